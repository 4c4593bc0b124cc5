"""Per-launch listing of the LAST forward in a rocprofv3 kernel trace (csv), split on a marker
kernel that runs once per forward (default: im2col3d).  usage: trace_last_call.py trace.csv [marker]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "im2col3d"
starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
last = rows[starts[-1]:]
tot = 0.0
for r in last:
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += us
    print("%8.1f  grid %8s x %4s  %s" % (us, r["Grid_Size_X"], r["Grid_Size_Y"], r["Kernel_Name"][:90]))
span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3
print("kernel sum %.1f us, span %.1f us, %d launches" % (tot, span, len(last)))
