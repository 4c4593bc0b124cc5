"""Busy-time union vs span of the last K steps of a rocprofv3 kernel trace (csv): how much of
the step the GPU runs at least one kernel, and the average number of kernels in flight.
usage: overlap.py trace.csv step_kernel_substring [last_steps]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mark = sys.argv[2]
last = int(sys.argv[3]) if len(sys.argv) > 3 else 5
ends = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
sel = rows[ends[-last - 1] + 1:ends[-1] + 1]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel)
span = iv[-1][1] - iv[0][0]
busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
ksum = sum(e - s for s, e in iv)
print("steps %d: span %.2f ms, busy %.2f ms (%.1f %%), kernel sum %.2f ms, mean concurrency %.2f"
      % (last, span / 1e6 / last, busy / 1e6 / last, 100.0 * busy / span, ksum / 1e6 / last, ksum / busy))
