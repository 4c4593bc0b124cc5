"""Effective clock per kernel family from a rocprofv3 --pmc GRBM_GUI_ACTIVE run:
GRBM_GUI_ACTIVE summed over the 8 XCDs / 8 / kernel duration (MI355X_MICROARCH 'DVFS give-back';
reads high on dispatches under ~0.3 ms).  Usage: python tools/clock_summary.py DIR [DIR ...]"""
import csv
import glob
import sys


def main():
    for d in sys.argv[1:]:
        fam = {}
        durs = {}                       # Dispatch_Id -> duration (ns) from the kernel trace
        for path in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    durs[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for path in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    if r.get("Counter_Name") != "GRBM_GUI_ACTIVE":
                        continue
                    name = r["Kernel_Name"].split("(")[0][:60]
                    if "End_Timestamp" in r:
                        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                    else:
                        dur = durs.get(r.get("Dispatch_Id"), 0)
                    a = fam.setdefault(name, [0.0, 0.0, 0])
                    a[0] += float(r["Counter_Value"])
                    a[1] += dur
                    a[2] += 1
        print(d)
        for name, (cyc, dur, n) in sorted(fam.items(), key=lambda kv: -kv[1][1])[:10]:
            if dur > 0:
                print("  %-60s n=%5d  %.3f GHz  (%.1f us avg)" % (name, n, cyc / 8 / dur, dur / n / 1e3))


if __name__ == "__main__":
    main()
