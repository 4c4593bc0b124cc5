"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE run
separately: they do not fit one pass on gfx950, MI355X_MICROARCH.md §rocprofv3 PMC slots).

Both counters are in KiB.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports
exactly half the bytes of a wide coalesced streaming read, so
    traffic_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024      per dispatch.

usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR [OUT_JSON [RUN_DESCRIPTION]]
Prints a table (calls, avg fetch/write MB per dispatch, corrected traffic) and, with
OUT_JSON, writes {kernel_name: {"traffic_bytes": .., "fetch_kib": .., "write_kib": .., "calls": ..}}
which bench.py reads to fill roofline.traffic for its dominant kernel."""
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % d)
    acc = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                a = acc.setdefault(r["Kernel_Name"], [0, 0.0])
                a[0] += 1
                a[1] += float(r["Counter_Value"])
    return {k: (n, v / n) for k, (n, v) in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    rows = []
    for k in sorted(set(fetch) & set(write)):
        n, fk = fetch[k]
        _, wk = write[k]
        tb = (2.0 * fk + wk) * 1024.0
        out[k] = {"traffic_bytes": tb, "fetch_kib": fk, "write_kib": wk, "calls": n}
        rows.append((tb * n, k, n, fk, wk, tb))
    print("%-90s %6s %12s %12s %14s" % ("kernel", "calls", "fetch MB", "write MB", "traffic MB"))
    for _, k, n, fk, wk, tb in sorted(rows, reverse=True)[:25]:
        print("%-90s %6d %12.2f %12.2f %14.2f" % (k[:90], n, fk * 1024 / 1e6, wk * 1024 / 1e6, tb / 1e6))
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                                 "traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 B per dispatch",
                       "run": sys.argv[4] if len(sys.argv) > 4 else "",
                       "kernels": out}, f, indent=1)


if __name__ == "__main__":
    main()
