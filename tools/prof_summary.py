"""Summarize a rocprofv3 kernel trace (SQLite results.db or kernel_stats/kernel_trace CSV)
into a per-kernel table: calls, total ms, avg us, share."""
import csv
import glob
import os
import sqlite3
import sys


def rows_from(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(n, d) for n, d in c.execute("select name, duration from kernels")]
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return out


def main(path, steps=None):
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) + \
            glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = cands[0]
    agg = {}
    for n, d in rows_from(path):
        a = agg.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    print("source: %s" % path)
    print("%-100s %7s %11s %10s %6s" % ("kernel", "calls", "total_ms", "avg_us", "share"))
    for n, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%-100s %7d %11.3f %10.2f %5.1f%%" % (n[:100], c, d / 1e6, d / c / 1e3, 100.0 * d / tot))
    print("total kernel time: %.3f ms%s" % (tot / 1e6, "" if not steps else "  (%.3f ms per step over %d steps)"
                                             % (tot / 1e6 / steps, steps)))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
