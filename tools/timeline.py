"""Busy/idle accounting of a rocprofv3 kernel trace over the timed window of a bench run:
wall time of the last N kernels' span, sum of kernel durations, union of busy intervals
(concurrency = sum / union), and the largest idle gaps.
usage: python tools/timeline.py run_kernel_trace.csv [last_seconds]"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:80]))
rows.sort()
end = max(e for _, e, _ in rows)
win = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2
rows = [r for r in rows if r[0] >= end - win * 1e9]
t0 = rows[0][0]
span = end - t0
tot = sum(e - s for s, e, _ in rows)
union, cur_s, cur_e, gaps = 0, rows[0][0], rows[0][1], []
for s, e, n in rows[1:]:
    if s > cur_e:
        union += cur_e - cur_s
        gaps.append((s - cur_e, cur_e - t0, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
print("kernels %d  span %.2f ms  sum %.2f ms  busy-union %.2f ms (%.1f%%)  concurrency %.2f" %
      (len(rows), span / 1e6, tot / 1e6, union / 1e6, 100.0 * union / span, tot / max(union, 1)))
gaps.sort(reverse=True)
print("idle gaps: total %.2f ms in %d gaps; largest:" % (sum(g for g, _, _ in gaps) / 1e6, len(gaps)))
for g, at, n in gaps[:12]:
    print("  %8.1f us at +%.2f ms before %s" % (g / 1e3, at / 1e6, n))
