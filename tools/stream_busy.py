"""Per-queue busy accounting of a rocprofv3 kernel trace over the last `last_seconds` of a run
(the training step's main dX chain vs its weight-gradient stream): for each hardware queue /
stream the kernel count, the sum of durations, the busy union and the span from its first
kernel to its last; plus the window's span and where each queue's last kernel ends.
usage: python tools/stream_busy.py run_kernel_trace.csv [last_seconds|@marker] [top]
  @marker: the window starts at the last launch of the first kernel whose name contains `marker`
  (e.g. @cast_multi: the teacher's input cast, the first kernel of a training step)."""
import csv
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


rows = []
with open(sys.argv[1]) as f:
    rd = csv.DictReader(f)
    key = "Stream_Id" if "Stream_Id" in rd.fieldnames else "Queue_Id"
    for r in rd:
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get(key, "?"), r["Kernel_Name"]))
end = max(r[1] for r in rows)
arg = sys.argv[2] if len(sys.argv) > 2 else "0.2"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 8
if arg.startswith("@"):
    start = max(r[0] for r in rows if arg[1:] in r[3])
else:
    start = end - float(arg) * 1e9
rows = [r for r in rows if r[0] >= start]
t0 = min(r[0] for r in rows)
print("window %.2f ms (%s), %d kernels, busy-union all %.2f ms" %
      ((end - t0) / 1e6, key, len(rows), union([(s, e) for s, e, _, _ in rows]) / 1e6))
by = defaultdict(list)
for r in rows:
    by[r[2]].append(r)
for q, rs in sorted(by.items(), key=lambda kv: -sum(e - s for s, e, _, _ in kv[1])):
    tot = sum(e - s for s, e, _, _ in rs)
    u = union([(s, e) for s, e, _, _ in rs])
    first, last = min(s for s, _, _, _ in rs), max(e for _, e, _, _ in rs)
    print("%s %s: %d kernels  sum %.2f ms  union %.2f ms  first +%.2f  last +%.2f ms" %
          (key, q, len(rs), tot / 1e6, u / 1e6, (first - t0) / 1e6, (last - t0) / 1e6))
    names = defaultdict(lambda: [0, 0])
    for s, e, _, n in rs:
        n = n.split("(")[0][:70]
        names[n][0] += 1
        names[n][1] += e - s
    for n, (c, d) in sorted(names.items(), key=lambda kv: -kv[1][1])[:top]:
        print("    %6d  %8.2f ms  %s" % (c, d / 1e6, n))
    rs.sort()
    gaps = [(rs[i + 1][0] - rs[i][1], rs[i][1], rs[i][3], rs[i + 1][3]) for i in range(len(rs) - 1)]
    big = [g for g in gaps if g[0] > 30000]
    print("    idle inside its span: %.2f ms; %d gaps > 30 us (%.2f ms), largest:" %
          (((last - first) - u) / 1e6, len(big), sum(g[0] for g in big) / 1e6))
    for g, at, a, b in sorted(big, reverse=True)[:top]:
        print("      %7.1f us at +%.2f ms  %s -> %s" % (g / 1e3, (at - t0) / 1e6, a.split("(")[0][:45],
                                                   b.split("(")[0][:45]))
# 2-ms buckets: which streams have a kernel running (busy fraction per stream)
qs = sorted(by)
print("timeline (busy fraction per 2 ms; columns " + " ".join(str(q) for q in qs) + ")")
for b0 in range(t0, end, 2000000):
    b1 = b0 + 2000000
    fr = []
    for q in qs:
        iv = [(max(s, b0), min(e, b1)) for s, e, _, _ in by[q] if e > b0 and s < b1]
        fr.append(union(iv) / 2e6 if iv else 0.0)
    print("  +%5.1f  " % ((b0 - t0) / 1e6) + " ".join("%4.2f" % f for f in fr))
