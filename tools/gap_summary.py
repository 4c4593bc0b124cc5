"""Idle gaps on one HIP queue of a rocprofv3 kernel trace (CSV), grouped by the kernel pair
around each gap: where a stream waits (host launch cost of tiny ops, cross-stream events).
usage: python tools/gap_summary.py TRACE.csv [--queue 1] [--step-kernel ema_kernel] [--steps 2]
       [--min-us 5]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--queue", default="1")
    ap.add_argument("--step-kernel", default="ema_kernel")
    ap.add_argument("--steps", type=int, default=2, help="window: the last N step-kernel intervals")
    ap.add_argument("--min-us", type=float, default=5.0)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["End_Timestamp"]) for r in rows if a.step_kernel in r["Kernel_Name"]]
    t0, t1 = marks[-1 - a.steps], marks[-1]
    win = [r for r in rows if int(r["Start_Timestamp"]) >= t0 and int(r["End_Timestamp"]) <= t1]
    q = [r for r in win if r["Queue_Id"] == a.queue]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in q)
    gaps, cnt, tot = collections.Counter(), collections.Counter(), 0
    for x, y in zip(q, q[1:]):
        g = int(y["Start_Timestamp"]) - int(x["End_Timestamp"])
        if g > a.min_us * 1e3:
            k = (x["Kernel_Name"][:48], y["Kernel_Name"][:48])
            gaps[k] += g
            cnt[k] += 1
            tot += g
    span = (t1 - t0) / a.steps / 1e6
    print("window: %d intervals of %.2f ms; queue %s busy %.2f ms, gaps > %.0f us %.2f ms (per interval)"
          % (a.steps, span, a.queue, busy / a.steps / 1e6, a.min_us, tot / a.steps / 1e6))
    for k, v in gaps.most_common(20):
        print("  %6.2f ms  n=%4d  %s  ->  %s" % (v / a.steps / 1e6, cnt[k] // a.steps, k[0], k[1]))


if __name__ == "__main__":
    main()
