"""Summarize a rocprofv3 kernel trace (SQLite results.db or kernel_stats/kernel_trace CSV)
into a per-kernel table: calls, total ms, avg us, share.

The per-step figure is DERIVED, never hand-entered: `--step-kernel NAME` names a kernel
launched a known number of times per step (`--per-step`, default 1), and steps = its calls /
per-step count.  E.g. the train step launches `ema_kernel` once (teacher EMA) and the
forward+loss step `loss_reduce_kernel` once per DINO loss.

`--last N` (with --step-kernel) keeps only the kernels of the LAST N steps: those that start after
the end of the step kernel's (N+1)-th-from-last launch and no later than its last launch (name the
step's LAST kernel, e.g. `center_ema` of the fwd+loss step).  A bench trace mixes the eager warm-up /
probe passes with the HIP-graph replays that follow them, so whole-trace averages mix two
launch patterns; the window holds replays only.  Every kernel's call count must then be a
multiple of N, or the summary refuses ("mixed trace") instead of printing per-step numbers."""
import argparse
import csv
import glob
import os
import sqlite3


def rows_from(path):
    """(name, duration ns, start ns, end ns) per dispatch"""
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(n, d, 0, d) for n, d in c.execute("select name, duration from kernels")]
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            out.append((r["Kernel_Name"], t1 - t0, t0, t1))
    return out


def main(path, step_kernel=None, per_step=1, last=0):
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) + \
            glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = cands[0]
    rows = rows_from(path)
    if last:
        if not step_kernel or path.endswith(".db"):
            raise SystemExit("--last needs --step-kernel and a kernel_trace CSV")
        ends = sorted(t1 for n, _, _, t1 in rows if step_kernel in n)
        need = (last + 1) * per_step
        if len(ends) < need:
            raise SystemExit("--last %d: only %d launches of '%s'" % (last, len(ends), step_kernel))
        t_start = ends[-need + per_step - 1] if per_step > 1 else ends[-need]
        t_end = ends[-1]                # kernels after the last step's step kernel belong to no step
        rows = [r for r in rows if t_start < r[2] <= t_end]
        bad = {}
        counts = {}
        for n, _, _, _ in rows:
            counts[n] = counts.get(n, 0) + 1
        for n, c in counts.items():
            if c % last:
                bad[n] = c
        if bad:
            raise SystemExit("mixed trace: in the last %d steps these kernels are not launched a whole number of "
                             "times per step: %s" % (last, sorted(bad.items())[:5]))
    agg = {}
    for n, d, _, _ in rows:
        a = agg.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    print("source: %s" % path)
    print("%-100s %7s %11s %10s %6s" % ("kernel", "calls", "total_ms", "avg_us", "share"))
    for n, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%-100s %7d %11.3f %10.2f %5.1f%%" % (n[:100], c, d / 1e6, d / c / 1e3, 100.0 * d / tot))
    line = "total kernel time: %.3f ms" % (tot / 1e6)
    if step_kernel:
        calls = sum(c for n, (c, _) in agg.items() if step_kernel in n)
        if calls and calls % per_step == 0:
            steps = calls // per_step
            line += "  (%.3f ms per step over %d steps: %d launches of '%s' / %d per step)" % (
                tot / 1e6 / steps, steps, calls, step_kernel, per_step)
        else:
            line += "  (steps not derivable: %d launches of '%s', %d per step)" % (calls, step_kernel, per_step)
    print(line)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--step-kernel", default=None, help="kernel-name substring launched a known number of times per step")
    ap.add_argument("--per-step", type=int, default=1)
    ap.add_argument("--last", type=int, default=0, help="summarize only the last N steps (graph replays)")
    a = ap.parse_args()
    main(a.path, a.step_kernel, a.per_step, a.last)
