"""Static check of gemm_4w.hip's untracked (inline-asm) global loads: between each such load and
the counted `s_waitcnt vmcnt` that retires it, no instruction may read or write the load's
destination VGPRs (a read sees stale data, a write is overwritten by the landing load -- the ABL 16
build that prefetched into dead registers faulted on the GPU).  Scans the code text from each
asm load to the first `s_waitcnt vmcnt(N)` with N <= the VMEM ops issued after it (both sides of any forward branch in between: a
superset of every path).
Usage: python tools/asm_pending_check.py <kernel .s from hipcc -save-temps>"""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def check(lines, name):
    bad, n = 0, 0
    i = 0
    while i < len(lines):
        ln = lines[i].strip()
        m = re.match(r"global_load_dwordx([24])\s+(v\[\d+:\d+\]),", ln)
        if m and i > 0 and "ASMSTART" in lines[i - 1]:
            n += 1
            dst = regs(m.group(2))
            younger = 0                   # VMEM ops issued after the load (text order)
            j = i + 1
            while j < len(lines):
                t = lines[j].strip()
                w = re.match(r"s_waitcnt vmcnt\((\d+)\)", t)
                if w and int(w.group(1)) <= younger:
                    break                 # retires the load (vmcnt counts in issue order)
                if re.match(r"(global|buffer|scratch)_(load|store|atomic)", t):
                    younger += 1
                if t.startswith("s_endpgm"):
                    print("%s: no wait for the load at line %d before s_endpgm" % (name, i + 1))
                    bad += 1
                    break
                if t and not t.startswith(";") and not t.startswith("."):
                    ops = re.split(r"[\s,]+", t)[1:]
                    hit = set()
                    for o in ops:
                        hit |= regs(o)
                    if hit & dst and not (t.startswith("global_load_dwordx") and "ASMSTART" in lines[j - 1]
                                           and not (regs(ops[0]) & dst)):
                        print("%s: line %d touches pending %s: %s" % (name, j + 1, sorted(hit & dst), t))
                        bad += 1
                j += 1
        i += 1
    return n, bad


def main():
    src = open(sys.argv[1]).read().split("\n")
    starts = [i for i, l in enumerate(src) if re.match(r"^_ZN4dsvt14gemm_4w_kernel\w+:", l)]
    total_bad = 0
    for k, s in enumerate(starts):
        e = next(i for i in range(s, len(src)) if src[i].startswith(".Lfunc_end"))
        name = src[s].split(":")[0]
        n, bad = check(src[s:e], name)
        print("%-60s asm loads %3d  violations %d" % (name[-60:], n, bad))
        total_bad += bad
    sys.exit(1 if total_bad else 0)


if __name__ == "__main__":
    main()
