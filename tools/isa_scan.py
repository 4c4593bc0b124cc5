"""Compiler-inserted LDS-DMA drains: compile csrc sources to gfx950 assembly and, for every kernel
that stages through LDS-DMA (global_load_lds), list each `s_waitcnt vmcnt(0)` that the next few
instructions follow with an LDS read -- the pattern that drains every in-flight prefetch stage
(r05: the wgrad kernel's builtin transposed reads, the GEMM epilogues' pending row-scale loads).
Inside a loop (the compiler's "in Loop" block comments) it runs per iteration.
usage: python tools/isa_scan.py [source.hip ...]   (default: the GEMM / wgrad / attention sources)"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dino-video-summarization-transformer_amd", "csrc")
DEFAULT = ["gemm.hip", "gemm_8ph.hip", "gemm_big.hip", "gemm_192.hip", "wgrad.hip", "attn_flash.hip"]


def scan(asm):
    out = []
    for f in re.split(r"\n(?=_Z[\w]+:)", asm):
        m = re.match(r"(_Z[\w]+):", f)
        if not m or "global_load_lds" not in f:
            continue
        lines = [l.strip() for l in f.split(".Lfunc_end")[0].split("\n")]
        hits, in_loop = 0, 0
        block_in_loop = False
        for k, l in enumerate(lines):
            if l.startswith(".LBB") or l.startswith("; %bb"):
                block_in_loop = "Loop" in l
            if l.startswith("s_waitcnt") and "vmcnt(0)" in l:
                nxt = [x for x in lines[k + 1:k + 8] if x and not x.startswith(";")]
                if any(x.startswith("ds_read") for x in nxt):
                    hits += 1
                    in_loop += block_in_loop
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        out.append((hits, in_loop, name))
    return out


def main():
    srcs = sys.argv[1:] or DEFAULT
    bad = 0
    with tempfile.TemporaryDirectory() as td:
        for s in srcs:
            path = s if os.path.isabs(s) else os.path.join(CSRC, s)
            asm = os.path.join(td, os.path.basename(s) + ".s")
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + CSRC,
                            "--cuda-device-only", "-S", "-o", asm, path], check=True, capture_output=True)
            for hits, in_loop, name in scan(open(asm).read()):
                flag = "LOOP" if in_loop else ("once" if hits else "ok")
                bad += in_loop
                print("%-5s drains %2d (in loops %2d)  %s" % (flag, hits, in_loop, name[:110]))
    print("kernels with a per-iteration drain before an LDS read: %d" % bad)


if __name__ == "__main__":
    main()
