"""Static checks on the gfx950 assembly of the 4-wave GEMM (csrc/gemm_4w.hip), CPU only (hipcc
cross-compiles): every untracked inline-asm global load (the epilogue prefetches and the residual
rows) is retired by a counted `s_waitcnt vmcnt(N)` before anything touches its destination
registers (tools/asm_pending_check.py), and no kernel of the file spills to scratch."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_gemm_4w_asm_loads_retired_before_use(tmp_path):
    src = os.path.join(ROOT, "dino-video-summarization-transformer_amd", "csrc", "gemm_4w.hip")
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function",
                        "-save-temps", "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o",
                        str(tmp_path / "g.o")], cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "ScratchSize [bytes/lane]: 0" in r.stderr
    assert not [ln for ln in r.stderr.splitlines() if "ScratchSize [bytes/lane]:" in ln and not ln.rstrip().endswith(
        "ScratchSize [bytes/lane]: 0 [-Rpass-analysis=kernel-resource-usage]")]
    asm = [f for f in os.listdir(tmp_path) if f.endswith(".s") and "gfx950" in f]
    assert asm
    c = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asm_pending_check.py"), str(tmp_path / asm[0])],
                       capture_output=True, text=True, timeout=300)
    print(c.stdout[-3000:])
    assert c.returncode == 0, c.stdout[-3000:]
    assert "asm loads  40" in c.stdout          # the LayerNorm-folded kernels prefetch 24 + 16 values
