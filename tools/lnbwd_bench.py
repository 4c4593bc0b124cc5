"""LayerNorm backward at the training shape (25 104 rows x 768, fp32 dy), through the C-ABI.
usage: python tools/lnbwd_bench.py [libdsvt.so path]   (A/B two builds in one process is not
possible with one ctypes handle; run once per library)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))
from dsvt import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = sys.argv[1]
import torch  # noqa: E402

from dsvt import ops  # noqa: E402

rows, C = 25104, 768
x = torch.randn(rows, C, device="cuda")
dy = torch.randn(rows, C, device="cuda")
gamma = torch.rand(C, device="cuda") + 0.5
dx = torch.zeros(rows, C, device="cuda")
dg = torch.zeros(C, device="cuda")
db = torch.zeros(C, device="cuda")
for _ in range(2):
    ops.layernorm_bwd(x, dy, gamma, 1e-6, dx, rows, dg, db)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    ops.layernorm_bwd(x, dy, gamma, 1e-6, dx, rows, dg, db)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print("%s: %.1f us per LN backward (x, dy, dx r/w: %.2f TB/s)" % (_lib.LIB_PATH, ms * 1e3, rows * C * 16 / ms / 1e9))
