"""Joint space-time attention at config 4's size (2 clips x 12 heads x L = 3137, head_dim 64):
time per launch and TFLOP/s (4 L^2 d per head) of the flash kernel (variant 0 = auto, 11-15 = its
workgroup shapes: 4 waves x 1 / 2 query tiles, 8 waves x 3+2 / 2+1 / 2+2) and the register-staged kernel
(variant 8), interleaved in one process.  NB clips (default 2), VARIANTS="0,11,..." """
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))
import torch  # noqa: E402

from dsvt import _lib, ops  # noqa: E402

nb, L, heads = int(os.environ.get("NB", 2)), int(os.environ.get("L", 3137)), 12
C = heads * 64
Q = torch.randn(nb * L, 3 * C, device="cuda").to(torch.bfloat16)
out = torch.empty(nb * L, C, device="cuda", dtype=torch.bfloat16)
fl = 4.0 * nb * heads * L * L * 64
res = {}
for rnd in range(3):
    for v in [int(x) for x in os.environ.get("VARIANTS", "0,11,12,13,14,15,8").split(",")]:
        _lib.call("dsvt_set_attn_variant", v)
        ops.attn_joint(Q, out, nb, L, heads, 0.125)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.attn_joint(Q, out, nb, L, heads, 0.125)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        res[v] = min(res.get(v, 1e9), us)
_lib.call("dsvt_set_attn_variant", 0)
for v, us in res.items():
    print("variant %d: %.1f us  %.1f TF/s" % (v, us, fl / us / 1e6))
