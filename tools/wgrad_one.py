"""One weight-gradient shape `reps` times (rocprofv3 counter passes of csrc/wgrad.hip).
usage: python tools/wgrad_one.py M N K [reps]   (DSVT_WGRAD_ABL=n: the diagnostic builds)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))
import torch  # noqa: E402

from dsvt import ops  # noqa: E402

M, N, K = map(int, sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
g = torch.zeros(N, K, device="cuda")
for _ in range(reps):
    ops.wgrad(dy, x, g, accumulate=True)
torch.cuda.synchronize()
print("done")
