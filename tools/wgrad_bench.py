"""Weight-gradient GEMM dW = dY^T . X at the training step's shapes (16 global clips: 25 104
rows; 48 local clips: 13 872 rows): dsvt wgrad kernel vs hipBLASLt (torch.mm, bf16 out).
usage: python tools/wgrad_bench.py [shape names]   (DSVT_WGRAD_ABL=n: csrc/wgrad.hip diagnostic builds)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402

from dsvt import ops  # noqa: E402

SHAPES = [("qkv_g", 25104, 2304, 768), ("proj_g", 25104, 768, 768), ("fc1_g", 25104, 3072, 768),
          ("fc2_g", 25104, 768, 3072), ("qkv_l", 13872, 2304, 768), ("fc2_l", 13872, 768, 3072),
          ("head_last", 80, 65536, 256)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


only = sys.argv[1:]          # optional shape names
for name, M, N, K in SHAPES:
    if only and name not in only:
        continue
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    g = torch.zeros(N, K, device="cuda")
    b = torch.zeros(N, device="cuda")
    t_d = timeit(lambda: ops.wgrad(dy, x, g, accumulate=True))
    t_b = timeit(lambda: ops.wgrad(dy, x, g, accumulate=True, db=b))
    t_t = timeit(lambda: g.add_(torch.mm(dy.t(), x)))
    fl = 2.0 * M * N * K
    print("%-10s M=%6d N=%6d K=%5d  dsvt %7.1f us %6.0f TF/s  (+bias %7.1f us)  hipBLASLt+add %7.1f us %6.0f TF/s" %
          (name, M, N, K, t_d * 1e3, fl / t_d / 1e9, t_b * 1e3, t_t * 1e3, fl / t_t / 1e9), flush=True)
