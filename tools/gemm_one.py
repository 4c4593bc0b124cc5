"""Run one GEMM shape with one kernel variant `reps` times (for rocprofv3 counter passes).
usage: python tools/gemm_one.py VARIANT M N K EPI [reps]
EPI 102 = the residual GEMM with the LayerNorm-statistics epilogue (dsvt_gemm_resid_stats_fwd, the
forward's dominant kernel gemm_8ph_kernel<2, true, 0, false, 2>)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))
import torch  # noqa: E402

from dsvt import _lib, ops  # noqa: E402

v, M, N, K, epi = map(int, sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
_lib.lib().dsvt_set_gemm_variant(v)
dev = torch.device("cuda")
A = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
b = torch.randn(N, device=dev)
stats = epi == 102
out = torch.zeros(M, N, device=dev, dtype=torch.float32 if epi in (_lib.EPI_BIAS_RESID, 102) else torch.bfloat16)
if stats:
    xb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    st = torch.empty(M, 12, 2, device=dev)
for _ in range(reps):
    if stats:
        ops.gemm_resid_stats(A, W, b, out, xb, st)
    else:
        ops.gemm(A, W, b, out, epilogue=epi)
torch.cuda.synchronize()
print("done")
