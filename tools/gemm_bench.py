"""GEMM micro-benchmark on the hot-path shapes (bf16, one process, interleaved variants).

Usage: python tools/gemm_bench.py [variant ...]     (variants are DSVT_GEMM_VARIANT values;
        default: the library's auto choice only).  Prints TFLOP/s per shape and variant and
        a max-abs-diff check of every variant against variant "old" (128x128 kernel)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402

from dsvt import _lib, ops  # noqa: E402

M_G, M_L = 16 * 1569, 48 * 289       # rows of the global (16 clips) / local (48 clips) backbone calls
SHAPES = [  # (name, M, N, K, epilogue)
    ("qkv_g", M_G, 2304, 768, _lib.EPI_BIAS),
    ("proj_g", M_G, 768, 768, _lib.EPI_BIAS_RESID),
    ("fc1_g", M_G, 3072, 768, _lib.EPI_BIAS_GELU),
    ("fc2_g", M_G, 768, 3072, _lib.EPI_BIAS_RESID),
    ("qkv_l", M_L, 2304, 768, _lib.EPI_BIAS),
    ("fc1_l", M_L, 3072, 768, _lib.EPI_BIAS_GELU),
    ("head", 64, 65536, 256, _lib.EPI_BIAS),
    ("fc1b_g", M_G, 3072, 768, _lib.EPI_BIAS),     # fc1 without the GELU: the epilogue's price
    ("fc1b_l", M_L, 3072, 768, _lib.EPI_BIAS),
    # backward dX GEMMs (bf16 out, N = 768): dY . W for fc1 (K = 3072), qkv (K = 2304), proj (K = 768)
    ("dxfc1_g", M_G, 768, 3072, _lib.EPI_BIAS),
    ("dxqkv_g", M_G, 768, 2304, _lib.EPI_BIAS),
    ("dxprj_g", M_G, 768, 768, _lib.EPI_BIAS),
    ("dxfc1_l", M_L, 768, 3072, _lib.EPI_BIAS),
    ("dxqkv_l", M_L, 768, 2304, _lib.EPI_BIAS),
]


if os.environ.get("DSVT_CUSTOM"):    # "name:M:N:K:epi,...": extra shapes (epi = the EPI_* number)
    for item in os.environ["DSVT_CUSTOM"].split(","):
        nm, m, n, k, e = item.split(":")
        SHAPES.append((nm, int(m), int(n), int(k), int(e)))


def set_variant(v):
    _lib.call("dsvt_set_gemm_variant", int(v))      # raises for an unknown variant


def run(M, N, K, epi, reps=20):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.randn(M, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g)
    out_dtype = torch.float32 if epi == _lib.EPI_BIAS_RESID else torch.bfloat16
    out = torch.zeros(M, N, device=dev, dtype=out_dtype)
    ops.gemm(A, W, b, out, epilogue=epi)
    torch.cuda.synchronize()
    first = out.clone()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.gemm(A, W, b, out, epilogue=epi)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return 2.0 * M * N * K / (ms * 1e-3) / 1e12, ms, first


def torch_ref(M, N, K, reps=20):
    """hipBLASLt through torch (F.linear, bf16) on the same shape: a known-good reference."""
    dev = torch.device("cuda")
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    torch.nn.functional.linear(A, W, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.nn.functional.linear(A, W, b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return 2.0 * M * N * K / (ms * 1e-3) / 1e12, ms


def main():
    variants = [int(v) for v in sys.argv[1:]] or [0]
    print("hipBLASLt (torch F.linear bf16):")
    for name, M, N, K, epi in SHAPES:
        if os.environ.get("DSVT_SHAPES"):
            break
        tf, ms = torch_ref(M, N, K)
        print("  %-7s %6d %6d %5d  %7.1f TF/s (%7.1f us)" % (name, M, N, K, tf, ms * 1e3), flush=True)
    print("%-7s %6s %6s %5s | " % ("shape", "M", "N", "K") + " | ".join("v%d TF/s (us)" % v for v in variants))
    only = os.environ.get("DSVT_SHAPES")
    for name, M, N, K, epi in SHAPES:
        if only and name not in only.split(","):
            continue
        if any(v in (14, 24, 34) for v in variants):
            epi = _lib.EPI_BIAS          # ablation builds exist for EPI_BIAS only
        best, ref, diffs = {}, None, {}
        for _round in range(3):          # interleaved rounds in one process; best of 3
            for v in variants:
                set_variant(v)
                try:
                    tf, ms, out = run(M, N, K, epi)
                except _lib.DsvtError:           # variant does not take this epilogue
                    tf, ms, out = 0.0, float("inf"), ref if ref is not None else torch.zeros(1)
                if ref is None:
                    ref = out.float()
                diffs[v] = (out.float() - ref).abs().max().item()
                if v not in best or ms < best[v][1]:
                    best[v] = (tf, ms)
        cells = ["%7.1f (%7.1f) d=%.1e" % (best[v][0], best[v][1] * 1e3, diffs[v]) for v in variants]
        print("%-7s %6d %6d %5d | " % (name, M, N, K) + " | ".join(cells), flush=True)
    set_variant(0)


if __name__ == "__main__":
    main()
