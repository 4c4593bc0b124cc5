"""Config 5 (Video Swin-T, 8 clips 8x224^2, bf16) per GEMM launch class: the in-library HIP-event
probe around each GEMM launch of one eager forward, grouped by (kernel, FLOPs, algorithmic bytes):
launches, average time, TF/s, GB/s, and the fraction of its own roofline max(FLOP / 2.5166 PF,
bytes / 8 TB/s).  Usage: python tools/swin_probe.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dsvt import ops  # noqa: E402
from dsvt._lib import PROBE_GEMM  # noqa: E402
from dsvt.models import SwinTransformer3D  # noqa: E402

PEAK_TF, HBM_GBS = 2516.6, 8000.0


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda")
    torch.manual_seed(1)
    m = SwinTransformer3D().to(dev)
    m.eval()
    m.dsvt_dtype = torch.bfloat16
    x = torch.randn(8, 3, 8, 224, 224, device=dev)
    with torch.no_grad():
        m(x)
        torch.cuda.synchronize()
        ops.probe_enable(PROBE_GEMM, 1 << 16)
        for _ in range(reps):
            m(x)
        torch.cuda.synchronize()
        ms, work, fam, tag, nbytes = ops.probe_read(1 << 16, with_bytes=True)
        ops.probe_disable()
    cls = {}
    for t, m_, w_, b_ in zip(tag, ms, work, nbytes):
        c = cls.setdefault((int(t), float(w_), float(b_)), [0, 0.0])
        c[0] += 1
        c[1] += float(m_)
    tot = sum(v[1] for v in cls.values()) / reps
    print("GEMM time per forward: %.1f us over %d launches" % (tot * 1e3, sum(v[0] for v in cls.values()) // reps))
    print("%-58s %4s %8s %7s %7s %8s %6s" % ("kernel", "n", "avg us", "GF", "MB", "GB/s", "frac"))
    for (t, w_, b_), (n, tms) in sorted(cls.items(), key=lambda kv: -kv[1][1]):
        avg = tms / n * 1e-3
        bound = max(w_ / (PEAK_TF * 1e12), b_ / (HBM_GBS * 1e9))
        print("%-58s %4d %8.1f %7.2f %7.1f %8.0f %6.3f" % (ops.gemm_kernel_name(t)[5:63], n // reps, avg * 1e6,
                                                            w_ / 1e9, b_ / 1e6, b_ / avg / 1e9, bound / avg))


if __name__ == "__main__":
    main()
