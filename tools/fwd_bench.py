"""North-star unit in isolation: ViT-B/16 divided space-time forward of 16 clips at 8x224^2
(the global crops of one 8-sample step), bf16, random init -- clips/s and the fraction of the
dense bf16 MFMA peak on executed / reference FLOPs, for the given stream splits.

usage: python tools/fwd_bench.py [--reps R] [--streams auto,1] [--clips 16] [--fold-ln 0|1]"""
import argparse
import os
import sys
import time
from functools import partial

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from bench import PEAK_TFLOPS, vit_fwd_flops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warm", type=int, default=3)
    ap.add_argument("--clips", type=int, default=16)
    ap.add_argument("--streams", default="auto,1")
    ap.add_argument("--fold-ln", default=None)
    args = ap.parse_args()
    from dsvt.models.timesformer import VisionTransformer
    torch.manual_seed(1)
    m = VisionTransformer(img_size=224, num_classes=0, embed_dim=768, depth=12, num_heads=12, qkv_bias=True,
                          norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=8,
                          attention_type="divided_space_time").cuda().eval()
    with torch.no_grad():
        for blk in m.blocks:
            blk.temporal_fc.weight.normal_(0, 0.02)
        m.time_embed.normal_(0, 0.02)
    m.dsvt_dtype = torch.bfloat16
    if args.fold_ln is not None and hasattr(m, "fold_ln"):
        m.fold_ln = bool(int(args.fold_ln))
    x = torch.randn(args.clips, 3, 8, 224, 224, device="cuda")
    exe, ref = vit_fwd_flops(8, 224, folded=True), vit_fwd_flops(8, 224)
    peak = PEAK_TFLOPS["bf16"]
    for st in args.streams.split(","):
        m.dsvt_streams = st
        with torch.no_grad():
            for _ in range(args.warm):
                m(x)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                y = m(x)
            torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / args.reps
        cps = args.clips / t
        print("streams=%-5s %8.1f clips/s  %.3f ms/fwd  frac_executed %.4f  frac_reference %.4f  finite %s" %
              (st, cps, t * 1e3, cps * exe / 1e12 / peak, cps * ref / 1e12 / peak, bool(torch.isfinite(y).all())),
              flush=True)


if __name__ == "__main__":
    main()
