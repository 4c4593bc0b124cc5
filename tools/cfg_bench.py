"""One BASELINE config's forward alone, for rocprofv3 / A-B runs: c2bb (the config-2 ViT-B/16
divided backbone, 16 clips 8x224^2), c4 (joint space-time ViT-B/16, 2 clips 16x224^2) or c5
(Video Swin-T, 8 clips 8x224^2); bf16, random init, synthetic input.

usage: python tools/cfg_bench.py c4 [--reps 5] [--warm 2] [--streams auto|1|2|3] [--ln-fold auto|on|off]"""
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

from bench import PEAK_TFLOPS, joint_flops, swin_t_flops, vit_fwd_flops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg", choices=["c2bb", "c4", "c5", "fs"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--streams", default=None)
    ap.add_argument("--ln-fold", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--graph", action="store_true", help="also time HIP-graph replays (as bench.py does)")
    ap.add_argument("--fpc", type=int, default=16, help="fs: frames per backbone call")
    args = ap.parse_args()
    from dsvt.models import SwinTransformer3D
    from dsvt.models.timesformer import VisionTransformer
    dev = torch.device("cuda")
    torch.manual_seed(1)
    if args.cfg == "fs":                # frame scoring: one 64-frame 224^2 video, local 3 / global 30 (bench.py)
        from dsvt.scoring import FrameScorer
        torch.manual_seed(2)
        fm = VisionTransformer(img_size=224, num_classes=0, embed_dim=768, depth=12, num_heads=12, qkv_bias=True,
                               norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=8,
                               attention_type="divided_space_time").to(dev).eval()
        fm.dsvt_dtype = torch.bfloat16
        sc = FrameScorer(fm, local_clip_size=3, global_clip_size=30, frames_per_call=args.fpc)
        video = torch.randn(64, 3, 224, 224, device=dev)

        class _M:                       # the scorer as a "model" of 64 "clips" (frames)
            def __call__(self, v):
                return sc.score(v)
        m, x, n, gf = _M(), video, 64, (vit_fwd_flops(3, 224) + vit_fwd_flops(30, 224)) / 1e9
    elif args.cfg == "c5":
        m = SwinTransformer3D().to(dev)
        m.eval()                        # returns None, as the reference's (swin_transformer.py:684-687)
        x = torch.randn(8, 3, 8, 224, 224, device=dev)
        n, gf = 8, swin_t_flops() / 1e9
    else:
        T, attn = (8, "divided_space_time") if args.cfg == "c2bb" else (16, "joint_space_time")
        m = VisionTransformer(img_size=224, num_classes=0, embed_dim=768, depth=12, num_heads=12, qkv_bias=True,
                              norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=T,
                              attention_type=attn).to(dev).eval()
        n = 16 if args.cfg == "c2bb" else 2
        x = torch.randn(n, 3, T, 224, 224, device=dev)
        gf = (vit_fwd_flops(8, 224, folded=True, cls_tail=m.cls_tail) if args.cfg == "c2bb" else joint_flops()) / 1e9
        if args.streams is not None:
            m.dsvt_streams = args.streams if args.streams == "auto" else int(args.streams)
        m.ln_fold = {"auto": "auto", "on": True, "off": False}[args.ln_fold]
    m.dsvt_dtype = torch.bfloat16
    with torch.no_grad():
        for _ in range(args.warm):
            m(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            m(x)
        torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / args.reps
    if args.graph:
        with torch.no_grad():
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                m(x)
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                m(x)
            g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                g.replay()
            torch.cuda.synchronize()
        tg = (time.perf_counter() - t0) / args.reps
        print("%s graph: %.2f clips/s, %.3f ms per replay" % (args.cfg, n / tg, tg * 1e3))
    print("%s: %.2f clips/s, %.3f ms per call, %.1f TFLOP/s executed (%.1f %% of the bf16 peak)"
          % (args.cfg, n / t, t * 1e3, n * gf / t / 1e3, 100 * n * gf / t / 1e3 / PEAK_TFLOPS["bf16"]))


if __name__ == "__main__":
    main()
