"""Backbone forward (16 divided 8x224^2 clips, bf16) with the batch split over 1..4 concurrent
HIP streams (VisionTransformer.dsvt_streams): clips/s per split and max |diff| vs no split."""
import os
import sys
import time
from functools import partial

import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "dino-video-summarization-transformer_amd"))
from dsvt.models.timesformer import VisionTransformer  # noqa: E402

B = int(os.environ.get("DSVT_SPLIT_B", "16"))
dev = "cuda"
torch.manual_seed(1)
m = VisionTransformer(img_size=224, num_classes=0, embed_dim=768, depth=12, num_heads=12, qkv_bias=True,
                      norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=8,
                      attention_type="divided_space_time").to(dev).eval()
m.dsvt_dtype = torch.bfloat16
x = torch.randn(B, 3, 8, 224, 224, device=dev)
ref = None
with torch.no_grad():
    for rnd in range(2):
        for k in (1, 2, 3, 4):
            m.dsvt_streams = k
            for _ in range(2):
                y = m(x)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(8):
                m(x)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 8
            if ref is None:
                ref = y.clone()
            print("round %d streams %d: %.1f clips/s  max|diff| %.3g" % (rnd, k, B / dt, (y - ref).abs().max().item()),
                  flush=True)
