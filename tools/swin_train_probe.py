"""bench.py's Swin-T DINO train-step measurement alone: python tools/swin_train_probe.py [clips]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

clips = int(sys.argv[1]) if len(sys.argv) > 1 else 8
print(bench.swin_train_bench(torch.bfloat16, torch.device("cuda"), clips=clips, steps=3, warmup=1), flush=True)
