"""Reproduce / check HIP-graph capture of a split-batch forward (VisionTransformer.dsvt_streams
> 1 inside a capture).  usage: DSVT_CAPTURE_SPLIT=1 python tools/capture_repro.py [nested]
nested: capture dino_forward (student + teacher on two streams, each splitting its batch)."""
import faulthandler
import os
import sys
from functools import partial

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from dsvt.models.timesformer import VisionTransformer  # noqa: E402
from dsvt.utils import MultiCropWrapper, dino_forward  # noqa: E402
from dsvt.vision_transformer import DINOHead  # noqa: E402

dev = torch.device("cuda")
nested = "nested" in sys.argv[1:]


def net(seed):
    torch.manual_seed(seed)
    bb = VisionTransformer(img_size=224, num_classes=0, embed_dim=768, depth=2, num_heads=12, qkv_bias=True,
                           norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=8).to(dev).eval()
    bb.dsvt_streams = 3
    return bb


if nested:
    s, t = MultiCropWrapper(net(1), DINOHead(768, 4096)).to(dev).eval(), \
        MultiCropWrapper(net(1), DINOHead(768, 4096)).to(dev).eval()
    x = [torch.randn(3, 3, 8, 224, 224, device=dev) for _ in range(2)] + \
        [torch.randn(3, 3, 8, 96, 96, device=dev) for _ in range(2)]

    def fwd():
        with torch.no_grad():
            a, b = dino_forward(s, t, x)
        return torch.cat([a, b])
else:
    m = net(1)
    x = torch.randn(6, 3, 8, 224, 224, device=dev)

    def fwd():
        with torch.no_grad():
            return m(x)
ref = fwd()
torch.cuda.synchronize()
print("eager ok", flush=True)
g = torch.cuda.CUDAGraph()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    fwd()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
print("capturing", flush=True)
with torch.cuda.graph(g):
    out = fwd()
print("captured", flush=True)
g.replay()
torch.cuda.synchronize()
print("replayed; max |diff| vs eager = %.3g" % (out - ref).abs().max().item(), flush=True)
