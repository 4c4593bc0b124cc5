"""Check HIP-graph capture of a split-batch forward (VisionTransformer.dsvt_streams > 1 inside a
capture).  usage: python tools/capture_repro.py [nested]
nested: capture dino_forward (student + teacher on two streams, each asking to split its batch).
Before dsvt.utils.nested_capture_fork the nested case died in capture_end (a two-level fork tree;
tools/capture_nested_min.py reproduces that with plain torch ops); now the inner splits run
unsplit inside a capture and both cases replay equal to eager."""
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


# bisection knobs: CAP_SERIAL_NETS=1 (dino_forward without the student/teacher fork), CAP_SERIAL_GROUPS=1
# (MultiCropWrapper groups in order), CAP_NO_RECORD=1 (Tensor.record_stream a no-op), CAP_K=<k> (chunks)
if os.environ.get("CAP_NO_RECORD") == "1":
    torch.Tensor.record_stream = lambda self, s: None
if os.environ.get("CAP_K"):
    _net = net

    def net(seed):   # noqa: F811
        bb = _net(seed)
        bb.dsvt_streams = int(os.environ["CAP_K"])
        return bb
if nested:
    s, t = MultiCropWrapper(net(1), DINOHead(768, 4096)).to(dev).eval(), \
        MultiCropWrapper(net(1), DINOHead(768, 4096)).to(dev).eval()
    if os.environ.get("CAP_SERIAL_GROUPS") == "1":
        s.concurrent_groups = t.concurrent_groups = False
    x = [torch.randn(3, 3, 8, 224, 224, device=dev) for _ in range(2)] + \
        [torch.randn(3, 3, 8, 96, 96, device=dev) for _ in range(2)]

    def fwd():
        with torch.no_grad():
            a, b = dino_forward(s, t, x, concurrent=os.environ.get("CAP_SERIAL_NETS") != "1")
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
