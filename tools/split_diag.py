"""Diagnose test_split_streams_bitwise_equal: max |diff| of split (k streams) vs unsplit CLS features,
per clip, with the CLS-only tail on / off, LayerNorm fold on, bf16; and k=1 run twice."""
import os
import sys
from functools import partial

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dino-video-summarization-transformer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from oracle import params as P  # noqa: E402


def main():
    from dsvt.models.timesformer import VisionTransformer
    sd = P.timesformer_state(2)
    m = VisionTransformer(img_size=224, patch_size=16, num_classes=0, embed_dim=768, depth=12, num_heads=12,
                          mlp_ratio=4, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=8)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.cuda().eval()
    m.dsvt_dtype = torch.bfloat16
    xs = [torch.from_numpy(P.clip(51, (3, 3, 4, 64, 64))).cuda(), torch.from_numpy(P.clip(52, (4, 3, 4, 64, 64))).cuda()]
    for tail in (True, False):
        for fold in (True, False):
            m.cls_tail, m.ln_fold = tail, fold
            with torch.no_grad():
                res = {}
                for k in (1, 1, 2, 3):
                    m.dsvt_streams = k
                    res.setdefault(k, []).append(m.forward_features(xs).float())
                torch.cuda.synchronize()
            base = res[1][0]
            d11 = (res[1][1] - base).abs().amax(1).tolist()
            d2 = (res[2][0] - base).abs().amax(1).tolist()
            d3 = (res[3][0] - base).abs().amax(1).tolist()
            print("tail=%d fold=%d  k1 again %s\n   k2 %s\n   k3 %s" % (tail, fold, ["%.1e" % v for v in d11],
                                                                      ["%.1e" % v for v in d2],
                                                                      ["%.1e" % v for v in d3]), flush=True)


if __name__ == "__main__":
    main()
