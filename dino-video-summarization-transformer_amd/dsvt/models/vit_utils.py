"""Init / layout helpers with the reference's semantics (models/vit_utils.py:62-179).
Parameter initialisation and module plumbing only -- no forward math lives here."""
import collections.abc
from itertools import repeat

import torch
import torch.nn as nn

IMAGENET_DEFAULT_MEAN = (0.485, 0.456, 0.406)   # models/vit_utils.py:20
IMAGENET_DEFAULT_STD = (0.229, 0.224, 0.225)    # models/vit_utils.py:21


def trunc_normal_(tensor, mean=0., std=1., a=-2., b=2.):
    """models/vit_utils.py:62-80: N(mean, std) truncated to [a, b] (absolute bounds)."""
    with torch.no_grad():
        return nn.init.trunc_normal_(tensor, mean=mean, std=std, a=a, b=b)


def _ntuple(n):
    def parse(x):
        if isinstance(x, collections.abc.Iterable):
            return x
        return tuple(repeat(x, n))
    return parse


to_2tuple = _ntuple(2)   # models/vit_utils.py:93


class DropPath(nn.Module):
    """models/vit_utils.py:152-179 (stochastic depth); a marker in dsvt: the drop is applied
    inside the fused residual epilogues (eval mode: identity)."""

    def __init__(self, drop_prob=None):
        super().__init__()
        self.drop_prob = drop_prob

    def extra_repr(self):
        return "drop_prob=%s" % (self.drop_prob,)
