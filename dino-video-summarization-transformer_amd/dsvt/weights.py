"""Storage-dtype views of nn.Parameters for the kernels.

bf16 mode: each weight is cast ONCE by the dsvt cast kernel and cached until the parameter
changes (tracked by its autograd version counter + storage pointer, so optimizer steps,
EMA updates, load_state_dict and .to() all invalidate it).  fp32 mode: the parameter
itself (no copy)."""
import torch

from . import ops


class WeightCache:
    def __init__(self):
        self._c = {}

    def getter(self, mode):
        def get(p, flat=False):
            t = p.detach()
            if flat:
                t = t.reshape(t.shape[0], -1)
            if t.dtype != torch.float32:
                raise TypeError("dsvt expects fp32 master parameters, got %s" % t.dtype)
            if mode == torch.float32:
                return t.contiguous()
            key = (id(p), flat)
            ent = self._c.get(key)
            if ent is not None and ent[0] == p._version and ent[1] == p.data_ptr():
                return ent[2]
            out = torch.empty(t.shape, device=t.device, dtype=mode)
            ops.cast(t.contiguous(), out)
            self._c[key] = (p._version, p.data_ptr(), out)
            return out
        return get

    def clear(self):
        self._c.clear()
