"""AdamW on libdsvt.so: the optimizer of the reference's SSL step
(`torch.optim.AdamW(params_groups)`, train_ssl.py:384; `optimizer.step()` at :551).

A torch.optim.Optimizer subclass, so param_groups (the lr / weight-decay schedules write them
each iteration, train_ssl.py:486-490), zero_grad and state_dict behave as the reference's.
step() is one multi-tensor HIP launch per (param group, step count) list -- parameters whose
.grad is None are skipped and do not count a step, like torch's (that is what the reference's
cancel_gradients_last_layer relies on in the first epoch, utils/utils.py:114-119).
"""
import torch

from ._lib import DsvtError, call


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        if lr < 0.0 or eps <= 0.0 or not (0.0 <= betas[0] < 1.0) or not (0.0 <= betas[1] < 1.0):
            raise ValueError("invalid AdamW hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        from . import ops
        from .utils import _tensor_list
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse or not p.is_cuda:
                    raise DsvtError("dsvt AdamW: dense GPU parameters only (no CPU fallback)")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)          # host scalar, like torch's non-capturable AdamW
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append(p)
            b1, b2 = group["betas"]
            for step, ps in sorted(by_step.items()):
                grads = [p.grad if p.grad.is_contiguous() else p.grad.contiguous() for p in ps]
                tl, pptr = _tensor_list(ps)
                _, gptr = _tensor_list(grads)
                _, mptr = _tensor_list([self.state[p]["exp_avg"] for p in ps])
                _, vptr = _tensor_list([self.state[p]["exp_avg_sq"] for p in ps])
                call("dsvt_adamw", pptr.data_ptr(), gptr.data_ptr(), mptr.data_ptr(), vptr.data_ptr(),
                     tl.sizes.data_ptr(), tl.ctensor.data_ptr(), tl.cstart.data_ptr(), tl.nchunks,
                     float(group["lr"]), float(group["weight_decay"]), float(b1), float(b2), float(group["eps"]),
                     step, ops._stream())
                for p in ps:            # written behind autograd's back: refresh the weight caches
                    torch.autograd.graph.increment_version(p)
        return loss
