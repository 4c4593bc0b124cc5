"""Drop-in for utils.utils.MultiCropWrapper (utils/utils.py:564-609), plus the concurrent
teacher/student forward of one DINO step."""
import os
import threading

import torch
import torch.nn as nn

_SIDE_STREAMS = {}
_SLOT_OF = {}          # cuda_stream handle of a side stream -> its slot
_FORK = threading.local()


def fork_depth():
    """How many run_concurrent forks the calling code runs inside (0 = none)."""
    return getattr(_FORK, "depth", 0)


def nested_capture_fork(device):
    """True when forking side streams from the current stream would be a NESTED fork inside a
    HIP-graph capture: the current stream is itself one of our side streams, forked from the
    capture's origin stream.  On this ROCm 7.2 / torch 2.10 stack a capture whose fork tree is
    two levels deep (origin -> side A -> side B, joined back B -> A -> origin) dies with a host
    segfault in capture_end even with no dsvt code in it (tools/capture_nested_min.py: plain
    torch elementwise ops, with or without allocations on B; one level -- origin -> A -> origin --
    captures and replays), so such a fork runs its items in order on the current stream instead."""
    return torch.cuda.is_current_stream_capturing() and torch.cuda.current_stream(device).cuda_stream in _SLOT_OF


def _slot_priority(slot):
    """DSVT_SIDE_PRIO="slot:prio,..." (A/B knob; integer slots only): HIP stream priority of a side
    stream (lower = higher priority; torch's range on this stack is -1 .. 0)."""
    import os
    spec = os.environ.get("DSVT_SIDE_PRIO")
    if not spec or not isinstance(slot, int):
        return 0
    for item in spec.split(","):
        k, v = item.split(":")
        if int(k) == slot:
            return int(v)
    return 0


def side_stream(device, slot):
    """A persistent non-default HIP stream per (device, slot), created on first use."""
    key = (torch.device(device), slot)
    st = _SIDE_STREAMS.get(key)
    if st is None:
        st = _SIDE_STREAMS[key] = torch.cuda.Stream(device=key[0], priority=_slot_priority(slot))
        _SLOT_OF[st.cuda_stream] = slot
    return st


def stream_slot(device):
    """The slot of the current stream if it is one of ours, else "main" (the default stream or
    a graph-capture stream): nested forks key their side streams on it, so the same streams
    serve eager warm-up and HIP-graph capture."""
    return _SLOT_OF.get(torch.cuda.current_stream(device).cuda_stream, "main")


def run_concurrent(thunks, device, slot0=0):
    """Run independent GPU work items on separate streams: thunk 0 on the current stream,
    thunk i on side stream slot0+i-1; every side stream first waits for the current
    stream's prior work, and the current stream waits for all of them before returning.
    Kernels of the different items then overlap on the chip (one backbone call's last,
    partly-filled wave of tiles runs beside another's full waves)."""
    if nested_capture_fork(device):         # see nested_capture_fork: in order, no fork
        return [fn() for fn in thunks]
    cur = torch.cuda.current_stream(device)
    results, used = [None] * len(thunks), []
    _FORK.depth = fork_depth() + 1
    try:
        for i, fn in enumerate(thunks):
            if i == 0:
                continue
            st = side_stream(device, slot0 + i - 1 if isinstance(slot0, int) else (slot0, i))
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                results[i] = fn()
            used.append(st)
        if thunks:
            results[0] = thunks[0]()
    finally:
        _FORK.depth -= 1
    for st in used:
        cur.wait_stream(st)
    for r in results:                      # outputs made on side streams are consumed on `cur`
        if isinstance(r, torch.Tensor) and r.is_cuda:
            r.record_stream(cur)
    return results


def prepare_weights(module):
    """Call prepare_weights() on every dsvt sub-module (storage-dtype weight copies produced
    on the current stream before work forks onto side streams)."""
    for m in module.modules():
        fn = getattr(m, "prepare_weights", None)
        if callable(fn):
            fn()


def dino_forward(student, teacher, images, n_global=2, concurrent=True):
    """train_ssl.py:523-527: teacher on the `n_global` global views, student on all views.
    The two networks are independent and their backbone calls run on concurrent streams."""
    if not concurrent:
        return student(images), teacher(images[:n_global])
    for net in (student, teacher):
        prepare_weights(net)
    s_out, t_out = run_concurrent([lambda: student(images), lambda: teacher(images[:n_global])],
                                  images[0].device, slot0=8)
    return s_out, t_out


def _inside_ddp():
    """True while a DistributedDataParallel forward is running this module."""
    try:
        from torch.nn.parallel import DistributedDataParallel as DDP
        return DDP._get_active_ddp_module() is not None
    except AttributeError:                      # pragma: no cover - older torch
        return True


class MultiCropWrapper(nn.Module):
    """Runs the backbone once per group of consecutive same-resolution crops and the head once
    on all features.  Unlike the reference it does not torch.cat the crops: the dsvt backbone
    takes the group as a list and writes every crop's tokens straight into one token tensor,
    and the features of all groups land in one preallocated buffer."""

    def __init__(self, backbone, head, vary_fr=False, concurrent_groups=True):
        super().__init__()
        self.concurrent_groups = concurrent_groups
        # training groups on separate streams: measured within noise of in-order (89.4 vs 90.2
        # clips/s, tools/train_step.py), so off by default
        self.concurrent_grad_groups = False
        if hasattr(backbone, 'fc'):
            backbone.fc, backbone.head = nn.Identity(), nn.Identity()
        self.backbone = backbone
        self.head = head
        self.vary_fr = vary_fr

    def forward(self, x, **kwargs):
        if not isinstance(x, list):
            x = [x]
        sizes = [inp.shape[-1] for inp in x]
        if self.vary_fr:                                   # utils/utils.py:588-592
            if len(x) == 10:
                idx_crops = [1, 2, 4, 6, 8, 10]
            elif len(x) == 2:
                idx_crops = [1, 2]
            else:
                raise ValueError("vary_fr supports 2 or 10 crops")
        else:                                              # unique_consecutive on widths (:584-587)
            idx_crops = []
            for i in range(1, len(sizes) + 1):
                if i == len(sizes) or sizes[i] != sizes[i - 1]:
                    idx_crops.append(i)
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            # training: autograd-tracked backbone calls, one per resolution group, in order (the
            # DropPath masks are drawn in that order).  Group i > 0 is launched on its own stream
            # when concurrent_grad_groups: autograd runs each group's backward on its forward's stream,
            # so the groups overlap in the backward as well
            if (len(idx_crops) > 1 and not kwargs and not self.concurrent_grad_groups
                    and hasattr(self.backbone, "forward_features_groups") and self.backbone._grad_path()):
                # dsvt: all groups through one autograd node (one set of gradient buffers)
                bounds = [0] + idx_crops
                feats = self.backbone.forward_features_groups([x[a:b] for a, b in zip(bounds[:-1], bounds[1:])])
                return self.head(feats)
            outs, start = [], 0
            cur = torch.cuda.current_stream(x[0].device) if x[0].is_cuda else None
            # DDP's reducer hooks stay bound to the stream its AccumulateGrad nodes were made on:
            # a group whose backward runs on a side stream hands it gradients before they are
            # complete (measured 0.24 relative error), so under DDP the groups run in order
            fork = self.concurrent_grad_groups and cur is not None and not _inside_ddp()
            used = []
            for gi, end in enumerate(idx_crops):
                group = x[start:end]

                def fwd(group=group):
                    if getattr(self.backbone, "takes_clip_lists", False):
                        return self.backbone.forward_features(group, **kwargs)
                    return self.backbone(torch.cat(group), **kwargs)
                if gi > 0 and fork:
                    st = side_stream(x[0].device, ("group", stream_slot(x[0].device), gi))
                    st.wait_stream(cur)
                    with torch.cuda.stream(st):
                        out = fwd()
                    used.append(st)
                    outs.append(out)
                else:
                    outs.append(fwd())
                start = end
            for st in used:
                cur.wait_stream(st)
            if used:
                for o in outs:
                    o.record_stream(cur)
            return self.head(torch.cat(outs) if len(outs) > 1 else outs[0])
        total = sum(inp.shape[0] for inp in x)
        # num_features: the backbone's output width (a Swin's is embed_dim * 2^(stages - 1))
        feats = torch.empty(total, getattr(self.backbone, "num_features", self.backbone.embed_dim), device=x[0].device,
                            dtype=torch.float32)
        jobs, start, row = [], 0, 0
        for end in idx_crops:
            group = x[start:end]
            n = sum(g.shape[0] for g in group)
            jobs.append((group, feats[row:row + n]))
            row += n
            start = end

        list_input = getattr(self.backbone, "takes_clip_lists", False)

        def job(group, out):
            if list_input:   # dsvt TimeSformer: the group's clips go in as a list (no cat copy)
                return lambda: self.backbone.forward_features(group, out=out, **kwargs)
            return lambda: out.copy_(self.backbone(torch.cat(group), **kwargs))   # utils.py:601
        thunks = [job(g, o) for g, o in jobs]
        if self.concurrent_groups and len(thunks) > 1 and feats.is_cuda:
            prepare_weights(self.backbone)            # weight copies made before the fork
            run_concurrent(thunks, feats.device)      # the resolution groups are independent
        else:
            for fn in thunks:
                fn()
        return self.head(feats)


# ---------------------------------------------------------------- training-step utilities
_TLISTS = {}      # tensor-list shape (device, numels) -> TensorList (size / chunk tables)
_TPTRS = {}       # (device, data pointers) -> device pointer table


def _tensor_list(tensors):
    """Cached device tables for a list of fp32 GPU tensors: (TensorList of its shape, pointer
    table).  Gradients are new buffers every step, so only their pointer table is rebuilt (one
    pinned, non-blocking copy); the shape tables are built once."""
    from .training import TensorList, check_fp32_contiguous
    check_fp32_contiguous(tensors, "multi-tensor op")
    dev = tensors[0].device
    skey = (dev, tuple(t.numel() for t in tensors))
    tl = _TLISTS.get(skey)
    if tl is None:
        tl = _TLISTS[skey] = TensorList(tensors, dev)
        if len(_TLISTS) > 64:
            _TLISTS.pop(next(iter(_TLISTS)))
    pkey = (dev, tuple(t.data_ptr() for t in tensors))
    ptr = _TPTRS.get(pkey)
    if ptr is None:
        ptr = _TPTRS[pkey] = TensorList.ptrs(tensors, dev)
        if len(_TPTRS) > 64:
            _TPTRS.pop(next(iter(_TPTRS)))
    return tl, ptr


def ema_update_(teacher_tensors, student_tensors, momentum):
    """teacher = m * teacher + (1 - m) * student over whole tensor lists in ONE launch
    (train_ssl.py:555-558 loops param by param)."""
    from . import ops
    from ._lib import call
    teacher_tensors = list(teacher_tensors)
    tl, tptr = _tensor_list(teacher_tensors)
    _, sptr = _tensor_list(list(student_tensors))
    call("dsvt_ema", tptr.data_ptr(), sptr.data_ptr(), tl.sizes.data_ptr(), tl.ctensor.data_ptr(),
         tl.cstart.data_ptr(), tl.nchunks, float(momentum), ops._stream())
    for t in teacher_tensors:   # written behind autograd's back: bump the version counters so the
        torch.autograd.graph.increment_version(t)   # storage-dtype weight caches refresh


def clip_gradients_(grads, clip):
    """utils/utils.py:102-111 per-tensor clipping (clip_coef = clip / (norm + 1e-6), applied when
    < 1) over a gradient list in three launches, no host sync; returns the norms (device)."""
    from . import ops
    from ._lib import call
    grads = list(grads)
    tl, gptr = _tensor_list(grads)
    norms = torch.empty(tl.ntensors, device=tl.sizes.device, dtype=torch.float32)
    ws = torch.empty(tl.nchunks, device=tl.sizes.device, dtype=torch.float32)
    call("dsvt_clip_grads", gptr.data_ptr(), tl.sizes.data_ptr(), tl.ctensor.data_ptr(), tl.cstart.data_ptr(),
         tl.first.data_ptr(), tl.nchunks, tl.ntensors, float(clip), norms.data_ptr(), ws.data_ptr(),
         ws.numel() * 4, ops._stream())
    return norms


def clip_gradients(model, clip):
    """utils/utils.py:102-111: returns the per-parameter gradient norms (a device tensor here;
    the reference returns a list of Python floats after one .item() sync per parameter)."""
    grads = [p.grad for p in model.parameters() if p.grad is not None]
    if not grads:
        return []
    return clip_gradients_(grads, clip)


def cancel_gradients_last_layer(epoch, model, freeze_last_layer):
    """utils/utils.py:114-119."""
    if epoch >= freeze_last_layer:
        return
    for n, p in model.named_parameters():
        if "last_layer" in n:
            p.grad = None


def get_params_groups(model):
    """utils/utils.py:612-623: no weight decay on biases and norm parameters."""
    regularized, not_regularized = [], []
    for name, param in model.named_parameters():
        if not param.requires_grad:
            continue
        if name.endswith(".bias") or len(param.shape) == 1:
            not_regularized.append(param)
        else:
            regularized.append(param)
    return [{'params': regularized}, {'params': not_regularized, 'weight_decay': 0.}]


def cosine_scheduler(base_value, final_value, epochs, niter_per_ep, warmup_epochs=0, start_warmup_value=0):
    """utils/utils.py:157-168."""
    from .training import np_cosine_scheduler
    return np_cosine_scheduler(base_value, final_value, epochs, niter_per_ep, warmup_epochs, start_warmup_value)
