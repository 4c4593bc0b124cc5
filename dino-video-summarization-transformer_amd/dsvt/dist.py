"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL ('nccl' backend on
ROCm = RCCL over xGMI) on the GPU, gloo for the CPU tests.

The DINO forward + loss has exactly ONE exchange per step: the sum of the teacher logits'
column sums for the center EMA (train_ssl.py:673-691, `dist.all_reduce(batch_center)` at
:686-688).  Everything else shards with no collective (weak scaling over clips; frame scoring
shards videos: replicas only)."""
import os

import torch
import torch.distributed as dist


def env_ranks():
    """(rank, world, local_rank) from the torch.distributed.run environment (1 process = 1 GPU)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(device=None, backend=None, timeout_s=None):
    """Initialise the default process group when WORLD_SIZE > 1 (env:// rendezvous; use
    MASTER_ADDR=127.0.0.1) -- utils/utils.py:437-469 of the reference.  backend defaults to
    'nccl' (RCCL over xGMI) for a GPU device, else gloo.  gloo on GPU tensors is the
    rehearsal mode for several ranks sharing one GPU (RCCL refuses duplicate devices)."""
    rank, world, _ = env_ranks()
    if world <= 1 or dist.is_initialized():
        return rank, world
    if backend is None:
        backend = "nccl" if device is not None and torch.device(device).type == "cuda" else "gloo"
    kw = {"device_id": torch.device(device)} if backend == "nccl" and device is not None else {}
    if timeout_s is not None:
        import datetime
        kw["timeout"] = datetime.timedelta(seconds=timeout_s)
    dist.init_process_group(backend, init_method="env://", **kw)
    if dist.get_world_size() != world:
        raise RuntimeError("process group has %d ranks, WORLD_SIZE says %d" % (dist.get_world_size(), world))
    return dist.get_rank(), dist.get_world_size()


def world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def center_batch_sum(colsum, rows):
    """All-reduce (sum, in place) the local teacher column sum [1, out_dim] over the ranks and
    return the EMA scale 1 / (rows * world) of train_ssl.py:688 (`batch_center /
    (len(teacher_output) * dist.get_world_size())`).  A no-op collective at world size 1."""
    world = world_size()
    if world > 1:
        dist.all_reduce(colsum)
    return 1.0 / (rows * world)


def backend():
    """The default process group's backend ('nccl' = RCCL, 'gloo'), or None at world size 1."""
    return dist.get_backend() if dist.is_available() and dist.is_initialized() else None


def max_over_ranks(value, device=None):
    """MAX of a host float over all ranks (bench timing: the slowest rank defines the step)."""
    if world_size() == 1:
        return float(value)
    if backend() == "gloo":
        device = None          # a host tensor: gloo reduces on the CPU anyway
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_range(n, rank, world):
    """Contiguous [lo, hi) share of n independent items (videos) for one rank; sizes differ by
    at most one and the shares tile [0, n) exactly."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


class BlockGradReducer:
    """Bucketed gradient all-reduce of the dsvt backbone, overlapped with its backward.

    The reference wraps the whole student in DDP (train_ssl.py:329), whose reducer all-reduces
    25 MB buckets as AccumulateGrad hooks fire during the backward.  The dsvt backbone backward
    is ONE autograd node (training.BackboneFn: all resolution groups, all blocks), so under plain
    DDP every backbone gradient becomes ready at once, at the very end, and ~86 M fp32 gradients
    are all-reduced after the compute instead of under it.  This reducer takes the backbone's
    parameters away from DDP (wrap_ddp: DDP keeps the DINO head) and lays their gradients out
    in one flat fp32 arena, one bucket per divided block (7.1 M values = 28 MB at ViT-B, DDP's
    bucket size) plus one for the embeddings and the final norm.  The backbone backward hands
    the arena views out as its gradient buffers and calls `launch(k)` as soon as block k's
    gradients are final (after the LAST resolution group's pass over it); the bucket's
    all-reduce is issued on the weight-gradient stream, so RCCL runs it while the dX chain of
    the blocks below continues.  `finish()` waits for all buckets (the averaging is RCCL's AVG;
    gloo sums and the arena is divided once).  Gradients equal DDP's: the bucket-wise average
    of the same fp32 per-rank gradients."""

    def __init__(self, backbone, group=None, ddp=None):
        self.bb, self.group, self.ddp = backbone, group, ddp
        self.world = dist.get_world_size(group)
        self.avg = dist.get_backend(group) == "nccl"
        self._works, self._arena, self._seeded = [], None, []
        self._local = False     # a no_sync backward left local sums in p.grad since the last sync
        backbone.dsvt_grad_reducer = self

    def params(self):
        """Backbone parameters that take gradients, per bucket: blocks 0..depth-1, then the rest."""
        buckets = [[p for p in blk.parameters() if p.requires_grad] for blk in self.bb.blocks]
        seen = {id(p) for b in buckets for p in b}
        buckets.append([p for p in self.bb.parameters() if p.requires_grad and id(p) not in seen])
        return buckets

    def active(self):
        """False inside DDP's no_sync() (gradient accumulation without communication)."""
        return self.ddp is None or getattr(self.ddp, "require_backward_grad_sync", True)

    def note_local(self):
        """Called for a backward inside no_sync(): the next synchronised arena seeds from p.grad."""
        self._local = True

    def arena(self, device):
        """A fresh flat fp32 arena for this backward (the returned views become p.grad), the
        id(p) -> view map the gradient buffers come from, and the ids of the views SEEDED with
        an existing p.grad.  Offsets are 256-byte aligned.

        Gradient accumulation (DDP.no_sync() micro-steps, then one synchronised step): the
        no_sync backwards leave LOCAL sums in p.grad.  DDP all-reduces the whole accumulated
        gradient on the sync step, so the arena starts from those sums (the backward then
        accumulates onto them) and the caller must REPLACE p.grad with the reduced view instead
        of letting autograd add it (`take_seeded`).  Only after such a no_sync backward
        (`note_local`): otherwise an existing p.grad (zeros left by zero_grad(set_to_none=False), a
        previous synchronised step's reduced sum) is already global, and autograd adds the reduced
        view onto it without an fp32 copy of every gradient through the arena."""
        buckets = self.params()
        sizes = [[(p.numel() + 63) // 64 * 64 for p in b] for b in buckets]
        flat = torch.empty(sum(sum(s) for s in sizes), device=device, dtype=torch.float32)
        views, self._slices, off = {}, [], 0
        self._seeded = []
        for b, s in zip(buckets, sizes):
            start = off
            for p, n in zip(b, s):
                v = flat[off:off + p.numel()].view(p.shape)
                views[id(p)] = v
                if self._local and p.grad is not None:
                    v.copy_(p.grad)
                    self._seeded.append(p)
                off += n
            self._slices.append(flat[start:off])
        self._arena, self._works, self._local = flat, [], False
        return views, {id(p) for p in self._seeded}

    def take_seeded(self):
        """Drop the accumulated p.grad of every seeded parameter (its sum is in the reduced
        arena view the backward returns, which autograd then installs as p.grad)."""
        for p in self._seeded:
            p.grad = None
        self._seeded = []

    def launch(self, k, side=None):
        """Start bucket k's all-reduce once everything queued so far (on the current stream and on
        `side`) has produced it; issued on `side` when given, so it overlaps the current stream."""
        buf = self._slices[k]
        if buf.numel() == 0:
            return
        op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
        if side is None:
            self._works.append(dist.all_reduce(buf, op=op, group=self.group, async_op=True))
            return
        side.wait_stream(torch.cuda.current_stream(buf.device))
        with torch.cuda.stream(side):
            self._works.append(dist.all_reduce(buf, op=op, group=self.group, async_op=True))

    def finish(self):
        """The current stream waits for every bucket; gloo's sums become averages."""
        for w in self._works:
            w.wait()
        if not self.avg and self._arena is not None:
            self._arena.div_(self.world)
        self._works, self._arena, self._slices = [], None, []


def wrap_ddp(student, device, overlap=True, **ddp_kw):
    """DDP over a MultiCropWrapper(dsvt backbone, head) the way train_ssl.py:329 does, with the
    backbone's gradients all-reduced bucket by bucket under its own backward (BlockGradReducer)
    when `overlap`; DDP then owns only the head's parameters.  The backbone's parameters and
    buffers are broadcast from rank 0 like DDP's own initial sync."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    ddp_kw.setdefault("broadcast_buffers", False)
    if device is not None and torch.device(device).type == "cuda":
        ddp_kw.setdefault("device_ids", [torch.device(device).index])
    bb = getattr(student, "backbone", None)
    if not overlap or bb is None or not hasattr(bb, "blocks"):
        return DDP(student, **ddp_kw)
    names = ["backbone." + n for n, _ in bb.named_parameters()] + ["backbone." + n for n, _ in bb.named_buffers()]
    DDP._set_params_and_buffers_to_ignore_for_model(student, names)
    with torch.no_grad():
        for t in list(bb.parameters()) + list(bb.buffers()):
            dist.broadcast(t.data, 0)
    ddp = DDP(student, **ddp_kw)
    BlockGradReducer(bb, ddp=ddp)
    return ddp
