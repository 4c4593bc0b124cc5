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
