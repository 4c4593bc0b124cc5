"""N > 1 data-parallel path on the CPU: gloo, world_size 2, one process per rank (the GPU runs
the same code over RCCL).  Covers dsvt.dist (incl. the overlapped per-block gradient buckets
of wrap_ddp / BlockGradReducer) and the product's dsvt.loss.DINOLoss.update_center
(the center column-sum all-reduce of train_ssl.py:673-691), the trainer's world-size lr
scaling, the bench's max-over-ranks timing, and the video sharding of frame scoring.
The GPU leg (DDP gradients through the HIP backward) is tests/test_gpu_dist.py."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dino-video-summarization-transformer_amd")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, errq):
    try:
        for p in (ROOT, PKG):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        import torch
        import torch.distributed as dist

        from dsvt import dist as ddist
        from oracle import dsvt_oracle as O

        r, w = ddist.init_from_env()                       # no device -> gloo
        assert (r, w) == (rank, world) and dist.get_backend() == "gloo"

        # one global batch of B_all clips, sharded over the ranks; D = out_dim
        B_all, D, ncrops, temp = 4, 64, 4, 0.04
        rng = np.random.default_rng(7)
        teacher = rng.standard_normal((2 * B_all, D)).astype(np.float32)   # [2 crops x B_all]
        student = rng.standard_normal((ncrops * B_all, D)).astype(np.float32)
        center = (0.1 * rng.standard_normal((1, D))).astype(np.float32)
        lo, hi = ddist.shard_range(B_all, rank, world)
        t_loc = np.concatenate([teacher[c * B_all + lo:c * B_all + hi] for c in range(2)])
        s_loc = np.concatenate([student[c * B_all + lo:c * B_all + hi] for c in range(ncrops)])

        # the product's DINOLoss.update_center on the rank's local column sum: the all-reduce and
        # the 1/(rows*world) scale run as shipped; only the center-EMA kernel launch (a GPU op,
        # csrc/dino_loss.hip) is replaced by its host arithmetic for this CPU test
        from dsvt import loss as dloss
        from dsvt import ops

        def center_ema_host(c, colsum, momentum, inv_count):
            c.mul_(momentum).add_(colsum.reshape(c.shape) * (inv_count * (1.0 - momentum)))
        ops.center_ema = center_ema_host
        lf = dloss.DINOLoss(D, ncrops, temp, temp, 0, 10)
        lf.center.copy_(torch.from_numpy(center))
        colsum = torch.from_numpy(t_loc.sum(0, keepdims=True))
        lf.update_center(colsum, t_loc.shape[0])
        c_dp = lf.center.numpy()
        _, c_full = O.dino_loss(student, teacher, center, ncrops, temp)   # single process, whole batch
        np.testing.assert_allclose(c_dp, c_full, rtol=1e-5, atol=1e-7)
        assert ddist.center_batch_sum(torch.zeros(1, D), t_loc.shape[0]) == pytest.approx(1.0 / (t_loc.shape[0] * world))
        # the oracle's own DP restatement agrees as well
        _, c_or = O.dino_loss(s_loc, t_loc, center, ncrops, temp, world_size=world, teacher_sum_all=colsum.numpy())
        np.testing.assert_allclose(c_or, c_full, rtol=1e-5, atol=1e-7)
        # DINOTrainer's linear lr scaling uses the world size (train_ssl.py:395-400)
        from dsvt.trainer import DINOTrainer
        net = torch.nn.Linear(4, 4)
        tr = DINOTrainer(net, torch.nn.Linear(4, 4), lf, lr=5e-4, epochs=2, niter_per_ep=3, warmup_epochs=1,
                         batch_size_per_gpu=8)
        assert tr.peak_lr == pytest.approx(5e-4 * 8 * world / 256.0)
        # every rank ends with the identical center (train_ssl.py: teacher stays in sync)
        got = [torch.zeros(1, D) for _ in range(world)]
        dist.all_gather(got, torch.from_numpy(c_dp))
        for g in got[1:]:
            assert torch.equal(g, got[0])

        # dist.wrap_ddp + BlockGradReducer (the overlapped per-block gradient buckets): initial
        # weights broadcast from rank 0, the backbone's parameters kept from DDP, buckets laid out
        # per block in one 256-B aligned arena and averaged bucket by bucket in any launch order
        class _Blk(torch.nn.Module):
            def __init__(self, seed):
                super().__init__()
                g = torch.Generator().manual_seed(seed)
                self.fc = torch.nn.Linear(6, 5)
                self.norm = torch.nn.LayerNorm(5)
                with torch.no_grad():
                    self.fc.weight.copy_(torch.randn(5, 6, generator=g))

        class _BB(torch.nn.Module):
            def __init__(self, seed):
                super().__init__()
                self.blocks = torch.nn.ModuleList([_Blk(seed + i) for i in range(3)])
                self.cls_token = torch.nn.Parameter(torch.full((1, 1, 5), float(seed)))

        class _MC(torch.nn.Module):
            def __init__(self, seed):
                super().__init__()
                self.backbone, self.head = _BB(seed), torch.nn.Linear(5, 3)

            def forward(self, x):
                return self.head(x)

        mc = _MC(100 + 10 * rank)                          # ranks start from different weights
        ddp = ddist.wrap_ddp(mc, None)
        red = mc.backbone.dsvt_grad_reducer
        assert red.ddp is ddp and red.active()
        assert torch.all(mc.backbone.cls_token == 100.0)    # rank 0's weights everywhere
        assert "backbone.blocks.0.fc.weight" in mc._ddp_params_and_buffers_to_ignore
        assert "head.weight" not in mc._ddp_params_and_buffers_to_ignore
        buckets = red.params()
        assert [len(b) for b in buckets] == [4, 4, 4, 1]
        views, seeded = red.arena(torch.device("cpu"))
        assert not seeded                                  # no accumulated p.grad yet
        for i, b in enumerate(buckets):
            for p in b:
                v = views[id(p)]
                assert v.shape == p.shape and (v.data_ptr() - red._arena.data_ptr()) % 256 == 0
                v.fill_(float(rank + 1) * (1 + i))
        for k in (3, 1, 0, 2):
            red.launch(k)
        red.finish()
        for i, b in enumerate(buckets):
            for p in b:                                   # mean over ranks of (rank + 1) * (i + 1)
                assert torch.allclose(views[id(p)], torch.full(p.shape, (i + 1) * (world + 1) / 2.0))
        ddp.require_backward_grad_sync = False             # DDP.no_sync(): no bucket traffic
        assert not red.active()
        # gradient accumulation: a no_sync micro-step leaves LOCAL sums in p.grad; the next
        # synchronised backward must all-reduce the accumulated total (DDP's semantics), so the
        # arena starts from p.grad and the reduced view replaces it (take_seeded)
        for i, b in enumerate(buckets):
            for p in b:
                p.grad = torch.full(p.shape, 10.0 * (rank + 1) + i)
        ddp.require_backward_grad_sync = True
        # an existing p.grad WITHOUT a no_sync backward before (zero_grad(set_to_none=False), a
        # previous synchronised step) is already global: not seeded, autograd adds onto it
        views, seeded = red.arena(torch.device("cpu"))
        assert not seeded
        red.note_local()                                   # what the no_sync backward records
        views, seeded = red.arena(torch.device("cpu"))
        assert seeded == {id(p) for b in buckets for p in b}
        for i, b in enumerate(buckets):
            for p in b:
                views[id(p)].add_(float(rank + 1))         # this micro-step's local gradient
        for k in range(len(buckets)):
            red.launch(k)
        red.finish()
        red.take_seeded()
        for i, b in enumerate(buckets):
            for p in b:                                   # mean over ranks of 11 (rank + 1) + i
                assert p.grad is None
                want = 11.0 * (world + 1) / 2.0 + i
                assert torch.allclose(views[id(p)], torch.full(p.shape, want)), (views[id(p)].flatten()[0], want)

        # bench: elapsed = MAX over ranks
        assert ddist.max_over_ranks(1.5 + rank) == pytest.approx(1.5 + world - 1)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # report to the parent; a hung peer is caught by the join timeout
        errq.put("rank %d: %r" % (rank, e))
        raise


def test_center_allreduce_and_timing_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not alive, "rank(s) hung"
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_world1_is_collective_free():
    from dsvt import dist as ddist
    import torch
    c = torch.ones(1, 8)
    assert ddist.world_size() == 1
    assert ddist.center_batch_sum(c, 4) == pytest.approx(0.25)
    assert torch.equal(c, torch.ones(1, 8))
    assert ddist.max_over_ranks(3.25) == 3.25


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 2), (64, 8), (5, 8), (1000, 3)])
def test_shard_range_tiles_exactly(n, world):
    from dsvt import dist as ddist
    spans = [ddist.shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1
