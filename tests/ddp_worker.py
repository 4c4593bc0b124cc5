"""One rank of the data-parallel DINO step test (tests/test_gpu_dist.py starts two of these).

The reference's config-3 data path (train_ssl.py:329 DDP wrap, :523-545 forward / loss /
backward, :686-688 center all-reduce, utils/utils.py:437-469 process-group init) on dsvt:
DDP(MultiCropWrapper(dsvt TimeSformer, DINOHead)) -> dsvt.loss.DINOLoss -> backward, each rank
on its half of the clips.  RCCL refuses two ranks on one GPU, so the two ranks share the box's
GPU over gloo (same DDP reducer, same bucketed all-reduce code path; only the transport
differs).  Rank 0 then re-runs the same step in one process on the WHOLE batch and checks the
all-reduced gradients, the loss and the center against it (fp32 parity mode, 1e-3 relative
to max |ref| per tensor) -- once with the backbone's gradients on DDP's own reducer and once on
dsvt.dist.wrap_ddp's per-block buckets overlapped with the backbone backward -- and both ranks check they hold bitwise-identical gradients.  A second
phase runs dsvt.trainer.DINOTrainer.step (clip + AdamW + EMA) under DDP and checks the student
and teacher parameters stay identical across the ranks.

Writes {"ok": bool, "msg": str, ...} to $DSVT_TEST_OUT.  Run by the test only.
"""
import json
import os
import sys
import traceback
from functools import partial

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "dino-video-summarization-transformer_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402

from oracle import params as P  # noqa: E402

# DSVT_DDP_CFG=tiny (default): a 64-wide depth-2 model, 4 clips of 2 x 4x64^2 + 2 x 4x32^2 crops.
# DSVT_DDP_CFG=vitb: ViT-B widths (embed 768, 12 heads, depth 2) on 2 clips of 2 x 8x224^2 +
# 2 x 8x96^2 crops, DINOHead(768 -> 2048 -> 256 -> 4096): the per-block gradient buckets of
# dist.BlockGradReducer at their real sizes (7.1 M values = 28 MB per block) and launch order
# under the real backward.
SIZE = os.environ.get("DSVT_DDP_CFG", "tiny")
if SIZE == "vitb":
    CFG = dict(embed_dim=768, num_heads=12, depth=2, img_size=224, num_frames=8)
    HEAD = dict(hidden_dim=2048, bottleneck_dim=256)
    OUT_DIM, B_ALL, NCROPS, T, G_SZ, L_SZ = 4096, 2, 4, 8, 224, 96
else:
    CFG = dict(embed_dim=64, num_heads=1, depth=2, img_size=64, num_frames=4)
    HEAD = dict(hidden_dim=128, bottleneck_dim=64)
    OUT_DIM, B_ALL, NCROPS, T, G_SZ, L_SZ = 512, 4, 4, 4, 64, 32
TOL = 1e-3


def build(seed_bb, seed_hd, use_bn=False):
    from dsvt.models.timesformer import VisionTransformer
    from dsvt.utils import MultiCropWrapper
    from dsvt.vision_transformer import DINOHead
    E = CFG["embed_dim"]
    bb = VisionTransformer(img_size=CFG["img_size"], patch_size=16, num_classes=0, embed_dim=E, depth=CFG["depth"],
                           num_heads=CFG["num_heads"], mlp_ratio=4, qkv_bias=True,
                           norm_layer=partial(nn.LayerNorm, eps=1e-6), drop_path_rate=0.0,
                           num_frames=CFG["num_frames"], attention_type="divided_space_time")
    bb.load_state_dict({k: torch.from_numpy(v) for k, v in P.timesformer_state(seed_bb, **CFG).items()})
    hd = DINOHead(E, OUT_DIM, use_bn=use_bn, **HEAD)
    sd = P.dino_head_bn_state(seed_hd, E, OUT_DIM, **HEAD) if use_bn else P.dino_head_state(seed_hd, E, OUT_DIM, **HEAD)
    hd.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    bb.dsvt_dtype = hd.dsvt_dtype = torch.float32
    return MultiCropWrapper(bb, hd).cuda()


def crops_all():
    """The whole batch: 2 global and 2 local crops of B_ALL clips."""
    return [P.clip(3100 + i, (B_ALL, 3, T, G_SZ, G_SZ)) for i in range(2)] + \
           [P.clip(3110 + i, (B_ALL, 3, T, L_SZ, L_SZ)) for i in range(2)]


def make_loss(center0):
    from dsvt.loss import DINOLoss
    lf = DINOLoss(OUT_DIM, NCROPS, 0.04, 0.04, 0, 10, student_temp=0.1, global_crops=2).cuda()
    lf.center.copy_(torch.from_numpy(center0))
    return lf


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-12))


_LOG = [None]


def log(msg):
    if _LOG[0] is not None:
        _LOG[0].write(msg + "\n")
        _LOG[0].flush()


def main():
    from dsvt import dist as ddist
    rank, world, _ = ddist.env_ranks()
    if os.environ.get("DSVT_TEST_LOGDIR"):
        _LOG[0] = open(os.path.join(os.environ["DSVT_TEST_LOGDIR"], "ddp_rank%d.log" % rank), "w")
    log("start")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    r, w = ddist.init_from_env(dev, backend="gloo", timeout_s=60)
    log("process group up")
    assert (r, w) == (rank, world) and world == 2, (r, w)
    info = {"rank": rank, "world": world, "backend": dist.get_backend()}

    center0 = (0.1 * P.clip(3120, (1, OUT_DIM))).astype(np.float32)
    full = crops_all()
    lo, hi = ddist.shard_range(B_ALL, rank, world)
    mine = [torch.from_numpy(c[lo:hi].copy()).to(dev) for c in full]

    # ---- phase 1: DDP gradients + center vs the single-process whole batch, with the backbone's
    # gradients on DDP's reducer (plain DDP) and on the overlapped per-block buckets (wrap_ddp)
    results = {}
    # *_accum: gradient accumulation -- one micro-step under DDP.no_sync() (local sums only),
    # then a synchronised one; DDP averages the ACCUMULATED gradient (the overlapped
    # buckets must reduce the no_sync sums too, dist.BlockGradReducer.arena seeding)
    # ddp_syncbn: DINOHead(use_bn=True) converted to SyncBatchNorm as train_ssl.py:319-321 does
    # (--use_bn_in_head): batch statistics over both ranks, and LOCAL weight / bias gradients that
    # DDP averages (torch's SyncBatchNorm semantics; ADVICE r04: dgamma / dbeta came out world_size
    # times too large when taken from the all-reduced sums)
    modes = ("ddp", "overlap", "overlap_1stream", "ddp_accum", "overlap_accum") + \
        (("ddp_syncbn",) if SIZE == "tiny" else ())
    bn_bufs = None
    for mode in modes:
        student = build(4101, 4102, use_bn=mode == "ddp_syncbn").train()
        if mode == "ddp_syncbn":
            student = nn.SyncBatchNorm.convert_sync_batchnorm(student)
            assert any(isinstance(m, nn.SyncBatchNorm) for m in student.head.modules())
        teacher = build(4201, 4202).eval()
        for p in teacher.parameters():
            p.requires_grad_(False)
        log("models built (%s)" % mode)
        if mode.startswith("ddp"):
            ddp = torch.nn.parallel.DistributedDataParallel(student, device_ids=[0], broadcast_buffers=False)
        else:
            ddp = ddist.wrap_ddp(student, dev)
            assert student.backbone.dsvt_grad_reducer is not None
            if mode == "overlap_1stream":                  # weight gradients and buckets on one stream
                student.backbone.dsvt_wgrad_stream = False
        log("ddp wrapped")
        loss_fn = make_loss(center0)
        if mode.endswith("_accum"):                         # micro-step 1: no gradient traffic
            with ddp.no_sync():
                s0 = ddp(mine)
                with torch.no_grad():
                    t0 = teacher(mine[:2])
                loss_fn(s0, t0, 0).backward()
            log("no_sync micro-step done")
        s_out = ddp(mine)                                   # train_ssl.py:523
        with torch.no_grad():
            t_out = teacher(mine[:2])                       # :527
        loss = loss_fn(s_out, t_out, 0)                     # center all-reduce inside (update_center)
        log("forward + loss done")
        loss.backward()                                     # bucketed gradient all-reduce
        log("backward done")
        torch.cuda.synchronize()
        names = [n for n, p in student.named_parameters() if p.requires_grad]
        grads = {n: p.grad.detach().float().cpu().numpy() for n, p in student.named_parameters() if p.requires_grad}
        missing = [n for n in names if student.get_parameter(n).grad is None]
        assert not missing, "no gradient for %s (%s)" % (missing, mode)
        flat = torch.cat([torch.from_numpy(grads[n]).reshape(-1) for n in names])
        peers = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(peers, flat)
        assert all(torch.equal(peers[0], x) for x in peers[1:]), "ranks hold different averaged gradients (%s)" % mode
        loss_sum = torch.tensor([float(loss.item())], dtype=torch.float64)
        dist.all_reduce(loss_sum)
        results[mode] = (grads, loss_sum, loss_fn.center.detach().cpu().numpy())
        if mode == "ddp_syncbn":
            bn_bufs = {n: b.detach().cpu().numpy().copy() for n, b in student.head.named_buffers()
                       if b.dtype != torch.int64}
        info["n_params"] = len(names)
        del ddp, student
    log("phase 1 collectives done")
    if rank == 0:
        from dsvt import ops
        allc = [torch.from_numpy(c).to(dev) for c in full]
        if "ddp_syncbn" in results:        # single process, whole batch, plain BatchNorm1d head
            ref = build(4101, 4102, use_bn=True).train()
            lf = make_loss(center0)
            lf.defer_center_update = True
            so = ref(allc)
            with torch.no_grad():
                to = teacher(allc[:2])
            loss_r = lf(so, to, 0)
            colsum, rows = lf.last_colsum
            ops.center_ema(lf.center, colsum, lf.center_momentum, 1.0 / rows)
            loss_r.backward()
            torch.cuda.synchronize()
            g_bn = {n: p.grad.cpu().numpy().copy() for n, p in ref.named_parameters() if p.requires_grad}
            l_bn, c_bn = loss_r, lf.center.cpu().numpy().copy()
            for n, b in ref.head.named_buffers():
                if n in bn_bufs:
                    info["bn_buf_err_" + n] = e = rel(bn_bufs[n], b.cpu().numpy())
                    assert e < 1e-4, "SyncBatchNorm running statistic %s: %.3g" % (n, e)
            del ref, lf
        ref = build(4101, 4102).train()
        lf = make_loss(center0)
        lf.defer_center_update = True      # a single process: its center update has no all-reduce

        def ref_step():
            so = ref(allc)
            with torch.no_grad():
                to = teacher(allc[:2])
            loss_r = lf(so, to, 0)
            colsum, rows = lf.last_colsum
            ops.center_ema(lf.center, colsum, lf.center_momentum, 1.0 / rows)
            loss_r.backward()
            return loss_r
        l_ref = ref_step()
        torch.cuda.synchronize()
        g_one = {n: p.grad.cpu().numpy().copy() for n, p in ref.named_parameters() if p.requires_grad}
        c_one = lf.center.cpu().numpy().copy()
        l_acc = ref_step()                 # accumulated onto the first step's gradients
        torch.cuda.synchronize()
        g_acc = {n: p.grad.cpu().numpy().copy() for n, p in ref.named_parameters() if p.requires_grad}
        c_acc = lf.center.cpu().numpy().copy()
        for mode, (grads, loss_sum, center_dp) in results.items():
            accum = mode.endswith("_accum")
            ref_g = g_bn if mode == "ddp_syncbn" else g_acc if accum else g_one
            errs = {n: rel(grads[n], ref_g[n]) for n in ref_g}
            if mode == "ddp_syncbn":
                # a train-mode BatchNorm removes any shift common to the batch, so the gradients of
                # the biases in front of it (the final-norm bias, the hidden Linears' biases) are
                # zero analytically -- rounding noise in both runs: checked against the gradient scale
                scale = max(float(np.abs(g).max()) for g in ref_g.values())
                for n in ref_g:
                    if float(np.abs(ref_g[n]).max()) < 1e-5 * scale:
                        errs[n] = float(np.abs(grads[n] - ref_g[n]).max()) / scale
            worst = max(errs, key=errs.get)
            info["worst_grad_" + mode] = [worst, errs[worst]]
            info["top_" + mode] = sorted(errs.items(), key=lambda kv: -kv[1])[:6]
            base = "ddp_accum" if accum else "ddp"
            if mode != base and mode != "ddp_syncbn":
                info["vs_ddp_" + mode] = max(rel(grads[n], results[base][0][n]) for n in grads)
        for mode, (grads, loss_sum, center_dp) in results.items():
            accum = mode.endswith("_accum")
            worst = info["worst_grad_" + mode][0]
            assert info["worst_grad_" + mode][1] < TOL, "%s grad %s rel err %.3g vs single-process full batch: %s" % (
                mode, worst, info["worst_grad_" + mode][1], info)
            l_mean = float(loss_sum.item()) / world
            lr_ = l_bn if mode == "ddp_syncbn" else l_acc if accum else l_ref
            info["loss_" + mode] = [l_mean, float(lr_.item())]
            assert abs(l_mean - float(lr_.item())) < TOL * abs(float(lr_.item())), info["loss_" + mode]
            ec = rel(center_dp, c_bn if mode == "ddp_syncbn" else c_acc if accum else c_one)
            info["center_err_" + mode] = ec
            assert ec < 1e-5, "center after the all-reduced update differs (%s): %.3g" % (mode, ec)
        del ref, lf
    dist.barrier()

    # ---- phase 2: whole training steps under DDP stay in sync across ranks
    if SIZE != "tiny":
        dist.destroy_process_group()
        return info
    from dsvt.trainer import DINOTrainer
    student = build(4101, 4102).train()
    teacher = build(4101, 4102).eval()
    ddp = ddist.wrap_ddp(student, dev)                 # the bench's wrapping (overlapped backbone buckets)
    tr = DINOTrainer(student, teacher, make_loss(center0), ddp=ddp, epochs=2, niter_per_ep=4, warmup_epochs=1,
                     batch_size_per_gpu=hi - lo, world_size=world)
    for it in (3, 4):                                  # it 3: last layer frozen (epoch 0); it 4: epoch 1
        tr.step(mine, it)
        log("trainer step %d done" % it)
    torch.cuda.synchronize()
    for tag, net in (("student", student), ("teacher", teacher)):
        flat = torch.cat([p.detach().float().reshape(-1).cpu() for p in net.parameters()])
        assert torch.isfinite(flat).all(), tag
        peers = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(peers, flat)
        assert all(torch.equal(peers[0], x) for x in peers[1:]), "%s parameters diverged across ranks" % tag
    dist.barrier()
    dist.destroy_process_group()
    return info


if __name__ == "__main__":
    out = os.environ["DSVT_TEST_OUT"]
    try:
        res = main()
        res["ok"] = True
        res["msg"] = "ok"
    except BaseException as e:  # noqa: BLE001 -- reported to the parent test
        res = {"ok": False, "msg": "%r\n%s" % (e, traceback.format_exc())}
    log("result: %s" % res["msg"][:2000])
    with open(out, "w") as f:
        json.dump(res, f)
    sys.exit(0 if res["ok"] else 1)
