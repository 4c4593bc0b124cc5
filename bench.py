#!/usr/bin/env python3
"""bench.py -- DINO-SVT forward + loss throughput on MI355X (BASELINE.json metric).

One STEP = the DINO fwd+loss of `--clips` multi-crop video clips per GPU (config 2):
  teacher: ViT-B/16 divided-ST backbone on the 2 global 8x224^2 crops of every clip,
  student: the same backbone architecture (own weights) on 2 global + 6 local 8x96^2 crops
           (MultiCropWrapper: one call per resolution group),
  DINOHead(768 -> 65536) on both, DINOLoss(ncrops=8) incl. the center update, whose teacher
  column sum is all-reduced over RCCL when N > 1.
value = clips/s over ALL ranks (weak scaling: `--clips` per GPU), inputs resident in HBM.

Usage:  python bench.py [--gpus N --steps K --warmup W]
        (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "dino-video-summarization-transformer_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "clips/sec (8-frame 224², ViT-B/16 DINO fwd+loss) at 1/2/4/8 MI355X; % MFMA roofline"
PEAK_TFLOPS = {"bf16": 2516.6, "f32": 157.3}   # dense, MI355X_MICROARCH.md chip table (2.4 GHz)
HBM_PEAK_GBS = 8000.0                          # HBM3E, MI355X_MICROARCH.md
IMAGENET_MEAN = (0.45, 0.45, 0.45)             # DATA.MEAN / STD defaults of the reference loader
IMAGENET_STD = (0.225, 0.225, 0.225)


# ----------------------------------------------------------------- algorithmic FLOPs
def vit_fwd_flops(T, S, C=768, depth=12, heads=12, mlp=4, patch=16, folded=False, cls_tail=False):
    """2*M*N*K over every matmul of one divided-ST clip forward, counted as the reference
    executes it (CLS replicated T times in the spatial branch).  8x224^2: 391.7 GFLOP,
    8x96^2: 70.7 GFLOP (391.66 / 70.70 from torch.utils.flop_counter).
    folded=True: what dsvt executes -- temporal proj and temporal_fc folded into one GEMM
    (VisionTransformer.fold_temporal_fc), i.e. one 2*R*C*C GEMM less per block.
    cls_tail=True: also what dsvt executes for a CLS-only forward (VisionTransformer.cls_tail):
    the last block's spatial queries and attention for the CLS rows only, attn.proj and the MLP
    on the CLS row only (Block._run_cls_tail)."""
    N = (S // patch) ** 2
    d = C // heads
    R = N * T
    rows_s = T * (1 + N)
    L = 1 + N * T
    per_block = (2 * R * C * 3 * C + 4 * N * heads * T * T * d + 2 * 2 * R * C * C          # temporal
                 + 2 * rows_s * C * 3 * C + 4 * T * heads * (1 + N) ** 2 * d + 2 * rows_s * C * C  # spatial
                 + 2 * 2 * L * C * mlp * C)                                                  # MLP
    if folded:
        per_block -= 2 * R * C * C
    tail = 0
    if cls_tail:   # last block: no patch-row queries, no patch-row proj / MLP
        tail = (4 * T * heads * (1 + N) * N * d + 2 * (rows_s - 1) * C * C + 2 * 2 * (L - 1) * C * mlp * C
                + 2 * (rows_s - 1) * C * C)                                      # + the patch rows' queries
    return depth * per_block - tail + 2 * R * (3 * patch * patch) * C


def head_flops(in_dim=768, hidden=2048, bottleneck=256, out_dim=65536):
    return 2 * (in_dim * hidden + hidden * hidden + hidden * bottleneck + bottleneck * out_dim)


def clip_flops(n_global=2, n_local=6, folded=False, cls_tail=False):
    """teacher (2 global) + student (2 global + 6 local) + heads on every crop row."""
    g = vit_fwd_flops(8, 224, folded=folded, cls_tail=cls_tail)
    l = vit_fwd_flops(8, 96, folded=folded, cls_tail=cls_tail)
    return 2 * n_global * g + n_local * l + (2 * n_global + n_local) * head_flops()


# ----------------------------------------------------------------- CPU baseline (oracle)
def host_cpu():
    """(model name, usable cores): the CPU model from /proc/cpuinfo (lscpu's "Model name"), and
    the cores this process may use -- its affinity mask, capped by the cgroup CPU quota."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:  # pragma: no cover
        pass
    cores = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            cores = max(1, min(cores, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return model, cores


def cpu_baseline(batches=(1, 4), reps=5):
    """The reference's own execution model on the host: eager torch fp32 on CPU, restated op
    for op in oracle/torch_cpu.py (the checker, pinned to the reference's golden vectors; never
    the product).  One DINO fwd+loss step of `b` multi-crop clips as the reference runs it
    (train_ssl.py:523-530: student on the 2b global + 6b local crops, one call per resolution
    group; teacher on the 2b global crops; DINOHead(65536) on every row; DINOLoss ncrops 8),
    1 warm-up + median of `reps`, torch.set_num_threads(usable cores)."""
    from oracle import params as P
    from oracle import torch_cpu as TC
    model, cores = host_cpu()
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    try:
        student, teacher = TC.TimeSformerCPU(P.timesformer_state(11), 12), TC.TimeSformerCPU(P.timesformer_state(12), 12)
        head_s = TC.DINOHeadCPU(P.dino_head_state(13, 768, 65536))
        head_t = TC.DINOHeadCPU(P.dino_head_state(14, 768, 65536))
        per_batch = {}
        for b in batches:
            gl = torch.from_numpy(P.clip(100 + b, (2 * b, 3, 8, 224, 224)))
            lo = torch.from_numpy(P.clip(200 + b, (6 * b, 3, 8, 96, 96)))
            center = torch.zeros(1, 65536)

            def step():
                s_out = head_s(torch.cat([student.forward_features(gl), student.forward_features(lo)]))
                t_out = head_t(teacher.forward_features(gl))
                return TC.dino_loss(s_out, t_out, center, 8, 0.04)
            step()
            times = []
            for _ in range(reps):
                t0 = time.perf_counter()
                step()
                times.append(time.perf_counter() - t0)
            per_batch[b] = (float(np.median(times)), times)
    finally:
        torch.set_num_threads(prev)
    best = max(per_batch, key=lambda b: b / per_batch[b][0])
    return {"value": round(best / per_batch[best][0], 4), "unit": "clips/s", "cores": int(cores), "kind": "port",
            "cpu_model": model,
            "per_batch": {str(b): {"clips_per_s": round(b / t, 4), "median_s": round(t, 3),
                                   "runs_s": [round(x, 3) for x in ts]} for b, (t, ts) in per_batch.items()},
            "sample": "DINO fwd+loss steps of %s multi-crop clip(s) (teacher 2x8x224^2 + student 2x8x224^2 + "
                      "6x8x96^2, DINOHead(65536), DINOLoss ncrops 8), torch %s CPU fp32 eager (oracle/torch_cpu.py), "
                      "%d threads, 1 warm-up + median of %d; value = the faster batch"
                      % ("/".join(map(str, batches)), torch.__version__, cores, reps)}


def pmc_traffic(kernel_name, path=os.path.join(ROOT, "profiles", "pmc_traffic.json")):
    """(HBM bytes per launch, source) of the dominant kernel from the committed PMC summary
    (tools/pmc_summary.py over separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this same
    bench command, gfx950 FETCH x2 correction applied).  Matched on the FULL instantiation name
    (dsvt.ops.gemm_kernel_name): (None, reason) when the summary has no entry for exactly that
    kernel -- never another instantiation's counters."""
    try:
        with open(path) as f:
            doc = json.load(f)
        kernels = doc["kernels"]
    except (OSError, ValueError, KeyError):
        return None, "no PMC summary at %s" % os.path.relpath(path, ROOT)
    v = kernels.get(kernel_name)
    if v is None:
        return None, "%s has no entry for %s" % (os.path.relpath(path, ROOT), kernel_name)
    return round(v["traffic_bytes"]), "%s (%s, %d dispatches)" % (os.path.relpath(path, ROOT),
                                                                 doc.get("run", "rocprofv3 --pmc"), v["calls"])


# ----------------------------------------------------------------- models / data
def build(dtype, device, seed=0):
    from functools import partial

    import torch.nn as nn

    from dsvt.loss import DINOLoss
    from dsvt.models.timesformer import VisionTransformer
    from dsvt.utils import MultiCropWrapper
    from dsvt.vision_transformer import DINOHead

    def net():
        bb = VisionTransformer(img_size=224, patch_size=16, num_classes=0, embed_dim=768, depth=12, num_heads=12,
                               mlp_ratio=4, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6),
                               drop_path_rate=0.1, num_frames=8, attention_type="divided_space_time")
        hd = DINOHead(768, 65536, norm_last_layer=True)
        bb.dsvt_dtype = hd.dsvt_dtype = dtype
        return MultiCropWrapper(bb, hd)

    torch.manual_seed(seed)
    student = net()
    teacher = net()
    teacher.load_state_dict(student.state_dict())          # train_ssl.py:330-333
    # random-init stand-in for the SVT weights: the temporal branch must not be a no-op
    # (reference zero-inits temporal_fc, SURVEY §5 defect 3)
    with torch.no_grad():
        for m in (student, teacher):
            for blk in m.backbone.blocks:
                blk.temporal_fc.weight.normal_(0, 0.02)
            m.backbone.time_embed.normal_(0, 0.02)
    for p in list(student.parameters()) + list(teacher.parameters()):
        p.requires_grad_(False)
    student = student.to(device).eval()
    teacher = teacher.to(device).eval()
    loss = DINOLoss(65536, 8, 0.04, 0.04, 0, 100).to(device)
    return student, teacher, loss


def synthetic_crops(clips, device, seed):
    """U8 uniform frames -> /255 -> (x - mean)/std, NCTHW fp32, resident on the GPU."""
    g = torch.Generator(device=device).manual_seed(seed)

    def crop(S):
        x = torch.randint(0, 256, (clips, 3, 8, S, S), generator=g, device=device, dtype=torch.uint8).float()
        return ((x / 255.0 - IMAGENET_MEAN[0]) / IMAGENET_STD[0]).contiguous()
    return [crop(224) for _ in range(2)] + [crop(96) for _ in range(6)]


# ----------------------------------------------------------------- config 3: SSL training step
def train_bench(args, device, rank, world, steps, warmup):
    """Config 3: the full DINO SSL step of train_ssl.py:466-573 per GPU --
    teacher fwd (2 global crops) + student fwd (2 global + 6 local, DropPath 0.1 active) + DINO
    loss with the RCCL center all-reduce + student backward on libdsvt with the DDP bucketed
    RCCL gradient all-reduce (world > 1) + per-parameter clipping + AdamW + teacher EMA.
    Weak scaling: `--clips` per GPU; value = all ranks' clips / max-over-ranks time."""
    from dsvt import dist as ddist
    from dsvt.trainer import DINOTrainer
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    student, teacher, dino_loss = build(dtype, device, seed=0)
    for p in student.parameters():
        p.requires_grad_(True)
    student.train()
    teacher.eval()          # the reference never sets eval on the teacher (SURVEY §5 defect 2); dsvt does
    ddp = None
    if world > 1:
        # the head on DDP's reducer, the backbone's gradients in per-block buckets all-reduced
        # under its own backward (dist.BlockGradReducer)
        ddp = ddist.wrap_ddp(student, device, overlap=getattr(args, "grad_overlap", True),
                             gradient_as_bucket_view=True)
    # the reference's defaults (train_ssl.py:50-151): lr 5e-4 scaled by clips * world / 256
    trainer = DINOTrainer(student, teacher, dino_loss, ddp=ddp, niter_per_ep=1000, epochs=100,
                          batch_size_per_gpu=args.clips, world_size=world,
                          concurrent_teacher=getattr(args, "concurrent_teacher", True))
    student.concurrent_grad_groups = getattr(args, "concurrent_groups", False)
    crops = synthetic_crops(args.clips, device, seed=4321 + rank)
    for i in range(warmup):
        trainer.step(crops, 2000 + i)       # past warm-up / first epoch: the last layer trains too
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = trainer.step(crops, 2000 + warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = ddist.max_over_ranks(time.perf_counter() - t0, device)
    loss_val = float(loss.item())
    if not np.isfinite(loss_val):
        raise SystemExit("bench: non-finite training loss %r" % loss_val)
    # the reference's own configuration: the teacher left in train mode (DropPath 0.1 active,
    # never .eval()'d: train_ssl.py:330-333), run under no_grad after the student -- the masked
    # training forward without saved activations (training.backbone_forward_nosave)
    elapsed_tt = float("nan")
    if not getattr(args, "no_teacher_train", False):      # tools/train_step.py traces skip it
        teacher.train()
        trainer.step(crops, 2000 + warmup + steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for i in range(steps):
            trainer.step(crops, 2001 + warmup + steps + i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed_tt = ddist.max_over_ranks(time.perf_counter() - t1, device)
        teacher.eval()
    g, l = vit_fwd_flops(8, 224), vit_fwd_flops(8, 96)
    fwd_s = 2 * g + 6 * l + 8 * head_flops()
    clip_gf = (2 * g + 2 * head_flops() + 3 * fwd_s) / 1e9      # teacher fwd + student fwd + 2x-fwd backward
    value = world * args.clips * steps / elapsed
    del trainer, student, teacher
    return {"metric": "clips/sec (DINO SSL train step: teacher fwd + student fwd/bwd + RCCL grad/center "
                      "all-reduce + AdamW + EMA)",
            "value": round(value, 3), "unit": "clips/s", "n_gpus": world, "steps": steps, "warmup": warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 3), "gflop_per_clip": round(clip_gf, 1),
            "tflops_per_gpu": round(value * clip_gf / 1e3 / world, 1), "loss": round(loss_val, 5),
            "parallelism": ("dp%d (%s bucketed all-reduce, %s)" % (
                world, "RCCL" if ddist.backend() == "nccl" else ddist.backend(),
                "backbone per-block buckets overlapped with its backward + DDP head"
                if getattr(args, "grad_overlap", True) else "DDP")) if world > 1 else "dp1",
            "optimizer": "dsvt AdamW (multi-tensor HIP kernel)",
            "drop_path": 0.1, "teacher_mode": "eval",
            "teacher_train_mode": {"value": round(world * args.clips * steps / elapsed_tt, 3),
                                   "ms_per_step": round(elapsed_tt / steps * 1e3, 3),
                                   "note": "the reference's teacher: train mode, DropPath 0.1, no_grad, "
                                           "sequential after the student (RNG order)"}}


def swin_train_bench(dtype, device, clips, steps, warmup):
    """DINOTrainer steps with the Video Swin-T student / teacher (--arch swin)."""
    from dsvt.loss import DINOLoss
    from dsvt.models import SwinTransformer3D
    from dsvt.trainer import DINOTrainer
    from dsvt.utils import MultiCropWrapper
    from dsvt.vision_transformer import DINOHead

    def net():
        bb = SwinTransformer3D(drop_path_rate=0.1)
        hd = DINOHead(768, 65536, norm_last_layer=True)
        bb.dsvt_dtype = hd.dsvt_dtype = dtype
        return MultiCropWrapper(bb, hd).to(device)
    torch.manual_seed(0)
    student = net()
    teacher = net()
    teacher.load_state_dict(student.state_dict())
    for p in teacher.parameters():
        p.requires_grad_(False)
    student.train()
    teacher.eval()
    loss_fn = DINOLoss(65536, 8, 0.04, 0.04, 0, 100).to(device)
    trainer = DINOTrainer(student, teacher, loss_fn, niter_per_ep=1000, epochs=100, batch_size_per_gpu=clips,
                          world_size=1)
    crops = synthetic_crops(clips, device, seed=777)
    for i in range(warmup):
        trainer.step(crops, 2000 + i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = trainer.step(crops, 2000 + warmup + i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    lv = float(loss.item())
    del trainer, student, teacher
    return {"value": round(clips * steps / el, 3), "unit": "clips/s", "ms_per_step": round(el / steps * 1e3, 2),
            "clips_per_step": clips, "steps": steps, "loss": round(lv, 5), "finite": bool(np.isfinite(lv)),
            "crops": "2 x 8x224^2 + 6 x 8x96^2", "drop_path": 0.1,
            "note": "Swin-T DINO SSL step (not a BASELINE metric; the --arch swin student)"}


# ----------------------------------------------------------------- configs 4 / 5: other backbones
def joint_flops(T=16, S=224, C=768, depth=12, heads=12, mlp=4, patch=16, cls_tail=False):
    """ViT-B/16 joint space-time forward: 899.35 GFLOP at 16x224^2.  cls_tail: what
    dsvt executes for a CLS-only forward (the last block's attention for the CLS query only, its
    proj and MLP on the CLS row only)."""
    N = (S // patch) ** 2
    L = 1 + N * T
    per_block = 2 * L * C * 3 * C + 4 * heads * L * L * (C // heads) + 2 * L * C * C + 2 * 2 * L * C * mlp * C
    tail = 0
    if cls_tail:
        tail = (4 * heads * (L - 1) * L * (C // heads) + 2 * (L - 1) * C * C + 2 * 2 * (L - 1) * C * mlp * C
                + 2 * (L - 1) * C * C)                                           # + the patch rows' queries
    return depth * per_block - tail + 2 * N * T * (3 * patch * patch) * C


def swin_t_flops(T=8, S=224, C=96, depths=(2, 2, 6, 2), window=(2, 7, 7), patch=(4, 4, 4)):
    """Video Swin-T forward at 8x224^2: 2*M*N*K of every Linear / Conv3d / window matmul."""
    D, H, W = T // patch[0], S // patch[1], S // patch[2]
    fl = 2 * D * H * W * C * 3 * patch[0] * patch[1] * patch[2]
    for i, depth in enumerate(depths):
        c = C * 2 ** i
        rows = D * H * W
        wd, wh, ww = min(window[0], D), min(window[1], H), min(window[2], W)
        n = wd * wh * ww
        rows_w = (-(-D // wd) * wd) * (-(-H // wh) * wh) * (-(-W // ww) * ww)
        fl += depth * (2 * rows_w * c * 3 * c + 4 * rows_w * n * c + 2 * rows_w * c * c + 2 * 2 * rows * c * 4 * c)
        if i < len(depths) - 1:
            H, W = (H + 1) // 2, (W + 1) // 2
            fl += 2 * D * H * W * 4 * c * 2 * c
    return fl


def other_configs(args, device):
    """Forward clips/s of the config-2 backbone alone (16 divided-attention 8x224^2 clips) and of
    BASELINE.json configs 4 (ViT-B/16 joint space-time, 16x224^2) and 5 (Video Swin-T, 8x224^2),
    and frames/s of the frame-scoring path (64 frames, local 3 / global 30), on one GPU, random
    init, synthetic normalized frames."""
    from functools import partial

    import torch.nn as nn

    from dsvt.models import SwinTransformer3D
    from dsvt.models.timesformer import VisionTransformer
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    res = {}

    def timed(fn, reps=5, warm=2):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    def graph_timed(fn, reps=10):
        """fn's kernels captured once in a HIP graph (as the fwd+loss step is) and replayed:
        the host's per-launch work leaves the timed region, every kernel still runs."""
        fn()
        torch.cuda.synchronize()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    # the north-star's own unit: the ViT-B/16 8x224^2 divided-attention backbone forward alone
    # (16 clips = the global crops of one 8-sample step), against the bf16 MFMA roofline
    torch.manual_seed(1)
    dm = VisionTransformer(img_size=224, num_classes=0, embed_dim=768, depth=12, num_heads=12, qkv_bias=True,
                           norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=8,
                           attention_type="divided_space_time").to(device).eval()
    dm.dsvt_dtype = dtype
    xd = torch.randn(16, 3, 8, 224, 224, device=device)
    with torch.no_grad():
        te = timed(lambda: dm(xd))
        t = graph_timed(lambda: dm(xd))
    ref_gf, exe_gf = vit_fwd_flops(8, 224), vit_fwd_flops(8, 224, folded=True, cls_tail=dm.cls_tail)
    peak = PEAK_TFLOPS[args.dtype]
    res["config2_backbone_fwd"] = {"value": round(16 / t, 2), "unit": "clips/s", "clips_per_step": 16,
                                   "launch": "hip_graph", "eager_value": round(16 / te, 2),
                                   "streams": "batch split over concurrent HIP streams (dsvt_streams=%s)"
                                              % dm.dsvt_streams,
                                   "gflop_per_clip": round(ref_gf / 1e9, 2),
                                   "tflops_executed": round(16 * exe_gf / t / 1e12, 1),
                                   "frac_executed": round(16 * exe_gf / t / 1e12 / peak, 4),
                                   "frac_reference_flops": round(16 * ref_gf / t / 1e12 / peak, 4)}
    del dm, xd
    if dtype == torch.bfloat16:
        # the fp32 PARITY mode of the headline step: the same config-2 fwd+loss
        # (8 multi-crop clips) with every kernel in fp32 -- the mode whose CLS embeddings / logits
        # meet the north star's 1e-3 against the reference, not only its loss
        from dsvt.utils import dino_forward
        s32, t32, l32 = build(torch.float32, device, seed=0)
        c32 = synthetic_crops(args.clips, device, seed=1234)

        def fwd_loss32():
            with torch.no_grad():
                so, to_ = dino_forward(s32, t32, c32, concurrent=True)
                return l32(so, to_, 0)
        t = timed(fwd_loss32, reps=3, warm=1)
        loss32 = float(fwd_loss32().item())
        res["config2_fwd_loss_fp32"] = {"value": round(args.clips / t, 3), "unit": "clips/s",
                                        "clips_per_step": args.clips, "launch": "eager", "dtype": "fp32",
                                        "loss": round(loss32, 5),
                                        "tflops_executed": round(args.clips * clip_flops(
                                            folded=s32.backbone.fold_temporal_fc, cls_tail=s32.backbone.cls_tail)
                                            / t / 1e12, 1),
                                        "note": "parity mode (v_mfma_f32_16x16x4f32 GEMMs, fp32 attention): the "
                                                "reference's numerics within 1e-3 on embeddings, logits and loss"}
        del s32, t32, l32, c32
        torch.cuda.empty_cache()
    jm = VisionTransformer(img_size=224, num_classes=0, embed_dim=768, depth=12, num_heads=12, qkv_bias=True,
                           norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=16,
                           attention_type="joint_space_time").to(device).eval()
    jm.dsvt_dtype = dtype
    xj = torch.randn(2, 3, 16, 224, 224, device=device)
    with torch.no_grad():
        te = timed(lambda: jm(xj))
        t = graph_timed(lambda: jm(xj))
    res["config4_joint16"] = {"value": round(2 / t, 2), "unit": "clips/s", "clips_per_step": 2,
                              "launch": "hip_graph", "eager_value": round(2 / te, 2),
                              "gflop_per_clip": round(joint_flops() / 1e9, 1),
                              "executed_gflop_per_clip": round(joint_flops(cls_tail=jm.cls_tail) / 1e9, 1),
                              "tflops": round(2 * joint_flops() / t / 1e12, 1),
                              "tflops_executed": round(2 * joint_flops(cls_tail=jm.cls_tail) / t / 1e12, 1)}
    del jm, xj
    sm = SwinTransformer3D().to(device)
    sm.eval()
    sm.dsvt_dtype = dtype
    xs = torch.randn(8, 3, 8, 224, 224, device=device)
    with torch.no_grad():
        te = timed(lambda: sm(xs))
        t = graph_timed(lambda: sm(xs))
    res["config5_swin_t"] = {"value": round(8 / t, 2), "unit": "clips/s", "clips_per_step": 8,
                             "launch": "hip_graph", "eager_value": round(8 / te, 2),
                             "gflop_per_clip": round(swin_t_flops() / 1e9, 2),
                             "tflops": round(8 * swin_t_flops() / t / 1e12, 1)}
    del sm, xs
    # the --arch swin SSL step (train_ssl.py:237-239 with the config-3 loop body): Swin-T student
    # (DropPath 0.1 as the reference's swin default 0.2 is the Swin-B one) and teacher with the
    # DINOHead(768, 65536), DINOLoss(ncrops 8), 8 clips of 2 global 8x224^2 + 6 local 8x96^2 crops --
    # not a BASELINE metric: evidence that the Swin training path runs at full size
    if not getattr(args, "no_swin_train", False):
        res["config5_swin_t_train"] = swin_train_bench(dtype, device, clips=8, steps=3, warmup=1)
    # frame scoring (a18 / a19): one F = 64-frame 224^2 video, local 3 / global 30
    # views per frame (dino_similarity.py:66-93), pairwise DINO loss per frame
    from dsvt.scoring import FrameScorer
    torch.manual_seed(2)
    fm = VisionTransformer(img_size=224, num_classes=0, embed_dim=768, depth=12, num_heads=12, qkv_bias=True,
                           norm_layer=partial(nn.LayerNorm, eps=1e-6), num_frames=8,
                           attention_type="divided_space_time").to(device).eval()
    fm.dsvt_dtype = dtype
    scorer = FrameScorer(fm, local_clip_size=3, global_clip_size=30)
    video = torch.randn(64, 3, 224, 224, device=device)
    with torch.no_grad():
        te = timed(lambda: scorer.score(video), reps=2, warm=1)
        t = graph_timed(lambda: scorer.score(video), reps=10)
    gf = (vit_fwd_flops(3, 224) + vit_fwd_flops(30, 224)) / 1e9
    res["frame_score"] = {"value": round(64 / t, 2), "unit": "frames/s", "frames": 64, "views": "local 3 / global 30",
                          "launch": "hip_graph (10 replays)", "eager_value": round(64 / te, 2), "dtype": args.dtype,
                          "gflop_per_frame": round(gf, 1), "tflops": round(64 * gf / t / 1e3, 1)}
    if dtype == torch.bfloat16:
        # the product output is the selected frames (frame_selection_loader.py:115-170).  The fp32
        # parity mode picks the reference's frames exactly (tests/test_gpu_model.py::
        # test_frame_scores_vitb_local3_global30); the bf16 mode moves a few picks by one frame.
        # Both modes are timed, and the bf16 picks are counted against the fp32 picks of the same
        # video (rates 1 / 4, N = 4 .. 24 picks, as the test does)
        from dsvt.selection import adaptive_frame_indices
        with torch.no_grad():
            s_bf = scorer.score(video).clone()
            fm.dsvt_dtype = torch.float32
            s_32 = scorer.score(video).clone()
            t32 = timed(lambda: scorer.score(video), reps=2, warm=1)
        fm.dsvt_dtype = dtype
        picked = moved = worst = 0
        for rate in (1, 4):
            for n_pick in (4, 8, 12, 16, 24):
                want, _ = adaptive_frame_indices(s_32, 64, 64 * rate, rate, n_pick)
                got, _ = adaptive_frame_indices(s_bf, 64, 64 * rate, rate, n_pick)
                want, got = np.asarray(want, np.int64), np.asarray(got, np.int64)
                picked += n_pick
                moved += int(np.sum(got != want))
                worst = max(worst, float(np.max(np.abs(got - want))) / rate)
        res["frame_score"].update({"picks_vs_fp32": picked, "picks_moved_vs_fp32": moved,
                                   "pick_mismatch_rate": round(moved / picked, 4), "max_shift_frames": worst})
        res["frame_score_fp32"] = {"value": round(64 / t32, 2), "unit": "frames/s", "frames": 64, "dtype": "fp32",
                                   "launch": "eager (2 reps)", "tflops": round(64 * gf / t32 / 1e3, 1),
                                   "picks": "the reference's frames (parity mode)"}
    return res


# ----------------------------------------------------------------- main
def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) outside torch.distributed.run: start N ranks of this script
    through torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) as CHILD
    processes -- this process never initialises the GPU -- and return their exit status.
    Fails loudly when fewer than N GPUs are visible (unless --shared-gpu rehearses it)."""
    import socket
    import subprocess
    ndev = torch.cuda.device_count()                    # does not initialise HIP
    if ndev < args.gpus and not args.shared_gpu:
        print("bench: --gpus %d requested but only %d GPU(s) are visible" % (args.gpus, ndev), file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clips", type=int, default=8, help="multi-crop clips per GPU per step (config 2: 8)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the per-kernel HIP-event probe")
    ap.add_argument("--serial", action="store_true",
                    help="run the backbone calls one after another (no stream overlap)")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every kernel eagerly instead of replaying the captured HIP graph")
    ap.add_argument("--no-train", action="store_true", help="skip the config-3 SSL training-step measurement")
    ap.add_argument("--ln-fold", default="auto", choices=["auto", "on", "off"],
                    help="LayerNorm folded into the GEMM that reads it (VisionTransformer.ln_fold; A/B)")
    ap.add_argument("--no-other", action="store_true", help="skip the config-4 / config-5 backbone measurements")
    ap.add_argument("--train-steps", type=int, default=5)
    ap.add_argument("--no-grad-overlap", dest="grad_overlap", action="store_false",
                    help="train leg at N>1: plain DDP over the whole student (no per-block backbone buckets)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 ('nccl' = RCCL over xGMI; 'gloo' only to rehearse "
                         "several ranks on one GPU with --shared-gpu)")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="rehearsal: allow N ranks on fewer GPUs (rank r uses GPU r %% count; needs --backend gloo)")
    args = ap.parse_args()

    from dsvt import dist as ddist

    rank, world, local_rank = ddist.env_ranks()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: start the N ranks before this process touches the GPU
        raise SystemExit(launch_ranks(args))
    if world != args.gpus:
        raise SystemExit("bench: --gpus %d but the torch.distributed.run environment has WORLD_SIZE=%d"
                         % (args.gpus, world))
    ndev = torch.cuda.device_count()                    # does not initialise HIP
    if world > ndev and not args.shared_gpu:
        raise SystemExit("bench: %d ranks but only %d GPU(s) visible" % (world, ndev))
    if args.shared_gpu and world > 1 and args.backend != "gloo":
        raise SystemExit("bench: --shared-gpu needs --backend gloo (RCCL refuses two ranks on one GPU)")
    local_rank = local_rank % max(ndev, 1)
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    rank, world = ddist.init_from_env(device, backend=args.backend)   # 'nccl' = RCCL over xGMI when world > 1
    from dsvt import ops

    # config 3 first: measured after the forward's HIP-graph capture and replays, the same training
    # step ran 86 instead of 99 clips/s (tools/train_step.py alone: 99-100)
    train_res = None
    if not args.no_train:
        train_res = train_bench(args, device, rank, world, args.train_steps, 2)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    from dsvt._lib import PROBE_GEMM

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    student, teacher, dino_loss = build(dtype, device)
    for net in (student, teacher):
        net.backbone.ln_fold = {"auto": "auto", "on": True, "off": False}[args.ln_fold]
    crops = synthetic_crops(args.clips, device, seed=1234 + rank)

    from dsvt.utils import dino_forward
    student.concurrent_groups = teacher.concurrent_groups = not args.serial

    dino_loss.defer_center_update = True   # center all-reduce + EMA outside the graph

    def forward_loss(concurrent=not args.serial):
        student.concurrent_groups = teacher.concurrent_groups = concurrent
        # the serial probe pass keeps every kernel alone on the chip: no split batches either
        student.backbone.dsvt_streams = teacher.backbone.dsvt_streams = "auto" if concurrent else 1
        with torch.no_grad():
            # student: 2 backbone calls (224 / 96 groups) + head on (2+6)*clips rows; teacher:
            # 1 backbone call + head on 2*clips rows -- three independent calls, overlapped
            s_out, t_out = dino_forward(student, teacher, crops, concurrent=concurrent)
            return dino_loss(s_out, t_out, 0)

    def center_update():
        colsum, rows = dino_loss.last_colsum
        dino_loss.update_center(colsum, rows)   # RCCL all-reduce of the teacher column sum when N > 1

    def step(concurrent=not args.serial):
        loss = forward_loss(concurrent)
        center_update()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- per-kernel measurement pass: eager, SERIAL launches (the probe brackets each launch
    # with HIP events on its stream; kernels sharing the chip with another stream would read
    # long), so the roofline is each kernel's own time -- same command as the rocprof summary
    probe = None
    if not args.no_probe:
        ops.probe_enable(PROBE_GEMM, 1 << 16)
        for _ in range(min(args.steps, 5)):
            step(concurrent=False)
        torch.cuda.synchronize()
        probe = ops.probe_read(1 << 16, with_bytes=True)
        ops.probe_disable()

    # ---- the timed run: the whole forward + loss of a step as ONE captured HIP graph (every
    # kernel of every step still runs; the graph only removes per-launch CPU work and gaps)
    graph = None
    if not args.no_graph:
        graph = torch.cuda.CUDAGraph()
        # capture on a stream of our own that has run the step eagerly once: its per-stream
        # scratch (the stream-K GEMM workspace, dsvt.ops) then exists before capture
        cap = torch.cuda.Stream()
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            forward_loss()
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, stream=cap):
            g_loss = forward_loss()
        torch.cuda.synchronize()

        def step(concurrent=None):  # noqa: F811
            graph.replay()
            center_update()
            return g_loss
        step()                                  # one replay before timing
        torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = ddist.max_over_ranks(time.perf_counter() - t0, device)
    loss_val = float(loss.item())
    if not np.isfinite(loss_val):
        raise SystemExit("bench: non-finite DINO loss %r -- the measured step is not valid" % loss_val)

    roofline = None
    if probe is not None:
        ms, work, fam, tag, nbytes = probe
        if len(ms):
            by_tag = {}
            for t, m_, w_ in zip(tag, ms, work):
                a = by_tag.setdefault(int(t), [0, 0.0, 0.0])
                a[0] += 1
                a[1] += float(m_)
                a[2] += float(w_)
            dom = max(by_tag, key=lambda t: by_tag[t][1])
            n, tms, tfl = by_tag[dom]
            peak = PEAK_TFLOPS[args.dtype]
            # per-launch roofline of the dominant kernel: each launch class (shape) is bound by
            # max(FLOP / MFMA peak, algorithmic bytes / HBM peak)
            classes = {}
            for t, m_, w_, b_ in zip(tag, ms, work, nbytes):
                if int(t) != dom:
                    continue
                c = classes.setdefault((float(w_), float(b_)), [0, 0.0])
                c[0] += 1
                c[1] += float(m_)
            cls_out, t_att, share = [], 0.0, {"mfma": 0.0, "hbm": 0.0}
            for (w_, b_), (cn, cms) in sorted(classes.items(), key=lambda kv: -kv[1][1]):
                avg_s = cms / cn * 1e-3
                t_f, t_b = w_ / (peak * 1e12), b_ / (HBM_PEAK_GBS * 1e9)
                bound = "hbm" if t_b > t_f else "mfma"
                share[bound] += cms
                t_att += cn * max(t_f, t_b)
                cls_out.append({"launches": cn, "gflop": round(w_ / 1e9, 2), "mbytes": round(b_ / 1e6, 1),
                                "bound": bound, "avg_us": round(avg_s * 1e6, 2),
                                "tflops": round(w_ / avg_s / 1e12, 1), "gbs": round(b_ / avg_s / 1e9, 1),
                                "frac_of_bound": round(max(t_f, t_b) / avg_s, 4)})
            bound = "hbm" if share["hbm"] > share["mfma"] else "mfma"
            if bound == "mfma":
                achieved, unit, pk = tfl / (tms * 1e-3) / 1e12, "TFLOP/s", peak
            else:
                tb = sum(c["mbytes"] * 1e6 * c["launches"] for c in cls_out)
                achieved, unit, pk = tb / (tms * 1e-3) / 1e9, "GB/s", HBM_PEAK_GBS
            all_ms = float(np.sum(ms))
            kname = ops.gemm_kernel_name(dom)
            traffic, traffic_src = pmc_traffic(kname)
            roofline = {"bound": bound, "achieved": round(achieved, 1), "peak": pk, "unit": unit,
                        "frac": round(achieved / pk, 4), "traffic": traffic, "traffic_source": traffic_src,
                        "traffic_over_algorithmic": (round(traffic / (sum(c["mbytes"] * 1e6 * c["launches"]
                                                                          for c in cls_out) / n), 3)
                                                     if traffic else None),
                        "frac_attainable": round(t_att / (tms * 1e-3), 4),
                        "kernel": kname, "launches": n,
                        "avg_launch_us": round(tms / n * 1e3, 2),
                        "flops_per_launch": tfl / n,
                        "launch_classes": cls_out,
                        "gemm_kernel_ms_per_step": round(all_ms / min(args.steps, 5), 3),
                        "measured": "HIP events around each launch, serial eager pass of the same step; "
                                    "frac_attainable = sum over launches of max(FLOP/MFMA peak, bytes/HBM peak) "
                                    "/ measured time",
                        "all_gemm_tflops": round(float(np.sum(work)) / (all_ms * 1e-3) / 1e12, 1)}

    value = world * args.clips * args.steps / elapsed
    step_ms = elapsed / args.steps * 1e3
    folded = student.backbone.fold_temporal_fc
    tail = student.backbone.cls_tail
    step_tflops = value * clip_flops(folded=folded, cls_tail=tail) / 1e12        # FLOPs the GPU executed
    out = {"metric": METRIC, "value": round(value, 3), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(step_ms, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
           "config": {"workload": "DINO-SVT fwd+loss: per clip teacher ViT-B/16 divided-ST on 2x8x224^2 global "
                                  "crops + student on 2x8x224^2 + 6x8x96^2 crops, DINOHead(768->65536), "
                                  "DINOLoss(ncrops=8) + center all-reduce",
                      "clips_per_gpu": args.clips, "global_batch": world * args.clips,
                      "gflop_per_clip": round(clip_flops() / 1e9, 1),
                      "executed_gflop_per_clip": round(clip_flops(folded=folded, cls_tail=tail) / 1e9, 1),
                      "last_block": ("CLS rows only past the spatial qkv (the reference discards the last block's "
                                     "patch-row outputs: x[:, 0] after the final norm)") if tail else "full",
                      "parallelism": "dp%d" % world,
                      "weights": "random init (torch seed 0)",
                      "launch": "eager" if graph is None else "hip_graph (forward+loss captured; center all-reduce eager)",
                      "streams": "serial" if args.serial else "3 backbone calls on concurrent HIP streams",
                      "layernorm": ("folded into the GEMM that reads it (dsvt_gemm_lnx_fwd)"
                                    if student.backbone.ln_fold else "LayerNorm pass + GEMM")},
           "step_roofline": {"achieved": round(step_tflops / world, 1), "peak": PEAK_TFLOPS[args.dtype],
                             "unit": "TFLOP/s per GPU", "flops": "executed",
                             "frac": round(step_tflops / world / PEAK_TFLOPS[args.dtype], 4),
                             "frac_reference_flops": round(value * clip_flops() / 1e12 / world
                                                           / PEAK_TFLOPS[args.dtype], 4)},
           "roofline": roofline, "loss": round(loss_val, 5),
           "world_size": world, "backend": ddist.backend() or "none",
           "rccl_ranks": world if ddist.backend() == "nccl" else 0}
    if train_res is not None:
        out["train_step"] = train_res
    if rank == 0 and world == 1 and not args.no_other:
        out["other_configs"] = other_configs(args, device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
