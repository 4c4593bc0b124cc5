"""One DINO-SVT SSL training step (train_ssl.py:466-573, `train_one_epoch` body) on dsvt:

  student(all crops) [DDP] -> teacher(global crops) [no grad] -> DINOLoss (center all-reduce)
  -> backward (DDP bucketed all-reduce of the student gradients over RCCL)
  -> per-parameter gradient clipping -> cancel last-layer grads in the first epoch(s)
  -> AdamW with the lr / wd schedules -> teacher EMA (one multi-tensor launch)

The order of the two forwards is the reference's (student first, train_ssl.py:523-527), so a
seeded run draws the DropPath masks in the same order.  The lr schedule applies the
reference's linear scaling rule lr * batch_size_per_gpu * world_size / 256
(train_ssl.py:395-400) when `batch_size_per_gpu` is given; without it `lr` is taken as the
already-scaled peak value.

Differences from the reference loop, all deliberate and documented:
  * no fp16 GradScaler: dsvt computes in bf16 storage / fp32 accumulate with fp32 master
    weights and fp32 gradients (no loss scaling needed);
  * the non-finite-loss check reads the loss once per step like the reference (optional,
    `check_finite`), but clipping returns device-side norms instead of 254 .item() syncs.
"""
import math

import torch

from .training import np_cosine_scheduler
from .utils import cancel_gradients_last_layer, clip_gradients, ema_update_, get_params_groups


class _TeacherStepSettings:
    """The teacher backbone's step-time settings, applied for the duration of the teacher call
    only (set permanently they also changed later uses of the same teacher object,
    e.g. eval or kNN feature extraction).  Inside a training step:
    - no batch split over streams of its own: the teacher runs beside the student on its own
      stream (146.6 / 146.7 vs 143.7 / 143.6 clips/s with the inference path's automatic 3-way
      split -- five streams contend, as in the forward bench);
    - no temporal_attn.proj -> temporal_fc fold: the EMA changes the weights every step, so the
      fold (an fp32 768^3 product per block, redone each step) costs more than the extra bf16 GEMM
      of the unfolded pair it saves."""

    SETTINGS = (("dsvt_streams", 1), ("fold_temporal_fc", False))

    def __init__(self, teacher):
        self.bb = getattr(teacher, "backbone", teacher)
        self.saved = []

    def __enter__(self):
        self.saved = [(k, getattr(self.bb, k)) for k, _ in self.SETTINGS if hasattr(self.bb, k)]
        for k, v in self.SETTINGS:
            if hasattr(self.bb, k):
                setattr(self.bb, k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved:
            setattr(self.bb, k, v)
        return False


class DINOTrainer:
    def __init__(self, student, teacher, dino_loss, lr=5e-4, min_lr=1e-6, weight_decay=0.04, weight_decay_end=0.4,
                 momentum_teacher=0.996, clip_grad=3.0, freeze_last_layer=1, epochs=100, niter_per_ep=1000,
                 warmup_epochs=10, n_global=2, ddp=None, batch_size_per_gpu=None, world_size=None,
                 optimizer="dsvt", concurrent_teacher=True):
        self.student = student                      # MultiCropWrapper (possibly DDP-wrapped: ddp)
        self.model = ddp if ddp is not None else student
        self.teacher = teacher
        self.dino_loss = dino_loss
        self.clip_grad = clip_grad
        self.concurrent_teacher = concurrent_teacher
        self.freeze_last_layer = freeze_last_layer
        self.n_global = n_global
        self.niter_per_ep = niter_per_ep
        if batch_size_per_gpu is not None:          # linear scaling rule (train_ssl.py:395-400)
            if world_size is None:
                from .dist import world_size as _ws
                world_size = _ws()
            lr = lr * (batch_size_per_gpu * world_size) / 256.
        self.peak_lr = lr
        # train_ssl.py:394-407: schedules
        self.lr_schedule = np_cosine_scheduler(lr, min_lr, epochs, niter_per_ep, warmup_epochs=warmup_epochs)
        self.wd_schedule = np_cosine_scheduler(weight_decay, weight_decay_end, epochs, niter_per_ep)
        self.momentum_schedule = np_cosine_scheduler(momentum_teacher, 1, epochs, niter_per_ep)
        groups = get_params_groups(student)
        if optimizer == "dsvt":                     # multi-tensor HIP AdamW (csrc/backward.hip)
            from .optim import AdamW
            self.optimizer = AdamW(groups)
        elif optimizer == "torch":
            self.optimizer = torch.optim.AdamW(groups)      # train_ssl.py:384
        else:
            raise ValueError("optimizer must be 'dsvt' or 'torch'")
        for p in teacher.parameters():
            p.requires_grad_(False)
        self._teacher_settings = _TeacherStepSettings(teacher)
        self._s_params = [p for p in student.parameters()]
        if ddp is None:          # gradients at fixed addresses: cached pointer tables (training.persistent_grad_arena)
            for m in (getattr(student, "backbone", None), getattr(student, "head", None)):
                if m is not None:
                    m.dsvt_persistent_grads = True
        self._t_params = [p for p in teacher.parameters()]

    def backward(self, loss):
        """zero_grad(set_to_none=True) + loss.backward() (train_ssl.py:538-545).  Every .grad is
        dropped first: the persistent gradient buffers (training.persistent_grad_arena) are then
        free, and the backward makes them the new .grad."""
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()

    def step(self, images, it, check_finite=False):
        epoch = it // self.niter_per_ep
        for i, pg in enumerate(self.optimizer.param_groups):       # train_ssl.py:486-490
            pg["lr"] = float(self.lr_schedule[it])
            if i == 0:
                pg["weight_decay"] = float(self.wd_schedule[it])
        if self.concurrent_teacher and images[0].is_cuda:
            # the teacher forward (no grad) is independent of the student's: it runs on its own
            # stream, overlapping the student forward's GEMM tails.  A teacher that draws random
            # numbers (train mode with DropPath: the reference's own setup) is ENQUEUED after the
            # student, so the host-side RNG draws keep the reference's order (:523-527); the GPU
            # still runs both forwards at once (the side stream waits only for the step's inputs)
            from .utils import side_stream
            main = torch.cuda.current_stream(images[0].device)
            side = side_stream(images[0].device, "teacher")
            side.wait_stream(main)
            # (student first for any teacher: 143.6 / 143.8 vs 143.1 / 143.3 clips/s teacher-first)
            s_out = self.model(images)                             # :523
            with torch.cuda.stream(side), torch.no_grad(), self._teacher_settings:
                t_out = self.teacher(images[:self.n_global])       # :527 (teacher on global views)
            main.wait_stream(side)
            t_out.record_stream(main)
        else:
            s_out = self.model(images)                             # :523
            with torch.no_grad(), self._teacher_settings:
                t_out = self.teacher(images[:self.n_global])       # :527 (teacher on global views)
        loss = self.dino_loss(s_out, t_out, epoch)
        if check_finite and not math.isfinite(loss.item()):        # :530-532
            raise FloatingPointError("Loss is %s, stopping training" % loss.item())
        self.backward(loss)
        if self.clip_grad:
            clip_gradients(self.student, self.clip_grad)           # :547-548
        cancel_gradients_last_layer(epoch, self.student, self.freeze_last_layer)
        self.optimizer.step()
        with torch.no_grad():                                      # :555-558 EMA
            ema_update_(self._t_params, self._s_params, float(self.momentum_schedule[it]))
        return loss
