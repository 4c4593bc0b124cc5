"""DINO losses on libdsvt.so.

`DINOLoss`         train_ssl.py:602-691 (two_token=False): centering + sharpening CE over
                   the 2*(ncrops-1) teacher/student pairs, then the center EMA with an
                   RCCL all-reduce of the teacher column sum.
`PairwiseDINOLoss` dino_similarity.py:120-135: CE of one teacher row vs one student row --
                   the per-frame importance score.
"""
import numpy as np
import torch
import torch.nn as nn

from . import ops
from ._lib import DsvtError
from .dist import center_batch_sum


def _fp32(t, name):
    if not t.is_cuda:
        raise DsvtError("%s must be on the GPU (no CPU fallback)" % name)
    return t.detach().float().contiguous()


class DINOLoss(nn.Module):
    def __init__(self, out_dim, ncrops, warmup_teacher_temp, teacher_temp, warmup_teacher_temp_epochs, nepochs,
                 student_temp=0.1, center_momentum=0.9, global_crops=2, two_token=False):
        super().__init__()
        if two_token:
            raise NotImplementedError("DINOLoss(two_token=True) is the out-of-scope two-token variant")
        self.student_temp = student_temp
        self.center_momentum = center_momentum
        self.n_crops = ncrops
        self.global_crops = global_crops
        self.two_token = two_token
        self.register_buffer("center", torch.zeros(1, out_dim))
        # When True, forward() leaves the center update to the caller: the teacher column sum
        # and row count are kept in `last_colsum` for update_center().  Lets a HIP graph hold
        # the forward while the RCCL all-reduce of the center runs outside it.
        self.defer_center_update = False
        self.last_colsum = None
        # train_ssl.py:627-631
        self.teacher_temp_schedule = np.concatenate((
            np.linspace(warmup_teacher_temp, teacher_temp, warmup_teacher_temp_epochs),
            np.ones(nepochs - warmup_teacher_temp_epochs) * teacher_temp))

    def forward(self, student_output, teacher_output, epoch):
        """Returns the 0-d loss tensor (device); updates `center` (train_ssl.py:633-671)."""
        if torch.is_grad_enabled() and student_output.requires_grad:
            return self._forward_train(student_output, teacher_output, epoch)
        s = _fp32(student_output, "student_output")
        t = _fp32(teacher_output, "teacher_output")
        if t.shape[0] % self.global_crops:
            raise ValueError("teacher rows %d not divisible by global_crops %d" % (t.shape[0], self.global_crops))
        B = t.shape[0] // self.global_crops
        if s.shape[0] != self.n_crops * B:
            # the reference would silently mis-chunk here (SURVEY §5 defect 10); fail loudly instead
            raise ValueError("student rows %d != ncrops %d x batch %d" % (s.shape[0], self.n_crops, B))
        temp = float(self.teacher_temp_schedule[epoch])
        loss, colsum = ops.dino_loss(s, t, self.center, B, self.n_crops, self.global_crops, self.student_temp, temp)
        self.last_colsum = (colsum, t.shape[0])
        if not self.defer_center_update:
            self.update_center(colsum, t.shape[0])
        return loss.reshape(())

    def _forward_train(self, student_output, teacher_output, epoch):
        """Differentiable w.r.t. the student logits (dsvt.training.LossFn); the teacher is
        detached as in train_ssl.py:651."""
        from .training import LossFn
        if not student_output.is_cuda:
            raise DsvtError("student_output must be on the GPU (no CPU fallback)")
        s = student_output.float()
        s = s if s.is_contiguous() else s.contiguous()
        t = _fp32(teacher_output, "teacher_output")
        B = t.shape[0] // self.global_crops
        if t.shape[0] % self.global_crops or s.shape[0] != self.n_crops * B:
            raise ValueError("student rows %d / teacher rows %d do not match ncrops %d, global_crops %d" %
                             (s.shape[0], t.shape[0], self.n_crops, self.global_crops))
        temp = float(self.teacher_temp_schedule[epoch])
        if self.center.dtype != torch.float32 or not self.center.is_contiguous():
            self.center = self.center.float().contiguous()
        loss, colsum = LossFn.apply(s, t, self.center, B, self.n_crops, self.global_crops, self.student_temp, temp)
        self.last_colsum = (colsum, t.shape[0])
        if not self.defer_center_update:
            self.update_center(colsum, t.shape[0])
        return loss

    @torch.no_grad()
    def update_center(self, colsum, rows):
        """train_ssl.py:673-691: all-reduce (RCCL 'nccl' backend on ROCm) of the teacher column
        sum, then center = m*center + (1-m)*sum/(rows*world)."""
        scale = center_batch_sum(colsum, rows)
        if self.center.dtype != torch.float32 or not self.center.is_contiguous():
            self.center = self.center.float().contiguous()
        ops.center_ema(self.center, colsum, self.center_momentum, scale)


class PairwiseDINOLoss(nn.Module):
    """dino_similarity.DINOLoss(out_dim, teacher_temp, student_temp=0.1)."""

    def __init__(self, out_dim, teacher_temp, student_temp=0.1):
        super().__init__()
        self.student_temp = student_temp
        self.register_buffer("center", torch.zeros(1, out_dim))
        self.teacher_temp = teacher_temp

    def per_row(self, student_output, teacher_output):
        """CE per row pair: [R] fp32 (the frame-importance scores of dino_similarity.py:87-88)."""
        s = _fp32(student_output, "student_output").reshape(-1, student_output.shape[-1])
        t = _fp32(teacher_output, "teacher_output").reshape(-1, teacher_output.shape[-1])
        return ops.pair_loss(s, t, self.center.float(), self.student_temp, self.teacher_temp)

    def forward(self, student_output, teacher_output):
        """dino_similarity.py:129-135: sum over the last dim, mean over the rest."""
        per = self.per_row(student_output, teacher_output)
        return per.reshape(()) if per.numel() == 1 else per.mean()
