"""Video DINO augmentation on libdsvt.so (the input producer of the training path).

Drop-in for `VideoDataAugmentationDINO` (datasets_custom/transform.py:661-749): same
constructor, same `__call__(image, from_list, no_aug, two_token)` and the same random draws --
the parameters are sampled on the host by the reference's own RNG calls in the reference's
order (torch CPU generator for the crop window, numpy for flip / jitter / grayscale and the
no-op blur / solarization draws), so a seeded run picks the same crops, flips and jitters.  The
pixel work -- uint8 -> [0, 1], crop + bicubic resize, flip, the colour-jitter chain, grayscale,
normalization -- is one or two `dsvt_video_augment` kernel launches per crop on frames that stay
on the GPU.  `augment_clip` is the fused form the loader wants: decoded [T, H, W, C] uint8 in,
[C, T', S, S] fp32 out with the temporal index_select folded in.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import call

MEAN, STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)      # transform.py:684-686
JITTER = (("brightness", 0.4, 1), ("contrast", 0.4, 2), ("saturation", 0.2, 3))   # color_jitter(.4, .4, .2)


class AugParams(ctypes.Structure):
    """dsvt_aug_params (include/dsvt.h)"""
    _fields_ = [("y0", ctypes.c_int32), ("x0", ctypes.c_int32), ("h", ctypes.c_int32), ("w", ctypes.c_int32),
                ("size", ctypes.c_int32), ("flip", ctypes.c_int32), ("n_ops", ctypes.c_int32),
                ("op", ctypes.c_int32 * 3), ("alpha", ctypes.c_float * 3), ("beta", ctypes.c_float * 3),
                ("gray", ctypes.c_int32), ("mean", ctypes.c_float * 3), ("std", ctypes.c_float * 3)]


_SIG = False


def _bind():
    global _SIG
    if not _SIG:
        f = _lib.lib().dsvt_video_augment
        p, i64 = ctypes.c_void_p, ctypes.c_int64
        f.argtypes = [p, ctypes.c_int, i64, i64, p, i64, i64, i64, i64, i64, i64, ctypes.POINTER(AugParams),
                      p, ctypes.c_int, p, ctypes.c_size_t, p]
        f.restype = ctypes.c_int
        _SIG = True


# ------------------------------------------------------------------ host-side random draws
def draw_crop_window(height, width, scale, ratio=(3. / 4., 4. / 3.)):
    """random_resized_crop's window (transform.py:134-169), same RNG calls in the same order.
    All ten attempts always run (the reference never breaks out): the LAST accepted attempt
    supplies (i, j) while h, w come from the last attempt, accepted or not; the window is then
    clipped by the slicing at :171."""
    area = height * width
    accepted = False
    i = j = 0
    for _ in range(10):
        target_area = area * torch.empty(1).uniform_(scale[0], scale[1]).item()
        log_ratio = torch.log(torch.tensor(ratio))
        aspect_ratio = torch.exp(torch.empty(1).uniform_(log_ratio[0], log_ratio[1])).item()
        w = int(round(np.sqrt(target_area * aspect_ratio)))
        h = int(round(np.sqrt(target_area / aspect_ratio)))
        if 0 < w <= width and 0 < h <= height:
            i = torch.randint(0, height - h + 1, size=(1,)).item()
            j = torch.randint(0, width - w + 1, size=(1,)).item()
            accepted = True
    if not accepted:                       # central-crop fallback (:155-167)
        in_ratio = float(width) / float(height)
        if in_ratio < min(ratio):
            w, h = width, int(round(width / min(ratio)))
        elif in_ratio > max(ratio):
            h, w = height, int(round(height * max(ratio)))
        else:
            w, h = width, height
        i, j = (height - h) // 2, (width - w) // 2
    hh, ww = min(i + h, height) - i, min(j + w, width) - j
    if hh <= 0 or ww <= 0:
        raise ValueError("random_resized_crop drew an empty window (the reference fails here too)")
    return i, j, hh, ww


def draw_flip_jitter_gray():
    """flip_and_color_jitter (transform.py:670-677): (flip, [(op code, alpha)...], gray)."""
    flip = bool(np.random.uniform() < 0.5)                       # horizontal_flip(prob=0.5)
    ops = []
    if np.random.uniform() < 0.8:
        order = np.random.permutation(np.arange(len(JITTER)))     # color_jitter :392
        for k in order:
            _, var, code = JITTER[k]
            ops.append((code, 1.0 + np.random.uniform(-var, var)))
    gray = bool(np.random.uniform() < 0.2)
    return flip, ops, gray


def make_params(window, size, flip=False, ops=(), gray=False, mean=MEAN, std=STD):
    y0, x0, h, w = window
    p = AugParams()
    p.y0, p.x0, p.h, p.w, p.size = int(y0), int(x0), int(h), int(w), int(size)
    p.flip, p.n_ops, p.gray = int(flip), len(ops), int(gray)
    for k, (code, alpha) in enumerate(ops):
        p.op[k] = code
        p.alpha[k] = np.float32(alpha)            # `tensor * alpha` runs in float32
        p.beta[k] = np.float32(1.0 - alpha)       # `tensor * (1 - alpha)`
    for c in range(3):
        p.mean[c], p.std[c] = np.float32(mean[c]), np.float32(std[c])
    return p


# ------------------------------------------------------------------ launches
def augment_clip(frames, params, frame_index=None, layout="cthw", channels_last=None):
    """One crop of a clip on the GPU.  frames: [T, C, H, W] or (channels_last) [T, H, W, C],
    uint8 or fp32, on the GPU.  frame_index: optional int32 [T'] (the loader's temporal
    index_select).  Returns fp32 [C, T', S, S] (layout "cthw") or [T', C, S, S] ("tchw")."""
    if not frames.is_cuda:
        raise _lib.DsvtError("augment_clip: frames must be on the GPU (no CPU fallback)")
    if frames.dtype not in (torch.uint8, torch.float32):
        raise _lib.DsvtError("augment_clip: frames must be uint8 or float32")
    _bind()
    if channels_last is None:
        channels_last = frames.shape[-1] == 3 and frames.shape[1] != 3
    if channels_last:
        T_in, H, W, C = frames.shape
        sT, sH, sW, sC = frames.stride()
    else:
        T_in, C, H, W = frames.shape
        sT, sC, sH, sW = frames.stride()
    if C != 3:
        raise _lib.DsvtError("augment_clip: 3 colour channels expected")
    fidx = None
    T = T_in
    if frame_index is not None:
        fidx = frame_index.to(device=frames.device, dtype=torch.int32).contiguous()
        T = fidx.numel()
    S = params.size
    out = torch.empty((3, T, S, S) if layout == "cthw" else (T, 3, S, S), device=frames.device, dtype=torch.float32)
    nbytes = int(_lib.lib().dsvt_workspace_bytes(_lib.WS_AUGMENT, _lib.F32, T, S, 0))
    ws = torch.empty(max(nbytes, 8), device=frames.device, dtype=torch.uint8)
    rc = _lib.lib().dsvt_video_augment(frames.data_ptr(), int(frames.dtype == torch.uint8), T_in, T,
                                       None if fidx is None else fidx.data_ptr(), H, W, sT, sC, sH, sW,
                                       ctypes.byref(params), out.data_ptr(), 1 if layout == "cthw" else 0,
                                       ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise _lib.DsvtError("dsvt_video_augment failed (%d): %s" % (rc, _lib.lib().dsvt_last_error().decode()))
    return out


class VideoDataAugmentationDINO(object):
    """transform.py:661-749 with the pixel work on the GPU.  Crops come back [T, C, S, S] fp32
    like the reference's; frames may be uint8 (scaled by 1/255 in the kernel) or fp32 [0, 1],
    [T, C, H, W] tensors (moved to the current GPU if they are on the host)."""

    def __init__(self, global_crops_scale=(0.4, 1.0), local_crops_scale=(0.05, 0.4), local_crops_number=8):
        self.global_crops_scale = global_crops_scale
        self.local_crops_scale = local_crops_scale
        self.local_crops_number = local_crops_number

    @staticmethod
    def _dev(frames):
        return frames if frames.is_cuda else frames.to("cuda", non_blocking=True)

    def _crop(self, frames, size, scale, extra_draws=()):
        frames = self._dev(frames)
        window = draw_crop_window(frames.shape[-2], frames.shape[-1], scale)
        flip, ops, gray = draw_flip_jitter_gray()
        for _ in extra_draws:               # the blur / solarization coin flips (no-ops in the reference)
            np.random.uniform()
        return augment_clip(frames, make_params(window, size, flip, ops, gray), layout="tchw", channels_last=False)

    def no_aug(self, frames):               # :698-701
        frames = self._dev(frames)
        H, W = frames.shape[-2:]
        return augment_clip(frames, make_params((0, 0, H, W), 224), layout="tchw", channels_last=False)

    def global_transform1(self, frames):    # :704-709
        return self._crop(frames, 224, self.global_crops_scale)

    def global_transform2(self, frames):    # :712-720
        return self._crop(frames, 224, self.global_crops_scale, extra_draws=("blur", "solarize"))

    def local_transform(self, frames):      # :723-729
        return self._crop(frames, 96, self.local_crops_scale, extra_draws=("blur",))

    def __call__(self, image, from_list=False, no_aug=False, two_token=False):   # :731-749
        if two_token:
            crops = [self.global_transform1(image[0]), self.no_aug(image[0]),
                     self.local_transform(image[1]), self.local_transform(image[2]),
                     self.no_aug(image[3]), self.no_aug(image[4])]
        elif no_aug:
            crops = [self.no_aug(x) for x in image]
        elif from_list:
            crops = [self.global_transform1(image[0]), self.global_transform2(image[1])]
            for local_image in image[2:]:
                crops.append(self.local_transform(local_image))
        else:
            crops = [self.global_transform1(image), self.global_transform2(image)]
            for _ in range(self.local_crops_number):
                crops.append(self.local_transform(image))
        return crops
