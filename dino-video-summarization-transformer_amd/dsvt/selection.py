"""Score -> frame selection on libdsvt.so (the consumer of the frame-importance scores).

Drop-in for the "adaptive" branch of `FrameSelectionLoader.__getitem__`
(datasets_custom/frame_selection_loader.py:115-166): the frame scores (a `loss_dict[key]`
list from the scores JSON, or the device tensor dsvt.scoring.FrameScorer returns) are turned
into N frame indices of the unsampled video and the N pre-sampled frames to stack, with the
reference's float64 numpy arithmetic reproduced bit-exactly by the `dsvt_select_frames` kernel
(pairwise np.sum, sequential cumsum, first arg-min, collision walk).  The frames are gathered on
the device by `dsvt_gather_rows`; nothing falls back to the host.
"""
import numpy as np
import torch

from . import _lib
from ._lib import call
from .ops import _stream  # noqa: F401  (the raw current-stream handle)


def adaptive_frame_indices(loss_list, n_frames, n_unsampled, pre_sampling_rate, N, device=None, return_cdf=False):
    """frame_selection_loader.py:115-166 minus the frame stacking.

    loss_list: sequence / ndarray / tensor of scores (float64 values; a float32 device tensor is
    widened exactly).  n_frames = frames.size(0) (pre-sampled), n_unsampled =
    frames_unsampled.size(0), pre_sampling_rate = the loader's `pre_sampling_rate`, N = frames
    to select.  Returns (indices: list of int -- the reference's `indices`, frame_pos: int32
    device tensor [N] -- the pre-sampled frame stacked for each slot[, cdf float64 [n]])."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type != "cuda":
        raise _lib.DsvtError("adaptive_frame_indices runs on the GPU (no CPU fallback)")
    if torch.is_tensor(loss_list):
        loss = loss_list.detach().to(device=dev, dtype=torch.float64).reshape(-1).contiguous()
    else:
        loss = torch.from_numpy(np.ascontiguousarray(np.asarray(loss_list, dtype=np.float64).reshape(-1))).to(dev)
    n = min(loss.numel(), int(n_frames))
    indices = torch.empty(int(N), device=dev, dtype=torch.int64)
    frame_pos = torch.empty(int(N), device=dev, dtype=torch.int32)
    cdf = torch.empty(n, device=dev, dtype=torch.float64) if return_cdf else None
    nbytes = int(_lib.lib().dsvt_workspace_bytes(_lib.WS_SELECT, _lib.F32, n, int(n_unsampled), 0))
    ws = torch.empty(nbytes, device=dev, dtype=torch.uint8)
    call("dsvt_select_frames", loss.data_ptr(), loss.numel(), int(n_frames), int(n_unsampled), int(pre_sampling_rate),
         int(N), indices.data_ptr(), frame_pos.data_ptr(), None if cdf is None else cdf.data_ptr(), ws.data_ptr(),
         nbytes, _stream())
    idx_list = [int(v) for v in indices.cpu().tolist()]
    return (idx_list, frame_pos, cdf) if return_cdf else (idx_list, frame_pos)


def gather_frames(frames, frame_pos):
    """torch.stack([frames[p] for p in frame_pos]) on the device (any dtype, rows = dim 0)."""
    if not frames.is_cuda or not frames.is_contiguous():
        raise _lib.DsvtError("gather_frames: frames must be a contiguous GPU tensor")
    pos = frame_pos.to(device=frames.device, dtype=torch.int32).contiguous()
    out = torch.empty((pos.numel(),) + tuple(frames.shape[1:]), device=frames.device, dtype=frames.dtype)
    row_bytes = frames[0].numel() * frames.element_size()
    call("dsvt_gather_rows", frames.data_ptr(), row_bytes, pos.data_ptr(), pos.numel(), out.data_ptr(), _stream())
    return out


def select_frames(frames, loss_list, n_unsampled, pre_sampling_rate, N):
    """The whole adaptive branch: returns (selected frames [N, ...] = torch.stack(selected_frames),
    indices) for the pre-sampled `frames` [F, C, H, W] (frame_selection_loader.py:113-166)."""
    idx, pos = adaptive_frame_indices(loss_list, frames.shape[0], n_unsampled, pre_sampling_rate, N,
                                      device=frames.device)
    return gather_frames(frames, pos), idx
