"""Frame-importance scoring (the repo's product output) on libdsvt.so.

dino_similarity.py:16-93: for every frame i of a (sampled, normalized, center-cropped)
video, the DINO loss between the backbone CLS of a short local clip around i (student
view) and of a long global clip around i (teacher view); same network, center 0,
teacher_temp 0.02, student_temp 0.3.  Windows follow
datasets_custom/dino_loss_loader.py:126-171 exactly (clamped at the video ends).

MI355X-first differences (same numbers):
  * the 2F views [2F, 3, 30, 224, 224] are never materialized: the patch-embed kernel
    gathers frames of a resident frame bank [F, 3, 224, 224] through an index map;
  * many frames per backbone call, and no per-frame `.item()` host sync
    (dino_similarity.py:87-88) -- scores stay on the device until the caller reads them.
"""
import json
import os

import numpy as np
import torch

from .loss import PairwiseDINOLoss


def view_windows(F, local_size, global_size):
    """Index form of get_views_of_video_same_size: per frame i, (j, k, l, m, G) such that the
    local view is frames[j:k] zero-padded to G frames and the global view frames[l:m]."""
    loc, glob = int(local_size / 2), int(global_size / 2)
    if F < global_size:
        global_size = F
    out = []
    for i in range(F):
        j, k, l, m = i - loc, i + loc + 1, i - glob, i + glob
        if j < 0:
            j, k = 0, local_size
        if k >= F:
            k, j = F, F - local_size
        if l < 0:
            l, m = 0, global_size
        if m >= F:
            m, l = F, F - global_size
        out.append((j, k, l, m, global_size))
    return out


def view_index(F, local_size, global_size):
    """(local_idx [F, local_size], global_idx [F, G]) int32 frame indices of the views the
    model consumes (dino_similarity.py:78-79: local = padded view[:, :, :local_size])."""
    if local_size % 2 == 0 or global_size % 2 == 1:
        # the reference's views only stack for odd local / even global sizes
        raise ValueError("local_clip_size must be odd and global_clip_size even (reference window rule)")
    if F < local_size:
        raise ValueError("video has %d frames < local_clip_size %d" % (F, local_size))
    w = view_windows(F, local_size, global_size)
    G = w[0][4]
    li = np.stack([np.arange(j, k) for (j, k, _, _, _) in w]).astype(np.int32)
    gi = np.stack([np.arange(l, m) for (_, _, l, m, _) in w]).astype(np.int32)
    assert li.shape == (F, local_size) and gi.shape == (F, G)
    return li, gi


def get_views_of_video_same_size(frames, local_size, global_size):
    """Tensor form of datasets_custom/dino_loss_loader.py:126-171 (data-loader side; kept for
    API compatibility -- the scorer itself uses view_index())."""
    F = frames.shape[0]
    views = []
    for (j, k, l, m, G) in view_windows(F, local_size, global_size):
        loc = frames[j:k].permute(1, 0, 2, 3)
        pad = torch.zeros(frames.shape[1], G, frames.shape[2], frames.shape[3], dtype=frames.dtype,
                          device=frames.device)
        pad[:, :local_size] = loc
        views.append(pad)
        views.append(frames[l:m].permute(1, 0, 2, 3))
    return torch.stack(views)


class FrameScorer:
    """Per-frame DINO-loss scores of a video with a (pretrained) dsvt TimeSformer."""

    def __init__(self, model, local_clip_size=3, global_clip_size=30, teacher_temp=0.02, student_temp=0.3,
                 frames_per_call=16):
        self.model = model
        self.local_clip_size = local_clip_size
        self.global_clip_size = global_clip_size
        self.loss = PairwiseDINOLoss(model.embed_dim, teacher_temp, student_temp).to(model.pos_embed.device)
        self.frames_per_call = frames_per_call

    @torch.no_grad()
    def score(self, frames):
        """frames [F, 3, H, W] fp32 on the GPU -> scores [F] fp32 (device)."""
        F = frames.shape[0]
        li, gi = view_index(F, self.local_clip_size, self.global_clip_size)
        dev = frames.device
        li_t = torch.from_numpy(li).to(dev)
        gi_t = torch.from_numpy(gi).to(dev)
        frames = frames.float().contiguous()
        scores = torch.empty(F, device=dev, dtype=torch.float32)
        n = self.frames_per_call
        for s0 in range(0, F, n):
            s1 = min(F, s0 + n)
            b = s1 - s0
            st = self.model.forward_frame_bank(frames, li_t[s0:s1].reshape(-1).contiguous(), b, li.shape[1])
            te = self.model.forward_frame_bank(frames, gi_t[s0:s1].reshape(-1).contiguous(), b, gi.shape[1])
            scores[s0:s1] = self.loss.per_row(st, te)
        return scores


def export_loss(loss_list, video_path, file_path):
    """dino_similarity.py:97-117: merge {video_name: [scores]} into a JSON file."""
    name, _ = os.path.splitext(os.path.basename(video_path))
    entry = {name: [float(v) for v in loss_list]}
    if os.path.exists(file_path):
        with open(file_path) as f:
            data = json.load(f)
        data.update(entry)
    else:
        data = entry
    with open(file_path, "w") as f:
        json.dump(data, f)
