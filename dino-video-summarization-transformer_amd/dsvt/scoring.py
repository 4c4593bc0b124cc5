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
    """(local_idx [F, Ts], global_idx [F, G]) int32 frame indices of the views the model
    consumes (dino_similarity.py:78-79: local = padded view[:, :, :local_size]).

    Same window arithmetic as dino_loss_loader.py:126-171, including its clamped edge cases:
    windows are Python slices (a negative start counts from the end), the local frames fill
    the first Ts = min(local_size, G) slots of the G-slot padded view with torch broadcasting
    (equal length, or one frame repeated -- e.g. F = 2, local 3: both local views are frame 1
    twice), G = min(global_size, F).  Raises ValueError exactly where the reference's view
    construction raises (assignment or stack shape mismatch: even local / odd global sizes in
    the middle of a video, some F < local_size)."""
    if F < 1:
        raise ValueError("empty video")
    w = view_windows(F, local_size, global_size)
    G = w[0][4]
    ts = min(local_size, G)
    ids = list(range(F))
    li = np.empty((F, ts), np.int32)
    gi = np.empty((F, G), np.int32)
    for i, (j, k, l, m, _) in enumerate(w):
        loc, glo = ids[j:k], ids[l:m]
        if len(loc) == 1:
            loc = loc * ts
        if len(loc) != ts or len(glo) != G:
            raise ValueError("the reference cannot build the views of a %d-frame video with local_clip_size %d "
                             "and global_clip_size %d (window %d has %d local / %d global frames)"
                             % (F, local_size, global_size, i, len(loc), len(glo)))
        li[i], gi[i] = loc, glo
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


DUMMY_FRAMES = 60   # dino_loss_loader.py:37-38: zeros(3, 60, crop, crop), 2 * global_clip_size of them


class FrameScorer:
    """Per-frame DINO-loss scores of a video with a (pretrained) dsvt TimeSformer.

    crop_size: the loader's center-crop size (dino_loss_loader.py:33, 92; 224 for the ViT-B
    checkpoints, default = the model's img_size).  A video whose frames are not crop_size^2
    takes the reference's dummy path (size_match, :103-107 and :115-123): its views are
    2 * global_clip_size all-zero clips of 60 frames, so the scoring loop yields
    global_clip_size identical scores -- DINO loss(model(zeros, local_clip_size frames),
    model(zeros, 60 frames)) -- whatever the video's length."""

    def __init__(self, model, local_clip_size=3, global_clip_size=30, teacher_temp=0.02, student_temp=0.3,
                 frames_per_call=8, crop_size=None):
        self.model = model
        self.local_clip_size = local_clip_size
        self.global_clip_size = global_clip_size
        self.loss = PairwiseDINOLoss(model.embed_dim, teacher_temp, student_temp).to(model.pos_embed.device)
        self.frames_per_call = frames_per_call
        # frame chunks on concurrent HIP streams (env DSVT_SCORE_STREAMS).  Bench video (64 frames, local 3 /
        # global 30), HIP graph, same box: 16 frames per call 376.4 / 377.5 frames/s on 2 streams vs
        # 367.4 / 367.5 on 1 and 373.7 / 374.1 on 4 (tools/r6_g15.sh); on 2 streams 8 frames per call
        # 383.5 / 384.0 vs 12: 379.9 / 383.5, 16: 374.9 / 376.6, 32: 380.6 / 381.5, 4: 338.2, and 8 on 3
        # streams 380.9 / 382.1 (tools/r6_g16.sh, r6_g17.sh)
        self.streams = 2
        self.crop_size = crop_size if crop_size is not None else model.patch_embed.img_size[0]
        self._views = {}
        # no LayerNorm folding: a frame's score is a difference of two close losses (the pairwise
        # DINO loss of its local and global views), so the fold's extra bf16 rounding of the
        # un-centred rows (error ~ sqrt(1 + mu^2 / sigma^2)) shows: bf16 scores measured 2.9e-2
        # of max vs the fp32 oracle with it, inside the 2e-2 bar without
        self.lnx = False

    @torch.no_grad()
    def dummy_scores(self, device):
        """The constant scores of a size-mismatched video (dino_similarity.py:73-90 over the
        dummy views): one score of the zero local / zero 60-frame global pair, repeated."""
        c = self.crop_size
        bank = torch.zeros(1, 3, c, c, device=device)
        ts = min(self.local_clip_size, DUMMY_FRAMES)
        st = self.model.forward_frame_bank(bank, torch.zeros(ts, dtype=torch.int32, device=device), 1, ts,
                                           lnx=self.lnx)
        te = self.model.forward_frame_bank(bank, torch.zeros(DUMMY_FRAMES, dtype=torch.int32, device=device), 1,
                                           DUMMY_FRAMES, lnx=self.lnx)
        return self.loss.per_row(st, te).expand(self.global_clip_size).contiguous()

    @torch.no_grad()
    def score(self, frames):
        """frames [F, 3, H, W] fp32 on the GPU -> scores fp32 (device): [F], or
        [global_clip_size] constant scores when H, W != crop_size (the dummy path)."""
        F = frames.shape[0]
        if tuple(frames.shape[-2:]) != (self.crop_size, self.crop_size):
            return self.dummy_scores(frames.device)
        dev = frames.device
        key = (F, dev)
        if key not in self._views:       # device index maps made once per video length (a HIP
            li, gi = view_index(F, self.local_clip_size, self.global_clip_size)    # graph replays them)
            self._views[key] = (li.shape[1], gi.shape[1], torch.from_numpy(li).to(dev), torch.from_numpy(gi).to(dev))
        ts, G, li_t, gi_t = self._views[key]
        frames = frames.float().contiguous()
        scores = torch.empty(F, device=dev, dtype=torch.float32)
        n = self.frames_per_call

        def chunk(s0):
            s1 = min(F, s0 + n)
            b = s1 - s0
            st = self.model.forward_frame_bank(frames, li_t[s0:s1].reshape(-1), b, ts, lnx=self.lnx)
            te = self.model.forward_frame_bank(frames, gi_t[s0:s1].reshape(-1), b, G, lnx=self.lnx)
            scores[s0:s1] = self.loss.per_row(st, te)
        starts = list(range(0, F, n))
        k = max(1, min(int(os.environ.get("DSVT_SCORE_STREAMS", self.streams)), len(starts)))
        from .utils import fork_depth
        if k > 1 and fork_depth() == 0:
            # the frame chunks are independent: k HIP streams, chunk i on stream i % k, so one
            # chunk's partly-filled last round of tiles runs beside another's full ones
            from .utils import prepare_weights, run_concurrent, stream_slot
            prepare_weights(self.model)           # weight copies and index maps made before the fork
            for t in (ts, G):
                self.model._indices(frames.shape[-2] // 16, frames.shape[-1] // 16, t, dev)
            groups = [starts[i::k] for i in range(k)]
            run_concurrent([(lambda g=g: [chunk(s0) for s0 in g]) for g in groups], dev,
                           slot0=("score", stream_slot(dev)))
        else:
            for s0 in starts:
                chunk(s0)
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
