"""Drop-in for utils.utils.MultiCropWrapper (utils/utils.py:564-609)."""
import torch
import torch.nn as nn


class MultiCropWrapper(nn.Module):
    """Runs the backbone once per group of consecutive same-resolution crops and the head once
    on all features.  Unlike the reference it does not torch.cat the crops: the dsvt backbone
    takes the group as a list and writes every crop's tokens straight into one token tensor,
    and the features of all groups land in one preallocated buffer."""

    def __init__(self, backbone, head, vary_fr=False):
        super().__init__()
        if hasattr(backbone, 'fc'):
            backbone.fc, backbone.head = nn.Identity(), nn.Identity()
        self.backbone = backbone
        self.head = head
        self.vary_fr = vary_fr

    def forward(self, x, **kwargs):
        if not isinstance(x, list):
            x = [x]
        sizes = [inp.shape[-1] for inp in x]
        if self.vary_fr:                                   # utils/utils.py:588-592
            if len(x) == 10:
                idx_crops = [1, 2, 4, 6, 8, 10]
            elif len(x) == 2:
                idx_crops = [1, 2]
            else:
                raise ValueError("vary_fr supports 2 or 10 crops")
        else:                                              # unique_consecutive on widths (:584-587)
            idx_crops = []
            for i in range(1, len(sizes) + 1):
                if i == len(sizes) or sizes[i] != sizes[i - 1]:
                    idx_crops.append(i)
        total = sum(inp.shape[0] for inp in x)
        feats = torch.empty(total, self.backbone.embed_dim, device=x[0].device, dtype=torch.float32)
        start, row = 0, 0
        for end in idx_crops:
            group = x[start:end]
            n = sum(g.shape[0] for g in group)
            self.backbone.forward_features(group, out=feats[row:row + n], **kwargs)
            row += n
            start = end
        return self.head(feats)
