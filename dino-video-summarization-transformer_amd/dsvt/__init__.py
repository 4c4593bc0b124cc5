"""dsvt -- MI355X-native (gfx950) DINO-SVT forward/loss hot path.

Host-side mirror of the reference's module API (models/, vision_transformer.py,
train_ssl.DINOLoss, dino_similarity.DINOLoss, utils.MultiCropWrapper) over the C-ABI
library libdsvt.so (include/dsvt.h).  No CPU or eager-PyTorch fallback exists: every op
raises when the HIP library or a GPU is missing.
"""
from . import _lib, ops  # noqa: F401
from ._lib import DsvtError  # noqa: F401

__version__ = "0.1.0"
