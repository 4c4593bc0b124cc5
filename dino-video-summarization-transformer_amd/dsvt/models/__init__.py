"""Drop-in for the reference's `models` package (models/__init__.py:1-3)."""
from .swin_transformer import SwinTransformer3D  # noqa: F401
from .timesformer import (TimeSformer, VisionTransformer, get_vit_base_patch16_224,  # noqa: F401
                          set_default_dtype, vit_base_patch16_224)


def get_aux_token_vit(cfg, no_head=False, **kwargs):
    """models/timesformer.py:612-628 -- the two-token research variant is OUT OF SCOPE
    (SURVEY §2.1); it also always fetches weights from a URL in the reference."""
    raise NotImplementedError("get_aux_token_vit (two-token variant) is out of scope for dsvt")
