"""Hand-written HIP/CDNA4 ops with PyTorch references (used on CPU and in numerics tests)."""
from .explore import explore_postprocess, explore_postprocess_reference, normalize_slices_reference
from .optim import FlatParams, FusedAdamPolyak, adam_polyak_reference
