"""Native gfx950 ops (HIP kernels in csrc/kernels) with autograd support."""
from .functional import (  # noqa: F401
    augment, batch_norm_act, cast_bf16_, checksum, conv2d, cross_entropy, global_avg_pool, linear, max_pool2d,
    sgd_flat_, weight_bf16,
)
from ._lib import available as native_available  # noqa: F401
