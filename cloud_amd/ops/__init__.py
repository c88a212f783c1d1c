"""MI355X compute ops: HIP/CDNA4 kernels with PyTorch reference fallbacks.

Every op takes NHWC activations, dispatches CUDA(HIP) tensors to the gfx950
kernels in ``cloud_amd/_C*.so`` and CPU tensors to an fp32-faithful PyTorch
reference (see :mod:`cloud_amd.ops._ext` for the fail-loudly policy).
"""
from ._ext import load as load_extension, ops_mode, use_native  # noqa: F401
from .batchnorm import bn_act  # noqa: F401
from .conv import conv2d_nhwc  # noqa: F401
from .gemm import linear  # noqa: F401
from .losses import backward_with_seed, softmax_cross_entropy, unit_seed  # noqa: F401
from .pooling import global_avg_pool_nhwc, global_max_pool_nhwc, max_pool2d_nhwc  # noqa: F401
from .dropout import dropout  # noqa: F401
