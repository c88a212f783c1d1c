"""Fused optimizers over flat parameter arenas (see :mod:`cloud_amd.optim.arena`)."""
from .arena import Arena, build_arenas, zero_grads  # noqa: F401
from .fused import SGD, Adam, AdamW, FusedOptimizer, RMSprop, get  # noqa: F401
