"""Native input pipeline (see :mod:`cloud_amd.data.loader`)."""
from .loader import DeviceLoader, NpyBatchLoader, write_npy_dataset  # noqa: F401
