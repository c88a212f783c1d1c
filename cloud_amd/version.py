"""Version of cloud_amd (API parity target: tensorflow_cloud 0.1.7.dev, ``TFC/version.py:16``)."""
__version__ = "0.1.0"
ARCH = "gfx950"
