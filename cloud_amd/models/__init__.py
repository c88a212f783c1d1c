"""Model zoo: the reference workloads re-built on cloud_amd NHWC ops."""
from .resnet import ResNet, resnet50  # noqa: F401
