"""Model zoo: the reference workloads re-built on cloud_amd NHWC ops."""
from .resnet import ResNet, resnet50  # noqa: F401
from .bert import BertConfig, BertForSequenceClassification, bert_base  # noqa: F401
