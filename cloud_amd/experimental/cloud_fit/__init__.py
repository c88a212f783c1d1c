"""``cloud_fit``: run ``model.fit`` for an in-memory model as a distributed job on this node."""
from .client import cloud_fit  # noqa: F401
