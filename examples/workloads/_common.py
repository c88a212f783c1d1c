"""Shared knobs for the ported reference workloads (sizes shrink under tests)."""
import os

SMALL = os.environ.get("CLOUD_AMD_EXAMPLE_SMALL") == "1"


def n(full, small):
    return small if SMALL else full
