"""Local node topology + job-label rules (replaces reference ``TFC/core/gcp.py``).

The reference mapped MachineConfigs onto GCP SKUs and regions.  On an MI355X
node the questions are: how many GPUs are visible, how much HBM each has, and
how they are wired (xGMI full mesh: 7 links per GPU).  Everything here avoids
initialising the GPU in the launcher process (device counting does not, on
this ROCm image), so spawned ranks own their devices.
"""
from __future__ import annotations

import os
import re
import subprocess

from .machine_config import HBM_GB_PER_GPU, AcceleratorType


def get_region():
    """Where jobs run: always the local node."""
    return os.environ.get("CLOUD_AMD_REGION", "local")


def get_project_name():
    return os.environ.get("CLOUD_AMD_PROJECT", "local")


def visible_gpu_count() -> int:
    env = os.environ.get("CLOUD_AMD_NUM_GPUS")
    if env is not None:
        return int(env)
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None and v.strip() != "":
            return len([x for x in v.split(",") if x.strip() != ""])
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # pragma: no cover
        return 0


def hbm_gb_per_gpu() -> float:
    return float(os.environ.get("CLOUD_AMD_HBM_GB", HBM_GB_PER_GPU))


def xgmi_links_per_gpu(n_gpus: int) -> int:
    """Point-to-point xGMI links usable by a collective among n_gpus (full mesh)."""
    return max(0, min(n_gpus, 8) - 1)


def describe_node():
    info = {"gpus": visible_gpu_count(), "hbm_gb_per_gpu": hbm_gb_per_gpu(), "arch": "gfx950"}
    info["xgmi_links_per_gpu"] = xgmi_links_per_gpu(info["gpus"])
    try:
        out = subprocess.run(["rocm-smi", "--showproductname"], capture_output=True, text=True, timeout=10)
        info["rocm_smi"] = out.stdout.strip().splitlines()[-3:] if out.returncode == 0 else None
    except Exception:
        info["rocm_smi"] = None
    return info


def get_accelerator_type(t: AcceleratorType) -> str:
    return t.value


def get_machine_type(cpu_cores, memory, accelerator_type) -> str:
    """A descriptive machine label for job metadata (reference gcp.py:93-116)."""
    if accelerator_type in (AcceleratorType.TPU_V2, AcceleratorType.TPU_V3):
        return "cloud_tpu"
    return "local-{}c-{}g".format(cpu_cores, memory)


_LABEL_RE = re.compile(r"^[a-z0-9_-]+$")


def validate_job_labels(job_labels):
    """Label rules kept from reference ``TFC/core/gcp.py:409-481`` (labels go to job.json)."""
    if not job_labels:
        print("No labels provided for the training job. Please consider creating labels to help "
              "with retrieval of job information (they are recorded in the job's job.json).")
    if len(job_labels) > 64:
        raise ValueError("Invalid job labels: too many labels. Expecting at most 64 labels. "
                         "Received {}.".format(len(job_labels)))
    for k, v in job_labels.items():
        if not k or not k[0].islower():
            raise ValueError("Invalid job labels: Label key must start with lowercase letters. "
                             "Received {}.".format(k))
        if not v or not v[0].islower():
            raise ValueError("Invalid job labels: Label value must start with lowercase letters. "
                             "Received {}.".format(v))
        if len(k) > 63:
            raise ValueError("Invalid job labels: Label key is too long. Expecting at most 63 characters. "
                             "Received {}.".format(k))
        if len(v) > 63:
            raise ValueError("Invalid job labels: Label value is too long for key {}. Expecting at most 63 "
                             "characters. Received {}.".format(k, v))
        if not _LABEL_RE.match(k):
            raise ValueError("Invalid job labels: Label key can only contain lowercase letters, numeric "
                             "characters, underscores and dashes. Received: {}.".format(k))
        if not _LABEL_RE.match(v):
            raise ValueError("Invalid job labels: Label value can only contain lowercase letters, numeric "
                             "characters, underscores and dashes. Received: {}.".format(v))
