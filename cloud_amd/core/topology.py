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


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"
# KFD io_link "type" values (hsakmttypes.h HSA_IOLINKTYPE_*): 2 = PCIe, 11 = xGMI.
IOLINK_PCIE, IOLINK_XGMI = 2, 11
# KFD mem_bank "heap_type": 1 = frame buffer public, 2 = frame buffer private (HBM).
_HBM_HEAPS = (1, 2)


def _read_props(path):
    out = {}
    try:
        with open(path) as f:
            for line in f:
                parts = line.split()
                if len(parts) == 2:
                    try:
                        out[parts[0]] = int(parts[1])
                    except ValueError:
                        out[parts[0]] = parts[1]
    except OSError:
        return None
    return out


def _subdirs(path):
    try:
        return sorted((d for d in os.listdir(path) if d.isdigit()), key=int)
    except OSError:
        return []


def kfd_root():
    """KFD topology root (``CLOUD_AMD_KFD_ROOT`` points tests at a fake tree)."""
    return os.environ.get("CLOUD_AMD_KFD_ROOT", KFD_NODES)


def kfd_gpu_nodes(root=None):
    """GPU agents from the KFD topology in sysfs, in HSA enumeration order.

    Reading sysfs never loads the HIP runtime, so the launcher can size a job
    before it forks any rank (the probe that replaces reference
    ``TFC/core/gcp.py:35-116``'s SKU tables).  Each entry: KFD node id,
    ``gfx_target_version`` (90500 = gfx950), SIMD and CU counts, HBM bytes and the
    xGMI / PCIe links to other KFD nodes (with KFD's link bandwidth fields)."""
    root = root or kfd_root()
    gpus = []
    for nid in _subdirs(root):
        node = os.path.join(root, nid)
        props = _read_props(os.path.join(node, "properties"))
        if not props or int(props.get("simd_count", 0)) <= 0:
            continue  # CPU agent
        hbm = 0
        for b in _subdirs(os.path.join(node, "mem_banks")):
            bp = _read_props(os.path.join(node, "mem_banks", b, "properties")) or {}
            if bp.get("heap_type") in _HBM_HEAPS:
                hbm += int(bp.get("size_in_bytes", 0))
        links = []
        for l in _subdirs(os.path.join(node, "io_links")):
            lp = _read_props(os.path.join(node, "io_links", l, "properties")) or {}
            links.append({"type": lp.get("type"), "to": lp.get("node_to"), "weight": lp.get("weight"),
                          "min_bandwidth": lp.get("min_bandwidth"), "max_bandwidth": lp.get("max_bandwidth")})
        simds = int(props.get("simd_count", 0))
        gpus.append({"node": int(nid), "gfx_target_version": props.get("gfx_target_version"),
                     "simd_count": simds, "cu_count": simds // max(int(props.get("simd_per_cu", 4)), 1),
                     "hbm_bytes": hbm, "unique_id": props.get("unique_id"),
                     "location_id": props.get("location_id"), "links": links})
    return gpus


def _visible_filter(n):
    """Indices kept by ``ROCR/HIP/CUDA_VISIBLE_DEVICES`` out of ``n`` enumerated GPUs."""
    idx = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        sel = [x.strip() for x in v.split(",") if x.strip() != ""]
        picked = []
        for s in sel:
            if s.isdigit() and int(s) < len(idx):
                picked.append(idx[int(s)])
            elif not s.isdigit():  # UUID-style selector: cannot be mapped without HIP; keep count
                picked.append(len(picked))
        idx = picked
    return idx


def visible_gpus(root=None):
    """The KFD GPU entries this process may use (visibility env applied)."""
    nodes = kfd_gpu_nodes(root)
    return [nodes[i] for i in _visible_filter(len(nodes)) if i < len(nodes)]


def visible_gpu_count(root=None) -> int:
    """Number of usable GPUs, from KFD sysfs (never initialises HIP).

    ``CLOUD_AMD_NUM_GPUS`` overrides (tests, dry runs).  Without a KFD topology
    (CPU container) the count is 0 unless a visibility variable names devices."""
    env = os.environ.get("CLOUD_AMD_NUM_GPUS")
    if env is not None:
        return int(env)
    nodes = kfd_gpu_nodes(root)
    if nodes:
        return len(visible_gpus(root))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None and v.strip() != "":
            return len([x for x in v.split(",") if x.strip() != ""])
    return 0


def hbm_gb_per_gpu(root=None) -> float:
    """HBM per GPU in GiB (the "288 GB" of the MI355X datasheet is 288 GiB): measured
    from the KFD memory banks when present, else the MI355X constant."""
    env = os.environ.get("CLOUD_AMD_HBM_GB")
    if env is not None:
        return float(env)
    gpus = visible_gpus(root)
    sizes = [g["hbm_bytes"] for g in gpus if g["hbm_bytes"] > 0]
    if sizes:
        return min(sizes) / 2**30
    return float(HBM_GB_PER_GPU)


def xgmi_matrix(root=None):
    """Visible-GPU x visible-GPU matrix of direct xGMI links (1 = link present)."""
    gpus = visible_gpus(root)
    ids = {g["node"]: i for i, g in enumerate(gpus)}
    m = [[0] * len(gpus) for _ in gpus]
    for i, g in enumerate(gpus):
        for l in g["links"]:
            if l["type"] == IOLINK_XGMI and l["to"] in ids:
                m[i][ids[l["to"]]] = 1
    return m


def xgmi_links_per_gpu(n_gpus: int, root=None) -> int:
    """Point-to-point xGMI links a GPU can use in a collective among ``n_gpus``.

    Measured from the KFD link table when it covers the job's GPUs (minimum over
    the first ``n_gpus`` visible GPUs); otherwise the MI355X full mesh (n-1)."""
    m = xgmi_matrix(root)
    if len(m) >= n_gpus > 0 and any(any(r) for r in m):
        return min(sum(m[i][:n_gpus]) for i in range(n_gpus))
    return max(0, min(n_gpus, 8) - 1)


def describe_node(root=None):
    gpus = visible_gpus(root)
    n = visible_gpu_count(root)
    info = {"gpus": n, "hbm_gb_per_gpu": round(hbm_gb_per_gpu(root), 1), "source": "kfd" if gpus else "constants"}
    gfx = {g["gfx_target_version"] for g in gpus}
    info["gfx_target_version"] = sorted(gfx)[0] if len(gfx) == 1 else sorted(gfx)
    info["arch"] = "gfx950" if gfx == {90500} or not gpus else "gfx%s" % sorted(gfx)
    info["cu_per_gpu"] = gpus[0]["cu_count"] if gpus else None
    info["xgmi_links_per_gpu"] = xgmi_links_per_gpu(n, root)
    info["xgmi_matrix"] = xgmi_matrix(root) if gpus else None
    return info


def rocm_smi_product():
    """Product names from rocm-smi (optional, diagnostics only)."""
    try:
        out = subprocess.run(["rocm-smi", "--showproductname"], capture_output=True, text=True, timeout=10)
        return out.stdout.strip().splitlines()[-3:] if out.returncode == 0 else None
    except Exception:
        return None


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
