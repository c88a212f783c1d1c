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


NUMA_ROOT = "/sys/devices/system/node"
CPU_ROOT = "/sys/devices/system/cpu"


def parse_cpulist(text):
    """Kernel cpulist syntax -> sorted ints: ``"0-3,8,10-11"`` -> [0, 1, 2, 3, 8, 10, 11]."""
    out = set()
    for part in (text or "").strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            out.update(range(int(lo), int(hi) + 1))
        else:
            out.add(int(part))
    return sorted(out)


def format_cpulist(cpus):
    """Sorted ints -> kernel cpulist syntax: [0, 1, 2, 5] -> ``"0-2,5"``."""
    cpus, out, i = sorted(cpus), [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else "%d-%d" % (cpus[i], cpus[j]))
        i = j + 1
    return ",".join(out)


def _cpu_agents(root):
    """KFD CPU agents in enumeration order: [(kfd node id, props)].  KFD creates one CPU
    agent per NUMA node, in NUMA order, so the k-th agent is NUMA node k."""
    out = []
    for nid in _subdirs(root):
        props = _read_props(os.path.join(root, nid, "properties"))
        if props and int(props.get("simd_count", 0)) == 0 and int(props.get("cpu_cores_count", 0)) > 0:
            out.append((int(nid), props))
    return out


def _links(root, nid):
    out = []
    for l in _subdirs(os.path.join(root, str(nid), "io_links")):
        lp = _read_props(os.path.join(root, str(nid), "io_links", l, "properties")) or {}
        if "node_to" in lp:
            out.append(lp)
    return out


def gpu_numa_nodes(root=None):
    """NUMA node of every visible GPU (None when unknown), from the KFD link table: the
    GPU's own PCIe link to a CPU agent, or else a CPU agent's link to the GPU (a job that
    sees one GPU of eight can read every CPU agent's links but only its own GPU's)."""
    root = root or kfd_root()
    cpus = _cpu_agents(root)
    numa_of_agent = {nid: k for k, (nid, _) in enumerate(cpus)}
    out = []
    for g in visible_gpus(root):
        numa = None
        for l in _links(root, g["node"]):
            if l.get("node_to") in numa_of_agent:
                numa = numa_of_agent[l["node_to"]]
                break
        if numa is None:
            for nid, _ in cpus:
                if any(l.get("node_to") == g["node"] for l in _links(root, nid)):
                    numa = numa_of_agent[nid]
                    break
        out.append(numa)
    return out


def numa_cpus(numa, root=None, kfd=None):
    """Logical CPUs of NUMA node ``numa``: sysfs ``node<k>/cpulist``, else the KFD CPU
    agent's ``cpu_core_id_base`` + ``cpu_cores_count``."""
    root = root or os.environ.get("CLOUD_AMD_NUMA_ROOT", NUMA_ROOT)
    try:
        with open(os.path.join(root, "node%d" % numa, "cpulist")) as f:
            cpus = parse_cpulist(f.read())
        if cpus:
            return cpus
    except OSError:
        pass
    agents = _cpu_agents(kfd or kfd_root())
    if numa < len(agents):
        p = agents[numa][1]
        base = int(p.get("cpu_core_id_base", 0))
        return list(range(base, base + int(p.get("cpu_cores_count", 0))))
    return []


def _cores(cpus, cpu_root=None):
    """Group logical CPUs into physical cores (SMT siblings together), ordered by first id."""
    cpu_root = cpu_root or os.environ.get("CLOUD_AMD_CPU_ROOT", CPU_ROOT)
    allowed, seen, cores = set(cpus), set(), []
    for c in sorted(cpus):
        if c in seen:
            continue
        sib = None
        try:
            with open(os.path.join(cpu_root, "cpu%d" % c, "topology", "thread_siblings_list")) as f:
                sib = [x for x in parse_cpulist(f.read()) if x in allowed]
        except OSError:
            pass
        core = sorted(set(sib or []) | {c})
        seen.update(core)
        cores.append(core)
    return cores


def rank_cpu_sets(gpus, root=None, numa_root=None, cpu_root=None, allowed=None):
    """CPU set for each rank of a job whose ranks drive visible GPUs ``gpus`` (list of
    visible-GPU indices, one per rank; None for a CPU rank): the cores of the GPU's NUMA
    node, split into disjoint contiguous groups of whole physical cores among the ranks on
    that node (4 ranks per socket on an 8x MI355X node), intersected with the CPUs this
    process may use.  None for a rank whose placement is unknown (no KFD / NUMA data)."""
    if allowed is None:
        try:
            allowed = set(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            allowed = None
    numa = gpu_numa_nodes(root)
    per_node = {}
    for r, g in enumerate(gpus):
        n = numa[g] if g is not None and g < len(numa) else None
        if n is not None:
            per_node.setdefault(n, []).append(r)
    out = [None] * len(gpus)
    for n, ranks in per_node.items():
        cpus = numa_cpus(n, numa_root, kfd=root)
        if allowed is not None:
            cpus = [c for c in cpus if c in allowed]
        cores = _cores(cpus, cpu_root)
        if len(cores) < len(ranks):
            continue  # fewer cores than ranks: leave placement to the scheduler
        k = len(ranks)
        for i, r in enumerate(ranks):
            lo, hi = i * len(cores) // k, (i + 1) * len(cores) // k
            out[r] = sorted(c for core in cores[lo:hi] for c in core)
    return out


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
