"""Machine configs, validation and job labels (parity: reference
core/tests/unit/{validate,gcp}_test.py expectations, adapted to a local MI355X node)."""
import os

import pytest

from cloud_amd.core import machine_config as mc
from cloud_amd.core import topology, validate


def test_accelerator_enum_and_auto():
    assert mc.AcceleratorType.AMD_INSTINCT_MI355X.value == "MI355X"
    assert mc.AcceleratorType.NO_ACCELERATOR in mc.AcceleratorType.all()
    with pytest.raises(ValueError, match="Invalid accelerator key"):
        mc.AcceleratorType.validate("H100")
    cfg = mc.MachineConfig()
    assert cfg.accelerator_type == mc.AcceleratorType.AMD_INSTINCT_MI355X
    assert cfg.accelerator_count == 1 and cfg.is_gpu and cfg.num_processes == 1


def test_common_configs():
    c = mc.COMMON_MACHINE_CONFIGS
    for k in ("CPU", "MI355X_1X", "MI355X_2X", "MI355X_4X", "MI355X_8X", "T4_1X", "V100_4X", "TPU"):
        assert k in c
    assert c["MI355X_8X"].accelerator_count == 8 and c["MI355X_8X"].num_processes == 8
    assert c["CPU"].accelerator_count == 0 and not c["CPU"].is_gpu and c["CPU"].num_processes == 1
    assert mc.is_tpu_config(c["TPU"]) and not mc.is_tpu_config(c["MI355X_1X"])


@pytest.mark.parametrize("kw,msg", [
    (dict(accelerator_type=mc.AcceleratorType.NO_ACCELERATOR, accelerator_count=2), "CPU machine"),
    (dict(accelerator_type="MI355X", accelerator_count=9), r"\[1, 8\]"),
    (dict(accelerator_type="MI355X", accelerator_count=0), r"\[1, 8\]"),
    (dict(cpu_cores=-1), "cpu_cores"),
])
def test_invalid_machine_configs(kw, msg):
    with pytest.raises(ValueError, match=msg):
        mc.MachineConfig(**kw)


def _ok_kwargs(tmp_path, **over):
    kw = dict(entry_point=None, requirements_txt=None, distribution_strategy="auto",
              chief_config=mc.COMMON_MACHINE_CONFIGS["MI355X_1X"], worker_config=mc.COMMON_MACHINE_CONFIGS["MI355X_1X"],
              worker_count=0, region="local", entry_point_args=None, stream_logs=False,
              docker_image_bucket_name=None, called_from_notebook=False)
    kw.update(over)
    return kw


def test_validate_ok(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    (tmp_path / "train.py").write_text("print(1)\n")
    (tmp_path / "req.txt").write_text("numpy\n")
    validate.validate(**_ok_kwargs(tmp_path, entry_point="train.py", requirements_txt="req.txt"))
    validate.validate(**_ok_kwargs(tmp_path, distribution_strategy=None))


@pytest.mark.parametrize("over,err", [
    (dict(entry_point="missing.py"), r"Invalid `entry_point`"),
    (dict(requirements_txt="nope.txt"), r"Invalid `requirements_txt`"),
    (dict(distribution_strategy="Mirrored"), r"Invalid `distribution_strategy`"),
    (dict(chief_config="gpu"), r"Invalid `chief_config`"),
    (dict(worker_count=-1), r"Invalid `worker_count`"),
    (dict(worker_count=1, worker_config=None), r"Invalid `worker_config`"),
    (dict(chief_config=mc.COMMON_MACHINE_CONFIGS["TPU"]), r"Invalid `chief_config`"),
    (dict(region=3), r"Invalid `region`"),
    (dict(entry_point_args="--x"), r"Invalid `entry_point_args`"),
    (dict(stream_logs="yes"), r"Invalid `stream_logs`"),
])
def test_validate_errors(tmp_path, monkeypatch, over, err):
    monkeypatch.chdir(tmp_path)
    with pytest.raises(ValueError, match=err):
        validate.validate(**_ok_kwargs(tmp_path, **over))


def test_validate_bad_suffix(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    (tmp_path / "train.txt").write_text("x")
    with pytest.raises(ValueError, match="Expected a python file or an iPython notebook"):
        validate.validate(**_ok_kwargs(tmp_path, entry_point="train.txt"))


def test_tpu_worker_rejected(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    with pytest.raises(ValueError, match="Expected worker_count=1"):
        validate.validate(**_ok_kwargs(tmp_path, worker_count=2, worker_config=mc.COMMON_MACHINE_CONFIGS["TPU"]))
    with pytest.raises(NotImplementedError):
        validate.validate(**_ok_kwargs(tmp_path, worker_count=1, worker_config=mc.COMMON_MACHINE_CONFIGS["TPU"]))


def test_node_capacity():
    c8 = mc.COMMON_MACHINE_CONFIGS["MI355X_8X"]
    validate.validate_node_capacity(c8, None, 0, available=8)
    with pytest.raises(ValueError, match="needs 16 GPUs"):
        validate.validate_node_capacity(c8, c8, 1, available=8)
    validate.validate_node_capacity(mc.COMMON_MACHINE_CONFIGS["CPU"], mc.COMMON_MACHINE_CONFIGS["CPU"], 3,
                                    available=0)


@pytest.mark.parametrize("labels,err", [
    ({"Key": "v"}, "Label key must start with lowercase"),
    ({"k": "V"}, "Label value must start with lowercase"),
    ({"k" * 64: "v"}, "Label key is too long"),
    ({"k": "v" * 64}, "Label value is too long"),
    ({"k.x": "v"}, "Label key can only contain"),
    ({"k": "v!"}, "Label value can only contain"),
    ({f"k{i}": "v" for i in range(65)}, "too many labels"),
])
def test_job_label_errors(labels, err):
    with pytest.raises(ValueError, match=err):
        topology.validate_job_labels(labels)


def test_job_labels_ok(capsys):
    topology.validate_job_labels({"team": "vision", "run_1": "a-b"})
    topology.validate_job_labels({})
    assert "No labels provided" in capsys.readouterr().out


def test_topology_counts(monkeypatch):
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "8")
    assert topology.visible_gpu_count() == 8
    monkeypatch.delenv("CLOUD_AMD_NUM_GPUS")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,3")
    assert topology.visible_gpu_count() == 2
    assert topology.xgmi_links_per_gpu(8) == 7
    assert topology.get_region() == os.environ.get("CLOUD_AMD_REGION", "local")


def _fake_kfd(root, n_gpus=8, hbm=288 * 2**30, mesh=True):
    """A KFD topology tree shaped like an 8x MI355X node: 2 CPU agents, then GPUs."""
    def write(path, props):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write("".join("%s %s\n" % kv for kv in props.items()))

    for c in range(2):
        write(os.path.join(root, str(c), "properties"), {"cpu_cores_count": 64, "simd_count": 0})
    for g in range(n_gpus):
        nid = 2 + g
        base = os.path.join(root, str(nid))
        write(os.path.join(base, "properties"), {"cpu_cores_count": 0, "simd_count": 1024, "simd_per_cu": 4,
                                                 "gfx_target_version": 90500, "unique_id": 1000 + g})
        write(os.path.join(base, "mem_banks", "0", "properties"), {"heap_type": 1, "size_in_bytes": hbm})
        links = [(2, g // 4)]  # PCIe link to its CPU agent
        if mesh:
            links += [(11, 2 + o) for o in range(n_gpus) if o != g]
        for i, (t, to) in enumerate(links):
            write(os.path.join(base, "io_links", str(i), "properties"),
                  {"type": t, "node_from": nid, "node_to": to, "weight": 15, "max_bandwidth": 153000})


def test_topology_kfd_probe(tmp_path, monkeypatch):
    for v in ("CLOUD_AMD_NUM_GPUS", "CLOUD_AMD_HBM_GB", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
              "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    root = str(tmp_path / "nodes")
    _fake_kfd(root)
    gpus = topology.kfd_gpu_nodes(root)
    assert [g["node"] for g in gpus] == list(range(2, 10))
    assert gpus[0]["cu_count"] == 256 and gpus[0]["gfx_target_version"] == 90500
    assert topology.visible_gpu_count(root) == 8
    assert abs(topology.hbm_gb_per_gpu(root) - 288.0) < 1e-6
    assert topology.xgmi_links_per_gpu(8, root) == 7
    assert topology.xgmi_links_per_gpu(4, root) == 3
    info = topology.describe_node(root)
    assert info["source"] == "kfd" and info["arch"] == "gfx950" and len(info["xgmi_matrix"]) == 8
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1,5,6")
    assert topology.visible_gpu_count(root) == 3
    assert [g["node"] for g in topology.visible_gpus(root)] == [3, 7, 8]
    assert topology.xgmi_links_per_gpu(3, root) == 2


def test_topology_kfd_no_mesh_falls_back(tmp_path, monkeypatch):
    for v in ("CLOUD_AMD_NUM_GPUS", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    root = str(tmp_path / "nodes")
    _fake_kfd(root, n_gpus=1, mesh=False)
    assert topology.visible_gpu_count(root) == 1
    assert topology.xgmi_links_per_gpu(1, root) == 0
    assert topology.visible_gpu_count(str(tmp_path / "missing")) == 0


def test_topology_real_mi355x_box_dump(monkeypatch):
    """KFD tree dumped on a gpurun box (an 8x MI355X node of which one GPU is exposed to
    the job: the other GPU nodes' properties are unreadable). Links of type 11 = xGMI."""
    for v in ("CLOUD_AMD_NUM_GPUS", "CLOUD_AMD_HBM_GB", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
              "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    root = os.path.join(os.path.dirname(__file__), "data", "kfd_mi355x_1of8")
    gpus = topology.kfd_gpu_nodes(root)
    assert len(gpus) == 1 and gpus[0]["gfx_target_version"] == 90500 and gpus[0]["cu_count"] == 256
    assert abs(topology.hbm_gb_per_gpu(root) - 288.0) < 0.5
    assert sum(1 for l in gpus[0]["links"] if l["type"] == topology.IOLINK_XGMI) == 7
    assert topology.xgmi_links_per_gpu(1, root) == 0


def _full_node_tree(tmp_path):
    """The real 1-of-8 KFD dump completed to all eight GPUs (the job that dumped it could
    read only its own GPU node's properties; the CPU agents' links, which decide NUMA
    placement, are all real), plus a fake sysfs NUMA / SMT tree: 2 sockets x 8 cores x 2
    threads (cpus n and n+32 are siblings)."""
    import shutil

    src = os.path.join(os.path.dirname(__file__), "data", "kfd_mi355x_1of8")
    kfd = tmp_path / "kfd"
    shutil.copytree(src, kfd)
    gpu_props = (kfd / "6" / "properties").read_text()
    for g in (2, 3, 4, 5, 7, 8, 9):
        (kfd / str(g) / "properties").write_text(gpu_props)
    numa = tmp_path / "node"
    cpu = tmp_path / "cpu"
    for k in range(2):
        (numa / ("node%d" % k)).mkdir(parents=True)
        (numa / ("node%d" % k) / "cpulist").write_text("%d-%d,%d-%d\n" % (16 * k, 16 * k + 15, 32 + 16 * k,
                                                                           32 + 16 * k + 15))
    for c in range(64):
        d = cpu / ("cpu%d" % c) / "topology"
        d.mkdir(parents=True)
        base = c % 32
        d.joinpath("thread_siblings_list").write_text("%d,%d\n" % (base, base + 32))
    return str(kfd), str(numa), str(cpu)


def test_rank_cpu_sets_eight_mi355x_ranks(tmp_path, monkeypatch):
    """each rank pinned to the cores local to its GPU.  KFD CPU agent 0
    (NUMA 0) links GPUs 2-5, agent 1 (NUMA 1) GPUs 6-9: ranks 0-3 split socket 0's cores,
    ranks 4-7 socket 1's, whole physical cores (both SMT threads) per rank, disjoint."""
    for v in ("CLOUD_AMD_NUM_GPUS", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    kfd, numa, cpu = _full_node_tree(tmp_path)
    monkeypatch.setenv("CLOUD_AMD_KFD_ROOT", kfd)
    monkeypatch.setenv("CLOUD_AMD_NUMA_ROOT", numa)
    monkeypatch.setenv("CLOUD_AMD_CPU_ROOT", cpu)
    assert topology.visible_gpu_count() == 8
    assert topology.gpu_numa_nodes() == [0, 0, 0, 0, 1, 1, 1, 1]
    sets = topology.rank_cpu_sets(list(range(8)), allowed=set(range(64)))
    want = []
    for k in range(2):
        for i in range(4):
            cores = list(range(16 * k + 4 * i, 16 * k + 4 * i + 4))
            want.append(sorted(cores + [c + 32 for c in cores]))
    assert sets == want
    assert topology.format_cpulist(sets[5]) == "20-23,52-55"
    # a restricted launcher (cgroup / taskset) only hands out CPUs it may use
    allowed = set(range(0, 8)) | set(range(32, 40)) | set(range(16, 32)) | set(range(48, 64))
    sets = topology.rank_cpu_sets(list(range(8)), allowed=allowed)
    assert sets[0] == [0, 1, 32, 33] and sets[3] == [6, 7, 38, 39] and sets[4] == want[4]
    # one GPU visible (the box the dump came from: KFD node 6 = NUMA 1)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "4")
    assert topology.gpu_numa_nodes() == [1]
    assert topology.rank_cpu_sets([0], allowed=set(range(64))) == [sorted(list(range(16, 32)) + list(range(48, 64)))]


def test_rank_cpu_sets_from_the_real_dump_alone(monkeypatch):
    """Only the real dump (no sysfs NUMA tree for it): the one visible GPU (KFD node 6)
    hangs off CPU agent 1, whose KFD cpu_core_id_base / cpu_cores_count give cores 128-255."""
    for v in ("CLOUD_AMD_NUM_GPUS", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    root = os.path.join(os.path.dirname(__file__), "data", "kfd_mi355x_1of8")
    monkeypatch.setenv("CLOUD_AMD_NUMA_ROOT", "/nonexistent")
    monkeypatch.setenv("CLOUD_AMD_CPU_ROOT", "/nonexistent")
    assert topology.gpu_numa_nodes(root) == [1]
    assert topology.rank_cpu_sets([0], root=root, allowed=set(range(512))) == [list(range(128, 256))]
    assert topology.rank_cpu_sets([None], root=root, allowed=set(range(512))) == [None]
