"""Cluster-shape vocabulary: ``AcceleratorType``, ``MachineConfig``,
``COMMON_MACHINE_CONFIGS`` (API parity with reference
``TFC/core/machine_config.py:25-185``).

MI355X-first semantics:

* ``AMD_INSTINCT_MI355X`` is the native accelerator; ``accelerator_type="auto"``
  resolves to it (the reference resolved "auto" to a P100).
* The legacy NVIDIA names stay importable so existing scripts keep working;
  on an MI355X node any GPU-type request runs on the local MI355X GPUs (the
  launcher logs the substitution).  TPU types are accepted for validation only:
  there is no TPU analogue and ``run()`` rejects TPU workers with a clear error.
* ``accelerator_count`` is GPUs per machine (chief or worker); one process is
  spawned per GPU.
"""
from __future__ import annotations

import enum


class AcceleratorType(enum.Enum):
    NO_ACCELERATOR = "CPU"
    AMD_INSTINCT_MI355X = "MI355X"
    NVIDIA_TESLA_K80 = "K80"
    NVIDIA_TESLA_P100 = "P100"
    NVIDIA_TESLA_V100 = "V100"
    NVIDIA_TESLA_P4 = "P4"
    NVIDIA_TESLA_T4 = "T4"
    TPU_V2 = "TPU_V2"
    TPU_V3 = "TPU_V3"

    @classmethod
    def all(cls):
        return tuple(cls)

    @classmethod
    def gpus(cls):
        return (cls.AMD_INSTINCT_MI355X, cls.NVIDIA_TESLA_K80, cls.NVIDIA_TESLA_P100, cls.NVIDIA_TESLA_V100,
                cls.NVIDIA_TESLA_P4, cls.NVIDIA_TESLA_T4)

    @classmethod
    def validate(cls, key):
        if key not in cls.all():
            raise ValueError("Invalid accelerator key provided: %s." % (key,))

    @classmethod
    def from_value(cls, v):
        if isinstance(v, cls):
            return v
        for m in cls:
            if m.value == v or m.name == v:
                return m
        raise ValueError("Invalid accelerator key provided: %s." % (v,))


# Per-node limits of an MI355X platform (8 OAM GPUs, 288 GB HBM3E each).
MAX_GPUS_PER_NODE = 8
HBM_GB_PER_GPU = 288


class MachineConfig:
    """Configuration of one machine (the chief or one worker) of a job."""

    def __init__(self, cpu_cores=8, memory=30, accelerator_type="auto", accelerator_count=1):
        self.cpu_cores = cpu_cores
        self.memory = memory
        if accelerator_type == "auto":
            accelerator_type = AcceleratorType.AMD_INSTINCT_MI355X
        elif isinstance(accelerator_type, str):
            accelerator_type = AcceleratorType.from_value(accelerator_type)
        self.accelerator_type = accelerator_type
        self.accelerator_count = accelerator_count
        self.validate()

    def validate(self):
        AcceleratorType.validate(self.accelerator_type)
        validate_machine_configuration(self.cpu_cores, self.memory, self.accelerator_type, self.accelerator_count)

    @property
    def is_gpu(self):
        return self.accelerator_type in AcceleratorType.gpus() and self.accelerator_count > 0

    @property
    def num_processes(self):
        """Processes the launcher spawns for this machine (one per GPU, else one)."""
        return self.accelerator_count if self.is_gpu else 1

    def to_dict(self):
        return {"cpu_cores": self.cpu_cores, "memory": self.memory,
                "accelerator_type": self.accelerator_type.value, "accelerator_count": self.accelerator_count}

    def __eq__(self, other):
        return isinstance(other, MachineConfig) and self.to_dict() == other.to_dict()

    def __repr__(self):
        return ("MachineConfig(cpu_cores={cpu_cores}, memory={memory}, accelerator_type={accelerator_type}, "
                "accelerator_count={accelerator_count})".format(**self.to_dict()))


def validate_machine_configuration(cpu_cores, memory, accelerator_type, accelerator_count):
    """Local-node analogue of the GCP SKU check (reference ``TFC/core/gcp.py:35-70``)."""
    if accelerator_type in (AcceleratorType.TPU_V2, AcceleratorType.TPU_V3):
        if accelerator_count != 8:
            raise ValueError("Invalid machine configuration: TPU configs need accelerator_count=8. "
                             "Received {}.".format(accelerator_count))
        return
    if not isinstance(accelerator_count, int) or accelerator_count < 0:
        raise ValueError("Invalid machine configuration: accelerator_count must be a non-negative "
                         "integer. Received {}.".format(accelerator_count))
    if accelerator_type == AcceleratorType.NO_ACCELERATOR and accelerator_count != 0:
        raise ValueError("Invalid machine configuration: a CPU machine has accelerator_count=0. "
                         "Received {}.".format(accelerator_count))
    if accelerator_type in AcceleratorType.gpus():
        if accelerator_count < 1 or accelerator_count > MAX_GPUS_PER_NODE:
            raise ValueError("Invalid machine configuration: accelerator_count must be in [1, {}] for "
                             "{}. Received {}.".format(MAX_GPUS_PER_NODE, accelerator_type.value,
                                                       accelerator_count))
    for name, v in (("cpu_cores", cpu_cores), ("memory", memory)):
        if v is not None and (not isinstance(v, (int, float)) or v <= 0):
            raise ValueError("Invalid machine configuration: {} must be positive. Received {}."
                             .format(name, v))


def _mk(cpu, mem, t, n):
    return MachineConfig(cpu_cores=cpu, memory=mem, accelerator_type=t, accelerator_count=n)


_M = AcceleratorType.AMD_INSTINCT_MI355X
COMMON_MACHINE_CONFIGS = {
    "CPU": _mk(4, 15, AcceleratorType.NO_ACCELERATOR, 0),
    "MI355X_1X": _mk(16, 256, _M, 1),
    "MI355X_2X": _mk(32, 512, _M, 2),
    "MI355X_4X": _mk(64, 1024, _M, 4),
    "MI355X_8X": _mk(128, 2048, _M, 8),
    # legacy names (run on local MI355X GPUs)
    "K80_1X": _mk(8, 30, AcceleratorType.NVIDIA_TESLA_K80, 1),
    "K80_4X": _mk(16, 60, AcceleratorType.NVIDIA_TESLA_K80, 4),
    "K80_8X": _mk(32, 120, AcceleratorType.NVIDIA_TESLA_K80, 8),
    "P100_1X": _mk(8, 30, AcceleratorType.NVIDIA_TESLA_P100, 1),
    "P100_4X": _mk(16, 60, AcceleratorType.NVIDIA_TESLA_P100, 4),
    "P4_1X": _mk(8, 30, AcceleratorType.NVIDIA_TESLA_P4, 1),
    "P4_4X": _mk(16, 60, AcceleratorType.NVIDIA_TESLA_P4, 4),
    "V100_1X": _mk(8, 30, AcceleratorType.NVIDIA_TESLA_V100, 1),
    "V100_4X": _mk(16, 60, AcceleratorType.NVIDIA_TESLA_V100, 4),
    "T4_1X": _mk(8, 30, AcceleratorType.NVIDIA_TESLA_T4, 1),
    "T4_4X": _mk(16, 60, AcceleratorType.NVIDIA_TESLA_T4, 4),
    "TPU": _mk(None, None, AcceleratorType.TPU_V3, 8),
}


def is_tpu_config(config):
    return bool(config) and getattr(config, "accelerator_type", None) in (AcceleratorType.TPU_V2,
                                                                          AcceleratorType.TPU_V3)
