"""Entry-point wrapper generation with automatic strategy selection.

Parity: reference ``TFC/core/preprocess.py:38-212``.  The generated wrapper

1. marks the process as remote (``TF_KERAS_RUNNING_REMOTELY=1`` for scripts
   written against the reference, plus ``CLOUD_AMD_RUNNING_REMOTELY=1``), so a
   ``run()`` call inside the user script becomes a no-op;
2. (``distribution_strategy="auto"``) installs a global strategy chosen from
   the cluster shape exactly as the reference does -- workers > 0 ->
   MultiWorkerMirrored, chief GPUs > 1 -> Mirrored, else OneDevice -- but
   OneDevice targets the CPU when the chief has no accelerator (the reference
   emitted ``/gpu:0`` even for CPU chiefs, relying on soft placement);
3. executes the user code: ``exec`` of the script, or the code cells of a
   notebook (read from the .ipynb JSON directly; lines starting with ``!``,
   ``%`` or ``#`` are dropped as in the reference).
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

from . import machine_config

HEADER = [
    "import os\n",
    "import time as _ca_time\n",
    'os.environ.setdefault("CLOUD_AMD_RANK_T0", repr(_ca_time.time()))\n',  # rank start, for the bench phases
    'os.environ["TF_KERAS_RUNNING_REMOTELY"]="1"\n',
    'os.environ["CLOUD_AMD_RUNNING_REMOTELY"]="1"\n',
    "import cloud_amd.parallel.strategy as _ca_strategy\n",
]


def strategy_lines(chief_config, worker_config, worker_count):
    if worker_count > 0:
        if machine_config.is_tpu_config(worker_config):
            raise NotImplementedError("TPUStrategy has no MI355X analogue")
        ctor = "strategy = _ca_strategy.MultiWorkerMirroredStrategy()\n"
    elif chief_config.is_gpu and chief_config.accelerator_count > 1:
        ctor = "strategy = _ca_strategy.MirroredStrategy()\n"
    elif chief_config.is_gpu:
        ctor = "strategy = _ca_strategy.OneDeviceStrategy(device='/gpu:0')\n"
    else:
        ctor = "strategy = _ca_strategy.OneDeviceStrategy(device='/cpu:0')\n"
    return [ctor, "_ca_strategy.experimental_set_strategy(strategy)\n"]


def notebook_code_lines(path):
    """Code-cell lines of an .ipynb (nbformat 4 JSON), magics/shell/comment lines dropped."""
    with open(path) as f:
        nb = json.load(f)
    lines = []
    for cell in nb.get("cells", []):
        if cell.get("cell_type") != "code":
            continue
        src = cell.get("source", [])
        if isinstance(src, str):
            src = src.splitlines(keepends=True)
        for line in src:
            if not line.endswith("\n"):
                line += "\n"
            lines.append(line)
        lines.append("\n")
    return [ln for ln in lines if not (ln.startswith("!") or ln.startswith("%") or ln.startswith("#"))]


def get_preprocessed_entry_point(entry_point, chief_config, worker_config, worker_count, distribution_strategy,
                                 called_from_notebook=False, notebook_lines=None, output_dir=None):
    """Write the wrapper script and return its path."""
    lines = list(HEADER)
    if distribution_strategy == "auto":
        lines.extend(strategy_lines(chief_config, worker_config, worker_count))
    if entry_point is None and not called_from_notebook:
        entry_point = sys.argv[0]
    if entry_point is not None and entry_point.endswith("py"):
        name = os.path.basename(entry_point)
        lines.append("__file__ = os.path.abspath({!r})\n".format(name))
        lines.append("exec(compile(open({0!r}).read(), {0!r}, 'exec'))\n".format(name))
    else:
        if notebook_lines is not None:
            code = notebook_lines
        elif entry_point is not None:
            code = notebook_code_lines(entry_point)
        else:
            raise RuntimeError("Unable to access the current notebook's code; pass entry_point='<notebook>.ipynb'.")
        lines.extend(code)
    fd, out = tempfile.mkstemp(suffix=".py", dir=output_dir)
    with os.fdopen(fd, "w") as f:
        f.writelines(lines)
    return out
