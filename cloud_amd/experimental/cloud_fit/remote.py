"""Job side of ``cloud_fit`` (reference ``experimental/cloud_fit/remote.py``).

``python -m cloud_amd.experimental.cloud_fit.remote --remote_dir D --distribution_strategy S``:
instantiate strategy S, load the model and the pickled fit arguments from D
inside ``strategy.scope()``, ``model.fit``, then the chief saves to
``D/output`` while every other worker saves to ``D/output/tmp/workers_<uuid>``
and deletes it (the reference's concurrent-write workaround, kept for layout
parity).  Chief detection keeps the reference quirk: task type ``chief`` OR
task index 0.
"""
from __future__ import annotations

import argparse
import logging
import os
import pickle
import shutil
import uuid

from ...parallel.strategy import is_chief_task
from . import utils

log = logging.getLogger("cloud_amd.cloud_fit")


def run(remote_dir, distribution_strategy):
    from ... import keras

    strategy = utils.SUPPORTED_DISTRIBUTION_STRATEGIES[distribution_strategy]()
    with strategy.scope():
        assets = os.path.join(remote_dir, "training_assets")

        def load(name):
            with open(os.path.join(assets, name), "rb") as f:
                return pickle.load(f)

        fit_kwargs = dict(load("fit_kwargs.pkl"))
        fit_kwargs.update(load("x.pkl"))
        vd = load("validation_data.pkl")
        if vd is not None:
            fit_kwargs["validation_data"] = vd
        cbs = load("callbacks.pkl")
        if cbs is not None:
            fit_kwargs["callbacks"] = cbs
        log.info("Loading model from %s", os.path.join(remote_dir, "model"))
        model = keras.models.load_model(os.path.join(remote_dir, "model"))
        model.fit(**fit_kwargs)
    # reference remote.py:130-145: the chief saves to output/, every other worker to a
    # temporary dir it deletes again (per-worker writes, not the collective model.save)
    from ...keras import saving

    if _is_current_worker_chief():
        saving._save_model(model, os.path.join(remote_dir, "output"))
    else:
        tmp = os.path.join(remote_dir, "output", "tmp", "workers_" + str(uuid.uuid4()))
        saving._save_model(model, tmp)
        _delete_dir(tmp)
    import torch.distributed as dist

    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
    return model


def _is_current_worker_chief():
    import torch.distributed as dist

    if dist.is_initialized():
        return dist.get_rank() == 0
    try:
        return is_chief_task()
    except ValueError:
        return True


def _delete_dir(path):
    shutil.rmtree(path, ignore_errors=True)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--remote_dir", required=True)
    ap.add_argument("--distribution_strategy", required=True)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    run(a.remote_dir, a.distribution_strategy)


if __name__ == "__main__":
    main()
