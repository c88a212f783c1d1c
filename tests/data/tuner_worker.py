"""Distributed-tuning worker used by tests/test_tuner.py (one process per tuner_id)."""
import os

import numpy as np


def build_model(hp):
    from cloud_amd import keras

    model = keras.Sequential([keras.layers.Dense(int(hp.Int("units", 8, 32, step=8)), activation="relu",
                                                 input_shape=(20,)), keras.layers.Dense(2)])
    model.compile(optimizer=keras.optimizers.SGD(hp.Float("lr", 1e-3, 1e-1, sampling="log")),
                  loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True), metrics=["acc"])
    return model


def run(tuner_id, device):
    from cloud_amd.parallel import strategy as S
    from cloud_amd.tuner import CloudTuner, HyperParameters

    S.experimental_set_strategy(S.OneDeviceStrategy("/cpu:0"))
    hps = HyperParameters()
    hps.Int("units", 8, 32, step=8)
    hps.Float("lr", 1e-3, 1e-1, sampling="log")
    rng = np.random.default_rng(0)
    x = rng.normal(size=(256, 20)).astype("float32")
    y = (x[:, 0] > 0).astype("int64")
    tuner = CloudTuner(build_model, project_id="p", region="r", objective="acc", hyperparameters=hps,
                       max_trials=int(os.environ.get("MAX_TRIALS", 6)), study_id=os.environ["STUDY_ID"], study_dir=os.environ["STUDY_DIR"],
                       directory=os.path.join(os.environ["STUDY_DIR"], "results", tuner_id))
    if os.environ.get("FAKE_FOOTPRINT_GB"):  # CPU stand-in for the measured HBM peak of a GPU trial
        from cloud_amd.utils import hbm

        hbm.report_footprint(float(os.environ["FAKE_FOOTPRINT_GB"]))
    tuner.search(x, y, epochs=2, batch_size=32)
