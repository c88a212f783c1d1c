"""cloud_fit: asset serialisation round trip and a real 2-process remote fit
(reference experimental/cloud_fit/tests/unit/{client,remote}_test.py)."""
import json
import os
import pickle

import numpy as np
import pytest

from cloud_amd import keras
from cloud_amd.experimental.cloud_fit import client, remote
from cloud_amd.parallel import strategy as S


class CountingCallback(keras.callbacks.Callback):
    def __init__(self, path):
        super().__init__()
        self.path = path

    def on_train_begin(self, logs=None):
        with open(os.path.join(self.path, f"cb_{os.getpid()}"), "w") as f:
            f.write("1")


def _model():
    m = keras.Sequential([keras.layers.Dense(16, activation="relu", input_shape=(8,)), keras.layers.Dense(2)])
    m.compile(optimizer=keras.optimizers.SGD(0.002), loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              metrics=["accuracy"])
    return m


def _data():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(128, 8)).astype("float32")
    return x, (x[:, 0] > 0).astype("int64")


def test_serialize_assets_layout(tmp_path):
    x, y = _data()
    client._serialize_assets(str(tmp_path), _model(), x=x, y=y, epochs=2, batch_size=16,
                             callbacks=[CountingCallback(str(tmp_path))], validation_data=(x, y))
    for f in client.ASSET_FILES:
        assert os.path.exists(tmp_path / "training_assets" / f)
    with open(tmp_path / "training_assets" / "fit_kwargs.pkl", "rb") as f:
        assert pickle.load(f) == {"epochs": 2, "batch_size": 16}
    assert os.path.exists(tmp_path / "model" / "weights.pt")


def test_strategy_name_validation(tmp_path):
    with pytest.raises(ValueError, match="not supported"):
        client.cloud_fit(_model(), str(tmp_path), distribution_strategy="TPUStrategy", x=_data()[0])


def test_default_job_spec_cpu(monkeypatch):
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "0")
    spec = client._default_job_spec(entry_point_args=["--remote_dir", "d"])
    assert spec["jobId"].startswith("cloud_fit_") and spec["trainingInput"]["worker_count"] == 1
    assert spec["trainingInput"]["args"] == ["--remote_dir", "d"]


def test_remote_run_in_process_fake_tf_config(tmp_path, monkeypatch):
    """remote_test.py:75-103: worker-only cluster, task worker:0 saves to output/."""
    x, y = _data()
    client._serialize_assets(str(tmp_path), _model(), x=x, y=y, epochs=1, batch_size=32,
                             callbacks=[CountingCallback(str(tmp_path))])
    monkeypatch.setenv("TF_CONFIG", json.dumps({"cluster": {"worker": ["localhost:9999", "localhost:9999"]},
                                                "task": {"type": "worker", "index": 0}}))
    monkeypatch.setattr(S, "MirroredStrategy", lambda: S.OneDeviceStrategy("/cpu:0"))
    from cloud_amd.experimental.cloud_fit import utils

    monkeypatch.setitem(utils.SUPPORTED_DISTRIBUTION_STRATEGIES, "MirroredStrategy",
                        lambda: S.OneDeviceStrategy("/cpu:0"))
    remote.run(str(tmp_path), "MirroredStrategy")
    assert os.path.exists(tmp_path / "output" / "weights.pt")
    assert len([f for f in os.listdir(tmp_path) if f.startswith("cb_")]) == 1
    m = keras.models.load_model(str(tmp_path / "output"))
    assert m.predict(x[:4]).shape == (4, 2)


def test_cloud_fit_two_process_job(tmp_path, monkeypatch):
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "0")
    monkeypatch.setenv("CLOUD_AMD_JOBS_DIR", str(tmp_path / "jobs"))
    x, y = _data()
    rd = str(tmp_path / "remote")
    job_id = client.cloud_fit(_model(), rd, x=x, y=y, epochs=2, batch_size=32,
                              callbacks=[CountingCallback(str(tmp_path))], job_id="cloud_fit_test")
    assert job_id == "cloud_fit_test"
    # returns at submission (reference client.py:227-286); the detached job finishes on its own
    from cloud_amd.core import launcher

    assert launcher.Job.attach(job_id).wait(300) == 0
    meta = json.load(open(tmp_path / "jobs" / job_id / "job.json"))
    assert meta["state"] == "SUCCEEDED" and meta["world_size"] == 2
    assert os.path.exists(os.path.join(rd, "output", "weights.pt"))
    assert not os.listdir(os.path.join(rd, "output", "tmp"))  # non-chief temp dirs removed
    assert len([f for f in os.listdir(tmp_path) if f.startswith("cb_")]) == 2  # fired once per replica
