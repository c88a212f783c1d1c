"""README MLP (reference README.md:60-90) on cloud_amd: run() in the script itself.

    python examples/mnist_mlp.py                # launches a job on this node, then exits
    CLOUD_AMD_EXAMPLE_CPU=1 python examples/mnist_mlp.py   # 2 CPU workers (gloo)

When the job starts, the same file runs again inside each rank: ``run()`` is a
no-op there (``remote()`` is True) and training proceeds under the strategy the
generated wrapper installed (Mirrored over the GPUs, or MultiWorkerMirrored).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import cloud_amd as tfc  # noqa: E402
from cloud_amd import keras  # noqa: E402

if os.environ.get("CLOUD_AMD_EXAMPLE_CPU") == "1":
    cfg = tfc.COMMON_MACHINE_CONFIGS["CPU"]
    tfc.run(chief_config=cfg, worker_config=cfg, worker_count=int(os.environ.get("WORKERS", 1)),
            stream_logs=True, entry_point_args=sys.argv[1:])
else:
    tfc.run(chief_config=tfc.COMMON_MACHINE_CONFIGS["MI355X_1X"], stream_logs=True, entry_point_args=sys.argv[1:])

epochs = int(os.environ.get("EPOCHS", 2))
(x_train, y_train), (x_test, y_test) = keras.datasets.mnist.load_data(n_train=8192, n_test=1024)
x_train = x_train.reshape(-1, 784).astype("float32") / 255
x_test = x_test.reshape(-1, 784).astype("float32") / 255
model = keras.Sequential([keras.layers.Dense(512, activation="relu", input_shape=(784,)),
                          keras.layers.Dropout(0.2), keras.layers.Dense(10, activation="softmax")])
model.compile(loss="sparse_categorical_crossentropy", optimizer=keras.optimizers.Adam(), metrics=["accuracy"])
hist = model.fit(x_train, y_train, epochs=epochs, batch_size=128, verbose=0)
loss, acc = model.evaluate(x_test, y_test, verbose=0)
from cloud_amd.parallel.strategy import get_strategy  # noqa: E402

s = get_strategy()
chk = float(sum(float(p.detach().double().sum()) for p in model.parameters()))
print("RESULT " + json.dumps({"rank": s.rank, "replicas": s.num_replicas_in_sync, "loss": hist.history["loss"],
                              "test_acc": acc, "weights_checksum": chk, "strategy": type(s).__name__}), flush=True)
