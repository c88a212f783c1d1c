#!/usr/bin/env python3
"""Generate the example notebooks (nbformat 4 JSON) from the cell lists below, so the
.ipynb files stay reviewable as Python.  Counterparts of the reference's notebooks:
core/tests/testdata/mnist_example_using_fit.ipynb, core/tests/examples/
{call_run_within_nb_on_colab,dogs_classification}.ipynb, tuner/tests/examples/
ai_platform_optimizer_tuner.ipynb, experimental/cloud_fit/tests/examples/cloud_fit.ipynb
-- rewritten for cloud_amd (local MI355X node, synthetic data, no cloud auth cells)."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def nb(cells):
    out = []
    for kind, src in cells:
        src = src.strip("\n") + "\n"
        lines = src.splitlines(keepends=True)
        if kind == "md":
            out.append({"cell_type": "markdown", "metadata": {}, "source": lines})
        else:
            out.append({"cell_type": "code", "execution_count": None, "metadata": {}, "outputs": [],
                        "source": lines})
    return {"cells": out, "metadata": {"kernelspec": {"display_name": "Python 3", "language": "python",
                                                     "name": "python3"},
                                       "language_info": {"name": "python"}},
            "nbformat": 4, "nbformat_minor": 4}


SETUP = """
import os
import sys
REPO = os.environ.get("CLOUD_AMD_REPO", os.path.abspath(os.path.join(os.getcwd(), "..", "..")))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
SMALL = os.environ.get("CLOUD_AMD_EXAMPLE_SMALL") == "1"
CPU = os.environ.get("CLOUD_AMD_EXAMPLE_CPU") == "1"
"""

MNIST_FIT = nb([
    ("md", "# Keras `fit` on MNIST (notebook entry point)\n"
           "Run by `examples/call_run_on_notebook_with_keras_fit.py` through `cloud_amd.run()`; the "
           "strategy comes from the generated wrapper. Synthetic MNIST-shaped data (no network)."),
    ("code", "from _common import n\nfrom cloud_amd import tf\nprint(tf.__version__)"),
    ("code", """
(x_train, y_train), (x_test, y_test) = tf.keras.datasets.mnist.load_data(n_train=n(60000, 1024),
                                                                          n_test=n(10000, 256))

def scale(image, label):
    return image.astype("float32") / 255, label

train_dataset = tf.data.Dataset.from_tensor_slices((x_train[..., None], y_train)).map(scale).shuffle(
    10000).batch(64)
eval_dataset = tf.data.Dataset.from_tensor_slices((x_test[..., None], y_test)).map(scale).batch(64)
"""),
    ("code", """
model = tf.keras.Sequential([
    tf.keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
    tf.keras.layers.MaxPooling2D(),
    tf.keras.layers.Flatten(),
    tf.keras.layers.Dense(64, activation="relu"),
    tf.keras.layers.Dense(10, activation="softmax"),
])
model.compile(loss="sparse_categorical_crossentropy", optimizer=tf.keras.optimizers.Adam(), metrics=["accuracy"])
"""),
    ("code", "# magics and shell lines are dropped by the notebook converter\n%time 1\n!echo skipped"),
    ("code", """
model.fit(train_dataset, epochs=n(3, 1))
loss, acc = model.evaluate(eval_dataset)
print("RESULT notebook_fit loss={:.4f} acc={:.4f}".format(loss, acc))
"""),
])

WITHIN_NB = nb([
    ("md", "# Calling `run()` from within a notebook\n"
           "Debug locally first; the `run()` cell then stages this notebook (its code cells become the "
           "job's entry point) and launches it on the node's MI355X GPUs. Inside the job `remote()` is "
           "True, `run()` is a no-op and the full training runs."),
    ("code", SETUP + "import cloud_amd as tfc\nfrom cloud_amd import tf"),
    ("code", """
(x_train, y_train), (x_test, y_test) = tf.keras.datasets.mnist.load_data(n_train=1024 if SMALL else 60000,
                                                                          n_test=256 if SMALL else 10000)
train = tf.data.Dataset.from_tensor_slices((x_train[..., None] / 255.0, y_train)).batch(64)
test = tf.data.Dataset.from_tensor_slices((x_test[..., None] / 255.0, y_test)).batch(64)
model = tf.keras.Sequential([
    tf.keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
    tf.keras.layers.MaxPooling2D(),
    tf.keras.layers.Flatten(),
    tf.keras.layers.Dense(64, activation="relu"),
    tf.keras.layers.Dense(10, activation="softmax"),
])
model.compile(loss="sparse_categorical_crossentropy", optimizer=tf.keras.optimizers.Adam(),
              metrics=["accuracy"])
"""),
    ("code", """
# local debug pass on a few batches
if not tfc.remote():
    model.fit(train.take(2), epochs=1)
"""),
    ("code", """
# launch: in Jupyter, entry_point=None finds this notebook; elsewhere name it explicitly
chief = tfc.COMMON_MACHINE_CONFIGS["CPU" if CPU else "MI355X_2X"]
tfc.run(entry_point="call_run_within_nb.ipynb" if not tfc.remote() else None, distribution_strategy="auto",
        chief_config=chief, worker_count=1 if CPU else 0,
        worker_config=tfc.COMMON_MACHINE_CONFIGS["CPU"] if CPU else None, stream_logs=True)
"""),
    ("code", """
if tfc.remote():
    model.fit(train, epochs=1 if SMALL else 5)
    model.save(os.environ.get("CLOUD_AMD_EXAMPLE_OUT", "mnist_model"))
loss, acc = model.evaluate(test)
print("RESULT within_nb remote={} loss={:.4f}".format(tfc.remote(), loss))
"""),
])

TUNER = nb([
    ("md", "# Hyper-parameter search with `CloudTuner` on the local study service\n"
           "The search space is given either as `HyperParameters` or as an AI-Platform-Optimizer "
           "`study_config`; several tuner loops (one per GPU on a node) share one study by `study_id`."),
    ("code", SETUP + "import tempfile\nimport cloud_amd.tuner as kt\nfrom cloud_amd import tf\n"
             "WORK = os.environ.get(\"CLOUD_AMD_EXAMPLE_OUT\", tempfile.mkdtemp())"),
    ("code", """
(x, y), (val_x, val_y) = tf.keras.datasets.mnist.load_data(n_train=512 if SMALL else 10000,
                                                            n_test=128 if SMALL else 2000)
x, val_x = x.astype("float32") / 255.0, val_x.astype("float32") / 255.0
"""),
    ("code", """
def build_model(hp):
    model = tf.keras.Sequential()
    model.add(tf.keras.layers.Flatten(input_shape=(28, 28)))
    for _ in range(hp.get("num_layers")):  # tunable depth
        model.add(tf.keras.layers.Dense(units=64, activation="relu"))
    model.add(tf.keras.layers.Dense(10, activation="softmax"))
    model.compile(optimizer=tf.keras.optimizers.Adam(learning_rate=hp.get("learning_rate")),
                  loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    return model
"""),
    ("code", """
HPS = kt.HyperParameters()
HPS.Float("learning_rate", min_value=1e-4, max_value=1e-2, sampling="log")
HPS.Int("num_layers", 2, 4)
tuner = kt.CloudTuner(build_model, objective="accuracy", hyperparameters=HPS, max_trials=2 if SMALL else 5,
                      directory=os.path.join(WORK, "t1"), study_dir=os.path.join(WORK, "studies"))
tuner.search_space_summary()
tuner.search(x=x, y=y, epochs=1 if SMALL else 5, validation_data=(val_x, val_y))
tuner.results_summary()
best = tuner.get_best_models(num_models=1)[0]
"""),
    ("code", """
STUDY_CONFIG = {
    "algorithm": "RANDOM_SEARCH",
    "metrics": [{"goal": "MAXIMIZE", "metric": "accuracy"}],
    "parameters": [
        {"parameter": "learning_rate", "type": "DISCRETE", "discrete_value_spec": {"values": [1e-4, 1e-3, 1e-2]}},
        {"parameter": "num_layers", "type": "INTEGER", "integer_value_spec": {"min_value": 2, "max_value": 4}},
    ],
}
"""),
    ("code", """
# several tuner loops on one study (threads here; one process per GPU with TrialScheduler)
from multiprocessing.dummy import Pool

STUDY_ID = "notebook_study_{}".format(os.getpid())

def one_loop(tuner_id):
    t = kt.CloudTuner(build_model, study_config=STUDY_CONFIG, study_id=STUDY_ID, max_trials=4 if SMALL else 10,
                      directory=os.path.join(WORK, "t2", str(tuner_id)), study_dir=os.path.join(WORK, "studies"))
    t.tuner_id = "tuner_{}".format(tuner_id)
    t.search(x=x, y=y, epochs=1, validation_data=(val_x, val_y))
    return t

with Pool(2) as pool:
    loops = pool.map(one_loop, range(2))
loops[0].results_summary()
print("RESULT tuner_nb trials={}".format(len(loops[0].oracle.get_best_trials(100))))
"""),
])

CLOUD_FIT = nb([
    ("md", "# `cloud_fit`: fit an in-memory model as a job\n"
           "The model, data and fit arguments are serialised under `remote_dir`; the job runs "
           "`cloud_amd.experimental.cloud_fit.remote` on the local launcher and the chief writes the "
           "trained model to `remote_dir/output`."),
    ("code", SETUP + "import tempfile\nimport uuid\nimport numpy as np\nfrom cloud_amd import tf\n"
             "from cloud_amd.experimental.cloud_fit import client\n"
             "REMOTE_DIR = os.environ.get(\"CLOUD_AMD_EXAMPLE_OUT\", tempfile.mkdtemp())"),
    ("code", """
# y = w*x + 1 with w trainable (starts at 0.5; the data says 0.5 -> 0.5, bias fixed at 6 / 1)
inp = tf.keras.layers.Input(shape=(1,), dtype="float32")
times_w = tf.keras.layers.Dense(1, kernel_initializer=tf.keras.initializers.Constant([[0.5]]), use_bias=False)
plus_1 = tf.keras.layers.Dense(1, kernel_initializer=tf.keras.initializers.Constant([[1.0]]),
                               bias_initializer=tf.keras.initializers.Constant([1.0]), trainable=False)
simple_model = tf.keras.Model(inp, plus_1(times_w(inp)))
simple_model.compile(loss="mse", optimizer=tf.keras.optimizers.SGD(0.002))
x = np.array([[9.0], [10.0], [11.0]] * 10, dtype=np.float32)
y = np.array([[xi[0] / 2.0 + 6] for xi in x], dtype=np.float32)
simple_model.fit(x, y, batch_size=len(x), epochs=1)  # local check first
"""),
    ("code", """
SIMPLE_REMOTE_DIR = os.path.join(REMOTE_DIR, str(uuid.uuid4()))
job_id = client.cloud_fit(model=simple_model, remote_dir=SIMPLE_REMOTE_DIR, x=x, y=y,
                          epochs=5 if SMALL else 100, batch_size=len(x), verbose=2)
"""),
    ("md", "`cloud_fit` returns as soon as the job is submitted; the job runs under its own supervisor "
           "(`python -m cloud_amd.jobs describe|stream-logs <job_id>` from any shell). Wait for it here:"),
    ("code", """
from cloud_amd.core.launcher import Job
assert Job.attach(job_id).wait() == 0
"""),
    ("code", """
trained = tf.keras.models.load_model(os.path.join(SIMPLE_REMOTE_DIR, "output"))
print("RESULT cloud_fit_nb job={} loss={:.4f}".format(job_id, trained.evaluate(x, y)))
"""),
])

DOGS = nb([
    ("md", "# ResNet-50 transfer learning, trained on the node's GPUs with `run()`\n"
           "Synthetic 120-class 224x224 images stand in for `stanford_dogs` (no network); "
           "`weights=None` (no download).  Same flow as `examples/call_run_within_script_with_keras_fit.py`."),
    ("code", SETUP + "import datetime\nimport numpy as np\nimport cloud_amd as tfc\nfrom cloud_amd import tf"),
    ("code", """
IMG_SIZE, NUM_CLASSES, BATCH_SIZE = (64, 120, 8) if SMALL else (224, 120, 64)
rng = np.random.default_rng(0)
n_train = 64 if SMALL else 4096
images = rng.random((n_train, IMG_SIZE, IMG_SIZE, 3), dtype=np.float32) * 255
labels = rng.integers(0, NUM_CLASSES, n_train)
ds = tf.data.Dataset.from_tensor_slices((images, labels)).map(
    lambda im, lb: (tf.keras.applications.resnet50.preprocess_input(im), lb))
ds_train = ds.batch(BATCH_SIZE, drop_remainder=True).prefetch(tf.data.AUTOTUNE)
ds_test = ds_train
"""),
    ("code", """
inputs = tf.keras.layers.Input(shape=(IMG_SIZE, IMG_SIZE, 3))
base_model = tf.keras.applications.ResNet50(weights=None, include_top=False, input_tensor=inputs)
h = tf.keras.layers.GlobalAveragePooling2D()(base_model.output)
h = tf.keras.layers.Dropout(0.5)(h)
model = tf.keras.Model(inputs, tf.keras.layers.Dense(NUM_CLASSES)(h))
base_model.trainable = False
model.compile(optimizer=tf.keras.optimizers.Adam(learning_rate=1e-2),
              loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True), metrics=["accuracy"])
"""),
    ("code", """
OUT = os.environ.get("CLOUD_AMD_EXAMPLE_OUT", "resnet-dogs")
callbacks = [tf.keras.callbacks.TensorBoard(log_dir=os.path.join(OUT, "logs",
                                                                 datetime.datetime.now().strftime("%Y%m%d-%H%M%S"))),
             tf.keras.callbacks.ModelCheckpoint(os.path.join(OUT, "save_at_{epoch}")),
             tf.keras.callbacks.EarlyStopping(monitor="val_loss", patience=3)]
if tfc.remote():
    epochs, train_data, test_data = (1 if SMALL else 50), ds_train, ds_test
else:
    epochs, train_data, test_data, callbacks = 1, ds_train.take(2), ds_test.take(2), None
model.fit(train_data, epochs=epochs, callbacks=callbacks, validation_data=test_data, verbose=2)
"""),
    ("code", """
tfc.run(entry_point="dogs_classification.ipynb" if not tfc.remote() else None, distribution_strategy="auto",
        chief_config=tfc.COMMON_MACHINE_CONFIGS["CPU" if CPU else "MI355X_8X"],
        job_labels={"job": "resnet-dogs", "team": "examples"}, stream_logs=True)
"""),
    ("code", """
if tfc.remote():
    model.save(os.path.join(OUT, "model"))
print("RESULT dogs remote={} loss={:.4f}".format(tfc.remote(), model.evaluate(test_data)[0]))
"""),
])


def main():
    files = {
        os.path.join(ROOT, "examples", "workloads", "mnist_example_using_fit.ipynb"): MNIST_FIT,
        os.path.join(ROOT, "examples", "notebooks", "call_run_within_nb.ipynb"): WITHIN_NB,
        os.path.join(ROOT, "examples", "notebooks", "cloud_tuner.ipynb"): TUNER,
        os.path.join(ROOT, "examples", "notebooks", "cloud_fit.ipynb"): CLOUD_FIT,
        os.path.join(ROOT, "examples", "notebooks", "dogs_classification.ipynb"): DOGS,
    }
    for path, content in files.items():
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(content, f, indent=1)
            f.write("\n")
        print(path)


if __name__ == "__main__":
    main()
