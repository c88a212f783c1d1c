"""Train locally first, then call run() inside the same script -- port of
reference ``TFC/core/tests/examples/call_run_within_script_with_keras_fit.py``
(ResNet-50 transfer learning on stanford_dogs).  Synthetic 120-class images of
the same shape replace tfds (no network); ``weights=None`` (no download).

Locally (``remote()`` False) one tiny epoch runs on a few batches; then
``run()`` launches the job on 2 MI355X and exits; inside the job the script
re-runs with ``remote()`` True and trains the full schedule under Mirrored."""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cloud_amd as tfc  # noqa: E402
from cloud_amd import tf  # noqa: E402

SMALL = os.environ.get("CLOUD_AMD_EXAMPLE_SMALL") == "1"
IMG_SIZE = 64 if SMALL else 224
NUM_CLASSES = 120
BATCH_SIZE = 8 if SMALL else 64
rng = np.random.default_rng(0)
n_train = 64 if SMALL else 2048
x = rng.random((n_train, IMG_SIZE, IMG_SIZE, 3), dtype=np.float32) * 255
y = rng.integers(0, NUM_CLASSES, n_train)
ds = tf.data.Dataset.from_tensor_slices((x, y))
ds_train = ds.map(lambda im, lb: (tf.keras.applications.resnet50.preprocess_input(im), lb)).batch(
    BATCH_SIZE, drop_remainder=True).prefetch(tf.data.AUTOTUNE)
ds_test = ds_train

inputs = tf.keras.layers.Input(shape=(IMG_SIZE, IMG_SIZE, 3))
base_model = tf.keras.applications.ResNet50(weights=None, include_top=False, input_tensor=inputs)
h = tf.keras.layers.GlobalAveragePooling2D()(base_model.output)
h = tf.keras.layers.Dropout(0.5)(h)
outputs = tf.keras.layers.Dense(NUM_CLASSES)(h)
model = tf.keras.Model(inputs, outputs)
base_model.trainable = False

# one directory for every rank of the job (the reference writes to a GCS bucket): the job
# directory run() created, else a fresh local one
ckpt_dir = os.environ.get("CLOUD_AMD_EXAMPLE_OUT") or (
    os.path.join(os.environ["CLOUD_AMD_JOB_DIR"], "model_out") if os.environ.get("CLOUD_AMD_JOB_DIR")
    else tempfile.mkdtemp())
callbacks = [
    tf.keras.callbacks.ModelCheckpoint(os.path.join(ckpt_dir, "save_at_{epoch}")),
    tf.keras.callbacks.TensorBoard(log_dir=os.path.join(ckpt_dir, "logs")),
    tf.keras.callbacks.EarlyStopping(monitor="val_loss", patience=3),
]
model.compile(optimizer=tf.keras.optimizers.Adam(learning_rate=1e-2),
              loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True), metrics=["accuracy"])

if tfc.remote():
    epochs, train_data, test_data = (1 if SMALL else 5), ds_train, ds_test
else:
    epochs, train_data, test_data, callbacks = 1, ds_train.take(2), ds_test.take(2), None
model.fit(train_data, epochs=epochs, callbacks=callbacks, validation_data=test_data, verbose=2)

if os.environ.get("CLOUD_AMD_EXAMPLE_CPU") == "1":  # CPU rehearsal: chief + 1 worker over gloo
    tfc.run(chief_config=tfc.COMMON_MACHINE_CONFIGS["CPU"], worker_config=tfc.COMMON_MACHINE_CONFIGS["CPU"],
            worker_count=1, stream_logs=True)
else:
    tfc.run(chief_config=tfc.COMMON_MACHINE_CONFIGS["MI355X_2X"], stream_logs=True)

if tfc.remote():
    save_path = os.path.join(ckpt_dir, "resnet-dogs")
    model.save(save_path)
    model = tf.keras.models.load_model(save_path)
loss, acc = model.evaluate(test_data)
print("RESULT within_script remote={} loss={:.4f}".format(tfc.remote(), loss))
