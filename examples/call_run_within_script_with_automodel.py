"""Model search inside a run() job -- counterpart of reference
``TFC/core/tests/examples/call_run_within_script_with_autokeras.py``.  AutoKeras is not
available here, so the "ImageClassifier(max_trials=2)" step is a cloud_amd
``RandomSearch`` over a small CNN family (depth, width, learning rate); the flow is the
same: run() first (the job re-runs this file remotely), search, evaluate, export the
best model to --path."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cloud_amd as tfc  # noqa: E402
import cloud_amd.tuner as kt  # noqa: E402
from cloud_amd import tf  # noqa: E402

parser = argparse.ArgumentParser(description="Model save path arguments.")
parser.add_argument("--path", required=True, type=str, help="Keras model save path")
args = parser.parse_args()
small = os.environ.get("CLOUD_AMD_EXAMPLE_SMALL") == "1"
cpu = os.environ.get("CLOUD_AMD_EXAMPLE_CPU") == "1"

# the job re-runs this file: forward its arguments (the reference example omitted them)
tfc.run(chief_config=tfc.COMMON_MACHINE_CONFIGS["CPU" if cpu else "MI355X_1X"], entry_point_args=sys.argv[1:],
        stream_logs=True)

(x_train, y_train), (x_test, y_test) = tf.keras.datasets.mnist.load_data(n_train=512 if small else 60000,
                                                                          n_test=128 if small else 10000)
x_train, x_test = x_train[..., None] / 255.0, x_test[..., None] / 255.0
print(x_train.shape, y_train.shape, y_train[:3])


def image_classifier(hp):
    m = tf.keras.Sequential([tf.keras.layers.InputLayer(input_shape=(28, 28, 1))])
    for i in range(hp.Int("conv_blocks", 1, 2)):
        m.add(tf.keras.layers.Conv2D(hp.Choice("filters_%d" % i, [16, 32]), 3, activation="relu"))
        m.add(tf.keras.layers.MaxPooling2D())
    m.add(tf.keras.layers.Flatten())
    m.add(tf.keras.layers.Dense(10, activation="softmax"))
    m.compile(optimizer=tf.keras.optimizers.Adam(hp.Float("lr", 1e-4, 1e-2, sampling="log")),
              loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    return m


clf = kt.RandomSearch(image_classifier, objective="val_accuracy", max_trials=2,
                      directory=os.path.join(args.path, "search"))
clf.search(x_train, y_train, epochs=1 if small else 10, validation_data=(x_test, y_test))
best = clf.get_best_models(1)[0]
acc = best.evaluate(x_test, y_test)[1]
print("Accuracy: {accuracy}".format(accuracy=acc))
best.save(os.path.join(args.path, "model"))
print("RESULT automodel remote={} acc={:.4f}".format(tfc.remote(), acc))
