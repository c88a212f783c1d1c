"""README MLP without a requirements file -- port of reference
``TFC/core/tests/testdata/mnist_example_using_fit_no_reqs.py``."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from _common import n  # noqa: E402

from cloud_amd import tf  # noqa: E402

(x_train, y_train), (_, _) = tf.keras.datasets.mnist.load_data(n_train=n(60000, 2048), n_test=16)
x_train = x_train.reshape((x_train.shape[0], 28 * 28)).astype("float32") / 255
model = tf.keras.Sequential([
    tf.keras.layers.Dense(512, activation="relu", input_shape=(28 * 28,)),
    tf.keras.layers.Dropout(0.2),
    tf.keras.layers.Dense(10, activation="softmax"),
])
model.compile(loss="sparse_categorical_crossentropy", optimizer=tf.keras.optimizers.Adam(), metrics=["accuracy"])
epochs = int(os.environ.get("MLP_EPOCHS", n(10, 1)))
t0 = time.time()
hist = model.fit(x_train, y_train, epochs=epochs, batch_size=128)
fit_s = time.time() - t0
print("RESULT mlp loss={:.4f} samples_per_s={:.1f} fit_s={:.3f}".format(hist.history["loss"][-1],
                                                                       epochs * len(x_train) / fit_s, fit_s))
