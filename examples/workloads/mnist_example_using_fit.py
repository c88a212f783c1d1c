"""Keras ``fit`` on MNIST with an LR schedule callback -- port of reference
``TFC/core/tests/testdata/mnist_example_using_fit.py`` (TF "distribute/keras"
tutorial).  Changes: ``import tensorflow as tf`` -> ``from cloud_amd import tf``;
``tfds.load("mnist")`` -> the synthetic ``keras.datasets.mnist`` (no network).
The strategy comes from the wrapper ``run()`` generates (or OneDevice when run
directly).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from _common import n  # noqa: E402

from cloud_amd import tf  # noqa: E402

print(tf.__version__)

(x_train, y_train), (x_test, y_test) = tf.keras.datasets.mnist.load_data(n_train=n(60000, 2048), n_test=n(10000, 512))
mnist_train = tf.data.Dataset.from_tensor_slices((x_train[..., None], y_train))
mnist_test = tf.data.Dataset.from_tensor_slices((x_test[..., None], y_test))

BUFFER_SIZE = 10000
BATCH_SIZE = 64


def scale(image, label):
    image = image.float() / 255 if hasattr(image, "float") else image.astype("float32") / 255
    return image, label


train_dataset = mnist_train.map(scale).cache().shuffle(BUFFER_SIZE).batch(BATCH_SIZE)
eval_dataset = mnist_test.map(scale).batch(BATCH_SIZE)

model = tf.keras.Sequential([
    tf.keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
    tf.keras.layers.MaxPooling2D(),
    tf.keras.layers.Flatten(),
    tf.keras.layers.Dense(64, activation="relu"),
    tf.keras.layers.Dense(10, activation="softmax"),
])
model.compile(loss="sparse_categorical_crossentropy", optimizer=tf.keras.optimizers.Adam(), metrics=["accuracy"])


def decay(epoch):
    if epoch < 3:
        return 1e-3
    elif 3 <= epoch < 7:
        return 1e-4
    return 1e-5


class PrintLR(tf.keras.callbacks.Callback):
    def on_epoch_end(self, epoch, logs=None):
        print("\nLearning rate for epoch {} is {}".format(epoch + 1, model.optimizer.lr.numpy()))


callbacks = [tf.keras.callbacks.LearningRateScheduler(decay), PrintLR()]
hist = model.fit(train_dataset, epochs=2, callbacks=callbacks)
loss, acc = model.evaluate(eval_dataset, verbose=0)
print("RESULT fit loss={:.4f} eval_acc={:.4f}".format(hist.history["loss"][-1], acc))
