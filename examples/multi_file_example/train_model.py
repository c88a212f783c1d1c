"""Training script importing a sibling module (the whole directory is staged
into ``jobs/<id>/app``) -- port of reference ``multi_file_example/train_model.py``."""
import os

from create_model import create_keras_model

import cloud_amd as tfc
from cloud_amd import tf

small = os.environ.get("CLOUD_AMD_EXAMPLE_SMALL") == "1"
(x_train, y_train), (x_test, y_test) = tf.keras.datasets.mnist.load_data(n_train=1024 if small else 60000,
                                                                        n_test=256 if small else 10000)


def scale(image, label):
    return image.astype("float32") / 255, label


train_dataset = tf.data.Dataset.from_tensor_slices((x_train[..., None], y_train)).map(scale).cache().shuffle(
    10000).batch(64)
eval_dataset = tf.data.Dataset.from_tensor_slices((x_test[..., None], y_test)).map(scale).batch(64)
model = create_keras_model()
epochs = (2 if small else 10) if tfc.remote() else 1
hist = model.fit(train_dataset, epochs=epochs)
print("RESULT multi_file remote={} epochs={} loss={:.4f}".format(tfc.remote(), epochs, hist.history["loss"][-1]))
