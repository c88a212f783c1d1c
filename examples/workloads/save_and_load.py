"""Checkpoint / save / load across strategies -- port of reference
``TFC/core/tests/testdata/save_and_load.py`` (TF "distribute/save_and_load"
tutorial).  Expects ``--path`` (model save directory)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from _common import n  # noqa: E402

from cloud_amd import tf  # noqa: E402

parser = argparse.ArgumentParser(description="A tutorial of argparse!")
parser.add_argument("--path", required=True, type=str, help="Keras model save path")
args = parser.parse_args()
model_save_path = args.path

mirrored_strategy = tf.distribute.MirroredStrategy()


def get_data():
    (xtr, ytr), (xte, yte) = tf.keras.datasets.mnist.load_data(n_train=n(60000, 1024), n_test=n(10000, 256))
    batch_size = 64 * mirrored_strategy.num_replicas_in_sync

    def scale(image, label):
        return image.astype("float32") / 255, label

    train = tf.data.Dataset.from_tensor_slices((xtr[..., None], ytr)).map(scale).cache().shuffle(10000).batch(
        batch_size)
    ev = tf.data.Dataset.from_tensor_slices((xte[..., None], yte)).map(scale).batch(batch_size)
    return train, ev


def get_model():
    with mirrored_strategy.scope():
        model_ = tf.keras.Sequential([
            tf.keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
            tf.keras.layers.MaxPooling2D(),
            tf.keras.layers.Flatten(),
            tf.keras.layers.Dense(64, activation="relu"),
            tf.keras.layers.Dense(10),
        ])
    model_.compile(loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer="adam",
                   metrics=["accuracy"])
    return model_


print("Initial training + saving model weights")
model = get_model()
train_dataset, eval_dataset = get_data()
checkpoint_path = "{}/cp.ckpt".format(model_save_path)
cp_callback = tf.keras.callbacks.ModelCheckpoint(filepath=checkpoint_path, save_weights_only=True, verbose=1)
model.fit(train_dataset, epochs=2, callbacks=[cp_callback])

print("Creating new model instance")
model = get_model()
print("Evaluating untrained model")
loss, acc = model.evaluate(eval_dataset, verbose=2)
print("Untrained model, accuracy: {:5.2f}%".format(100 * acc))

print("Loading model weights")
another_strategy = tf.distribute.OneDeviceStrategy("/cpu:0")
with another_strategy.scope():
    model.load_weights(checkpoint_path)
print("Evaluating model with loaded weights")
loss, acc_restored = model.evaluate(eval_dataset, verbose=2)
print("Restored model, accuracy: {:5.2f}%".format(100 * acc_restored))

print("Saving model")
model.save(model_save_path)

print("Restore model and train without dist strat")
restored_keras_model = tf.keras.models.load_model(model_save_path)
restored_keras_model.fit(train_dataset, epochs=2)

print("Restore model and training using a different strategy")
with another_strategy.scope():
    restored_keras_model_ds = tf.keras.models.load_model(model_save_path)
    restored_keras_model_ds.fit(train_dataset, epochs=2)
print("RESULT save_and_load untrained_acc={:.4f} restored_acc={:.4f}".format(acc, acc_restored))
