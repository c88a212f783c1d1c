"""KerasTuner random search on CIFAR-10 with augmentation -- port of reference
``TFC/core/tests/testdata/keras_tuner_cifar_example.py``.  ``kerastuner.tuners``
-> :mod:`cloud_amd.tuner` (same RandomSearch surface, local study service)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from _common import SMALL, n  # noqa: E402

from cloud_amd import tf  # noqa: E402
from cloud_amd import tuner as tuners  # noqa: E402

parser = argparse.ArgumentParser(description="Keras model save path")
parser.add_argument("--path", required=True, type=str, help="Keras model save path")
parser.add_argument("--directory", default="test_dir")
args = parser.parse_args()


def build_model(hp):
    data_augmentation = tf.keras.Sequential([
        tf.keras.layers.experimental.preprocessing.RandomFlip(),
        tf.keras.layers.experimental.preprocessing.RandomRotation(0.1),
        tf.keras.layers.experimental.preprocessing.RandomWidth(0.1),
        tf.keras.layers.experimental.preprocessing.RandomHeight(0.1),
    ])
    inputs = tf.keras.Input(shape=(32, 32, 3))
    x = data_augmentation(inputs)
    x = tf.keras.layers.Conv2D(32, (3, 3), padding="same",
                               activation=hp.Choice("conv_activation_0", values=["relu", "elu"], default="relu"))(x)
    for i in range(hp.Int("num_blocks", 1, 3)):
        for j in range(hp.Int("num_conv_{}".format(i), 1, 3)):
            x = tf.keras.layers.Conv2D(
                hp.Int("filter_{}_{}".format(i, j), 16, n(256, 32), step=16), (3, 3), padding="same",
                activation=hp.Choice("conv_activation_{}_{}".format(i, j), values=["relu", "elu"], default="relu"))(x)
        x = tf.keras.layers.MaxPooling2D(pool_size=(2, 2))(x)
    x = tf.keras.layers.Dropout(rate=hp.Float("dropout_1", min_value=0.0, max_value=0.9, default=0.25, step=0.05))(x)
    x = tf.keras.layers.GlobalMaxPooling2D()(x)
    x = tf.keras.layers.Dense(n(512, 64), activation="relu")(x)
    outputs = tf.keras.layers.Dense(10, activation="softmax")(x)
    model = tf.keras.Model(inputs, outputs)
    lr_schedule = tf.keras.optimizers.schedules.ExponentialDecay(
        initial_learning_rate=hp.Choice("initial_learning_rate", [1e-1, 1e-2, 1e-3]), decay_steps=100000,
        decay_rate=hp.Choice("decay_rate", [0.5, 0.75, 0.95]), staircase=True)
    model.compile(loss="sparse_categorical_crossentropy",
                  optimizer=tf.keras.optimizers.RMSprop(learning_rate=lr_schedule),
                  metrics=["sparse_categorical_accuracy"])
    return model


tuner = tuners.RandomSearch(build_model, objective="val_sparse_categorical_accuracy", max_trials=n(5, 2),
                            executions_per_trial=n(3, 1), directory=args.directory)
tuner.search_space_summary()

(x_train, y_train), (x_test, y_test) = tf.keras.datasets.cifar10.load_data(n_train=n(50000, 512),
                                                                          n_test=n(10000, 128))
BUFFER_SIZE, BATCH_SIZE = 10000, 64


def scale(image, label):
    return image.astype("float32") / 255, label


train_dataset = tf.data.Dataset.from_tensor_slices((x_train, y_train)).map(scale).cache().shuffle(BUFFER_SIZE).batch(
    BATCH_SIZE)
test_dataset = tf.data.Dataset.from_tensor_slices((x_test, y_test)).map(scale).batch(BATCH_SIZE)
tuner.search(train_dataset, epochs=n(2, 1), validation_data=test_dataset,
             callbacks=[tf.keras.callbacks.EarlyStopping(monitor="val_loss", patience=3, mode="min")])
print("Tuner results summary")
tuner.results_summary()
best_model = tuner.get_best_models(num_models=1)[0]
scores = best_model.evaluate(x_test.astype("float32") / 255, y_test, verbose=1)
print("Test loss:", scores[0])
print("Test accuracy:", scores[1])
print("Saving best model")
best_model.save(args.path)
print("RESULT tuner best_acc={:.4f}".format(scores[1]))
