"""Model factory imported by train_model.py -- port of reference
``TFC/core/tests/examples/multi_file_example/create_model.py``."""
from cloud_amd import tf


def create_keras_model():
    model = tf.keras.Sequential([
        tf.keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
        tf.keras.layers.MaxPooling2D(),
        tf.keras.layers.Flatten(),
        tf.keras.layers.Dense(64, activation="relu"),
        tf.keras.layers.Dense(10, activation="softmax"),
    ])
    model.compile(loss="sparse_categorical_crossentropy", optimizer=tf.keras.optimizers.Adam(),
                  metrics=["sparse_categorical_accuracy"])
    return model
