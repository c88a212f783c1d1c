"""run() on the KerasTuner search workload on 4 GPUs -- port of reference
``TFC/core/tests/examples/call_run_on_script_with_keras_tuner_search.py``
(``V100_4X`` -> ``MI355X_4X``)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cloud_amd as tfc  # noqa: E402

parser = argparse.ArgumentParser(description="Model save path arguments.")
parser.add_argument("--path", required=True, type=str, help="Keras model save path")
args = parser.parse_args()
os.chdir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "workloads"))
tfc.run(entry_point="keras_tuner_cifar_example.py", distribution_strategy="auto",
        chief_config=tfc.COMMON_MACHINE_CONFIGS["MI355X_4X"], worker_count=0,
        entry_point_args=["--path", os.path.abspath(args.path)], stream_logs=True)
