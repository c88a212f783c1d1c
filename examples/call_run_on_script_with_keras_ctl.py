"""run() on a custom-training-loop script that creates its own strategy
(``distribution_strategy=None``) with one extra worker -- port of reference
``TFC/core/tests/examples/call_run_on_script_with_keras_ctl.py``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cloud_amd as tfc  # noqa: E402

os.chdir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "workloads"))
cpu = os.environ.get("CLOUD_AMD_EXAMPLE_CPU") == "1"
cfg = tfc.COMMON_MACHINE_CONFIGS["CPU"] if cpu else tfc.COMMON_MACHINE_CONFIGS["MI355X_1X"]
tfc.run(entry_point="mnist_example_using_ctl.py", distribution_strategy=None, chief_config=cfg, worker_config=cfg,
        worker_count=1, stream_logs=True)
