"""run() on a separate training script with auto strategy -- port of reference
``TFC/core/tests/examples/call_run_on_script_with_keras_fit.py``: 2 MI355X on
the chief -> MirroredStrategy over RCCL (one process per GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cloud_amd as tfc  # noqa: E402

os.chdir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "workloads"))
tfc.run(
    entry_point="mnist_example_using_fit.py",
    distribution_strategy="auto",
    chief_config=tfc.MachineConfig(cpu_cores=8, memory=30, accelerator_type=tfc.AcceleratorType.AMD_INSTINCT_MI355X,
                                   accelerator_count=2),
    worker_count=0,
    stream_logs=True,
)
