"""run() on a notebook entry point -- counterpart of reference
``TFC/core/tests/examples/call_run_on_notebook_with_keras_fit.py``: the notebook's code
cells (magics, shell lines and comments dropped) become the job's script; 2 MI355X on
the chief -> MirroredStrategy (one process per GPU over RCCL)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cloud_amd as tfc  # noqa: E402

os.chdir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "workloads"))
cpu = os.environ.get("CLOUD_AMD_EXAMPLE_CPU") == "1"
tfc.run(
    entry_point="mnist_example_using_fit.ipynb",
    distribution_strategy="auto",
    chief_config=(tfc.COMMON_MACHINE_CONFIGS["CPU"] if cpu else
                  tfc.MachineConfig(cpu_cores=8, memory=30, accelerator_type=tfc.AcceleratorType.AMD_INSTINCT_MI355X,
                                    accelerator_count=2)),
    worker_count=0,
    stream_logs=True,
)
