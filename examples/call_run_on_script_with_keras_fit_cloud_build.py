"""run() with ``docker_image_bucket_name`` -- counterpart of reference
``TFC/core/tests/examples/call_run_on_script_with_keras_fit_cloud_build.py``.  There is
no Cloud Build here: the bucket name selects the "remote build" staging path, which on
the local node means the job directory is staged and recorded in the manifest exactly
as for a local build; the argument is kept so reference scripts run unchanged."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cloud_amd as tfc  # noqa: E402

parser = argparse.ArgumentParser(description="Model cloud bucket name argument.")
parser.add_argument("--bucket_name", required=True, type=str, help="Cloud bucket name")
args = parser.parse_args()
os.chdir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "workloads"))
cpu = os.environ.get("CLOUD_AMD_EXAMPLE_CPU") == "1"
tfc.run(
    entry_point="mnist_example_using_fit_no_reqs.py",
    distribution_strategy="auto",
    chief_config=tfc.COMMON_MACHINE_CONFIGS["CPU" if cpu else "MI355X_2X"],
    worker_count=0,
    stream_logs=True,
    docker_image_bucket_name=args.bucket_name,
)
