"""Launch train_model.py (which imports create_model.py) through run() -- port of
reference ``multi_file_example/scale_model.py``; run from this directory."""
import os

import cloud_amd as tfc

if os.environ.get("CLOUD_AMD_EXAMPLE_CPU") == "1":
    tfc.run(entry_point="train_model.py", requirements_txt="requirements.txt",
            chief_config=tfc.COMMON_MACHINE_CONFIGS["CPU"], stream_logs=True)
else:
    tfc.run(entry_point="train_model.py", requirements_txt="requirements.txt", stream_logs=True)
