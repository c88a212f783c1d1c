"""Stream-priority probe: run a bench script in-process with its main (critical-path) compute on
a high-priority HIP stream, the weight-gradient side stream staying at normal priority.

    python scripts/prio_probe.py bench/bert_base_synth.py --steps 20 --warmup 5
"""
import os
import runpy
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    script = sys.argv[1]
    s = torch.cuda.Stream(priority=-1)
    sys.argv = [script, "--via-run", "0"] + sys.argv[2:]
    with torch.cuda.stream(s):
        runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
