"""The probnum25 paper's timing configurations alone (bench.paper_configs: n = 2^10 per task, SI lattice
alpha = 2 / DSI net alpha = 4, f and (f, grad f)), for rocprofv3 kernel traces of the multitask fit
(k_mt_spec_iter + k_spec_reduce_step) and the single-task fits.  Prints one JSON line per config.

    python tools/paper_kernels.py [--no-warm]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch.set_default_dtype(torch.float64)


def main():
    import bench
    import fastgaussianprocesses_amd as F
    dev = torch.device("cuda", 0)
    for c in bench.paper_configs(F, dev, warm="--no-warm" not in sys.argv):
        print(json.dumps(c), flush=True)


if __name__ == "__main__":
    main()
