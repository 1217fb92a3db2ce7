"""Load golden fixtures (tests/golden/*.npz, produced by tests/golden/make_golden*.py)."""
import glob
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_names(family=None, multitask=False):
    """Single-task fixtures (make_golden.py) by default; multitask=True: the multitask /
    derivative-informed ones (make_golden_multitask.py, names mt_* / deriv_*)."""
    # (c5_*: the benched C5 regime of make_golden_c5.py, read by tests/test_gpu_multioutput.py only;
    # c4_*: the benched C4 work of make_golden_c4.py, read by tests/test_gpu_bench_path.py and
    # tests/test_bench_accounting.py only; c2_ / c3_: the benched C2 / C3 work of make_golden_c23.py, read by
    # tests/test_gpu_bench_path.py and tests/test_native_cpu.py only; single_extras: make_golden_single_extras.py, read by
    # tests/test_gpu_single_extras.py only)
    names = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                   if not os.path.basename(p).startswith(("c5_", "c4_", "c2_", "c3_", "single_extras")))
    mt = [n for n in names if n.startswith("mt_") or n.startswith("deriv_")]
    names = mt if multitask else [n for n in names if n not in mt]
    if family is not None:
        names = [n for n in names if n.startswith(family)]
    return names


def load_golden(name):
    with np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}
