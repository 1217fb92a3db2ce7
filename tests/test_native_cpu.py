"""CPU-only checks: the C-ABI library loads and exports every symbol of include/fgp_hip.h, the host
logic (point sets, argument validation) matches the reference, and nothing runs without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import fastgaussianprocesses_amd as F
from fastgaussianprocesses_amd import _native as N
from tests.golden_util import golden_names, load_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
torch.set_default_dtype(torch.float64)


def header_functions():
    src = open(os.path.join(ROOT, "include", "fgp_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(fgp_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(N.LIB_PATH)
    names = header_functions()
    assert len(names) >= 12
    for name in names:
        assert hasattr(lib, name), "libfgp_hip.so does not export %s" % name
    assert set(names) <= set(N.exported_symbols()), "ctypes binding misses: %s" % (set(names) - set(N.exported_symbols()))


def test_abi_version_and_error_reporting():
    lib = N.lib()
    assert lib.fgp_abi_version() == N.ABI_VERSION
    # validation failures return an error code without touching a device
    rc = lib.fgp_fftbr(None, 0, 1, None, 1, 25, 0, None)
    assert rc == -2
    assert b"log2n" in lib.fgp_last_error()
    rc = lib.fgp_fftbr(None, 0, 1, None, 3, 4, 0, None)
    assert rc == -1


def test_struct_layouts_match_header(tmp_path):
    """Compile a probe against include/fgp_hip.h with gcc and compare sizeof/offsetof of every field
    with the ctypes mirrors in _native.py."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "fgp_hip.h"', "int main(void) {"]
    expect = []
    for cname, cls in (("fgp_nll_desc", N.NllDesc), ("fgp_fit_desc", N.FitDesc), ("fgp_pred_desc", N.PredDesc),
                       ("fgp_mt_layout", N.MtLayout), ("fgp_mt_fit_desc", N.MtFitDesc)):
        lines.append('printf("%%zu\\n", sizeof(%s));' % cname)
        expect.append(ctypes.sizeof(cls))
        for fname, _ in cls._fields_:
            lines.append('printf("%%zu\\n", offsetof(%s, %s));' % (cname, fname))
            expect.append(getattr(cls, fname).offset)
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    assert got == expect


def test_ops_refuse_cpu_tensors():
    with pytest.raises(RuntimeError, match="HIP device"):
        F.ops.fftbr(torch.zeros(8))
    with pytest.raises(RuntimeError, match="HIP device"):
        F.ops.fwht(torch.zeros(8))
    with pytest.raises(RuntimeError, match="HIP device"):
        F.FastGPLattice(2, device="cpu")


def test_power_of_two_guard():
    with pytest.raises(AssertionError):
        F.ops.log2_exact(12)
    assert F.ops.log2_exact(1 << 20) == 20


@pytest.mark.parametrize("name", golden_names())
def test_product_point_sets_match_golden(name):
    g = load_golden(name)
    n = 2 ** int(g["m"])
    d = int(g["d"])
    if str(g["family"]) == "lattice":
        s = F.Lattice(d, generating_vector=g["z"], shift=g["shift"])
        assert np.array_equal(s(0, n), g["x"])
        if n > 1:  # incremental generation == one-shot generation
            assert np.array_equal(np.vstack([s(0, n // 2), s(n // 2, n)]), g["x"])
    else:
        s = F.DigitalNetB2(d, generating_matrices=g["C"].astype(np.uint64), t=int(g["t"]),
                           shift=g["shift"].astype(np.uint64))
        assert np.array_equal(s(0, n, return_binary=True).astype(np.int64), g["xb"])
        assert np.array_equal(s(0, n), g["x"])


def test_default_sobol_matrices_are_nets():
    # the first 2^m points of each 1-D projection are a permutation of {k / 2^m}
    C = F.seqs.sobol_matrices(8, t=32)
    s = F.DigitalNetB2(8, generating_matrices=C, t=32, randomize="FALSE")
    xb = s(0, 256, return_binary=True)
    for j in range(8):
        assert sorted((xb[:, j] >> np.uint64(24)).tolist()) == list(range(256))


def test_lattice_coefficient_matches_reference_formula():
    # (-1)^(alpha+1) (2 pi)^(2 alpha) / (2 alpha)!
    import math
    for a in (1, 2, 3, 4):
        exact = (-1) ** (a + 1) * (2 * math.pi) ** (2 * a) / math.factorial(2 * a)
        assert abs(F.ops.lattice_coefficient(a) - exact) <= 1e-13 * abs(exact)


def test_bench_c2_c3_point_sets_are_the_fixtures():
    """bench.SingleGP's point sets -- Lattice(3, seed=7), DigitalNetB2(3, seed=7) -- are the ones the REAL reference ran
    on in tests/golden/c2_m16_d3_it50.npz / c3_m16_d3_a2_it50.npz (generating vector / matrices and shifts)."""
    import os
    g2 = np.load(os.path.join(os.path.dirname(__file__), "golden", "c2_m16_d3_it50.npz"))
    s = F.Lattice(3, seed=7)
    assert np.array_equal(np.asarray(s.z)[:3], g2["z"]) and np.array_equal(s.shift, g2["shift"])
    g3 = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_m16_d3_a2_it50.npz"))
    s = F.DigitalNetB2(3, seed=7)
    assert int(g3["t"]) == s.t
    assert np.array_equal(s.C[:, :g3["C"].shape[1]], g3["C"].astype(np.uint64))
    assert np.array_equal(s.shift, g3["shift"].astype(np.uint64))
