"""bench.py roofline accounting on CPU: algorithmic bytes per fit kernel for the full-length, the
half-length (R2C) and the real-even (RE) lattice kernels, and the lookup of the committed PMC
traffic for the kernel and grid the bench reports."""
import bench
import fastgaussianprocesses_amd as F


def test_stage_bytes_full_length(monkeypatch):
    monkeypatch.setenv("FGP_R2C", "0")
    n, d, P = 2 ** 20, 5, 8
    sb = bench.stage_bytes(n, d, P, parts_array=False)
    assert sb == {"k_fwd_rows": 16 * n * P, "k_fwd_cols": 40 * n * P, "k_bwd_rows": 16 * n * P}
    sb = bench.stage_bytes(n, d, P, parts_array=True)
    assert sb["k_fwd_rows"] == (16 * n + 8 * n * d) * P and sb["k_fwd_cols"] == 40 * n * P


def test_stage_bytes_half_length(monkeypatch):
    monkeypatch.setenv("FGP_R2C", "1")
    n, d, P = 2 ** 20, 5, 8
    assert bench.r2c_active(n) and not bench.r2c_active(2 ** 16)
    sb = bench.stage_bytes(n, d, P, parts_array=False)
    # work of n/2 complex values: 8n per pass; the column kernel also reads Y at the mirror pairs'
    # primaries only (n/2 values of the even Y: 4n)
    assert sb == {"k_fwd_rows": 8 * n * P, "k_fwd_cols": 20 * n * P, "k_bwd_rows": 8 * n * P}
    # below 2^17 the full-length kernels run
    assert bench.stage_bytes(2 ** 16, d, P, False)["k_fwd_cols"] == 40 * 2 ** 16 * P


def test_stage_bytes_real_even(monkeypatch):
    monkeypatch.delenv("FGP_R2C", raising=False)
    n, d, P = 2 ** 20, 5, 8
    N1 = n // (2 * 2 ** bench.re_row_log2())      # rows of the n/2-point transform (2048 by default)
    assert bench.fit_variant(n, parts_array=False) == "re"
    assert bench.fit_variant(n, parts_array=True) == "r2c"          # RE needs the parts generator
    assert bench.fit_variant(2 ** 16, parts_array=False) == "full"
    sb = bench.stage_bytes(n, d, P, parts_array=False)
    # n/4 complex values of work per pass (4n B); Y read as the pairs (Y_2k, Y_2k+1) of those n/4
    # frequencies (4n B); the Nyquist column (N1 complex) and its N1/2 adjoint values
    assert sb == {"k_fwd_rows": (4 * n + 16 * N1) * P, "k_fwd_cols": (12 * n + 20 * N1) * P,
                  "k_bwd_rows": (4 * n + 4 * N1) * P}
    N2 = 2 ** bench.re_row_log2()
    assert bench.fit_grid(n, P, "re") == {"k_fwd_rows": (P * N1 // 2, N2 // 8), "k_fwd_cols": (P * n // 16384, 256),
                                           "k_bwd_rows": (P * N1 // 2, N2 // 8)}


def test_pmc_traffic_lookup_matches_kernel_and_grid():
    """The committed profiles the bench line prices on (profiles/r03i_*): PMC traffic, VALU instructions
    and the rocprofv3 average of the dominant kernel k_spec_tile at the bench grid; exact name match."""
    n, P, d = 2 ** 20, 8, 5
    wg = bench.spec_tile_grid(n, d, P)
    assert wg == 512
    t = bench.pmc_traffic("k_spec_tile", wg * 256)
    assert t is not None and t > 0
    # PMC traffic within 2 % of the algorithmic bytes: the spectra and Y read once, no re-reads
    sb = bench.stage_bytes(n, d, P, parts_array=False, variant="spectral_fused")["k_spec_tile"]
    assert abs(t - sb) <= 0.02 * sb
    assert bench.pmc_traffic("k_spec", wg * 256) is None           # exact name match, not a prefix
    assert bench.pmc_traffic("k_spec_tile", 12345) is None
    assert bench.pmc_valu_insts("k_spec_tile", wg * 256) > 0
    assert bench.rocprof_avg_us("k_spec_tile", wg * 256) > 0


def test_path_choice():
    """The cost model (fit_engine.spectral_wanted): spectral for the BASELINE configs C2-C5 and the C4
    shifts, the transform kernels for one large high-dimensional problem."""
    assert F.fit_engine.spectral_wanted(0, 2 ** 16, 3, 1)                 # C2
    assert F.fit_engine.spectral_wanted(1, 2 ** 16, 3, 1)                 # C3
    assert F.fit_engine.spectral_wanted(0, 2 ** 20, 5, 8)                 # C4, 8 shifts sharing one basis
    assert F.fit_engine.spectral_wanted(0, 2 ** 18, 3, 1)                 # C5 shared hyper-parameters
    assert F.fit_engine.spectral_wanted(0, 2 ** 18, 3, 512)               # C5 per-output hyper-parameters
    assert not F.fit_engine.spectral_wanted(0, 2 ** 22, 5, 1)
    assert not F.fit_engine.spectral_wanted(0, 2 ** 20, 7, 8)             # d > 6


def test_gpus_flag_starts_a_launcher_child(monkeypatch, capsys):
    """bench.py --gpus N (N > 1, no WORLD_SIZE): the parent runs torch.distributed.run with N ranks over the same
    arguments as a child process and relays only rank 0's JSON line (no GPU call in the parent)."""
    import io
    import subprocess
    import sys
    seen = {}

    class FakeProc(object):
        def __init__(self, cmd, stdout=None, env=None, text=None):
            seen["cmd"], seen["env"] = cmd, env
            self.stdout = io.StringIO('some launcher chatter\n{"metric": "m", "n_gpus": 3}\n')

        def wait(self):
            return 0
    monkeypatch.setattr(subprocess, "Popen", FakeProc)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "3", "--steps", "2"])
    try:
        bench.main()
    except SystemExit as e:
        assert e.code == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "3"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "3", "--steps", "2"]
    assert capsys.readouterr().out.strip() == '{"metric": "m", "n_gpus": 3}'


def test_c4_fixture_inputs_are_the_benched_shifts():
    """tests/golden/c4_m20_d5_it50.npz (the real reference over bench.py's exact C4 work) holds the inputs bench.py
    generates: the shift seeds of rank 0, the package's default generating vector, the shifts of seqs.Lattice
    (default_rng(seed)), 51 loss-history rows per shift (50 Rprop iterations + the final evaluation)."""
    import os
    import numpy as np
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "c4_m20_d5_it50.npz"))
    d = int(g["d"])
    assert list(g["seeds"]) == bench.shard_seeds(0, 1, 8)[:2]
    for p, seed in enumerate(g["seeds"]):
        s = F.Lattice(d, seed=int(seed), randomize="SHIFT")
        assert np.array_equal(s.z, g["z"]) and np.array_equal(s.shift, g["shift"][p])
    assert g["loss_hist"].shape == (2, int(g["its"]) + 1)
    assert np.isfinite(g["pmean"]).all() and (g["pvar"] >= 0).all()


def test_timed_region_stats_takes_the_launches_between_the_markers(tmp_path):
    """tools/timed_region_stats.py: only the kernels between the first two k_clock_stamp launches count (bench.py
    brackets its timed loop with them), in kstats_grid's table format that bench.rocprof_avg_us reads."""
    import csv
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rows = []
    t = 0

    def add(name, dur, grid=131072):
        nonlocal t
        rows.append({"Kernel_Name": name, "Grid_Size_X": str(grid), "Start_Timestamp": str(t),
                     "End_Timestamp": str(t + dur)})
        t += dur

    add("void fgp::k_spec_tile<5, 2, false, false>(fgp::Nll, fgp::FitFuse)", 40000)    # eager, before
    add("fgp::k_clock_stamp(unsigned long long*)", 2000, 64)
    for _ in range(3):
        add("void fgp::k_spec_tile<5, 2, false, false>(fgp::Nll, fgp::FitFuse)", 37000)
    add("fgp::k_clock_stamp(unsigned long long*)", 2000, 64)
    add("void fgp::k_spec_tile<5, 2, false, false>(fgp::Nll, fgp::FitFuse)", 45000)    # eager, after
    add("fgp::k_clock_stamp(unsigned long long*)", 2000, 64)
    path = tmp_path / "trace.csv"
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "timed_region_stats.py"), str(path)],
                         capture_output=True, text=True, check=True).stdout
    stats = tmp_path / "timed.txt"
    stats.write_text(out)
    assert bench.rocprof_avg_us("k_spec_tile<5, 2, false, false>", 131072, path=str(stats)) == 37.0
    assert "timed region: 3 launches" in out
