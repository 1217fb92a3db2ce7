"""bench.py roofline accounting on CPU: algorithmic bytes per fit kernel for the full-length and the
half-length (R2C) lattice kernels, and the lookup of the committed PMC
traffic for the kernel and grid the bench reports."""
import bench


def test_stage_bytes_full_length(monkeypatch):
    monkeypatch.setenv("FGP_R2C", "0")
    n, d, P = 2 ** 20, 5, 8
    sb = bench.stage_bytes(n, d, P, parts_array=False)
    assert sb == {"k_fwd_rows": 16 * n * P, "k_fwd_cols": 40 * n * P, "k_bwd_rows": 16 * n * P}
    sb = bench.stage_bytes(n, d, P, parts_array=True)
    assert sb["k_fwd_rows"] == (16 * n + 8 * n * d) * P and sb["k_fwd_cols"] == 40 * n * P


def test_stage_bytes_half_length(monkeypatch):
    monkeypatch.delenv("FGP_R2C", raising=False)
    n, d, P = 2 ** 20, 5, 8
    assert bench.r2c_active(n) and not bench.r2c_active(2 ** 16)
    sb = bench.stage_bytes(n, d, P, parts_array=False)
    # work of n/2 complex values: 8n per pass; the column kernel also reads Y at the mirror pairs'
    # primaries only (n/2 values of the even Y: 4n)
    assert sb == {"k_fwd_rows": 8 * n * P, "k_fwd_cols": 20 * n * P, "k_bwd_rows": 8 * n * P}
    # below 2^17 the full-length kernels run
    assert bench.stage_bytes(2 ** 16, d, P, False)["k_fwd_cols"] == 40 * 2 ** 16 * P


def test_pmc_traffic_lookup_matches_kernel_and_grid():
    n, P = 2 ** 20, 8
    t = bench.pmc_traffic("k_fwd_cols_r2c", P * (n // 2) // 4096 * 256)
    assert t is not None and t > 0
    # the full-length kernel name must not match the R2C entry (exact name match, not a suffix)
    assert bench.pmc_traffic("k_fwd_cols", P * (n // 2) // 4096 * 256) is None
    assert bench.pmc_traffic("k_fwd_cols_r2c", 12345) is None
