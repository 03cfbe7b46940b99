"""The HIP top-k's algorithm (tools/topk_model.py) against the oracle (libstdc++)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from oracle import mx_oracle as O  # noqa: E402
from topk_model import topk_model  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")


def check_rows(rows, k):
    _, want = O.topk(rows, k)
    for r, w in zip(rows, want):
        got, _ = topk_model(r, k)
        assert np.array_equal(got, w), (k, r.tolist())


@pytest.mark.parametrize("name", ["deit", "deit30", "dit", "cross"])
def test_model_on_golden_ties(name):
    d = np.load(os.path.join(G, "topk_ties.npz"))
    check_rows(d[f"{name}_pred"][:256], int(d[f"{name}_k"]))


@pytest.mark.parametrize("n", [5, 17, 64, 65, 120, 197, 256, 300])
@pytest.mark.parametrize("nd", [1, 2, 3, 7, 1000])
def test_model_random_small_alphabets(n, nd):
    rng = np.random.default_rng(n * 1000 + nd)
    for k in sorted({1, 2, 3, 4, min(n, 20), min(n, 77), min(n, 154), n // 2 or 1, n}):
        rows = rng.integers(0, nd, (12, n)).astype(np.float32)
        if nd == 1000:
            rows = rng.standard_normal((12, n)).astype(np.float32)
        check_rows(rows, k)


def test_model_special_values():
    rng = np.random.default_rng(5)
    rows = rng.integers(-3, 3, (64, 197)).astype(np.float32)
    rows[rows == 2] = np.nan
    rows[rows == -3] = -np.inf
    rows[rows == -2] = -0.0
    rows[rows == 1] = np.inf
    for k in (1, 3, 20, 100, 197):
        check_rows(rows, k)


@pytest.mark.parametrize("n", [60, 120, 197, 256, 1000])
@pytest.mark.parametrize("k", [20, 30, 77, 154, 256])
def test_model_depth_limit_fallbacks(n, k):
    if k > n or k * 64 <= n:
        pytest.skip("not an nth_element case")
    row = O.antiqsort_row(n, k)
    _, want = O.topk(row[None], k)
    got, fallbacks = topk_model(row, k)
    assert np.array_equal(got, want[0])
    if k >= 77:
        assert fallbacks >= 1  # the adversary does reach the heap fallback here


def test_wave_model_matches_libstdcxx():
    """The one-wave-per-row top-k (tools/wave_topk_model.py, step for step the HIP
    mxa_topk_wave.hpp: rank-form partition with slot tables, pending-range stack,
    boundary bits, stable rank per final segment) against libstdc++ (oracle/topk_ref.cpp)
    on ex_pred rows, small-integer tie rows and antiqsort depth-limit rows."""
    from tools.wave_topk_model import wave_topk
    rng = np.random.default_rng(7)
    q = rng.standard_normal((1, 64, 64), dtype=np.float32)
    kk = rng.standard_normal((1, 197, 64), dtype=np.float32)
    aq, ak = O.approx_operands(q, kk, "ex_pred")
    pred = O.exact_matmul_f32(aq, np.swapaxes(ak, -1, -2)).reshape(-1, 197)
    for k in (20, 30):
        _, want = O.topk(pred, k)
        for r in range(len(pred)):
            np.testing.assert_array_equal(wave_topk(pred[r], k), want[r])
    for n, k in [(256, 154), (100, 99), (300, 17), (512, 300), (5, 3), (17, 17), (40, 1), (64, 2)]:
        for _ in range(6):
            v = rng.integers(0, 4, size=n).astype(np.float32)
            np.testing.assert_array_equal(wave_topk(v, k), O.topk(v[None], k)[1][0])
        a = O.antiqsort_row(n, k)
        np.testing.assert_array_equal(wave_topk(a, k), O.topk(a[None], k)[1][0])
