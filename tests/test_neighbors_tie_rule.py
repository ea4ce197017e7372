"""Why f4's order among exactly equal distances is a documented rule, not a
reference parity target.

The reference's kNN order on ties comes from numpy: sklearn's brute force
ranks a CSR row with np.argpartition + np.argsort, and the subset lists are
merged with np.argsort(np.hstack(...)) (reference neighbors/base.py:119-128).
numpy 2.x dispatches both to SIMD kernels (x86-simd-sort) chosen at run time
from the host CPU's features, and those kernels order equal keys differently.
So the same reference code on the same data gives different tie orders on
an AVX-512, an AVX2 and a baseline x86 host: there is no single reference
order to reproduce.  This test shows it on the host at hand (skipped where
the features to switch are absent) and pins the rule the HIP path keeps:
(distance, index) ascending, the order a stable sort of the merged lists
gives (the reference's own order on every tie-free row, checked bit-exact in
test_neighbors_golden.py / test_gpu_neighbors.py).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

SNIPPET = r"""
import numpy as np
rng = np.random.default_rng(0)
a = rng.integers(0, 5, (200, 3000)).astype(np.float64)
p = np.argpartition(a, 9, axis=1)[:, :10]
s = np.argsort(np.take_along_axis(a, p, 1), axis=1)
o = np.take_along_axis(p, s, 1)
np.save(OUT, o)
"""

AVX512 = ("AVX512F AVX512CD AVX512_SKX AVX512_CLX AVX512_CNL AVX512_ICL "
          "AVX512_SPR")
AVX2 = "AVX2 FMA3 F16C " + AVX512


def _found():
    try:
        from numpy._core._multiarray_umath import __cpu_features__ as f
    except ImportError:  # pragma: no cover - older numpy layout
        from numpy.core._multiarray_umath import __cpu_features__ as f
    return f


def _order(tmp_path, tag, disable):
    out = str(tmp_path / f"{tag}.npy")
    env = dict(os.environ)
    if disable:
        env["NPY_DISABLE_CPU_FEATURES"] = disable
    subprocess.run([sys.executable, "-c", f"OUT = {out!r}\n" + SNIPPET],
                   env=env, check=True, timeout=120)
    return np.load(out)


def test_numpy_tie_order_depends_on_the_host_simd(tmp_path):
    f = _found()
    if not (f.get("AVX512F") and f.get("AVX2")):
        pytest.skip("host lacks AVX-512 / AVX2: nothing to switch")
    full = _order(tmp_path, "full", None)
    no512 = _order(tmp_path, "no512", AVX512)
    base = _order(tmp_path, "base", AVX2)
    rng = np.random.default_rng(0)
    a = rng.integers(0, 5, (200, 3000)).astype(np.float64)
    for o in (full, no512, base):
        v = np.take_along_axis(a, o, 1)
        # every build returns the 10 smallest, sorted: only ties differ
        assert np.array_equal(v, np.sort(a, axis=1)[:, :10])
    assert not (np.array_equal(full, no512) and np.array_equal(no512, base))


def test_oracle_tie_rule_is_distance_then_index():
    """The rule the kernels keep (TopK in dkm_neighbors.hip) and the oracle
    states: ascending (distance, index); NaN distances after +inf."""
    from oracle.neighbors_oracle import kneighbors_exact
    rng = np.random.default_rng(1)
    fit = rng.integers(0, 3, (300, 2)).astype(np.float64)
    fit[7] = np.nan
    q = rng.integers(0, 3, (40, 2)).astype(np.float64)
    d, i = kneighbors_exact(fit, q, 300)
    for r in range(40):
        fin = ~np.isnan(d[r])
        assert np.all(np.diff(d[r][fin]) >= 0)
        same = np.diff(d[r][fin]) == 0
        assert np.all(np.diff(i[r][fin])[same] > 0)
        assert i[r, -1] == 7 and np.isnan(d[r, -1])
