"""GPU parity of the large-d path (d > 128): the MFMA GEMM screen
(dkm_gemm.hip; bf16x3, and the single-product mode auto picks) + exact
candidate evaluation + exact re-check, against the CPU oracle and against
golden vectors produced by the reference itself.

Bar (BASELINE.json north star): labels bit-exact; centres within 1e-9
relative in fp64 (1e-4 for fp32 samples); sums within 1e-12 of the oracle's
sequential fp64 sums.
"""
import hashlib

import numpy as np
import pytest
from sklearn.datasets import make_blobs

from oracle import kmeans_oracle as orc
from tests.conftest import load_golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _close(a, b, rtol):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = np.maximum(np.abs(b), 1.0)
    err = np.max(np.abs(a - b) / scale) if a.size else 0.0
    assert err <= rtol, "max rel err %g > %g" % (err, rtol)


def _load(x, n):
    from dislib_amd.data import load_data
    return load_data(x, subset_size=n)


def _run(x, C, mode="bf16x3", kind="partial", prev=None):
    """One assignment call through the C ABI; returns labels, sums, counts,
    re-checked count."""
    from dislib_amd import _device, _lib
    dev = torch.device("cuda")
    ds = _load(x, x.shape[0])
    dd = ds._device_data()
    k, d = C.shape
    Ct = torch.from_numpy(np.ascontiguousarray(C)).to(dev)
    ws = _device.Workspace(k, d, dd.n, dev)
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    m = {"exact": _lib.MODE_EXACT, "bf16x3": _lib.MODE_BF16X3,
         "bf16": _lib.MODE_BF16, "auto": _lib.MODE_AUTO}[mode]
    _device.prepare(Ct, ws, acc)
    if kind == "partial":
        lab = torch.full((dd.n,), -7, dtype=torch.int32, device=dev)
        _device.partial_sum(dd, Ct, ws, lab, acc, m)
    elif kind == "delta":
        lab = torch.from_numpy(prev.astype(np.int32)).to(dev)
        _device.assign_delta(dd, Ct, ws, lab, acc, m)
    else:
        lab = torch.full((dd.n,), -7, dtype=torch.int32, device=dev)
        _device.predict(dd, Ct, ws, lab, m)
    a = acc.cpu().numpy()
    return (lab.cpu().numpy(), a[:k * d].reshape(k, d), a[k * d:],
            _device.rechecked(ws))


def _data(n, d, k, seed, dtype=np.float64):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, d)) * rng.uniform(0.5, 8)
    x += rng.uniform(-5, 5, (1, d))
    C = x[rng.choice(n, k, replace=False)] + rng.standard_normal((k, d)) * 0.1
    return x.astype(dtype), C


@pytest.mark.parametrize("n,d,k,seed", [
    (3000, 129, 40, 0),      # one 32-feature stage of padding
    (2000, 200, 300, 1),     # two centre tiles, second one ragged
    (1500, 257, 600, 2),     # d % 8 != 0: unaligned split loads
    (1200, 1024, 700, 3),    # C4 feature count
    (800, 300, 3, 4),        # k < 4: padding centres in the kept lists
    (600, 2048, 64, 5),      # 64 K-stages
    (70, 160, 9, 6),         # a single partial sample tile
])
@pytest.mark.parametrize("gmode", ["bf16x3", "bf16"])
def test_gemm_partial_sum_vs_oracle(n, d, k, seed, gmode):
    x, C = _data(n, d, k, seed)
    lab, sums, cnt, _ = _run(x, C, mode=gmode)
    rl, rs, rc = orc.partial_sum(x, C)
    assert np.array_equal(lab, rl)
    assert np.array_equal(cnt, rc.astype(np.float64))
    _close(sums, rs, 1e-12)
    plab, _, _, _ = _run(x, C, mode=gmode, kind="predict")
    assert np.array_equal(plab, rl)


@pytest.mark.parametrize("gmode", ["bf16x3", "bf16"])
def test_gemm_fp32_samples(gmode):
    x, C = _data(3000, 300, 100, 7, np.float32)
    lab, sums, cnt, _ = _run(x, C, mode=gmode)
    rl, rs, rc = orc.partial_sum(x, C)
    assert np.array_equal(lab, rl)
    assert np.array_equal(cnt, rc.astype(np.float64))
    _close(sums, rs, 1e-4)


@pytest.mark.parametrize("d,k", [(200, 300), (1024, 600)])
@pytest.mark.parametrize("gmode", ["bf16x3", "bf16"])
def test_gemm_delta_equals_difference_of_partial_sums(d, k, gmode):
    x, C = _data(4000, d, k, d + k)
    prev = np.random.default_rng(1).integers(-1, k, x.shape[0])
    lab, sums, cnt, _ = _run(x, C, mode=gmode, kind="delta", prev=prev)
    rl, rs, rc = orc.partial_sum(x, C)
    assert np.array_equal(lab, rl)
    ps = np.zeros((k, d))
    pc = np.zeros(k)
    ok = prev >= 0
    np.add.at(ps, prev[ok], x[ok])
    np.add.at(pc, prev[ok], 1)
    _close(sums, rs - ps, 1e-11)
    assert np.array_equal(cnt, rc - pc)


@pytest.mark.parametrize("gmode", ["bf16x3", "bf16"])
def test_gemm_candidate_and_recheck_branches(gmode):
    """Force every decision branch of the merge: (a) several centres within
    the bound in DIFFERENT centre tiles (complete candidate list: exact
    evaluation of the candidates), (b) more than 3 near-identical centres
    in ONE tile (incomplete: k_recheck_exact over all centres), (c) exact
    ties (first index wins)."""
    rng = np.random.default_rng(11)
    d, k = 300, 700
    base = rng.uniform(-4, 4, (k, d))
    C = base.copy()
    # (a) centre 5 ~ centre 400 ~ centre 650 (tiles 0, 1, 2)
    C[400] = C[5] + 1e-9 * rng.standard_normal(d)
    C[650] = C[5] + 1e-9 * rng.standard_normal(d)
    # (b) centres 100..105 (all in tile 0) nearly identical
    for j in range(101, 106):
        C[j] = C[100] + 1e-9 * rng.standard_normal(d)
    # (c) exact duplicates in tiles 1 and 2: the first index must win
    C[520] = C[300].copy()
    C[300] = C[600].copy()
    xs = []
    for c in (5, 100, 300, 520, 600):
        xs.append(C[c] + 0.01 * rng.standard_normal((200, d)))
    xs.append(rng.uniform(-4, 4, (400, d)))
    x = np.vstack(xs)
    lab, sums, cnt, nre = _run(x, C, mode=gmode)
    rl, rs, rc = orc.partial_sum(x, C)
    assert np.array_equal(lab, rl)
    assert np.array_equal(cnt, rc.astype(np.float64))
    _close(sums, rs, 1e-12)
    assert nre >= 200              # branch (b) went to the exact re-check


@pytest.mark.parametrize("scale", [1e-30, 1e-3, 1.0, 1e6])
@pytest.mark.parametrize("gmode", ["bf16x3", "bf16"])
def test_gemm_near_ties_across_scales(scale, gmode):
    rng = np.random.default_rng(int(np.log10(scale) + 60))
    d, k = 192, 40
    C = rng.uniform(-10, 10, (k, d)) * scale
    xs = []
    for _ in range(3000):
        a, b = rng.choice(k, 2, replace=False)
        u = C[a] - C[b]
        w = rng.standard_normal(d)
        w -= w.dot(u) / u.dot(u) * u
        eps = rng.choice([0.0, 1.0]) * rng.uniform(-1, 1) * \
            10.0 ** -rng.integers(6, 16)
        xs.append(0.5 * (C[a] + C[b]) + 0.2 * scale * w + eps * u)
    x = np.array(xs)
    lab, _, _, _ = _run(x, C, mode=gmode)
    assert np.array_equal(lab, orc.predict_labels(x, C))


@pytest.mark.parametrize("gmode", ["bf16x3", "bf16"])
def test_gemm_nonfinite_samples_go_exact(gmode):
    x, C = _data(1000, 160, 20, 12)
    x[3, 7] = np.nan
    x[9, 0] = np.inf
    x[11] = 1e200
    lab, _, _, _ = _run(x, C, mode=gmode)
    ok = np.isfinite(x).all(axis=1)
    rl = orc.predict_labels(x, C)
    assert np.array_equal(lab, rl)
    assert ok.sum() == 998


@pytest.mark.parametrize("gmode", ["bf16x3", "bf16"])
def test_gemm_c4_shape_vs_exact_kernel(gmode):
    """d = 1024, k = 4096 (BASELINE configs[3]) on 20k samples: every label
    against the exact kernel (the reference arithmetic for every pair, pinned
    to the oracle by the parity tests), 400 of them against the oracle."""
    d, k, n = 1024, 4096, 20000
    x, _ = make_blobs(n_samples=n, n_features=d, centers=k,
                      center_box=(-10, 10), random_state=15)
    rng = np.random.default_rng(4)
    C = x[rng.choice(n, k, replace=False)] + rng.standard_normal((k, d))
    lab, sums, cnt, _ = _run(x, C, mode=gmode)
    ref, _, _, _ = _run(x[:4000], C, mode="exact", kind="predict")
    assert np.array_equal(lab[:4000], ref)
    assert cnt.sum() == n
    sub = rng.choice(n, 400, replace=False)
    assert np.array_equal(lab[sub], orc.predict_labels(x[sub], C))
    # sums: one cluster's rows add up exactly as the oracle's chain does
    j = int(np.argmax(cnt))
    _close(sums[j], x[lab == j].sum(axis=0), 1e-12)


@pytest.mark.parametrize("gmode", ["bf16x3", "bf16"])
def test_gemm_c4_shape_fp32_samples(gmode):
    """The fp32 variant of configs[3] (reported separately by bench.py):
    fp32 samples at d = 1024, k = 4096 on 20k rows -- fp64 distances, so
    labels bit-exact against the exact kernel and the oracle; fp32 partial
    sums within 1e-4 relative of the oracle's."""
    d, k, n = 1024, 4096, 20000
    x, _ = make_blobs(n_samples=n, n_features=d, centers=k,
                      center_box=(-10, 10), random_state=16)
    x = x.astype(np.float32)
    rng = np.random.default_rng(5)
    C = x[rng.choice(n, k, replace=False)].astype(np.float64) + \
        rng.standard_normal((k, d))
    lab, sums, cnt, _ = _run(x, C, mode=gmode)
    ref, _, _, _ = _run(x[:4000], C, mode="exact", kind="predict")
    assert np.array_equal(lab[:4000], ref)
    assert cnt.sum() == n
    sub = rng.choice(n, 400, replace=False)
    assert np.array_equal(lab[sub], orc.predict_labels(x[sub], C))
    for j in np.argsort(cnt)[-3:]:
        ref_sum = x[lab == j].sum(axis=0, dtype=np.float32)
        _close(sums[j], ref_sum, 1e-4)


def test_f15_c4mini_fit_predict_vs_reference():
    """Golden vectors of the reference's own KMeans at the C4 shape:
    make_blobs(20000 x 1024, 4096 centres), KMeans(4096, max_iter=2, tol=0,
    random_state=0).fit_predict (tests/golden/gen_golden_big.py)."""
    from dislib_amd.cluster import KMeans
    g = load_golden("f15_c4mini")
    x, _ = make_blobs(n_samples=20_000, n_features=1024, centers=4096,
                      center_box=(-10, 10), random_state=15)
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["x_sha"])
    ds = _load(x, 5000)
    km = KMeans(n_clusters=4096, max_iter=2, tol=0, random_state=0)
    km.fit_predict(ds)
    assert km.n_iter == int(g["n_iter"])
    lab = ds.labels_int32()
    assert np.array_equal(lab, g["labels"].astype(np.int32))
    assert np.array_equal(np.bincount(lab, minlength=4096), g["counts"])
    C = km.centers
    R = np.random.RandomState(1).standard_normal((1024, 8))
    tol = 1e-9 * (np.abs(C) @ np.abs(R)) + 1e-12
    assert (np.abs(C @ R - g["proj"]) <= tol).all()
    _close(C.sum(axis=1), g["rowsum"], 1e-9)
    _close(C[g["top"]], g["top_rows"], 1e-9)
