"""GPU parity of the label-hinted threshold pass of the single-product
screen: k_screen_b2 (centres on the lanes, dkm_b2.hip) and the k_screen_b1
it replaces (mode flag DKM_MODE_B1), against the oracle's restatement of the
reference assignment (dislib cluster/kmeans/base.py:171-173, 204-205).

The image variant also checks the image itself against the fp64 -> fp32 ->
bf16 roundings (test_sample_image_layout).  Shapes cover every K-step count the kernels instantiate that the LDS admits,
k % 32 != 0 (hints pointing into a partial last block), an odd number of
centre blocks (the pipeline's tail), k > 1024 (own masks of several words),
and a shape whose b2 image does not fit LDS (the b1 fallback).  Hint kinds:
the right labels, 30 % wrong, and exact duplicate centres placed in EVERY
centre block with the hint on the later copy -- every block position then
takes the append branch, and the first index must win the exact tie.
"""
import os

import numpy as np
import pytest

from oracle import kmeans_oracle as orc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


_VARIANT = {"name": "img"}


@pytest.fixture(params=["img", "b2", "b1", "sorted"])
def variant(request, monkeypatch):
    """img: k_screen_b2 streaming the sample image; b2: the same kernel
    converting X itself; b1: k_screen_b1 (DKM_MODE_B1); sorted: k_screen_b2
    over the label-sorted image (the fit's default from iteration 2), built
    from a shuffled copy of the hints, with block skipping."""
    from dislib_amd import _device
    monkeypatch.setattr(_device, "X_IMAGE", request.param in ("img",
                                                             "sorted"))
    monkeypatch.setitem(_VARIANT, "name", request.param)
    yield request.param


def _hinted(x, C, hint, acc_kind="partial"):
    from dislib_amd import _device, _lib
    from dislib_amd.data import load_data
    dev = torch.device("cuda", 0)
    ds = load_data(x, subset_size=x.shape[0])
    dd = ds._device_data()
    k, d = C.shape
    Ct = torch.from_numpy(np.ascontiguousarray(C)).to(dev)
    ws = _device.Workspace(k, d, dd.n, dev)
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    lab = torch.from_numpy(np.asarray(hint).astype(np.int32)).to(dev)
    mode = _lib.MODE_BF16
    image = None
    v = _VARIANT["name"]
    if v == "b1":
        mode |= _lib.MODE_B1
    _device.prepare(Ct, ws, acc)
    if v == "sorted":
        if not _lib.lib().dkm_x_image_sorted_ok(k, d):
            pytest.skip("(k, d) does not take the sorted image")
        # grouped by the incoming labels themselves: the image's label copy
        # must equal them (the fit builds it from the labels it passes)
        image = _device.sorted_image(dd, lab, k, ws)
        assert image[0] is not None
    if acc_kind == "partial":
        _device.partial_sum(dd, Ct, ws, lab, acc, mode, image=image)
    else:
        _device.assign_delta(dd, Ct, ws, lab, acc, mode, image=image)
    a = acc.cpu().numpy()
    return lab.cpu().numpy(), a[:k * d].reshape(k, d), a[k * d:]


def _problem(n, d, k, seed):
    rng = np.random.default_rng(seed)
    blobs = rng.uniform(-10, 10, (k, d))
    x = blobs[rng.integers(0, k, n)] + rng.standard_normal((n, d))
    C = blobs + rng.standard_normal((k, d)) * 0.3
    return rng, x, C


def _dups_every_block(rng, C):
    """An exact copy of some centre in every 32-centre block (a different
    slot per block); returns (copy, original) index pairs."""
    k = C.shape[0]
    nkb = (k + 31) // 32
    pairs = []
    used = set()
    for b in range(nkb):
        j = min(32 * b + (5 * b + 3) % 32, k - 1)
        p = (j + 37 + 11 * b) % k
        if j in used or p in used or j == p:
            continue
        used.update((j, p))
        C[j] = C[p]
        pairs.append((j, p))
    return pairs


@pytest.mark.parametrize("d,k", [(16, 300), (32, 600), (64, 1000), (64, 990),
                                 (48, 777), (96, 500), (16, 2000),
                                 (128, 560)])
@pytest.mark.parametrize("kind", ["exact", "noisy", "dups"])
def test_threshold_pass_shapes(variant, d, k, kind):
    n = 30000
    rng, x, C = _problem(n, d, k, 1000 * d + k)
    if kind == "dups":
        pairs = _dups_every_block(rng, C)
        # samples at both copies of each pair: an exact tie between them
        m = len(pairs)
        idx = rng.integers(0, n, 40 * m)
        for t, i in enumerate(idx):
            j, p = pairs[t % m]
            x[i] = C[p] + rng.standard_normal(d)
    rl, rs, rc = orc.partial_sum(x, C)
    if kind == "exact":
        hint = rl
    elif kind == "noisy":
        hint = np.where(rng.random(n) < 0.3, rng.integers(0, k, n), rl)
    else:
        # hint = the LATER copy of a duplicated pair (the reference picks the
        # first index: the pass must find the earlier copy as a tie)
        _, inv = np.unique(C, axis=0, return_inverse=True)
        inv = np.asarray(inv).reshape(-1)
        last = {}
        for c in range(k):
            last[inv[c]] = c
        hint = np.array([last[inv[c]] for c in rl])
        assert (hint != rl).sum() > 0
    lab, sums, cnt = _hinted(x, C, hint)
    assert np.array_equal(lab, rl), (lab != rl).sum()
    assert np.array_equal(cnt, rc.astype(np.float64))
    err = np.max(np.abs(sums - rs) / np.maximum(np.abs(rs), 1.0))
    assert err <= 1e-12


@pytest.mark.parametrize("d,k", [(64, 1000), (16, 2000)])
def test_threshold_pass_delta(variant, d, k):
    """dkm_assign_delta with previous labels as the hint (the fit loop's
    call): labels exact and the delta of the sums."""
    n = 30000
    rng, x, C = _problem(n, d, k, 7 * d + k)
    prev = orc.predict_labels(x, C + 0.2 * rng.standard_normal(C.shape))
    prev[rng.random(n) < 0.01] = -1
    rl, rs, rc = orc.partial_sum(x, C)
    lab, sums, cnt = _hinted(x, C, prev, acc_kind="delta")
    assert np.array_equal(lab, rl)
    ps = np.zeros((k, d))
    pc = np.zeros(k)
    ok = prev >= 0
    np.add.at(ps, prev[ok], x[ok])
    np.add.at(pc, prev[ok], 1)
    assert np.array_equal(cnt, rc - pc)
    err = np.max(np.abs(sums - (rs - ps)) / np.maximum(np.abs(rs), 1.0))
    assert err <= 1e-11


def test_threshold_pass_tail_and_hint_edge_cases(variant):
    """n not a multiple of 32 (a partial last tile), hints at -1, k, k-1
    (the last, partially filled block) and 0, a constant hint for a whole
    wave tile, and a crowded group (overfull kept lists: top-3 fallback)."""
    n, d, k = 20011, 64, 1000
    rng, x, C = _problem(n, d, k, 5)
    z = rng.uniform(-10, 10, d)
    C[960:] = z + 0.05 * rng.standard_normal((40, d))
    near = rng.random(n) < 0.05
    x[near] = z + rng.standard_normal((int(near.sum()), d))
    rl, rs, rc = orc.partial_sum(x, C)
    hint = rl.copy()
    sel = rng.random(n)
    hint[sel < 0.02] = -1
    hint[(sel >= 0.02) & (sel < 0.04)] = k
    hint[(sel >= 0.04) & (sel < 0.06)] = k - 1
    hint[(sel >= 0.06) & (sel < 0.08)] = 0
    hint[64:96] = 17
    lab, sums, cnt = _hinted(x, C, hint)
    assert np.array_equal(lab, rl)
    assert np.array_equal(cnt, rc.astype(np.float64))


def test_refresh_skipped_once_converged(monkeypatch):
    """The periodic full recomputation of the running sums is skipped when
    no delta since the last one moved a sample (the sums are then exactly
    those of the current assignment): a fit that converges early makes
    fewer full passes than it < max_iter / REFRESH, and still matches the
    oracle (labels bit-exact, centres 1e-9, n_iter)."""
    from sklearn.datasets import make_blobs

    import dislib_amd.cluster.kmeans as km_mod
    from dislib_amd import _device
    from dislib_amd.cluster import KMeans
    from dislib_amd.data import load_data
    x, _ = make_blobs(n_samples=20000, n_features=64, centers=200,
                      center_box=(-10, 10), random_state=4)
    ref = orc.OracleKMeans(n_clusters=200, max_iter=14, tol=0,
                           random_state=0)
    rl = ref.fit([x[i:i + 5000] for i in range(0, 20000, 5000)],
                 set_labels=True)
    calls = []
    real = _device.partial_sum

    def counted(*a, **kw):
        calls.append(1)
        return real(*a, **kw)
    monkeypatch.setattr(_device, "partial_sum", counted)
    monkeypatch.setattr(km_mod, "REFRESH", 2)
    ds = load_data(x, 5000)
    km = KMeans(n_clusters=200, max_iter=14, tol=0, random_state=0)
    km.fit_predict(ds)
    assert km.n_iter == ref.n_iter
    assert np.array_equal(ds.labels_int32(), rl)
    err = np.max(np.abs(km.centers - ref.centers) /
                 np.maximum(np.abs(ref.centers), 1.0))
    assert err <= 1e-9
    assert 1 <= len(calls) < 7, len(calls)


@pytest.mark.parametrize("n,d", [(1000, 64), (77, 20), (33, 128), (64, 1)])
def test_sample_image_layout(n, d):
    """dkm_x_image_f64: 32-row tiles of dpad16(d) / 16 K-steps; lane l of
    K-step ks holds row l & 31, features 16 ks + 8 (l >> 5) + 0..7, rounded
    fp64 -> fp32 -> bf16 (nearest even); rows and features past n, d zero;
    then fp32 |x|^2 of the fp32 values per row (32 per tile)."""
    from dislib_amd import _device, _lib
    so = _lib.lib()
    rng = np.random.default_rng(n + d)
    x = rng.standard_normal((n, d)) * 10.0 ** rng.integers(-3, 4, (n, 1))
    X = torch.from_numpy(x).cuda()
    nb = so.dkm_x_image_bytes(n, d, _lib.IMAGE_SINGLE)
    nt, nks = (n + 31) // 32, (d + 15) // 16
    assert nb == nt * nks * 1024 + nt * 128
    img = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    _lib.check(so.dkm_x_image_f64(_device.ptr(X), n, d, d, _lib.IMAGE_SINGLE,
                                  _device.ptr(img), nb, _device.stream_ptr()),
               "image")
    raw = img.cpu().numpy()
    tiles = raw[:nt * nks * 1024].view(np.uint16).reshape(nt, nks, 64, 8)
    xx = raw[nt * nks * 1024:].view(np.float32)
    # fp32 -> bf16 round to nearest even (finite values)
    f = np.zeros((nt * 32, nks * 16), np.float32)
    f[:n, :d] = x.astype(np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    bf = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    bf = bf.reshape(nt, 32, nks, 2, 8)            # tile, row, ks, half, j
    want = bf.transpose(0, 2, 3, 1, 4).reshape(nt, nks, 64, 8)
    assert np.array_equal(tiles, want)
    ref = (f.astype(np.float64) ** 2).sum(1)
    assert np.all(np.abs(xx - ref) <= 2.0 ** -23 * ref)
    assert np.all(xx[n:] == 0)


def test_threshold_pass_non_finite_rows(variant):
    """Rows holding NaN or +-inf (and rows whose squares overflow fp32) in a
    tile of ordinary rows: the screen sends them to the exact path, they do
    not disturb the other rows' labels or counts, and every label -- the
    non-finite rows' too -- is the reference's: np.argmin over their NaN
    (first NaN) or all-inf (first index) distances (base.py:173)."""
    n, d, k = 20011, 64, 1000
    rng, x, C = _problem(n, d, k, 23)
    bad = rng.choice(n, 200, replace=False)
    x[bad[:50], rng.integers(0, d, 50)] = np.nan
    x[bad[50:100], rng.integers(0, d, 50)] = np.inf
    x[bad[100:150], rng.integers(0, d, 50)] = -np.inf
    x[bad[150:]] *= 1e25                       # |x|^2 overflows fp32
    rl, rs, rc = orc.partial_sum(x, C)
    hint = rl.copy()
    lab, sums, cnt = _hinted(x, C, hint)
    assert np.all((lab >= 0) & (lab < k))
    assert np.array_equal(lab, rl)
    assert np.array_equal(cnt, rc.astype(np.float64))
