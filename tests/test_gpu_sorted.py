"""The label-sorted sample image (DKM_IMAGE_SORTED, dkm_x_image_sorted_*)
and the block skipping of k_screen_b2 over it.

The reference assigns every sample by computing its distance to every
centre (dislib cluster/kmeans/base.py:171-173).  The build screens the
rows of a label-sorted image tile by tile and skips the 32-centre blocks
the triangle inequality proves farther than the tile's hinted centre.  The
labels must not depend on that: they are checked against the oracle, and
against the same fit without the image.
"""
import numpy as np
import pytest
from sklearn.datasets import make_blobs

from oracle import kmeans_oracle as orc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("n,d,k", [(1000, 64, 300), (77, 24, 40),
                                   (4100, 128, 200), (64, 16, 2000)])
def test_sorted_image_layout(n, d, k):
    """Rows grouped by label (labels outside [0, k) after them, -1 past n),
    the label copy equal to labels[perm], and each tile the SINGLE image's
    tile of the permuted rows (fp64 -> fp32 -> bf16, |x|^2 in fp32)."""
    from dislib_amd import _device, _lib
    from dislib_amd.data import load_data
    so = _lib.lib()
    if not so.dkm_x_image_sorted_ok(k, d):
        pytest.skip("(k, d) does not take the sorted image")
    rng = np.random.default_rng(n + d + k)
    x = rng.standard_normal((n, d)) * 10.0 ** rng.integers(-2, 3, (n, 1))
    lab = rng.integers(-1, k + 1, n).astype(np.int32)
    dev = torch.device("cuda", 0)
    dd = load_data(x, subset_size=n)._device_data()
    ws = _device.Workspace(k, d, n, dev)
    img, kind = _device.sorted_image(dd, torch.from_numpy(lab).to(dev), k, ws)
    assert kind == _lib.IMAGE_SORTED
    _check_sorted_layout(img.cpu().numpy(), x, lab, k)


def _check_sorted_layout(raw, x, lab, k):
    n, d = x.shape
    nt, nks = (n + 31) // 32, (d + 15) // 16
    tb = nt * nks * 1024
    tiles = raw[:tb].view(np.uint16).reshape(nt, nks, 64, 8)
    xx = raw[tb:tb + nt * 128].view(np.float32)
    perm = raw[tb + nt * 128:tb + nt * 256].view(np.int32)
    plab = raw[tb + nt * 256:tb + nt * 384].view(np.int32)
    assert np.all(perm[n:] == -1) and np.all(plab[n:] == -1)
    p = perm[:n]
    assert np.array_equal(np.sort(p), np.arange(n))       # a permutation
    lp = lab[p]
    ok = (lp >= 0) & (lp < k)
    m = int(ok.sum())
    assert ok[:m].all() and not ok[m:].any()              # unlabelled last
    assert np.all(np.diff(lp[:m]) >= 0)                   # grouped, in order
    # the label copy holds labels outside [0, k) as -1 (a negative copy is
    # read as a re-check marker by the label sync)
    assert np.array_equal(plab[:n], np.where((lp >= 0) & (lp < k), lp, -1))
    f = np.zeros((nt * 32, nks * 16), np.float32)
    f[:n, :d] = x[p].astype(np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    bf = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    want = bf.reshape(nt, 32, nks, 2, 8).transpose(0, 2, 3, 1, 4).reshape(
        nt, nks, 64, 8)
    assert np.array_equal(tiles, want)
    ref = (f.astype(np.float64) ** 2).sum(1)
    assert np.all(np.abs(xx - ref) <= 2.0 ** -23 * ref)


def _fit(x, k, iters, sorted_on, monkeypatch, subset=None):
    import dislib_amd.cluster.kmeans as km_mod
    from dislib_amd.cluster import KMeans
    from dislib_amd.data import load_data
    monkeypatch.setattr(km_mod, "SORTED_IMAGE", sorted_on)
    ds = load_data(x, subset or x.shape[0])
    km = KMeans(n_clusters=k, max_iter=iters, tol=0, random_state=0)
    km.fit_predict(ds)
    return km, ds.labels_int32()


def test_sorted_fit_matches_oracle(monkeypatch):
    """A C3-shaped fit (d = 64, k = 1000, blobs) through the label-sorted
    image from iteration 2 on: labels bit-exact and centres within 1e-9 of
    the oracle, and blocks were really skipped."""
    from dislib_amd import _device
    x, _ = make_blobs(n_samples=60_000, n_features=64, centers=300,
                      center_box=(-10, 10), random_state=7)
    ref = orc.OracleKMeans(n_clusters=1000, max_iter=6, tol=0,
                           random_state=0)
    rl = ref.fit([x[i:i + 20_000] for i in range(0, 60_000, 20_000)],
                 set_labels=True)
    seen = {}
    real = _device.sorted_image

    def spy(*a, **kw):
        out = real(*a, **kw)
        seen["built"] = out[0] is not None
        return out
    monkeypatch.setattr(_device, "sorted_image", spy)
    km, lab = _fit(x, 1000, 6, True, monkeypatch, 20_000)
    assert seen.get("built")
    assert km.n_iter == ref.n_iter
    assert np.array_equal(lab, np.asarray(rl))
    err = np.max(np.abs(km.centers - ref.centers) /
                 np.maximum(np.abs(ref.centers), 1.0))
    assert err <= 1e-9


@pytest.mark.parametrize("seed,blobs,std", [(0, 1000, 1.0), (1, 50, 4.0),
                                            (2, 3000, 0.3)])
def test_sorted_and_unsorted_fits_agree(monkeypatch, seed, blobs, std):
    """400k x 64, k = 1000 on device blobs (the bench generator): the fit
    with and without the sorted image gives identical labels, centres and
    iteration counts, for well-separated blobs (most blocks skipped), few
    wide blobs (crowded centres: little to skip) and tight ones."""
    from dislib_amd import _device
    from dislib_amd.cluster.kmeans import _Lloyd, _init_centers
    from dislib_amd.data import Dataset, Subset
    import dislib_amd.cluster.kmeans as km_mod
    n, d, k = 400_000, 64, 1000
    dev = torch.device("cuda", 0)
    X = torch.empty((n, d), dtype=torch.float64, device=dev)
    _device.make_blobs(X, seed * n, blobs, seed=seed, box=10.0, std=std)
    out = {}
    for on in (False, True):
        monkeypatch.setattr(km_mod, "SORTED_IMAGE", on)
        ds = Dataset(n_features=d)
        ds.append(Subset(X))
        st = _Lloyd(ds, _init_centers(d, False, k, seed), 0.0, True, "auto",
                    dev)
        for _ in range(7):
            st.step()
        out[on] = (st.labels[:n].cpu().numpy(), st.C.cpu().numpy(),
                   st.screened_blocks(), st.simg is not None)
    assert out[True][3] and not out[False][3]
    assert np.array_equal(out[True][0], out[False][0])
    err = np.max(np.abs(out[True][1] - out[False][1]) /
                 np.maximum(np.abs(out[False][1]), 1.0))
    assert err <= 1e-12
    tiles, done, blocks, handed = out[True][2]
    assert 0 <= handed <= tiles
    assert 0 < blocks <= 32 * tiles
    if blobs == 1000:       # separated blobs: most blocks are cleared
        assert blocks < 16 * tiles, (blocks, tiles)


@pytest.mark.parametrize("n,d,k,f32,out", [(5000, 64, 300, False, 0.0),
                                           (4100, 128, 200, True, 0.0),
                                           (777, 16, 2000, False, 0.0),
                                           (3000, 40, 100, False, 0.0),
                                           (9000, 24, 64, True, 0.0),
                                           (6000, 64, 500, False, 0.1)])
def test_sorted_image_sums_fused(n, d, k, f32, out):
    """dkm_x_image_sorted_sums_*: the image of dkm_x_image_sorted_*, and acc += the dkm_label_sums_* result (fp64
    atomics: equal up to the order of the additions); d = 40 (three 16-wide
    slices) takes the image, then the separate sums."""
    from dislib_amd import _device, _lib
    from dislib_amd.data import load_data
    so = _lib.lib()
    if not so.dkm_x_image_sorted_ok(k, d):
        pytest.skip("(k, d) does not take the sorted image")
    rng = np.random.default_rng(n + d + k)
    x = rng.standard_normal((n, d)) * 10.0 ** rng.integers(-2, 3, (n, 1))
    if f32:
        x = x.astype(np.float32)
    lab = rng.integers(0, k, n).astype(np.int32)
    lab[: n // 3] = rng.integers(0, 3, n // 3)          # a few big clusters
    if out:       # labels outside [0, k): sorted after the others, no sums
        m = rng.random(n) < out
        lab[m] = np.where(rng.random(int(m.sum())) < 0.5, -1, k)
    dev = torch.device("cuda", 0)
    dd = load_data(x, subset_size=n)._device_data()
    ws = _device.Workspace(k, d, n, dev)
    lt = torch.from_numpy(lab).to(dev)
    img0, _ = _device.sorted_image(dd, lt, k, ws)
    want = torch.full((k * (d + 1),), 0.5, dtype=torch.float64, device=dev)
    _device.label_sums(dd, ws, lt, want, k)
    acc = torch.full_like(want, 0.5)
    img1, kind = _device.sorted_image(dd, lt, k, ws, acc=acc)
    assert kind == _lib.IMAGE_SORTED
    # the order within a cluster is the counting sort's (not fixed): each
    # image is checked for the layout on its own
    _check_sorted_layout(img1.cpu().numpy(), x, lab, k)
    _check_sorted_layout(img0.cpu().numpy(), x, lab, k)
    a, w = acc.cpu().numpy(), want.cpu().numpy()      # [sums k x d | counts]
    assert np.array_equal(a[k * d:], w[k * d:])
    scale = np.zeros((k, d))
    ok = (lab >= 0) & (lab < k)
    np.add.at(scale, lab[ok], np.abs(x[ok].astype(np.float64)))
    assert np.all(np.abs(a[:k * d] - w[:k * d]) <=
                  1e-13 * (scale.ravel() + 1.0))


@pytest.mark.parametrize("seed,frac_out", [(0, 0.0), (1, 0.01), (2, 0.2)])
def test_sorted_delta_lists_the_moved_rows(seed, frac_out):
    """The incremental pass over the label-sorted image: the label sync lists
    the moved rows with their previous labels (no label copy, no scan), and
    the delta is sums(new) - sums(previous) with previous labels outside
    [0, k) contributing nothing; labels bit-exact against the oracle, and the
    image's label copy follows them."""
    from dislib_amd import _device, _lib
    from dislib_amd.data import load_data
    so = _lib.lib()
    n, d, k = 60_000, 64, 1000
    if not so.dkm_x_image_sorted_ok(k, d):
        pytest.skip("(k, d) does not take the sorted image")
    rng = np.random.default_rng(seed)
    blobs = rng.uniform(-10, 10, (300, d))
    x = blobs[rng.integers(0, 300, n)] + rng.standard_normal((n, d))
    C = x[rng.choice(n, k, replace=False)] + 0.05 * rng.standard_normal((k, d))
    prev = orc.predict_labels(x, C + 0.3 * rng.standard_normal(C.shape))
    out = rng.random(n) < frac_out
    # previous labels outside [0, k), including markers' own range (-2,
    # INT32_MIN): they contribute nothing and the rows are listed as moved
    u = rng.random(int(out.sum()))
    prev[out] = np.where(u < 0.25, -1, np.where(u < 0.5, k, np.where(
        u < 0.75, -2, np.iinfo(np.int32).min)))
    dev = torch.device("cuda", 0)
    dd = load_data(x, subset_size=n)._device_data()
    ws = _device.Workspace(k, d, n, dev)
    lab = torch.from_numpy(prev.astype(np.int32)).to(dev)
    img = _device.sorted_image(dd, lab, k, ws)
    assert img[1] == _lib.IMAGE_SORTED
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    Ct = torch.from_numpy(C).to(dev)
    _device.prepare(Ct, ws, acc)
    _device.assign_delta(dd, Ct, ws, lab, acc, _lib.MODE_AUTO, image=img)
    rl, rs, rc = orc.partial_sum(x, C)
    got = lab.cpu().numpy()
    assert np.array_equal(got, rl), (got != rl).sum()
    raw = img[0].cpu().numpy()
    nt, nks = (n + 31) // 32, (d + 15) // 16
    tb = nt * nks * 1024
    perm = raw[tb + nt * 128:tb + nt * 256].view(np.int32)[:n]
    plab = raw[tb + nt * 256:tb + nt * 384].view(np.int32)[:n]
    assert np.array_equal(plab, rl[perm])
    a = acc.cpu().numpy()
    ps = np.zeros((k, d))
    pc = np.zeros(k)
    ok = (prev >= 0) & (prev < k)
    np.add.at(ps, prev[ok], x[ok])
    np.add.at(pc, prev[ok], 1)
    assert np.array_equal(a[k * d:], rc - pc)
    err = np.max(np.abs(a[:k * d].reshape(k, d) - (rs - ps)) /
                 np.maximum(np.abs(rs), 1.0))
    assert err <= 1e-11


@pytest.mark.parametrize("d,ldx", [(60, 60), (64, 65), (64, 66)])
def test_fit_shapes_without_the_sorted_image(d, ldx):
    """Auto-mode fits whose samples the single-product screen cannot read as
    16-B pieces (d % 8 != 0, or rows 8 B apart): no sorted image is built,
    and the fit matches the oracle (it used to fail with DKM_E_ARG at the
    first iteration over the image)."""
    from dislib_amd.cluster.kmeans import KMeans, _Lloyd, _init_centers
    from dislib_amd.data import Dataset, Subset
    n, k = 20_000, 1000
    rng = np.random.default_rng(d + ldx)
    blobs = rng.uniform(-10, 10, (200, d))
    xw = np.zeros((n, ldx))
    xw[:, :d] = blobs[rng.integers(0, 200, n)] + rng.standard_normal((n, d))
    dev = torch.device("cuda", 0)
    Xw = torch.from_numpy(xw).to(dev)
    ds = Dataset(n_features=d)
    ds.append(Subset(Xw[:, :d]))
    st = _Lloyd(ds, _init_centers(d, False, k, 3), 0.0, True, "auto", dev)
    # (a strided view is copied to 16-B rows on upload: then the image is
    # legal; d % 8 != 0 never takes it)
    assert not (st.sorting and d % 8)
    for _ in range(4):
        st.step()
    x = xw[:, :d]
    C = _init_centers(d, False, k, 3)
    for _ in range(4):
        lab, s, c = orc.partial_sum(x, C)
        nz = c > 0
        C = C.copy()
        C[nz] = s[nz] / c[nz, None]
    got = st.labels[:n].cpu().numpy()
    assert np.array_equal(got, lab), (got != lab).sum()
    err = np.max(np.abs(st.C.cpu().numpy() - C) / np.maximum(np.abs(C), 1.0))
    assert err <= 1e-9


@pytest.mark.parametrize("shift,spread", [(0.0, 1.0), (50.0, 1.0),
                                          (-3.0, 0.01)])
def test_translated_single_product_screen_vs_oracle(shift, spread):
    """DKM_MODE_TRANSLATE: the centres-on-lanes single-product screen over
    -2 (c - m) (m = the centres' mean) with the bound's x.c term on
    max ||c - m||: labels equal the oracle's for crowded centres far from the
    origin (shift), tight crowds (spread) and the reference's U[0, 1) init,
    with the sums / counts of the same assignment."""
    from dislib_amd import _device, _lib
    from dislib_amd.data import load_data
    rng = np.random.default_rng(int(abs(shift) * 7 + spread * 100))
    n, d, k = 60000, 64, 1000
    blobs = rng.uniform(-10, 10, (50, d)) + shift
    x = blobs[rng.integers(0, 50, n)] + rng.standard_normal((n, d))
    C = shift + spread * rng.random((k, d))
    dev = torch.device("cuda", 0)
    dd = load_data(x, subset_size=n)._device_data()
    ws = _device.Workspace(k, d, n, dev)
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    Ct = torch.from_numpy(C).to(dev)
    lab = torch.full((n,), -1, dtype=torch.int32, device=dev)
    _device.prepare(Ct, ws, acc)
    mode = _lib.MODE_BF16 | _lib.MODE_NOHINT | _lib.MODE_TRANSLATE
    _device.partial_sum(dd, Ct, ws, lab, acc, mode)
    rl, rs, rc = orc.partial_sum(x, C)
    assert np.array_equal(lab.cpu().numpy(), rl)
    a = acc.cpu().numpy()
    assert np.array_equal(a[k * d:], rc.astype(np.float64))
    err = np.max(np.abs(a[:k * d].reshape(k, d) - rs) /
                 np.maximum(np.abs(rs), 1.0))
    assert err <= 1e-11


def test_translated_first_iteration_fit_matches(monkeypatch):
    """A label-sorted-image fit whose first assignment takes the translated
    single-product screen equals the bf16x3 first assignment: labels,
    centres and iteration count (400k x 64, k = 1000, device blobs)."""
    from dislib_amd import _device
    from dislib_amd.cluster.kmeans import _Lloyd, _init_centers
    from dislib_amd.data import Dataset, Subset
    import dislib_amd.cluster.kmeans as km_mod
    n, d, k = 400_000, 64, 1000
    dev = torch.device("cuda", 0)
    X = torch.empty((n, d), dtype=torch.float64, device=dev)
    _device.make_blobs(X, 0, k, seed=3, box=10.0, std=1.0)
    out = {}
    for on in (False, True):
        monkeypatch.setattr(km_mod, "TRANSLATE_FIRST", on)
        ds = Dataset(n_features=d)
        ds.append(Subset(X))
        st = _Lloyd(ds, _init_centers(d, False, k, 3), 0.0, True, "auto",
                    dev)
        for _ in range(4):
            st.step()
        out[on] = (st.labels[:n].cpu().numpy(), st.C.cpu().numpy())
    assert np.array_equal(out[True][0], out[False][0])
    err = np.max(np.abs(out[True][1] - out[False][1]) /
                 np.maximum(np.abs(out[False][1]), 1.0))
    assert err <= 1e-12
