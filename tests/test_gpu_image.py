"""The d <= 32 split sample image (DKM_IMAGE_SPLIT) and k_screen_w32's
image path (dislib_amd/csrc/dkm_b2.hip k_x_image_split, dkm_dense.hip
k_screen_w32<IMG>): the image against the fp64 -> fp32 -> bf16 hi / lo
roundings, and delta launches through it against the oracle's restatement
of the reference assignment (cluster/kmeans/base.py:171-173) -- labels
bit-exact, the delta of the sums -- with and without the image."""
import numpy as np
import pytest

from oracle import kmeans_oracle as orc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _bf16_rne(f):
    u = f.view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


@pytest.mark.parametrize("n,d", [(1000, 32), (77, 20), (33, 16), (64, 5)])
def test_split_image_layout(n, d):
    from dislib_amd import _device, _lib
    so = _lib.lib()
    rng = np.random.default_rng(n + d)
    x = rng.standard_normal((n, d)) * 10.0 ** rng.integers(-3, 4, (n, 1))
    X = torch.from_numpy(x).cuda()
    nb = so.dkm_x_image_bytes(n, d, _lib.IMAGE_SPLIT)
    nt = (n + 31) // 32
    assert nb == nt * 4096 + nt * 128
    img = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    _lib.check(so.dkm_x_image_f64(_device.ptr(X), n, d, d, _lib.IMAGE_SPLIT,
                                  _device.ptr(img), nb, _device.stream_ptr()),
               "image")
    raw = img.cpu().numpy()
    tiles = raw[:nt * 4096].view(np.uint16).reshape(nt, 2, 2, 64, 8)
    xx = raw[nt * 4096:].view(np.float32)
    f = np.zeros((nt * 32, 32), np.float32)
    f[:n, :d] = x.astype(np.float32)
    hi = _bf16_rne(f)
    hif = (hi.astype(np.uint32) << 16).view(np.float32)
    lo = _bf16_rne((f - hif).astype(np.float32))
    for part, want in ((0, hi), (1, lo)):
        # tile, row, half h, slice s, j: features 16 h + 8 s + j
        w = want.reshape(nt, 32, 2, 2, 8).transpose(0, 3, 2, 1, 4)
        w = w.reshape(nt, 2, 64, 8)
        assert np.array_equal(tiles[:, part], w), part
    ref = (f.astype(np.float64) ** 2).sum(1)
    assert np.all(np.abs(xx - ref) <= 2.0 ** -23 * ref)
    assert np.all(xx[n:] == 0)


@pytest.mark.parametrize("image", [True, False])
@pytest.mark.parametrize("d,k", [(32, 100), (20, 300), (16, 10), (8, 64)])
def test_w32_delta_through_the_image(monkeypatch, image, d, k):
    """C2's AUTO pick is asserted in test_c2_shape_reads_the_split_image."""
    from dislib_amd import _device, _lib
    from dislib_amd.data import load_data
    monkeypatch.setattr(_device, "X_IMAGE", image)
    rng = np.random.default_rng(d * k)
    n = 40011
    blobs = rng.uniform(-10, 10, (k, d))
    x = blobs[rng.integers(0, k, n)] + rng.standard_normal((n, d))
    C = blobs + 0.3 * rng.standard_normal((k, d))
    prev = orc.predict_labels(x, C + 0.2 * rng.standard_normal(C.shape))
    prev[rng.random(n) < 0.01] = -1
    dev = torch.device("cuda", 0)
    dd = load_data(x, subset_size=n)._device_data()
    ws = _device.Workspace(k, d, n, dev)
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    Ct = torch.from_numpy(C).to(dev)
    lab = torch.from_numpy(prev.astype(np.int32)).to(dev)
    _device.prepare(Ct, ws, acc)
    # the bf16x3 screen (AUTO's pick wherever the sums fit LDS, e.g. C2)
    mode = _lib.MODE_BF16X3
    assert _lib.lib().dkm_x_image_kind(k, d, mode) == _lib.IMAGE_SPLIT
    _device.assign_delta(dd, Ct, ws, lab, acc, mode)
    assert (_lib.IMAGE_SPLIT in dd.images) == image
    rl, rs, rc = orc.partial_sum(x, C)
    got = lab.cpu().numpy()
    assert np.array_equal(got, rl), (got != rl).sum()
    a = acc.cpu().numpy()
    ps = np.zeros((k, d))
    pc = np.zeros(k)
    ok = prev >= 0
    np.add.at(ps, prev[ok], x[ok])
    np.add.at(pc, prev[ok], 1)
    assert np.array_equal(a[k * d:], rc - pc)
    err = np.max(np.abs(a[:k * d].reshape(k, d) - (rs - ps)) /
                 np.maximum(np.abs(rs), 1.0))
    assert err <= 1e-11


def test_image_kind_per_config():
    """C2 reads the split image, C3 the single one, C4 the GEMM tiles
    (round 4); the exact mode takes none."""
    from dislib_amd import _lib
    so = _lib.lib()
    assert so.dkm_x_image_kind(100, 32, _lib.MODE_AUTO) == _lib.IMAGE_SPLIT
    assert so.dkm_x_image_kind(1000, 64, _lib.MODE_AUTO) == _lib.IMAGE_SINGLE
    assert so.dkm_x_image_kind(4096, 1024, _lib.MODE_AUTO) == _lib.IMAGE_GEMM
    assert so.dkm_x_image_kind(4096, 1024, _lib.MODE_EXACT) == _lib.IMAGE_NONE


@pytest.mark.parametrize("n,d,k,f32", [(40011, 32, 100, False),
                                       (9000, 20, 64, False),
                                       (5000, 16, 10, True),
                                       (777, 8, 300, False)])
def test_full_sums_pass_builds_the_split_image(n, d, k, f32):
    """DKM_IMAGE_BUILD: the d <= 32 screen's full-sums pass (a fit's
    iteration 0) writes the split image while it converts X: the hi / lo
    tiles equal dkm_x_image_*'s bit for bit, |x|^2 is the screen's own fp32
    sum (within 2^-22 of the exact one), and the call's labels and sums are
    the oracle's; a delta launch through the fused image then matches the
    oracle too."""
    from dislib_amd import _device, _lib
    from dislib_amd.data import load_data
    so = _lib.lib()
    rng = np.random.default_rng(n + d + k)
    blobs = rng.uniform(-10, 10, (k, d))
    x = blobs[rng.integers(0, k, n)] + rng.standard_normal((n, d))
    if f32:
        x = x.astype(np.float32)
    C = blobs + 0.3 * rng.standard_normal((k, d))
    dev = torch.device("cuda", 0)
    dd = load_data(x, subset_size=n)._device_data()
    ws = _device.Workspace(k, d, n, dev)
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    Ct = torch.from_numpy(C).to(dev)
    lab = torch.full((n,), -1, dtype=torch.int32, device=dev)
    mode = _lib.MODE_BF16X3
    _device.prepare(Ct, ws, acc)
    img, kind = dd.screen_image(k, mode)
    assert kind == _lib.IMAGE_SPLIT | _lib.IMAGE_BUILD
    img.fill_(0xAB)                       # garbage: the call must write all
    _device.partial_sum(dd, Ct, ws, lab, acc, mode)
    assert not dd._unbuilt
    rl, rs, rc = orc.partial_sum(x, C)
    assert np.array_equal(lab.cpu().numpy(), rl)
    a = acc.cpu().numpy()
    assert np.array_equal(a[k * d:], rc.astype(np.float64))
    err = np.max(np.abs(a[:k * d].reshape(k, d) - rs) /
                 np.maximum(np.abs(rs), 1.0))
    assert err <= (1e-4 if f32 else 1e-11)
    # against the separate builder
    nb = so.dkm_x_image_bytes(n, d, _lib.IMAGE_SPLIT)
    ref = torch.zeros(nb, dtype=torch.uint8, device=dev)
    fn = so.dkm_x_image_f32 if f32 else so.dkm_x_image_f64
    _lib.check(fn(_device.ptr(dd.X), n, d, d, _lib.IMAGE_SPLIT,
                  _device.ptr(ref), nb, _device.stream_ptr()), "image")
    nt = (n + 31) // 32
    got, want = img.cpu().numpy(), ref.cpu().numpy()
    assert np.array_equal(got[:nt * 4096], want[:nt * 4096])
    gx = got[nt * 4096:nt * 4096 + 4 * n].view(np.float32)
    wx = want[nt * 4096:nt * 4096 + 4 * n].view(np.float32)
    assert np.all(np.abs(gx - wx) <= 2.0 ** -22 * wx)
    # a delta launch through the fused image
    C2 = C + 0.2 * rng.standard_normal(C.shape)
    Ct2 = torch.from_numpy(C2).to(dev)
    acc.zero_()
    _device.prepare(Ct2, ws, acc)
    _device.assign_delta(dd, Ct2, ws, lab, acc, mode)
    rl2, _, _ = orc.partial_sum(x, C2)
    assert np.array_equal(lab.cpu().numpy(), rl2)


@pytest.mark.parametrize("n,d,k,f32", [(150001, 160, 300, False),
                                       (70000, 200, 129, True)])
def test_bf16x3_gemm_pass_builds_the_gemm_image(n, d, k, f32):
    """DKM_IMAGE_BUILD on the GEMM shapes (round 6): the bf16x3 iteration's
    chunk splits also write the single-product image (hi tiles + norms) of
    every chunk, byte for byte what dkm_x_image_* builds in its own pass;
    the call's labels and sums are the oracle's, and a single-product delta
    launch through the fused image matches the oracle too."""
    from dislib_amd import _device, _lib
    from dislib_amd.data import load_data
    so = _lib.lib()
    rng = np.random.default_rng(n + d + k)
    blobs = rng.uniform(-10, 10, (k, d))
    x = blobs[rng.integers(0, k, n)] + rng.standard_normal((n, d))
    if f32:
        x = x.astype(np.float32)
    C = blobs + 0.3 * rng.standard_normal((k, d))
    dev = torch.device("cuda", 0)
    dd = load_data(x, subset_size=n)._device_data()
    ws = _device.Workspace(k, d, n, dev)
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    Ct = torch.from_numpy(C).to(dev)
    lab = torch.full((n,), -1, dtype=torch.int32, device=dev)
    _device.prepare(Ct, ws, acc)
    img, kind = dd.screen_image(k, _lib.MODE_AUTO)
    assert kind == _lib.IMAGE_GEMM | _lib.IMAGE_BUILD
    img.fill_(0xAB)
    _device.partial_sum(dd, Ct, ws, lab, acc, _lib.MODE_BF16X3,
                        image=(img, kind))
    assert not dd._unbuilt
    rl, rs, rc = orc.partial_sum(x, C)
    assert np.array_equal(lab.cpu().numpy(), rl)
    a = acc.cpu().numpy()
    assert np.array_equal(a[k * d:], rc.astype(np.float64))
    err = np.max(np.abs(a[:k * d].reshape(k, d) - rs) /
                 np.maximum(np.abs(rs), 1.0))
    assert err <= (1e-4 if f32 else 1e-11)
    nb = so.dkm_x_image_bytes(n, d, _lib.IMAGE_GEMM)
    ref = torch.full((img.numel(),), 0xAB, dtype=torch.uint8, device=dev)
    fn = so.dkm_x_image_f32 if f32 else so.dkm_x_image_f64
    _lib.check(fn(_device.ptr(dd.X), n, d, d, _lib.IMAGE_GEMM,
                  _device.ptr(ref), nb, _device.stream_ptr()), "image")
    assert torch.equal(img, ref)
    # a single-product delta launch through the fused image
    C2 = C + 0.2 * rng.standard_normal(C.shape)
    Ct2 = torch.from_numpy(C2).to(dev)
    acc.zero_()
    _device.prepare(Ct2, ws, acc)
    _device.assign_delta(dd, Ct2, ws, lab, acc, _lib.MODE_AUTO)
    rl2, _, _ = orc.partial_sum(x, C2)
    assert np.array_equal(lab.cpu().numpy(), rl2)
