"""Label parity at the bench sizes (BASELINE.json configs[1..4] per GPU).

The other GPU tests pin every kernel branch on inputs the oracle finishes in
seconds.  These run the product fit loop (``_Lloyd``: image build, bf16x3
iteration 0, the delta path, the sums from labels) at the FULL per-GPU
sizes ``bench.py`` times -- where X is 25.6 GB (C2), 64 GB plus a 16.5 GB
bf16 image (C3) or 82 GB (C4), so every 32-bit byte offset of the data,
the image and the label scratch has wrapped many times -- and check:

* the labels of ~40k rows sampled over the whole range, plus windows around
  every 2^20-th row (2^18-th at d = 1024: each crosses a 2 GiB multiple of
  the X, image or label offsets) and the first and last tiles, against the
  oracle's restatement of the reference assignment (dislib
  cluster/kmeans/base.py:171-173, np.linalg.norm + np.argmin) under the
  centres that assignment used -- bit-exact;
* every label in [0, k), and the fit state's counts equal to a bincount of
  all n labels (so they sum to n);
* ``predict`` (the top-3 pass, no hint) under the final centres on the
  same rows.

Three Lloyd iterations per config, tol = 0.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import kmeans_oracle as orc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _rows_to_check(n, n_random, window_every, seed):
    rng = np.random.default_rng(seed)
    idx = [rng.choice(n, min(n, n_random), replace=False),
           np.arange(min(n, 96)), np.arange(max(0, n - 96), n)]
    for w in range(window_every, n, window_every):
        idx.append(np.arange(max(0, w - 16), min(n, w + 16)))
    return np.unique(np.concatenate(idx))


def _oracle_labels(rows, C, sparse=False):
    """orc.predict_labels over row chunks on THREADS threads (numpy releases
    the GIL in the ufunc loops)."""
    if sparse:
        return orc.predict_labels(rows, C, sparse=True)
    parts = np.array_split(np.arange(rows.shape[0]), THREADS)
    with ThreadPoolExecutor(THREADS) as ex:
        out = list(ex.map(lambda ix: orc.predict_labels(rows[ix], C), parts))
    return np.concatenate(out)


def _fit_and_check(ds, C0, k, d, rows_of, idx, sparse=False, iters=3):
    from dislib_amd import _device, _lib
    from dislib_amd.cluster.kmeans import _Lloyd
    dev = torch.device("cuda", 0)
    st = _Lloyd(ds, C0, 0.0, True, "auto", dev)
    n = st.dd.n
    for _ in range(iters - 1):
        st.step()
    C_used = st.C.cpu().numpy()          # the centres iteration `iters` uses
    st.step()
    lab = st.labels[:n]
    assert int(lab.min()) >= 0 and int(lab.max()) < k
    cnt = torch.bincount(lab.long(), minlength=k).cpu().numpy()
    assert int(cnt.sum()) == n
    state_counts = st.state[k * d:].cpu().numpy()
    assert np.array_equal(state_counts, cnt.astype(np.float64))
    it = torch.from_numpy(idx).to(dev)
    got = lab[it].cpu().numpy()
    rows = rows_of(idx)
    want = _oracle_labels(rows, C_used if not sparse else
                          _csr(C_used), sparse)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, ("fit labels differ at rows", idx[bad[:10]],
                           got[bad[:10]], want[bad[:10]])
    # predict under the final centres (no hint: the top-3 / full screens)
    C_fin = st.C.cpu().numpy()
    plab = torch.empty(n, dtype=torch.int32, device=dev)
    _device.prepare(st.C, st.ws, None, csr=sparse)   # the final centres
    _device.predict(st.dd, st.C, st.ws, plab, _lib.MODE_AUTO)
    pgot = plab[it].cpu().numpy()
    pwant = _oracle_labels(rows, C_fin if not sparse else _csr(C_fin), sparse)
    bad = np.nonzero(pgot != pwant)[0]
    assert bad.size == 0, ("predict labels differ at rows", idx[bad[:10]])
    del st, plab, lab
    torch.cuda.empty_cache()


def _csr(C):
    import scipy.sparse as sp
    return sp.csr_matrix(C)


def _dense_config(n, d, k, f32=False, n_random=40_000, window=1 << 20):
    from dislib_amd import _device
    from dislib_amd.cluster.kmeans import _init_centers
    from dislib_amd.data import Dataset, Subset
    dev = torch.device("cuda", 0)
    free = torch.cuda.mem_get_info(dev)[0]
    need = n * d * 8 * (1.6 if not f32 else 1.0) + n * 64
    if need > free:
        pytest.skip("needs %.0f GB of HBM, %.0f free" % (need / 1e9, free / 1e9))
    X = torch.empty((n, d), dtype=torch.float64, device=dev)
    _device.make_blobs(X, 0, k, seed=0, box=10.0, std=1.0)   # bench's data
    if f32:
        X = X.to(torch.float32)
        torch.cuda.empty_cache()
    ds = Dataset(n_features=d)
    for i in range(0, n, 1_000_000):
        ds.append(Subset(X[i:i + 1_000_000]))
    idx = _rows_to_check(n, n_random, window, n + d + k)
    C0 = _init_centers(d, False, k, 0)

    def rows_of(ix):
        return X[torch.from_numpy(ix).to(dev)].cpu().numpy()
    try:
        _fit_and_check(ds, C0, k, d, rows_of, idx)
    finally:
        del ds, X
        torch.cuda.empty_cache()


def test_c2_full_size_labels():
    """configs[1]: 100M x 32 fp64, k = 100 (the headline; split image)."""
    _dense_config(100_000_000, 32, 100)


def test_c3_full_size_labels():
    """configs[2]'s per-GPU shard: 125M x 64 fp64, k = 1000 (64 GB of X,
    16.5 GB single image, the b2 screen)."""
    _dense_config(125_000_000, 64, 1000)


def test_c4_full_size_labels():
    """configs[3]: 10M x 1024 fp64, k = 4096 (82 GB; the GEMM screen)."""
    _dense_config(10_000_000, 1024, 4096, n_random=1500, window=1 << 18)


def test_c4_fp32_full_size_labels():
    """configs[3], fp32 samples (fp64 distances, fp32 sums)."""
    _dense_config(10_000_000, 1024, 4096, f32=True, n_random=1000,
                  window=1 << 19)


def test_c5_full_size_labels():
    """configs[4]: CSR 10M x 10k, 10 stored entries per row, k = 256."""
    import bench
    from dislib_amd.cluster.kmeans import _init_centers
    from dislib_amd.data import Dataset, Subset
    n, d, k = 10_000_000, 10_000, 256
    X = bench.csr_rows(0, n, d, 10, seed=1)
    ds = Dataset(n_features=d, sparse=True)
    for i in range(0, n, 1_000_000):
        ds.append(Subset(X[i:i + 1_000_000]))
    idx = _rows_to_check(n, 20_000, 1 << 20, 5)
    C0 = _init_centers(d, True, k, 0).toarray()
    _fit_and_check(ds, C0, k, d, lambda ix: X[ix], idx, sparse=True)
