"""CPU tests of the host-side mirror of the reference interface: Dataset /
Subset / load_data semantics (reference tests/test_data.py), KMeans
constructor (tests/test_kmeans.py:13-27), label materialisation rules, and
the loud failure of compute paths without a GPU."""
import numpy as np
import pytest
import scipy.sparse as sp
from sklearn.datasets import make_blobs

import dislib_amd
from dislib_amd.cluster import KMeans
from dislib_amd.data import Dataset, Subset, load_data
from dislib_amd.data.classes import _DeviceLabels


def test_init_params():
    km = KMeans(n_clusters=2, max_iter=1, tol=1e-4, arity=2, random_state=666)
    assert (km._n_clusters, km._max_iter, km._tol, km._random_state,
            km._arity) == (2, 1, 1e-4, 666, 2)
    assert km.centers is None and km.n_iter == 0
    d = KMeans()
    assert (d._n_clusters, d._max_iter, d._tol, d._arity, d._verbose) == \
        (8, 10, 1e-4, 50, False)
    with pytest.raises(ValueError):
        KMeans(mode="bogus")


def test_load_data_with_labels():
    x, y = make_blobs(n_samples=1500, random_state=0)
    data = load_data(x=x, y=y, subset_size=100)
    assert len(data) == 15
    rx = np.concatenate([s.samples for s in data])
    ry = np.concatenate([s.labels for s in data])
    assert (rx == x).all() and (ry == y).all()


def test_load_data_without_labels_dense_and_sparse():
    x = np.random.random((100, 2))
    ds = load_data(x=x, subset_size=10)
    assert np.array_equal(ds.samples, x) and len(ds) == 10 and not ds.sparse
    xs = sp.csr_matrix(x)
    ds = load_data(x=xs, subset_size=10)
    assert np.array_equal(ds.samples.toarray(), x) and ds.sparse
    assert ds.labels is None


@pytest.mark.parametrize("size,sizes", [(30, [30, 30, 30, 10]),
                                        (25, [25] * 4), (100, [100]),
                                        (1, [1] * 100)])
def test_subsets_sizes(size, sizes):
    data = np.random.random((100, 1))
    assert load_data(data, subset_size=size).subsets_sizes() == sizes
    assert load_data(sp.csr_matrix(data), subset_size=size).subsets_sizes() \
        == sizes


def test_subset_copies_samples_and_set_label():
    a = np.random.random((25, 8))
    s = Subset(samples=a)
    a[0, 0] = 99.0
    assert s.samples[0, 0] != 99.0
    s.set_label(15, 3)
    assert s.labels[15] == 3 and s.labels.dtype == object
    assert s.labels[0] is None


def test_subset_concatenate_and_getitem():
    s1 = Subset(np.zeros((13, 2)), labels=np.zeros(13))
    s1.concatenate(Subset(np.zeros((11, 2)), labels=np.zeros(11)))
    assert s1.samples.shape[0] == 24 and s1.labels.shape[0] == 24
    s = Subset(samples=np.array([range(10), range(10, 20)]),
               labels=np.array([3, 4]))
    it = s[1]
    assert (it.samples == np.arange(10, 20)).all() and it.labels == 4


class _FakeTensor:
    """Stands in for a device int32 tensor (``.cpu().numpy()``)."""

    def __init__(self, a):
        self.a = np.asarray(a, dtype=np.int32)

    def cpu(self):
        return self

    def numpy(self):
        return self.a


def test_device_labels_materialise_like_set_label():
    x = np.arange(12, dtype=float).reshape(6, 2)
    ds = load_data(x, subset_size=4)
    ds._attach_device_labels(_FakeTensor([1, 0, 2, 1, 0, 0]))
    lab = ds.labels
    # reference: object array of np.int64 (set_label on a None label array)
    assert lab.dtype == object and isinstance(lab[0], np.int64)
    assert list(lab) == [1, 0, 2, 1, 0, 0]
    assert ds.labels_int32().dtype == np.int32


def test_device_labels_overwrite_existing_keep_dtype():
    x = np.arange(12, dtype=float).reshape(6, 2)
    ds = load_data(x, subset_size=3, y=np.full(6, 7.5))
    before = [s._labels for s in ds]
    ds._attach_device_labels(_FakeTensor([2, 2, 1, 0, 1, 2]))
    lab = ds.labels
    assert lab.dtype == np.float64 and list(lab) == [2, 2, 1, 0, 1, 2]
    # written in place into the Subsets' existing arrays
    assert all(s.labels is b for s, b in zip(ds, before))


def test_device_labels_src_is_shared_and_fetched_once():
    calls = []

    class T(_FakeTensor):
        def cpu(self):
            calls.append(1)
            return self

    src = _DeviceLabels(T([0, 1, 2]))
    assert list(src.host()) == [0, 1, 2] and list(src.host()) == [0, 1, 2]
    assert len(calls) == 1


def test_install_as_dislib_aliases_modules():
    import sys
    saved = {k: sys.modules.get(k) for k in ("dislib", "dislib.cluster",
                                             "dislib.data")}
    try:
        dislib_amd.install_as_dislib()
        from dislib.cluster import KMeans as K2
        from dislib.data import load_data as ld2
        assert K2 is KMeans and ld2 is load_data
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def test_shard_range_partitions_subsets():
    from dislib_amd import shard_range
    for n in (1, 7, 10, 100, 1000):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_shard_dataset_views():
    from dislib_amd import shard_dataset
    ds = load_data(np.random.random((100, 3)), subset_size=10)
    parts = [shard_dataset(ds, r, 3) for r in range(3)]
    assert [len(p) for p in parts] == [3, 3, 4]
    assert parts[1][0] is ds[3]


def test_compute_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    ds = load_data(np.random.random((10, 2)), subset_size=5)
    with pytest.raises(RuntimeError, match="GPU"):
        KMeans(n_clusters=2, random_state=0).fit(ds)


def test_randomstate_instance_rejected():
    ds = load_data(np.random.random((10, 2)), subset_size=5)
    with pytest.raises(TypeError):
        KMeans(n_clusters=2, random_state=np.random.RandomState(0)).fit(ds)


def test_device_must_be_a_gpu():
    """KMeans(device=...) names the GPU that runs the kernels; anything
    that is not a ROCm device is rejected before any launch."""
    pytest.importorskip("torch")
    from dislib_amd import _device
    with pytest.raises(ValueError, match="ROCm GPU"):
        _device.resolve("cpu")


def test_sparse_epsilon_query_host_checks():
    """The sparse epsilon query (dbscan classes.py:130) rejects dense
    Subsets before any device call, and concatenates CSR Subsets into one
    matrix with sorted column indices (the order scipy's products follow)."""
    import scipy.sparse as sp
    from dislib_amd.cluster.dbscan import _concat_csr, compute_neighbours
    from dislib_amd.data import load_data
    with pytest.raises(ValueError):
        compute_neighbours(1.0, 2, True, 0, 5,
                           *list(load_data(np.zeros((10, 3)), subset_size=5)))
    rng = np.random.default_rng(3)
    m = sp.random(50, 20, density=0.3, format="csr", random_state=rng)
    ip, ix, dv = m.indptr, m.indices.copy(), m.data.copy()
    for i in range(50):          # reverse the entries of every row
        ix[ip[i]:ip[i + 1]] = ix[ip[i]:ip[i + 1]][::-1].copy()
        dv[ip[i]:ip[i + 1]] = dv[ip[i]:ip[i + 1]][::-1].copy()
    u = sp.csr_matrix((dv, ix, ip), shape=m.shape)
    c = _concat_csr(list(load_data(u, subset_size=15)))
    assert c.has_sorted_indices
    assert (c != m).nnz == 0


def test_sparse_epsilon_query_refuses_duplicates_and_nonfinite():
    """a non-canonical CSR row with a duplicate column would get
    other products than scipy's csr_matmat (every stored pair): refused
    loudly; equal columns in DIFFERENT rows are fine.  NaN / inf raise like
    sklearn's pairwise_distances input check (dbscan classes.py:130)."""
    from dislib_amd.cluster.dbscan import _concat_csr
    from dislib_amd.data import load_data
    dup = sp.csr_matrix((np.array([1., 2, 3, 4]), np.array([1, 1, 0, 2]),
                         np.array([0, 2, 2, 4])), shape=(3, 3))
    with pytest.raises(ValueError, match="duplicate"):
        _concat_csr(list(load_data(dup, subset_size=3)))
    ok = sp.csr_matrix((np.array([1., 2, 3, 4]), np.array([1, 2, 2, 3]),
                        np.array([0, 2, 2, 4])), shape=(3, 4))
    assert _concat_csr(list(load_data(ok, subset_size=3))).nnz == 4
    for bad, msg in ((np.nan, "NaN"), (np.inf, "infinity")):
        b = ok.copy()
        b.data[1] = bad
        with pytest.raises(ValueError, match=msg):
            _concat_csr(list(load_data(b, subset_size=3)))


def test_sparse_kmeans_nonfinite_raises_before_the_device():
    """The sparse k-means path raises sklearn's ValueError on NaN / inf
    samples (base.py:169 -> pairwise_distances' check_array)."""
    from dislib_amd._device import assert_all_finite
    assert_all_finite(np.array([0.0, 1.0]))
    with pytest.raises(ValueError, match="Input contains NaN"):
        assert_all_finite(np.array([0.0, np.nan, np.inf]))
    with pytest.raises(ValueError, match="infinity"):
        assert_all_finite(np.array([-np.inf]))
