"""Loader -> HIP path end to end (SURVEY.md section 8 row f1 feeding a7):
the reference's F7 sparse fixture written as a LibSVM file, read back by
``load_libsvm_file`` (C++ parser, one-shot CSR upload) and clustered on the
GPU must reproduce the reference's golden labels / centres."""
import numpy as np
import pytest
import scipy.sparse as sp

from tests.conftest import load_golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _write_libsvm(path, x, y):
    # repr() is the shortest round-trip spelling: the file holds x exactly
    with open(path, "w") as f:
        for i in range(x.shape[0]):
            a, b = x.indptr[i], x.indptr[i + 1]
            toks = ["%d:%r" % (j + 1, float(v))
                    for j, v in zip(x.indices[a:b], x.data[a:b])]
            f.write(" ".join([repr(float(y[i]))] + toks) + "\n")


@pytest.mark.parametrize("store_sparse", [True, False])
def test_libsvm_file_to_gpu_kmeans_matches_golden(tmp_path, store_sparse):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dislib_amd.cluster import KMeans
    from dislib_amd.data import load_libsvm_file
    g = load_golden("f07_sparse")
    xs = sp.csr_matrix((g["data"], g["indices"], g["indptr"]),
                       shape=tuple(g["shape"]))
    p = tmp_path / "f07.svm"
    _write_libsvm(str(p), xs, np.arange(xs.shape[0], dtype=np.float64))
    ds = load_libsvm_file(str(p), 200, xs.shape[1], store_sparse)
    km = KMeans(n_clusters=8, random_state=170)
    km.fit_predict(ds)
    lab = np.asarray(ds.labels.astype(np.int64))
    if store_sparse:
        assert km.n_iter == g["sparse_n_iter"]
        assert np.array_equal(lab, g["sparse_labels"])
        ref = g["sparse_centers"]
        got = km.centers.toarray()
    else:
        assert np.array_equal(lab, g["dense_labels"])
        ref, got = g["dense_centers"], km.centers
    err = np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1.0))
    assert err <= 1e-9
