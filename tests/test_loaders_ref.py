"""Dataset loaders against the REFERENCE loaders' own outputs
(tests/golden/loaders_ref.npz, written by gen_golden_loaders.py through
``dislib.data.load_libsvm_file(s)`` / ``load_txt_file(s)``): the same input
bytes through ``dislib_amd.data`` must give bit-identical Subsets -- CSR
arrays or dense samples, labels and their dtype.  Host code only (CPU)."""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from dislib_amd.data import (load_libsvm_file, load_libsvm_files,
                             load_txt_file, load_txt_files)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "loaders_ref.npz")
# (name, loader, kwargs) -- the cases of gen_golden_loaders.cases()
CASES = [
    ("svm_one", load_libsvm_file, dict(subset_size=50, n_features=40)),
    ("svm_zero_crlf", load_libsvm_file, dict(subset_size=33, n_features=25)),
    ("svm_dense", load_libsvm_file, dict(subset_size=40, n_features=12,
                                         store_sparse=False)),
    ("txt_last", load_txt_file, dict(subset_size=40, n_features=6,
                                     delimiter=",", label_col="last")),
    ("txt_first_ws", load_txt_file, dict(subset_size=25, n_features=4,
                                         delimiter=None, label_col="first")),
    ("txt_nolabel_onerow", load_txt_file, dict(subset_size=20, n_features=4,
                                               delimiter=",")),
    ("svm_dir", load_libsvm_files, dict(n_features=20)),
    ("txt_dir", load_txt_files, dict(n_features=5, delimiter=",",
                                     label_col="last")),
]


def _bits(a):
    a = np.asarray(a)
    if a.dtype.kind == "f":
        return a.dtype.str, a.shape, a.view(np.uint8).tobytes()
    return a.dtype.str, a.shape, a.tobytes()


def _check_subset(s, g, prefix):
    x = s.samples
    if prefix + "indptr" in g:
        assert sp.issparse(x)
        x = x.tocsr()
        assert tuple(x.shape) == tuple(g[prefix + "shape"])
        assert np.array_equal(x.indptr, g[prefix + "indptr"])
        assert np.array_equal(x.indices, g[prefix + "indices"])
        assert _bits(x.data) == _bits(g[prefix + "data"])
    else:
        assert not sp.issparse(x)
        assert _bits(x) == _bits(g[prefix + "dense"])
    if bool(g[prefix + "has_labels"]):
        assert _bits(s.labels) == _bits(g[prefix + "labels"])
    else:
        assert s.labels is None


@pytest.mark.parametrize("name,loader,kw", CASES, ids=[c[0] for c in CASES])
def test_loader_matches_reference_output(tmp_path, name, loader, kw):
    g = np.load(GOLDEN)
    if loader in (load_libsvm_files, load_txt_files):
        p = tmp_path / name
        p.mkdir()
        pre = "%s/in/" % name
        for key in g.files:
            if key.startswith(pre):
                (p / key[len(pre):]).write_bytes(g[key].tobytes())
        ds = loader(str(p), **kw)
        names = os.listdir(str(p))        # both walk os.listdir order
        assert len(ds) == int(g["%s/n_subsets" % name]) == len(names)
        for fn, s in zip(names, ds):
            _check_subset(s, g, "%s/out/%s/" % (name, fn))
    else:
        p = tmp_path / name
        p.write_bytes(g["%s/in" % name].tobytes())
        ds = loader(str(p), **kw)
        assert len(ds) == int(g["%s/n_subsets" % name])
        for i, s in enumerate(ds):
            _check_subset(s, g, "%s/out/%d/" % (name, i))
