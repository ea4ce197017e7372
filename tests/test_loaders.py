"""Dataset file loaders vs the oracle's
restatement of ``dislib/data/base.py:42-238`` (sklearn load_svmlight_file /
np.genfromtxt per chunk of ``subset_size`` raw lines).  Host code only: the
parsers in ``libdkm.so`` (``dkm_io.cpp``) run without a GPU, so these are CPU
tests.  Bar: bit-exact samples (CSR arrays included) and labels."""
import gzip
import os

import numpy as np
import pytest
import scipy.sparse as sp

from dislib_amd.data import (load_libsvm_file, load_libsvm_files,
                             load_txt_file, load_txt_files)
from dislib_amd.data.base import parse_libsvm, parse_txt
from oracle import loaders_oracle as orc

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _same(a, b):
    """bit-exact equality of two arrays (NaN == NaN, -0.0 != 0.0)."""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype.kind == "f":
        return np.array_equal(a.view(np.uint64 if a.itemsize == 8 else
                                     np.uint32),
                              b.astype(a.dtype).view(
                                  np.uint64 if a.itemsize == 8 else
                                  np.uint32))
    return np.array_equal(a, b)


def _check(ds, ref, sparse):
    assert len(ds) == len(ref)
    for s, (x, y) in zip(ds, ref):
        if sparse:
            assert sp.issparse(s.samples) and sp.issparse(x)
            assert s.samples.shape == x.shape
            assert _same(s.samples.indptr, x.indptr)
            assert _same(s.samples.indices, x.indices)
            assert _same(s.samples.data, x.data)
        else:
            assert not sp.issparse(s.samples)
            assert _same(s.samples, x)
        if y is None:
            assert s.labels is None
        else:
            assert _same(s.labels, y)


def _libsvm_text(rng, n, d, one_based=True, extras=True, crlf=False,
                 density=0.05):
    out = []
    base = 1 if one_based else 0
    for i in range(n):
        if extras and i % 17 == 5:
            out.append("# a comment line")
        if extras and i % 23 == 7:
            out.append("   ")
        cols = np.flatnonzero(rng.random(d) < density)
        vals = rng.standard_normal(cols.size) * 10.0 ** rng.integers(
            -5, 5, cols.size)
        lab = ["%d" % rng.integers(-1, 3), "%.17g" % rng.standard_normal(),
               "+1"][i % 3]
        toks = [lab]
        if extras and i % 11 == 3:
            toks.append("qid:%d" % i)
        fmt = ["%.17g", "%r", "%.6e", "%g"]
        toks += ["%d:%s" % (c + base, fmt[j % 4] % v if fmt[j % 4] != "%r"
                            else repr(float(v)))
                 for j, (c, v) in enumerate(zip(cols, vals))]
        line = "\t".join(toks) if i % 5 == 0 else " ".join(toks)
        if extras and i % 13 == 2:
            line += "  # trailing comment 3:4"
        out.append(line)
    nl = "\r\n" if crlf else "\n"
    return nl.join(out) + nl


@pytest.mark.parametrize("subset_size", [1, 7, 50, 1000])
@pytest.mark.parametrize("store_sparse", [True, False])
def test_libsvm_file_matches_reference(tmp_path, subset_size, store_sparse):
    rng = np.random.default_rng(subset_size)
    p = tmp_path / "a.svm"
    p.write_text(_libsvm_text(rng, 300, 120))
    ds = load_libsvm_file(str(p), subset_size, 130, store_sparse)
    ref = orc.load_file(str(p), subset_size, "libsvm", 130,
                        store_sparse=store_sparse)
    _check(ds, ref, store_sparse)
    assert ds.sparse == store_sparse
    assert ds.n_features == 130


def test_libsvm_zero_based_auto_shift_is_per_chunk(tmp_path):
    # zero-based file: chunks that happen to have no index 0 are shifted by
    # sklearn's "auto" heuristic in the reference -- reproduced per chunk
    rng = np.random.default_rng(3)
    p = tmp_path / "z.svm"
    p.write_text(_libsvm_text(rng, 200, 40, one_based=False, density=0.1))
    for ss in (3, 10, 200):
        ds = load_libsvm_file(str(p), ss, 40)
        _check(ds, orc.load_file(str(p), ss, "libsvm", 40,
                                 store_sparse=True), True)


def test_libsvm_crlf_and_lone_cr(tmp_path):
    rng = np.random.default_rng(4)
    txt = _libsvm_text(rng, 120, 30, crlf=True)
    p = tmp_path / "crlf.svm"
    p.write_bytes(txt.encode())
    _check(load_libsvm_file(str(p), 9, 31),
           orc.load_file(str(p), 9, "libsvm", 31, store_sparse=True), True)
    q = tmp_path / "cr.svm"
    q.write_bytes(txt.replace("\r\n", "\r").encode())
    _check(load_libsvm_file(str(q), 9, 31),
           orc.load_file(str(q), 9, "libsvm", 31, store_sparse=True), True)


def test_libsvm_no_trailing_newline_and_empty(tmp_path):
    p = tmp_path / "t.svm"
    p.write_text("1 1:2 3:4\n-1 2:0.5")
    _check(load_libsvm_file(str(p), 1, 5),
           orc.load_file(str(p), 1, "libsvm", 5, store_sparse=True), True)
    e = tmp_path / "e.svm"
    e.write_text("")
    assert len(load_libsvm_file(str(e), 4, 5)) == 0
    c = tmp_path / "c.svm"            # a chunk of comment lines only
    c.write_text("# x\n# y\n1 1:1\n")
    _check(load_libsvm_file(str(c), 2, 5),
           orc.load_file(str(c), 2, "libsvm", 5, store_sparse=True), True)


@pytest.mark.parametrize("body", [
    "1 3:1 2:1\n",          # unsorted
    "1 2:1 2:3\n",          # duplicate
    "1 -1:2\n",             # negative index
    "1 2:abc\n",            # bad value
    "x 2:1\n",              # bad target
    "1 2\n",                # no colon
    "1 1:1 9:1\n",          # n_features too small (8)
])
def test_libsvm_errors_like_reference(tmp_path, body):
    p = tmp_path / "bad.svm"
    p.write_text("1 1:1\n" + body)
    with pytest.raises(ValueError):
        orc.load_file(str(p), 10, "libsvm", 8, store_sparse=True)
    with pytest.raises(ValueError):
        load_libsvm_file(str(p), 10, 8)


def test_libsvm_multithreaded_parse_equals_single(tmp_path):
    rng = np.random.default_rng(5)
    txt = _libsvm_text(rng, 6000, 400, density=0.08)
    assert len(txt) > (1 << 20)          # takes the threaded path
    buf = txt.encode()
    one = parse_libsvm(buf, nthreads=1)
    many = parse_libsvm(buf, nthreads=7)
    assert one[0] == many[0]
    for a, b in zip(one[1:], many[1:]):
        assert _same(a, b)
    p = tmp_path / "big.svm"
    p.write_bytes(buf)
    _check(load_libsvm_file(str(p), 1000, 401),
           orc.load_file(str(p), 1000, "libsvm", 401, store_sparse=True),
           True)


def test_libsvm_files_one_subset_per_file(tmp_path):
    rng = np.random.default_rng(6)
    d = tmp_path / "dir"
    d.mkdir()
    for i in range(4):
        (d / ("f%d" % i)).write_text(_libsvm_text(rng, 30 + 10 * i, 50))
    for sparse in (True, False):
        _check(load_libsvm_files(str(d), 60, sparse),
               orc.load_files(str(d), "libsvm", 60, store_sparse=sparse),
               sparse)


def _csv_text(rng, n, d, delim=",", extras=True):
    out = []
    for i in range(n):
        if extras and i % 19 == 4:
            out.append("# comment")
        if extras and i % 29 == 9:
            out.append("")
        v = rng.standard_normal(d) * 10.0 ** rng.integers(-3, 4, d)
        f = ["%.17g" % x for x in v]
        if extras and i % 7 == 1:
            f[i % d] = ""                 # missing -> nan
        if extras and i % 31 == 2:
            f[(i + 1) % d] = "abc"        # unconvertible -> nan
        if extras and i % 9 == 0:
            f[0] = " %s " % f[0]
        line = delim.join(f) if delim is not None else "  ".join(f)
        if extras and i % 15 == 6:
            line += "#tail"
        out.append(line)
    return "\n".join(out) + "\n"


@pytest.mark.parametrize("label_col", [None, "first", "last"])
@pytest.mark.parametrize("subset_size", [1, 13, 500])
def test_txt_file_matches_reference(tmp_path, label_col, subset_size):
    rng = np.random.default_rng(subset_size + 1)
    p = tmp_path / "a.csv"
    p.write_text(_csv_text(rng, 200, 9))
    if subset_size == 1 and label_col is not None:
        # genfromtxt squeezes 1-row chunks: the reference's samples[:, 1:]
        # raises there, and so does the loader
        with pytest.raises(IndexError):
            orc.load_file(str(p), 1, "txt", 9, delimiter=",",
                          label_col=label_col)
        with pytest.raises(IndexError):
            load_txt_file(str(p), 1, 9, label_col=label_col)
        return
    ds = load_txt_file(str(p), subset_size, 9, label_col=label_col)
    ref = orc.load_file(str(p), subset_size, "txt", 9, delimiter=",",
                        label_col=label_col)
    _check(ds, ref, False)


def test_txt_whitespace_and_other_delimiters(tmp_path):
    rng = np.random.default_rng(8)
    p = tmp_path / "w.txt"
    p.write_text(_csv_text(rng, 150, 6, delim=None, extras=False))
    _check(load_txt_file(str(p), 40, 6, delimiter=None),
           orc.load_file(str(p), 40, "txt", 6, delimiter=None), False)
    q = tmp_path / "s.txt"
    q.write_text(_csv_text(rng, 150, 6, delim=";"))
    _check(load_txt_file(str(q), 40, 6, delimiter=";"),
           orc.load_file(str(q), 40, "txt", 6, delimiter=";"), False)


def test_txt_column_mismatch_raises(tmp_path):
    p = tmp_path / "m.csv"
    p.write_text("1,2,3\n4,5\n")
    with pytest.raises(ValueError):
        orc.load_file(str(p), 10, "txt", 3, delimiter=",")
    with pytest.raises(ValueError):
        load_txt_file(str(p), 10, 3)


@pytest.mark.parametrize("ending", ["\n", "\r\n", "\r"])
def test_txt_width_changes_between_chunks(tmp_path, ending):
    """genfromtxt runs per chunk in the reference: a file whose width
    changes at a chunk boundary loads (one width per Subset); a change
    inside a chunk raises ValueError in both."""
    rng = np.random.default_rng(12)
    a = _csv_text(rng, 30, 3, extras=False).splitlines()
    b = _csv_text(rng, 20, 5, extras=False).splitlines()
    p = tmp_path / "r.csv"
    p.write_bytes((ending.join(a + b) + ending).encode())
    ds = load_txt_file(str(p), 10, 5)
    ref = orc.load_file(str(p), 10, "txt", 5, delimiter=",")
    _check(ds, ref, False)
    assert [s.samples.shape[1] for s in ds] == [3, 3, 3, 5, 5]
    with pytest.raises(ValueError):
        orc.load_file(str(p), 25, "txt", 5, delimiter=",")
    with pytest.raises(ValueError):
        load_txt_file(str(p), 25, 5)


def test_txt_files(tmp_path):
    rng = np.random.default_rng(9)
    d = tmp_path / "csvdir"
    d.mkdir()
    for i in range(3):
        (d / str(i)).write_text(_csv_text(rng, 50 + i, 5))
    _check(load_txt_files(str(d), 5, label_col="last"),
           orc.load_files(str(d), "txt", 5, delimiter=",", label_col="last"),
           False)


def test_reference_fixture_other4(tmp_path):
    """``tests/files/other/4`` of the reference (a real data file; the
    csv/libsvm fixtures are Git-LFS pointers), committed gzipped."""
    raw = gzip.open(os.path.join(GOLDEN, "other4.txt.gz")).read()
    p = tmp_path / "4"
    p.write_bytes(raw)
    ds = load_txt_file(str(p), 300, 0, delimiter=" ")
    ref = orc.load_file(str(p), 300, "txt", 0, delimiter=" ")
    _check(ds, ref, False)
    # the reference test's own expectation (test_data.py:129-144 style)
    full = np.loadtxt(str(p), delimiter=" ")
    assert _same(np.concatenate([s.samples for s in ds]), full)
    # multithreaded parse of the 1.1 MB file equals the single-thread one
    one, many = parse_txt(raw, " ", nthreads=1), parse_txt(raw, " ", 8)
    assert one[0] == many[0] and _same(one[1], many[1])


def test_libsvm_loader_feeds_kmeans_host_image(tmp_path):
    """The loader's concatenated CSR (the one-shot HBM upload image) equals
    the vstack of its Subsets."""
    rng = np.random.default_rng(10)
    p = tmp_path / "k.svm"
    p.write_text(_libsvm_text(rng, 257, 64))
    ds = load_libsvm_file(str(p), 32, 64)
    img = ds._host_image
    st = sp.vstack([s.samples for s in ds], format="csr")
    assert img.shape == st.shape
    assert _same(img.indptr, st.indptr) and _same(img.indices, st.indices)
    assert _same(img.data, st.data)
    ds.append(ds[0])
    assert ds._host_image is None      # invalidated by a mutation


def test_parser_abi_argument_checks():
    """C-ABI error behaviour of the loader entry points (host-only)."""
    import ctypes
    from dislib_amd import _lib
    so = _lib.load()
    cnt = np.zeros(4, np.int64)
    p = ctypes.c_void_p(cnt.ctypes.data)
    assert so.dkm_libsvm_count(None, 5, 1, p) == 10001        # NULL buffer
    assert b"bad arguments" in so.dkm_last_error()
    assert so.dkm_txt_count(None, 0, 300, 1, p) == 10001      # bad delimiter
    assert so.dkm_libsvm_count(None, 0, 1, p) == 0            # empty input
    assert list(cnt[:3]) == [0, 0, 0]
    buf = np.frombuffer(b"1 1:2 1:3\n", np.uint8)
    ptr = np.zeros(2, np.int64)
    ind, dat = np.empty(2, np.int32), np.empty(2)
    y, rl = np.empty(1), np.empty(1, np.int64)
    a = [ctypes.c_void_p(x.ctypes.data) for x in (buf, ptr, ind, dat, y, rl)]
    rc = so.dkm_libsvm_parse(a[0], buf.size, 1, a[1], a[2], a[3], a[4], a[5])
    assert rc == 10004 and b"sorted and unique" in so.dkm_last_error()
    assert b"(line 1)" in so.dkm_last_error()
