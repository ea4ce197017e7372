"""CPU: the f4 oracle (oracle/neighbors_oracle.py) against the golden vectors
the reference itself wrote (tests/golden/gen_golden_neighbors.py):
NearestNeighbors.kneighbors (neighbors/base.py:40-87) and the DBSCAN epsilon
query _compute_neighbours (cluster/dbscan/classes.py:124-141)."""
import os

import numpy as np
import pytest

from oracle import neighbors_oracle as orc

G = np.load(os.path.join(os.path.dirname(__file__), "golden",
                         "neighbors_ref.npz"))
KNN = sorted({k.split("__")[0] for k in G.files if k.startswith("kn_")})
DB = sorted({k.split("__")[0] for k in G.files if k.startswith("db_")})


def _blocks(x, sub):
    return [x[i:i + sub] for i in range(0, len(x), sub)]


def knn_case(name):
    sub, kn = (int(v) for v in G[name + "__meta"])
    return (G[name + "__xf"], G[name + "__xq"], sub, kn,
            G[name + "__dist"], G[name + "__ind"])


def kd_tree_regime(xf, sub, kn):
    return xf.shape[1] <= 15 and kn < sub // 2


@pytest.mark.parametrize("name", KNN)
def test_oracle_kneighbors_is_the_reference(name):
    xf, xq, sub, kn, dist, ind = knn_case(name)
    d, i = orc.kneighbors(_blocks(xf, sub), _blocks(xq, sub), kn)
    assert np.array_equal(i, ind)
    assert np.array_equal(d, dist)


@pytest.mark.parametrize("name", KNN)
def test_sequential_restatement(name):
    """The GPU contract (one brute-force pass, sequential squared sums,
    ascending (r, index)) against the reference: bit-exact in sklearn's
    kd_tree regime, within the GEMM expansion's rounding otherwise."""
    xf, xq, sub, kn, dist, ind = knn_case(name)
    d, i = orc.kneighbors_exact(xf, xq, kn)
    assert np.array_equal(i, ind), name
    if kd_tree_regime(xf, sub, kn):
        assert np.array_equal(d, dist), name
    else:
        # |x|^2 - 2 x.y + |y|^2 in fp64: error ~ eps (|x|^2 + |y|^2) on the
        # squared distance (sqrt magnifies it near 0: compare squares)
        scale2 = (xf ** 2).sum(1).max() + (xq ** 2).sum(1).max()
        assert np.max(np.abs(d ** 2 - dist ** 2)) <= 1e-13 * scale2, name


@pytest.mark.parametrize("name", DB)
def test_oracle_epsilon_query_is_the_reference(name):
    x = G[name + "__x"]
    sub, eps, ms, b, e = G[name + "__meta"]
    nl, cp = orc.compute_neighbours(eps, ms, int(b), int(e), x)
    off = G[name + "__offsets"]
    ref = G[name + "__neigh"]
    assert len(nl) == len(off) - 1
    for r, v in enumerate(nl):
        assert np.array_equal(v, ref[off[r]:off[r + 1]]), (name, r)
    assert np.array_equal(np.array(cp), G[name + "__core"])


GS = np.load(os.path.join(os.path.dirname(__file__), "golden",
                          "neighbors_sparse_ref.npz"))
DBS = sorted({k.split("__")[0] for k in GS.files if k.startswith("dbs_")})
KNS = sorted({k.split("__")[0] for k in GS.files if k.startswith("kns_")})


def sparse_case(name):
    """(indptr, indices, data, shape, meta, offsets, neigh, core) of a
    sparse epsilon-query golden (classes.py:130, sparse=True)."""
    return tuple(GS[name + "__" + f] for f in (
        "indptr", "indices", "data", "shape", "meta", "offsets", "neigh",
        "core"))


@pytest.mark.parametrize("name", DBS)
def test_oracle_sparse_epsilon_query_is_the_reference(name):
    ip, ix, dv, shape, meta, off, ref, core = sparse_case(name)
    sub, eps, ms, b, e = meta
    nl, cp = orc.compute_neighbours_csr(eps, ms, int(b), int(e), ip, ix, dv,
                                        f32=dv.dtype == np.float32)
    assert len(nl) == len(off) - 1
    for r, v in enumerate(nl):
        assert_same_up_to_ties(v, ref[off[r]:off[r + 1]], ip, ix, dv,
                               int(b) + r, (name, r))
    assert np.array_equal(np.array(cp), core)


def assert_same_up_to_ties(v, w, ip, ix, dv, q, what):
    """Identical lists, except that runs of exactly equal distances may be
    permuted: the reference's np.argsort (introsort) does not order equal
    keys by index (dbs_empty: empty rows, all at distance 0)."""
    if np.array_equal(v, w):
        return
    r = orc.csr_sq_distances(ip, ix, dv, q)
    dist = np.sqrt(r.astype(np.float32) if dv.dtype == np.float32 else r)
    assert np.array_equal(np.sort(v), np.sort(w)), what
    assert np.array_equal(dist[v], dist[w]), what


def test_oracle_sparse_distances_are_sklearns_expansion():
    """The restated distances against sklearn's own pairwise_distances on
    the golden inputs (bit for bit, the sqrt of the restated squares)."""
    sk = pytest.importorskip("sklearn.metrics")
    sp = pytest.importorskip("scipy.sparse")
    for name in DBS:
        ip, ix, dv, shape, *_ = sparse_case(name)
        m = sp.csr_matrix((dv, ix, ip), shape=tuple(shape))
        for q in (0, 7, int(shape[0]) - 1):
            want = sk.pairwise_distances(m[q], m).ravel()
            r = orc.csr_sq_distances(ip, ix, dv, q)
            # float32 Subsets: sklearn's upcast path (fp64 squares cast to
            # float32, float32 sqrt)
            got = np.sqrt(r.astype(np.float32) if dv.dtype == np.float32
                          else r)
            assert got.dtype == want.dtype, name
            assert np.array_equal(got, want), (name, q)


def sparse_knn_case(name):
    """(fit csr, query csr, d, subset, n_neighbors, dist, ind) of a sparse
    kneighbors golden; csr = (indptr, indices, data)."""
    f = tuple(GS[name + "__f" + a] for a in ("indptr", "indices", "data"))
    q = tuple(GS[name + "__q" + a] for a in ("indptr", "indices", "data"))
    sub, kn, d = (int(v) for v in GS[name + "__meta"])
    return f, q, d, sub, kn, GS[name + "__dist"], GS[name + "__ind"]


def assert_knn_same_up_to_ties(dist, ind, rdist, rind, what):
    """Distances bit-exact; indices equal except among exactly equal
    distances, which the reference's argpartition / quicksort argsort order
    arbitrarily (the whole tie group at the list's end may also be a
    different subset of it)."""
    assert np.array_equal(dist, rdist), what
    if np.array_equal(ind, rind):
        return
    for r in np.nonzero((ind != rind).any(1))[0]:
        for v in np.unique(dist[r]):
            at = dist[r] == v
            if v == dist[r, -1]:
                continue        # the last tie group may be another subset
            assert np.array_equal(np.sort(ind[r, at]), np.sort(rind[r, at])), \
                (what, r)


@pytest.mark.parametrize("name", KNS)
def test_oracle_sparse_kneighbors_is_the_reference(name):
    f, q, d, sub, kn, dist, ind = sparse_knn_case(name)
    got_d, got_i = orc.kneighbors_csr(f, q, kn,
                                      f32=f[2].dtype == np.float32)
    assert_knn_same_up_to_ties(got_d, got_i, dist, ind, name)
    # the indices name rows at the reported distances
    fm = sp_matrix(f, d)
    qm = sp_matrix(q, d)
    for r in (0, qm.shape[0] // 2, qm.shape[0] - 1):
        rr = orc.csr_sq_distances_to(qm[r].indices,
                                     qm[r].data.astype(np.float64), *f)
        want = np.sqrt(rr.astype(np.float32) if f[2].dtype == np.float32
                       else rr)
        assert np.array_equal(want[ind[r]], dist[r]), (name, r)
    del fm


def sp_matrix(csr, d):
    sp = pytest.importorskip("scipy.sparse")
    ip, ix, dv = csr
    return sp.csr_matrix((dv, ix, ip), shape=(ip.size - 1, d))
