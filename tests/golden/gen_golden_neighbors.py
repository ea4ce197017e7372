"""Golden vectors for the distance-primitive reuse rows,
produced by the REFERENCE itself:

* ``dislib.neighbors.NearestNeighbors.kneighbors``
  (``/root/reference/dislib/neighbors/base.py:40-87``: sklearn
  ``NearestNeighbors`` per (query Subset, fit Subset) pair, merged by
  ``_merge_queries``);
* the DBSCAN epsilon query ``_compute_neighbours``
  (``/root/reference/dislib/cluster/dbscan/classes.py:124-141``, distances by
  ``_vec_matrix_euclid`` ``:153-154``).

Run in the development container only:
``python tests/golden/gen_golden_neighbors.py`` -- like ``gen_golden.py`` it
imports the reference under the sequential PyCOMPSs stub.  Nothing of the
reference is copied: inputs are seeded synthetic matrices (stored, they are
small), outputs are what the reference returned.  Writes
``neighbors_ref.npz`` and ``neighbors_sparse_ref.npz`` (the epsilon query
and kneighbors on sparse Subsets).
"""
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

# (name, n_fit, n_query or None (query = fit), d, subset, n_neighbors, kind)
KNN_CASES = [
    ("kn_doc", 100, None, 5, 25, 10, "uniform"),     # the docstring example
    ("kn_blobs", 300, None, 3, 50, 5, "blobs"),      # kd_tree regime
    ("kn_d20", 200, None, 20, 40, 7, "uniform"),     # d > 15: brute regime
    ("kn_half", 120, None, 4, 30, 16, "uniform"),    # k >= n_fit // 2: brute
    ("kn_other", 200, 100, 6, 50, 4, "blobs"),       # queries != fit data
    ("kn_one", 90, None, 2, 30, 1, "uniform"),       # single neighbour
    ("kn_40", 400, None, 3, 100, 40, "blobs"),       # > 32: two passes
    ("kn_70", 300, None, 4, 100, 70, "uniform"),     # > 64, brute regime
]
# (name, n, d, subset, epsilon, min_samples, begin, end)
DB_CASES = [
    ("db_blobs", 400, 2, 100, 0.5, 5, 0, 400),
    ("db_d10", 300, 10, 75, 1.6, 8, 50, 250),
    ("db_d130", 150, 130, 50, 16.3, 3, 10, 140),
    ("db_none", 120, 3, 40, 1e-3, 2, 0, 120),        # only the point itself
]
# sparse Subsets (the pairwise_distances branch, classes.py:130):
# (name, n, d, subset, density, epsilon, min_samples, begin, end)
DB_SPARSE_CASES = [
    ("dbs_small", 200, 50, 50, 0.1, 0.8, 3, 0, 200),
    ("dbs_wide", 300, 2000, 100, 0.005, 2.3, 2, 20, 280),   # ~10 nnz / row
    ("dbs_empty", 150, 30, 50, 0.03, 0.3, 2, 0, 150),       # empty rows
    ("dbs_blobs", 240, 20, 60, None, 5.5, 4, 30, 210),      # thresholded blobs
    ("dbs_f32", 250, 40, 50, 0.15, 1.1, 3, 0, 250),         # float32 Subsets
]
# sparse kneighbors (sklearn brute force on CSR):
# (name, n_fit, n_query or None (query = fit), d, subset, density, n_neighbors)
KNN_SPARSE_CASES = [
    ("kns_small", 200, None, 50, 50, 0.1, 5),
    ("kns_wide", 300, None, 2000, 100, 0.005, 8),   # mostly disjoint rows
    ("kns_empty", 150, None, 30, 50, 0.03, 4),      # empty rows: ties at 0
    ("kns_other", 240, 120, 20, 60, None, 6),       # queries != fit data
    ("kns_40", 400, None, 30, 100, 0.2, 40),        # > 32: two passes
    ("kns_f32", 300, None, 40, 100, 0.15, 6),       # float32 Subsets
]


def _data(rng, n, d, kind):
    import numpy as np
    if kind == "blobs":
        c = rng.uniform(-5, 5, (4, d))
        return c[rng.integers(0, 4, n)] + rng.standard_normal((n, d))
    return rng.random((n, d)) * np.linspace(1.0, 3.0, d)


def generate():
    import numpy as np
    from dislib.data import load_data
    from dislib.neighbors import NearestNeighbors
    from dislib.cluster.dbscan.classes import _compute_neighbours

    out = {}
    for i, (name, nf, nq, d, sub, kn, kind) in enumerate(KNN_CASES):
        rng = np.random.default_rng(100 + i)
        xf = _data(rng, nf, d, kind)
        xq = xf if nq is None else _data(rng, nq, d, kind)
        knn = NearestNeighbors(n_neighbors=kn)
        knn.fit(load_data(xf, subset_size=sub))
        dist, ind = knn.kneighbors(load_data(xq, subset_size=sub))
        out[name + "__xf"] = xf
        out[name + "__xq"] = xq
        out[name + "__meta"] = np.array([sub, kn])
        out[name + "__dist"] = np.asarray(dist)
        out[name + "__ind"] = np.asarray(ind)
        print("kneighbors", name, np.asarray(dist).shape)
    for i, (name, n, d, sub, eps, ms, b, e) in enumerate(DB_CASES):
        rng = np.random.default_rng(200 + i)
        x = _data(rng, n, d, "blobs" if i % 2 == 0 else "uniform")
        ds = load_data(x, subset_size=sub)
        nl, cp = _compute_neighbours(eps, ms, False, b, e, *list(ds))
        lens = np.array([len(v) for v in nl], dtype=np.int64)
        out[name + "__x"] = x
        out[name + "__meta"] = np.array([sub, eps, ms, b, e], dtype=np.float64)
        out[name + "__offsets"] = np.concatenate([[0], np.cumsum(lens)])
        out[name + "__neigh"] = (np.concatenate(nl).astype(np.int64)
                                 if len(nl) else np.zeros(0, np.int64))
        out[name + "__core"] = np.asarray(cp, dtype=bool)
        print("dbscan", name, int(lens.sum()), "neighbours")
    np.savez_compressed(os.path.join(HERE, "neighbors_ref.npz"), **out)
    print("wrote neighbors_ref.npz")
    import scipy.sparse as sp
    out = {}
    for i, (name, n, d, sub, dens, eps, ms, b, e) in enumerate(
            DB_SPARSE_CASES):
        rng = np.random.default_rng(300 + i)
        if dens is None:
            x = _data(rng, n, d, "blobs")
            x[np.abs(x) < 1.0] = 0.0
            x = sp.csr_matrix(x)
        else:
            x = sp.random(n, d, density=dens, format="csr", random_state=rng,
                          data_rvs=lambda k: rng.uniform(-1, 1, k))
        if name.endswith("_f32"):
            x = x.astype(np.float32)
        x.sort_indices()
        ds = load_data(x, subset_size=sub)
        nl, cp = _compute_neighbours(eps, ms, True, b, e, *list(ds))
        lens = np.array([len(v) for v in nl], dtype=np.int64)
        out[name + "__indptr"] = x.indptr.astype(np.int64)
        out[name + "__indices"] = x.indices.astype(np.int32)
        out[name + "__data"] = x.data
        out[name + "__shape"] = np.array(x.shape, dtype=np.int64)
        out[name + "__meta"] = np.array([sub, eps, ms, b, e], dtype=np.float64)
        out[name + "__offsets"] = np.concatenate([[0], np.cumsum(lens)])
        out[name + "__neigh"] = (np.concatenate(nl).astype(np.int64)
                                 if len(nl) else np.zeros(0, np.int64))
        out[name + "__core"] = np.asarray(cp, dtype=bool)
        print("dbscan sparse", name, x.nnz, "nnz", int(lens.sum()),
              "neighbours")
    for i, (name, nf, nq, d, sub, dens, kn) in enumerate(KNN_SPARSE_CASES):
        rng = np.random.default_rng(400 + i)

        def _csr(n):
            if dens is None:
                x = _data(rng, n, d, "blobs")
                x[np.abs(x) < 1.0] = 0.0
                x = sp.csr_matrix(x)
            else:
                x = sp.random(n, d, density=dens, format="csr",
                              random_state=rng,
                              data_rvs=lambda k: rng.uniform(-1, 1, k))
            if name.endswith("_f32"):
                x = x.astype(np.float32)
            x.sort_indices()
            return x
        xf = _csr(nf)
        xq = xf if nq is None else _csr(nq)
        knn = NearestNeighbors(n_neighbors=kn)
        fds = load_data(xf, subset_size=sub)
        knn.fit(fds)
        dist, ind = knn.kneighbors(fds if nq is None else
                                   load_data(xq, subset_size=sub))
        for tag, x in (("f", xf), ("q", xq)):
            out["%s__%sindptr" % (name, tag)] = x.indptr.astype(np.int64)
            out["%s__%sindices" % (name, tag)] = x.indices.astype(np.int32)
            out["%s__%sdata" % (name, tag)] = x.data
        out[name + "__meta"] = np.array([sub, kn, d], dtype=np.int64)
        out[name + "__dist"] = np.asarray(dist)
        out[name + "__ind"] = np.asarray(ind)
        print("kneighbors sparse", name, np.asarray(dist).shape)
    np.savez_compressed(os.path.join(HERE, "neighbors_sparse_ref.npz"), **out)
    print("wrote neighbors_sparse_ref.npz")


def main():
    try:
        import dislib  # noqa: F401
        import pycompss  # noqa: F401
        ok = True
    except ImportError:
        ok = False
    if ok:
        generate()
        return
    if not os.path.isdir(REF):
        print("reference not present; golden vectors are committed -- skip")
        return
    sys.path.insert(0, HERE)
    from gen_golden import SHIM
    shim = tempfile.mkdtemp(prefix="dkm_shim_")
    for rel, body in SHIM.items():
        p = os.path.join(shim, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(body)
    env = dict(os.environ, PYTHONPATH=shim + ":" + REF,
               PYTHONDONTWRITEBYTECODE="1")
    sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)],
                             env=env, cwd=REF))


if __name__ == "__main__":
    main()
