"""Generate golden vectors by running the REFERENCE dislib (v0.2.0) k-means.

Run in the development container only:  ``python tests/golden/gen_golden.py``

The reference lives read-only at /root/reference and needs PyCOMPSs, which is
not installed; like the reference's own ``run_coverage.sh:3-4`` we run it in
PyCOMPSs *sequential* semantics through a tiny stub package (``@task`` is the
identity, ``compss_wait_on`` returns its argument), plus two scikit-learn API
drift shims (``sklearn.utils.fixes.logsumexp``; keyword-only ``n_features`` of
``load_svmlight_file``).  No reference source is copied: this script imports
it and records inputs/outputs as ``.npz`` data.

Inputs that are cheap to regenerate (sklearn ``make_blobs`` with a fixed
seed) are not stored; the fixture stores their sha256 instead so the tests
can assert they rebuilt the identical matrix.
"""
import hashlib
import io
import os
import subprocess
import sys
import tempfile
import contextlib

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

SHIM = {
    "pycompss/__init__.py": "",
    "pycompss/api/__init__.py": "",
    "pycompss/api/api.py": (
        "def compss_wait_on(*objs, **kw):\n"
        "    return objs[0] if len(objs) == 1 else list(objs)\n"
        "def barrier(*a, **k):\n    pass\n"
        "def compss_delete_object(*a, **k):\n    pass\n"),
    "pycompss/api/task.py": (
        "def task(*dargs, **dkw):\n"
        "    def deco(f):\n        return f\n"
        "    return deco\n"),
    "pycompss/api/parameter.py": (
        "IN='IN'; OUT='OUT'; INOUT='INOUT'; FILE_IN='FILE_IN'\n"
        "FILE_OUT='FILE_OUT'; FILE_INOUT='FILE_INOUT'\n"),
    "sitecustomize.py": (
        "import sklearn.utils.fixes as _f\nimport scipy.special as _s\n"
        "if not hasattr(_f, 'logsumexp'):\n    _f.logsumexp = _s.logsumexp\n"
        "import sklearn.datasets as _d\n_orig = _d.load_svmlight_file\n"
        "def _wrap(f, n_features=None, *a, **k):\n"
        "    return _orig(f, n_features=n_features, *a, **k)\n"
        "_d.load_svmlight_file = _wrap\n"),
}


def sha(a):
    import numpy as np
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _record_trace(KMeans):
    """Wrap ``_recompute_centers`` to record the centres after each update."""
    orig = KMeans._recompute_centers

    def rec(self, partials):
        orig(self, partials)
        c = self.centers
        self._trace.append(c.toarray().copy() if hasattr(c, "toarray")
                           else c.copy())
    KMeans._recompute_centers = rec


def generate():
    import numpy as np
    import scipy.sparse as sp
    from sklearn.datasets import make_blobs
    from dislib.cluster import KMeans
    from dislib.data import Dataset, Subset, load_data

    _record_trace(KMeans)

    def km(**kw):
        m = KMeans(**kw)
        m._trace = []
        return m

    def labels_of(ds):
        lab = ds.labels
        return None if lab is None else np.asarray(lab.astype(np.int64))

    out = {}

    # F1/F2 -- tests/test_kmeans.py:29-63 (toy integer data)
    ds = Dataset(n_features=2)
    ds.append(Subset(np.array([[1, 2], [2, 1]])))
    ds.append(Subset(np.array([[-1, -2], [-2, -1]])))
    m = km(n_clusters=2, random_state=666)
    m.fit(ds)
    test_set = load_data(np.array([[1, 2], [2, 1], [-1, -2], [-2, -1],
                                   [10, 10], [-10, -10]]), subset_size=2)
    m.predict(test_set)
    out["f01_toy"] = dict(centers=m.centers, n_iter=m.n_iter,
                          trace=np.array(m._trace),
                          predict_labels=labels_of(test_set))

    # F3 -- tests/test_kmeans.py:65-83 (blobs filtered to 610 rows)
    x, y = make_blobs(n_samples=1500, random_state=170)
    xf = np.vstack((x[y == 0][:500], x[y == 1][:100], x[y == 2][:10]))
    ds = load_data(xf, subset_size=300)
    m = km(n_clusters=3, random_state=170)
    m.fit_predict(ds)
    out["f03_blobs610"] = dict(x=xf, centers=m.centers, n_iter=m.n_iter,
                               labels=labels_of(ds), trace=np.array(m._trace))

    # F4 -- config-1 mini (make_blobs 20000x50, 10 blobs, subset 2000)
    x, _ = make_blobs(n_samples=20000, n_features=50, centers=10,
                      random_state=0)
    ds = load_data(x, subset_size=2000)
    m = km(n_clusters=10, max_iter=5, tol=0, random_state=0)
    m.fit_predict(ds)
    out["f04_c1mini"] = dict(x_sha=sha(x), centers=m.centers, n_iter=m.n_iter,
                             labels=labels_of(ds), trace=np.array(m._trace))

    # F5 -- config-2 shape mini (k=100, d=32)
    x, _ = make_blobs(n_samples=20000, n_features=32, centers=100,
                      center_box=(-10, 10), random_state=1)
    ds = load_data(x, subset_size=5000)
    m = km(n_clusters=100, max_iter=3, tol=0, random_state=0)
    m.fit_predict(ds)
    out["f05_c2mini"] = dict(x_sha=sha(x), centers=m.centers, n_iter=m.n_iter,
                             labels=labels_of(ds), trace=np.array(m._trace))

    # F6 -- config-3 shape mini (k=1000, d=64)
    x, _ = make_blobs(n_samples=10000, n_features=64, centers=50,
                      center_box=(-10, 10), random_state=2)
    ds = load_data(x, subset_size=5000)
    m = km(n_clusters=1000, max_iter=2, tol=0, random_state=0)
    m.fit_predict(ds)
    out["f06_c3mini"] = dict(x_sha=sha(x), centers=m.centers, n_iter=m.n_iter,
                             labels=labels_of(ds), trace=np.array(m._trace))

    # F7 -- sparse CSR vs dense (synthetic replacement for the LFS fixture
    # tests/files/libsvm/2 used by tests/test_kmeans.py:85-101)
    xs = sp.random(2000, 780, density=0.01, format="csr", random_state=170,
                   dtype=np.float64)
    dss = load_data(xs, subset_size=200)
    m = km(n_clusters=8, random_state=170)
    m.fit_predict(dss)
    sparse_centers = m.centers.toarray()
    sparse_trace = np.array(m._trace)
    sparse_labels = labels_of(dss)
    sparse_n_iter = m.n_iter
    pred_set = load_data(xs, subset_size=500)
    m.predict(pred_set)
    sparse_pred = labels_of(pred_set)
    dsd = load_data(xs.toarray(), subset_size=200)
    m2 = km(n_clusters=8, random_state=170)
    m2.fit_predict(dsd)
    out["f07_sparse"] = dict(
        indptr=xs.indptr, indices=xs.indices, data=xs.data,
        shape=np.array(xs.shape), sparse_centers=sparse_centers,
        sparse_trace=sparse_trace, sparse_labels=sparse_labels,
        sparse_n_iter=sparse_n_iter, sparse_predict=sparse_pred,
        dense_centers=m2.centers, dense_labels=labels_of(dsd),
        dense_n_iter=m2.n_iter, dense_trace=np.array(m2._trace))

    # F8 -- exact ties and sqrt ties (first index wins), predict only
    rng = np.random.RandomState(8)
    xs8, cs8 = [], []
    # exact ties: equal squared distances
    xs8.append([0.0, 0.0, 0.0])
    cs_exact = np.array([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0],
                         [5.0, 5.0, 5.0]])
    # sqrt ties: s_a > s_b but sqrt(s_a) == sqrt(s_b); put a first
    from oracle_path import pairwise_sum  # noqa: E402
    found = []
    while len(found) < 6:
        x0 = rng.uniform(-3, 3, 3)
        cb = rng.uniform(-3, 3, 3)
        for _ in range(200):
            ca = cb.copy()
            j = rng.randint(3)
            ca[j] = np.nextafter(ca[j], ca[j] + rng.choice([-1, 1]) * 10.0)
            sa = pairwise_sum((x0 - ca) ** 2)
            sb = pairwise_sum((x0 - cb) ** 2)
            if sa > sb and np.sqrt(sa) == np.sqrt(sb):
                found.append((x0, ca, cb))
                break
    sqrt_tie_x = np.array([f[0] for f in found])
    sqrt_tie_c = np.array([[f[1], f[2]] for f in found])
    tie_pred = []
    for x0, ca, cb in found:
        m = km(n_clusters=2)
        m.centers = np.array([ca, cb])
        t = load_data(x0[None, :], subset_size=1)
        m.predict(t)
        tie_pred.append(int(labels_of(t)[0]))
    m = km(n_clusters=4)
    m.centers = cs_exact
    t = load_data(np.array(xs8), subset_size=1)
    m.predict(t)
    exact_tie = labels_of(t)
    # near ties for the screening path: samples almost equidistant
    cen = rng.uniform(-10, 10, (16, 24))
    near = []
    for i in range(512):
        a, b = rng.randint(16), rng.randint(16)
        if a == b:
            b = (a + 1) % 16
        mid = 0.5 * (cen[a] + cen[b])
        u = cen[a] - cen[b]
        v = rng.standard_normal(24)
        v -= v.dot(u) / u.dot(u) * u
        xq = mid + 0.3 * v + (rng.uniform(-1, 1) * 10.0 ** -rng.randint(6, 16)) * u
        near.append(xq)
    near = np.array(near)
    m = km(n_clusters=16)
    m.centers = cen.copy()
    t = load_data(near, subset_size=100)
    m.predict(t)
    out["f08_ties"] = dict(exact_x=np.array(xs8), exact_c=cs_exact,
                           exact_labels=exact_tie, sqrt_x=sqrt_tie_x,
                           sqrt_c=sqrt_tie_c, sqrt_labels=np.array(tie_pred),
                           near_x=near, near_c=cen,
                           near_labels=labels_of(t))

    # F9 -- empty clusters keep their U[0,1) initial centre
    rng = np.random.RandomState(9)
    x9 = np.vstack([rng.normal(5, 0.1, (100, 2)), rng.normal(-5, 0.1, (100, 2))])
    ds = load_data(x9, subset_size=50)
    m = km(n_clusters=6, max_iter=4, random_state=9)
    m.fit_predict(ds)
    out["f09_empty"] = dict(x=x9, centers=m.centers, n_iter=m.n_iter,
                            labels=labels_of(ds), trace=np.array(m._trace))

    # F10 -- fp32 samples: fp64 distances, fp32 partial sums
    x, _ = make_blobs(n_samples=3000, n_features=8, centers=4, random_state=3)
    x32 = x.astype(np.float32)
    ds = load_data(x32, subset_size=500)
    m = km(n_clusters=4, max_iter=5, tol=0, random_state=3)
    m.fit_predict(ds)
    out["f10_fp32"] = dict(x=x32, centers=m.centers, n_iter=m.n_iter,
                           labels=labels_of(ds), trace=np.array(m._trace))

    # F11 -- max_iter=0 runs one iteration; tol boundary
    x, _ = make_blobs(n_samples=400, n_features=3, centers=3, random_state=11)
    ds = load_data(x, subset_size=100)
    m0 = km(n_clusters=3, max_iter=0, random_state=11)
    m0.fit(ds)
    mt = km(n_clusters=3, max_iter=50, tol=1e-1, random_state=11)
    buf = io.StringIO()
    mt._verbose = True
    with contextlib.redirect_stdout(buf):
        mt.fit(ds)
    out["f11_iters"] = dict(x=x, n_iter_max0=m0.n_iter, centers_max0=m0.centers,
                            n_iter_tol=mt.n_iter, centers_tol=mt.centers,
                            verbose=np.array(buf.getvalue()))

    # F12 -- fit_predict labels are the last assignment, not predict(final)
    x, _ = make_blobs(n_samples=1000, n_features=2, centers=5, random_state=7)
    ds = load_data(x, subset_size=250)
    m = km(n_clusters=5, max_iter=2, tol=0, random_state=7)
    m.fit_predict(ds)
    fp_labels = labels_of(ds)
    ds2 = load_data(x, subset_size=250)
    m.predict(ds2)
    out["f12_lastassign"] = dict(x=x, centers=m.centers, fit_predict=fp_labels,
                                 predict=labels_of(ds2))

    # F13 -- 120 Subsets: arity-50 and arity-2 merge-tree order
    x, _ = make_blobs(n_samples=6000, n_features=4, centers=6, random_state=13)
    res = {}
    for ar in (50, 2):
        ds = load_data(x, subset_size=50)
        m = km(n_clusters=6, max_iter=4, tol=0, arity=ar, random_state=13)
        m.fit_predict(ds)
        res["centers_a%d" % ar] = m.centers
        res["trace_a%d" % ar] = np.array(m._trace)
        res["labels_a%d" % ar] = labels_of(ds)
    out["f13_arity"] = dict(x=x, **res)

    # F14 -- preloaded float labels are overwritten in place, dtype kept
    x, yb = make_blobs(n_samples=300, n_features=2, centers=3, random_state=14)
    ds = load_data(x, subset_size=100, y=yb.astype(np.float64))
    m = km(n_clusters=3, random_state=14)
    m.fit_predict(ds)
    lab = ds.labels
    out["f14_prelabels"] = dict(x=x, y=yb.astype(np.float64),
                                labels=np.asarray(lab),
                                labels_dtype=np.array(str(lab.dtype)),
                                centers=m.centers)

    for name, d in out.items():
        arrs = {k: (np.asarray(v) if v is not None else np.array([]))
                for k, v in d.items()}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
        print("wrote", name)


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
    shim = tempfile.mkdtemp(prefix="dkm_shim_")
    for rel, body in SHIM.items():
        p = os.path.join(shim, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(body)
    # oracle_path: makes oracle.pairwise_sum importable for tie construction
    with open(os.path.join(shim, "oracle_path.py"), "w") as f:
        f.write("import sys\nsys.path.insert(0, %r)\n"
                "from oracle.kmeans_oracle import pairwise_sum\n"
                % os.path.dirname(os.path.dirname(HERE)))
    env = dict(os.environ, PYTHONPATH=shim + ":" + REF,
               PYTHONDONTWRITEBYTECODE="1")
    sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)],
                             env=env, cwd=REF))


if __name__ == "__main__":
    main()
