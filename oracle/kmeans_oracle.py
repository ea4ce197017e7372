"""CPU oracle for dislib's k-means Lloyd path -- TEST INFRASTRUCTURE ONLY.

This module is a numpy restatement of the reference algorithm in
``/root/reference/dislib/cluster/kmeans/base.py`` (dislib v0.2.0).  It is the
*checker*: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product path (``dislib_amd``) never
imports, calls or falls back to anything in ``oracle/``.

Parity pin: every function below is checked bit-for-bit against golden
vectors produced by the reference itself (``tests/golden/gen_golden.py``,
which imports ``/root/reference`` under a sequential PyCOMPSs shim) in
``tests/test_oracle_golden.py``.

Arithmetic facts the restatement relies on (all verified in this container,
numpy 2.2.6):

* ``np.linalg.norm(v - C, axis=1)`` (base.py:204-205) is
  ``sqrt(add.reduce((v - C)**2, axis=1))``; ``add.reduce`` over a contiguous
  row sums in numpy's *pairwise* order (8 accumulators for 8 <= n <= 128,
  recursive halving at multiples of 8 above 128, plain loop below 8) inside
  iterator buffers of 8192 elements that are added sequentially.  The same
  reduction over a 3-D ``(m, k, d)`` temporary gives identical bits, which is
  what :func:`dense_distances` uses.  :func:`pairwise_sum` states the order
  explicitly (it is the model the HIP kernels implement).
* ``np.argmin`` returns the first index of the minimum (base.py:173,200).
* ``partials[c][0] += sample`` (base.py:178) is a sequential per-element add
  in sample order; ``np.add.at`` performs exactly that chain.
* fp32 samples give fp64 distances (the centres are fp64) but fp32 partial
  sums; integer samples give integer (exact) partial sums.
"""
import numpy as np

PW_BLOCKSIZE = 128        # numpy loops_utils.h PW_BLOCKSIZE
NPY_BUFSIZE = 8192        # numpy default ufunc buffer size (elements)


# --------------------------------------------------------------------------
# Summation order model (numpy add.reduce, used by np.linalg.norm axis=1)
# --------------------------------------------------------------------------
def _pairwise_block(a, lo, n):
    """numpy ``@TYPE@_pairwise_sum`` over ``a[lo:lo+n]`` (python floats)."""
    if n < 8:
        res = -0.0
        for i in range(n):
            res = res + a[lo + i]
        return res
    if n <= PW_BLOCKSIZE:
        r = [a[lo + j] for j in range(8)]
        i = 8
        stop = n - (n % 8)
        while i < stop:
            for j in range(8):
                r[j] = r[j] + a[lo + i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res = res + a[lo + i]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return _pairwise_block(a, lo, n2) + _pairwise_block(a, lo + n2, n - n2)


def pairwise_sum(a):
    """Sum of the 1-D sequence ``a`` in the exact order ``np.add.reduce`` uses
    for a contiguous float64 row (buffer chunks of 8192, pairwise inside)."""
    a = [float(v) for v in a]
    res = 0.0
    for s in range(0, len(a), NPY_BUFSIZE):
        res = res + _pairwise_block(a, s, min(NPY_BUFSIZE, len(a) - s))
    return res


def vec_matrix_euclid(vector, matrix):
    """``_vec_matrix_euclid`` -- reference base.py:204-205 (verbatim math)."""
    return np.linalg.norm(vector - matrix, axis=1)


def vec_euclid(vec1, vec2):
    """``_vec_euclid`` -- reference base.py:208-209 (BLAS dot based norm)."""
    return np.linalg.norm(vec1 - vec2)


def _chunk_rows(n, k, d, budget=1 << 22):
    return max(1, int(budget // max(1, k * d)))


def dense_distances(X, C):
    """Distances of every row of X to every centre, bit-identical to calling
    ``vec_matrix_euclid(x, C)`` per row (reference base.py:171-172)."""
    X = np.asarray(X)
    C = np.asarray(C, dtype=np.float64)
    n, d = X.shape
    k = C.shape[0]
    out = np.empty((n, k), dtype=np.float64)
    step = _chunk_rows(n, k, d)
    for s in range(0, n, step):
        diff = X[s:s + step, None, :] - C[None, :, :]
        np.multiply(diff, diff, out=diff)
        np.sqrt(np.add.reduce(diff, axis=2), out=out[s:s + step])
    return out


# --------------------------------------------------------------------------
# Sparse distances: sklearn.metrics.pairwise._euclidean_distances (1.7.2,
# metrics/pairwise.py:391-442) as reached from base.py:169,196.
# --------------------------------------------------------------------------
def _seq_sq_norm(vals):
    # sklearn utils/sparsefuncs_fast.pyx:26-44 -- sequential over stored nnz
    acc = 0.0
    for v in vals:
        acc = acc + float(v) * float(v)
    return acc


def sparse_row_distances(idx, val, C_dense, c_norm2):
    """sqrt(max(0, ((-2*dot) + ||x||^2) + ||c||^2)) with scipy csr_matmat's
    sequential dot (x's stored order) -- one CSR sample vs dense centres."""
    k = C_dense.shape[0]
    dot = np.zeros(k)
    for j, v in zip(idx, val):
        dot = dot + float(v) * C_dense[:, j]          # per-centre sequential
    xx = _seq_sq_norm(val)
    dist = -2.0 * dot
    dist = dist + xx
    dist = dist + c_norm2
    np.maximum(dist, 0.0, out=dist)
    return np.sqrt(dist)


def centre_sq_norms_sparse(C_csr):
    """Row norms of the CSR centre matrix, sequential over stored entries."""
    C_csr = C_csr.tocsr()
    out = np.empty(C_csr.shape[0])
    for r in range(C_csr.shape[0]):
        out[r] = _seq_sq_norm(C_csr.data[C_csr.indptr[r]:C_csr.indptr[r + 1]])
    return out


def sparse_distances(X_csr, C_csr):
    C_dense = np.asarray(C_csr.toarray(), dtype=np.float64)
    cn = centre_sq_norms_sparse(C_csr)
    X_csr = X_csr.tocsr()
    out = np.empty((X_csr.shape[0], C_dense.shape[0]))
    for i in range(X_csr.shape[0]):
        a, b = X_csr.indptr[i], X_csr.indptr[i + 1]
        out[i] = sparse_row_distances(X_csr.indices[a:b], X_csr.data[a:b],
                                      C_dense, cn)
    return out


# --------------------------------------------------------------------------
# Tasks of the Lloyd iteration
# --------------------------------------------------------------------------
def init_centers(n_features, sparse, n_clusters, random_state):
    """``_init_centers`` -- reference base.py:155-163."""
    if isinstance(random_state, np.random.RandomState):
        # np.random.seed rejects a RandomState instance (Appendix B.1)
        raise TypeError("random_state must be an int or None")
    np.random.seed(random_state)
    centers = np.random.random((n_clusters, n_features))
    if sparse:
        from scipy.sparse import csr_matrix
        centers = csr_matrix(centers)
    return centers


def _sum_dtype(x_dtype):
    if np.issubdtype(x_dtype, np.floating):
        return x_dtype
    if np.issubdtype(x_dtype, np.bool_):
        return np.int64
    return np.result_type(x_dtype, np.int64)


def partial_sum(samples, centers, sparse=False):
    """``_partial_sum`` -- reference base.py:166-181.

    Returns (labels int64[n], sums[k, d] in the samples' accumulation dtype,
    counts int64[k]).  Empty clusters have sums == 0 and counts == 0, which
    adds exactly like the reference's integer ``0`` placeholder.
    """
    k = centers.shape[0]
    if sparse:
        dist = sparse_distances(samples, centers)
        labels = np.argmin(dist, axis=1)
        X = samples.toarray()
    else:
        X = np.asarray(samples)
        dist = dense_distances(X, centers)
        labels = np.argmin(dist, axis=1)
    sums = np.zeros((k, X.shape[1]), dtype=_sum_dtype(X.dtype))
    np.add.at(sums, labels, X)                       # sequential, sample order
    counts = np.bincount(labels, minlength=k).astype(np.int64)
    return labels.astype(np.int64), sums, counts


def predict_labels(samples, centers, sparse=False):
    """``_predict`` -- reference base.py:194-201."""
    if sparse:
        return np.argmin(sparse_distances(samples, centers), axis=1)
    return np.argmin(dense_distances(np.asarray(samples), centers), axis=1)


def merge_tree(partials, arity):
    """``_recompute_centers`` reduction loop + ``_merge`` -- base.py:137-141,
    184-191.  ``partials`` is a list of (sums, counts); returns the root."""
    partials = list(partials)
    while len(partials) > 1:
        group = partials[:arity]
        partials = partials[arity:]
        acc_s = group[0][0].copy()
        acc_c = group[0][1].copy()
        for s, c in group[1:]:
            acc_s += s
            acc_c += c
        partials.append((acc_s, acc_c))
    return partials[0]


def recompute_centers(centers, root, sparse=False):
    """base.py:145-147 -- in place; empty clusters keep their old centre.

    Sparse partial sums are scipy CSR rows, and scipy's scalar true-divide is
    ``self._mul_scalar(1./other)`` (scipy/sparse/_base.py ``_divide``): the
    sparse centre is ``sum * (1.0 / count)``, not ``sum / count``."""
    sums, counts = root
    for idx in range(centers.shape[0]):
        if counts[idx] != 0:
            cnt = int(counts[idx])        # a Python int, as in the reference
            if sparse:
                centers[idx] = sums[idx] * (1.0 / cnt)
            else:
                centers[idx] = sums[idx] / cnt    # fp32 sums stay fp32 here
    return centers


def converged_diff(centers, old_centers, sparse=False):
    """``_converged`` criterion -- base.py:122-135."""
    if sparse:
        from sklearn.metrics import pairwise_distances
        diff = 0
        for i in range(centers.shape[0]):
            diff += pairwise_distances(centers[i], old_centers[i])
        return diff
    diff = 0
    for i, c in enumerate(centers):
        diff += vec_euclid(c, old_centers[i])
    return diff


class OracleKMeans:
    """Sequential restatement of ``KMeans`` (base.py:9-147) over a list of
    Subset sample blocks.  ``trace`` records the centres after each update."""

    def __init__(self, n_clusters=8, max_iter=10, tol=1e-4, arity=50,
                 random_state=None, verbose=False):
        self.n_clusters = n_clusters
        self.max_iter = max_iter
        self.tol = tol
        self.arity = arity
        self.random_state = random_state
        self.verbose = verbose
        self.centers = None
        self.n_iter = 0
        self.trace = []

    def fit(self, blocks, sparse=False, set_labels=False):
        d = blocks[0].shape[1]
        self.centers = init_centers(d, sparse, self.n_clusters,
                                    self.random_state)
        if sparse:
            self.centers = self.centers.toarray()
        old = None
        it = 0
        labels = None
        self.trace = []
        while True:
            if old is not None:
                diff = converged_diff(
                    _as_sparse(self.centers) if sparse else self.centers,
                    _as_sparse(old) if sparse else old, sparse)
                if self.verbose:
                    print("Iteration %s - Convergence crit. = %s" % (it, diff))
                if diff < self.tol ** 2 or it >= self.max_iter:
                    break
            old = self.centers.copy()
            parts = []
            lab = []
            for b in blocks:
                cen = _as_sparse(old) if sparse else old
                l_, s_, c_ = partial_sum(b, cen, sparse)
                parts.append((s_, c_))
                lab.append(l_)
            recompute_centers(self.centers, merge_tree(parts, self.arity), sparse)
            self.trace.append(self.centers.copy())
            labels = np.concatenate(lab) if lab else None
            it += 1
        self.n_iter = it
        return labels if set_labels else None

    def predict(self, blocks, sparse=False):
        cen = _as_sparse(self.centers) if sparse else self.centers
        return np.concatenate([predict_labels(b, cen, sparse) for b in blocks])


def _as_sparse(c):
    from scipy.sparse import csr_matrix
    return csr_matrix(c)


# --------------------------------------------------------------------------
# Synthetic make_blobs generator shared with the HIP generator (the bench's
# on-device data).  Counter-based, so any row range can be regenerated here.
# --------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def _splitmix64(z):
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _splitmix64_np(z):
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def blob_centres(n_blobs, d, seed, box=10.0):
    """Blob centres: U(-box, box) from the counter hash (row-major)."""
    ctr = np.arange(n_blobs * d, dtype=np.uint64) + np.uint64(seed) * np.uint64(0x100000000)
    with np.errstate(over="ignore"):
        u = (_splitmix64_np(ctr ^ np.uint64(0xC0FFEE)) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    return ((2.0 * u - 1.0) * box).reshape(n_blobs, d)


def make_blobs_rows(row0, nrows, d, n_blobs, seed, box=10.0, std=1.0):
    """Rows [row0, row0+nrows) of the synthetic blob matrix.  Sample i belongs
    to blob hash(i) % n_blobs; element (i, j) = centre + std * N(0,1) with the
    normal drawn by Box-Muller from two hashed uniforms.  Mirrors
    ``dkm_make_blobs_f64`` bit-for-bit except for libm's log/cos rounding,
    which may differ by an ulp between host and device."""
    cen = blob_centres(n_blobs, d, seed, box)
    rows = np.arange(row0, row0 + nrows, dtype=np.uint64)
    sm = np.uint64(seed) << np.uint64(40)
    with np.errstate(over="ignore"):
        blob = (_splitmix64_np(rows ^ sm ^ np.uint64(0xB10B)) % np.uint64(n_blobs)).astype(np.int64)
        ctr = (rows[:, None] * np.uint64(d) + np.arange(d, dtype=np.uint64)[None, :]) ^ sm
        h1 = _splitmix64_np(ctr * np.uint64(2))
        h2 = _splitmix64_np(ctr * np.uint64(2) + np.uint64(1))
    u1 = ((h1 >> np.uint64(11)).astype(np.float64) + 1.0) * (2.0 ** -53)
    u2 = (h2 >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    z = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
    return cen[blob] + std * z, blob
