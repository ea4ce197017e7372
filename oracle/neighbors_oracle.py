"""CPU oracle for the distance-primitive reuse rows --
TEST INFRASTRUCTURE ONLY.

Restates, in numpy/scikit-learn, the two reference call sites that reuse
k-means' distance primitive:

* ``NearestNeighbors.kneighbors`` (``/root/reference/dislib/neighbors/
  base.py:40-87``): sklearn ``NearestNeighbors(n_neighbors)`` fitted on each
  fit Subset and queried with each query Subset (``_get_neighbors``
  ``:103-111``), the per-pair results merged left to right
  (``_merge_queries`` ``:90-100``: global indices by running offsets, then
  per row the ``n_neighbors`` smallest of the concatenated distances by
  ``np.sort`` / ``np.argsort``, ``_min_distances`` / ``_min_indices``
  ``:114-126``), and the query Subsets' results stacked (``:131-133``).
* the DBSCAN epsilon query ``_compute_neighbours`` (``/root/reference/
  dislib/cluster/dbscan/classes.py:124-141``): for every sample of rows
  ``[begin, end)`` of the concatenated Subsets, the indices of all samples
  with ``_vec_matrix_euclid`` distance ``< epsilon`` (``:153-154``; numpy's
  pairwise order, the k-means oracle's ``vec_matrix_euclid``), sorted by
  distance, and the core flag ``count >= min_samples``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module; ``dislib_amd`` never does.

Parity pin: ``tests/test_neighbors_golden.py`` checks both restatements
against ``tests/golden/neighbors_ref.npz``, which the reference itself wrote
(``tests/golden/gen_golden_neighbors.py``).

Arithmetic the GPU kernels follow (and :func:`seq_distances` states):
sklearn picks ``kd_tree`` when ``d <= 15`` and ``n_neighbors < n_fit // 2``
(``sklearn/neighbors/_base.py`` ``_fit``), whose Euclidean ``rdist`` is the
sequential sum ``r = 0; r += (x_t - y_t)**2`` over t = 0..d-1 (no FMA) and
whose reported distance is ``sqrt(r)``.  Otherwise it runs ``brute``, whose
Euclidean distances come from the GEMM expansion
``|x|^2 - 2 x.y + |y|^2`` (BLAS order: not reproducible bit for bit, so
that regime is compared within a stated tolerance).

One reference quirk is not restated: ``_merge_queries`` iterates
``range(n_samples)`` with ``n_samples`` the size of the *fit* Subset
(``base.py:96``), which only equals the number of query rows when both
Subsets have the same size (every reference test and example); this oracle
and the GPU path use the query rows.
"""
import numpy as np

from .kmeans_oracle import vec_matrix_euclid


# --------------------------------------------------------------------------
# kneighbors (neighbors/base.py:40-133)
# --------------------------------------------------------------------------
def _get_neighbors(q_samples, f_samples, n_neighbors):
    """``_get_neighbors`` (base.py:103-111)."""
    from sklearn.neighbors import NearestNeighbors as SKNeighbors
    knn = SKNeighbors(n_neighbors=n_neighbors)
    knn.fit(X=f_samples)
    dist, ind = knn.kneighbors(X=q_samples)
    return dist, ind, f_samples.shape[0]


def _merge_queries(queries):
    """``_merge_queries`` (base.py:90-100) with the query-row count."""
    final_dist, final_ind, offset = queries[0]
    final_ind = final_ind.copy()
    for dist, ind, n_samples in queries[1:]:
        ind = ind + offset
        offset += n_samples
        rows, num = final_dist.shape
        comb_d = np.hstack((final_dist, dist))
        comb_i = np.hstack((final_ind, ind))
        m_ind = np.array([np.argsort(comb_d[i])[:num] for i in range(rows)])
        final_ind = np.array([comb_i[i][m_ind[i]] for i in range(rows)])
        final_dist = np.array([np.sort(comb_d[i])[:num] for i in range(rows)])
    return final_dist, final_ind


def kneighbors(fit_blocks, query_blocks, n_neighbors):
    """The reference's ``kneighbors`` over lists of Subset sample blocks."""
    dists, inds = [], []
    for qb in query_blocks:
        parts = [_get_neighbors(qb, fb, n_neighbors) for fb in fit_blocks]
        d, i = _merge_queries(parts)
        dists.append(d)
        inds.append(i)
    return np.vstack(dists), np.vstack(inds)


def seq_distances(q, X):
    """sklearn KD-tree Euclidean distance of q to every row of X:
    ``sqrt(sum_t (q_t - x_t)**2)`` summed sequentially from 0."""
    X = np.asarray(X, dtype=np.float64)
    q = np.asarray(q, dtype=np.float64)
    r = np.zeros(X.shape[0])
    for t in range(X.shape[1]):
        df = q[t] - X[:, t]
        r = r + df * df
    return np.sqrt(r)


def kneighbors_exact(fit, query, n_neighbors):
    """Brute force over the whole fit set with :func:`seq_distances`,
    ascending (distance, index): the GPU kernel's contract."""
    fit = np.asarray(fit, dtype=np.float64)
    out_d = np.empty((len(query), n_neighbors))
    out_i = np.empty((len(query), n_neighbors), dtype=np.int64)
    idx = np.arange(len(fit))
    for r, q in enumerate(np.asarray(query, dtype=np.float64)):
        dist = seq_distances(q, fit)
        order = np.lexsort((idx, dist))[:n_neighbors]
        out_d[r] = dist[order]
        out_i[r] = order
    return out_d, out_i


# --------------------------------------------------------------------------
# DBSCAN epsilon query (cluster/dbscan/classes.py:124-141)
# --------------------------------------------------------------------------
def compute_neighbours(epsilon, min_samples, begin_idx, end_idx, samples):
    """Dense ``_compute_neighbours`` over the concatenated samples.  Lists
    are ordered by (distance, index): the reference's ``np.argsort`` is the
    same order except among exactly equal distances."""
    samples = np.asarray(samples)
    neighbour_list, core_points = [], []
    for sample in samples[begin_idx:end_idx]:
        dist = vec_matrix_euclid(sample, samples).flatten()
        neigh = np.where(dist < epsilon)[0]
        neigh = neigh[np.lexsort((neigh, dist[neigh]))]
        neighbour_list.append(neigh)
        core_points.append(neigh.size >= min_samples)
    return neighbour_list, core_points


# --------------------------------------------------------------------------
# sparse epsilon query (cluster/dbscan/classes.py:124-141, sparse=True)
# --------------------------------------------------------------------------
def _seq_row_sums(indptr, vals):
    """Per-row sums of ``vals`` (one per stored entry) accumulated from 0 in
    stored order -- the loop of sklearn's ``_sqeuclidean_row_norms_sparse``;
    vectorised over rows, one entry position at a time."""
    n = indptr.size - 1
    lens = np.diff(indptr)
    acc = np.zeros(n)
    for k in range(int(lens.max()) if n else 0):
        rows = np.nonzero(lens > k)[0]
        acc[rows] = acc[rows] + vals[indptr[rows] + k]
    return acc


def csr_sq_distances(indptr, indices, data, q):
    """``pairwise_distances(row q, X) ** 2`` before the sqrt, as sklearn 1.7
    (``metrics/pairwise.py`` ``_euclidean_distances``, fp64) computes it for
    CSR input with sorted indices: ``XX = row_norms(q)``, ``YY =
    row_norms(X)`` (stored-order sums), ``D = -2 * (q @ X.T)`` (scipy
    ``csr_matmat``: the products ``q_c * x_c`` of the matching columns summed
    from 0 in q's stored order), ``D += XX``, ``D += YY``,
    ``np.maximum(D, 0)``."""
    indptr = np.asarray(indptr, np.int64)
    qa, qb = indptr[q], indptr[q + 1]
    return csr_sq_distances_to(np.asarray(indices)[qa:qb],
                               np.asarray(data, np.float64)[qa:qb],
                               indptr, indices, data)


def csr_sq_distances_to(qi, qv, indptr, indices, data, yy=None):
    """:func:`csr_sq_distances` of a query row given by its sorted column
    indices ``qi`` and values ``qv`` against every row of the CSR matrix
    (``yy``: its precomputed stored-order row norms, optional)."""
    indptr = np.asarray(indptr, np.int64)
    indices = np.asarray(indices)
    data = np.asarray(data, np.float64)
    if yy is None:
        yy = _seq_row_sums(indptr, data * data)
    xx = 0.0
    for v in qv:
        xx += v * v
    # the matching query entry of every stored entry (or none)
    if qi.size:
        pos = np.minimum(np.searchsorted(qi, indices), qi.size - 1)
        match = qi[pos] == indices
        with np.errstate(all="ignore"):
            prod = qv[pos] * data
    else:
        match = np.zeros(indices.size, bool)
        prod = np.zeros(indices.size)
    n = indptr.size - 1
    lens = np.diff(indptr)
    dot = np.zeros(n)
    for k in range(int(lens.max()) if n else 0):
        rows = np.nonzero(lens > k)[0]
        at = indptr[rows] + k
        m = match[at]
        dot[rows[m]] = dot[rows[m]] + prod[at[m]]
    r = -2.0 * dot
    r += xx
    r += yy
    return np.maximum(r, 0.0)


def kneighbors_csr(f_csr, q_csr, n_neighbors, f32=False):
    """Sparse ``kneighbors`` (reference neighbors/base.py:40-111 on CSR
    Subsets): sklearn fits brute force on CSR and ranks by
    ``pairwise_distances_chunked(squared=True)`` -- the squared distances of
    :func:`csr_sq_distances_to` -- then reports ``sqrt``.  ``f_csr`` /
    ``q_csr`` = (indptr, indices, data) with sorted indices.  Returns
    ``(dist, ind)`` ascending by (squared distance, fit row); the
    reference's argpartition / argsort order equal distances arbitrarily.
    ``f32``: float32 Subsets -- sklearn's ``_euclidean_distances_upcast``
    computes the same fp64 squares, casts them to float32, then max and
    sqrt in float32."""
    fp, fi, fd = (np.asarray(a) for a in f_csr)
    qp, qi, qd = (np.asarray(a) for a in q_csr)
    fd = fd.astype(np.float64)
    yy = _seq_row_sums(fp.astype(np.int64), fd * fd)
    nq = qp.size - 1
    dist = np.empty((nq, n_neighbors))
    ind = np.empty((nq, n_neighbors), np.int64)
    rows = np.arange(fp.size - 1)
    for q in range(nq):
        a, b = qp[q], qp[q + 1]
        r = csr_sq_distances_to(qi[a:b], qd[a:b].astype(np.float64), fp, fi,
                                fd, yy)
        if f32:
            r = r.astype(np.float32)
        o = np.lexsort((rows, r))[:n_neighbors]
        dist[q] = np.sqrt(r[o])
        ind[q] = o
    return dist, ind


def compute_neighbours_csr(epsilon, min_samples, begin_idx, end_idx,
                           indptr, indices, data, f32=False):
    """Sparse ``_compute_neighbours``: same lists and flags as the dense
    form, distances by :func:`csr_sq_distances` then ``sqrt``.  ``f32``:
    float32 Subsets (the squares cast to float32, float32 sqrt, and numpy
    compares ``dist < epsilon`` in float32)."""
    n = len(indptr) - 1
    neighbour_list, core_points = [], []
    data = np.asarray(data, np.float64)
    for q in range(*slice(begin_idx, end_idx).indices(n)):
        r = csr_sq_distances(indptr, indices, data, q)
        dist = np.sqrt(r.astype(np.float32) if f32 else r)
        neigh = np.where(dist < epsilon)[0]
        neigh = neigh[np.lexsort((neigh, dist[neigh]))]
        neighbour_list.append(neigh)
        core_points.append(neigh.size >= min_samples)
    return neighbour_list, core_points
