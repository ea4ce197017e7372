"""``dislib.neighbors.NearestNeighbors`` on the GPU distance primitive
(SURVEY.md 8 f4).

Reference: ``/root/reference/dislib/neighbors/base.py:7-133``.  There,
``kneighbors`` fits a scikit-learn ``NearestNeighbors`` on every fit Subset,
queries it with every query Subset (``_get_neighbors`` ``:103-111``) and
merges the per-pair lists by sort (``_merge_queries`` ``:90-100``).  Here
both Datasets stay resident in HBM and one ``dkm_knn_f64`` call ranks every
fit row for every query row: the distance is sklearn's KD-tree Euclidean
``sqrt(sum_t (q_t - x_t)**2)`` summed sequentially (what sklearn runs for
d <= 15), neighbours ascending by (squared distance, fit row).  For d > 15
sklearn switches to its GEMM-expanded brute force, whose rounding no fixed
order reproduces; the distances here are the exactly ordered ones
(DESIGN.md section 7).

Differences from the reference (documented, not reproduced):
* ``_merge_queries`` walks ``range(n_samples)`` with the *fit* Subset size
  (``base.py:96``); the rows are the query rows here.
* ``n_neighbors`` beyond 32 runs in passes of 32 columns (the kernel's
  register-resident top-k), each starting after the previous pass's last
  (distance, index).
* Sparse Subsets: sklearn fits brute force on CSR and ranks by
  ``pairwise_distances_chunked(squared=True)`` (its ArgKmin reduction
  refuses sparse-sparse pairs): ``dkm_knn_csr_f64`` computes the same
  ``((-2 q.x) + ||q||^2) + ||x||^2`` in the same order (the sparse epsilon
  query's arithmetic), so the distances are bit-exact; rows are read with
  sorted column indices, and a row holding a duplicate column is refused.
  A dense query against sparse fit data (or the reverse) raises ValueError:
  the reference's kd_tree refuses the one, and the other takes a
  dense-times-sparse product whose order is scipy's, not pinned here.
* Ties: the reference merges with ``np.argsort`` (quicksort, unstable);
  here equal distances come out by ascending fit row.
"""
import ctypes
import numbers

import numpy as np

from .. import _lib
from .._device import on, ptr, stream_ptr, torch


class NearestNeighbors:
    """Unsupervised neighbour search (reference ``base.py:7-38``).

    Parameters
    ----------
    n_neighbors : int, optional (default=5)
        Number of neighbours for :meth:`kneighbors` queries.
    device : keyword-only, optional
        GPU to run on (default: the current device).
    """


    def __init__(self, n_neighbors=5, *, device=None):
        self._n_neighbors = n_neighbors
        self._fit_dataset = None
        self._device = device

    def fit(self, dataset):
        """Keep ``dataset`` as the fitted data (reference ``base.py:30-38``)."""
        self._fit_dataset = dataset

    def kneighbors(self, dataset, n_neighbors=None, return_distance=True):
        """Distances and fit-row indices of the ``n_neighbors`` nearest fit
        samples of every sample of ``dataset`` (reference ``base.py:40-87``).

        Returns ``(dist, ind)`` -- or ``ind`` when ``return_distance`` is
        False -- as ``(n_samples, n_neighbors)`` float64 / int64 arrays.
        """
        if n_neighbors is None:
            n_neighbors = self._n_neighbors
        if self._fit_dataset is None:
            raise ValueError("NearestNeighbors: call fit() first")
        _check_n_neighbors(n_neighbors, self._fit_dataset)
        if dataset.sparse or self._fit_dataset.sparse:
            if not (dataset.sparse and self._fit_dataset.sparse):
                raise ValueError("NearestNeighbors: the query and the fitted "
                                 "Dataset must both be sparse or both dense")
            return self._kneighbors_csr(dataset, n_neighbors,
                                        return_distance)
        t = torch()
        fit_dd = self._fit_dataset._device_data(self._device)
        q_dd = dataset._device_data(fit_dd.device)
        so = _lib.lib()
        nq, nx, d = q_dd.n, fit_dd.n, fit_dd.d
        if q_dd.d != d:
            raise ValueError("X has %d features, but NearestNeighbors is "
                             "expecting %d features as input" % (q_dd.d, d))
        with on(fit_dd.device):
            X = _as_f64(fit_dd.X)
            Q = _as_f64(q_dd.X)
            out_d = t.empty((nq, n_neighbors), dtype=t.float64,
                            device=fit_dd.device)
            out_i = t.empty((nq, n_neighbors), dtype=t.int64,
                            device=fit_dd.device)
            if nq:
                wsb = int(so.dkm_knn_workspace_bytes(nq, nx, n_neighbors))
                ws = t.empty(max(wsb, 1), dtype=t.uint8, device=fit_dd.device)
                _lib.check(so.dkm_knn_f64(
                    ptr(Q), nq, Q.stride(0), ptr(X), nx, X.stride(0), d,
                    n_neighbors, ctypes.c_void_p(ws.data_ptr()), wsb,
                    ptr(out_d), ptr(out_i), stream_ptr()), "dkm_knn_f64")
            ind = out_i.cpu().numpy()
            if not return_distance:
                return ind
            return out_d.cpu().numpy(), ind


    def _kneighbors_csr(self, dataset, n_neighbors, return_distance):
        """CSR Subsets: both Datasets concatenated to one CSR matrix each
        (sorted indices, finite, no duplicate columns) and ranked by
        ``dkm_knn_csr_f64``."""
        from ..cluster.dbscan import _concat_csr
        from .._device import resolve
        t = torch()
        xf = _concat_csr(list(self._fit_dataset), "NearestNeighbors")
        same = dataset is self._fit_dataset
        xq = xf if same else _concat_csr(list(dataset), "NearestNeighbors")
        nq, nx, d = xq.shape[0], xf.shape[0], xf.shape[1]
        if xq.shape[1] != d:
            raise ValueError("X has %d features, but NearestNeighbors is "
                             "expecting %d features as input"
                             % (xq.shape[1], d))
        dev = resolve(self._device)
        so = _lib.lib()
        with on(dev):
            f = _csr_to(xf, dev)
            q = f if same else _csr_to(xq, dev)
            out_d = t.empty((nq, n_neighbors), dtype=t.float64, device=dev)
            out_i = t.empty((nq, n_neighbors), dtype=t.int64, device=dev)
            # float32 on both sides: sklearn's upcast path (r rounded to
            # float32, float32 sqrt)
            f32 = 1 if (getattr(xf, "dkm_f32", False) and
                        getattr(xq, "dkm_f32", False)) else 0
            if nq:
                wsb = int(so.dkm_knn_workspace_bytes(nq, nx, n_neighbors))
                ws = t.empty(max(wsb, 1), dtype=t.uint8, device=dev)
                _lib.check(so.dkm_knn_csr_f64(
                    ptr(q[0]), ptr(q[1]), ptr(q[2]), nq, ptr(f[0]),
                    ptr(f[1]), ptr(f[2]), nx, d, n_neighbors, f32,
                    ctypes.c_void_p(ws.data_ptr()), wsb, ptr(out_d),
                    ptr(out_i), stream_ptr()), "dkm_knn_csr_f64")
            ind = out_i.cpu().numpy()
            if not return_distance:
                return ind
            dist = out_d.cpu().numpy()
            # float32 Subsets: sklearn returns float32 distances (the
            # values are float32 already)
            return (dist.astype(np.float32) if f32 else dist), ind


def _csr_to(m, dev):
    """(indptr int64, indices int32, data fp64) device tensors of a CSR
    matrix (one-element arrays for an all-zero matrix, so every pointer is
    a valid device address)."""
    t = torch()
    indptr = t.from_numpy(m.indptr.astype(np.int64)).to(dev)
    indices = np.ascontiguousarray(m.indices, dtype=np.int32)
    data = np.ascontiguousarray(m.data, dtype=np.float64)
    if data.size == 0:
        indices = np.zeros(1, np.int32)
        data = np.zeros(1, np.float64)
    return indptr, t.from_numpy(indices).to(dev), t.from_numpy(data).to(dev)


def _as_f64(x):
    t = torch()
    return x if x.dtype == t.float64 else x.to(t.float64)


def _check_n_neighbors(n_neighbors, fit_dataset):
    """sklearn's argument checks, per fit Subset as the reference meets
    them (``_get_neighbors`` fits one model per Subset)."""
    if isinstance(n_neighbors, bool) or \
            not isinstance(n_neighbors, numbers.Integral):
        raise TypeError("n_neighbors does not take %s value, enter integer "
                        "value" % type(n_neighbors))
    if n_neighbors <= 0:
        raise ValueError("Expected n_neighbors > 0. Got %d" % n_neighbors)
    for s in fit_dataset:
        n_fit = int(s.samples.shape[0])
        if n_neighbors > n_fit:
            raise ValueError(
                "Expected n_neighbors <= n_samples_fit, but n_neighbors = %d,"
                " n_samples_fit = %d" % (n_neighbors, n_fit))
    if len(fit_dataset) == 0:
        raise ValueError("NearestNeighbors: the fitted Dataset is empty")
