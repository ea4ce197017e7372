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
* Sparse Subsets are not supported on this path.
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
            raise ValueError("NearestNeighbors: sparse Subsets are not "
                             "supported by the GPU path")
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
