"""DBSCAN's epsilon query on the GPU distance primitive.

Reference: ``_compute_neighbours`` of
``/root/reference/dislib/cluster/dbscan/classes.py:124-141`` -- for every
sample of rows ``[begin_idx, end_idx)`` of the concatenated Subsets, the
indices of all samples whose ``_vec_matrix_euclid`` distance (``:153-154``,
numpy's ``sqrt(add.reduce((x - s)**2))`` in its pairwise order) is below
``epsilon``, ordered by distance, and whether there are at least
``min_samples`` of them.  The rest of DBSCAN (grid regions, equivalence
merging) is out of scope.

Here the concatenated samples are uploaded once and ``dkm_radius_count_f64``
/ ``dkm_radius_fill_f64`` compute the same fp64 distances (bit-exact: the
k-means exact arithmetic), select ``dist < epsilon``, and sort each list by
(distance, index).  The reference's ``np.argsort`` gives the same order
except among exactly equal distances, which it may order differently.

Sparse Subsets (``sparse=True``, the reference's ``pairwise_distances``
branch, ``:130``) go through ``dkm_radius_count_csr_f64`` /
``dkm_radius_fill_csr_f64``: sklearn 1.7's fp64 CSR expansion
``sqrt(max(-2 q.x + |q|^2 + |x|^2, 0))`` in its own operation order.  The
concatenated CSR matrix is taken with sorted column indices (a sorted copy
when a Subset's are not; scipy's products then follow the same order).
"""
import ctypes

import numpy as np

from .. import _lib
from .._device import _is_torch, on, ptr, resolve, stream_ptr, torch
from .._device import assert_all_finite as _device_assert_finite


def compute_neighbours(epsilon, min_samples, sparse, begin_idx, end_idx,
                       *subsets, device=None):
    """Same arguments and results as the reference task: a list of int64
    index arrays (one per query sample) and a list of core-point flags."""
    if sparse:
        return _compute_neighbours_csr(epsilon, min_samples, begin_idx,
                                       end_idx, subsets, device)
    t = torch()
    dev = resolve(device)
    with on(dev):
        X = _concat(subsets, dev)
        n, d = X.shape
        b, e = _slice_bounds(begin_idx, end_idx, n)
        Q = X[b:e]
        nq = e - b
        if nq == 0:
            return [], []
        so = _lib.lib()
        counts = t.empty(nq, dtype=t.int64, device=dev)
        _lib.check(so.dkm_radius_count_f64(
            ptr(Q), nq, X.stride(0), ptr(X), n, X.stride(0), d,
            float(epsilon), ptr(counts), stream_ptr()), "dkm_radius_count")
        c = counts.cpu().numpy()
        offsets = np.concatenate([[0], np.cumsum(c)]).astype(np.int64)
        total = int(offsets[-1])
        off_d = t.from_numpy(offsets).to(dev)
        out_i = t.empty(max(total, 1), dtype=t.int64, device=dev)
        out_d = t.empty(max(total, 1), dtype=t.float64, device=dev)
        wsb = int(so.dkm_radius_workspace_bytes(nq, total))
        ws = t.empty(wsb, dtype=t.uint8, device=dev)
        _lib.check(so.dkm_radius_fill_f64(
            ptr(Q), nq, X.stride(0), ptr(X), n, X.stride(0), d,
            float(epsilon), ptr(off_d), ctypes.c_void_p(ws.data_ptr()), wsb,
            ptr(out_i), ptr(out_d), stream_ptr()), "dkm_radius_fill")
        idx = out_i[:total].cpu().numpy()
    neigh = [idx[offsets[i]:offsets[i + 1]] for i in range(nq)]
    core = [bool(c[i] >= min_samples) for i in range(nq)]
    return neigh, core


def _compute_neighbours_csr(epsilon, min_samples, begin_idx, end_idx,
                            subsets, device):
    m = _concat_csr(subsets)
    t = torch()
    dev = resolve(device)
    n, d = m.shape
    b, e = _slice_bounds(begin_idx, end_idx, n)
    nq = e - b
    if nq == 0:
        return [], []
    so = _lib.lib()
    with on(dev):
        indptr = t.from_numpy(m.indptr.astype(np.int64)).to(dev)
        indices = t.from_numpy(
            np.ascontiguousarray(m.indices, dtype=np.int32)).to(dev)
        data = t.from_numpy(
            np.ascontiguousarray(m.data, dtype=np.float64)).to(dev)
        if data.numel() == 0:  # keep valid device pointers
            indices = t.zeros(1, dtype=t.int32, device=dev)
            data = t.zeros(1, dtype=t.float64, device=dev)
        counts = t.empty(nq, dtype=t.int64, device=dev)
        f32 = 1 if getattr(m, "dkm_f32", False) else 0
        _lib.check(so.dkm_radius_count_csr_f64(
            ptr(indptr), ptr(indices), ptr(data), n, d, b, nq,
            float(epsilon), f32, ptr(counts), stream_ptr()),
            "dkm_radius_count_csr")
        c = counts.cpu().numpy()
        offsets = np.concatenate([[0], np.cumsum(c)]).astype(np.int64)
        total = int(offsets[-1])
        off_d = t.from_numpy(offsets).to(dev)
        out_i = t.empty(max(total, 1), dtype=t.int64, device=dev)
        out_d = t.empty(max(total, 1), dtype=t.float64, device=dev)
        wsb = int(so.dkm_radius_workspace_bytes(nq, total))
        ws = t.empty(wsb, dtype=t.uint8, device=dev)
        _lib.check(so.dkm_radius_fill_csr_f64(
            ptr(indptr), ptr(indices), ptr(data), n, d, b, nq,
            float(epsilon), f32, ptr(off_d), ctypes.c_void_p(ws.data_ptr()),
            wsb, ptr(out_i), ptr(out_d), stream_ptr()),
            "dkm_radius_fill_csr")
        idx = out_i[:total].cpu().numpy()
    neigh = [idx[offsets[i]:offsets[i + 1]] for i in range(nq)]
    core = [bool(c[i] >= min_samples) for i in range(nq)]
    return neigh, core


def _concat_csr(subsets, who="compute_neighbours"):
    """The concatenated sparse samples as one CSR matrix with sorted column
    indices (``_concatenate_subsets`` -> ``vstack``, classes.py:144-150).
    Also the fit / query matrix of the sparse kNN (``who`` names the caller
    in the errors)."""
    import scipy.sparse as sp
    if not subsets:
        raise ValueError("%s: no Subsets" % who)
    parts = []
    for s in subsets:
        x = s.samples
        if not sp.issparse(x):
            raise ValueError("%s: sparse=True needs sparse Subsets" % who)
        parts.append(x)
    m = sp.csr_matrix(parts[0] if len(parts) == 1 else
                      sp.vstack(parts, format="csr"))
    f32 = m.dtype == np.float32   # sklearn's float32 (upcast) path
    m = sp.csr_matrix(m, dtype=np.float64)
    if not m.has_sorted_indices:
        m = m.sorted_indices()
    if m.shape[1] > np.iinfo(np.int32).max:
        raise ValueError("%s: too many features" % who)
    # duplicate column entries in a row (legal while a scipy matrix is not
    # in canonical format): scipy's csr_matmat multiplies every stored pair
    # in stored order, which the kernel's merge of two sorted rows does not
    # reproduce -- refuse them loudly instead of returning other distances
    ind = m.indices
    if ind.size > 1:
        same = ind[1:] == ind[:-1]
        if same.any():
            row_start = np.zeros(ind.size, bool)
            row_start[m.indptr[:-1][np.diff(m.indptr) > 0]] = True
            if (same & ~row_start[1:]).any():
                raise ValueError(
                    "%s: sparse samples hold duplicate column entries; call "
                    "sum_duplicates() on them first" % who)
    _device_assert_finite(m.data)
    m.dkm_f32 = bool(f32)
    return m


def _concat(subsets, dev):
    """The concatenated samples as one fp64 (n, d) device matrix
    (``_concatenate_subsets``, classes.py:144-150)."""
    t = torch()
    if not subsets:
        raise ValueError("compute_neighbours: no Subsets")
    parts = []
    for s in subsets:
        x = s.samples
        if _is_torch(x):
            parts.append(x.to(dev, dtype=t.float64))
        else:
            if hasattr(x, "toarray"):
                raise ValueError("compute_neighbours: sparse Subsets are not"
                                 " supported by the GPU path")
            parts.append(t.from_numpy(np.ascontiguousarray(
                np.asarray(x, dtype=np.float64))).to(dev))
    X = parts[0] if len(parts) == 1 else t.cat(parts, 0)
    return X.contiguous()


def _slice_bounds(begin, end, n):
    """``samples[begin:end]`` bounds with Python slice semantics."""
    b, e, _ = slice(begin, end).indices(n)
    return b, max(b, e)
