"""C5-style sparse bench line (BASELINE configs[4], scaled by --n): CSR rows
with --nnz entries in --d columns (strictly increasing random columns,
values U(0,1)), k centres, the fit loop's Lloyd step through the same
_Lloyd driver as bench.py, then predict.  Prints one JSON line.

  python tools/bench_csr.py --n 10000000 --d 10000 --nnz 10 --k 256
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=10_000)
    ap.add_argument("--nnz", type=int, default=10)
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--subset", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    gap = max(1, a.d // a.nnz - 1)
    cols = np.cumsum(rng.integers(1, gap + 1, (a.n, a.nnz)), axis=1) - 1
    indptr = np.arange(0, a.n * a.nnz + 1, a.nnz, dtype=np.int64)
    data = rng.random(a.n * a.nnz)
    X = sp.csr_matrix((data, cols.reshape(-1).astype(np.int32), indptr),
                      shape=(a.n, a.d))
    import torch
    from dislib_amd.cluster.kmeans import _Lloyd, _init_centers
    from dislib_amd.data import Dataset, Subset
    dev = torch.device("cuda", 0)
    ds = Dataset(n_features=a.d, sparse=True)
    for i in range(0, a.n, a.subset):
        ds.append(Subset(X[i:i + a.subset]))
    st = _Lloyd(ds, _init_centers(a.d, True, a.k, 0).toarray(), 0.0, False,
                "auto", dev)
    torch.cuda.synchronize()
    st.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        st.prepare()
        st.partial()
        st.reduce_update()
        st.read_flags()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # one full (refresh) assignment + sums, and predict, timed alone
    from dislib_amd import _device, _lib
    t0 = time.perf_counter()
    st.prepare()
    _device.partial_sum(st.dd, st.C, st.ws, st.labels, st.acc,
                        _lib.MODE_AUTO)
    torch.cuda.synchronize()
    full_ms = (time.perf_counter() - t0) * 1e3
    lab = torch.empty(st.dd.n, dtype=torch.int32, device=dev)
    _device.predict(st.dd, st.C, st.ws, lab, _lib.MODE_AUTO)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        _device.predict(st.dd, st.C, st.ws, lab, _lib.MODE_AUTO)
    torch.cuda.synchronize()
    pred_ms = (time.perf_counter() - t0) / a.steps * 1e3
    nnz = a.n * a.nnz
    out = {"metric": "KMeans samples·iters/sec (sparse CSR fit)",
           "value": a.n * a.steps / el, "unit": "samples·iters/s",
           "ms_per_step": el / a.steps * 1e3, "dtype": "f64",
           "config": {"workload": "CSR %dx%d, %d nnz/row, k=%d" %
                      (a.n, a.d, a.nnz, a.k), "nnz": nnz},
           "bytes_per_step": 12 * nnz + 8 * (a.n + 1),
           "hbm_gbs": (12 * nnz + 8 * (a.n + 1)) / (el / a.steps) / 1e9,
           # k_csr_screen gathers fp32 centre columns (C^T): 4 B a value
           "gather_bytes_per_step": 4 * nnz * a.k,
           "gather_tbs": 4 * nnz * a.k / (el / a.steps) / 1e12,
           "full_sums_iteration_ms": full_ms,
           "predict_ms": pred_ms,
           "predict_samples_per_s": a.n / (pred_ms * 1e-3),
           "rechecked_total": st.rechecked()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
