"""Throughput of the f4 rows on one MI355X, with the
reference's CPU algorithm timed beside it on a bounded sample.

  python tools/bench_neighbors.py [--nfit N] [--nq Q] [--d D] [--kn K]
                                  [--eps-n N] [--eps E] [--eps-q Q]

kneighbors: queries/s against a fit set of nfit rows (dkm_knn_f64), with
  the fp64 VALU rate of its distance work (3 d ops per pair: sub, mul, add)
  against the vector fp64 instruction peak (78.6 TF/s counts an FMA as 2).
  CPU: the reference algorithm (oracle.neighbors_oracle.kneighbors: sklearn
  NearestNeighbors per (query Subset, fit Subset) pair + the sort merge) on
  a sample of query rows, one process.
kneighbors on CSR: queries/s of dkm_knn_csr_f64 (sp-kq queries against the
  sp-n CSR rows); CPU: the reference algorithm on CSR Subsets (sklearn brute
  force per Subset pair + the sort merge) on a sample of query rows.
epsilon query: queries/s of dkm_radius_count + fill (+ sort) over eps-n
  rows; CPU: the reference's per-sample _vec_matrix_euclid loop
  (oracle.neighbors_oracle.compute_neighbours) on a sample of queries.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FP64_VALU_PEAK = 78.6e12   # flop/s, FMA = 2 (MI355X_MICROARCH.md)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--nfit", type=int, default=1_000_000)
    p.add_argument("--nq", type=int, default=100_000)
    p.add_argument("--d", type=int, default=8)
    p.add_argument("--kn", type=int, default=5)
    p.add_argument("--subset", type=int, default=100_000)
    p.add_argument("--eps-n", type=int, default=400_000)
    p.add_argument("--eps-q", type=int, default=100_000)
    p.add_argument("--eps", type=float, default=0.25)
    p.add_argument("--sp-n", type=int, default=200_000)
    p.add_argument("--sp-d", type=int, default=10_000)
    p.add_argument("--sp-nnz", type=int, default=10)
    p.add_argument("--sp-q", type=int, default=50_000)
    p.add_argument("--sp-eps", type=float, default=1.5)
    p.add_argument("--sp-kq", type=int, default=20_000)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--no-cpu", action="store_true")
    a = p.parse_args()

    rng = np.random.default_rng(0)
    import scipy.sparse as sp
    xs = sp.random(a.sp_n, a.sp_d, density=a.sp_nnz / a.sp_d, format="csr",
                   random_state=rng)
    xs.sort_indices()
    xf = rng.random((a.nfit, a.d))
    xq = rng.random((a.nq, a.d))
    xe = rng.random((a.eps_n, a.d))
    cpu = {}
    if not a.no_cpu:
        from oracle import neighbors_oracle as orc
        blocks = [xf[i:i + a.subset] for i in range(0, a.nfit, a.subset)]
        m = 2000
        t0 = time.perf_counter()
        orc.kneighbors(blocks, [xq[:m]], a.kn)
        el = time.perf_counter() - t0
        cpu["knn"] = {"value": m / el, "unit": "queries/s", "cores": 1,
                      "kind": "port", "seconds": el,
                      "sample": "%d query rows against the full fit set "
                                "(%d Subsets of %d), sklearn per Subset "
                                "pair + sort merge" % (m, len(blocks),
                                                       a.subset)}
        m = 200
        t0 = time.perf_counter()
        orc.compute_neighbours(a.eps, 5, 0, m, xe)
        el = time.perf_counter() - t0
        cpu["eps"] = {"value": m / el, "unit": "queries/s", "cores": 1,
                      "kind": "port", "seconds": el,
                      "sample": "%d query rows against %d rows, the "
                                "reference's per-sample numpy loop"
                                % (m, a.eps_n)}
        from sklearn.metrics import pairwise_distances
        m = 100
        t0 = time.perf_counter()
        for i in range(m):
            dist = pairwise_distances(xs[i], xs).ravel()
            np.argsort(dist[np.where(dist < a.sp_eps)[0]])
        el = time.perf_counter() - t0
        cpu["eps_csr"] = {"value": m / el, "unit": "queries/s", "cores": 1,
                          "kind": "reference", "seconds": el,
                          "sample": "%d query rows against %d CSR rows, the "
                                    "reference's per-sample sklearn "
                                    "pairwise_distances loop" % (m, a.sp_n)}
        m = 500
        sblocks = [xs[i:i + a.subset] for i in range(0, a.sp_n, a.subset)]
        t0 = time.perf_counter()
        orc.kneighbors(sblocks, [xs[:m]], a.kn)
        el = time.perf_counter() - t0
        cpu["knn_csr"] = {"value": m / el, "unit": "queries/s", "cores": 1,
                          "kind": "port", "seconds": el,
                          "sample": "%d CSR query rows against %d CSR rows "
                                    "(%d Subsets), sklearn brute force per "
                                    "Subset pair + sort merge"
                                    % (m, a.sp_n, len(sblocks))}

    import torch
    from dislib_amd.cluster.dbscan import compute_neighbours
    from dislib_amd.data import load_data
    from dislib_amd.neighbors import NearestNeighbors
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    fit = load_data(torch.from_numpy(xf).to(dev), subset_size=a.subset)
    qry = load_data(torch.from_numpy(xq).to(dev), subset_size=a.subset)
    nn = NearestNeighbors(n_neighbors=a.kn)
    nn.fit(fit)
    nn.kneighbors(qry)                         # warm-up (uploads, JIT)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        nn.kneighbors(qry)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    pairs = float(a.nq) * a.nfit
    flops = 3.0 * a.d * pairs
    knn = {"workload": "kneighbors: %d queries x %d fit rows, d=%d, k=%d "
                       "(sklearn kd_tree regime)" % (a.nq, a.nfit, a.d, a.kn),
           "value": a.nq / t, "unit": "queries/s", "seconds": t,
           "pairs_per_s": pairs / t,
           "roofline": {"bound": "valu_fp64", "achieved": flops / t / 1e12,
                        "peak": FP64_VALU_PEAK / 2 / 1e12,
                        "unit": "T fp64 ops/s (sub, mul, add: one op each)",
                        "frac": flops / t / (FP64_VALU_PEAK / 2)},
           "includes": "device->host copy of the (nq x k) results"}
    if "knn" in cpu:
        knn["cpu_baseline"] = cpu["knn"]
        knn["gpu_over_cpu"] = knn["value"] / cpu["knn"]["value"]

    xe_d = torch.from_numpy(xe).to(dev)
    subs = list(load_data(xe_d, subset_size=a.subset))
    compute_neighbours(a.eps, 5, False, 0, a.eps_q, *subs)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        nl, _ = compute_neighbours(a.eps, 5, False, 0, a.eps_q, *subs)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    pairs = float(a.eps_q) * a.eps_n
    eps = {"workload": "DBSCAN epsilon query: %d queries x %d rows, d=%d, "
                       "eps=%g" % (a.eps_q, a.eps_n, a.d, a.eps),
           "value": a.eps_q / t, "unit": "queries/s", "seconds": t,
           "pairs_per_s": pairs / t,
           "neighbours": int(sum(len(v) for v in nl)),
           "includes": "two distance passes (count, fill), the sort, the "
                       "host prefix sum and the device->host copy of the "
                       "lists"}
    if "eps" in cpu:
        eps["cpu_baseline"] = cpu["eps"]
        eps["gpu_over_cpu"] = eps["value"] / cpu["eps"]["value"]
    sp_subs = list(load_data(xs, subset_size=a.subset))
    compute_neighbours(a.sp_eps, 5, True, 0, a.sp_q, *sp_subs)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        nl, _ = compute_neighbours(a.sp_eps, 5, True, 0, a.sp_q, *sp_subs)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    pairs = float(a.sp_q) * a.sp_n
    eps_csr = {"workload": "DBSCAN epsilon query, sparse: %d queries x %d "
                           "CSR rows, d=%d, %d nnz/row, eps=%g"
                           % (a.sp_q, a.sp_n, a.sp_d, a.sp_nnz, a.sp_eps),
               "value": a.sp_q / t, "unit": "queries/s", "seconds": t,
               "pairs_per_s": pairs / t,
               "neighbours": int(sum(len(v) for v in nl)),
               "includes": "host concatenation + upload of the CSR arrays, "
                           "two passes, the sort and the copy back"}
    if "eps_csr" in cpu:
        eps_csr["cpu_baseline"] = cpu["eps_csr"]
        eps_csr["gpu_over_cpu"] = eps_csr["value"] / cpu["eps_csr"]["value"]
    sp_fit = load_data(xs, subset_size=a.subset)
    sp_q = load_data(xs[:a.sp_kq], subset_size=a.subset)
    nn = NearestNeighbors(n_neighbors=a.kn)
    nn.fit(sp_fit)
    nn.kneighbors(sp_q)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        nn.kneighbors(sp_q)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    pairs = float(a.sp_kq) * a.sp_n
    knn_csr = {"workload": "kneighbors, sparse: %d queries x %d CSR rows, "
                           "d=%d, %d nnz/row, k=%d"
                           % (a.sp_kq, a.sp_n, a.sp_d, a.sp_nnz, a.kn),
               "value": a.sp_kq / t, "unit": "queries/s", "seconds": t,
               "pairs_per_s": pairs / t,
               "includes": "host concatenation + upload of both CSR "
                           "matrices, the partial lists, the merge and the "
                           "copy back"}
    if "knn_csr" in cpu:
        knn_csr["cpu_baseline"] = cpu["knn_csr"]
        knn_csr["gpu_over_cpu"] = knn_csr["value"] / cpu["knn_csr"]["value"]
    print(json.dumps({"kneighbors": knn, "epsilon_query": eps,
                      "epsilon_query_csr": eps_csr,
                      "kneighbors_csr": knn_csr}), flush=True)


if __name__ == "__main__":
    main()
