"""One rank of a multi-process KMeans fit on the GPU, started by
tests/test_gpu_dist.py through torch.distributed.run (not a test module).

Every rank builds the same seeded dataset, takes its contiguous block of
Subsets (``shard_dataset``), runs the product ``KMeans.fit_predict`` (HIP
kernels, per-iteration all-reduce of [sums | counts]) and writes its
centres, n_iter, labels and initial centres to ``<out>.<rank>.npz``.
With ``--backend gloo`` (the default) every rank shares cuda:0 (RCCL
refuses two ranks on one device) and the collective is the same ``_shard``
entry point the ``nccl`` path takes.  With ``--backend nccl`` rank r runs on
cuda:r and the per-iteration all-reduce goes through libdkm's own RCCL
communicator (dkm_allreduce_*); the rank records its (nranks, rank) as
that communicator reports them.

  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1
      --master-port P tests/dist_worker.py --case NAME --out PREFIX
      [--backend nccl]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = {
    # name: (n, d, blobs, k, subset, max_iter, tol, random_state, refresh)
    "dense": (24000, 16, 12, 12, 1000, 12, 0.0, 0, 3),
    "gemm": (6000, 200, 20, 40, 500, 4, 0.0, 3, 2),
    "none": (9000, 8, 6, 6, 1000, 8, 1e-6, None, 8),
    "ragged": (7001, 24, 9, 9, 700, 5, 0.0, 5, 8),
    # k x d sums beyond LDS: the single-product screen with label hints
    # (k_screen_b2) on both ranks, delta sums, refresh every 3
    "b2": (24000, 64, 200, 200, 2000, 6, 0.0, 0, 3),
    # CSR Subsets (the sparse screen + exact resolve), 10 entries per row
    "csr": (2000, 300, 0, 8, 250, 4, 0.0, 2, 2),
    # world 4 (LAYOUT: Subset sizes instead of `subset`): ragged Subsets;
    # 3 Subsets over 4 ranks (rank 0 -- whose REFRESH and initial centres
    # win -- owns no rows and still joins every all-reduce); the
    # single-product screen with the per-rank label-sorted image
    "ragged4": (7001, 24, 9, 9, 0, 6, 0.0, 5, 2),
    "empty4": (9500, 16, 12, 12, 0, 8, 0.0, 1, 3),
    "sorted4": (24000, 64, 200, 200, 0, 8, 0.0, 0, 3),
}
LAYOUT = {
    "ragged4": [700, 1300, 50, 2100, 900, 1, 1600, 350],
    "empty4": [3000, 2500, 4000],
    "sorted4": [5000, 7000, 3000, 9000],
}


def subsets(case):
    """[(row0, row1)] of the case's Subsets."""
    n, sub = CASES[case][0], CASES[case][4]
    sizes = LAYOUT.get(case) or [min(sub, n - i) for i in range(0, n, sub)]
    assert sum(sizes) == n
    edges = np.concatenate([[0], np.cumsum(sizes)])
    return [(int(a), int(b)) for a, b in zip(edges[:-1], edges[1:])]


def data(case):
    from sklearn.datasets import make_blobs
    n, d, blobs = CASES[case][:3]
    if case == "csr":
        import scipy.sparse as sp
        rng = np.random.default_rng(11)
        cols = np.sort(np.stack([rng.choice(d, 10, replace=False)
                                 for _ in range(n)]), axis=1)
        indptr = np.arange(0, 10 * n + 1, 10)
        return sp.csr_matrix((rng.random(10 * n), cols.reshape(-1),
                              indptr), shape=(n, d))
    x, _ = make_blobs(n_samples=n, n_features=d, centers=blobs,
                      center_box=(-8, 8), random_state=42)
    return x


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--case", required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--backend", default="gloo")
    a = p.parse_args()
    import torch
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    dev = rank if a.backend == "nccl" else 0
    torch.cuda.set_device(dev)
    if a.backend == "nccl":
        dist.init_process_group("nccl",
                                device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group("gloo")
    import dislib_amd.cluster.kmeans as km_mod
    from dislib_amd import shard_dataset
    from dislib_amd.cluster import KMeans
    from dislib_amd.data import Dataset, Subset
    n, d, blobs, k, sub, iters, tol, rs, refresh = CASES[a.case]
    km_mod.REFRESH = refresh if rank == 0 else 1000   # rank 0's value wins
    init = {}
    orig = km_mod._init_centers

    def rec(*args):
        c = orig(*args)
        init["c"] = np.array(c.toarray() if hasattr(c, "toarray") else c)
        return c
    km_mod._init_centers = rec
    x = data(a.case)
    full = Dataset(n_features=d, sparse=a.case == "csr")
    for lo, hi in subsets(a.case):
        full.append(Subset(x[lo:hi]))
    ds = shard_dataset(full)
    km = KMeans(n_clusters=k, max_iter=iters, tol=tol, random_state=rs)
    km.fit_predict(ds)
    cen = km.centers.toarray() if hasattr(km.centers, "toarray") else \
        km.centers
    from dislib_amd import _shard
    info = _shard.comm_info(dev) if a.backend == "nccl" else None
    lab = ds.labels_int32()
    np.savez("%s.%d.npz" % (a.out, rank), centers=cen,
             n_iter=km.n_iter, init=init["c"], nrows=np.array(
                 sum(s.samples.shape[0] for s in ds)),
             labels=lab if lab is not None else np.zeros(0, np.int32),
             refresh=np.array(km_mod.REFRESH),
             comm=np.array(info if info else (0, -1)))
    dist.barrier()
    _shard.finalize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
