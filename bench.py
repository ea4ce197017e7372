"""Lloyd-iteration throughput of dislib_amd's KMeans on MI355X.

Workload (BASELINE.json configs[1]): KMeans k=100 on 100M x 32 fp64 dense
make_blobs data per GPU, synthetic, generated on the device by the library's
counter-based generator (100 blobs, centres U(-10,10), std 1), Subsets of 1M
rows, initial centres np.random.seed(0); np.random.random((k, d)).

A "step" is one Lloyd iteration over all resident samples: centre prep ->
fused assign + per-cluster sum/count (HIP) -> RCCL all-reduce of
[sums | counts] (N > 1) -> centre update + convergence criterion (HIP) ->
4-byte flag read.  Weak scaling: every rank owns n samples.

Prints ONE JSON line (rank 0) with metric/value/unit, the roofline of the
dominant kernel (dkm_partial_sum, timed with HIP events on its stream) and a
CPU baseline (the oracle, rank 0, N=1 only, bounded sample).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "KMeans samples·iters/sec at 1/2/4/8 GPUs + % of HBM/MFMA roofline"
HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3       # vector/matrix fp32 (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--n", type=int, default=100_000_000,
                   help="samples per GPU")
    p.add_argument("--d", type=int, default=32)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--subset", type=int, default=1_000_000)
    p.add_argument("--mode", default="auto")
    p.add_argument("--labels", action="store_true",
                   help="fit_predict (write labels) instead of fit")
    p.add_argument("--no-cpu", action="store_true",
                   help="skip the CPU baseline")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--traffic-json", default=os.path.join(
        ROOT, "profiles", "r01_traffic.json"))
    return p.parse_args()


def cpu_baseline(d, k, target_s, centers):
    """Oracle (numpy restatement of the reference, vectorised) on the host:
    one Lloyd iteration's partial sums, one task per Subset over a process
    pool, BLAS threads = 1.  Bounded sample sized for ~target_s seconds."""
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
    import multiprocessing as mp
    from oracle import kmeans_oracle as orc
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    # probe: single-core rate on a small block
    probe = 4000
    xb, _ = orc.make_blobs_rows(0, probe, d, k, seed=0)
    t0 = time.perf_counter()
    orc.partial_sum(xb, centers)
    rate1 = probe / (time.perf_counter() - t0)
    rows_per_task = 25_000
    n_tasks = max(cores, int(rate1 * cores * target_s / rows_per_task))
    tasks = [(i * rows_per_task, rows_per_task, d, k) for i in range(n_tasks)]
    ctx = mp.get_context("fork")
    with ctx.Pool(cores) as pool:
        pool.map(_cpu_gen, tasks[:cores])          # warm the workers
        blocks = pool.map(_cpu_gen, tasks)
        t0 = time.perf_counter()
        parts = pool.starmap(_cpu_task, [(b, centers) for b in blocks])
        root = orc.merge_tree(parts, 50)
        orc.recompute_centers(centers.copy(), root)
        el = time.perf_counter() - t0
    n = n_tasks * rows_per_task
    # faithful per-sample-loop variant (the reference's own cost model)
    xs, _ = orc.make_blobs_rows(0, 2000, d, k, seed=0)
    t0 = time.perf_counter()
    for s in xs:
        np.argmin(orc.vec_matrix_euclid(s, centers))
    faithful = 2000 / (time.perf_counter() - t0)
    return {"value": n / el, "unit": "samples·iters/s", "cores": cores,
            "kind": "port",
            "sample": "%d rows (%d Subsets of %d) of the same make_blobs "
                      "workload, one Lloyd iteration (distances+argmin+"
                      "sums+arity-50 merge), vectorised numpy oracle, one "
                      "process per core, BLAS threads 1" %
                      (n, n_tasks, rows_per_task),
            "seconds": el,
            "faithful_per_sample_loop_1core": faithful}


def _cpu_gen(args):
    from oracle import kmeans_oracle as orc
    row0, n, d, k = args
    return orc.make_blobs_rows(row0, n, d, k, seed=0)[0]


def _cpu_task(block, centers):
    from oracle import kmeans_oracle as orc
    _, s, c = orc.partial_sum(block, centers)
    return (s, c)


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    # CPU baseline first, before anything touches the GPU: its worker pool is
    # forked from a process with no HIP state and is gone before GPU init.
    cpu = None
    if world == 1 and not a.no_cpu:
        from dislib_amd.cluster.kmeans import _init_centers as _ic
        cpu = cpu_baseline(a.d, a.k, a.cpu_seconds, _ic(a.d, False, a.k, 0))

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from dislib_amd import _device, _lib
    from dislib_amd.cluster.kmeans import _Lloyd, _init_centers
    from dislib_amd.data import Dataset, Subset

    n, d, k = a.n, a.d, a.k
    X = torch.empty((n, d), dtype=torch.float64, device=dev)
    # global rows [rank*n, (rank+1)*n): the ranks shard one dataset
    _device.make_blobs(X, rank * n, k, seed=0, box=10.0, std=1.0)
    ds = Dataset(n_features=d)
    for i in range(0, n, a.subset):
        ds.append(Subset(X[i:i + a.subset]))
    centers0 = _init_centers(d, False, k, 0)
    st = _Lloyd(ds, centers0, 0.0, a.labels, a.mode, dev)
    torch.cuda.synchronize()

    for _ in range(a.warmup):
        st.step()

    ev = [(torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        st.prepare()
        ev[i][0].record()
        st.partial()                  # the dominant kernel(s), same stream
        ev[i][1].record()
        st.reduce_update()
        st.flag.item()                # the per-iteration convergence read
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    if world > 1:
        t = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern_ms = float(t[0]), float(t[1])
    rechecked = st.rechecked()

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    total = n * world * a.steps
    value = total / el
    bytes_per_launch = n * d * 8 + (n * 4 if a.labels else 0)
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    flops = 2.0 * k * d * n
    # HBM bytes per launch from the committed PMC passes (tools/pmc_session.sh
    # -> tools/pmc_summary.py --traffic-out), scaled to this launch's rows
    traffic = None
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            if tj.get("d") == d and tj.get("k") == k:
                traffic = n * (tj["hbm_read_bytes_per_sample"] +
                               tj["hbm_write_bytes_per_sample"])
        except (OSError, ValueError, KeyError):
            traffic = None
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "samples·iters/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": el / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (on-device counter-based make_blobs, 100 blobs)",
        "config": {"workload": "KMeans k=%d on %dM x %d fp64 dense per GPU "
                               "(BASELINE configs[1])" % (k, n // 10**6, d),
                   "n_per_gpu": n, "d": d, "k": k, "subset_size": a.subset,
                   "mode": a.mode, "labels": bool(a.labels),
                   "parallelism": "dp%d" % world},
        "roofline": {"bound": "hbm", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "dkm_partial_sum (k_screen + k_recheck)",
                     "kernel_ms": kern_ms,
                     "fp32_screen_tflops": flops / (kern_ms * 1e-3) / 1e12,
                     "fp32_peak_tflops": FP32_PEAK_TFLOPS},
        "rechecked_samples": rechecked,
    }
    if cpu is not None:
        cpu["gpu_over_cpu"] = value / cpu["value"]
        out["cpu_baseline"] = cpu
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
