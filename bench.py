"""Lloyd-iteration throughput of dislib_amd's KMeans on MI355X.

Headline workload (BASELINE.json configs[1], the metric's config): KMeans
k=100 on 100M x 32 fp64 dense make_blobs data per GPU, synthetic, generated
on the device by the library's counter-based generator (k blobs, centres
U(-10,10), std 1), Subsets of 1M rows, initial centres
np.random.seed(0); np.random.random((k, d)).

A "step" is one Lloyd iteration over all resident samples: centre prep ->
fused assign + per-cluster sum/count (HIP) -> all-reduce of [sums | counts]
(RCCL through libdkm, N > 1) -> centre update + convergence criterion
(HIP) -> 4-byte flag read.  Weak scaling: every rank owns n samples.

Timing follows SURVEY 8(d): W warmup iterations run on a throwaway fit;
the K timed steps are ONE whole fit from the initial centres (iteration 0,
the image builds and the mass migration of iterations 1-2 included; tol =
0, so exactly K iterations), bracketed by barrier + synchronize.  `value` =
n x N x K / that wall time.  The steady-state figures (the fit's last
ceil(K/2) iterations) are reported beside it, never as `value`.

Prints ONE JSON line (rank 0): metric/value/unit for the headline config,
its roofline (the assignment call -- the dominant kernels -- timed with HIP
events on its stream over the timed fit, and over its steady iterations),
a CPU baseline (the oracle on this host, rank 0, N=1 only, bounded sample),
the fit_predict variant (labels written), per-iteration wall and kernel
times, and under "extra_configs" the other single-GPU BASELINE configs
measured the same way in the same run: configs[0] (C1), configs[2]'s
per-GPU shard (125M x 64, k=1000, the north-star target), configs[3] (10M
x 1024, k=4096, fp64 and fp32; MFMA) and configs[4] (CSR 10M x 10k, 10
entries per row, k=256: fit and predict).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--only-headline]
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
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6        # fp64 vector = matrix
L2_PEAK_TBS = 34.5             # aggregate L2 (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--n", "--rows", dest="n", type=int, default=100_000_000,
                   help="samples per GPU (headline config)")
    p.add_argument("--d", type=int, default=32)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--subset", type=int, default=1_000_000)
    p.add_argument("--mode", default="auto")
    p.add_argument("--labels", action="store_true",
                   help="headline = fit_predict (labels written)")
    p.add_argument("--only-headline", action="store_true",
                   help="skip the fit_predict and extra-config runs")
    p.add_argument("--no-cpu", action="store_true",
                   help="skip the CPU baselines")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--extras-scale", type=float, default=1.0,
                   help="scale the extra configs' rows per GPU (rehearsals "
                        "only; their lines then name the scaled size)")
    p.add_argument("--backend", default="nccl",
                   help="process-group backend for N > 1 (nccl = RCCL; gloo "
                        "only to rehearse several ranks on one GPU)")
    p.add_argument("--traffic-json", default=None,
                   help="PMC traffic summary for the headline (default: "
                        "profiles/traffic/d<d>_k<k>.json when present)")
    return p.parse_args()


# ---------------------------------------------------------------------------
# CPU baseline: the oracle (numpy restatement of the reference, pinned to the
# reference's golden vectors) timed on this host
# ---------------------------------------------------------------------------
def cpu_share():
    """Worker processes for the CPU baseline: the CPU share the GPU box
    grants this job (OMP_NUM_THREADS, 16 per GPU there) within the
    affinity mask; the whole machine's thread count is reported beside."""
    aff = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS", "")
    share = int(env) if env.isdigit() and int(env) > 0 else aff
    return max(1, min(share, aff)), aff


def progress(msg):
    """One line per stage on stderr (long runs: the log keeps growing)."""
    sys.stderr.write("bench [%s] %s\n" % (time.strftime("%H:%M:%S"), msg))
    sys.stderr.flush()


def cpu_baseline(d, k, target_s, centers, n_blobs, share, csr_nnz=0):
    """One Lloyd iteration's partial sums on a bounded sample of the same
    workload, one Subset per task over a process pool of `share` = (cores,
    machine threads) workers (BLAS threads 1), then the arity-50 merge and
    the centre update -- the reference's task graph (base.py:113-147) run
    by the vectorised oracle.  csr_nnz > 0: CSR rows of the C5 generator
    (the oracle's sklearn-order sparse distances, base.py:169)."""
    cores, machine = share
    progress("cpu baseline d=%d k=%d nnz=%d" % (d, k, csr_nnz))
    os.environ["OMP_NUM_THREADS"] = "1"        # BLAS threads of the workers
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    import multiprocessing as mp
    from oracle import kmeans_oracle as orc
    sparse = csr_nnz > 0
    # probe: single-core rate on a small block (smaller for large k*d)
    probe = 500 if sparse else int(max(16, min(4000, 3e8 / (k * d))))
    xb = _cpu_gen((0, probe, d, n_blobs, csr_nnz))
    t0 = time.perf_counter()
    orc.partial_sum(xb, centers, sparse=sparse)
    rate1 = probe / (time.perf_counter() - t0)
    rows_per_task = int(max(16, min(2000 if sparse else 25_000,
                                    rate1 * 0.5)))
    n_tasks = max(cores, int(rate1 * cores * target_s / rows_per_task))
    tasks = [(i * rows_per_task, rows_per_task, d, n_blobs, csr_nnz)
             for i in range(n_tasks)]
    ctx = mp.get_context("fork")
    with ctx.Pool(cores) as pool:
        pool.map(_cpu_gen, tasks[:cores])          # warm the workers
        blocks = pool.map(_cpu_gen, tasks)
        t0 = time.perf_counter()
        parts = pool.starmap(_cpu_task, [(b, centers, sparse)
                                         for b in blocks])
        root = orc.merge_tree(parts, 50)
        orc.recompute_centers(centers.copy(), root, sparse=sparse)
        el = time.perf_counter() - t0
    n = n_tasks * rows_per_task
    out = {"value": n / el, "unit": "samples·iters/s", "cores": cores,
           "kind": "port",
           "sample": "%d rows (%d Subsets of %d) of the same %s workload, "
                     "one Lloyd iteration (distances+argmin+sums+arity-50 "
                     "merge), vectorised numpy oracle, one process per core "
                     "of this job's CPU share, BLAS threads 1" %
                     (n, n_tasks, rows_per_task,
                      "CSR" if sparse else "make_blobs"),
           "seconds": el,
           "per_core": n / el / cores,
           "machine_threads": machine,
           "note": "cores = the CPU share the GPU box grants one GPU's job "
                   "(OMP_NUM_THREADS = 16; the harness caps a job's worker "
                   "pools at that share, not the %d-thread affinity mask); "
                   "the oracle scales linearly over Subsets, so per_core x "
                   "machine_threads bounds a whole-machine run" % machine}
    if not sparse:
        # faithful per-sample-loop variant (the reference's own cost model)
        m = int(max(4, min(2000, rate1 * 0.02)))
        xs = _cpu_gen((0, m, d, n_blobs, 0))
        t0 = time.perf_counter()
        for row in xs:
            np.argmin(orc.vec_matrix_euclid(row, centers))
        out["faithful_per_sample_loop_1core"] = \
            m / (time.perf_counter() - t0)
    return out


def csr_rows(row0, n, d, nnz, seed=0):
    """C5 rows [row0, row0 + n): nnz strictly increasing random columns of
    d per row, values U(0, 1); counter-based per row block so that any
    range regenerates identically (host numpy, scipy CSR)."""
    import scipy.sparse as sp
    rng = np.random.default_rng([seed, row0, n])
    gap = max(1, d // nnz - 1)
    cols = np.cumsum(rng.integers(1, gap + 1, (n, nnz)), axis=1) - 1
    indptr = np.arange(0, n * nnz + 1, nnz, dtype=np.int64)
    data = rng.random(n * nnz)
    return sp.csr_matrix((data, cols.reshape(-1).astype(np.int32), indptr),
                         shape=(n, d))


def _cpu_gen(args):
    from oracle import kmeans_oracle as orc
    row0, n, d, nb, nnz = args
    if nnz:
        return csr_rows(row0, n, d, nnz, seed=1)
    return orc.make_blobs_rows(row0, n, d, nb, seed=0)[0]


def _cpu_task(block, centers, sparse=False):
    from oracle import kmeans_oracle as orc
    _, s, c = orc.partial_sum(block, centers, sparse=sparse)
    return (s, c)


# ---------------------------------------------------------------------------
# one configuration on the GPU(s)
# ---------------------------------------------------------------------------
def run_config(torch, dist, dev, rank, world, n, d, k, subset, steps, warmup,
               mode, labels, n_blobs=None, f32=False, csr_nnz=0, host_x=None):
    """One configuration, timed as SURVEY 8(d) defines the metric: the wall
    time of a whole Lloyd loop, from after the data is resident and the
    centres are initialised through the last convergence decision.

    * W warmup iterations of a throwaway fit on the same resident data (code
      objects, allocator); its sample images are then dropped, so the timed
      fit builds every image it uses, as a first fit on a dataset does;
    * the timed fit: a fresh fit state from the initial centres, then exactly
      K iterations with tol = 0 (barrier + synchronize on both sides), so
      iteration 0 -- the most expensive one -- is inside the timed region;
    * per iteration: HIP events around the assignment call (the dominant
      kernels, on their stream) and the host clock after the iteration's
      flag read (the per-iteration sync), so every iteration's wall time and
      kernel time are reported; the "steady" figures are the last ceil(K/2)
      iterations of the same fit;
    * every workspace / image allocation's host time (_device.ALLOC_LOG)."""
    progress("gpu n=%d d=%d k=%d steps=%d warmup=%d%s" % (
        n, d, k, steps, warmup, " csr" if csr_nnz else ""))
    from dislib_amd import _device, _shard
    from dislib_amd.cluster.kmeans import _Lloyd, _init_centers
    from dislib_amd.data import Dataset, Subset
    n_blobs = n_blobs or k
    tp0 = time.perf_counter()
    if host_x is not None:
        # C1: the reference's own make_blobs (host numpy), rank's slice
        X = torch.from_numpy(np.ascontiguousarray(
            host_x[rank * n:(rank + 1) * n])).to(dev)
        C0 = _init_centers(d, False, k, 0)
    elif csr_nnz:
        # global rows [rank*n, (rank+1)*n): the ranks shard one dataset
        X = csr_rows(rank * n, n, d, csr_nnz, seed=1)
        C0 = _init_centers(d, True, k, 0).toarray()
    else:
        X = torch.empty((n, d), dtype=torch.float64, device=dev)
        _device.make_blobs(X, rank * n, n_blobs, seed=0, box=10.0, std=1.0)
        if f32:              # fp32 samples: fp64 distances, fp32 sums
            X = X.to(torch.float32)
            torch.cuda.empty_cache()
        C0 = _init_centers(d, False, k, 0)
    ds = Dataset(n_features=d, sparse=bool(csr_nnz))
    for i in range(0, n, subset):
        ds.append(Subset(X[i:i + subset]))
    dd = ds._device_data(dev)             # resident before the fit starts
    torch.cuda.synchronize()
    phases = {"data_s": time.perf_counter() - tp0}
    del _device.ALLOC_LOG[:]
    # warmup: a throwaway fit of W iterations
    tw = time.perf_counter()
    if warmup > 0:
        st = _Lloyd(ds, C0, 0.0, labels, mode, dev)
        for _ in range(warmup):
            st.step()
        torch.cuda.synchronize()
        del st
    dd.drop_images()
    phases["warmup_fit_s"] = time.perf_counter() - tw
    ts = time.perf_counter()
    st = _Lloyd(ds, C0, 0.0, labels, mode, dev)
    torch.cuda.synchronize()
    phases["fit_state_s"] = time.perf_counter() - ts
    ev = [(torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    wall = []
    nlog = len(_device.ALLOC_LOG)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tl = t0
    for i in range(steps):
        st.prepare()
        ev[i][0].record()
        st.partial()                  # the dominant kernel(s), same stream
        ev[i][1].record()
        st.reduce_update()
        st.read_flags()               # the per-iteration convergence read
        tn = time.perf_counter()
        wall.append(tn - tl)
        tl = tn
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern = [s.elapsed_time(e) for s, e in ev]
    ns = (steps + 1) // 2                 # the steady iterations: the last half
    kern_ms = float(np.mean(kern))
    steady_kern_ms = float(np.mean(kern[-ns:]))
    steady_ms = float(np.mean(wall[-ns:])) * 1e3
    phases["fit_allocs"] = [{"what": w, "bytes": b, "s": round(s, 6)}
                            for w, b, s in _device.ALLOC_LOG[nlog:]]
    phases["warmup_allocs_s"] = round(sum(s for _, _, s in
                                          _device.ALLOC_LOG[:nlog]), 6)
    pred_ms = None
    if csr_nnz:                       # predict on the final centres
        from dislib_amd import _lib
        lab = torch.empty(st.dd.n, dtype=torch.int32, device=dev)
        _device.predict(st.dd, st.C, st.ws, lab, _lib.MODE_AUTO)
        torch.cuda.synchronize()
        tp = time.perf_counter()
        for _ in range(3):
            _device.predict(st.dd, st.C, st.ws, lab, _lib.MODE_AUTO)
        torch.cuda.synchronize()
        pred_ms = (time.perf_counter() - tp) / 3 * 1e3
        del lab
    if world > 1:
        t = torch.tensor([el, kern_ms, steady_kern_ms, steady_ms],
                         dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern_ms, steady_kern_ms, steady_ms = (float(x) for x in t)
    info = _shard.comm_info(dev.index) if world > 1 else None
    out = {"el": el, "kern_ms": kern_ms, "steady_kern_ms": steady_kern_ms,
           "steady_ms": steady_ms, "steady_iters": ns,
           "iter_ms": [round(w * 1e3, 3) for w in wall],
           "iter_kern_ms": [round(x, 3) for x in kern],
           "phases": phases, "rechecked": st.rechecked(),
           "pred_ms": pred_ms,
           "collective": ("libdkm-rccl" if info else "torch.distributed")
           if world > 1 else "none",
           "rccl_ranks": info[0] if info else None,
           # the sample image the screen streamed: the fit's label-sorted
           # image (3), else the dataset's cached one (dkm_x_image_*), if any
           "image_kind": 3 if getattr(st, "simg", None) is not None else
           (max(st.dd.images) if getattr(st.dd, "images", None) else 0),
           # single-product screen counters (threshold tiles, decided,
           # centre blocks screened over the sorted image), whole fit
           "counters": st.screened_blocks() if not csr_nnz and
           getattr(st, "sorting", False) else None,
           "nkb": (k + 31) // 32}
    del st, ds, X, dd
    torch.cuda.empty_cache()
    return out


def traffic_for(n, d, k, path=None, csr_nnz=0):
    """HBM bytes per assignment call from the committed PMC passes
    (tools/pmc_session.sh -> tools/pmc_summary.py --traffic-out): the
    per-sample read + write bytes of the screen and re-check kernels,
    scaled to n; None when no summary for this (d, k) is committed."""
    path = path or os.path.join(ROOT, "profiles", "traffic",
                                ("csr%d_" % csr_nnz if csr_nnz else "") +
                                "d%d_k%d.json" % (d, k))
    try:
        tj = json.load(open(path))
        if tj.get("d") == d and tj.get("k") == k:
            return n * (tj["hbm_read_bytes_per_sample"] +
                        tj["hbm_write_bytes_per_sample"])
    except (OSError, ValueError, KeyError):
        pass
    return None


def skip_fields(r):
    """Block skipping over the label-sorted image: the
    fraction of (tile, 32-centre block) pairs the threshold passes of the
    whole fit screened."""
    c = r.get("counters")
    if not c or not c[0]:
        return None
    return {"threshold_tiles": c[0], "tiles_decided": c[1],
            "blocks_screened": c[2],
            "screened_frac": c[2] / (c[0] * r["nkb"])}


def fit_fields(r, n, world):
    """Per-iteration record of the timed fit (K iterations from
    the initial centres, tol = 0): wall time per iteration (host clock after
    each flag read), assignment-kernel time per iteration (HIP events), the
    steady figure (the fit's last ceil(K/2) iterations) and the host-side
    phases (data generation, warmup fit, fit-state setup, allocations)."""
    return {"iter_ms": r["iter_ms"], "iter_kernel_ms": r["iter_kern_ms"],
            "steady_ms_per_step": r["steady_ms"],
            "steady_value": n * world / (r["steady_ms"] * 1e-3),
            "phases": r["phases"]}


def screen_products(k, d):
    """bf16 MFMA products per term of the d <= 128 screen auto mode runs
    (dkm_dense.hip `assign`: the single-product screen when k x d sums do
    not fit an 80 KB LDS budget beside the fragments; bf16x3 otherwise)."""
    lds_stride = d if d % 2 else d + 1
    frags = ((k + 31) // 32) * (4096 + 128) if d <= 32 else \
        ((k + 15) // 16) * (((d + 31) // 32) * 2048 + 64)
    return 3 if frags + (k * lds_stride + k) * 8 <= 80 * 1024 else 1


def roofline(n, d, k, r, labels, es=8, csr_nnz=0, traffic=None):
    """Roofline of the assignment call (the dominant kernels), timed with
    HIP events on its stream over the timed fit (`kernel_ms`: the mean over
    its K iterations, iteration 0 included -- the SURVEY 8(d) loop), with
    `step_frac` the same work over the fit's wall time per iteration and
    `steady` the same figures over the fit's last ceil(K/2) iterations.

    * d <= 128: HBM-bound on the algorithmic bytes, the X read (es d per
      sample);
    * d > 128: MFMA-bound, the executed flops of the single-product GEMM
      screen (2 k d per sample over the padded tiles) against the dense bf16
      peak;
    * CSR (C5): the HBM bytes of the rows (12 B per stored entry + 8 B of
      indptr + 8 B of labels); the gather of bf16 centre columns from L2
      (2 B per stored entry and centre) beside it.
    `traffic` (PMC bytes per steady launch, profiles/traffic/) gives
    `steady.physical`."""
    sec = r["kern_ms"] * 1e-3
    step_sec = r["el"] / len(r["iter_ms"])
    st_sec = r["steady_kern_ms"] * 1e-3
    st_step = r["steady_ms"] * 1e-3
    if csr_nnz:
        work = n * (12 * csr_nnz + 8 + 8)
        g = n * csr_nnz * k * 2
        out = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
               "bytes_per_sample": 12 * csr_nnz + 16,
               "kernel": "dkm_assign_delta_csr / dkm_partial_sum_csr (screen "
                         "+ merge + resolve)",
               "l2_gather": {"bytes_per_sample": csr_nnz * k * 2,
                             "table": "bf16 C^T (d x k)",
                             "achieved_tbs": g / st_sec / 1e12,
                             "peak_tbs": L2_PEAK_TBS,
                             "frac": g / st_sec / 1e12 / L2_PEAK_TBS,
                             "note": "steady launches"}}
        scale, peak = 1e9, HBM_PEAK_GBS
    elif d <= 128:
        # the fit streams X once per iteration, es * d bytes
        # per sample (the labels the delta path reads and writes are not
        # counted)
        work = n * es * d
        ik = r.get("image_kind", 0)
        # bytes the screen actually streams per sample: the resident bf16
        # image (SPLIT: hi + lo, 4 KB per 32-row tile; SINGLE: 1 KB per
        # 16-feature K-step per tile) + fp32 |x|^2, or X itself; + labels
        if ik == 2:
            sb = 4096 // 32 + 4 + 8
        elif ik == 1:
            sb = (d + 15) // 16 * 1024 // 32 + 4 + 8
        elif ik == 3:          # + the row's sample index and label copy
            sb = (d + 15) // 16 * 1024 // 32 + 4 + 8 + 4
        else:
            sb = es * d + 8
        out = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
               "bytes_per_sample": es * d,
               "kernel": "dkm_assign_delta / dkm_partial_sum (screen + "
                         "re-check + sums)",
               # MFMA products per x.c term of the steady screen: bf16x3 (3)
               # when the fp64 sums fit LDS beside the centre fragments,
               # else the single-product screen (1)
               "mfma_products": screen_products(k, d),
               "image": {0: "none (X converted in the screen)",
                         1: "bf16 single (resident, built in the fit)",
                         2: "bf16 hi+lo split (resident, built in the "
                            "fit)",
                         3: "bf16 single, rows grouped by label (built in "
                            "the fit; block skipping)"}[ik],
               "streamed_bytes_per_sample": sb}
        scale, peak = 1e9, HBM_PEAK_GBS
    else:
        # auto mode runs the single-product GEMM screen (bf16 hi x hi on
        # hi-only tiles, features padded to 32) in the steady iterations
        dp, kp = (d + 31) // 32 * 32, (k + 255) // 256 * 256
        work = 2.0 * kp * dp * n
        out = {"bound": "mfma", "unit": "TFLOP/s", "peak": BF16_PEAK_TFLOPS,
               "flops_per_sample": 2.0 * kp * dp,
               "kernel": "dkm_assign (single-product bf16 GEMM screen + "
                         "exact candidates + sums)",
               "mfma_products": 1,
               "image": ("bf16 GEMM tiles (resident, built in the fit)"
                         if r.get("image_kind", 0) == 4 else
                         "none (X split per chunk on a second stream)")}
        scale, peak = 1e12, BF16_PEAK_TFLOPS

    def rate(s):
        return work / s / scale

    out.update({"achieved": rate(sec), "frac": rate(sec) / peak,
                "kernel_ms": r["kern_ms"],
                "step_frac": rate(step_sec) / peak,
                "timed": "mean over the K iterations of the timed fit "
                         "(iteration 0 included)"})
    st = {"iterations": r["steady_iters"], "kernel_ms": r["steady_kern_ms"],
          "achieved": rate(st_sec), "frac": rate(st_sec) / peak,
          "ms_per_step": r["steady_ms"], "step_frac": rate(st_step) / peak}
    if traffic:
        st["physical"] = {"hbm_bytes_per_sample": traffic / n,
                          "achieved_gbs": traffic / st_sec / 1e9,
                          "frac": traffic / st_sec / 1e9 / HBM_PEAK_GBS,
                          "note": "PMC FETCH_SIZE x2 + WRITE_SIZE (gfx950 "
                                  "correction) per steady launch, "
                                  "profiles/traffic/"}
    if d <= 128 and not csr_nnz:
        ik = out["streamed_bytes_per_sample"]
        st["streamed_gbs"] = n * ik / st_sec / 1e9
        st["streamed_frac"] = n * ik / st_sec / 1e9 / HBM_PEAK_GBS
        st["mfma_bf16_tflops_executed"] = \
            2.0 * screen_products(k, d) * k * d * n / st_sec / 1e12
    out["steady"] = st
    out["traffic"] = traffic
    out["binding"] = binding_for(d, k, csr_nnz)
    return out


def binding_for(d, k, csr_nnz):
    """The resource that actually limits the steady dominant kernel, from
    the PMC passes committed under profiles/ (DESIGN.md 5): the algorithmic
    `frac` prices fp64 X bytes or executed MFMA flops, which the screens
    that read a resident bf16 image do not stream."""
    if csr_nnz:
        return ("latency of the bf16 C^T gathers: k_csr_screen waits "
                "(SQ_WAIT_ANY) 70% of its wave cycles at 8 waves per SIMD "
                "with 96% L2 hits; neither HBM nor L2 bandwidth saturates "
                "(profiles/r05/pmc/c5_csr_pmc_summary_10M_bf16.txt)")
    if d > 128:
        return ("the LDS-read + MFMA loop of k_gemm_screen1: 2 waves per "
                "SIMD, SQ_WAIT_INST_ANY 38% of wave cycles, 1.7x the "
                "algorithmic HBM bytes "
                "(profiles/r05/pmc/c4_pmc_summary_10M.txt)")
    if k * d > 32 * 128:
        return ("instruction issue of k_screen_sorted over the label-sorted "
                "image: VALU:MFMA 7.4:1, SALU 6 per MFMA, SQ_WAIT_ANY 35% "
                "and SQ_WAIT_INST_ANY 28% of wave cycles; 173 B/sample of "
                "HBM traffic per steady iteration "
                "(profiles/r06/pmc/c3_pmc_summary_20M.txt)")
    return ("instruction issue of k_screen_w32 over the split image: "
            "VALU:MFMA 13.4:1, SQ_WAIT_ANY 47% of wave cycles; 143 "
            "B/sample of HBM traffic per steady iteration, streamed at "
            "about half of HBM (profiles/r06/pmc/c2_pmc_summary_20M.txt)")


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    sc = a.extras_scale
    extras = [] if a.only_headline else [
        # (name, n, d, k, subset, steps, warmup, fp32 samples, csr nnz/row);
        # steps = the SURVEY 8(d) iteration count of the config (C1 10, C3
        # 10, C4 5, C5 5): the timed fit is that whole Lloyd loop
        ("KMeans k=10 on 100k x 50 fp64 make_blobs per GPU (BASELINE "
         "configs[0], the reference's CPU-runnable parity case)", 100_000,
         50, 10, 10_000, 10, 2, False, "c1"),
        ("KMeans k=1000 on 125M x 64 fp64 dense per GPU (BASELINE "
         "configs[2] per-GPU shard; north-star target)",
         125_000_000, 64, 1000, 1_000_000, 10, 2, False, 0),
        ("KMeans k=4096 on 10M x 1024 fp64 dense per GPU (BASELINE "
         "configs[3], MFMA-bound)", 10_000_000, 1024, 4096, 1_000_000, 5, 1,
         False, 0),
        ("KMeans k=4096 on 10M x 1024 fp32 dense per GPU (BASELINE "
         "configs[3], fp32 variant reported separately)", 10_000_000, 1024,
         4096, 1_000_000, 5, 1, True, 0),
        ("KMeans k=256 on sparse CSR 10M x 10k at 0.1% density per GPU "
         "(BASELINE configs[4], fit + predict)", 10_000_000, 10_000, 256,
         1_000_000, 5, 1, False, 10),
    ]

    # CPU baselines first, before anything touches the GPU: their worker
    # pools are forked from a process with no HIP state and are gone before
    # GPU init.
    cpu = {}
    if world == 1 and not a.no_cpu:
        from dislib_amd.cluster.kmeans import _init_centers as _ic
        share = cpu_share()       # before the workers' BLAS settings below
        cpu["head"] = cpu_baseline(a.d, a.k, a.cpu_seconds,
                                   _ic(a.d, False, a.k, 0), a.k, share)
        for i, (_, n, d, k, *_r, f32, nnz) in enumerate(extras):
            if f32:
                continue          # the fp64 line's baseline covers the shape
            nz = 0 if nnz == "c1" else nnz
            cpu[i] = cpu_baseline(d, k, a.cpu_seconds / (4 if nnz == "c1"
                                                         else 2),
                                  _ic(d, bool(nz), k, 0), k, share,
                                  csr_nnz=nz)

    import torch
    import torch.distributed as dist

    from dislib_amd import _lib
    build_flags = int(_lib.load().dkm_build_flags())
    # one rank per GPU; a rehearsal with more ranks than GPUs (gloo) shares
    ndev = max(1, torch.cuda.device_count())
    torch.cuda.set_device(local % ndev)
    dev = torch.device("cuda", local % ndev)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.backend)

    def check_collective(r):
        # under nccl the Lloyd loop's all-reduce must be libdkm's RCCL
        # communicator over all ranks, never the silent torch fallback
        if world > 1 and a.backend == "nccl" and (
                r["collective"] != "libdkm-rccl" or r["rccl_ranks"] != world):
            sys.stderr.write("bench: collective %s over %s ranks, expected "
                             "libdkm-rccl over %d\n" % (
                                 r["collective"], r["rccl_ranks"], world))
            raise SystemExit(3)

    r = run_config(torch, dist, dev, rank, world, a.n, a.d, a.k, a.subset,
                   a.steps, a.warmup, a.mode, a.labels)
    check_collective(r)
    fp = None
    if not a.only_headline and not a.labels:
        fp = run_config(torch, dist, dev, rank, world, a.n, a.d, a.k,
                        a.subset, a.steps, a.warmup, a.mode, True)
    ex = []
    for i, (name, n, d, k, sub, steps, warm, f32, nnz) in enumerate(extras):
        hx = None
        if nnz == "c1":
            from sklearn.datasets import make_blobs
            hx = make_blobs(n_samples=n * world, n_features=d, centers=k,
                            cluster_std=1.0, random_state=0)[0]
            nnz = 0
        elif sc != 1.0:
            n = max(sub, int(n * sc) // sub * sub)
            name += " [scaled to %d rows per GPU]" % n
        rr = run_config(torch, dist, dev, rank, world, n, d, k, sub, steps,
                        warm, a.mode, False, f32=f32, csr_nnz=nnz, host_x=hx)
        check_collective(rr)
        e = {"workload": name, "n_per_gpu": n, "d": d, "k": k,
             "dtype": "f32 samples (f64 distances)" if f32 else "f64",
             "value": n * world * steps / rr["el"],
             "unit": "samples·iters/s", "ms_per_step": rr["el"] / steps * 1e3,
             "steps": steps, "warmup": warm,
             "roofline": roofline(n, d, k, rr, False, 4 if f32 else 8,
                                  csr_nnz=nnz, traffic=None if f32 else
                                  traffic_for(n, d, k, csr_nnz=nnz)),
             "rechecked_samples": rr["rechecked"],
             "block_skip": skip_fields(rr)}
        e.update(fit_fields(rr, n, world))
        if nnz:
            e["nnz_per_row"] = nnz
            e["predict_ms"] = rr["pred_ms"]
            e["predict_samples_per_s"] = n / (rr["pred_ms"] * 1e-3)
        if world > 1:
            e["rccl_ranks"] = rr["rccl_ranks"]
        ci = i if i in cpu else (i - 1 if f32 and (i - 1) in cpu else None)
        if ci is not None:
            cb = dict(cpu[ci])
            if ci != i:     # fp32 samples: the same fp64-distance arithmetic
                cb["note"] = ("the fp64 line's measurement: the reference's "
                              "fp32 path computes the same fp64 distances "
                              "(base.py:204-205 on fp32 rows upcast)")
            cb["gpu_over_cpu"] = e["value"] / cb["value"]
            e["cpu_baseline"] = cb
        ex.append(e)

    if rank != 0:
        from dislib_amd import _shard
        _shard.finalize()
        if world > 1:
            dist.destroy_process_group()
        return

    value = a.n * world * a.steps / r["el"]
    rf = roofline(a.n, a.d, a.k, r, a.labels,
                  traffic=traffic_for(a.n, a.d, a.k, a.traffic_json))
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "samples·iters/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": r["el"] / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (on-device counter-based make_blobs, k blobs)",
        "config": {"workload": "KMeans k=%d on %dM x %d fp64 dense per GPU "
                               "(BASELINE configs[1]); timed = one whole "
                               "Lloyd loop of `steps` iterations from the "
                               "initial centres, tol = 0 (SURVEY 8(d))" % (
                                   a.k, a.n // 10**6, a.d),
                   "n_per_gpu": a.n, "d": a.d, "k": a.k,
                   "subset_size": a.subset, "mode": a.mode,
                   "labels": bool(a.labels),
                   "parallelism": "dp%d" % world},
        "roofline": rf,
        "rechecked_samples": r["rechecked"],
        "block_skip": skip_fields(r),
        "collective": r["collective"],
    }
    out.update(fit_fields(r, a.n, world))
    if world > 1:
        out["rccl_ranks"] = r["rccl_ranks"]
    if build_flags:
        out["timing_only_build"] = build_flags   # A/B probe library
    if fp is not None:
        out["fit_predict"] = {
            "value": a.n * world * a.steps / fp["el"],
            "ms_per_step": fp["el"] / a.steps * 1e3,
            "roofline": roofline(a.n, a.d, a.k, fp, True)}
    if "head" in cpu:
        cpu["head"]["gpu_over_cpu"] = value / cpu["head"]["value"]
        out["cpu_baseline"] = cpu["head"]
    if ex:
        out["extra_configs"] = ex
    print(json.dumps(out), flush=True)
    from dislib_amd import _shard
    _shard.finalize()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
