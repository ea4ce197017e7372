"""Time the large-d assignment path (bf16x3 GEMM screen) on device data.

  python tools/bench_gemm.py [--n 1000000] [--d 1024] [--k 4096] [--reps 3]
                             [--centres data|init] [--f32]

Reports ms per dkm_partial_sum call, the executed bf16 MFMA rate
(3 products, or 1 with --mode bf16, x 2 k dpad flops per sample) against the 2.5 PF dense peak, and
the number of samples sent to the exact paths.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--d", type=int, default=1024)
    p.add_argument("--k", type=int, default=4096)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--centres", default="data", choices=["data", "init"])
    p.add_argument("--f32", action="store_true")
    p.add_argument("--mode", default="bf16x3", choices=["bf16x3", "bf16"])
    p.add_argument("--kind", default="partial",
                   choices=["partial", "predict", "delta"])
    a = p.parse_args()
    import torch
    from dislib_amd import _device, _lib
    from dislib_amd.data import Dataset, Subset
    dev = torch.device("cuda")
    n, d, k = a.n, a.d, a.k
    X = torch.empty((n, d), dtype=torch.float64, device=dev)
    _device.make_blobs(X, 0, k, seed=0, box=10.0, std=1.0)
    if a.f32:
        X = X.float()
    if a.centres == "init":
        np.random.seed(0)
        C = torch.from_numpy(np.random.random((k, d))).to(dev)
    else:
        g = torch.Generator(device="cpu").manual_seed(1)
        idx = torch.randperm(n, generator=g)[:k].to(dev)
        C = X[idx].double() + 0.5
    ds = Dataset(n_features=d)
    ds.append(Subset(X))
    dd = ds._device_data()
    ws = _device.Workspace(k, d, n, dev)
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    lab = torch.full((n,), -1, dtype=torch.int32, device=dev)
    m = _lib.MODE_BF16X3 if a.mode == "bf16x3" else _lib.MODE_BF16
    times = []
    for r in range(a.reps + 1):
        _device.prepare(C, ws, acc)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if a.kind == "partial":
            _device.partial_sum(dd, C, ws, lab, acc, m)
        elif a.kind == "predict":
            _device.predict(dd, C, ws, lab, m)
        else:
            _device.assign_delta(dd, C, ws, lab, acc, m)
        torch.cuda.synchronize()
        if r:
            times.append(time.perf_counter() - t0)
    ms = 1e3 * float(np.median(times))
    dpad = (d + 31) // 32 * 32
    kpad = (k + 255) // 256 * 256
    flops = (6.0 if a.mode == "bf16x3" else 2.0) * n * kpad * dpad
    out = {"n": n, "d": d, "k": k, "kind": a.kind, "f32": a.f32,
           "centres": a.centres, "ms": ms, "ms_all": [1e3 * t for t in times],
           "bf16_tflops": flops / ms * 1e-9,
           "frac_bf16_peak": flops / ms * 1e-9 / 2500.0,
           "alg_fp64_equiv_tflops": 2.0 * n * k * d / ms * 1e-9,
           "rechecked_total": _device.rechecked(ws)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
