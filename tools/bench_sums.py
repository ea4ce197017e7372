"""Time dkm_label_sums (counting sort by label + segmented sums) on fp64 and
fp32 copies of the same rows, with labels in row order (sequential reads)
or random (a gather of whole rows):
  python tools/bench_sums.py [--n 10000000] [--d 1024] [--k 4096] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--d", type=int, default=1024)
    p.add_argument("--k", type=int, default=4096)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    import torch
    from dislib_amd import _device
    from dislib_amd.data import Dataset, Subset
    dev = torch.device("cuda", 0)
    n, d, k = a.n, a.d, a.k
    X = torch.empty((n, d), dtype=torch.float64, device=dev)
    _device.make_blobs(X, 0, k, seed=0, box=10.0, std=1.0)
    labs = {"ordered": (torch.arange(n, device=dev) * k // n).to(torch.int32),
            "random": torch.randint(0, k, (n,), device=dev,
                                    dtype=torch.int32)}
    ws = _device.Workspace(k, d, n, dev)
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    out = {}
    for dt in ("f64", "f32"):
        Xd = X if dt == "f64" else X.float()
        ds = Dataset(n_features=d)
        ds.append(Subset(Xd))
        dd = ds._device_data()
        for name, lab in labs.items():
            ts = []
            for r in range(a.reps + 1):
                acc.zero_()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                _device.label_sums(dd, ws, lab, acc, k)
                torch.cuda.synchronize()
                if r:
                    ts.append(1e3 * (time.perf_counter() - t0))
            ms = min(ts)
            gbs = n * d * Xd.element_size() / ms * 1e-6
            out[f"{dt}_{name}"] = {"ms": round(ms, 3), "GB/s": round(gbs, 1)}
            print(dt, name, out[f"{dt}_{name}"], flush=True)
        del dd, ds
        if dt == "f32":
            del Xd
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
