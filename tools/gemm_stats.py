"""Per-iteration diagnostics of the GEMM screen (d > 128) on the bench data:
wall time, samples re-checked (candidate + overflow lists) and samples on
the overflow scan (k_gemm_full), from the workspace header.

  python tools/gemm_stats.py [--n N] [--d D] [--k K] [--iters I]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def header(ws):
    h = ws.buf[:128].cpu().numpy().view(np.uint64)
    return int(h[7]), int(h[15])   # rechecked_total, reserved[4]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=2_000_000)
    p.add_argument("--d", type=int, default=1024)
    p.add_argument("--k", type=int, default=4096)
    p.add_argument("--iters", type=int, default=4)
    a = p.parse_args()
    import torch
    from dislib_amd import _device
    from dislib_amd.cluster.kmeans import _Lloyd, _init_centers
    from dislib_amd.data import Dataset, Subset
    dev = torch.device("cuda", 0)
    X = torch.empty((a.n, a.d), dtype=torch.float64, device=dev)
    _device.make_blobs(X, 0, a.k, seed=0, box=10.0, std=1.0)
    ds = Dataset(n_features=a.d)
    for i in range(0, a.n, 1_000_000):
        ds.append(Subset(X[i:i + 1_000_000]))
    st = _Lloyd(ds, _init_centers(a.d, False, a.k, 0), 0.0, False, "auto",
                dev)
    r0, f0 = header(st.ws)
    for it in range(a.iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        r1, f1 = header(st.ws)
        print("iter %d  %.1f ms  rechecked %d  overflow-scan %d"
              % (it, el * 1e3, r1 - r0, f1 - f0), flush=True)
        r0, f0 = r1, f1


if __name__ == "__main__":
    main()
