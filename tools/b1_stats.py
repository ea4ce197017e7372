"""Per-iteration diagnostics of the single-product screen's threshold pass
(C3 shape by default): wave tiles that ran the threshold pass, tiles that
kept its result (the rest redid the tile with the top-3 pass), re-checked
samples, and the step time.   python tools/b1_stats.py [--n N] [--iters I]
Reads the workspace header counters (WsHeader.reserved[0..1],
rechecked_total) that k_screen_b1 / the re-check kernels accumulate."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=20_000_000)
    p.add_argument("--d", type=int, default=64)
    p.add_argument("--k", type=int, default=1000)
    p.add_argument("--iters", type=int, default=12)
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
    prev = np.zeros(3, np.int64)
    for it in range(a.iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        h = st.ws.buf[:256].cpu().numpy().view(np.uint64)
        cur = np.array([h[11], h[12], h[7]], dtype=np.int64)
        dlt = cur - prev
        prev = cur
        print("iter %2d  %7.2f ms  threshold tiles %9d  "
              "kept %9d  rechecked %9d" % (it, el * 1e3, dlt[0],
                                           dlt[1], dlt[2]), flush=True)


if __name__ == "__main__":
    main()
