"""Probe: the C2 headline shape (100M x 32, k = 100) through the label-sorted
single-product path (k_screen_sorted / k_screen_b2 + delta sums) instead of
auto mode's bf16x3 split-image screen with in-LDS full sums.  Prints the
per-iteration wall time of both fits (tol = 0) and checks that the labels
agree at the end.
  python tools/c2_sorted_probe.py [--n 100000000] [--d 32] [--k 100] [--iters 10]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=100_000_000)
    p.add_argument("--d", type=int, default=32)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--iters", type=int, default=10)
    a = p.parse_args()
    import torch
    from dislib_amd import _device, _lib
    from dislib_amd.cluster import kmeans as km
    from dislib_amd.data import Dataset, Subset
    dev = torch.device("cuda", 0)
    X = torch.empty((a.n, a.d), dtype=torch.float64, device=dev)
    _device.make_blobs(X, 0, a.k, seed=0, box=10.0, std=1.0)
    ds = Dataset(n_features=a.d)
    for i in range(0, a.n, 1_000_000):
        ds.append(Subset(X[i:i + 1_000_000]))
    ds._device_data(dev)
    C0 = km._init_centers(a.d, False, a.k, 0)
    labs = {}
    for name in ("auto", "sorted"):
        st = km._Lloyd(ds, C0, 0.0, False, "auto", dev)
        if name == "sorted":
            st.sorting = bool(_lib.lib().dkm_x_image_sorted_ok(a.k, a.d))
        ts = []
        for it in range(a.iters):
            if name == "sorted" and it == 1:
                st.mode = _lib.MODE_BF16   # single product from iteration 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.step()
            torch.cuda.synchronize()
            ts.append(round(1e3 * (time.perf_counter() - t0), 2))
        labs[name] = st.labels[:a.n].clone()
        print(name, "ms/iter", ts, "steady(2..)",
              round(sum(ts[2:]) / max(1, len(ts) - 2), 3),
              "whole", round(sum(ts) / len(ts), 3), flush=True)
        del st
        torch.cuda.empty_cache()
    print("labels equal:", bool(torch.equal(labs["auto"], labs["sorted"])),
          flush=True)


if __name__ == "__main__":
    main()
