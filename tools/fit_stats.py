"""Per-iteration statistics of one fit on the bench data (diagnostics):
wall time, samples re-checked (candidate / re-check lists), threshold-pass
tiles and centre blocks screened over the label-sorted image, and labels
changed.

  python tools/fit_stats.py [--n N] [--d D] [--k K] [--iters I]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=125_000_000)
    p.add_argument("--d", type=int, default=64)
    p.add_argument("--k", type=int, default=1000)
    p.add_argument("--iters", type=int, default=10)
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
    prev_lab = None
    r0, c0 = 0, (0, 0, 0)
    for it in range(a.iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        rc = st.rechecked()
        cc = st.screened_blocks() if st.sorting else (0, 0, 0)
        lab = st.labels[:st.dd.n]
        moved = int((lab != prev_lab).sum()) if prev_lab is not None else -1
        prev_lab = lab.clone()
        tiles = cc[0] - c0[0]
        print("it %d  %.2f ms  rechecked %d  moved %d  tiles %d  decided %d  "
              "blocks/tile %.2f" % (
                  it, ms, rc - r0, moved, tiles, cc[1] - c0[1],
                  (cc[2] - c0[2]) / tiles if tiles else 0.0), flush=True)
        r0, c0 = rc, cc


if __name__ == "__main__":
    main()
