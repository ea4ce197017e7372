"""Per-iteration diagnostics of a label-sorted-image fit (C3 by default):
samples that changed label, image tiles whose rows do not all carry the
tile's first label, centre blocks screened and tiles handed to the general
pass, and the step time.

  python tools/c3_diag.py [--n 125000000] [--d 64] [--k 1000] [--iters 10]
                          [--resort-at IT]

--resort-at IT: before iteration IT, rebuild the label-sorted image from the
current labels (dkm_x_image_sorted, the buffer reused) and print its time:
whether one re-sort pays back through cheaper screens.
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=125_000_000)
    p.add_argument("--d", type=int, default=64)
    p.add_argument("--k", type=int, default=1000)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--resort-at", type=int, default=-1)
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
    ds._device_data(dev)
    st = _Lloyd(ds, _init_centers(a.d, False, a.k, 0), 0.0, False, "auto",
                dev)
    nt = (a.n + 31) // 32
    tile_b = (a.d + 15) // 16 * 1024
    prev_c = (0, 0, 0, 0)
    for it in range(a.iters):
        if it == a.resort_at and st.simg is not None:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with st._on():
                st.simg = _device.sorted_image(st.dd, st.labels[:a.n], a.k,
                                               st.ws, old=st.simg)
            torch.cuda.synchronize()
            print({"resort_ms": round((time.perf_counter() - t0) * 1e3, 2)},
                  flush=True)
        before = st.labels[:a.n].clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        moved = int((st.labels[:a.n] != before).sum())
        lists = _device.screen_lists(st.ws)
        c = st.screened_blocks()
        dc = tuple(x - y for x, y in zip(c, prev_c))
        prev_c = c
        line = {"it": it, "ms": round(ms, 2), "moved": moved,
                "tiles": dc[0], "decided": dc[1], "blocks": dc[2],
                "fallback": dc[3], "recheck": lists[0], "two": lists[1],
                "many": lists[2], "overflow": lists[3]}
        if dc[0]:
            line["blocks_per_tile"] = round(dc[2] / dc[0], 2)
        if st.simg is not None:
            img = st.simg[0]
            off = nt * tile_b + nt * 128 + nt * 128
            plab = img[off:off + nt * 128].view(torch.int32).view(nt, 32)
            perm = img[nt * tile_b + nt * 128:off].view(torch.int32).view(
                nt, 32)
            ok = perm >= 0
            first = plab[:, :1]
            mixed = ((plab != first) & ok).any(dim=1)
            line["mixed_tiles"] = int(mixed.sum())
            line["mixed_frac"] = round(int(mixed.sum()) / nt, 4)
            line["rows_not_first"] = int(((plab != first) & ok).sum())
        print(line, flush=True)


if __name__ == "__main__":
    main()
