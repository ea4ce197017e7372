"""Re-screen diagnostics (round 6): one C3-shape assignment against the
initial centres (bf16x3, iteration 0 of a fit) and one single-product call
(iteration 1's), with the workspace header's list counters: the re-check
list the screen left (rtotal) and the samples k_cand2 / k_recheck_list
took (rechecked_total delta), and the call time.

  python tools/rescreen_diag.py [--n 20000000]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def hdr(ws):
    import torch
    h = ws.buf[:256].cpu().numpy()
    rt = int(h[76:80].view(np.uint32)[0])
    tot = int(h[56:64].view(np.uint64)[0])
    q = int(h[48:52].view(np.uint32)[0])
    return rt, tot, q


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=20_000_000)
    p.add_argument("--d", type=int, default=64)
    p.add_argument("--k", type=int, default=1000)
    a = p.parse_args()
    import torch
    from dislib_amd import _device, _lib
    from dislib_amd.cluster.kmeans import _init_centers
    from dislib_amd.data import Dataset, Subset
    dev = torch.device("cuda", 0)
    X = torch.empty((a.n, a.d), dtype=torch.float64, device=dev)
    _device.make_blobs(X, 0, a.k, seed=0, box=10.0, std=1.0)
    ds = Dataset(n_features=a.d)
    ds.append(Subset(X))
    dd = ds._device_data(dev)
    C = torch.from_numpy(_init_centers(a.d, False, a.k, 0)).to(dev)
    ws = _device.Workspace(a.k, a.d, dd.n, dev)
    acc = torch.zeros(a.k * (a.d + 1), dtype=torch.float64, device=dev)
    lab = torch.full((dd.n,), -1, dtype=torch.int32, device=dev)
    C1 = C
    for name, mode in (("bf16x3 (iteration 0)", _lib.MODE_BF16X3),
                       ("bf16x3 again", _lib.MODE_BF16X3),
                       ("single, no hint (iteration 1)",
                        _lib.MODE_BF16 | _lib.MODE_NOHINT)):
        if "iteration 1" in name:
            C = C1
        _device.prepare(C, ws, acc)
        torch.cuda.synchronize()
        r0 = hdr(ws)
        t0 = time.perf_counter()
        _device.predict(dd, C, ws, lab, mode)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        r1 = hdr(ws)
        print("%-32s %8.2f ms  re-check list %d  taken by cand2+list %d  "
              "overflow %d" % (name, el * 1e3, r1[0], r1[1] - r0[1], r1[2]),
              flush=True)
        if "iteration 0" in name:
            # centres of the first assignment (host), for the next call
            labs = lab.cpu().numpy()
            x = X.cpu().numpy() if a.n <= 20_000_000 else None
            if x is not None:
                cc = C.cpu().numpy()
                for j in range(a.k):
                    m = labs == j
                    if m.any():
                        cc[j] = x[m].mean(0)
                C1 = torch.from_numpy(cc).to(dev)


if __name__ == "__main__":
    main()
