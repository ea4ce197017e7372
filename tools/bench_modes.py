"""A/B the assignment kernels in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Times dkm_partial_sum per mode with
HIP events on torch's current stream and checks that every mode produces the
same labels as the exact kernel on the same centres.

  python tools/bench_modes.py --n 100000000 --d 32 --k 100 --rounds 5
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--modes", default="screen32,bf16x3")
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--centres", default="fitted",
                    help="fitted (2 Lloyd steps from the U[0,1) init) | init")
    a = ap.parse_args()
    import torch
    from dislib_amd import _device, _lib
    from dislib_amd.cluster.kmeans import _Lloyd, _init_centers, _MODES
    from dislib_amd.data import Dataset, Subset
    dev = torch.device("cuda")
    X = torch.empty((a.n, a.d), dtype=torch.float64, device=dev)
    _device.make_blobs(X, 0, a.k, seed=0)
    if a.fp32:
        X = X.float()
    ds = Dataset(n_features=a.d)
    ds.append(Subset(X))
    st = _Lloyd(ds, _init_centers(a.d, False, a.k, 0), 0.0, True, "auto",
                dev)
    if a.centres == "fitted":
        st.step()
        st.step()
    dd, C, ws = st.dd, st.C, st.ws
    acc = st.acc
    modes = a.modes.split(",")
    lab = {m: torch.empty(a.n, dtype=torch.int32, device=dev) for m in modes}
    times = {m: [] for m in modes}
    ptimes = {m: [] for m in modes}
    rech = {}
    for r in range(a.rounds):
        for m in modes:
            _device.prepare(C, ws, acc)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            before = _device.rechecked(ws)
            e0.record()
            _device.partial_sum(dd, C, ws, lab[m], acc, _MODES[m])
            e1.record()
            torch.cuda.synchronize()
            times[m].append(e0.elapsed_time(e1))
            rech[m] = _device.rechecked(ws) - before
            e0.record()
            _device.predict(dd, C, ws, lab[m], _MODES[m])
            e1.record()
            torch.cuda.synchronize()
            ptimes[m].append(e0.elapsed_time(e1))
    ref = lab[modes[0]].cpu().numpy()
    out = {}
    bytes_ = a.n * a.d * (4 if a.fp32 else 8)
    for m in modes:
        t = np.array(times[m])
        same = bool(np.array_equal(lab[m].cpu().numpy(), ref))
        out[m] = {"median_ms": float(np.median(t)), "min_ms": float(t.min()),
                  "predict_median_ms": float(np.median(ptimes[m])),
                  "GBps": bytes_ / (np.median(t) * 1e-3) / 1e9,
                  "rechecked": rech[m], "labels_equal_first": same}
    print(json.dumps({"n": a.n, "d": a.d, "k": a.k, "fp32": a.fp32,
                      "centres": a.centres, "modes": out}, indent=1))


if __name__ == "__main__":
    main()
