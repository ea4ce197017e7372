"""Find samples where a screen mode disagrees with the exact kernel and report
what the reference arithmetic says about them (gap between the two best
distances vs the screen bound).  Diagnostic tool, not part of the product.

  python tools/debug_mismatch.py --n 300000
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300000)
    ap.add_argument("--nfit", type=int, default=4000000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--k", type=int, default=100)
    a = ap.parse_args()
    import torch
    from dislib_amd import _device, _lib
    from dislib_amd.cluster.kmeans import KMeans
    from dislib_amd.data import Dataset, Subset
    from oracle import kmeans_oracle as orc
    dev = torch.device("cuda")
    X = torch.empty((a.nfit, a.d), dtype=torch.float64, device=dev)
    _device.make_blobs(X, 0, a.k, seed=0)
    ds = Dataset(n_features=a.d)
    ds.append(Subset(X))
    km = KMeans(n_clusters=a.k, max_iter=3, tol=0, random_state=0)
    km.fit(ds)
    C = km.centers
    xs = X[:a.n].contiguous()
    sub = Dataset(n_features=a.d)
    sub.append(Subset(xs))
    dd = sub._device_data()
    Ct = torch.from_numpy(C).to(dev)
    ws = _device.Workspace(a.k, a.d, a.n, dev)
    acc = torch.zeros(a.k * (a.d + 1), dtype=torch.float64, device=dev)
    out = {}
    labs = {}
    reps = int(os.environ.get("DBG_REPS", "1"))
    for name, m in [("exact", _lib.MODE_EXACT),
                    ("screen32", _lib.MODE_SCREEN32),
                    ("bf16x3", _lib.MODE_BF16X3)]:
        for kind in ["partial", "predict"] * reps:
            lab = torch.full((a.n,), -7, dtype=torch.int32, device=dev)
            _device.prepare(Ct, ws, acc)
            if kind == "partial":
                _device.partial_sum(dd, Ct, ws, lab, acc, m)
            else:
                _device.predict(dd, Ct, ws, lab, m)
            torch.cuda.synchronize()
            key = (name, kind)
            r = 0
            while (name, "%s%d" % (kind, r)) in labs:
                r += 1
            labs[(name, "%s%d" % (kind, r))] = lab.cpu().numpy()
    ref = labs[("exact", "partial0")]
    xh = xs.cpu().numpy()
    cn = np.sqrt((C * C).sum(1))
    for key, lab in labs.items():
        bad = np.nonzero(lab != ref)[0]
        info = {"n_bad": int(bad.size), "n_neg": int((lab < 0).sum())}
        ex = []
        for i in bad[:8]:
            dist = orc.dense_distances(xh[i:i + 1], C)[0]
            o = np.argsort(dist)
            xn = float(np.sqrt((xh[i] ** 2).sum()))
            ex.append({"i": int(i), "got": int(lab[i]), "ref": int(ref[i]),
                       "d2_best": float(dist[o[0]] ** 2),
                       "d2_2nd": float(dist[o[1]] ** 2),
                       "d2_got": float(dist[lab[i]] ** 2)
                       if 0 <= lab[i] < a.k else None,
                       "xn": xn, "cmax": float(cn.max()),
                       "i_mod_32": int(i % 32), "i_mod_16": int(i % 16)})
        info["examples"] = ex
        if bad.size:
            info["bad_mod16_hist"] = np.bincount(bad % 16, minlength=16).tolist()
            info["bad_first"] = bad[:20].tolist()
        out["%s/%s" % key] = info
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
