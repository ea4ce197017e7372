"""Reproduce test_gpu_b2::test_threshold_pass_shapes[sorted-dups-d-k] and
describe the rows whose label differs from the oracle (debug aid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import test_gpu_b2 as tb  # noqa: E402
from oracle import kmeans_oracle as orc  # noqa: E402


def main(d=48, k=777):
    from dislib_amd import _device
    _device.X_IMAGE = True
    tb._VARIANT["name"] = "sorted"
    n = 30000
    rng, x, C = tb._problem(n, d, k, 1000 * d + k)
    pairs = tb._dups_every_block(rng, C)
    m = len(pairs)
    idx = rng.integers(0, n, 40 * m)
    for t, i in enumerate(idx):
        j, p = pairs[t % m]
        x[i] = C[p] + rng.standard_normal(d)
    rl, rs, rc = orc.partial_sum(x, C)
    _, inv = np.unique(C, axis=0, return_inverse=True)
    inv = np.asarray(inv).reshape(-1)
    last = {}
    for c in range(k):
        last[inv[c]] = c
    hint = np.array([last[inv[c]] for c in rl])
    from dislib_amd import _lib
    from dislib_amd.data import load_data
    dev = torch.device("cuda", 0)
    ds = load_data(x, subset_size=x.shape[0])
    dd = ds._device_data()
    Ct = torch.from_numpy(np.ascontiguousarray(C)).to(dev)
    ws = _device.Workspace(k, d, dd.n, dev)
    acc = torch.zeros(k * (d + 1), dtype=torch.float64, device=dev)
    labt = torch.from_numpy(np.asarray(hint).astype(np.int32)).to(dev)
    _device.prepare(Ct, ws, acc)
    image = _device.sorted_image(dd, labt, k, ws)
    nt = (n + 31) // 32
    tb_ = (d + 15) // 16 * 1024
    img = image[0]
    perm0 = img[nt * tb_ + nt * 128:nt * tb_ + nt * 256].view(torch.int32).cpu().numpy().copy()
    plab0 = img[nt * tb_ + nt * 256:nt * tb_ + nt * 384].view(torch.int32).cpu().numpy().copy()
    _device.partial_sum(dd, Ct, ws, labt, acc, _lib.MODE_BF16, image=image)
    lab = labt.cpu().numpy()
    for t in (329, 636):
        print("device tile", t, "plab", plab0[t * 32:(t + 1) * 32].tolist())
        print("   perm hints", hint[perm0[t * 32:(t + 1) * 32]].tolist())
    bad = np.nonzero(lab != rl)[0]
    print("pairs", pairs)
    print("bad rows", len(bad))
    order = np.argsort(hint, kind="stable")
    pos = np.empty(n, np.int64)
    pos[order] = np.arange(n)
    order = np.argsort(hint, kind="stable")
    pos = np.empty(n, np.int64)
    pos[order] = np.arange(n)
    if os.environ.get("DKM_LIB", "").endswith(("dbg4.so", "dbg5.so")):
        where = np.empty(n, np.int64)
        where[perm0[perm0 >= 0]] = np.nonzero(perm0 >= 0)[0]
        for i in (5081, 5236, 6637):
            t = where[i] // 32
            print("   device tile", t, "plab", plab0[t * 32:(t + 1) * 32].tolist(),
                  "row at", where[i] % 32)
            m = int(lab[i]) & 0x3fffffff
            print("row", i, "ref", rl[i], "hint", hint[i], "blocks",
                  [b for b in range(32) if m >> b & 1])
        return
    if os.environ.get("DKM_LIB", "").endswith("dbg3.so"):
        dup = np.nonzero(hint != rl)[0]
        cd = lab[dup]
        u, c = np.unique(cd, return_counts=True)
        print("dup-row codes", dict(zip(u.tolist(), c.tolist())))
        for i in dup[(cd % 100) // 10 == 0][:8]:
            t = pos[i] // 32
            rows = order[t * 32:(t + 1) * 32]
            print("row", i, "code", lab[i], "ref", rl[i], "hint", hint[i],
                  "tile", t, "hints", hint[rows].tolist())
        codes = lab[lab >= 1000000]
        u, c = np.unique(codes // 10000, return_counts=True)
        print("bmask popcounts", dict(zip(u.tolist(), c.tolist())))
        return
    for i in bad[:20]:
        t = pos[i] // 32
        rows = order[t * 32:(t + 1) * 32]
        print("row", i, "got", lab[i], "ref", rl[i], "hint", hint[i],
              "tile", t, "tile hints", sorted(set(hint[rows].tolist())))
        dist = np.sqrt(((x[i] - C) ** 2).sum(1))
        o = np.argsort(dist)[:4]
        print("   nearest", o.tolist(), dist[o].tolist())


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
