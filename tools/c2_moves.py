"""Per-iteration moves of a C2 fit (100M x 32, k = 100): labels changed,
rows left undecided by the screen, and the assignment call's time.
Diagnostic only (the bench line is bench.py's).  usage: c2_moves.py [n] [iters]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from dislib_amd import _device  # noqa: E402
from dislib_amd.cluster.kmeans import _Lloyd, _init_centers  # noqa: E402
from dislib_amd.data import Dataset, Subset  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 8
d, k = 32, 100
dev = torch.device("cuda:0")
X = torch.empty((n, d), dtype=torch.float64, device=dev)
_device.make_blobs(X, 0, k, seed=0, box=10.0, std=1.0)
ds = Dataset(n_features=d)
for i in range(0, n, 10_000_000):
    ds.append(Subset(X[i:i + 10_000_000]))
C0 = _init_centers(d, False, k, 0)
st = _Lloyd(ds, C0, 0.0, False, "auto", dev)
prev = None
for it in range(iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(
        enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    st.assign()
    e1.record()
    st.reduce_update()
    st.read_flags()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    lab = st.labels[:n].clone()
    moved = -1 if prev is None else int((lab != prev).sum())
    hdr = st.rechecked()
    cnt = np.bincount(lab.cpu().numpy(), minlength=k)
    print("it %d assign %.2f ms wall %.2f ms moved %d (%.2f%%) nonempty %d "
          "max cluster %.1f%% rechecked %s" % (
              it, e0.elapsed_time(e1), wall, moved, 100.0 * moved / n,
              int((cnt > 0).sum()), 100.0 * cnt.max() / n, hdr), flush=True)
    prev = lab
