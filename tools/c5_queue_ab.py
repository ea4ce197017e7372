"""C5 (CSR 10M x 10k, 10 nnz, k = 256): the fit's step time with the
workspace queue at n (the CSR screen then runs in two chunks of n / 2) and
at 2n (one chunk), alternating in one process.  Diagnostic only.
usage: c5_queue_ab.py [n] [rounds]"""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from dislib_amd import _device  # noqa: E402
from dislib_amd.cluster.kmeans import _Lloyd, _init_centers  # noqa: E402
from dislib_amd.data import Dataset, Subset  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
d, k, nnz, steps = 10_000, 256, 10, 6
dev = torch.device("cuda", 0)
X = bench.csr_rows(0, n, d, nnz, seed=1)
ds = Dataset(n_features=d, sparse=True)
for i in range(0, n, 1_000_000):
    ds.append(Subset(X[i:i + 1_000_000]))
ds._device_data(dev)
C0 = _init_centers(d, True, k, 0).toarray()
for r in range(rounds):
    for mult in (1, 2):
        st = _Lloyd(ds, C0, 0.0, False, "auto", dev)
        if mult != 1:
            st.ws = _device.Workspace(k, d, min(mult * n, 1 << 27), dev)
        ts = []
        for _ in range(steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.step()
            st.read_flags()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print("round %d queue %dn: ms per step %s, mean of last 3 %.3f" % (
            r, mult, [round(t, 3) for t in ts], sum(ts[-3:]) / 3),
            flush=True)
        del st
        torch.cuda.empty_cache()
