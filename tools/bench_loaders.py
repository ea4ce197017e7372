"""Loader throughput: ``load_libsvm_file`` /
``load_txt_file`` (C++ parser in libdkm.so) vs the reference's path (the
oracle's restatement: sklearn ``load_svmlight_file`` / ``np.genfromtxt`` per
chunk of ``subset_size`` lines, sequential PyCOMPSs mode).  With a GPU it
also times the one-shot HBM upload of the parsed CSR.
usage: python tools/bench_loaders.py [--rows N] [--d D] [--nnz Z]"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(
    __file__))))
from dislib_amd.data import load_libsvm_file, load_txt_file  # noqa: E402
from oracle import loaders_oracle as orc  # noqa: E402


def write_libsvm(path, rows, d, nnz, seed=0):
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for a in range(0, rows, 100000):
            m = min(100000, rows - a)
            cols = np.sort(np.argsort(rng.random((m, d)), axis=1)[:, :nnz]
                           if d <= 64 else
                           rng.choice(d, size=(m, nnz * 2))[:, :nnz], axis=1)
            vals = rng.random((m, nnz))
            lines = []
            for i in range(m):
                c = np.unique(cols[i])
                lines.append("%d " % (i % 2) + " ".join(
                    "%d:%r" % (j + 1, float(v))
                    for j, v in zip(c, vals[i, :c.size])))
            f.write("\n".join(lines) + "\n")


def write_csv(path, rows, d, seed=0):
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for a in range(0, rows, 100000):
            m = min(100000, rows - a)
            np.savetxt(f, rng.standard_normal((m, d)), delimiter=",",
                       fmt="%.17g")


def timed(fn):
    t = time.perf_counter()
    r = fn()
    return r, time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=500000)
    ap.add_argument("--d", type=int, default=10000)
    ap.add_argument("--nnz", type=int, default=10)
    ap.add_argument("--csv-rows", type=int, default=200000)
    ap.add_argument("--csv-d", type=int, default=32)
    ap.add_argument("--subset", type=int, default=100000)
    ap.add_argument("--ref-rows", type=int, default=100000,
                    help="rows of the file the (slow) reference path reads")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    from dislib_amd.data.base import _threads
    out = {"parser_threads": _threads(),
           "affinity_cpus": len(os.sched_getaffinity(0))}
    p = os.path.join(tmp, "x.svm")
    write_libsvm(p, a.rows, a.d, a.nnz)
    mb = os.path.getsize(p) / 1e6
    ds, t = timed(lambda: load_libsvm_file(p, a.subset, a.d))
    out["libsvm"] = {"rows": a.rows, "d": a.d, "nnz_row": a.nnz, "MB": mb,
                     "s": t, "MB_per_s": mb / t}
    q = os.path.join(tmp, "r.svm")
    write_libsvm(q, a.ref_rows, a.d, a.nnz, seed=1)
    mbq = os.path.getsize(q) / 1e6
    _, tq = timed(lambda: orc.load_file(q, a.subset, "libsvm", a.d,
                                        store_sparse=True))
    _, tn = timed(lambda: load_libsvm_file(q, a.subset, a.d))
    out["libsvm_ref_sample"] = {"rows": a.ref_rows, "MB": mbq,
                                "reference_s": tq, "native_s": tn,
                                "reference_MB_per_s": mbq / tq,
                                "speedup": tq / tn}
    c = os.path.join(tmp, "x.csv")
    write_csv(c, a.csv_rows, a.csv_d)
    mbc = os.path.getsize(c) / 1e6
    _, tc = timed(lambda: load_txt_file(c, a.subset, a.csv_d))
    _, tcr = timed(lambda: orc.load_file(c, a.subset, "txt", a.csv_d,
                                         delimiter=","))
    out["txt"] = {"rows": a.csv_rows, "d": a.csv_d, "MB": mbc, "s": tc,
                  "MB_per_s": mbc / tc, "reference_s": tcr,
                  "reference_MB_per_s": mbc / tcr, "speedup": tcr / tc}
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            dd, tu = timed(lambda: (ds._device_data(),
                                    torch.cuda.synchronize())[0])
            out["libsvm"]["upload_s"] = tu
    except ImportError:
        pass
    for f in (p, q, c):
        os.remove(f)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
