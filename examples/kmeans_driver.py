"""K-means driver: the drop-in for dislib's ``examples/kmeans-driver.py``
(reference lines 12-74), run on MI355X through ``dislib_amd``.

Command line and output are the reference's: read a LibSVM or text file (or
a directory of them) into a Dataset, fit ``KMeans(n_clusters, max_iter,
arity, verbose=True)``, print ``[clusters, arity, part_size, read_time,
fit_time]``.  The reference's ``pycompss.api.api.barrier()`` becomes a
device synchronisation.

One addition: ``--make-blobs N`` first writes the BASELINE configs[0] input
-- ``make_blobs(N, FEATURES, centers=CLUSTERS, random_state=0)`` as CSV with
the blob id in the last column -- so the config-1 plumbing run is

  python examples/kmeans_driver.py --make-blobs 100000 -f 50 -c 10 \\
      -p 10000 -i 10 --dense /tmp/c1.csv
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dislib_amd import data as dsd  # noqa: E402
from dislib_amd.cluster import KMeans  # noqa: E402

# (flags, keyword arguments) of the reference driver's options, in its order
_OPTIONS = [
    (("--libsvm",), dict(action="store_true",
                         help="read files in libsvm format")),
    (("-dt", "--detailed_times"), dict(action="store_true",
                                       help="time the read and the fit "
                                            "separately")),
    (("-a", "--arity"), dict(type=int, default=50, metavar="CASCADE_ARITY",
                             help="merge arity (no effect on the GPU; "
                                  "default 50)")),
    (("-c", "--clusters"), dict(type=int, default=2, metavar="N_CLUSTERS",
                                help="number of clusters (default 2)")),
    (("-p", "--part_size"), dict(type=int, default=100, metavar="PART_SIZE",
                                 help="rows per Subset (default 100; "
                                      "ignored for a directory)")),
    (("-i", "--iteration"), dict(type=int, default=5,
                                 metavar="MAX_ITERATIONS",
                                 help="maximum iterations (default 5)")),
    (("-f", "--features"), dict(type=int, required=True,
                                metavar="N_FEATURES")),
    (("--dense",), dict(action="store_true",
                        help="keep the samples dense")),
]


def _parser():
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    for flags, kw in _OPTIONS:
        p.add_argument(*flags, **kw)
    p.add_argument("--make-blobs", type=int, default=0, metavar="N_SAMPLES",
                   help="write make_blobs(N_SAMPLES, FEATURES, "
                        "centers=CLUSTERS, random_state=0) to train_data "
                        "first (CSV, label last)")
    p.add_argument("train_data", type=str,
                   help="a file, or a directory of files (one Subset each)")
    return p


def _sync():
    """pycompss barrier(): every queued device operation has finished."""
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _write_blobs(path, n, d, k):
    import numpy as np
    from sklearn.datasets import make_blobs
    x, y = make_blobs(n_samples=n, n_features=d, centers=k, random_state=0)
    np.savetxt(path, np.column_stack([x, y]), delimiter=",", fmt="%.17g")


def _read(a):
    """The reference's four loader branches (file/directory x libsvm/txt)."""
    many = os.path.isdir(a.train_data)
    if a.libsvm:
        kw = dict(store_sparse=not a.dense)
        if many:
            return dsd.load_libsvm_files(a.train_data, a.features, **kw)
        return dsd.load_libsvm_file(a.train_data, subset_size=a.part_size,
                                    n_features=a.features, **kw)
    if many:
        return dsd.load_txt_files(a.train_data, a.features, label_col="last")
    return dsd.load_txt_file(a.train_data, subset_size=a.part_size,
                             n_features=a.features, label_col="last")


def main(argv=None):
    a = _parser().parse_args(argv)
    if a.make_blobs:
        _write_blobs(a.train_data, a.make_blobs, a.features, a.clusters)
    t0 = time.time()
    dataset = _read(a)
    read_time = 0
    if a.detailed_times:
        _sync()
        read_time = time.time() - t0
        t0 = time.time()
    km = KMeans(n_clusters=a.clusters, max_iter=a.iteration, arity=a.arity,
                verbose=True)
    km.fit(dataset)
    _sync()
    print([a.clusters, a.arity, a.part_size, read_time, time.time() - t0])
    return km, dataset


if __name__ == "__main__":
    main()
