"""The k-means driver keeps the reference driver's command line
(examples/kmeans-driver.py:14-37): same flags, defaults and positional."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_driver_flags_and_defaults():
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import kmeans_driver
    a = kmeans_driver._parser().parse_args(["-f", "7", "data.txt"])
    assert (a.libsvm, a.detailed_times, a.arity, a.clusters, a.part_size,
            a.iteration, a.features, a.dense, a.train_data) == \
        (False, False, 50, 2, 100, 5, 7, False, "data.txt")
    a = kmeans_driver._parser().parse_args(
        ["--libsvm", "-dt", "-a", "3", "-c", "4", "-p", "9", "-i", "2",
         "--features", "11", "--dense", "d"])
    assert (a.libsvm, a.detailed_times, a.arity, a.clusters, a.part_size,
            a.iteration, a.features, a.dense) == \
        (True, True, 3, 4, 9, 2, 11, True)
