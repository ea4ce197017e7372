"""dislib_amd -- MI355X-native drop-in for dislib's k-means Lloyd path.

``from dislib_amd.cluster import KMeans`` and
``from dislib_amd.data import Dataset, Subset, load_data`` mirror
``dislib.cluster.KMeans`` / ``dislib.data`` (dislib v0.2.0).
:func:`install_as_dislib` registers the same modules under the ``dislib``
names so unmodified user code (``from dislib.cluster import KMeans``) runs on
the GPU path.
"""
import sys

name = "dislib_amd"
__version__ = "0.1.0"

from dislib_amd._shard import shard_dataset, shard_range  # noqa: E402,F401


def install_as_dislib():
    """Alias ``dislib``, ``dislib.cluster``, ``dislib.data`` and
    ``dislib.neighbors`` to this package (the k-means path, its data
    containers and the kNN reuse of its distance primitive)."""
    import types
    from dislib_amd import cluster, data, neighbors
    pkg = types.ModuleType("dislib")
    pkg.__path__ = []
    pkg.name = "dislib"
    pkg.cluster = cluster
    pkg.data = data
    pkg.neighbors = neighbors
    sys.modules["dislib"] = pkg
    sys.modules["dislib.neighbors"] = neighbors
    sys.modules["dislib.cluster"] = cluster
    sys.modules["dislib.data"] = data
    return pkg
