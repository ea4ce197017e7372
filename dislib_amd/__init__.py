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
    """Alias ``dislib``, ``dislib.cluster`` and ``dislib.data`` to this
    package (only the k-means path and its data containers)."""
    import types
    from dislib_amd import cluster, data
    pkg = types.ModuleType("dislib")
    pkg.__path__ = []
    pkg.name = "dislib"
    pkg.cluster = cluster
    pkg.data = data
    sys.modules["dislib"] = pkg
    sys.modules["dislib.cluster"] = cluster
    sys.modules["dislib.data"] = data
    return pkg
