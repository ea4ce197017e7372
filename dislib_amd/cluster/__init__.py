from dislib_amd.cluster.kmeans import KMeans

__all__ = ['KMeans']
