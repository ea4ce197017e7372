from dislib_amd.neighbors.base import NearestNeighbors

__all__ = ["NearestNeighbors"]
