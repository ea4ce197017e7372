from dislib_amd.data.classes import Dataset, Subset
from dislib_amd.data.base import load_data

__all__ = ['Dataset', 'Subset', 'load_data']
