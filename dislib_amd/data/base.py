"""``load_data`` -- reference ``dislib/data/base.py:11-39``.

Slices an in-memory array (ndarray, CSR matrix, or a device ``torch``
tensor) into Subsets of ``subset_size`` rows.  The libsvm/txt file loaders
of the reference (``data/base.py:42-238``) are outside the k-means hot path
 and are not provided in this round.
"""
from scipy.sparse import issparse

from .classes import Dataset, Subset


def load_data(x, subset_size, y=None):
    """Loads data into a Dataset of Subsets of ``subset_size`` samples."""
    dataset = Dataset(n_features=x.shape[1], sparse=issparse(x))
    for i in range(0, x.shape[0], subset_size):
        if y is not None:
            subset = Subset(x[i: i + subset_size], y[i: i + subset_size])
        else:
            subset = Subset(x[i: i + subset_size])
        dataset.append(subset)
    return dataset
