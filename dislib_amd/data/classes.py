"""``Dataset`` / ``Subset`` -- the data containers of dislib's k-means path.

Mirrors the members of ``dislib.data.Dataset`` and ``dislib.data.Subset``
(reference ``dislib/data/classes.py:8-364``) that the k-means path and its
callers use, with the same semantics:

* ``Subset(samples, labels=None)`` copies ``samples`` (classes.py:298-304);
* ``Subset.set_label`` lazily creates an object array of ``None`` and writes
  into it, or into the existing label array keeping its dtype (:339-357);
* ``Dataset.labels`` concatenates the non-``None`` Subset labels, or is
  ``None`` (:226-229, :257-266).

MI355X-native additions: a Dataset keeps an HBM image of its samples
(:class:`dislib_amd._device.DeviceData`) so Lloyd iterations never re-upload
data, and labels produced on the device stay there (int32) until a Subset's
``labels`` is read (the reference's ``collect()`` sync point, :223-224).
Samples may also be device tensors (``torch.Tensor`` on ``cuda``) -- then the
data never touches the host.
"""
import numpy as np
import scipy.sparse as sp
from scipy.sparse import issparse


def _nrows(x):
    return int(x.shape[0])


def _is_device_tensor(x):
    return type(x).__module__.startswith("torch") and hasattr(x, "is_cuda")


def _freeze(x):
    """Make a host sample array (or a CSR matrix's arrays) read-only: the
    HBM copy is its image, so an in-place edit must fail loudly instead of
    leaving later fits on stale device data (the reference re-reads the
    samples on every task).  A visible side effect on caller-owned arrays,
    documented on ``Dataset``; assign a new array to change a Subset's
    samples, which re-uploads.  When the samples are a view (``x.base`` is
    an array, e.g. the slices ``load_data`` makes of the caller's matrix),
    only the view is frozen: the caller's own matrix stays writable, and a
    write through it is not caught (``Dataset`` says so)."""
    if isinstance(x, np.ndarray):
        x.setflags(write=False)
    elif issparse(x):
        for a in (getattr(x, "data", None), getattr(x, "indices", None),
                  getattr(x, "indptr", None)):
            if isinstance(a, np.ndarray):
                a.setflags(write=False)


class _DeviceLabels:
    """Labels of a whole Dataset, resident on the device (int32)."""

    def __init__(self, tensor):
        self.tensor = tensor
        self._host = None

    def host(self):
        if self._host is None:
            self._host = self.tensor.cpu().numpy().astype(np.int64)
        return self._host


class Subset(object):
    """A block of samples (ndarray, CSR matrix, or device tensor) with
    optional labels.  Reference: ``data/classes.py:280-364``."""

    def __init__(self, samples, labels=None):
        if _is_device_tensor(samples):
            # HBM-resident block: kept by reference (a view), never copied
            self.samples = samples
        else:
            self.samples = samples.copy()
        if labels is not None:
            self._labels = np.array(labels)
        else:
            self._labels = None
        self._pending = None          # (DeviceLabels, start, end)

    # -- labels ------------------------------------------------------------
    def _materialise(self):
        if self._pending is None:
            return
        src, a, b = self._pending
        self._pending = None
        vals = src.host()[a:b]
        if self._labels is None:
            # reference: np.array([None] * n) then labels[idx] = np.int64
            self._labels = np.array(list(vals), dtype=object)
        elif self._labels.dtype == object:
            self._labels[:] = list(vals)   # np.int64 objects, in place
        else:
            self._labels[:] = vals    # in place, keeping the existing dtype

    @property
    def labels(self):
        self._materialise()
        return self._labels

    @labels.setter
    def labels(self, value):
        self._pending = None
        self._labels = value

    def _set_device_labels(self, src, start, end):
        self._pending = (src, start, end)

    def set_label(self, index, label):
        """Reference ``Subset.set_label`` (classes.py:339-357)."""
        self._materialise()
        if self._labels is None:
            self._labels = np.array([None] * _nrows(self.samples))
        self._labels[index] = label

    # -- misc members of the reference Subset ------------------------------
    def copy(self):
        return Subset(samples=self.samples, labels=self.labels)

    def concatenate(self, subset):
        assert issparse(self.samples) == issparse(subset.samples), \
            "Cannot concatenate sparse data with non-sparse data."
        assert (self.labels is None) == (subset.labels is None), \
            "Cannot concatenate labeled data with non-labeled data"
        if issparse(self.samples):
            self.samples = sp.vstack([self.samples, subset.samples])
        else:
            self.samples = np.concatenate([self.samples, subset.samples])
        if self.labels is not None:
            self._labels = np.concatenate([self.labels, subset.labels])

    def __getitem__(self, item):
        if self.labels is not None:
            return Subset(self.samples[item], self.labels[item])
        return Subset(self.samples[item])


class Dataset(object):
    """Ordered list of Subsets.  Reference: ``data/classes.py:8-277``.

    Device residency: the first device use (a fit, a predict, a neighbour
    query) uploads the samples to HBM and keeps them there.  From then on
    the host arrays behind it -- each Subset's ``samples`` ndarray and the
    arrays of a CSR matrix -- are made read-only, so that an in-place write fails loudly instead of leaving
    the device copy stale (the reference re-reads samples on every task).
    To change the data, assign new arrays to the Subsets (``ds[i].samples
    = new``); the next device use uploads them.  Device tensors given as
    samples are tracked by their version counter instead.  Not caught: a
    write through an array the samples are views of (``load_data(x)``
    slices ``x``; ``x`` itself stays writable) -- treat such an array as
    read-only while the Dataset is in use, or pass a copy."""

    def __init__(self, n_features, sparse=False):
        self._subsets = list()
        self.n_features = n_features
        self._sizes = list()
        self._max_features = None
        self._min_features = None
        self._samples = None
        self._labels = None
        self._sparse = sparse
        self._device = None        # DeviceData cache
        self._host_image = None    # loader's concatenated CSR (one upload)
        self._host_image_sig = None

    def __getitem__(self, item):
        return self._subsets.__getitem__(item)

    def __len__(self):
        return len(self._subsets)

    def __iter__(self):
        return self._subsets.__iter__()

    def append(self, subset, n_samples=None):
        self._subsets.append(subset)
        self._sizes.append(n_samples)
        self._reset_attributes()

    def extend(self, subsets):
        self._subsets.extend(subsets)
        self._sizes.extend([None] * len(subsets))
        self._reset_attributes()

    def subset_size(self, index):
        if self._sizes[index] is None:
            self._sizes[index] = _nrows(self._subsets[index].samples)
        return self._sizes[index]

    def subsets_sizes(self):
        for i in range(len(self)):
            self.subset_size(i)
        return list(self._sizes)

    def min_features(self):
        if self._min_features is None:
            self._compute_min_max()
        return self._min_features

    def max_features(self):
        if self._max_features is None:
            self._compute_min_max()
        return self._max_features

    def collect(self):
        """No-op: there are no futures (kept for API compatibility)."""
        return None

    @property
    def labels(self):
        self._update_labels()
        return self._labels

    @property
    def samples(self):
        self._update_samples()
        return self._samples

    @property
    def sparse(self):
        return self._sparse

    def labels_int32(self):
        """Fast accessor: labels as an int32 ndarray straight from the device
        (no object array).  None if no labels."""
        parts = []
        for s in self._subsets:
            if s._pending is not None:
                src, a, b = s._pending
                parts.append(src.host()[a:b].astype(np.int32))
            elif s._labels is not None:
                parts.append(np.asarray(s._labels).astype(np.int32))
        return np.concatenate(parts) if parts else None

    def _reset_attributes(self):
        self._max_features = None
        self._min_features = None
        self._samples = None
        self._labels = None
        self._device = None
        self._host_image = None

    def _compute_min_max(self):
        mm = []
        for s in self._subsets:
            x = s.samples
            mn, mx = x.min(axis=0), x.max(axis=0)
            if issparse(x):
                mn, mx = mn.toarray()[0], mx.toarray()[0]
            mm.append(np.array([np.asarray(mn), np.asarray(mx)]))
        self._min_features = np.nanmin(mm, axis=0)[0]
        self._max_features = np.nanmax(mm, axis=0)[1]

    def _update_labels(self):
        labels_list = [s.labels for s in self._subsets if s.labels is not None]
        if len(labels_list) > 0:
            self._labels = np.concatenate(labels_list)

    def _update_samples(self):
        if len(self._subsets) > 0:
            self._samples = self._subsets[0].samples
            concat_f = sp.vstack if self._sparse else np.concatenate
            for s in self._subsets[1:]:
                self._samples = concat_f((self._samples, s.samples))

    # -- device residency --------------------------------------------------
    def _signature(self):
        """Identity of the Subsets' sample objects: any reassignment
        (``ds[i].samples = ...``, ``Subset.concatenate``, a new Subset)
        changes it, and so does an in-place write into a device tensor
        (its ``_version`` counter).  Host arrays cannot change in place
        unseen: they are made read-only once uploaded (``_freeze``)."""
        return tuple((id(s.samples), tuple(s.samples.shape),
                      getattr(s.samples, "_version", None))
                     for s in self._subsets)

    def _device_data(self, device=None):
        """The HBM image of the samples, rebuilt when the Subsets' sample
        objects or the requested device changed since the upload (the
        reference reads Subset samples afresh on every call)."""
        from .._device import DeviceData, resolve
        dev = resolve(device) if device is not None else None
        sig = self._signature()
        dd = self._device
        if dd is None or dd.signature != sig or \
                (dev is not None and dd.device != dev):
            if self._host_image is not None and \
                    self._host_image_sig != sig:
                self._host_image = None     # loader image of other samples
            dd = DeviceData(self, device)
            dd.signature = sig
            self._device = dd
            for s in self._subsets:
                _freeze(s.samples)
        return dd

    def _set_host_image(self, image):
        self._host_image = image
        self._host_image_sig = self._signature()

    def _attach_device_labels(self, labels_tensor):
        src = _DeviceLabels(labels_tensor)
        off = 0
        for s in self._subsets:
            n = _nrows(s.samples)
            s._set_device_labels(src, off, off + n)
            off += n
        self._labels = None
