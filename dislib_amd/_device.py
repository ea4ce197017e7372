"""Device residency and thin launch wrappers around ``libdkm.so``.

PyTorch is used only as the device allocator / stream provider: tensors are
HBM buffers whose ``data_ptr()`` goes through the C ABI.  All compute is in
the HIP kernels of ``dislib_amd/csrc``.

``DeviceData`` is the HBM image of a :class:`dislib_amd.data.Dataset`: every
Subset's rows concatenated into one row-major matrix (or one CSR matrix),
with the Subset boundaries kept as row offsets.  It replaces PyCOMPSs'
per-task pickling of Subsets (reference ``cluster/kmeans/base.py:113-115``,
``data/classes.py:298-304``): the data is uploaded once and stays resident
for every Lloyd iteration.
"""
import ctypes

import numpy as np

from . import _lib

# False: never build the sample image (the screen then converts X itself;
# identical labels -- the parity tests switch it through this attribute)
X_IMAGE = True
# HBM left free after an image is allocated
_IMAGE_HEADROOM = 4 << 30
# (what, bytes, host seconds) of every workspace / image allocation: lets a
# caller (bench.py) attribute host time inside a fit to its allocations
ALLOC_LOG = []


def _alloc(what, nbytes, fn):
    import time
    t0 = time.perf_counter()
    out = fn()
    ALLOC_LOG.append((what, int(nbytes), time.perf_counter() - t0))
    return out


def torch():
    import torch as _t
    return _t


def stream_ptr():
    t = torch()
    return ctypes.c_void_p(t.cuda.current_stream().cuda_stream)


def resolve(device=None):
    """A concrete ``torch.device('cuda', i)``: ``None`` / ``'cuda'`` mean the
    current device, so a fit keeps using the GPU it started on."""
    t = torch()
    dev = t.device(device if device is not None else "cuda")
    if dev.type != "cuda":
        raise ValueError("dislib_amd runs on a ROCm GPU, got device %s" % dev)
    if dev.index is None:
        dev = t.device("cuda", t.cuda.current_device())
    return dev


def on(device):
    """Context in which launches go to ``device``: HIP launches and
    ``stream_ptr()`` use the current device, so every entry point that
    touches the data of a Dataset runs inside ``with on(dd.device):``."""
    return torch().cuda.device(device)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class DeviceData:
    """HBM image of a Dataset (dense or CSR)."""

    def __init__(self, dataset, device=None):
        self.device = resolve(device)
        self.images = {}            # sample images by kind (screen_image)
        self._unbuilt = set()       # kinds allocated, not yet built
        self._image_failed = set()
        subsets = list(dataset)
        self.sizes = [int(s.samples.shape[0]) for s in subsets]
        self.offsets = np.concatenate([[0], np.cumsum(self.sizes)]).astype(
            np.int64)
        self.n = int(self.offsets[-1])
        self.d = int(dataset.n_features)
        self.sparse = bool(dataset.sparse)
        if self.sparse:
            self._upload_csr(subsets, getattr(dataset, "_host_image", None))
        else:
            self._upload_dense(subsets)

    # -- dense -------------------------------------------------------------
    def _upload_dense(self, subsets):
        t = torch()
        dev_parts = [s.samples for s in subsets
                     if _is_torch(s.samples)]
        if dev_parts and len(dev_parts) == len(subsets):
            # already device-resident (e.g. bench data): view/concat on device
            xs = [s.samples for s in subsets]
            dt = xs[0].dtype
            self.dtype = np.float32 if dt == t.float32 else np.float64
            X = _adjacent_view(xs)
            if X is None:
                X = xs[0] if len(xs) == 1 else t.cat(xs, 0)
            self.X = X.to(self.device, dtype=(t.float32 if self.dtype ==
                                             np.float32 else t.float64))
            self.X = self.X.contiguous()
            return
        arrs = [np.asarray(s.samples) for s in subsets]
        dts = {a.dtype for a in arrs}
        if dts == {np.dtype(np.float32)}:
            self.dtype = np.float32
        else:
            # fp64 samples; integer samples are exact in fp64 below 2**53
            self.dtype = np.float64
        host = np.concatenate([a.astype(self.dtype, copy=False)
                               for a in arrs]) if arrs else \
            np.zeros((0, self.d), self.dtype)
        host = np.ascontiguousarray(host.reshape(self.n, self.d))
        self.X = t.from_numpy(host).to(self.device)
        self.int_input = any(np.issubdtype(a.dtype, np.integer) for a in arrs)

    # -- CSR ---------------------------------------------------------------
    def _upload_csr(self, subsets, image=None):
        import scipy.sparse as sp
        t = torch()
        if image is not None and image.shape == (self.n, self.d):
            m = image      # file loaders: the parser's concatenated output
        else:
            mats = [sp.csr_matrix(s.samples) for s in subsets]
            m = sp.vstack(mats, format="csr") if mats else \
                sp.csr_matrix((0, self.d))
        # keep each row's stored order: it is the reference's dot order
        assert_all_finite(m.data)
        self.dtype = np.float64
        self.indptr = t.from_numpy(m.indptr.astype(np.int64)).to(self.device)
        self.indices = t.from_numpy(m.indices.astype(np.int32)).to(
            self.device)
        self.data = t.from_numpy(m.data.astype(np.float64)).to(self.device)

    # -- the sample image ---------------------------------------------------
    def screen_image(self, k, mode):
        """The resident bf16 operand image of X (dkm_x_image_*) when the
        screen that (k, d, mode) selects reads one, as (tensor, kind); kept
        with the data, which is immutable (one image per kind).  On first
        use it is only allocated and returned as kind | IMAGE_BUILD: the
        assignment call that receives it builds it (the d <= 32 screen's
        full-sums pass writes it while it converts X anyway) and
        :meth:`image_built` records that.  (None, 0) when not useful,
        disabled (DKM_X_IMAGE=0) or when it would leave less than 4 GiB of
        HBM free."""
        if self.sparse or not X_IMAGE or self.n == 0:
            return None, 0
        so = _lib.lib()
        kind = int(so.dkm_x_image_kind(int(k), self.d, int(mode)))
        if kind == 0:
            return None, 0
        if self.images.get(kind) is not None:
            return self.images[kind], kind | (
                _lib.IMAGE_BUILD if kind in self._unbuilt else 0)
        if kind in self._image_failed:
            return None, 0
        t = torch()
        nb = int(so.dkm_x_image_bytes(self.n, self.d, kind))
        free = t.cuda.mem_get_info(self.device)[0]
        if nb == 0 or nb + _IMAGE_HEADROOM > free:
            self._image_failed.add(kind)
            return None, 0
        img = _alloc("image%d" % kind, nb, lambda: t.empty(
            nb, dtype=t.uint8, device=self.device))
        self.images[kind] = img
        self._unbuilt.add(kind)
        return img, kind | _lib.IMAGE_BUILD

    def image_built(self, kind):
        """The call that received kind | IMAGE_BUILD returned: built."""
        self._unbuilt.discard(kind & ~_lib.IMAGE_BUILD)

    def drop_images(self):
        """Free the resident sample images (up to 16.5 GB at C3): later
        calls convert X in the screen, or build an image again."""
        self.images = {}
        self._unbuilt = set()
        self._image_failed = set()

    # -- helpers -----------------------------------------------------------
    def subset_slices(self):
        return [(int(a), int(b)) for a, b in zip(self.offsets[:-1],
                                                 self.offsets[1:])]


def assert_all_finite(values):
    """The sparse path's input check: the reference computes its sparse
    distances with sklearn's ``pairwise_distances`` (kmeans/base.py:169,
    196; dbscan/classes.py:130), whose ``check_array`` raises ValueError on
    NaN or inf in either operand -- with these messages."""
    v = np.asarray(values)
    if v.size and not np.isfinite(v).all():
        if np.isnan(v).any():
            raise ValueError("Input contains NaN.")
        raise ValueError("Input contains infinity or a value too large for "
                         "dtype('float64').")


def _adjacent_view(xs):
    """One (n, d) view over row blocks that are consecutive slices of one
    device buffer (e.g. ``load_data`` of a device tensor): no copy."""
    t = torch()
    x0 = xs[0]
    if x0.dim() != 2 or x0.stride(1) != 1:
        return None
    ld, es = x0.stride(0), x0.element_size()
    nxt = x0.data_ptr()
    for x in xs:
        if (x.dim() != 2 or x.dtype != x0.dtype or x.stride(1) != 1 or
                x.shape[1] != x0.shape[1] or
                (x.shape[0] > 1 and x.stride(0) != ld) or
                x.data_ptr() != nxt or x.device != x0.device):
            return None
        nxt += x.shape[0] * ld * es
    n = sum(int(x.shape[0]) for x in xs)
    return t.as_strided(x0, (n, x0.shape[1]), (ld, 1))


def _is_torch(x):
    try:
        import torch as _t
        return isinstance(x, _t.Tensor)
    except ImportError:          # pragma: no cover
        return False


class Workspace:
    """Caller-owned scratch for the C ABI (``dkm_workspace_bytes``)."""

    def __init__(self, k, d, n_queue, device):
        t = torch()
        so = _lib.lib()
        self.k, self.d = int(k), int(d)
        self.nbytes = int(so.dkm_workspace_bytes(self.k, self.d,
                                                 int(n_queue)))
        if self.nbytes == 0:
            raise _lib.DkmError("dkm_workspace_bytes: bad k/d")
        self.buf = _alloc("workspace", self.nbytes, lambda: t.zeros(
            self.nbytes, dtype=t.uint8, device=device))
        preload(self.buf.device)

    @property
    def p(self):
        return ctypes.c_void_p(self.buf.data_ptr())


_PRELOADED = set()


def preload(device):
    """Load the library's kernels on ``device`` now (``dkm_preload``), once
    per process and device: the runtime loads each source file's kernels on
    first launch, several ms apiece, which otherwise lands inside the first
    Lloyd iterations."""
    t = torch()
    idx = t.device(device).index
    if idx in _PRELOADED:
        return
    with on(device):
        _lib.check(_lib.lib().dkm_preload(), "dkm_preload")
    _PRELOADED.add(idx)


# ---------------------------------------------------------------------------
# launch wrappers (all stream-ordered on torch's current stream)
# ---------------------------------------------------------------------------
def prepare(C, ws, acc, csr=False):
    so = _lib.lib()
    k, d = C.shape
    _lib.check(so.dkm_prepare_centers(ptr(C), k, d,
                                      _lib.PREP_CSR if csr else 0, ws.p,
                                      ws.nbytes, ptr(acc), stream_ptr()),
               "dkm_prepare_centers")


def _image_for(dd, k, mode, labels, image):
    """The image an assignment call streams: ``image`` = (tensor, kind) when
    the caller owns one (the fit's label-sorted image), else the dataset's
    cached image for the screen (k, mode) selects (labels needed: the
    image screens write labels only)."""
    if image is not None:
        return image
    if labels is None:
        return None, 0
    return dd.screen_image(k, mode)


def partial_sum(dd, C, ws, labels, acc, mode, image=None):
    so = _lib.lib()
    k = C.shape[0]
    if dd.sparse:
        _lib.check(so.dkm_partial_sum_csr_f64(
            ptr(dd.indptr), ptr(dd.indices), ptr(dd.data), dd.n, dd.d,
            ptr(C), k, ws.p, ws.nbytes, ptr(labels), ptr(acc), stream_ptr()),
            "dkm_partial_sum_csr_f64")
        return
    img, kind = _image_for(dd, k, mode, labels, image)
    if img is not None:
        fn = so.dkm_partial_sum_img_f32 if dd.dtype == np.float32 else \
            so.dkm_partial_sum_img_f64
        _lib.check(fn(ptr(dd.X), ptr(img), kind, img.numel(), dd.n, dd.d,
                      dd.X.stride(0), ptr(C), k, ws.p, ws.nbytes, ptr(labels),
                      ptr(acc), mode, stream_ptr()), "dkm_partial_sum_img")
        dd.image_built(kind)
        return
    fn = so.dkm_partial_sum_f32 if dd.dtype == np.float32 else \
        so.dkm_partial_sum_f64
    _lib.check(fn(ptr(dd.X), dd.n, dd.d, dd.X.stride(0), ptr(C), k, ws.p,
                  ws.nbytes, ptr(labels), ptr(acc), mode, stream_ptr()),
               "dkm_partial_sum")


def assign_delta(dd, C, ws, labels, delta, mode, image=None):
    """Incremental assignment: labels in/out, delta +=."""
    so = _lib.lib()
    k = C.shape[0]
    if dd.sparse:
        _lib.check(so.dkm_assign_delta_csr_f64(
            ptr(dd.indptr), ptr(dd.indices), ptr(dd.data), dd.n, dd.d,
            ptr(C), k, ws.p, ws.nbytes, ptr(labels), ptr(delta),
            stream_ptr()), "dkm_assign_delta_csr_f64")
        return
    img, kind = _image_for(dd, k, mode, labels, image)
    if img is not None:
        fn = so.dkm_assign_delta_img_f32 if dd.dtype == np.float32 else \
            so.dkm_assign_delta_img_f64
        _lib.check(fn(ptr(dd.X), ptr(img), kind, img.numel(), dd.n, dd.d,
                      dd.X.stride(0), ptr(C), k, ws.p, ws.nbytes, ptr(labels),
                      ptr(delta), mode, stream_ptr()), "dkm_assign_delta_img")
        dd.image_built(kind)
        return
    fn = so.dkm_assign_delta_f32 if dd.dtype == np.float32 else \
        so.dkm_assign_delta_f64
    _lib.check(fn(ptr(dd.X), dd.n, dd.d, dd.X.stride(0), ptr(C), k, ws.p,
                  ws.nbytes, ptr(labels), ptr(delta), mode, stream_ptr()),
               "dkm_assign_delta")


def sorted_image_ok(dd, k):
    """Does the fit's auto mode on (k, d) run the single-product screen that
    takes a label-sorted image (dkm_x_image_sorted_ok)?"""
    if dd.sparse or dd.n == 0 or not X_IMAGE:
        return False
    # the screen that maintains the image reads 16-B pieces of X's rows
    # (dkm_dense.hip launch_screen `vec`): rows a multiple of 16 B apart,
    # X 16-B aligned (d % 8 == 0 is checked by dkm_x_image_sorted_ok)
    isz = dd.X.element_size()
    if (dd.X.stride(0) * isz) % 16 or dd.X.data_ptr() % 16:
        return False
    so = _lib.lib()
    return (int(so.dkm_x_image_kind(int(k), dd.d, _lib.MODE_AUTO)) ==
            _lib.IMAGE_SINGLE and bool(so.dkm_x_image_sorted_ok(int(k), dd.d)))


def sorted_image(dd, labels, k, ws, old=None, acc=None):
    """dkm_x_image_sorted_*: the sample image with its rows grouped by
    ``labels`` (a fit's current assignment), as (tensor, IMAGE_SORTED); the
    buffer of ``old`` is reused.  (None, 0) when it would leave less than
    4 GiB of HBM free or the workspace's label scratch is shorter than n
    (then ``acc`` is untouched).  With ``acc``: also acc += the [sums |
    counts] of X by ``labels`` (dkm_x_image_sorted_sums_*, one pass over X).
    The image carries a copy of the labels: pass it to every later call
    that updates them (partial_sum / assign_delta ``image=``)."""
    t = torch()
    so = _lib.lib()
    nb = int(so.dkm_x_image_bytes(dd.n, dd.d, _lib.IMAGE_SORTED))
    if old is not None and old[0] is not None and old[0].numel() >= nb:
        img = old[0]
    else:
        free = t.cuda.mem_get_info(dd.device)[0]
        if nb == 0 or nb + _IMAGE_HEADROOM > free:
            return None, 0
        img = _alloc("image_sorted", nb, lambda: t.empty(
            nb, dtype=t.uint8, device=dd.device))
    if int(so.dkm_workspace_bytes(int(k), dd.d, dd.n)) > ws.nbytes:
        return None, 0
    f32 = dd.dtype == np.float32
    if acc is not None:
        fn = so.dkm_x_image_sorted_sums_f32 if f32 else \
            so.dkm_x_image_sorted_sums_f64
        _lib.check(fn(ptr(dd.X), dd.n, dd.d, dd.X.stride(0), ptr(labels),
                      int(k), ws.p, ws.nbytes, ptr(img), nb, ptr(acc),
                      stream_ptr()), "dkm_x_image_sorted_sums")
        return img, _lib.IMAGE_SORTED
    fn = so.dkm_x_image_sorted_f32 if f32 else so.dkm_x_image_sorted_f64
    _lib.check(fn(ptr(dd.X), dd.n, dd.d, dd.X.stride(0), ptr(labels), int(k),
                  ws.p, ws.nbytes, ptr(img), nb, stream_ptr()),
               "dkm_x_image_sorted")
    return img, _lib.IMAGE_SORTED


def label_sums(dd, ws, labels, acc, k):
    """acc += [sums | counts] of X by labels (dkm_label_sums_*)."""
    so = _lib.lib()
    fn = so.dkm_label_sums_f32 if dd.dtype == np.float32 else \
        so.dkm_label_sums_f64
    _lib.check(fn(ptr(dd.X), dd.n, dd.d, dd.X.stride(0), ptr(labels), int(k),
                  ws.p, ws.nbytes, ptr(acc), stream_ptr()), "dkm_label_sums")


def add_(y, x, nonzero=None):
    """y += x; with ``nonzero`` (a device int32 element view): 1 there if any
    x != 0, else 0."""
    so = _lib.lib()
    if nonzero is None:
        _lib.check(so.dkm_add_f64(ptr(y), ptr(x), y.numel(), stream_ptr()),
                   "dkm_add_f64")
    else:
        _lib.check(so.dkm_add_f64_nz(ptr(y), ptr(x), y.numel(), ptr(nonzero),
                                     stream_ptr()), "dkm_add_f64_nz")


def add_dd_(hi, lo, x, nonzero=None):
    """(hi, lo) += x compensated (hi = the rounded running sums)."""
    so = _lib.lib()
    _lib.check(so.dkm_add_f64_dd(ptr(hi), ptr(lo), ptr(x), hi.numel(),
                                 ptr(nonzero), stream_ptr()), "dkm_add_f64_dd")


def predict(dd, C, ws, labels, mode):
    so = _lib.lib()
    k = C.shape[0]
    if dd.sparse:
        _lib.check(so.dkm_predict_csr_f64(
            ptr(dd.indptr), ptr(dd.indices), ptr(dd.data), dd.n, dd.d,
            ptr(C), k, ws.p, ws.nbytes, ptr(labels), stream_ptr()),
            "dkm_predict_csr_f64")
        return
    fn = so.dkm_predict_f32 if dd.dtype == np.float32 else so.dkm_predict_f64
    _lib.check(fn(ptr(dd.X), dd.n, dd.d, dd.X.stride(0), ptr(C), k, ws.p,
                  ws.nbytes, ptr(labels), mode, stream_ptr()),
               "dkm_predict")


def update(acc, C, sums_mode, tol, diff, flag):
    so = _lib.lib()
    k, d = C.shape
    _lib.check(so.dkm_update_centers(ptr(acc), ptr(C), k, d, sums_mode,
                                     float(tol), ptr(diff), ptr(flag),
                                     stream_ptr()), "dkm_update_centers")


def make_blobs(X, row0, n_blobs, seed, box=10.0, std=1.0, blob=None):
    so = _lib.lib()
    n, d = X.shape
    _lib.check(so.dkm_make_blobs_f64(ptr(X), int(row0), n, d, int(n_blobs),
                                     int(seed), float(box), float(std),
                                     ptr(blob), stream_ptr()),
               "dkm_make_blobs_f64")


def rechecked(ws):
    so = _lib.lib()
    out = ctypes.c_int64(0)
    _lib.check(so.dkm_screen_stats(ws.p, ctypes.byref(out), stream_ptr()),
               "dkm_screen_stats")
    return int(out.value)


def screen_counters(ws):
    """(threshold-pass tiles, tiles it decided, centre blocks screened over
    the label-sorted image, sorted-image tiles the steady-state pass handed
    to the general one) accumulated over the workspace's life."""
    so = _lib.lib()
    out = (ctypes.c_int64 * 4)()
    _lib.check(so.dkm_screen_counters(ws.p, out, stream_ptr()),
               "dkm_screen_counters")
    return tuple(int(x) for x in out)


def screen_lists(ws):
    """(re-check list, two-candidate, 3..6-candidate entries, overflowed
    samples) the last single-product screen launch left (diagnostics)."""
    so = _lib.lib()
    out = (ctypes.c_int64 * 4)()
    _lib.check(so.dkm_screen_lists(ws.p, ws.nbytes, out, stream_ptr()),
               "dkm_screen_lists")
    return tuple(int(x) for x in out)
