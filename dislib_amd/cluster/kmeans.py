"""``KMeans`` -- drop-in for ``dislib.cluster.KMeans`` (dislib v0.2.0,
``dislib/cluster/kmeans/base.py:9-147``) running the Lloyd iteration on
MI355X through ``libdkm.so``.

Same constructor, attributes and semantics as the reference:

* ``KMeans(n_clusters=8, max_iter=10, tol=1e-4, arity=50, random_state=None,
  verbose=False)`` stores ``_n_clusters, _max_iter, _tol, _random_state,
  _arity, _verbose``; ``centers`` is None and ``n_iter`` 0 until fitted.
* initial centres are ``np.random.seed(random_state);
  np.random.random((k, d))`` (base.py:155-163), CSR-wrapped for sparse data;
* each iteration assigns every sample to the first nearest centre under the
  reference's exact fp64 arithmetic, sums/counts per cluster, replaces
  non-empty centres by their mean (empty ones keep theirs) and stops when
  ``sum_c ||c_new - c_old|| < tol**2`` or ``n_iter >= max_iter``
  (base.py:98-147) -- so at least one iteration always runs;
* ``fit_predict`` labels come from the last assignment (before the final
  update); ``predict`` labels from ``centers``.

Differences (documented in DESIGN.md): the per-Subset tasks become one fused
kernel launch over the device-resident data, and the partial sums are
accumulated in a different order than the reference's sequential
Subset-then-arity-tree order, so centres agree to ~1e-15 relative instead of
bit-for-bit; ``arity`` is kept but has no effect on the GPU (no reduction
tree).  Extra keyword-only arguments select the assignment arithmetic
(``mode``: "auto" | "exact" | "screen32" | "bf16x3" | "bf16", identical
labels) and the device.
"""
import numpy as np
from scipy.sparse import csr_matrix, issparse

from .. import _lib, _shard

_MODES = {"auto": _lib.MODE_AUTO, "exact": _lib.MODE_EXACT,
          "screen32": _lib.MODE_SCREEN32, "bf16x3": _lib.MODE_BF16X3,
          "bf16": _lib.MODE_BF16}


def _init_centers(n_features, sparse, n_clusters, random_state):
    """Reference ``_init_centers`` (base.py:155-163), host-side."""
    np.random.seed(random_state)
    centers = np.random.random((n_clusters, n_features))
    if sparse:
        centers = csr_matrix(centers)
    return centers


class KMeans:
    """Perform K-means clustering (Lloyd) on MI355X.

    Parameters match ``dislib.cluster.KMeans``; ``mode`` and ``device`` are
    keyword-only extensions.  Under ``torch.distributed`` with more than one
    rank, each rank passes its own shard Dataset (see
    :func:`dislib_amd.shard_dataset`) and the per-iteration [sums | counts]
    are all-reduced (RCCL).
    """

    def __init__(self, n_clusters=8, max_iter=10, tol=1e-4, arity=50,
                 random_state=None, verbose=False, *, mode="auto",
                 device=None):
        self._n_clusters = n_clusters
        self._max_iter = max_iter
        self._tol = tol
        self._random_state = random_state
        self._arity = arity
        self.centers = None
        self.n_iter = 0
        self._verbose = verbose
        if mode not in _MODES:
            raise ValueError("mode must be one of %s" % sorted(_MODES))
        self._mode = mode
        self._device = device
        self._rechecked = 0

    # -- public API (base.py:64-96) ----------------------------------------
    def fit(self, dataset):
        """Compute K-means clustering."""
        self._do_fit(dataset, False)

    def fit_predict(self, dataset):
        """Cluster and set the labels of ``dataset``'s Subsets."""
        self._do_fit(dataset, True)

    def predict(self, dataset):
        """Set each sample's label to its closest centre."""
        if self.centers is None:
            raise ValueError("KMeans.predict before fit")
        from .._device import Workspace, on, predict, prepare, torch
        t = torch()
        _lib.lib()
        dd = dataset._device_data(self._device)
        if dd.n == 0:
            return
        with on(dd.device):
            self._predict_on(dataset, dd, t, Workspace, predict, prepare)

    def _predict_on(self, dataset, dd, t, Workspace, predict, prepare):
        centers = self.centers.toarray() if issparse(self.centers) else \
            np.asarray(self.centers, dtype=np.float64)
        k, d = centers.shape
        if d != dd.d:
            raise ValueError("centers have %d features, data %d" % (d, dd.d))
        if dd.sparse:
            from .._device import assert_all_finite
            assert_all_finite(centers)
        C = t.from_numpy(np.ascontiguousarray(centers)).to(dd.device)
        ws = Workspace(k, d, min(dd.n, 1 << 24), dd.device)
        labels = t.empty(dd.n, dtype=t.int32, device=dd.device)
        prepare(C, ws, None, csr=dd.sparse)
        predict(dd, C, ws, labels, _MODES[self._mode])
        dataset._attach_device_labels(labels)

    # -- Lloyd loop (base.py:98-147) -----------------------------------------
    def _do_fit(self, dataset, set_labels):
        if isinstance(self._random_state, np.random.RandomState):
            raise TypeError("random_state must be an int or None "
                            "(np.random.seed, as in the reference)")
        _lib.lib()                          # no GPU / no libdkm: raise here
        sparse = dataset.sparse
        centers = _init_centers(dataset.n_features, sparse, self._n_clusters,
                                self._random_state)
        state = _Lloyd(dataset, centers.toarray() if sparse else centers,
                       self._tol, set_labels, self._mode, self._device,
                       broadcast_init=self._random_state is None)
        iteration = 0
        while True:
            conv = state.step()
            iteration += 1
            if self._verbose:
                dv = state.criterion()
                crit = np.array([[dv]]) if sparse else np.float64(dv)
                print("Iteration %s - Convergence crit. = %s"
                      % (iteration, crit))
            if conv or iteration >= self._max_iter:
                break
        self._rechecked = state.rechecked()
        host = state.centers_host()
        self.centers = csr_matrix(host) if sparse else host
        self.n_iter = iteration
        state.attach_labels()


# Full recomputation of the running [sums | counts] every REFRESH
# iterations (1 = every iteration).  The running state is compensated
# (dkm_add_f64_dd: hi + lo, TwoSum), so a delta update adds no rounding of
# the old sums: between refreshes the state differs from a fresh
# recomputation only by the deltas' own rounding, <= ~2^-52 x (the moved
# rows' magnitude) per iteration and element -- the error of ONE fresh
# fp64 sum whenever the rows moved since the refresh weigh no more than the
# cluster.  With a plain fp64 state every add also rounded |S_old| (the
# drift grew as REFRESH x 2^-52 |S|), which is what the old 8-iteration
# refresh bounded; the fit tests pin the centres at 1e-9 of the oracle.
# A refresh is also skipped when no delta since the last one held a
# nonzero: then no sample changed cluster and the running sums are
# bit-identical to that last full recomputation.
REFRESH = 64

# The fit's label-sorted sample image (dkm_x_image_sorted_*, DESIGN.md
# 3.11): built from the labels of iteration SORT_AT (the first assignment
# against centres that are means of samples), together with that
# iteration's full sums in one pass over X (dkm_x_image_sorted_sums_*); it
# groups each 32-row tile under one label so the single-product screen skips
# the centre blocks the triangle inequality clears.  Labels are identical
# without it (the tests switch it off through this module attribute).
SORTED_IMAGE = True
SORT_AT = 1
# the first assignment of a label-sorted-image fit: the single-product
# screen over translated centres (DKM_MODE_TRANSLATE) instead of bf16x3.
# Off: at C3 the translated screen still leaves ~40 % of the rows two or
# more candidates against the U[0, 1) centres (its 2B window is 4 x 2^-8
# x |x| max |c - m|), and the iteration took 93 ms against bf16x3's 73.5
# (profiles/r06/c3/r06h_translate_iters.txt).  Labels are identical either
# way; the tests run both.
TRANSLATE_FIRST = False


class _Lloyd:
    """Device state of one fit: resident data, centres, labels, workspace and
    the packed [sums | counts] of the current assignment (``state``).

    ``step()`` is one Lloyd iteration: prepare -> fused assignment (HIP) ->
    all-reduce of the per-rank buffer (RCCL when N > 1) -> centre update +
    criterion (HIP) -> one 4-byte flag read (the reference's per-iteration
    sync, base.py:143).  The fit uses the incremental assignment
    (dkm_assign_delta*: only samples whose label changed move their row
    between clusters; dense and CSR) and recomputes ``state`` from scratch
    (dkm_partial_sum) on the first and every REFRESH-th iteration, which
    bounds the rounding drift of the running sums."""

    def __init__(self, dataset, centers, tol, set_labels, mode="auto",
                 device=None, broadcast_init=False):
        from .._device import Workspace, on, torch
        t = torch()
        self.dataset = dataset
        self.dd = dd = dataset._device_data(device)
        self._on = lambda: on(dd.device)
        self.sparse = dd.sparse
        k, d = centers.shape
        if d != dd.d:
            raise ValueError("centres have %d features, data %d" % (d, dd.d))
        self.k, self.d = k, d
        self.C = t.from_numpy(np.ascontiguousarray(centers, dtype=np.float64)
                              ).to(dd.device)
        if broadcast_init:
            _shard.broadcast_(self.C)     # ranks must start identically
        # label scratch for n samples; a CSR fit's screen keeps 24 B of
        # state per sample there (one centre slice), so 2n lets it run in one
        # chunk (two chunks of n / 2: 6.64-6.71 against 6.45 ms per C5 step,
        # tools/c5_queue_ab.py)
        nq = 2 * dd.n if dd.sparse else dd.n
        self.ws = Workspace(k, d, max(1, min(nq, 1 << 27)), dd.device)
        self.acc = t.empty(k * (d + 1), dtype=t.float64, device=dd.device)
        self.state = t.zeros(k * (d + 1), dtype=t.float64, device=dd.device)
        self.state_lo = t.zeros_like(self.state)   # compensation term
        self.diff = t.zeros(k + 1, dtype=t.float64, device=dd.device)
        # [converged, delta nonzero]: read together once per iteration
        self.flag = t.zeros(2, dtype=t.int32, device=dd.device)
        self.dirty = False     # a delta since the last full recomputation
                               # moved a sample
        self._was_full = True
        self.labels = t.full((max(dd.n, 1),), -1, dtype=t.int32,
                             device=dd.device)
        self.set_labels = set_labels
        self.it = 0
        if self.sparse:
            self.sums_mode = _lib.SUMS_RECIP
        elif dd.dtype == np.float32:
            self.sums_mode = _lib.SUMS_F32
        else:
            self.sums_mode = _lib.SUMS_F64
        self.mode = _MODES[mode]
        self.tol = tol
        if REFRESH < 1:
            raise ValueError("REFRESH must be >= 1, got %d" % REFRESH)
        # every rank must refresh on the same iterations (their delta states
        # are summed): rank 0's setting wins
        self.refresh = _shard.broadcast_int(REFRESH, dd.device)
        from .._device import sorted_image_ok
        # the label-sorted image: auto mode on the single-product shapes
        self.sorting = (SORTED_IMAGE and mode == "auto" and
                        sorted_image_ok(dd, k))
        self.simg = None          # (tensor, IMAGE_SORTED) once built

    def prepare(self):
        """Per-iteration centre data + zeroed accumulator."""
        from .._device import prepare
        with self._on():
            prepare(self.C, self.ws, self.acc, csr=self.sparse)

    def _full(self):
        # iteration 1 recomputes too: its labels are the first against
        # centres that are means of samples, and most samples move (a delta
        # pass would add and subtract most rows: 2x a full pass at C3)
        return self.it <= 1 or (self.it % self.refresh == 0 and self.dirty)

    def partial(self):
        """The hot kernel: fused assignment over all resident samples, full
        partial sums (dkm_partial_sum_*) or incremental (dkm_assign_delta_*).
        """
        from .._device import (assign_delta, label_sums, partial_sum,
                               predict, sorted_image)
        if self.dd.n == 0:
            return
        mode = self.mode
        image = None
        if mode == _lib.MODE_AUTO and self.it == 0:
            # the first iteration scores against the initial centres
            # (U[0, 1)^d, crowded): the plain single-product screen would
            # leave most samples undecided.  The shapes of the label-sorted
            # image take it with the translated centres (DKM_MODE_TRANSLATE:
            # the bf16 error scales with max ||c - mean||, and k_cand2 / the
            # bf16x3 re-screen take what it leaves); the others screen with
            # bf16x3
            if self.sorting and TRANSLATE_FIRST:
                mode = _lib.MODE_BF16 | _lib.MODE_NOHINT | \
                    _lib.MODE_TRANSLATE
            else:
                mode = _lib.MODE_BF16X3
            if self.sorting:
                image = (None, 0)
            else:
                # the image the later (auto) iterations stream: a d <= 32
                # or GEMM-shaped bf16x3 pass writes it as it converts X
                # (DKM_IMAGE_BUILD); other shapes take none here
                image = self.dd.screen_image(self.k, _lib.MODE_AUTO)
                if (image[0] is None or not image[1] & _lib.IMAGE_BUILD or
                        image[1] & ~_lib.IMAGE_BUILD not in
                        (_lib.IMAGE_SPLIT, _lib.IMAGE_GEMM)):
                    image = None   # none, or built: this pass streams X
        elif self.sorting:
            if self.it <= SORT_AT:
                # the labels of the initial centres are poor hints (most
                # samples move): the top-3 pass directly, and no image yet
                # (X is converted in the screen; the sorted image is built
                # from this iteration's labels)
                mode |= _lib.MODE_NOHINT
                image = (None, 0)
            else:
                image = self.simg or (None, 0)
        with self._on():
            if self.sorting and self.it == SORT_AT:
                # labels only, then the sorted image and this iteration's
                # full sums in one pass over X (iteration 1 always recomputes
                # in full: _full())
                lab = self.labels[:self.dd.n]
                predict(self.dd, self.C, self.ws, lab, mode)
                simg = sorted_image(self.dd, lab, self.k, self.ws,
                                    acc=self.acc)
                if simg[0] is None:
                    label_sums(self.dd, self.ws, lab, self.acc, self.k)
                self.simg = simg if simg[0] is not None else None
                return
            if self._full():
                partial_sum(self.dd, self.C, self.ws, self.labels, self.acc,
                            mode, image=image)
            else:
                assign_delta(self.dd, self.C, self.ws, self.labels, self.acc,
                             mode, image=image)

    def assign(self):
        self.prepare()
        self.partial()

    def reduce_update(self):
        from .._device import add_dd_, update
        with self._on():
            _shard.allreduce_sum_(self.acc)
            self._was_full = self._full()
            if self._was_full:
                self.state.copy_(self.acc)
                self.state_lo.zero_()
            else:
                # every rank adds the same all-reduced delta: the ranks'
                # nonzero flags, and so their refresh decisions, agree
                add_dd_(self.state, self.state_lo, self.acc, self.flag[1:])
            update(self.state, self.C, self.sums_mode, self.tol, self.diff,
                   self.flag[:1])
        self.it += 1

    def read_flags(self):
        """The iteration's one device->host read (the reference's
        per-iteration sync, base.py:143): converged?, and whether the delta
        moved a sample (the refresh bookkeeping)."""
        conv, nz = self.flag.tolist()
        if self._was_full:
            self.dirty = False
        elif nz:
            self.dirty = True
        return bool(conv)

    def step(self):
        self.assign()
        self.reduce_update()
        return self.read_flags()

    def criterion(self):
        return float(self.diff[0].item())

    def screened_blocks(self):
        """Diagnostics of the label-sorted image: (tiles threshold-screened,
        centre blocks screened) accumulated over the workspace's life."""
        from .._device import screen_counters
        with self._on():
            return screen_counters(self.ws)

    def rechecked(self):
        from .._device import rechecked
        with self._on():
            return 0 if self.sparse else rechecked(self.ws)

    def centers_host(self):
        return self.C.cpu().numpy()

    def attach_labels(self):
        if self.set_labels and self.dd.n > 0:
            self.dataset._attach_device_labels(self.labels[:self.dd.n])
