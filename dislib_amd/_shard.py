"""Multi-GPU sharding for the Lloyd iteration (one process per GPU).

Replaces the reference's distribution layer -- PyCOMPSs tasks over Subsets
plus the ``_merge`` arity tree (``cluster/kmeans/base.py:113-117, 137-143,
184-191``) -- with sample sharding and ONE all-reduce per iteration:

* every rank owns a contiguous block of whole Subsets (:func:`shard_range`),
* every rank computes [sums | counts] of its samples into one packed fp64
  buffer of k*(d+1) values (:mod:`dislib_amd._device`),
* one in-place RCCL all-reduce (SUM) over xGMI through libdkm's C ABI
  (``dkm_allreduce_sum_f64``, ``dislib_amd/csrc/dkm_comm.cpp``) gives every
  rank the global buffer -- under a ``nccl`` process group the library's
  own communicator is brought up on first use (the 128-byte RCCL id goes
  from rank 0 to the others through ``torch.distributed``, which is only
  the rendezvous); under ``gloo`` (CPU tests, or several ranks sharing one
  GPU) the same reduction runs through ``torch.distributed.all_reduce``,
* every rank runs the identical centre update, so the centres and the
  convergence decision are replicated without a broadcast.

Only the centre initialisation is broadcast (when ``random_state`` is None
the ranks' draws would differ).  The same functions run over ``gloo`` for the
CPU tests.
"""


def _dist():
    try:
        import torch.distributed as dist
    except ImportError:       # pragma: no cover
        return None
    if not dist.is_available() or not dist.is_initialized():
        return None
    return dist


def world():
    d = _dist()
    return (d.get_rank(), d.get_world_size()) if d is not None else (0, 1)


def active():
    return world()[1] > 1


def shard_range(n_subsets, rank, world_size):
    """Contiguous, balanced block of Subset indices owned by ``rank``."""
    if world_size < 1 or not (0 <= rank < world_size):
        raise ValueError("bad rank/world_size")
    lo = (n_subsets * rank) // world_size
    hi = (n_subsets * (rank + 1)) // world_size
    return lo, hi


def shard_dataset(dataset, rank=None, world_size=None):
    """The Dataset of this rank's Subsets (views of the originals)."""
    from .data.classes import Dataset
    if rank is None or world_size is None:
        rank, world_size = world()
    lo, hi = shard_range(len(dataset), rank, world_size)
    out = Dataset(n_features=dataset.n_features, sparse=dataset.sparse)
    out.extend([dataset[i] for i in range(lo, hi)])
    return out


_COMM = {}   # device index -> True once libdkm's RCCL communicator is up,
             # False when the ranks agreed to use torch.distributed instead


def _dkm_comm(t, d):
    """libdkm's RCCL communicator for ``t``'s device, brought up on first
    use (every rank reaches its first all-reduce together).  None when the
    group is not ``nccl`` or ``t`` is not a GPU tensor.

    The ranks agree on the path BEFORE the collective ncclCommInitRank
    (which blocks until every rank has joined): each rank checks that
    librccl loads, rank 0 also creates the id, and one MIN all-reduce of
    those flags decides for all.  Only after a successful init do the ranks
    agree once more; a rank whose init failed then destroys nothing but its
    own device's communicator."""
    import ctypes

    import torch

    from . import _lib
    if d.get_backend() != "nccl" or not t.is_cuda:
        return None
    dev = t.device.index
    if dev in _COMM:
        return dev if _COMM[dev] else None
    so = _lib.lib()
    rank, world = d.get_rank(), d.get_world_size()

    def all_ok(flag):
        f = torch.tensor([1 if flag else 0], dtype=torch.int32,
                         device=t.device)
        d.all_reduce(f, op=d.ReduceOp.MIN)
        return int(f[0]) == 1

    buf = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
    ok = so.dkm_allreduce_available() == 0
    if rank == 0 and ok:
        ok = so.dkm_allreduce_unique_id(buf) == 0
    if not all_ok(ok):
        _COMM[dev] = False
        return None
    obj = [bytes(buf.raw) if rank == 0 else None]
    d.broadcast_object_list(obj, src=0)
    rc = so.dkm_allreduce_init_rank(obj[0], world, rank, dev)
    if not all_ok(rc == 0):
        so.dkm_allreduce_finalize_device(dev)
        _COMM[dev] = False
        return None
    _COMM[dev] = True
    return dev


def comm_info(device):
    """(ranks, rank) of libdkm's RCCL communicator on ``device``, or None
    when it has none (single process, gloo, or the torch.distributed
    fallback)."""
    import ctypes

    from . import _lib
    if not _COMM.get(device):
        return None
    n, r = ctypes.c_int(0), ctypes.c_int(0)
    _lib.check(_lib.lib().dkm_allreduce_comm_info(device, ctypes.byref(n),
                                                  ctypes.byref(r)),
               "dkm_allreduce_comm_info")
    return n.value, r.value


def finalize():
    """Destroy libdkm's RCCL communicators (before the process group)."""
    if any(_COMM.values()):
        from . import _lib
        _lib.check(_lib.lib().dkm_allreduce_finalize(),
                   "dkm_allreduce_finalize")
    _COMM.clear()


def allreduce_sum_(t):
    """In-place SUM of a contiguous fp64 buffer over all ranks."""
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return t
    dev = _dkm_comm(t, d)
    if dev is None:
        d.all_reduce(t, op=d.ReduceOp.SUM)
        return t
    import ctypes

    import torch

    from . import _lib
    if t.dtype != torch.float64 or not t.is_contiguous():
        raise ValueError("allreduce_sum_: contiguous float64 buffer expected")
    _lib.check(_lib.lib().dkm_allreduce_sum_f64(
        ctypes.c_void_p(t.data_ptr()), t.numel(), dev,
        ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)),
        "dkm_allreduce_sum_f64")
    return t


def broadcast_(t, src=0):
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.broadcast(t, src=src)
    return t


def broadcast_int(value, device=None):
    """Rank 0's integer on every rank (the value itself when not
    distributed).  ``device``: where the collective runs (nccl: the GPU)."""
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return int(value)
    import torch
    dev = device if d.get_backend() == "nccl" else "cpu"
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    d.broadcast(t, src=0)
    return int(t[0])


def agree(flag_value):
    """True iff every rank holds the same integer flag (debug check)."""
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return True
    import torch
    dev = "cuda" if d.get_backend() == "nccl" else "cpu"
    t = torch.tensor([flag_value, -flag_value], dtype=torch.int64, device=dev)
    d.all_reduce(t, op=d.ReduceOp.MAX)
    return int(t[0]) == flag_value and int(-t[1]) == flag_value
