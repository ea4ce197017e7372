"""Multi-GPU sharding for the Lloyd iteration (one process per GPU).

Replaces the reference's distribution layer -- PyCOMPSs tasks over Subsets
plus the ``_merge`` arity tree (``cluster/kmeans/base.py:113-117, 137-143,
184-191``) -- with sample sharding and ONE all-reduce per iteration:

* every rank owns a contiguous block of whole Subsets (:func:`shard_range`),
* every rank computes [sums | counts] of its samples into one packed fp64
  buffer of k*(d+1) values (:mod:`dislib_amd._device`),
* ``torch.distributed.all_reduce(SUM)`` -- RCCL over xGMI for the ``nccl``
  backend -- gives every rank the global buffer,
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


def allreduce_sum_(t):
    """In-place SUM over all ranks (RCCL for CUDA tensors on ``nccl``)."""
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(t, op=d.ReduceOp.SUM)
    return t


def broadcast_(t, src=0):
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.broadcast(t, src=src)
    return t


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
