"""Multi-process (world_size 2, 4 and 8, gloo, CPU) tests of the N>1 path's host
logic: Subset sharding, the packed [sums | counts] all-reduce that replaces
the reference's `_merge` arity tree (cluster/kmeans/base.py:137-143), the
init-centre broadcast, and replicated convergence decisions.  The per-rank
partial sums come from the oracle (the GPU kernels are covered by the -m gpu
parity tests)."""
import functools
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, "ERR %r" % (e,)))
    finally:
        dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r, v in res.items():
        assert not (isinstance(v, str) and v.startswith("ERR")), v
    return res


def _lloyd_emulation(rank, world):
    """Distributed Lloyd loop with oracle partial sums on each rank's shard
    and the product's comm helpers; returns (centres, n_iter)."""
    from sklearn.datasets import make_blobs
    from dislib_amd import _shard
    from dislib_amd.data import load_data
    from oracle import kmeans_oracle as orc
    x, _ = make_blobs(n_samples=3000, n_features=5, centers=4,
                      random_state=4)
    ds = load_data(x, subset_size=250)            # 12 Subsets
    mine = _shard.shard_dataset(ds, rank, world)
    k, d = 4, 5
    C = orc.init_centers(d, False, k, 4)
    it = 0
    while True:
        acc = np.zeros(k * (d + 1))
        for s in mine:
            _, sums, cnt = orc.partial_sum(s.samples, C)
            acc[:k * d] += sums.ravel()
            acc[k * d:] += cnt
        t = torch.from_numpy(acc)
        _shard.allreduce_sum_(t)
        acc = t.numpy()
        old = C.copy()
        cnt = acc[k * d:]
        sums = acc[:k * d].reshape(k, d)
        for c in range(k):
            if cnt[c] != 0:
                C[c] = sums[c] / cnt[c]
        it += 1
        diff = sum(np.linalg.norm(C[c] - old[c]) for c in range(k))
        conv = int(diff < 1e-4 ** 2 or it >= 10)
        assert _shard.agree(conv)
        if conv:
            return C, it


def _lloyd_sizes(rank, world, sizes):
    """The distributed Lloyd loop of _lloyd_emulation over Subsets of the
    given sizes (ragged; fewer Subsets than ranks leaves ranks empty):
    (centres, n_iter, rows owned, labels of the last assignment)."""
    from sklearn.datasets import make_blobs
    from dislib_amd import _shard
    from dislib_amd.data import Dataset, Subset
    from oracle import kmeans_oracle as orc
    x, _ = make_blobs(n_samples=sum(sizes), n_features=5, centers=4,
                      random_state=7)
    ds = Dataset(n_features=5)
    edges = np.concatenate([[0], np.cumsum(sizes)])
    for a, b in zip(edges[:-1], edges[1:]):
        ds.append(Subset(x[a:b]))
    mine = _shard.shard_dataset(ds, rank, world)
    k, d = 4, 5
    C = orc.init_centers(d, False, k, 7)
    _shard.broadcast_(torch.from_numpy(C))
    it = 0
    while True:
        acc = np.zeros(k * (d + 1))
        labs = []
        for s in mine:
            lab, sums, cnt = orc.partial_sum(s.samples, C)
            labs.append(lab)
            acc[:k * d] += sums.ravel()
            acc[k * d:] += cnt
        t = torch.from_numpy(acc)
        _shard.allreduce_sum_(t)      # every rank joins, empty or not
        acc = t.numpy()
        old = C.copy()
        cnt = acc[k * d:]
        sums = acc[:k * d].reshape(k, d)
        for c in range(k):
            if cnt[c] != 0:
                C[c] = sums[c] / cnt[c]
        it += 1
        diff = sum(np.linalg.norm(C[c] - old[c]) for c in range(k))
        conv = int(diff < 1e-4 ** 2 or it >= 10)
        assert _shard.agree(conv)
        if conv:
            rows = sum(s.samples.shape[0] for s in mine)
            return C, it, rows, (np.concatenate(labs) if labs else
                                 np.zeros(0, np.int64))


def _allreduce_matches_global(rank, world):
    from dislib_amd import _shard
    from dislib_amd.data import load_data
    from oracle import kmeans_oracle as orc
    rng = np.random.default_rng(0)
    x = rng.standard_normal((1000, 3))
    C = rng.standard_normal((6, 3))
    ds = load_data(x, subset_size=100)
    mine = _shard.shard_dataset(ds, rank, world)
    acc = np.zeros(6 * 4)
    for s in mine:
        _, sums, cnt = orc.partial_sum(s.samples, C)
        acc[:18] += sums.ravel()
        acc[18:] += cnt
    t = torch.from_numpy(acc.copy())
    _shard.allreduce_sum_(t)
    _, gs, gc = orc.partial_sum(x, C)
    ok_counts = np.array_equal(t.numpy()[18:], gc.astype(float))
    err = np.max(np.abs(t.numpy()[:18] - gs.ravel()))
    return ok_counts, float(err), len(mine)


def _broadcast_init(rank, world):
    from dislib_amd import _shard
    c = torch.from_numpy(np.random.default_rng(rank + 10).random((3, 2)))
    _shard.broadcast_(c)
    return c.numpy().copy()


def test_allreduce_of_partials_equals_global_sums():
    res = _run(_allreduce_matches_global)
    for r, (ok, err, nsub) in res.items():
        assert ok and err < 1e-12 and nsub == 5


def test_broadcast_makes_init_identical():
    res = _run(_broadcast_init)
    assert np.array_equal(res[0], res[1])


def test_distributed_lloyd_matches_single_process():
    from sklearn.datasets import make_blobs
    from oracle import kmeans_oracle as orc
    res = _run(_lloyd_emulation)
    (c0, i0), (c1, i1) = res[0], res[1]
    assert np.array_equal(c0, c1) and i0 == i1      # replicated state
    x, _ = make_blobs(n_samples=3000, n_features=5, centers=4,
                      random_state=4)
    ref = orc.OracleKMeans(n_clusters=4, random_state=4)
    ref.fit([x[i:i + 250] for i in range(0, 3000, 250)])
    assert i0 == ref.n_iter
    np.testing.assert_allclose(c0, ref.centers, rtol=1e-12, atol=1e-12)


def _shard_under_world(rank, world):
    from dislib_amd import _shard
    from dislib_amd.data import load_data
    ds = load_data(np.zeros((70, 2)), subset_size=10)
    m = _shard.shard_dataset(ds)      # rank/world from the process group
    return _shard.world(), len(m)


def test_shard_dataset_under_world():
    res = _run(_shard_under_world)
    assert res[0] == ((0, 2), 3) and res[1] == ((1, 2), 4)


@pytest.mark.parametrize("sizes", [
    [700, 1300, 50, 2100, 900, 1, 1600, 350],     # ragged, 2 per rank
    [3000, 2500, 4000],                           # rank 0 owns nothing
    [10, 20],                                     # two empty ranks
])
def test_world4_ragged_and_empty_shards(sizes):
    """World size 4: ragged Subsets and ranks without rows (which still join
    every all-reduce) give the single-process result: identical centres
    and n_iter on every rank, every row labelled once, the oracle's fit."""
    _check_ragged(sizes, 4)


@pytest.mark.parametrize("sizes", [
    [700, 1300, 50, 2100, 900, 1, 1600, 350, 10, 20, 3000],  # 1-2 per rank
    [3000, 2500, 4000, 5],                        # four empty ranks
])
def test_world8_ragged_and_empty_shards(sizes):
    """World size 8 (the driver's largest scaling run, rehearsed on gloo):
    the same checks as world 4."""
    _check_ragged(sizes, 8)


def _check_ragged(sizes, world):
    from sklearn.datasets import make_blobs
    from oracle import kmeans_oracle as orc
    res = _run(functools.partial(_lloyd_sizes, sizes=sizes), world=world)
    c0, i0, _, _ = res[0]
    for r in range(world):
        assert np.array_equal(res[r][0], c0) and res[r][1] == i0
    assert sum(res[r][2] for r in range(world)) == sum(sizes)
    if len(sizes) < world:
        assert sum(res[r][2] == 0 for r in range(world)) >= world - len(sizes)
    x, _ = make_blobs(n_samples=sum(sizes), n_features=5, centers=4,
                      random_state=7)
    edges = np.concatenate([[0], np.cumsum(sizes)])
    ref = orc.OracleKMeans(n_clusters=4, random_state=7)
    rl = ref.fit([x[a:b] for a, b in zip(edges[:-1], edges[1:])],
                 set_labels=True)
    assert i0 == ref.n_iter
    np.testing.assert_allclose(c0, ref.centers, rtol=1e-12, atol=1e-12)
    lab = np.concatenate([res[r][3] for r in range(world)])
    assert np.array_equal(lab, rl)
