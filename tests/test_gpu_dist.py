"""Multi-process / collective tests on the GPU.

* The RCCL all-reduce behind the C ABI (``dkm_allreduce_*``): world size 1
  through both set-up paths (one box = one GPU, and RCCL refuses two ranks
  on one device).
* The product Lloyd loop at world size 2 and 4: processes on cuda:0 (gloo on
  the CUDA buffers), each fitting its shard with the HIP kernels (world 4:
  ragged Subsets, an empty rank, the per-rank sorted image), against
  the oracle on the whole dataset -- labels bit-exact, centres within 1e-9,
  n_iter, the delta/refresh state kept consistent across ranks (rank 0's
  REFRESH wins) and ``random_state=None`` (rank 0's draw is used).
"""
import ctypes
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
from scipy.sparse import csr_matrix

from oracle import kmeans_oracle as orc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def test_rccl_allreduce_world1_both_setups():
    from dislib_amd import _lib
    so = _lib.lib()
    buf = torch.arange(1000, dtype=torch.float64, device="cuda") * 0.5
    ref = buf.clone()
    devs = (ctypes.c_int * 1)(0)
    _lib.check(so.dkm_allreduce_init(1, devs), "init")
    _lib.check(so.dkm_allreduce_sum_f64(ctypes.c_void_p(buf.data_ptr()),
                                        buf.numel(), 0, _stream()), "sum")
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    # a second communicator on the same device is refused
    assert so.dkm_allreduce_init(1, devs) == 10001
    _lib.check(so.dkm_allreduce_finalize(), "finalize")
    uid = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
    _lib.check(so.dkm_allreduce_unique_id(uid), "unique_id")
    _lib.check(so.dkm_allreduce_init_rank(bytes(uid.raw), 1, 0, 0), "rank")
    _lib.check(so.dkm_allreduce_sum_f64(ctypes.c_void_p(buf.data_ptr()),
                                        buf.numel(), 0, _stream()), "sum")
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    assert so.dkm_allreduce_sum_f64(None, 5, 0, _stream()) == 10001
    _lib.check(so.dkm_allreduce_finalize(), "finalize")
    assert so.dkm_allreduce_sum_f64(ctypes.c_void_p(buf.data_ptr()), 5, 0,
                                    _stream()) == 10001   # no communicator


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_world2(case, tmp_path, backend="gloo", world=2):
    out = str(tmp_path / case)
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(world), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_worker.py"), "--case", case,
           "--out", out, "--backend", backend]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [dict(np.load("%s.%d.npz" % (out, i))) for i in range(world)]


def _backends():
    """gloo always (two ranks on cuda:0); nccl -- one rank per GPU through
    libdkm's RCCL communicator (base.py:137-143's _merge) -- on any box
    with two or more GPUs (skipped on one)."""
    return ["gloo", pytest.param("nccl", marks=pytest.mark.skipif(
        torch.cuda.device_count() < 2, reason="RCCL world 2 needs 2 GPUs"))]


def _check_vs_oracle(case, rs_):
    """The fit of every rank against the oracle on the whole dataset from
    the same initial centres: replicated centres / n_iter / init, labels
    bit-exact (concatenated in rank order), centres within 1e-9."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dist_worker as w
    n, d, blobs, k, sub, iters, tol, rs, refresh = w.CASES[case]
    r0 = rs_[0]
    for r in rs_[1:]:
        assert np.array_equal(r0["centers"], r["centers"])
        assert int(r0["n_iter"]) == int(r["n_iter"])
        if rs is not None:   # with None each rank draws; rank 0's is used
            assert np.array_equal(r0["init"], r["init"])
    x = w.data(case)
    blocks = [x[a:b] for a, b in w.subsets(case)]
    ref = orc.OracleKMeans(n_clusters=k, max_iter=iters, tol=tol,
                           random_state=0)
    real_init = orc.init_centers
    # (the reference wraps sparse initial centres in a CSR matrix)
    orc.init_centers = lambda d_, sparse, *a: (
        csr_matrix(r0["init"]) if sparse else r0["init"].copy())
    try:
        rl = ref.fit(blocks, sparse=case == "csr", set_labels=True)
    finally:
        orc.init_centers = real_init
    assert int(r0["n_iter"]) == ref.n_iter
    assert sum(int(r["nrows"]) for r in rs_) == n
    lab = np.concatenate([r["labels"] for r in rs_])
    assert np.array_equal(lab, rl)
    rc = ref.centers.toarray() if hasattr(ref.centers, "toarray") else \
        ref.centers
    err = np.max(np.abs(r0["centers"] - rc) / np.maximum(np.abs(rc), 1.0))
    assert err <= 1e-9, err


@pytest.mark.parametrize("backend", _backends())
@pytest.mark.parametrize("case", ["dense", "gemm", "none", "ragged", "b2",
                                  "csr"])
def test_world2_fit_predict_vs_oracle(case, backend, tmp_path):
    res = _run_world2(case, tmp_path, backend)
    if backend == "nccl":   # libdkm's communicator spans both ranks
        assert tuple(res[0]["comm"]) == (2, 0)
        assert tuple(res[1]["comm"]) == (2, 1)
    _check_vs_oracle(case, res)


@pytest.mark.parametrize("case", ["ragged4", "empty4", "sorted4"])
def test_world4_fit_predict_vs_oracle(case, tmp_path):
    """Four ranks on cuda:0 (gloo on the CUDA buffers): ragged Subsets, a
    rank with no rows (rank 0, whose REFRESH and initial centres win), and
    the single-product screen with a label-sorted image per rank and the
    delta/refresh state -- every rank's fit against the oracle on the whole
    dataset (base.py:113-117, 137-143)."""
    res = _run_world2(case, tmp_path, "gloo", world=4)
    if case == "empty4":
        assert int(res[0]["nrows"]) == 0 and len(res[0]["labels"]) == 0
    _check_vs_oracle(case, res)
