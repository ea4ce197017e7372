"""CPU tests of the drop-in boundary: libdkm.so loads and exports every
entry point that include/dkm.h declares (no compute call without a GPU)."""
import ctypes
import os
import re

import pytest

from dislib_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dkm.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dkm_\w+)\s*\(", src)))


def test_header_declares_the_hot_path():
    syms = declared_symbols()
    for s in ("dkm_partial_sum_f64", "dkm_partial_sum_f32", "dkm_predict_f64",
              "dkm_update_centers", "dkm_prepare_centers",
              "dkm_partial_sum_csr_f64", "dkm_predict_csr_f64",
              "dkm_last_error", "dkm_workspace_bytes"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    so = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(so, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_load_and_host_only_calls():
    so = _lib.load()
    assert so.dkm_abi_version() == _lib.ABI_VERSION
    assert so.dkm_workspace_bytes(100, 32, 0) > 100 * 32 * 4
    assert so.dkm_workspace_bytes(0, 32, 0) == 0
    # argument validation happens before any device work
    rc = so.dkm_update_centers(None, None, 0, 0, 0, 0.0, None, None, None)
    assert rc == 10001 and b"bad" in so.dkm_last_error()


def test_missing_library_is_loud(tmp_path):
    with pytest.raises(_lib.DkmError, match="not found"):
        _lib.load(str(tmp_path / "nope.so"))


def test_constants_match_header():
    src = open(HEADER).read()
    consts = dict(re.findall(r"#define (DKM_\w+) (\d+)", src))
    assert int(consts["DKM_ABI_VERSION"]) == _lib.ABI_VERSION
    assert int(consts["DKM_MODE_EXACT"]) == _lib.MODE_EXACT
    assert int(consts["DKM_MODE_SCREEN32"]) == _lib.MODE_SCREEN32
    assert int(consts["DKM_SUMS_F32"]) == _lib.SUMS_F32
    assert int(consts["DKM_SUMS_RECIP"]) == _lib.SUMS_RECIP
    assert int(consts["DKM_PREP_CSR"]) == _lib.PREP_CSR


def test_knn_workspace_covers_both_paths():
    """kNN beyond 32 neighbours takes the two-scan path (32 < kn <= 2048)
    and reruns in passes of 32 when a candidate list overflows, so its
    workspace covers both; beyond 2048 only the passes'.  Host-only."""
    so = _lib.load()
    passes = so.dkm_knn_workspace_bytes(5000, 100000, 32)
    assert passes > 0
    for kn in (33, 1000, 2048):
        two = so.dkm_knn_workspace_bytes(5000, 100000, kn)
        assert two >= passes
        # the two-scan chunk: per query the candidate cap (4096 x 12 B)
        assert two >= 5000 * 4096 * 12
    assert so.dkm_knn_workspace_bytes(5000, 100000, 2049) < \
        so.dkm_knn_workspace_bytes(5000, 100000, 2048)
    # queries past the 8192-query chunk reuse its workspace
    big = so.dkm_knn_workspace_bytes(100000, 100000, 1000)
    assert big < 100000 * 4096 * 12
    assert so.dkm_knn_workspace_bytes(10, 5, 6) == 0   # kn > nx
