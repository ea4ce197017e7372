"""CPU guard on the generated gfx950 ISA (compiles the kernels to device
assembly with the Makefile's flags; no GPU needed).

ROCm 7.2 hipcc on gfx950 produced a packed-fp32 (v_pk_fma_f32) operand
hazard in the screen kernel: lanes 48-63 read a source VGPR already
overwritten by a later VALU op.  The kernels
therefore must contain no v_pk_*_f32 instruction.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dislib_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def _flags():
    mk = open(os.path.join(CSRC, "Makefile")).read()
    m = re.search(r"^FLAGS\s*:=\s*(.*?)(?<!\\)\n", mk, re.S | re.M)
    flags = m.group(1).replace("\\\n", " ").replace("$(ARCH)", "gfx950")
    return [f for f in flags.split() if f not in ("-fPIC",)]


SOURCES = ["dkm_dense.hip", "dkm_util.hip", "dkm_sparse.hip", "dkm_b2.hip",
           "dkm_gemm.hip", "dkm_sums.hip", "dkm_neighbors.hip"]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not present")
def test_no_packed_fp32_valu(tmp_path):
    """Every kernel source (compiled concurrently): no v_pk_*_f32."""
    procs = {}
    for src in SOURCES:
        out = tmp_path / (src + ".s")
        cmd = [HIPCC] + _flags() + ["-S", "--cuda-device-only",
                                    os.path.join(CSRC, src), "-o", str(out)]
        procs[src] = (subprocess.Popen(cmd, cwd=CSRC,
                                       stdout=subprocess.DEVNULL,
                                       stderr=subprocess.DEVNULL), out)
    for src, (p, out) in procs.items():
        assert p.wait() == 0, "hipcc -S failed on %s" % src
        asm = out.read_text()
        bad = sorted(set(re.findall(r"\bv_pk_\w*f32\b", asm)))
        assert not bad, "packed fp32 VALU in %s: %s" % (src, bad)
    assert "-fno-slp-vectorize" in _flags()


def test_product_build_has_no_timing_probe():
    """The in-tree libdkm.so was built without any result-invalidating A/B
    probe (DKM_AB_B1_PROBE, DKM_DBG_NOCOMPUTE, DKM_DBG_NOLOAD): those exist
    for timing-only variant libraries (csrc/variants.sh)."""
    import sys
    sys.path.insert(0, ROOT)
    from dislib_amd import _lib
    assert _lib.load().dkm_build_flags() == 0
    src = open(os.path.join(CSRC, "Makefile")).read()
    for m in ("DKM_AB_B1_PROBE", "DKM_DBG_NOCOMPUTE", "DKM_DBG_NOLOAD"):
        assert m not in src
