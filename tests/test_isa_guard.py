"""CPU guards on the generated gfx950 ISA and on the build (compiles the
kernels to device assembly with the Makefile's flags; no GPU needed).

* ROCm 7.2 hipcc on gfx950 produced a packed-fp32 (v_pk_fma_f32) operand
  hazard in the screen kernel: lanes 48-63 read a source VGPR already
  overwritten by a later VALU op.  The kernels
  therefore must contain no v_pk_*_f32 instruction.
* hipcc's hazard recognizer does not pad inline-asm operands: an asm VALU
  read of an MFMA result right after the MFMA read stale values (DESIGN.md
  3.12).  tools/isa_hazard.py walks the control flow back from every asm
  VALU operand; no kernel may have such a read.
* The in-tree library must be a product build: no A/B variant object and
  no result-invalidating probe (dkm_build_flags() == 0), and a probe build
  must report itself.

Every source of the Makefile's SRCS is checked (dkm_sorted.hip and
dkm_cand.hip included), compiled once for all checks.
"""
import ctypes
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dislib_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_hazard  # noqa: E402

MK = open(os.path.join(CSRC, "Makefile")).read()


def _flags():
    m = re.search(r"^FLAGS\s*:=\s*(.*?)(?<!\\)\n", MK, re.S | re.M)
    flags = m.group(1).replace("\\\n", " ").replace("$(ARCH)", "gfx950")
    return [f for f in flags.split() if f not in ("-fPIC",)]


def _xflags(src):
    """Per-file XFLAGS_<stem> of the Makefile."""
    m = re.search(r"^XFLAGS_%s\s*:=\s*(.*)$" % re.escape(src[:-4]), MK, re.M)
    return m.group(1).split() if m else []


def _sources():
    m = re.search(r"^SRCS\s*:=\s*(.*?)(?<!\\)\n", MK, re.S | re.M)
    return m.group(1).replace("\\\n", " ").split()


SOURCES = _sources()


def test_sources_come_from_the_makefile():
    for s in ("dkm_sorted.hip", "dkm_cand.hip", "dkm_b2.hip", "dkm_dense.hip",
              "dkm_gemm.hip", "dkm_sparse.hip"):
        assert s in SOURCES


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    """Device assembly of every kernel source, compiled concurrently."""
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not present")
    tmp = tmp_path_factory.mktemp("asm")
    procs = {}
    for src in SOURCES:
        out = tmp / (src + ".s")
        cmd = [HIPCC] + _flags() + _xflags(src) + [
            "-S", "--cuda-device-only", os.path.join(CSRC, src), "-o",
            str(out)]
        procs[src] = (subprocess.Popen(cmd, cwd=CSRC,
                                       stdout=subprocess.DEVNULL,
                                       stderr=subprocess.DEVNULL), out)
    res = {}
    for src, (p, out) in procs.items():
        assert p.wait() == 0, "hipcc -S failed on %s" % src
        res[src] = out.read_text()
    return res


def test_no_packed_fp32_valu(asm):
    """Every kernel source: no v_pk_*_f32."""
    for src, text in asm.items():
        bad = sorted(set(re.findall(r"\bv_pk_\w*f32\b", text)))
        assert not bad, "packed fp32 VALU in %s: %s" % (src, bad)
    assert "-fno-slp-vectorize" in _flags()


def test_no_inline_asm_read_of_an_unwaited_mfma_result(asm):
    """No asm VALU operand is an MFMA destination still in its hazard
    window on any path (tools/isa_hazard.py)."""
    checked = 0
    for src, text in asm.items():
        bad = isa_hazard.check_asm(text)
        assert not bad, "%s: %s" % (src, bad[:5])
        checked += text.count(";;#ASMSTART")
    assert checked > 100          # the screens' asm blocks were seen


KERNEL = r"""
#include <hip/hip_runtime.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void k(const bf16x8 *a, const bf16x8 *b, float *out, float ninf) {
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[threadIdx.x],
                                                b[threadIdx.x], acc, 0, 0, 0);
#if FIXED
  const float m = __builtin_amdgcn_fmed3f(acc[0], acc[15], ninf);
#else
  const float m = ninf;
#endif
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(acc[1]), "v"(acc[2]),
      "v"(m));
  out[threadIdx.x] = r;
}
"""


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not present")
@pytest.mark.parametrize("fixed", [0, 1])
def test_hazard_checker_catches_the_min16_pattern(tmp_path, fixed):
    """The checker flags an asm read right after the MFMA (the bug of
    DESIGN.md 3.12) and passes min16's form (a compiler-visible read of
    the accumulator first)."""
    src = tmp_path / "k.hip"
    src.write_text(KERNEL)
    out = tmp_path / "k.s"
    subprocess.run([HIPCC] + _flags() + ["-DFIXED=%d" % fixed, "-S",
                                         "--cuda-device-only", str(src),
                                         "-o", str(out)], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    bad = isa_hazard.check_asm(out.read_text())
    assert bool(bad) == (not fixed), bad


def test_hazard_checker_follows_branches():
    """Back edges and branch targets are followed; s_nop counts N + 1."""
    text = """
f:
\tv_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], v[0:15]
\ts_cbranch_scc1 .LBB0_2
\ts_nop 3
.LBB0_2:
\t;;#ASMSTART
\tv_min3_f32 v30, v1, v2, v3
\t;;#ASMEND
\ts_endpgm
"""
    bad = isa_hazard.check_asm(text)
    assert bad and bad[0][2] == "v1"
    ok = text.replace("s_nop 3", "s_nop 15").replace(
        "s_cbranch_scc1 .LBB0_2", "s_nop 11")
    assert not isa_hazard.check_asm(ok)


def _lib_flags(path):
    so = ctypes.CDLL(path)
    so.dkm_build_flags.restype = ctypes.c_int
    return so.dkm_build_flags()


def test_product_build_has_no_timing_probe():
    """The in-tree libdkm.so was built without any A/B variant object or
    result-invalidating probe (those exist for csrc/variants*.sh builds)."""
    sys.path.insert(0, ROOT)
    from dislib_amd import _lib
    assert _lib.load().dkm_build_flags() == 0
    for m in ("DKM_AB_", "DKM_DBG_"):
        assert m not in MK


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not present")
@pytest.mark.parametrize("defs,flag", [
    ("-DDKM_AB_SORTED_BSCALE=2", 1 | 2),
    ("-DDKM_AB_SORTED_DBG=3", 1 | 2),
    ("-DDKM_AB_SBS=512", 2)])
def test_probe_build_reports_itself(tmp_path, defs, flag):
    """A library whose dkm_sorted object carries an A/B knob (as
    variants_b2.sh builds it) reports DKM_BUILD_AB_VARIANT, plus
    DKM_BUILD_TIMING_ONLY for the result-invalidating knobs."""
    objs = [os.path.join(CSRC, s[:-4] + ".o") for s in SOURCES
            if s != "dkm_sorted.hip"] + [os.path.join(CSRC, "dkm_io.o"),
                                         os.path.join(CSRC, "dkm_comm.o")]
    if not all(os.path.exists(o) for o in objs):
        pytest.skip("product objects not built (make -C dislib_amd/csrc)")
    obj = tmp_path / "dkm_sorted.o"
    subprocess.run([HIPCC] + _flags() + ["-fPIC"] + _xflags("dkm_sorted.hip")
                   + ["-DDKM_AB_VARIANT=1", defs, "-c",
                      os.path.join(CSRC, "dkm_sorted.hip"), "-o", str(obj)],
                   check=True, cwd=CSRC, stdout=subprocess.DEVNULL,
                   stderr=subprocess.DEVNULL)
    lib = tmp_path / "libdkm_probe.so"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-pthread",
                    "-o", str(lib)] + objs + [str(obj), "-ldl"], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    assert _lib_flags(str(lib)) == flag
