// dkm_b2.h -- device helpers shared by the centres-on-lanes screens
// (k_screen_b2 in dkm_b2.hip, k_screen_sorted in dkm_sorted.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "dkm_internal.h"
#include "dkm_screen.h"

namespace dkm {

constexpr uint32_t PACK2 = 9, PACK2_MASK = (1u << PACK2) - 1;
constexpr int B2_ENT = 3;    // kept (score, centre) per sample besides p
constexpr int B2_RTHR = 4;   // over-full samples a wave tolerates per tile

// min of an MFMA accumulator's 16 values without fminf's NaN
// canonicalisation.  The first step is a compiler-visible VALU read of the
// accumulator (v_med3 against ninf, an opaque -inf): LLVM's hazard
// recognizer does not look at inline-asm operands, so an asm read right
// after the MFMA that writes a[] got no wait states and read stale values
// (k_screen_sorted at 3 K-steps missed kept pairs).  The rest is one asm
// statement, so that the compiler pads no nops between its dependent steps.
template <class V16>
__device__ __forceinline__ float min16(const V16 &a, float ninf) {
  const float m = __builtin_amdgcn_fmed3f(a[0], a[15], ninf);
  float r, t0, t1, t2, t3;
  asm("v_min3_f32 %1, %5, %6, %7\n\t"
      "v_min3_f32 %2, %8, %9, %10\n\t"
      "v_min3_f32 %3, %11, %12, %13\n\t"
      "v_min3_f32 %4, %14, %15, %16\n\t"
      "v_min3_f32 %1, %1, %2, %3\n\t"
      "v_min3_f32 %4, %4, %17, %18\n\t"
      "v_min3_f32 %0, %1, %4, %19"
      : "=v"(r), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3)
      : "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]),
        "v"(a[7]), "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]), "v"(a[12]),
        "v"(a[13]), "v"(a[14]), "v"(m));
  return r;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the workspace pointers the kernels read (the whole WsView as a kernel
// argument kept ~60 SGPRs of unused pointers live: 82 SGPRs spilled)
struct B2View {
  WsHeader *hdr;
  const uint16_t *b1frag;
  const float *cn32f, *cn32;
  int2 *tlist, *clist;
  int4 *nlist;
  int32_t *tcount, *ccount, *ncount;
  // block skipping (IMG_SORTED): mind[p * MIND_LD + cb] = a lower bound on
  // min_{j in block cb, j != p} |c_p - c_j| (dkm_util.hip k_mind); nullptr
  // = no skipping
  const float *mind;
  // DKM_MODE_TRANSLATE: b1frag holds -2 (c - m); the bound's x.c magnitude
  // term takes max ||c - m|| (hdr->umax_bits) instead of max ||c||
  int transl;
};

inline B2View b2_view(const WsView &v, bool sorted, bool transl = false) {
  B2View bv;
  bv.hdr = v.hdr;
  bv.b1frag = transl ? v.b1frag_t : v.b1frag;
  bv.transl = transl ? 1 : 0;
  bv.cn32f = v.cn32f;
  bv.cn32 = v.cn32;
  bv.tlist = v.tlist;
  bv.clist = v.clist;
  bv.nlist = v.nlist;
  bv.tcount = v.tcount;
  bv.ccount = v.ccount;
  bv.ncount = v.ncount;
  bv.mind = sorted ? v.mind : nullptr;
  return bv;
}

// The steady-state threshold pass over the label-sorted image
// (dkm_sorted.hip).  Returns 1 (nothing launched) when it does not apply;
// tiles it cannot finish are listed in `fall` (count *nfall, zeroed here)
// for k_screen_b2's tile-list mode.
int launch_screen_sorted(int64_t n, int d, int k, const WsView &v,
                         int32_t *lab_out, XImage img, int cus, hipStream_t s,
                         int *nseg, int32_t *fall, uint32_t *nfall);

}  // namespace dkm
