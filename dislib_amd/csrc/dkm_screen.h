// dkm_screen.h -- device helpers shared by the MFMA screens (dkm_dense.hip,
// dkm_b2.hip): precision ids, score packing, the rigorous screen bound,
// lane shuffles and the fragment vector types.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dkm {

enum { P_F32 = 0, P_B3 = 1, P_B1 = 2 };

constexpr uint32_t PACK_BITS = 7;
constexpr uint32_t PACK_MASK = (1u << PACK_BITS) - 1;
constexpr int GROUP_BLOCKS = 1 << (PACK_BITS - 2);  // 16-centre blocks/group

template <int PREC>
__device__ __forceinline__ float screen_bound(int d, float xn, float cm,
                                              bool packed) {
  float rel;
  if (PREC == P_F32)
    rel = (d + 6.0f) * 0x1.0p-24f;
  else
    rel = 3.1f * 0x1.0p-16f + (3.0f * d + 6.0f) * 0x1.0p-23f;
  const float s = xn + cm;
  const float mag = 2.0f * xn * cm + cm * cm;
  float b = 2.0f * rel * mag;
  if (packed) b += 0x1.0p-16f * mag;
  b += 16.0f * 0x1.0p-52f * s * s;
  b += (8.0f * d) * 0x1.0p-120f * (s + 1.0f);
  return b * 1.0001f;  // covers the fp32 evaluation of this bound
}

__device__ __forceinline__ float pack_score(float s, uint32_t idx) {
  return __uint_as_float((__float_as_uint(s) & ~PACK_MASK) | idx);
}

// A value the compiler cannot see through (a v_mov it must keep).  The
// screen keeps -inf and the packing mask in VGPRs this way, so that
// med3(a, b, -inf) stays one v_med3 (a visible -inf is folded into fminf,
// which costs two NaN-canonicalising v_max) and the packing stays one
// v_and_or_b32 with the wave-uniform tag in an SGPR.
__device__ __forceinline__ uint32_t opaque_u32(uint32_t v) {
  uint32_t r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}
__device__ __forceinline__ uint32_t opaque_s32(uint32_t v) {
  uint32_t r;
  asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "s"(v));
  return r;
}
// set bits of a wave mask below this lane (v_mbcnt: no 64-bit lane mask)
__device__ __forceinline__ int lane_prefix(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi(
      (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// min without fminf's NaN canonicalisation: the screen's NaN/Inf samples
// are caught by its `sane` test either way.  ninf = opaque -inf.
__device__ __forceinline__ float min_nc(float a, float b, float ninf) {
  return __builtin_amdgcn_fmed3f(a, b, ninf);
}

// The two values x and x' of lane l and lane l ^ (16 or 32), in some order:
// v_permlane{16,32}_swap instead of an LDS ds_bpermute round trip.  Callers
// combine the pair symmetrically, so the order does not matter.
template <int OFF>
__device__ __forceinline__ void pair_xor(float x, float &a, float &b) {
  const uint32_t u = __float_as_uint(x);
  if constexpr (OFF == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
  }
}
template <int OFF>
__device__ __forceinline__ void pair_xor(int x, int &a, int &b) {
  float fa, fb;
  pair_xor<OFF>(__int_as_float(x), fa, fb);
  a = __float_as_int(fa);
  b = __float_as_int(fb);
}

// Per-launch constants of screen_bound: 2B = k_mag * mag + k_s2 * s^2 +
// k_s1 * (s + 1), s = xn + cm, mag = 2 xn cm + cm^2 (same terms, pre-summed;
// the 1.0001 factor covers the fp32 evaluation of either form).
struct BoundK {
  float k_mag, k_s2, k_s1, two_cm, cm2, cm, xn_scale;
};
template <int PREC>
__device__ __forceinline__ BoundK bound_consts(int d, float cm) {
  float rel;
  if (PREC == P_F32)
    rel = (d + 6.0f) * 0x1.0p-24f;
  else
    rel = 3.1f * 0x1.0p-16f + (3.0f * d + 6.0f) * 0x1.0p-23f;
  BoundK k;
  k.k_mag = 2.0f * (2.0f * rel + 0x1.0p-16f) * 1.0001f;
  k.k_s2 = 2.0f * 16.0f * 0x1.0p-52f * 1.0001f;
  k.k_s1 = 2.0f * (8.0f * d) * 0x1.0p-120f * 1.0001f;
  k.two_cm = 2.0f * cm;
  k.cm2 = cm * cm;
  k.cm = cm;
  // v_sqrt_f32 (<= 1 ulp) instead of the correctly rounded sqrtf: 4 more ulp
  k.xn_scale = 1.0f + (d + 8) * 0x1.0p-24f;
  // wave-uniform: keep them in SGPRs (in VGPRs they were spilled, and the
  // reload's vmcnt(0) waited for the prefetched tile)
  auto u = [](float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
  };
  k.k_mag = u(k.k_mag);
  k.k_s2 = u(k.k_s2);
  k.k_s1 = u(k.k_s1);
  k.two_cm = u(k.two_cm);
  k.cm2 = u(k.cm2);
  k.cm = u(k.cm);
  k.xn_scale = u(k.xn_scale);
  return k;
}
// 2B for a sample with fp32 |x|^2 = xx (packed scores)
__device__ __forceinline__ float bound2_fast(const BoundK &k, float xx,
                                            float &xn) {
  xn = __builtin_amdgcn_sqrtf(__builtin_amdgcn_fmed3f(xx, 0x1.0p-100f,
                                                      INFINITY)) *
       k.xn_scale;
  const float s = xn + k.cm;
  const float mag = fmaf(xn, k.two_cm, k.cm2);
  float b = k.k_mag * mag;
  b = fmaf(k.k_s2 * s, s, b);
  return fmaf(k.k_s1, s + 1.0f, b);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

}  // namespace dkm
