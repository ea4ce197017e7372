// dkm_dense.hip -- dense assignment (+ per-cluster sum/count) kernels.
//
// Replaces the per-Subset task `_partial_sum` of dislib
// (cluster/kmeans/base.py:166-181) and `_predict` (:194-201).  One launch
// covers every Subset resident on the device: the partial sums are additive,
// so the per-Subset task split of the reference is not needed on a GPU.
//
// Label arithmetic (bit-exact with the reference):
//   dist_j = sqrt(pairwise_sum((x - c_j)^2))  [np.linalg.norm, base.py:204-5]
//   label  = first j with minimal dist_j      [np.argmin, base.py:173]
//
// Kernels
//   k_exact_reg<MAXD>  lane = sample, x in VGPRs, centres (fp64) in LDS: the
//                      reference arithmetic for every (sample, centre).
//   k_exact_gen        lane = sample, any d, x/centres through the caches.
//   k_screen           MFMA screen: s_j = |c_j|^2 - 2 x.c_j (fp32 or bf16x3
//                      split precision), a rigorous error bound decides
//                      whether the screened winner IS the reference winner;
//                      otherwise the label is left for the re-check.
//   k_recheck_lane     undecided samples, compacted per wave, lane per
//                      sample: fp32 re-screen, then the reference
//                      arithmetic on the remaining candidate centres.
//   k_recheck_exact    the reference arithmetic on all centres (any d, k).
//
// Toolchain note (ROCm 7.2, gfx950): no packed-fp32 VALU (v_pk_fma_f32 and
// friends) in these kernels.  hipcc reused a source VGPR of a v_pk_fma_f32
// as the destination of a VALU op three instructions later, and lanes 48-63
// of the packed op read the clobbered value: ~1e-5 of the labels went wrong
// at random (tools/debug_mismatch.py pinned it to MFMA row 13 = lanes 48-63,
// element 1).  Scalar fmaf + -fno-slp-vectorize; tests check the ISA.
//
// Accumulation (acc = [sums k*d | counts k], fp64):
//   full   every sample adds its row (partial_sum semantics);
//   delta  incremental: labels[] holds the previous assignment; only samples
//          whose label changes add +x to the new and -x to the old cluster
//          (dkm_assign_delta).
// Both go to block-private LDS accumulators (odd row stride, flushed once
// per block) when they fit, else to fp64 global atomics.  Delta in LDS
// matters: in the first iterations most labels move, and global atomics on
// k rows serialise (a 100M x 32, k = 100 delta pass took 650 ms that way).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "dkm_internal.h"

namespace dkm {

constexpr int BLOCK = 256;
constexpr size_t LDS_BUDGET = 80 * 1024;  // per block -> >= 2 blocks / CU

// Accumulation mode bits: AM_ON (accumulate at all), AM_DELTA (incremental:
// only label changes move rows), AM_INLDS (block-private LDS accumulators,
// flushed once per block; else fp64 global atomics).
enum : int { AM_NONE = 0, AM_ON = 1, AM_DELTA = 2, AM_INLDS = 4 };
__host__ __device__ __forceinline__ bool am_full(int m) {
  return (m & (AM_ON | AM_DELTA)) == AM_ON;
}

struct DevInfo {
  int cus = 256;
};
static DevInfo dev_info() {
  static thread_local int cached_dev = -1;
  static thread_local DevInfo info;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return info;
  if (dev != cached_dev) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess)
      info.cus = p.multiProcessorCount;
    cached_dev = dev;
  }
  return info;
}

template <class TX>
__device__ __forceinline__ double ld_x(const TX *p) {
  return (double)(*p);
}

// LDS accumulators: row stride of an odd number of doubles, so that the
// rows of different clusters start in different banks (a 32-double row is
// exactly one 256-B bank row: unpadded, every cluster's feature t sits in
// the same bank and same-feature adds of different clusters serialise).
__host__ __device__ __forceinline__ int lds_stride(int d) {
  return (d & 1) ? d : d + 1;
}
__host__ __device__ __forceinline__ int64_t lds_acc_len(int64_t k, int d) {
  return k * lds_stride(d) + k;
}

__device__ __forceinline__ void lds_add(double *p, double v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Where one kernel's sums go: LDS rows (odd stride) or the global acc.
struct AccTarget {
  double *rows;
  double *cnt;
  int stride;
  bool lds;
  __device__ __forceinline__ void add(int row, int t, double v) const {
    double *p = rows + (int64_t)row * stride + t;
    if (lds)
      lds_add(p, v);
    else
      atomic_add_f64(p, v);
  }
  __device__ __forceinline__ void count(int row, double v) const {
    if (lds)
      lds_add(cnt + row, v);
    else
      atomic_add_f64(cnt + row, v);
  }
};

__device__ __forceinline__ AccTarget acc_target(int amode, double *lds_acc,
                                                double *acc, int64_t k,
                                                int d) {
  if (amode & AM_INLDS) {
    const int ds = lds_stride(d);
    return AccTarget{lds_acc, lds_acc + k * ds, ds, true};
  }
  return AccTarget{acc, acc + k * d, d, false};
}

// Accumulate one sample (lane-per-sample kernels): +x to `label`, and in
// delta mode (only when the label changed) -x from `prev`.
template <class TX>
__device__ __forceinline__ void acc_row_lane(int amode, const AccTarget &a,
                                             int d, int label, int prev,
                                             const TX *xrow) {
  if (!(amode & AM_ON)) return;
  const bool delta = amode & AM_DELTA;
  if (delta && label == prev) return;
  const bool sub = delta && prev >= 0;
  for (int t = 0; t < d; ++t) {
    const double x = ld_x(xrow + t);
    a.add(label, t, x);
    if (sub) a.add(prev, t, -x);
  }
  a.count(label, 1.0);
  if (sub) a.count(prev, -1.0);
}

__device__ __forceinline__ void zero_lds_acc(double *lds_acc, int64_t k,
                                             int d) {
  const int64_t len = lds_acc_len(k, d);
  for (int64_t e = threadIdx.x; e < len; e += blockDim.x) lds_acc[e] = 0.0;
}

__device__ __forceinline__ void flush_lds_acc(const double *lds_acc,
                                              double *acc, int64_t k, int d) {
  const int ds = lds_stride(d);
  const int64_t kd = k * d;
  for (int64_t e = threadIdx.x; e < kd + k; e += blockDim.x) {
    const double v = e < kd ? lds_acc[(e / d) * ds + (e % d)]
                            : lds_acc[k * ds + (e - kd)];
    if (v != 0.0) atomic_add_f64(acc + e, v);
  }
}

// ---------------------------------------------------------------------------
// exact, register-resident x (d <= MAXD), fp64 centres in LDS
// ---------------------------------------------------------------------------
template <int MAXD, class TX>
__global__ void __launch_bounds__(BLOCK)
    k_exact_reg(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                const double *__restrict__ C, int k, int32_t *labels,
                double *acc, int amode) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double *cl = smem;                         // k*d centres
  double *lds_acc = smem + (int64_t)k * d;   // accumulators (AM_INLDS)
  const int64_t kd = (int64_t)k * d;
  for (int64_t e = threadIdx.x; e < kd; e += blockDim.x) cl[e] = C[e];
  if (amode & AM_INLDS) zero_lds_acc(lds_acc, k, d);
  __syncthreads();
  const AccTarget at = acc_target(amode, lds_acc, acc, k, d);

  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += stride) {
    const TX *xr = X + i * ldx;
    double x[MAXD];
#pragma unroll
    for (int t = 0; t < MAXD; ++t) x[t] = t < d ? ld_x(xr + t) : 0.0;
    // argmin over sqrt'd distances, first index on ties (np.argmin); sqrt
    // is monotone, so a centre can only win (or tie) when s < best_s.
    double best_s = exact_sqdist_reg<MAXD>(x, cl, d);
    double best = sqrt(best_s);
    int bi = 0;
    for (int j = 1; j < k; ++j) {
      const double s = exact_sqdist_reg<MAXD>(x, cl + (int64_t)j * d, d);
      if (s < best_s) {
        const double dist = sqrt(s);
        if (dist < best) {
          best = dist;
          bi = j;
        }
        best_s = s;
      }
    }
    const int prev = (amode & AM_DELTA) ? labels[i] : -1;
    if (labels) labels[i] = bi;
    acc_row_lane(amode, at, d, bi, prev, xr);
  }
  if (amode & AM_INLDS) {
    __syncthreads();
    flush_lds_acc(lds_acc, acc, k, d);
  }
}

// ---------------------------------------------------------------------------
// exact, any d: x and centres through the cache hierarchy
// ---------------------------------------------------------------------------
template <class TX>
__device__ __forceinline__ int exact_label_lane(const TX *xr, int d,
                                                const double *C, int k) {
  double best_s = pw_sum(SqDiff<TX>{xr, C}, d);
  double best = sqrt(best_s);
  int bi = 0;
  for (int j = 1; j < k; ++j) {
    const double s = pw_sum(SqDiff<TX>{xr, C + (int64_t)j * d}, d);
    if (s < best_s) {
      const double dist = sqrt(s);
      if (dist < best) {
        best = dist;
        bi = j;
      }
      best_s = s;
    }
  }
  return bi;
}

template <class TX>
__global__ void __launch_bounds__(BLOCK)
    k_exact_gen(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                const double *__restrict__ C, int k, int32_t *labels,
                double *acc, int amode) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double *lds_acc = smem;
  if (amode & AM_INLDS) {
    zero_lds_acc(lds_acc, k, d);
    __syncthreads();
  }
  const AccTarget at = acc_target(amode, lds_acc, acc, k, d);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += stride) {
    const TX *xr = X + i * ldx;
    const int bi = exact_label_lane(xr, d, C, k);
    const int prev = (amode & AM_DELTA) ? labels[i] : -1;
    if (labels) labels[i] = bi;
    acc_row_lane(amode, at, d, bi, prev, xr);
  }
  if (amode & AM_INLDS) {
    __syncthreads();
    flush_lds_acc(lds_acc, acc, k, d);
  }
}

// ---------------------------------------------------------------------------
// MFMA screen.  Score s_j = |c_j|^2 - 2 x.c_j on matrix cores, a rigorous
// bound B on |(s_j + |x|^2) - numpy_dist_j^2|, and the exact re-check of
// every sample whose best two scores are not 2B apart.
//
// Precisions (PREC):
//   P_F32  v_mfma_f32_16x16x4_f32 (exact f32 fma chains) on x32 = fl32(x),
//          c32 = fl32(c).  Bound: conversions 2u|x.c|, the d-term chain
//          d*u*sum|x c|, fp32 |c|^2 (u|c|^2), final fma (u|s|), u = 2^-24.
//   P_B3   v_mfma_f32_16x16x32_bf16 on bf16 hi/lo splits of x32 and c:
//          x.c ~ xh.ch + xh.cl + xl.ch (products exact in fp32); split
//          remainder <= 3.1 * 2^-16 sum|x c| (incl. the x -> x32 rounding),
//          fp32 accumulation of 3d products bounded as (3d + 6) roundings of
//          2^-23 (no assumption about the MFMA's internal adder), fp32
//          |c|^2 and final fma.
// Both doubled for safety, plus numpy's fp64 rounding (16 * 2^-52 (|x| +
// cmax)^2), an absolute underflow floor, and |x.c| <= |x| cmax.  |x| is
// computed in fp32 and inflated (relative error <= (d + 4) 2^-24).
// ---------------------------------------------------------------------------
enum { P_F32 = 0, P_B3 = 1 };

template <int PREC>
__device__ __forceinline__ float screen_bound(int d, float xn, float cm) {
  float rel;
  if (PREC == P_F32)
    rel = (d + 6.0f) * 0x1.0p-24f;
  else
    rel = 3.1f * 0x1.0p-16f + (3.0f * d + 6.0f) * 0x1.0p-23f;
  const float s = xn + cm;
  float b = 2.0f * rel * (2.0f * xn * cm + cm * cm);
  b += 16.0f * 0x1.0p-52f * s * s;
  b += (8.0f * d) * 0x1.0p-120f * (s + 1.0f);
  return b * 1.0001f;  // covers the fp32 evaluation of this bound
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int SB = 256;  // screen block: 4 waves

// Eight consecutive features t0..t0+7 of one row, as fp64.  VEC: d % 8 == 0
// and 16-B aligned rows, so the 8 features are in range iff t0 < d.
template <bool VEC, class TX>
__device__ __forceinline__ void load8(const TX *xr, int t0, int d,
                                      double (&o)[8]) {
  if (VEC) {
    if (t0 < d) {
      if constexpr (sizeof(TX) == 8) {
        const double2 *p = (const double2 *)(xr + t0);
        const double2 a = p[0], b = p[1], c = p[2], e = p[3];
        o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
        o[4] = c.x; o[5] = c.y; o[6] = e.x; o[7] = e.y;
      } else {
        const float4 *p = (const float4 *)(xr + t0);
        const float4 a = p[0], b = p[1];
        o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
        o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
      }
    } else {
#pragma unroll
      for (int m = 0; m < 8; ++m) o[m] = 0.0;
    }
  } else {
#pragma unroll
    for (int m = 0; m < 8; ++m)
      o[m] = (t0 + m < d) ? (double)xr[t0 + m] : 0.0;
  }
}

// One wave = NB blocks of 16 samples per step.  Lane l = (q = l >> 4,
// j = l & 15) holds features ks*32 + 8q + m (m < 8) of sample j of every
// block (4 x 16-B loads per lane per 32 features).  Outside the full-
// accumulation modes the fp64 tile registers are reloaded with the NEXT
// step's rows as soon as they are converted, so one tile is in flight during
// the MFMA/scoring of the current one.  The MFMA output gives lane (q, j)
// the dots of centres cb*16 + 4q + i (i < 4) with sample j; each lane keeps a
// top-2 (fma, cmp, cndmask, med3, min per score), two xor-shuffles merge the
// four lanes of a sample.  lab_out[si] = label, or -(prev + 2) when the
// screen cannot decide (the re-check resolves it; prev = -1 outside
// AM_DELTA).
template <int PREC, int NKS, int NB, bool VEC, class TX>
__global__ void __launch_bounds__(SB)
    k_screen(const TX *__restrict__ X, int64_t n, int d, int64_t ldx, int k,
             WsView v, int32_t *__restrict__ lab_out, double *acc, int amode,
             int64_t base) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nkb = (int)(kpad16(k) / 16);
  // fragment region: nkb*NKS blocks of 2 KB (f32: 8 floats per lane;
  // bf16x3: 8 hi + 8 lo bf16 per lane)
  char *frag = (char *)smem;
  float *cn = (float *)(frag + (int64_t)nkb * NKS * 2048);  // nkb*16
  double *lds_acc = (double *)(cn + nkb * 16);
  {
    const f32x4 *src = (const f32x4 *)(PREC == P_F32 ? (const void *)v.cfrag
                                                     : (const void *)v.bfrag);
    f32x4 *dst = (f32x4 *)frag;
    for (int e = threadIdx.x; e < nkb * NKS * 128; e += SB) dst[e] = src[e];
    for (int e = threadIdx.x; e < nkb * 16; e += SB) cn[e] = v.cnpad[e];
    if (amode & AM_INLDS) zero_lds_acc(lds_acc, k, d);
  }
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  const bool full_acc = am_full(amode);
  const bool delta = amode & AM_DELTA;
  const AccTarget at = acc_target(amode, lds_acc, acc, k, d);
  __syncthreads();

  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & 15;
  const int64_t wv = (int64_t)blockIdx.x * (SB / 64) + (threadIdx.x >> 6);
  const int64_t step = (int64_t)gridDim.x * (SB / 64) * 16 * NB;

  double tile[NB][NKS][8];
  auto load_tile = [&](int64_t s0) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      int64_t si = s0 + 16 * b + j;
      si = si < n ? si : n - 1;  // clamp: always a readable row
      const TX *xr = X + si * ldx;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
        load8<VEC>(xr, ks * 32 + 8 * q, d, tile[b][ks]);
    }
  };

  int64_t s0 = base + wv * 16 * NB;
  if (s0 < n) load_tile(s0);
  for (; s0 < n; s0 += step) {
    // ---- convert the tile (fp64 -> fp32 -> operands), |x|^2 in fp32 ----
    float xx[NB];
    float xf[PREC == P_F32 ? NB : 1][NKS][8];
    bf16x8 xh[PREC == P_B3 ? NB : 1][NKS], xl[PREC == P_B3 ? NB : 1][NKS];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      xx[b] = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const float x32 = (float)tile[b][ks][m];
          xx[b] = fmaf(x32, x32, xx[b]);
          if constexpr (PREC == P_F32) {
            xf[b][ks][m] = x32;
          } else {
            const __bf16 h = (__bf16)x32;
            xh[b][ks][m] = h;
            xl[b][ks][m] = (__bf16)(x32 - (float)h);  // exact subtraction
          }
        }
      xx[b] += __shfl_xor(xx[b], 16, WAVE);
      xx[b] += __shfl_xor(xx[b], 32, WAVE);
    }
    // ---- the next step's rows stream in while this one computes ----
    const int64_t s_next = s0 + step;
    if (!full_acc && s_next < n) load_tile(s_next);

    float b1[NB], b2[NB];
    int i1[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      b1[b] = INFINITY;
      b2[b] = INFINITY;
      i1[b] = 0;
    }
    // MFMA chain of centre block cb into acc[]; consumed one chain later so
    // that the next block's MFMAs overlap this block's VALU scoring.
    auto chain = [&](int cb, f32x4 (&accv)[NB]) {
#pragma unroll
      for (int b = 0; b < NB; ++b) accv[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const char *blk = frag + ((int64_t)cb * NKS + ks) * 2048;
        if constexpr (PREC == P_F32) {
          const f32x4 a0 = *(const f32x4 *)(blk + lane * 32);
          const f32x4 a1 = *(const f32x4 *)(blk + lane * 32 + 16);
          const float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
          for (int m = 0; m < 8; ++m)
#pragma unroll
            for (int b = 0; b < NB; ++b)
              accv[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                  a[m], xf[b][ks][m], accv[b], 0, 0, 0);
        } else {
          const bf16x8 ah = *(const bf16x8 *)(blk + lane * 16);
          const bf16x8 al = *(const bf16x8 *)(blk + 1024 + lane * 16);
#pragma unroll
          for (int b = 0; b < NB; ++b)
            accv[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, xh[b][ks],
                                                              accv[b], 0, 0, 0);
#pragma unroll
          for (int b = 0; b < NB; ++b)
            accv[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, xl[b][ks],
                                                              accv[b], 0, 0, 0);
#pragma unroll
          for (int b = 0; b < NB; ++b)
            accv[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, xh[b][ks],
                                                              accv[b], 0, 0, 0);
        }
      }
    };
    auto score = [&](int cb, const f32x4 (&accv)[NB]) {
      const float4 cn4 = *(const float4 *)(cn + cb * 16 + 4 * q);
      const float cnv[4] = {cn4.x, cn4.y, cn4.z, cn4.w};
      const int cbase = cb * 16 + 4 * q;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // scalar fmaf on purpose: no v_pk_*_f32 anywhere (see the header
        // note on packed-VALU operand hazards; built -fno-slp-vectorize)
        float sc[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) sc[b] = fmaf(-2.f, accv[b][i], cnv[i]);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          // b1 <= b2: new second = med3(b1, b2, s); ties -> b2 == b1
          i1[b] = sc[b] < b1[b] ? cbase + i : i1[b];
          b2[b] = __builtin_amdgcn_fmed3f(b1[b], b2[b], sc[b]);
          b1[b] = fminf(b1[b], sc[b]);
        }
      }
    };
    f32x4 acc_a[NB], acc_b[NB];
    chain(0, acc_a);
    int cb = 0;
    for (; cb + 2 <= nkb; cb += 2) {  // ping-pong: no runtime-indexed arrays
      chain(cb + 1, acc_b);
      score(cb, acc_a);
      if (cb + 2 < nkb) chain(cb + 2, acc_a);
      score(cb + 1, acc_b);
    }
    if (cb < nkb) score(cb, acc_a);  // odd block count: final chain in acc_a
    // merge the top-2 of the four lanes of a sample (first index on ties)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int off = 16; off <= 32; off <<= 1) {
        const float ob1 = __shfl_xor(b1[b], off, WAVE);
        const float ob2 = __shfl_xor(b2[b], off, WAVE);
        const int oi1 = __shfl_xor(i1[b], off, WAVE);
        const bool other = ob1 < b1[b] || (ob1 == b1[b] && oi1 < i1[b]);
        b2[b] = other ? fminf(b1[b], ob2) : fminf(b2[b], ob1);
        i1[b] = other ? oi1 : i1[b];
        b1[b] = other ? ob1 : b1[b];
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int64_t si = s0 + 16 * b + j;
      if (si >= n) continue;
      const float xn = sqrtf(xx[b]) * (1.0f + (d + 4) * 0x1.0p-24f);
      const float B = screen_bound<PREC>(d, xn, cm);
      const bool sane = (xn < 1e18f) && (xn * cm < 1e30f);
      const bool unique = sane && (b2[b] - b1[b] > 2.0f * B);
      const int lab = i1[b];
      int prev = -1;
      if (delta) prev = lab_out[si];  // 16 lanes x 4 B, coalesced
      if (q == 0) lab_out[si] = unique ? lab : -(prev + 2);
      if (!unique) continue;  // label + sums by the re-check
      if (full_acc) {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
          for (int m = 0; m < 8; ++m) {
            const int t = ks * 32 + 8 * q + m;
            if (t < d) at.add(lab, t, tile[b][ks][m]);
          }
        if (q == 0) at.count(lab, 1.0);
      } else if (delta && lab != prev) {
        // rare after the first iterations: reload the row (L2) and move it
        const TX *xr = X + si * ldx;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
          for (int m = 0; m < 8; ++m) {
            const int t = ks * 32 + 8 * q + m;
            if (t < d) {
              const double x = ld_x(xr + t);
              at.add(lab, t, x);
              if (prev >= 0) at.add(prev, t, -x);
            }
          }
        if (q == 0) {
          at.count(lab, 1.0);
          if (prev >= 0) at.count(prev, -1.0);
        }
      }
    }
    if (full_acc && s_next < n) load_tile(s_next);  // the tile was in use
  }
  if (amode & AM_INLDS) {
    __syncthreads();
    flush_lds_acc(lds_acc, acc, k, d);
  }
}

// Exact re-check of the samples the screen left undecided (lab_out < 0,
// encoding the previous label as -(prev + 2)).  Waves scan 64 labels at a
// time (coalesced, no shared counter).
//   k_recheck_lane (d <= 128, fp32 centres fit in LDS): each wave compacts
//     its undecided samples into an LDS list and resolves them 64 at a time,
//     lane = sample.  Stage 1 re-screens in fp32 VALU (x in VGPRs, centres
//     broadcast from LDS) -- the P_F32 arithmetic and bound, ~2^-24 instead
//     of bf16x3's ~2^-16 -- and keeps the label when the best two scores are
//     2B apart.  Otherwise stage 2 runs the reference arithmetic on the
//     candidates only (score <= best + 2B: the reference winner is always
//     among them, and every other centre is strictly farther after sqrt,
//     DESIGN.md 3.1).
//   k_recheck_exact (any d, k): wave per sample, lanes over centres, the
//     reference arithmetic on every centre.
template <class TX>
__device__ __forceinline__ void recheck_accumulate(int amode,
                                                   const AccTarget &at,
                                                   const TX *xr, int d,
                                                   int bi, int prev,
                                                   int lane) {
  if (!(amode & AM_ON)) return;
  const bool delta = amode & AM_DELTA;
  if (delta && bi == prev) return;
  const bool sub = delta && prev >= 0;
  for (int t = lane; t < d; t += 64) {
    const double x = ld_x(xr + t);
    at.add(bi, t, x);
    if (sub) at.add(prev, t, -x);
  }
  if (lane == 0) {
    at.count(bi, 1.0);
    if (sub) at.count(prev, -1.0);
  }
}

__device__ __forceinline__ void recheck_finish_count(
    unsigned long long mine, unsigned long long *blk_count, const WsView &v) {
  if ((threadIdx.x & 63) == 0 && mine)
    __hip_atomic_fetch_add(blk_count, mine, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  if (threadIdx.x == 0 && *blk_count)
    atomicAdd((unsigned long long *)&v.hdr->rechecked_total, *blk_count);
}

constexpr int RL_CAP = 128;  // per-wave list: a full batch + one chunk

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

static size_t recheck_lane_lds(int64_t k, int64_t d) {
  const int64_t dp = round_up(d, 4);
  return (size_t)round_up((k * dp + k) * 4, 8) +
         (size_t)(BLOCK / 64) * RL_CAP * 8;
}

template <int MAXD, bool VEC, class TX>
__global__ void __launch_bounds__(BLOCK)
    k_recheck_lane(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                   int k, WsView v, int32_t *__restrict__ lab_out,
                   double *acc, int amode, int64_t base) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int dp = (int)round_up(d, 4);  // c32 row stride (dkm_util)
  float *cl = (float *)smem;           // fp32 centres, k x dp (zero padded)
  float *cnl = cl + (int64_t)k * dp;   // |c|^2 fp32
  int64_t *lists =
      (int64_t *)((char *)smem + round_up(((int64_t)k * dp + k) * 4, 8));
  double *lds_acc = (double *)(lists + (BLOCK / 64) * RL_CAP);
  __shared__ unsigned long long blk_count;
  if (threadIdx.x == 0) blk_count = 0;
  {
    const f32x4 *src = (const f32x4 *)v.c32;
    f32x4 *dst = (f32x4 *)cl;
    for (int64_t e = threadIdx.x; e < (int64_t)k * dp / 4; e += BLOCK)
      dst[e] = src[e];
    for (int e = threadIdx.x; e < k; e += BLOCK) cnl[e] = v.cn32[e];
  }
  if (amode & AM_INLDS) zero_lds_acc(lds_acc, k, d);
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  const AccTarget at = acc_target(amode, lds_acc, acc, k, d);
  __syncthreads();

  const int lane = threadIdx.x & 63;
  int64_t *wl = lists + (threadIdx.x >> 6) * RL_CAP;

  // one undecided sample per lane
  auto resolve = [&](int64_t i) {
    const int prev = -lab_out[i] - 2;
    const TX *xr = X + i * ldx;
    float xf[MAXD];
    float xx = 0.f;
#pragma unroll
    for (int b = 0; b < MAXD / 8; ++b) {
      double o[8];
      if (8 * b < d) {
        load8<VEC>(xr, 8 * b, d, o);
      } else {
#pragma unroll
        for (int m = 0; m < 8; ++m) o[m] = 0.0;
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        xf[8 * b + m] = (float)o[m];
        xx = fmaf(xf[8 * b + m], xf[8 * b + m], xx);
      }
    }
    // fp32 score of centre j: fma chain over features (padding adds 0 * 0)
    auto score = [&](int j) {
      const float *cr = cl + (int64_t)j * dp;
      float dot = 0.f;
#pragma unroll
      for (int t4 = 0; t4 < MAXD / 4; ++t4) {
        if (4 * t4 < dp) {
          const f32x4 c4 = *(const f32x4 *)(cr + 4 * t4);
          dot = fmaf(xf[4 * t4 + 0], c4.x, dot);
          dot = fmaf(xf[4 * t4 + 1], c4.y, dot);
          dot = fmaf(xf[4 * t4 + 2], c4.z, dot);
          dot = fmaf(xf[4 * t4 + 3], c4.w, dot);
        }
      }
      return fmaf(-2.f, dot, cnl[j]);
    };
    float b1 = INFINITY, b2 = INFINITY;
    int i1 = 0;
    for (int j = 0; j < k; ++j) {
      const float sc = score(j);
      i1 = sc < b1 ? j : i1;
      b2 = __builtin_amdgcn_fmed3f(b1, b2, sc);
      b1 = fminf(b1, sc);
    }
    const float xn = sqrtf(xx) * (1.0f + (d + 4) * 0x1.0p-24f);
    const float B = screen_bound<P_F32>(d, xn, cm);
    const bool sane = (xn < 1e18f) && (xn * cm < 1e30f) && (b1 < 1e30f);
    int bi = i1;
    if (!(sane && b2 - b1 > 2.0f * B)) {
      const float lim = b1 + 2.0f * B;
      double best = INFINITY;
      bi = -1;
      for (int j = 0; j < k; ++j) {
        if (sane && !(score(j) <= lim)) continue;
        const SqDiffT<TX> f{xr, v.ct64 + j, (int64_t)k};
        const double dist = sqrt(pw_leaf(f, 0, d));
        if (dist < best || bi < 0) {
          best = dist;
          bi = j;
        }
      }
    }
    lab_out[i] = bi;
    if (!(amode & AM_ON)) return;
    const bool delta = amode & AM_DELTA;
    if (delta && bi == prev) return;
    const bool sub = delta && prev >= 0;
    for (int t = 0; t < d; ++t) {
      const double x = ld_x(xr + t);
      at.add(bi, t, x);
      if (sub) at.add(prev, t, -x);
    }
    at.count(bi, 1.0);
    if (sub) at.count(prev, -1.0);
  };

  // Scan: 4 labels per lane (int4), 256 per wave step, the next step's
  // labels in flight while this one resolves (a wave's list only holds
  // samples of steps it has already scanned, so the prefetch is never stale).
  // a0 aligns the int4 loads; lanes outside [base, n) read nothing.
  const int64_t wv = (int64_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
  const int64_t nwv = (int64_t)gridDim.x * (BLOCK / 64);
  const int64_t a0 =
      base - (int64_t)(((uintptr_t)(lab_out + base) >> 2) & 3);
  auto load4 = [&](int64_t c0, int (&o)[4]) {
    const int64_t i0 = c0 + 4 * lane;
    if (i0 >= base && i0 + 3 < n) {
      const int4 q4 = *(const int4 *)(lab_out + i0);
      o[0] = q4.x; o[1] = q4.y; o[2] = q4.z; o[3] = q4.w;
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        o[c] = (i0 + c >= base && i0 + c < n) ? lab_out[i0 + c] : 0;
    }
  };
  unsigned long long mine = 0;
  int cnt = 0;  // wave-uniform list length
  int cur[4] = {0, 0, 0, 0};
  int64_t c0 = a0 + wv * 256;
  if (c0 < n) load4(c0, cur);
  for (; c0 < n; c0 += nwv * 256) {
    int nxt[4] = {0, 0, 0, 0};
    if (c0 + nwv * 256 < n) load4(c0 + nwv * 256, nxt);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const unsigned long long mask = __ballot(cur[c] < 0);
      if (cur[c] < 0)
        wl[cnt + __popcll(mask & ((1ull << lane) - 1))] = c0 + 4 * lane + c;
      const int add = __popcll(mask);
      mine += add;
      cnt += add;
      if (cnt >= 64) {
        wave_lds_sync();
        resolve(wl[lane]);
        const int rem = cnt - 64;
        const int64_t tail = lane < rem ? wl[64 + lane] : 0;
        wave_lds_sync();
        if (lane < rem) wl[lane] = tail;
        cnt = rem;
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) cur[c] = nxt[c];
  }
  wave_lds_sync();
  if (lane < cnt) resolve(wl[lane]);
  recheck_finish_count(mine, &blk_count, v);
  if (amode & AM_INLDS) flush_lds_acc(lds_acc, acc, k, d);
}

template <bool SMALL, class TX>
__global__ void __launch_bounds__(BLOCK)
    k_recheck_exact(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                    int k, WsView v, int32_t *__restrict__ lab_out,
                    double *acc, int amode, int64_t base) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double *lds_acc = smem;
  __shared__ unsigned long long blk_count;
  if (threadIdx.x == 0) blk_count = 0;
  if (amode & AM_INLDS) zero_lds_acc(lds_acc, k, d);
  const AccTarget at = acc_target(amode, lds_acc, acc, k, d);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wv = (int64_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
  const int64_t nwv = (int64_t)gridDim.x * (BLOCK / 64);
  unsigned long long mine = 0;
  for (int64_t c0 = base + wv * 64; c0 < n; c0 += nwv * 64) {
    const int64_t li = c0 + lane;
    const int lv = li < n ? lab_out[li] : 0;
    unsigned long long mask = __ballot(lv < 0);
    mine += __popcll(mask);
    while (mask) {
      const int bit = __ffsll((long long)mask) - 1;
      mask &= mask - 1;
      const int64_t i = c0 + bit;
      const int prev = -__shfl(lv, bit, WAVE) - 2;
      const TX *xr = X + i * ldx;
      double best = INFINITY;
      int bi = 0x7fffffff;  // lanes without a centre never win
      for (int jc = lane; jc < k; jc += 64) {
        const SqDiffT<TX> f{xr, v.ct64 + jc, (int64_t)k};
        const double dist = sqrt(SMALL ? pw_leaf(f, 0, d) : pw_sum(f, d));
        if (dist < best || bi == 0x7fffffff) {
          best = dist;
          bi = jc;
        }
      }
      wave_argmin(best, bi);
      if (lane == 0) lab_out[i] = bi;
      recheck_accumulate(amode, at, xr, d, bi, prev, lane);
    }
  }
  recheck_finish_count(mine, &blk_count, v);
  if (amode & AM_INLDS) flush_lds_acc(lds_acc, acc, k, d);
}

__global__ void k_add(double *__restrict__ y, const double *__restrict__ x,
                      int64_t n) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x)
    y[e] += x[e];
}

// ---------------------------------------------------------------------------
// host dispatch
// ---------------------------------------------------------------------------
static int pick_maxd(int d) {
  if (d <= 8) return 8;
  if (d <= 16) return 16;
  if (d <= 32) return 32;
  if (d <= 64) return 64;
  return 0;
}

static unsigned grid_for(int64_t n, const void *kern, int block, size_t lds) {
  int per_cu = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block,
                                                   lds) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int64_t cap = (int64_t)dev_info().cus * per_cu;
  const int64_t need = (n + block - 1) / block;
  return (unsigned)std::max<int64_t>(1, std::min(need, cap));
}

// acc_kind: 0 = none (predict), 1 = full accumulation, 2 = delta
static int acc_mode(int acc_kind, bool lds_fits) {
  if (acc_kind == 0) return AM_NONE;
  return AM_ON | (acc_kind == 2 ? AM_DELTA : 0) | (lds_fits ? AM_INLDS : 0);
}

template <class TX>
static int launch_exact(const TX *X, int64_t n, int d, int64_t ldx,
                        const double *C, int k, int32_t *labels, double *acc,
                        int acc_kind, hipStream_t s) {
  const int64_t kd = (int64_t)k * d;
  const size_t c_bytes = (size_t)kd * 8;
  const size_t a_bytes = (size_t)lds_acc_len(k, d) * 8;
  const int maxd = pick_maxd(d);
  const bool creg = maxd > 0 && c_bytes <= LDS_BUDGET;
  const size_t base = creg ? c_bytes : 0;
  const int amode = acc_mode(acc_kind, base + a_bytes <= LDS_BUDGET);
  const size_t lds = base + ((amode & AM_INLDS) ? a_bytes : 0);
  if (creg) {
#define DKM_EXACT_CASE(M)                                                   \
  case M: {                                                                 \
    const void *kf = (const void *)k_exact_reg<M, TX>;                      \
    unsigned g = grid_for(n, kf, BLOCK, lds);                               \
    k_exact_reg<M, TX><<<g, BLOCK, lds, s>>>(X, n, d, ldx, C, k, labels,    \
                                             acc, amode);                   \
    break;                                                                  \
  }
    switch (maxd) {
      DKM_EXACT_CASE(8)
      DKM_EXACT_CASE(16)
      DKM_EXACT_CASE(32)
      DKM_EXACT_CASE(64)
    }
#undef DKM_EXACT_CASE
  } else {
    const void *kf = (const void *)k_exact_gen<TX>;
    unsigned g = grid_for(n, kf, BLOCK, lds);
    k_exact_gen<TX><<<g, BLOCK, lds, s>>>(X, n, d, ldx, C, k, labels, acc,
                                          amode);
  }
  return check_launch("exact assignment");
}

static size_t screen_lds_fixed(int64_t k, int64_t d) {
  // fragments (kpad16 x dpad32 x 4 B, both precisions) + |c|^2
  return (size_t)(kpad16(k) * dpad32(d) * 4 + kpad16(k) * 4);
}

static bool screen_ok(int64_t k, int64_t d) {
  return k >= 2 && d <= 128 && screen_lds_fixed(k, d) <= LDS_BUDGET;
}

template <int PREC, int NKS, int NB, bool VEC, class TX>
static int launch_screen_t(const TX *X, int64_t end, int d, int64_t ldx,
                           int k, const WsView &v, int32_t *lab_out,
                           double *acc, int amode, int64_t base, size_t lds,
                           hipStream_t s) {
  const void *kf = (const void *)k_screen<PREC, NKS, NB, VEC, TX>;
  int per_cu = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, SB, lds) !=
          hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int64_t cap = (int64_t)dev_info().cus * per_cu;
  const int64_t per_block = 16 * NB * (SB / 64);
  const int64_t need = (end - base + per_block - 1) / per_block;
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min(need, cap));
  k_screen<PREC, NKS, NB, VEC, TX><<<g, SB, lds, s>>>(X, end, d, ldx, k, v,
                                                      lab_out, acc, amode,
                                                      base);
  return check_launch("screen assignment");
}

template <int PREC, bool VEC, class TX>
static int launch_screen_nks(const TX *X, int64_t end, int d, int64_t ldx,
                             int k, const WsView &v, int32_t *lab_out,
                             double *acc, int amode, int64_t base, size_t lds,
                             hipStream_t s) {
  switch (dpad32(d) / 32) {
    case 1:
      return launch_screen_t<PREC, 1, 2, VEC, TX>(X, end, d, ldx, k, v,
                                                  lab_out, acc, amode, base,
                                                  lds, s);
    case 2:
      return launch_screen_t<PREC, 2, 1, VEC, TX>(X, end, d, ldx, k, v,
                                                  lab_out, acc, amode, base,
                                                  lds, s);
    case 3:
      return launch_screen_t<PREC, 3, 1, VEC, TX>(X, end, d, ldx, k, v,
                                                  lab_out, acc, amode, base,
                                                  lds, s);
    case 4:
      return launch_screen_t<PREC, 4, 1, VEC, TX>(X, end, d, ldx, k, v,
                                                  lab_out, acc, amode, base,
                                                  lds, s);
  }
  return fail(DKM_E_ARG, "screen: d too large");
}

template <int MAXD, bool VEC, class TX>
static void launch_recheck_lane_t(unsigned g, size_t lds, hipStream_t s,
                                  const TX *X, int64_t end, int d,
                                  int64_t ldx, int k, const WsView &v,
                                  int32_t *lab_out, double *acc, int amode,
                                  int64_t base) {
  k_recheck_lane<MAXD, VEC, TX><<<g, BLOCK, lds, s>>>(X, end, d, ldx, k, v,
                                                       lab_out, acc, amode,
                                                       base);
}

template <int MAXD, class TX>
static const void *recheck_lane_fn(bool vec) {
  return vec ? (const void *)k_recheck_lane<MAXD, true, TX>
             : (const void *)k_recheck_lane<MAXD, false, TX>;
}

template <class TX>
static int launch_recheck(const TX *X, int64_t end, int d, int64_t ldx, int k,
                          const WsView &v, int32_t *lab_out, double *acc,
                          int acc_kind, bool vec, int64_t base,
                          hipStream_t s) {
  const size_t a_bytes = (size_t)lds_acc_len(k, d) * 8;
  const size_t fb = recheck_lane_lds(k, d);
  const bool lane = d <= 128 && fb <= LDS_BUDGET;
  const int maxd = d <= 32 ? 32 : d <= 64 ? 64 : 128;
  const size_t fixed = lane ? fb : 0;
  const int amode = acc_mode(acc_kind, fixed + a_bytes <= LDS_BUDGET);
  const size_t lds = fixed + ((amode & AM_INLDS) ? a_bytes : 0);
  const bool small = d <= 128;
  const void *kf =
      !lane   ? (small ? (const void *)k_recheck_exact<true, TX>
                       : (const void *)k_recheck_exact<false, TX>)
      : maxd == 32 ? recheck_lane_fn<32, TX>(vec)
      : maxd == 64 ? recheck_lane_fn<64, TX>(vec)
                   : recheck_lane_fn<128, TX>(vec);
  int per_cu = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, BLOCK, lds) !=
          hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int64_t waves = (end - base + 3 + (lane ? 255 : 63)) / (lane ? 256 : 64);
  const unsigned g = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>((int64_t)dev_info().cus * per_cu,
                           (waves + BLOCK / 64 - 1) / (BLOCK / 64)));
  if (lane) {
#define DKM_RL(M)                                                            \
  (vec ? launch_recheck_lane_t<M, true, TX>(g, lds, s, X, end, d, ldx, k, v, \
                                            lab_out, acc, amode, base)       \
       : launch_recheck_lane_t<M, false, TX>(g, lds, s, X, end, d, ldx, k,   \
                                             v, lab_out, acc, amode, base))
    if (maxd == 32)
      DKM_RL(32);
    else if (maxd == 64)
      DKM_RL(64);
    else
      DKM_RL(128);
#undef DKM_RL
  } else if (small) {
    k_recheck_exact<true, TX><<<g, BLOCK, lds, s>>>(X, end, d, ldx, k, v,
                                                     lab_out, acc, amode, base);
  } else {
    k_recheck_exact<false, TX><<<g, BLOCK, lds, s>>>(X, end, d, ldx, k, v,
                                                      lab_out, acc, amode, base);
  }
  return check_launch("exact re-check");
}

// Screen + exact re-check over [0, n).  Labels go to `labels` when given,
// else to the workspace scratch (queue region), in chunks of its capacity.
template <class TX>
static int launch_screen(int prec, const TX *X, int64_t n, int d,
                         int64_t ldx, int k, const WsView &v, size_t wsb,
                         int32_t *labels, double *acc, int acc_kind,
                         hipStream_t s) {
  const size_t fixed = (size_t)((const char *)v.queue - (const char *)v.hdr);
  const int64_t nq =
      std::min<int64_t>((int64_t)((wsb - fixed) / 4), INT32_MAX);
  if (!labels && nq < 1)
    return fail(DKM_E_WORKSPACE, "screen: no label scratch");
  const int64_t chunk = labels ? n : nq;
  const size_t fb = screen_lds_fixed(k, d);
  const size_t a_bytes = (size_t)lds_acc_len(k, d) * 8;
  const int amode = acc_mode(acc_kind, fb + a_bytes <= LDS_BUDGET);
  const size_t lds = fb + ((amode & AM_INLDS) ? a_bytes : 0);
  const bool vec = (d % 8 == 0) && (ldx % (16 / (int64_t)sizeof(TX)) == 0) &&
                   (((uintptr_t)X % 16) == 0);
  for (int64_t base = 0; base < n; base += chunk) {
    const int64_t end = std::min(n, base + chunk);
    int32_t *lab_out = labels ? labels : v.queue - base;
    int r;
    if (prec == P_F32)
      r = vec ? launch_screen_nks<P_F32, true, TX>(X, end, d, ldx, k, v,
                                                   lab_out, acc, amode, base,
                                                   lds, s)
              : launch_screen_nks<P_F32, false, TX>(X, end, d, ldx, k, v,
                                                    lab_out, acc, amode, base,
                                                    lds, s);
    else
      r = vec ? launch_screen_nks<P_B3, true, TX>(X, end, d, ldx, k, v,
                                                  lab_out, acc, amode, base,
                                                  lds, s)
              : launch_screen_nks<P_B3, false, TX>(X, end, d, ldx, k, v,
                                                   lab_out, acc, amode, base,
                                                   lds, s);
    if (r) return r;
    if ((r = launch_recheck<TX>(X, end, d, ldx, k, v, lab_out, acc,
                                acc_kind, vec, base, s)))
      return r;
  }
  return 0;
}

template <class TX>
static int assign(const TX *X, int64_t n, int64_t d, int64_t ldx,
                  const double *C, int64_t k, const void *ws, size_t wsb,
                  int32_t *labels, double *acc, int acc_kind, int mode,
                  void *stream, const char *who) {
  if (n < 0 || d <= 0 || k <= 0 || ldx < d)
    return fail(DKM_E_ARG, std::string(who) + ": bad n/d/k/ldx");
  if (d > INT32_MAX || k > INT32_MAX)
    return fail(DKM_E_ARG, std::string(who) + ": d/k too large");
  if (n == 0) return 0;
  if (!X || !C) return fail(DKM_E_ARG, std::string(who) + ": NULL X/C");
  if (!labels && !acc)
    return fail(DKM_E_ARG, std::string(who) + ": nothing to write");
  hipStream_t s = (hipStream_t)stream;
  if (mode == DKM_MODE_AUTO)
    mode = screen_ok(k, d) ? DKM_MODE_SCREEN_BF16X3 : DKM_MODE_EXACT;
  if (mode == DKM_MODE_EXACT)
    return launch_exact<TX>(X, n, (int)d, ldx, C, (int)k, labels, acc,
                            acc_kind, s);
  if (mode == DKM_MODE_SCREEN32 || mode == DKM_MODE_SCREEN_BF16X3) {
    if (!screen_ok(k, d))
      return launch_exact<TX>(X, n, (int)d, ldx, C, (int)k, labels, acc,
                              acc_kind, s);
    WsView v;
    if (int r = ws_view(ws, wsb, k, d, &v)) return r;
    return launch_screen<TX>(mode == DKM_MODE_SCREEN32 ? P_F32 : P_B3, X, n,
                             (int)d, ldx, (int)k, v, wsb, labels, acc,
                             acc_kind, s);
  }
  return fail(DKM_E_ARG, std::string(who) + ": bad mode");
}

}  // namespace dkm

using namespace dkm;

extern "C" {

int dkm_partial_sum_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                        const double *C, int64_t k, const void *ws,
                        size_t ws_bytes, int32_t *labels, double *acc,
                        int mode, void *stream) {
  if (!acc) return fail(DKM_E_ARG, "partial_sum: acc is NULL");
  return assign<double>(X, n, d, ldx, C, k, ws, ws_bytes, labels, acc, 1,
                        mode, stream, "dkm_partial_sum_f64");
}

int dkm_partial_sum_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                        const double *C, int64_t k, const void *ws,
                        size_t ws_bytes, int32_t *labels, double *acc,
                        int mode, void *stream) {
  if (!acc) return fail(DKM_E_ARG, "partial_sum: acc is NULL");
  return assign<float>(X, n, d, ldx, C, k, ws, ws_bytes, labels, acc, 1,
                       mode, stream, "dkm_partial_sum_f32");
}

int dkm_assign_delta_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                         const double *C, int64_t k, const void *ws,
                         size_t ws_bytes, int32_t *labels, double *delta,
                         int mode, void *stream) {
  if (!labels || !delta)
    return fail(DKM_E_ARG, "assign_delta: labels and delta are required");
  return assign<double>(X, n, d, ldx, C, k, ws, ws_bytes, labels, delta, 2,
                        mode, stream, "dkm_assign_delta_f64");
}

int dkm_assign_delta_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                         const double *C, int64_t k, const void *ws,
                         size_t ws_bytes, int32_t *labels, double *delta,
                         int mode, void *stream) {
  if (!labels || !delta)
    return fail(DKM_E_ARG, "assign_delta: labels and delta are required");
  return assign<float>(X, n, d, ldx, C, k, ws, ws_bytes, labels, delta, 2,
                       mode, stream, "dkm_assign_delta_f32");
}

int dkm_predict_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                    const double *C, int64_t k, const void *ws,
                    size_t ws_bytes, int32_t *labels, int mode, void *stream) {
  if (!labels) return fail(DKM_E_ARG, "predict: labels is NULL");
  return assign<double>(X, n, d, ldx, C, k, ws, ws_bytes, labels, nullptr, 0,
                        mode, stream, "dkm_predict_f64");
}

int dkm_predict_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                    const double *C, int64_t k, const void *ws,
                    size_t ws_bytes, int32_t *labels, int mode, void *stream) {
  if (!labels) return fail(DKM_E_ARG, "predict: labels is NULL");
  return assign<float>(X, n, d, ldx, C, k, ws, ws_bytes, labels, nullptr, 0,
                       mode, stream, "dkm_predict_f32");
}

int dkm_add_f64(double *y, const double *x, int64_t n, void *stream) {
  if ((!y || !x) && n > 0) return fail(DKM_E_ARG, "add: NULL");
  if (n <= 0) return 0;
  const int64_t g = std::min<int64_t>((n + 255) / 256, 4096);
  k_add<<<(unsigned)g, 256, 0, (hipStream_t)stream>>>(y, x, n);
  return check_launch("dkm_add_f64");
}

}  // extern "C"
