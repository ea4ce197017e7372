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
#include <cstdio>
#include <cstdlib>
#include <string>

#include "dkm_internal.h"

namespace dkm {

constexpr int BLOCK = 256;
constexpr size_t LDS_BUDGET = 80 * 1024;  // per block -> >= 2 blocks / CU
constexpr size_t LDS_PER_CU = 160 * 1024;

// Accumulation mode bits: AM_ON (accumulate at all), AM_DELTA (incremental:
// only label changes move rows), AM_INLDS (block-private LDS accumulators,
// flushed once per block; else fp64 global atomics).
// AM_MLIST (k_screen_w32, with AM_DELTA and without AM_ON): the rows the
// screen moves are listed (v.smoved, count hdr->nmoved; previous labels in
// v.queue[row]) for sorted_sums_moved instead of added in the screen.
enum : int { AM_NONE = 0, AM_ON = 1, AM_DELTA = 2, AM_INLDS = 4,
             AM_MLIST = 8 };
constexpr int W32_MLB = 256;  // AM_MLIST: moved rows staged per wave (LDS)
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

// Workgroups of `block` threads resident per CU, for sizing the persistent
// (grid-stride) grids: the smallest of the VGPR-file limit (512 registers
// per lane per SIMD, 8-register granule, at most 6 waves per SIMD for the
// ~100-SGPR kernels here), the LDS limit (160 KiB per CU) and 32 waves per
// CU (MI355X_MICROARCH.md "Register files", "Residency").  The occupancy
// API answered 1 for the 512-thread screen where 3 fit (2 instead of 6
// waves per SIMD), so it is not used.  A/B builds (variants.sh) may pin the
// count with -DDKM_AB_BLOCKS_PER_CU=n and print the numbers with
// -DDKM_AB_VERBOSE; the product build has neither.
static int resident_blocks(const void *kf, int block, size_t lds) {
#ifdef DKM_AB_BLOCKS_PER_CU
  return DKM_AB_BLOCKS_PER_CU;
#endif
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, kf) != hipSuccess) return 1;
  const int waves = (block + 63) / 64;
  const int alloc = std::max(8, (fa.numRegs + 7) / 8 * 8);
  const int wps = std::min(6, 512 / alloc);
  const int by_regs = (4 * wps) / waves;
  const size_t l = lds + fa.sharedSizeBytes;
  const int by_lds = l ? (int)(LDS_PER_CU / l) : 32;
  const int own =
      std::max(1, std::min(std::min(by_regs, by_lds), 32 / waves));
#ifdef DKM_AB_VERBOSE
  {
    int api = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, kf, block, lds) !=
        hipSuccess)
      api = -1;
    fprintf(stderr, "dkm: block %d lds %zu vgpr %d -> %d/CU (api %d)\n",
            block, l, fa.numRegs, own, api);
  }
#endif
  return own;
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
    // NaN distances rank first (np.argmin's first-NaN rule): argmin_key
    const double s0 = exact_sqdist_reg<MAXD>(x, cl, d);
    double best_s = argmin_key(s0);
    double best = argmin_key(sqrt(s0));
    int bi = 0;
    for (int j = 1; j < k; ++j) {
      const double s = exact_sqdist_reg<MAXD>(x, cl + (int64_t)j * d, d);
      const double ks = argmin_key(s);
      if (ks < best_s) {
        const double dist = argmin_key(sqrt(s));
        if (dist < best) {
          best = dist;
          bi = j;
        }
        best_s = ks;
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
  const double s0 = pw_sum(SqDiff<TX>{xr, C}, d);
  double best_s = argmin_key(s0);
  double best = argmin_key(sqrt(s0));
  int bi = 0;
  for (int j = 1; j < k; ++j) {
    const double s = pw_sum(SqDiff<TX>{xr, C + (int64_t)j * d}, d);
    const double ks = argmin_key(s);
    if (ks < best_s) {
      const double dist = argmin_key(sqrt(s));
      if (dist < best) {
        best = dist;
        bi = j;
      }
      best_s = ks;
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
// The centre fragments hold -2c (exact scaling) and each MFMA chain starts
// from |c|^2, so the chain's output IS the score (no VALU epilogue).
//
// Precisions (PREC):
//   P_F32  v_mfma_f32_16x16x4_f32 (exact f32 fma chains) on x32 = fl32(x),
//          c32 = fl32(c).  Bound: conversions 2u|x.c|, the d-term chain
//          d*u*(|c|^2 + sum|2 x c|), fp32 |c|^2 (u|c|^2), u = 2^-24.
//   P_B3   v_mfma_f32_16x16x32_bf16 on bf16 hi/lo splits of x32 and -2c:
//          x.c ~ xh.ch + xh.cl + xl.ch (products exact in fp32); split
//          remainder <= 3.1 * 2^-16 sum|x c| (incl. the x -> x32 rounding),
//          fp32 accumulation of |c|^2 and 3d products bounded as (3d + 6)
//          roundings of 2^-23 (no assumption about the MFMA's internal
//          adder), fp32 |c|^2.
// Both doubled for safety, plus numpy's fp64 rounding (16 * 2^-52 (|x| +
// cmax)^2), an absolute underflow floor, and |x.c| <= |x| cmax.  |x| is
// computed in fp32 and inflated (relative error <= (d + 4) 2^-24).
//
// Index packing: the screen replaces the low PACK_BITS mantissa bits of each
// score by a wave-uniform tag (16-centre block within its group of 32 blocks,
// accumulator row i < 4); the lane's q supplies the rest of the centre index
// (cb * 16 + 4q + i) when the group is folded.  One v_and_or, one v_med3 and
// one v_min (med3 against -inf, no NaN canonicalisation) per score keep a
// top-2 of (value, index) pairs.  Packing
// moves a score by < 2^PACK_BITS ulp <= 2^-16 |s|, |s| <= |c|^2 + 2|x||c|;
// `packed` adds that to B (both compared scores move, and the test is
// s2 - s1 > 2B).
// ---------------------------------------------------------------------------
}  // namespace dkm

#include "dkm_screen.h"
#include "dkm_b2.h"

namespace dkm {


#ifndef DKM_SB
#define DKM_SB 512
#endif
// NB1: 16-sample blocks per wave step at d <= 32.  WPE: waves per SIMD the
// d <= 32 screen is compiled for (6 -> <= 80 VGPRs -> three 512-thread
// blocks per CU; NB1 = 2 needs ~150 VGPRs, one block per CU); d <= 64: 4.
#ifndef DKM_NB1
#define DKM_NB1 1
#endif
#ifndef DKM_WPE
#define DKM_WPE 6
#endif
// CHUNK (fragments staged through LDS): one 512-thread block per CU (the
// chunk fills the LDS), so 2 waves per SIMD whatever the registers: compiled
// for 2 waves per EU (up to 256 VGPRs) instead of d <= 64's 4 -- C3
// iteration 0's bf16x3 screen 60-61 -> 54 ms (r05nb kernel traces).  Two
// 16-sample blocks per wave step (half the L2 -> LDS fragment traffic per
// row) measured slower, 68.5 ms: NB_CHUNK stays 1.
#ifndef DKM_NB_CHUNK
#define DKM_NB_CHUNK 1
#endif
#define DKM_SCREEN_WPE(NKS, CHUNK) \
  __attribute__((amdgpu_waves_per_eu( \
      (CHUNK) ? 2 : DKM_WPE <= 0 ? 1 : (NKS) == 1 ? DKM_WPE : (NKS) == 2 ? 4 : 1)))
constexpr int SB = DKM_SB;  // screen block: SB/64 waves share one LDS image

// A/B switches, compile-time only (variants.sh -DDKM_AB_...=1; all off in the
// product build): no W32 screen, delta sums always / never by k_label_sums,
// no per-wave undecided lists, post-screen sums by k_label_sums instead of
// the sorted sums.
#ifndef DKM_AB_LABEL_SUMS
#define DKM_AB_LABEL_SUMS 0
#endif
#ifndef DKM_AB_NO_W32
#define DKM_AB_NO_W32 0
#endif
#ifndef DKM_AB_NO_C32
#define DKM_AB_NO_C32 0
#endif
constexpr bool AB_NO_C32 = DKM_AB_NO_C32;
#ifndef DKM_AB_NO_GEMM_BUILD
#define DKM_AB_NO_GEMM_BUILD 0
#endif
constexpr bool AB_NO_GEMM_BUILD = DKM_AB_NO_GEMM_BUILD;
#ifndef DKM_AB_NO_MLIST
#define DKM_AB_NO_MLIST 0
#endif
constexpr bool AB_NO_MLIST = DKM_AB_NO_MLIST;
#ifndef DKM_AB_DELTA_POST
#define DKM_AB_DELTA_POST 0
#endif
#ifndef DKM_AB_NO_POST
#define DKM_AB_NO_POST 0
#endif
#ifndef DKM_AB_NO_LIST
#define DKM_AB_NO_LIST 0
#endif
constexpr bool AB_NO_W32 = DKM_AB_NO_W32, AB_DELTA_POST = DKM_AB_DELTA_POST,
               AB_NO_POST = DKM_AB_NO_POST, AB_NO_LIST = DKM_AB_NO_LIST,
               AB_LABEL_SUMS = DKM_AB_LABEL_SUMS;

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

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// One undecided sample per lane (the screen's tail and k_recheck_lane).
// Stage 1 re-screens in fp32 VALU (x in VGPRs, fp32 centres `cl` of row
// stride dp and |c|^2 `cnl`, in LDS or global memory) -- the P_F32
// arithmetic and bound, ~2^-24 instead of bf16x3's ~2^-16 -- and keeps the
// label when the best two scores are 2B apart.  Otherwise stage 2 runs the
// reference arithmetic on the candidates only (score <= best + 2B: the
// reference winner is always among them, and every other centre is
// strictly farther after sqrt).  Writes lab_out[i] and moves
// the row between the accumulators as amode says (prev = previous label).
// STAGE1_ONLY: return false (writing nothing) when stage 1 cannot decide,
// so the caller can batch the rare stage-2 samples into full waves.
template <int MAXD, bool VEC, class TX, bool STAGE1_ONLY = false>
__device__ __forceinline__ bool resolve_lane(
    const TX *__restrict__ X, int64_t ldx, int d, int k, int64_t i, int prev,
    const float *cl, const float *cnl, int dp, float cm, const double *ct64,
    int32_t *lab_out, int amode, const AccTarget &at) {
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
  // fp32 score of centre jc: fma chain over features (padding adds 0 * 0).
  // cl / cnl are the workspace's global fp32 centres, read through the
  // constant address space: jc is wave-uniform, so the rows arrive by scalar
  // loads into SGPRs (an LDS broadcast of the same row costs the full LDS
  // return bandwidth, twice the VALU time of the fma chain).
  typedef const __attribute__((address_space(4))) float cfloat;
  typedef const __attribute__((address_space(4))) f32x4 cf32x4;
  cfloat *clc = (cfloat *)cl;
  cfloat *cnc = (cfloat *)cnl;
  // full rows (dp == MAXD): no per-chunk branch, so the row's scalar loads
  // issue together (one wait instead of one per 4 features)
  const bool full = dp == MAXD;
  auto score = [&](int jc) {
    cfloat *cr = clc + (int64_t)jc * dp;
    float dot = 0.f;
    if (full) {
#pragma unroll
      for (int t4 = 0; t4 < MAXD / 4; ++t4) {
        const f32x4 c4 = *(cf32x4 *)(cr + 4 * t4);
        dot = fmaf(xf[4 * t4 + 0], c4.x, dot);
        dot = fmaf(xf[4 * t4 + 1], c4.y, dot);
        dot = fmaf(xf[4 * t4 + 2], c4.z, dot);
        dot = fmaf(xf[4 * t4 + 3], c4.w, dot);
      }
    } else {
#pragma unroll
      for (int t4 = 0; t4 < MAXD / 4; ++t4) {
        if (4 * t4 < dp) {
          const f32x4 c4 = *(cf32x4 *)(cr + 4 * t4);
          dot = fmaf(xf[4 * t4 + 0], c4.x, dot);
          dot = fmaf(xf[4 * t4 + 1], c4.y, dot);
          dot = fmaf(xf[4 * t4 + 2], c4.z, dot);
          dot = fmaf(xf[4 * t4 + 3], c4.w, dot);
        }
      }
    }
    return fmaf(-2.f, dot, cnc[jc]);
  };
  float b1 = INFINITY, b2 = INFINITY;
  int i1 = 0;
#ifndef DKM_S1_UNROLL
#define DKM_S1_UNROLL 4
#endif
#pragma unroll DKM_S1_UNROLL
  for (int jc = 0; jc < k; ++jc) {
    const float sc = score(jc);
    i1 = sc < b1 ? jc : i1;
    b2 = __builtin_amdgcn_fmed3f(b1, b2, sc);
    b1 = fminf(b1, sc);
  }
  const float xn = sqrtf(xx) * (1.0f + (d + 4) * 0x1.0p-24f);
  const float B = screen_bound<P_F32>(d, xn, cm, false);
  const bool sane = (xn < 1e18f) && (xn * cm < 1e30f) && (b1 < 1e30f);
  int bi = i1;
  if (!(sane && b2 - b1 > 2.0f * B)) {
    if constexpr (STAGE1_ONLY) return false;
    const float lim = b1 + 2.0f * B;
    double best = INFINITY;
    bi = -1;
#pragma unroll 1
    for (int jc = 0; jc < k; ++jc) {
      if (sane && !(score(jc) <= lim)) continue;
      const SqDiffT<TX> f{xr, ct64 + jc, ct_ld(k)};
      const double dist = argmin_key(sqrt(pw_leaf(f, 0, d)));
      if (dist < best || bi < 0) {
        best = dist;
        bi = jc;
      }
    }
  }
  lab_out[i] = bi;
  if (!(amode & AM_ON)) return true;
  const bool delta = amode & AM_DELTA;
  if (delta && bi == prev) return true;
  const bool sub = delta && prev >= 0;
  for (int t = 0; t < d; ++t) {
    const double x = ld_x(xr + t);
    at.add(bi, t, x);
    if (sub) at.add(prev, t, -x);
  }
  at.count(bi, 1.0);
  if (sub) at.count(prev, -1.0);
  return true;
}

// One wave = NB blocks of 16 samples per step.  Lane l = (q = l >> 4,
// j = l & 15) holds features ks*32 + 8q + m (m < 8) of sample j of every
// block (4 x 16-B loads per lane per 32 features).  Outside the full-
// accumulation modes the fp64 tile registers are reloaded with the NEXT
// step's rows as soon as they are converted, so one tile is in flight during
// the MFMA/scoring of the current one.  The MFMA output gives lane (q, j)
// the scores of centres cb*16 + 4q + i (i < 4) with sample j; each lane
// keeps a packed top-2 per group of 128 centres (v_and_or, v_med3, v_min
// per score), merges it into a running (value, index) top-2 per group, and
// two xor-shuffles merge the four lanes of a sample.  lab_out[si] = label,
// or -(prev + 2) when the screen cannot decide (the re-check resolves it;
// prev = -1 outside AM_DELTA).
//
// CHUNK (k x d too large for LDS, e.g. k = 1000, d = 64): the fragments pass
// through LDS in chunks of chb 16-centre blocks for every block step; the
// sample loop is block-uniform (waves past n compute on zero rows and write
// nothing) so that every wave reaches the chunk barriers.  L2 -> LDS traffic
// per block step = all fragments (k * dpad * 4 B) per 16 * NB * SB/64 rows.
//
// T3 (CHUNK bf16x3: C3's iteration 0 against the U[0, 1) initial centres):
// each lane keeps a packed top-3 (one more v_med3 per score) and the running
// top-3 carries the first two centres' indices, so the decision is
// three-way like the single-product screens': s2 - s1 > 2B -> the label;
// else s3 - s1 > 2B -> the two candidates go to the wave's candidate list
// (k_cand2 applies the reference arithmetic to both; use_list bit 2, labels-
// only launches with d % 8 == 0); else the re-check list.  Against U[0, 1)
// centres ~2 % of the rows are near-ties under the bf16x3 bound, nearly all
// with two candidates (tools/exp note in DESIGN.md 3.13): they no longer
// cost a fp32 re-scan of all k centres each.
template <int PREC, int NKS, int NB, bool VEC, class TX, bool CHUNK,
          bool T3P = false>
__global__ void __launch_bounds__(SB) DKM_SCREEN_WPE(NKS, CHUNK)
    k_screen(const TX *__restrict__ X, int64_t n, int d, int64_t ldx, int k,
             WsView v, int32_t *__restrict__ lab_out, double *acc, int amode,
             int64_t base, int use_list, int chb) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nkb = (int)(kpad16(k) / 16);
  const int lkb = CHUNK ? chb : nkb;  // blocks resident in LDS at a time
  // fragment region: lkb*NKS blocks of 2 KB (f32: 8 floats per lane;
  // bf16x3: 8 hi + 8 lo bf16 per lane)
  char *frag = (char *)smem;
  float *cn = (float *)(frag + (int64_t)lkb * NKS * 2048);  // lkb*16
  double *lds_acc = (double *)(cn + lkb * 16);
  const f32x4 *fsrc = (const f32x4 *)(PREC == P_F32 ? (const void *)v.cfrag
                                                    : (const void *)v.bfrag);
  // LDS <- fragment blocks [c0, c1)
  auto load_chunk = [&](int c0, int c1) {
    const f32x4 *src = fsrc + (int64_t)c0 * NKS * 128;
    f32x4 *dst = (f32x4 *)frag;
    for (int e = threadIdx.x; e < (c1 - c0) * NKS * 128; e += SB)
      dst[e] = src[e];
    for (int e = threadIdx.x; e < (c1 - c0) * 16; e += SB)
      cn[e] = v.cnpad[c0 * 16 + e];
  };
  if (!CHUNK) load_chunk(0, nkb);
  if (amode & AM_INLDS) zero_lds_acc(lds_acc, k, d);
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  const BoundK bk = bound_consts<PREC>(d, cm);
  const float ninf = __uint_as_float(opaque_u32(0xff800000u));
  const uint32_t vmask = opaque_u32(~PACK_MASK);
  const bool full_acc = am_full(amode);
  const bool delta = amode & AM_DELTA;
  const AccTarget at = acc_target(amode, lds_acc, acc, k, d);
  __syncthreads();

  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t wv = (int64_t)blockIdx.x * (SB / 64) + wid;
  const int64_t step = (int64_t)gridDim.x * (SB / 64) * 16 * NB;
  const int64_t seg = (int64_t)blockIdx.x * (SB / 64) + wid;
  int2 *wl = v.tlist + seg * TL_CAP;  // this wave's undecided samples
  const bool listing = (use_list & 1) && seg < TL_SEGS;
  int tl_cnt = 0;   // wave-uniform: listed samples
  int tl_over = 0;  // wave-uniform: undecided samples left for the re-check
  constexpr bool T3 = T3P && CHUNK && PREC == P_B3;
  // two-candidate list (T3, labels-only launches): (offset, c1 | c2 << 16)
  const bool list2 = T3 && (use_list & 2) && v.clist && seg < B1_SEGS;
  int2 *cl = list2 ? v.clist + seg * B1_CAP : nullptr;
  int cl_cnt = 0;
  const float pinf = __uint_as_float(opaque_u32(0x7f800000u));
  (void)pinf;

  double tile[NB][NKS][8];
  // delta: the previous labels of the tile's samples travel with the tile
  // (a label load issued at use time exposed a full HBM latency per step)
  int pv[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) pv[b] = -1;
  // VEC steps: buffer loads off a per-step SGPR descriptor (base = the
  // step's first row, 32-bit lane offsets, no 64-bit lane pointers); rows
  // past n fall outside num_records and read as 0 (no clamp needed)
  const bool off32 =
      (int64_t)16 * NB * ldx * (int64_t)sizeof(TX) < (1ll << 31);
  const uint32_t lane_off = (uint32_t)(j * ldx * (int64_t)sizeof(TX)) +
                            (uint32_t)(8 * q * sizeof(TX));
  auto load_tile = [&](int64_t s0) {
    if (VEC && off32) {
      const int64_t rows = std::max<int64_t>(0, n - s0);
      const int64_t xb = rows * ldx * (int64_t)sizeof(TX);
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(X + std::min(s0, n) * ldx), 0,
          (int)std::min<int64_t>(xb, 0x7fffffff), 0x00020000);
      if (delta) {
        const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(lab_out + std::min(s0, n)), 0,
            (int)std::min<int64_t>(rows * 4, 0x7fffffff), 0x00020000);
#pragma unroll
        for (int b = 0; b < NB; ++b)
          pv[b] = (int)__builtin_amdgcn_raw_buffer_load_b32(
              rl, (16 * b + j) * 4, 0, 0);
      }
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const uint32_t ob = lane_off + (uint32_t)(16 * b * ldx * sizeof(TX));
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          if (ks * 32 + 8 * q < d) {
            const uint32_t o = ob + ks * 32 * sizeof(TX);
            if constexpr (sizeof(TX) == 8) {
#pragma unroll
              for (int p4 = 0; p4 < 4; ++p4) {
                const double2 v2 = __builtin_bit_cast(
                    double2,
                    __builtin_amdgcn_raw_buffer_load_b128(rx, o + 16 * p4, 0, 0));
                tile[b][ks][2 * p4] = v2.x;
                tile[b][ks][2 * p4 + 1] = v2.y;
              }
            } else {
#pragma unroll
              for (int p4 = 0; p4 < 2; ++p4) {
                const float4 v4 = __builtin_bit_cast(
                    float4,
                    __builtin_amdgcn_raw_buffer_load_b128(rx, o + 16 * p4, 0, 0));
                tile[b][ks][4 * p4] = v4.x;
                tile[b][ks][4 * p4 + 1] = v4.y;
                tile[b][ks][4 * p4 + 2] = v4.z;
                tile[b][ks][4 * p4 + 3] = v4.w;
              }
            }
          } else {
#pragma unroll
            for (int m = 0; m < 8; ++m) tile[b][ks][m] = 0.0;
          }
        }
      }
      return;
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      int64_t si = s0 + 16 * b + j;
      si = si < n ? si : n - 1;  // clamp: always a readable row
      if (delta) pv[b] = lab_out[si];
      const TX *xr = X + si * ldx;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
        load8<VEC>(xr, ks * 32 + 8 * q, d, tile[b][ks]);
    }
  };

  // CHUNK: iterate on the block's first row so the trip count is
  // block-uniform (every wave reaches the chunk barriers)
  const int64_t wofs = (int64_t)wid * 16 * NB;
  int64_t s0 = base + wv * 16 * NB;
  if (s0 < n) load_tile(s0);
  for (; (CHUNK ? s0 - wofs : s0) < n; s0 += step) {
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
        for (int m = 0; m < 8; m += 2) {
          const float x0 = (float)tile[b][ks][m];
          const float x1 = (float)tile[b][ks][m + 1];
          xx[b] = fmaf(x0, x0, xx[b]);
          xx[b] = fmaf(x1, x1, xx[b]);
          if constexpr (PREC == P_F32) {
            xf[b][ks][m] = x0;
            xf[b][ks][m + 1] = x1;
          } else {
            // one v_cvt_pk_bf16_f32 per pair; the hi parts back as fp32 by
            // shift / mask; lo = x - hi is exact
            const bf16x2 h2 = __builtin_convertvector(f32x2{x0, x1}, bf16x2);
            const uint32_t hu = __builtin_bit_cast(uint32_t, h2);
            const float h0 = __uint_as_float(hu << 16);
            const float h1 = __uint_as_float(hu & 0xffff0000u);
            const bf16x2 l2 =
                __builtin_convertvector(f32x2{x0 - h0, x1 - h1}, bf16x2);
            xh[b][ks][m] = h2[0];
            xh[b][ks][m + 1] = h2[1];
            xl[b][ks][m] = l2[0];
            xl[b][ks][m + 1] = l2[1];
          }
        }
      float xa, xb;
      pair_xor<16>(xx[b], xa, xb);
      xx[b] = xa + xb;
      pair_xor<32>(xx[b], xa, xb);
      xx[b] = xa + xb;
    }
    int prv[NB];  // this step's previous labels (pv is refilled below)
#pragma unroll
    for (int b = 0; b < NB; ++b) prv[b] = pv[b];
    // ---- the next step's rows stream in while this one computes ----
    const int64_t s_next = s0 + step;
#ifndef DKM_DBG_NOLOAD
    if (!full_acc && s_next < n) load_tile(s_next);
#endif

    // running (value, centre index) top-2 of this lane over all groups
    // (T3: top-3, the second's index in ri2)
    float r1[NB], r2[NB], r3[NB];
    int ri[NB], ri2[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      r1[b] = INFINITY;
      r2[b] = INFINITY;
      r3[b] = INFINITY;
      ri[b] = 0;
      ri2[b] = 0;
    }
    // MFMA chain of centre block cb into accv[], started from |c|^2; consumed
    // one chain later so that the next block's MFMAs overlap this block's
    // VALU scoring.
    int cbase = 0;  // first LDS-resident block (CHUNK)
    auto chain = [&](int cb, f32x4 (&accv)[NB]) {
      const f32x4 c4 = *(const f32x4 *)(cn + (cb - cbase) * 16 + 4 * q);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const char *blk = frag + ((int64_t)(cb - cbase) * NKS + ks) * 2048;
        if constexpr (PREC == P_F32) {
          const f32x4 a0 = *(const f32x4 *)(blk + lane * 32);
          const f32x4 a1 = *(const f32x4 *)(blk + lane * 32 + 16);
          const float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
          for (int m = 0; m < 8; ++m)
#pragma unroll
            for (int b = 0; b < NB; ++b)
              accv[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                  a[m], xf[b][ks][m], (ks == 0 && m == 0) ? c4 : accv[b], 0,
                  0, 0);
        } else {
          const bf16x8 ah = *(const bf16x8 *)(blk + lane * 16);
          const bf16x8 al = *(const bf16x8 *)(blk + 1024 + lane * 16);
#pragma unroll
          for (int b = 0; b < NB; ++b)
            accv[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                ah, xh[b][ks], ks == 0 ? c4 : accv[b], 0, 0, 0);
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
#ifdef DKM_DBG_NOCOMPUTE
    for (int b = 0; b < NB; ++b) {
      r1[b] = xx[b];
      r2[b] = 1e20f;
    }
#else
    for (int c0 = 0; c0 < nkb; c0 += lkb) {
    const int c1 = min(nkb, c0 + lkb);
    if (CHUNK) {
      __syncthreads();  // every wave is done with the previous chunk
      load_chunk(c0, c1);
      __syncthreads();
    }
    cbase = c0;
    for (int g0 = c0; g0 < c1; g0 += GROUP_BLOCKS) {
      const int g1 = min(c1, g0 + GROUP_BLOCKS);
      float b1[NB], b2[NB], b3[NB];  // packed, this group
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        b1[b] = INFINITY;
        b2[b] = INFINITY;
        b3[b] = INFINITY;
      }
      auto score = [&](int cb, const f32x4 (&accv)[NB]) {
        const uint32_t ib = (uint32_t)((cb - g0) * 4);  // wave-uniform tag
        uint32_t tag[4];  // opaque SGPRs: one v_and_or_b32 per score
        const uint32_t t0 = opaque_s32(ib);
#pragma unroll
        for (int i = 0; i < 4; ++i) tag[i] = t0 + i;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            // scalar ops on purpose: no v_pk_*_f32 anywhere (see the header
            // note on packed-VALU operand hazards; built -fno-slp-vectorize)
            const float sp = __uint_as_float(
                (__float_as_uint(accv[b][i]) & vmask) | tag[i]);
            // b1 <= b2 (<= b3): new third = med3(b2, b3, s), new second =
            // med3(b1, b2, s)
            if constexpr (T3) b3[b] = __builtin_amdgcn_fmed3f(b2[b], b3[b], sp);
            b2[b] = __builtin_amdgcn_fmed3f(b1[b], b2[b], sp);
            b1[b] = min_nc(b1[b], sp, ninf);
          }
        }
      };
      f32x4 acc_a[NB], acc_b[NB];
      chain(g0, acc_a);
      int cb = g0;
      for (; cb + 2 <= g1; cb += 2) {  // ping-pong: no runtime-indexed arrays
        chain(cb + 1, acc_b);
        score(cb, acc_a);
        if (cb + 2 < g1) chain(cb + 2, acc_a);
        score(cb + 1, acc_b);
      }
      if (cb < g1) score(cb, acc_a);  // odd block count: last chain in acc_a
      // fold the group's packed top-2 into the running (value, index) top-2
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const uint32_t tg = __float_as_uint(b1[b]) & PACK_MASK;
        const int gi = (g0 + (int)(tg >> 2)) * 16 + 4 * q + (int)(tg & 3);
        const bool nw = b1[b] < r1[b];
        if constexpr (T3) {
          // merge sorted (r1, r2, r3) with (b1, b2, b3): the third smallest
          // of the union is min(r3, b3, max(r1, b2), max(r2, b1)); ties keep
          // the running entry (earlier groups: lower indices)
          const uint32_t t2 = __float_as_uint(b2[b]) & PACK_MASK;
          const int gi2 = (g0 + (int)(t2 >> 2)) * 16 + 4 * q + (int)(t2 & 3);
          r3[b] = min_nc(min_nc(r3[b], b3[b], ninf),
                         min_nc(__builtin_amdgcn_fmed3f(r1[b], b2[b], pinf),
                                __builtin_amdgcn_fmed3f(r2[b], b1[b], pinf),
                                ninf),
                         ninf);
          const bool s2 = nw ? (b2[b] < r1[b]) : (b1[b] < r2[b]);
          const float v2 = nw ? (s2 ? b2[b] : r1[b]) : (s2 ? b1[b] : r2[b]);
          ri2[b] = nw ? (s2 ? gi2 : ri[b]) : (s2 ? gi : ri2[b]);
          r2[b] = v2;
        } else {
          r2[b] = nw ? min_nc(r1[b], b2[b], ninf) : min_nc(r2[b], b1[b], ninf);
        }
        ri[b] = nw ? gi : ri[b];
        r1[b] = nw ? b1[b] : r1[b];
      }
    }
    }  // chunks
#endif
    // merge the top-2 of the four lanes of a sample
    // (symmetric in the pair: both lanes get the same result whichever
    // order pair_xor hands the two sides over)
    auto merge2 = [&](float &v1, float &v2, int &vi, float a1, float a2,
                      int ai, float c1, float c2, int ci) {
      const bool tc = (c1 < a1) | ((c1 == a1) & (ci < ai));
      v1 = tc ? c1 : a1;
      vi = tc ? ci : ai;
      v2 = tc ? min_nc(a1, c2, ninf) : min_nc(a2, c1, ninf);
    };
    // T3: merge two (value, index) top-3 lists with the first two indices
    // (symmetric in the pair: both lanes hold the same result)
    auto merge3 = [&](int b, float a1, float a2, float a3, int ai, int ai2,
                      float c1, float c2, float c3, int ci, int ci2) {
      const bool tc = (c1 < a1) | ((c1 == a1) & (ci < ai));
      const float x = tc ? a1 : c1, y = tc ? c2 : a2;
      const int xi = tc ? ai : ci, yi = tc ? ci2 : ai2;
      const bool ty = (y < x) | ((y == x) & (yi < xi));
      r3[b] = min_nc(min_nc(a3, c3, ninf),
                     min_nc(__builtin_amdgcn_fmed3f(a1, c2, pinf),
                            __builtin_amdgcn_fmed3f(a2, c1, pinf), ninf),
                     ninf);
      r1[b] = tc ? c1 : a1;
      ri[b] = tc ? ci : ai;
      r2[b] = ty ? y : x;
      ri2[b] = ty ? yi : xi;
    };
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float a1, c1, a2, c2;
      int ai, ci;
      if constexpr (T3) {
        float a3, c3;
        int aj, cj;
#define DKM_T3_ROUND(OFF)                                          \
  pair_xor<OFF>(r1[b], a1, c1);                                    \
  pair_xor<OFF>(r2[b], a2, c2);                                    \
  pair_xor<OFF>(r3[b], a3, c3);                                    \
  pair_xor<OFF>(ri[b], ai, ci);                                    \
  pair_xor<OFF>(ri2[b], aj, cj);                                   \
  merge3(b, a1, a2, a3, ai, aj, c1, c2, c3, ci, cj);
        DKM_T3_ROUND(16)
        DKM_T3_ROUND(32)
#undef DKM_T3_ROUND
        continue;
      }
      pair_xor<16>(r1[b], a1, c1);
      pair_xor<16>(r2[b], a2, c2);
      pair_xor<16>(ri[b], ai, ci);
      merge2(r1[b], r2[b], ri[b], a1, a2, ai, c1, c2, ci);
      pair_xor<32>(r1[b], a1, c1);
      pair_xor<32>(r2[b], a2, c2);
      pair_xor<32>(ri[b], ai, ci);
      merge2(r1[b], r2[b], ri[b], a1, a2, ai, c1, c2, ci);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int64_t si = s0 + 16 * b + j;
      float xn;
      const float B2 = bound2_fast(bk, xx[b], xn);
      const bool sane = (xn < 1e18f) & (xn * cm < 1e30f) & (r1[b] < 1e30f);
      const bool unique = sane & (r2[b] - r1[b] > B2);
      const int prev = delta ? prv[b] : -1;
      // T3: exactly two candidates -> the candidate list (k_cand2)
      bool two = false;
      if constexpr (T3) {
        two = list2 && si < n && sane && !unique && (r3[b] - r1[b] > B2);
        const uint64_t mc = __ballot(q == 0 && two);
        const int addc = __popcll(mc);
        if (cl_cnt + addc <= B1_CAP) {
          if (q == 0 && two)
            cl[cl_cnt + lane_prefix(mc)] =
                make_int2((int)(si - base), ri[b] | (ri2[b] << 16));
          cl_cnt += addc;
        } else {
          two = false;   // list full: the re-check list takes it
        }
      }
      const bool und = si < n && !unique && !two;
      // undecided samples join the wave's list (resolved in the tail) while
      // it has room; the rest are counted for the re-check pass
      const uint64_t um = __ballot(q == 0 && und);
      const int add = __popcll(um);
      if (listing && tl_cnt + add <= TL_CAP) {
        if (q == 0 && und)
          wl[tl_cnt + lane_prefix(um)] =
              make_int2((int)(si - base), prev);
        tl_cnt += add;
      } else {
        tl_over += add;
      }
      if (si >= n) continue;
      const int lab = ri[b];
      // an unchanged delta label is already in place: no store
      if (q == 0 && !(unique && lab == prev))
        lab_out[si] = unique ? lab : -(prev + 2);
      if (!unique) continue;  // label + sums by the tail / re-check
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
  if (lane == 0) {
    if (listing) v.tcount[seg] = tl_cnt;
    if (list2) v.ccount[seg] = cl_cnt;
    if (tl_over) atomicAdd(&v.hdr->qcount, (uint32_t)tl_over);
  }
  if (amode & AM_INLDS) {
    __syncthreads();
    flush_lds_acc(lds_acc, acc, k, d);
  }
}


// ---------------------------------------------------------------------------
// bf16x3 screen on v_mfma_f32_32x32x16_bf16 for d <= 32 (16-B aligned rows):
// one wave step = 32 samples (B columns) x 32-centre blocks (A rows).  Lane
// l = (r = l & 31, h = l >> 5) holds the 16 contiguous features 16h..16h+15
// of sample r (K-slice ks takes features 16h + 8ks + j, the same permuted K
// order as the W32 fragments built by k_frag), so a sample's partial |x|^2
// and top-2 need one permlane32 swap to merge, and every per-sample cost
// (conversion, merge, bound, label, list) is paid by 2 lanes instead of the
// 16x16 kernel's 4.  Accumulator register g holds centre
// cb*32 + (g & 3) + 8 (g >> 2) + 4h; the packing tag is (block in group) x 16
// + g, PACK_BITS = 7 -> groups of 8 blocks.  Same bound, same exactness
// argument and the same list / label / accumulation contract as k_screen.
// ---------------------------------------------------------------------------
constexpr int SBW = 256;  // k_screen_w32 block: 4 waves, 3 blocks per CU
constexpr int W32_SCR = 2048 + 128 + 128;  // per-wave LDS scratch
__device__ __forceinline__ void wave_sync_w() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// cache policy of k_screen_w32's streaming row loads (0 = default; 2 = NT)
#ifndef DKM_XLOAD_AUX
#define DKM_XLOAD_AUX 0
#endif
#ifndef DKM_W32_WPE
#define DKM_W32_WPE 3
#endif
// HINT (image delta launches, k <= W32_HINT_KMAX: the steady iterations of
// C2): a threshold pass, as k_screen_b2's.  With p = the row's incoming
// label, s_hat_p comes from v_dot2 products of the same bf16x3 operands
// (within the bound of the MFMA scores), T = s_hat_p + 2B, and a centre
// whose score exceeds T can neither win nor tie.  Each 32-centre block is
// tested as a whole -- one min over the 16 accumulators against T -- and
// only a block with some score <= T (rare once labels settle) runs the
// packed top-2 update; p's own accumulator starts from +2^100 (a poisoned
// copy of its norm chunk), so p's block does not hit on p itself.  Per
// score: about 0.6 VALU instead of the top-2's 3 (VALU:MFMA 13:1, the
// limit of this kernel, round-5 PMC).  The decision over {p} and the kept
// scores is the same rule, exactly: every centre left out is > T.
constexpr int W32_HINT_KMAX = 256;
template <class TX, bool IMG, bool HINT = false>
__global__ void __launch_bounds__(SBW) __attribute__((
    amdgpu_waves_per_eu(DKM_W32_WPE)))
    k_screen_w32(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                 int k, WsView v, int32_t *__restrict__ lab_out, double *acc,
                 int amode, int64_t base, int use_list, XImage img,
                 int build) {
  constexpr int GB = 8;  // 32-centre blocks per packing group
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nkb = (int)(kpad32(k) / 32);
  char *frag = (char *)smem;                          // nkb x 4 KB
  float *cn = (float *)(frag + (int64_t)nkb * 4096);  // nkb x 32
  double *lds_acc = (double *)(cn + nkb * 32);
  {
    const f32x4 *src = (const f32x4 *)v.b32frag;
    f32x4 *dst = (f32x4 *)frag;
    for (int e = threadIdx.x; e < nkb * 256; e += SBW) dst[e] = src[e];
    for (int e = threadIdx.x; e < nkb * 32; e += SBW) cn[e] = v.cn32f[e];
  }
  if (amode & AM_INLDS) zero_lds_acc(lds_acc, k, d);
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  const BoundK bk = bound_consts<P_B3>(d, cm);
  const float ninf = __uint_as_float(opaque_u32(0xff800000u));
  const uint32_t vmask = opaque_u32(~PACK_MASK);
  const bool full_acc = am_full(amode);
  const bool delta = amode & AM_DELTA;
  const AccTarget at = acc_target(amode, lds_acc, acc, k, d);
  char *scr0 = (char *)((amode & AM_INLDS) ? lds_acc + lds_acc_len(k, d)
                                           : lds_acc);
  // HINT: centre p's norm chunk (the 16 norms of its block half) with p's
  // own slot +2^100, 16 floats per centre, in place of the waves' scratch
  // (the image launches use none)
  float *pcn = (float *)scr0;
  if constexpr (HINT) {
    for (int e = threadIdx.x; e < k * 16; e += SBW) {
      const int p = e >> 4, g = e & 15, q = p & 31;
      const int gp = (q & 3) | ((q >> 3) << 2);
      pcn[e] = g == gp ? 0x1.0p100f
                       : v.cn32f[(p >> 5) * 32 + 16 * ((q >> 2) & 1) + g];
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // per-wave scratch (W32_SCR bytes) after the accumulators: the transpose
  // of one 16-feature half of the tile (bf16 hi then lo, 32 rows x 32 B
  // each), |x|^2 per sample, the decided labels (full sums)
  char *scr = scr0 + wid * W32_SCR;
  char *s_hi = scr, *s_lo = scr + 1024;
  float *s_xx = (float *)(scr + 2048);
  int *s_lab = (int *)(scr + 2176);
  const int64_t wv = (int64_t)blockIdx.x * (SBW / 64) + wid;
  const int64_t step = (int64_t)gridDim.x * (SBW / 64) * 32;
  const int64_t seg = wv;
  int2 *wl = v.tlist + seg * TL_CAP;
  const bool listing = use_list && seg < TL_SEGS;
  int tl_cnt = 0, tl_over = 0;
  // AM_MLIST: this wave's staged moved rows (after the scratch and the
  // threshold norms), reserved in the global list W32_MLB at a time
  const bool mlist = (amode & AM_MLIST) != 0;
  int *mbuf = (int *)(scr0 + (IMG ? 0 : (SBW / 64) * W32_SCR) +
                      (HINT ? kpad32(k) * 64 : 0)) +
              wid * W32_MLB;
  int mcnt = 0;  // wave-uniform
  auto mflush = [&]() {
    wave_sync_w();
    int at0 = 0;
    if (lane == 0) at0 = atomicAdd(&v.hdr->nmoved, mcnt);
    at0 = __shfl(at0, 0, 64);
    for (int e = lane; e < mcnt; e += 64) v.smoved[at0 + e] = mbuf[e];
    wave_sync_w();
    mcnt = 0;
  };

  // Whole 128-B lines per wave-instruction (tools/membench.hip: loading
  // each lane's own 16 features touched 64 lines per instruction and
  // streamed X at 3.9 TB/s; whole lines 6.2 TB/s).  Half c of the tile
  // (features 16c .. 16c + 15, one line per fp64 row) is read by lanes
  // l = (row RI i + l / LR, 16-B piece l % LR); the lanes convert their
  // pieces to bf16 hi + lo, and the half reaches its consumer lanes
  // (h = c) through a 2 KB LDS transpose.  The loading lanes keep the raw
  // values for the full sums and sum |x|^2 of their rows.
  constexpr int EPL = 16 / (int)sizeof(TX);  // elements per 16-B piece
  constexpr int LR = 16 / EPL;                // lanes per row line (8 | 4)
  constexpr int RI = 64 / LR;                 // rows per instruction
  constexpr int IC = 32 / RI;                 // instructions per half
  typedef TX txv __attribute__((ext_vector_type(EPL)));
  txv raw[2][IC];
  int pv = -1;
  const int lrow = lane / LR, lpos = lane % LR;
  uint32_t lane_off[IC];
#pragma unroll
  for (int i = 0; i < IC; ++i)
    lane_off[i] = (uint32_t)((RI * i + lrow) * ldx * (int64_t)sizeof(TX)) +
                  (uint32_t)(16 * lpos);
  const bool two = d > 16;  // the second half holds features
  auto load_tile = [&](int64_t s0) {
    const int64_t rows = std::max<int64_t>(0, n - s0);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(X + std::min(s0, n) * ldx), 0,
        (int)std::min<int64_t>(rows * ldx * (int64_t)sizeof(TX), 0x7fffffff),
        0x00020000);
    if (delta) {
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(lab_out + std::min(s0, n)), 0,
          (int)std::min<int64_t>(rows * 4, 0x7fffffff), 0x00020000);
      pv = (int)__builtin_amdgcn_raw_buffer_load_b32(rl, r * 4, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < IC; ++i) {
        if (c == 1 && !two) {
          raw[c][i] = txv{};
          continue;
        }
        raw[c][i] = __builtin_bit_cast(
            txv, __builtin_amdgcn_raw_buffer_load_b128(
                     rx, lane_off[i] + 16 * c * (int)sizeof(TX), 0,
                     DKM_XLOAD_AUX));
      }
  };
  auto tx_addr = [](int row, int q) {  // 16-B quarter q of a 32-B row
    return 32 * row + 16 * (q ^ ((row >> 3) & 1));
  };

  // IMG (IMG_SPLIT image, delta / labels-only launches): the tile's hi and
  // lo slices and |x|^2 come ready in operand order, 4 whole-line 16-B
  // loads per lane, the next tile's in flight while this one is scored
  bf16x8 qi[4];
  float qxx = 0.f;
  int qpv = -1;
  auto load_img = [&](int64_t s0) {
    const bf16x8 *src =
        (const bf16x8 *)(img.tiles + (s0 >> 5) * 2048) + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) qi[q] = __builtin_nontemporal_load(src + 64 * q);
    qxx = __builtin_nontemporal_load(img.xx + s0 + r);
    if (delta) {
      const int64_t rows = std::max<int64_t>(0, n - s0);
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(lab_out + std::min(s0, n)), 0,
          (int)std::min<int64_t>(rows * 4, 0x7fffffff), 0x00020000);
      qpv = (int)__builtin_amdgcn_raw_buffer_load_b32(rl, r * 4, 0, 0);
    }
  };
  int64_t s0 = base + wv * 32;
  if (s0 < n) {
    if constexpr (IMG)
      load_img(s0);
    else
      load_tile(s0);
  }
  for (; s0 < n; s0 += step) {
    bf16x8 xh[2], xl[2];
    float xx;
    int prv;
    const int64_t s_next = s0 + step;
    if constexpr (IMG) {
      xh[0] = qi[0];
      xh[1] = qi[1];
      xl[0] = qi[2];
      xl[1] = qi[3];
      xx = qxx;
      prv = qpv;
      if (s_next < n) load_img(s_next);
    } else {
    float xp[IC];
#pragma unroll
    for (int i = 0; i < IC; ++i) xp[i] = 0.f;
    // features past d: lim recomputed per tile (opaque), or the lane masks
    // are hoisted into long-lived SGPR pairs
    const int lim = (int)opaque_u32((uint32_t)(d - EPL * lpos));
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      wave_sync_w();  // the previous readers of the transpose are done
#pragma unroll
      for (int i = 0; i < IC; ++i) {
        float xf[EPL];
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const float x = (float)raw[c][i][e];
          xf[e] = 16 * c + e < lim ? x : 0.f;
          xp[i] = fmaf(xf[e], xf[e], xp[i]);
        }
        const int row = RI * i + lrow;
#pragma unroll
        for (int e = 0; e < EPL; e += 2) {
          // one v_cvt_pk_bf16_f32 per pair; hi back as fp32 by shift /
          // mask; lo = x - hi is exact
          const bf16x2 h2 = __builtin_convertvector(f32x2{xf[e], xf[e + 1]},
                                                    bf16x2);
          const uint32_t hu = __builtin_bit_cast(uint32_t, h2);
          const bf16x2 l2 = __builtin_convertvector(
              f32x2{xf[e] - __uint_as_float(hu << 16),
                    xf[e + 1] - __uint_as_float(hu & 0xffff0000u)},
              bf16x2);
          // feature 16c + EPL lpos + e: quarter (EPL lpos + e) / 8
          const int f = EPL * lpos + e;
          const int o = tx_addr(row, f >> 3) + 2 * (f & 7);
          *(bf16x2 *)(s_hi + o) = h2;
          *(bf16x2 *)(s_lo + o) = l2;
        }
      }
      wave_sync_w();
      if (h == c) {
        xh[0] = *(const bf16x8 *)(s_hi + tx_addr(r, 0));
        xh[1] = *(const bf16x8 *)(s_hi + tx_addr(r, 1));
        xl[0] = *(const bf16x8 *)(s_lo + tx_addr(r, 0));
        xl[1] = *(const bf16x8 *)(s_lo + tx_addr(r, 1));
      }
    }
#pragma unroll
    for (int i = 0; i < IC; ++i) {
#pragma unroll
      for (int m = 1; m < LR; m <<= 1) xp[i] += __shfl_xor(xp[i], m, 64);
      if (lpos == 0) s_xx[RI * i + lrow] = xp[i];
    }
    wave_sync_w();
    xx = s_xx[r];
    prv = pv;
    if (build) {
      // DKM_IMAGE_BUILD: this tile of the split image (k_x_image_split's
      // layout: hi slices 0, 1 then lo 0, 1, lane l = row l & 31, features
      // 16 (l >> 5) + 8 s ..) and the screen's own fp32 |x|^2 -- the image
      // launches of later iterations then score exactly these operands
      bf16x8 *dst = (bf16x8 *)(img.tiles + (s0 >> 5) * 2048) + lane;
      dst[0] = xh[0];
      dst[64] = xh[1];
      dst[128] = xl[0];
      dst[192] = xl[1];
      if (h == 0) ((float *)img.xx)[s0 + r] = xx;
    }
    if (!full_acc && s_next < n) load_tile(s_next);
    }  // !IMG

    float r1 = INFINITY, r2 = INFINITY;
    int ri = 0;
    typedef float f32x16 __attribute__((ext_vector_type(16)));
    float xn;
    const float B2 = bound2_fast(bk, xx, xn);
    // HINT: p, s_hat_p (v_dot2 over this lane's 16 features of the bf16x3
    // operands, the two halves added), T
    const int p = prv;
    const bool pok = HINT && p >= 0 && p < k;
    float shp = INFINITY, T = INFINITY;
    if constexpr (HINT) {
      float dg = 0.f;
      if (pok) {
        const char *pf = frag + (int64_t)(p >> 5) * 4096 +
                         ((p & 31) + 32 * h) * 16;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 ch = *(const bf16x8 *)(pf + ks * 2048);
          const bf16x8 cl = *(const bf16x8 *)(pf + ks * 2048 + 1024);
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const bf16x2 c2h{ch[j], ch[j + 1]};
            dg = __builtin_amdgcn_fdot2_f32_bf16(
                bf16x2{xh[ks][j], xh[ks][j + 1]}, c2h, dg, false);
            dg = __builtin_amdgcn_fdot2_f32_bf16(
                bf16x2{xl[ks][j], xl[ks][j + 1]}, c2h, dg, false);
            dg = __builtin_amdgcn_fdot2_f32_bf16(
                bf16x2{xh[ks][j], xh[ks][j + 1]}, bf16x2{cl[j], cl[j + 1]},
                dg, false);
          }
        }
      }
      float da, db;
      pair_xor<32>(dg, da, db);
      dg = da + db;
      if (pok) {
        const int q = p & 31;
        shp = cn[(p >> 5) * 32 + 16 * ((q >> 2) & 1) +
                 ((q & 3) | ((q >> 3) << 2))] + dg;
        T = shp + B2;
      }
    }
    auto chain = [&](int cb, f32x16 &accv) {
      const bool pz = HINT && pok && (p >> 5) == cb && ((p >> 2) & 1) == h;
      const f32x4 *c4p =
          (const f32x4 *)(pz ? pcn + p * 16 : cn + cb * 32 + 16 * h);
      const f32x4 c0 = c4p[0], c1 = c4p[1], c2 = c4p[2], c3 = c4p[3];
      accv = f32x16{c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                    c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const char *blk = frag + ((int64_t)cb * 2 + ks) * 2048;
        const bf16x8 ah = *(const bf16x8 *)(blk + lane * 16);
        const bf16x8 al = *(const bf16x8 *)(blk + 1024 + lane * 16);
        accv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xh[ks], accv, 0, 0,
                                                       0);
        accv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xl[ks], accv, 0, 0,
                                                       0);
        accv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, xh[ks], accv, 0, 0,
                                                       0);
      }
    };
    if constexpr (HINT) {
      // the threshold pass: a block with no score <= T is done in 8 VALU
      auto test = [&](int cb, const f32x16 &accv) {
        const bool hit = min16(accv, ninf) <= T;
        if (__ballot(hit) == 0) return;
        if (hit) {
          float b1 = INFINITY, b2 = INFINITY;
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const float sq =
                __uint_as_float((__float_as_uint(accv[g]) & vmask) | g);
            b2 = __builtin_amdgcn_fmed3f(b1, b2, sq);
            b1 = min_nc(b1, sq, ninf);
          }
          const int g = (int)(__float_as_uint(b1) & 15);
          const int gi = cb * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
          const bool nw = b1 < r1;
          r2 = nw ? min_nc(r1, b2, ninf) : min_nc(r2, b1, ninf);
          ri = nw ? gi : ri;
          r1 = nw ? b1 : r1;
        }
      };
      f32x16 acc_a, acc_b;
      chain(0, acc_a);
      int cb = 0;
      for (; cb + 2 <= nkb; cb += 2) {
        chain(cb + 1, acc_b);
        test(cb, acc_a);
        if (cb + 2 < nkb) chain(cb + 2, acc_a);
        test(cb + 1, acc_b);
      }
      if (cb < nkb) test(cb, acc_a);
    }
    for (int g0 = 0; !HINT && g0 < nkb; g0 += GB) {
      const int g1 = min(nkb, g0 + GB);
      float b1 = INFINITY, b2 = INFINITY;
      auto score = [&](int cb, const f32x16 &accv) {
        const uint32_t t0 = opaque_s32((uint32_t)((cb - g0) * 16));
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const float sp =
              __uint_as_float((__float_as_uint(accv[g]) & vmask) | (t0 + g));
          b2 = __builtin_amdgcn_fmed3f(b1, b2, sp);
          b1 = min_nc(b1, sp, ninf);
        }
      };
      f32x16 acc_a, acc_b;
      chain(g0, acc_a);
      int cb = g0;
      for (; cb + 2 <= g1; cb += 2) {
        chain(cb + 1, acc_b);
        score(cb, acc_a);
        if (cb + 2 < g1) chain(cb + 2, acc_a);
        score(cb + 1, acc_b);
      }
      if (cb < g1) score(cb, acc_a);
      const uint32_t tg = __float_as_uint(b1) & PACK_MASK;
      const int g = (int)(tg & 15);
      const int gi = (g0 + (int)(tg >> 4)) * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
      const bool nw = b1 < r1;
      r2 = nw ? min_nc(r1, b2, ninf) : min_nc(r2, b1, ninf);
      ri = nw ? gi : ri;
      r1 = nw ? b1 : r1;
    }
    {  // merge the two lanes of a sample (symmetric in the pair)
      float a1, c1, a2, c2;
      int ai, ci;
      pair_xor<32>(r1, a1, c1);
      pair_xor<32>(r2, a2, c2);
      pair_xor<32>(ri, ai, ci);
      const bool tc = (c1 < a1) | ((c1 == a1) & (ci < ai));
      r1 = tc ? c1 : a1;
      ri = tc ? ci : ai;
      r2 = tc ? min_nc(a1, c2, ninf) : min_nc(a2, c1, ninf);
    }
    if (HINT && pok) {
      // the kept scores (all <= T) with p's: every other centre is > T
      const bool tk = (shp < r1) | ((shp == r1) & (p < ri));
      r2 = tk ? r1 : min_nc(r2, shp, ninf);
      ri = tk ? p : ri;
      r1 = tk ? shp : r1;
    }
    const int64_t si = s0 + r;
    const bool sane = (xn < 1e18f) & (xn * cm < 1e30f) & (r1 < 1e30f);
    const bool unique = sane & (r2 - r1 > B2);
    const bool und = si < n && !unique;
    const int prev = delta ? prv : -1;
    const uint64_t um = __ballot(h == 0 && und);
    const int add = __popcll(um);
    if (listing && tl_cnt + add <= TL_CAP) {
      if (h == 0 && und)
        wl[tl_cnt + lane_prefix(um)] =
            make_int2((int)(si - base), prev);
      tl_cnt += add;
    } else {
      tl_over += add;
    }
    if (!IMG && full_acc) {
      // the loading lanes add their pieces of the decided rows
      if (h == 0) s_lab[r] = si < n && unique ? ri : -1;
      wave_sync_w();
#pragma unroll
      for (int i = 0; i < IC; ++i) {
        const int row = RI * i + lrow;
        const int lb = s_lab[row];
        if (lb >= 0) {
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
              const int t = 16 * c + EPL * lpos + e;
              if (t < d) at.add(lb, t, (double)raw[c][i][e]);
            }
          if (lpos == 0) at.count(lb, 1.0);
        }
      }
    }
    if (si < n) {
      const int lab = ri;
      if (h == 0 && !(unique && lab == prev))
        lab_out[si] = unique ? lab : -(prev + 2);
      if (unique) {
        if (full_acc) {
          // added above
        } else if (delta && lab != prev && !mlist) {
          const TX *xr = X + si * ldx;
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int m = 0; m < 8; ++m) {
              const int t = 16 * h + 8 * ks + m;
              if (t < d) {
                const double x = ld_x(xr + t);
                at.add(lab, t, x);
                if (prev >= 0) at.add(prev, t, -x);
              }
            }
          if (h == 0) {
            at.count(lab, 1.0);
            if (prev >= 0) at.count(prev, -1.0);
          }
        }
      }
    }
    if (mlist) {
      // a row the screen moved: listed with its previous label
      const bool mv = h == 0 && si < n && unique && ri != prev;
      const uint64_t mm = __ballot(mv);
      if (mm) {
        const int c = __popcll(mm);
        if (mcnt + c > W32_MLB) mflush();
        if (mv) {
          mbuf[mcnt + lane_prefix(mm)] = (int)si;
          v.queue[si] = prev;
        }
        mcnt += c;
      }
    }
    if (!IMG && full_acc && s_next < n) load_tile(s_next);
  }
  if (mlist && mcnt) mflush();
  if (lane == 0) {
    if (listing) v.tcount[seg] = tl_cnt;
    if (tl_over) atomicAdd(&v.hdr->qcount, (uint32_t)tl_over);
  }
  if (amode & AM_INLDS) {
    __syncthreads();
    flush_lds_acc(lds_acc, acc, k, d);
  }
}

// ---------------------------------------------------------------------------
// The chunked bf16x3 screen on v_mfma_f32_32x32x16_bf16 (k_screen_c32):
// labels-only launches with k x d fragments beyond LDS and 32 < d <= 64
// (C3's first assignment, against the crowded initial centres).  k_screen's
// 16x16x32 form read each fragment for 16 samples; this one reads it for 32
// -- half the MFMA and LDS instructions per score and half the L2 -> LDS
// fragment traffic per sample -- with the per-score work unchanged (the
// packed top-2 of k_screen_w32's non-hinted pass).  Centres on the A rows in
// b1frag's order (block cb, K-step ks: lane (r, h) holds -2c[32cb + r][16ks
// + 8h + j], hi in b1frag, lo in b1frag_lo), staged through LDS in chunks of
// C32_CB blocks; lane (r, h) of a wave holds sample r's features 16ks + 8h +
// j as the B operand, converted from its fp64 row at the step's start (a
// prefetched row cost 64 VGPRs: 2 waves per SIMD).  Output as k_screen's: labels, or
// -(prev + 2) and the wave's undecided list.
constexpr int SB32C = 512;  // 8 waves share each LDS chunk
// 32-centre blocks per chunk: what LDS_BUDGET holds, rounded down to whole
// packing groups of 8 (9 at NK = 4 left a one-block group and a short last
// chunk: 8 is 1 ms faster at C3, profiles/r06/c3ab/r06zi_c32_cb8_ab.txt)
template <int NK>
constexpr int c32_cb() {
  constexpr int c = (int)(LDS_BUDGET / (NK * 2048 + 128));
  return c >= 8 ? c / 8 * 8 : c;
}
template <class TX, int NK>
__global__ void __launch_bounds__(SB32C) __attribute__((amdgpu_waves_per_eu(4)))
    k_screen_c32(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                 int k, WsView v, int32_t *__restrict__ lab_out, int64_t base,
                 int use_list) {
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  constexpr int CB = c32_cb<NK>();
  constexpr int GB = 8;  // 32-centre blocks per packing group (128 tags)
  extern __shared__ __attribute__((aligned(16))) double smem[];
  char *frag = (char *)smem;                           // CB x NK x 2 KB
  float *cnl = (float *)(frag + (int64_t)CB * NK * 2048);  // CB x 32
  const int nkb = (int)(kpad32(k) / 32);
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  const BoundK bk = bound_consts<P_B3>(d, cm);
  const float ninf = __uint_as_float(opaque_u32(0xff800000u));
  const uint32_t vmask = opaque_u32(~PACK_MASK);
  const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t seg = (int64_t)blockIdx.x * (SB32C / 64) + wid;
  const int64_t step = (int64_t)gridDim.x * (SB32C / 64) * 32;
  int2 *wl = v.tlist + seg * TL_CAP;
  const bool listing = use_list && seg < TL_SEGS;
  int tl_cnt = 0, tl_over = 0;
  // LDS <- blocks [c0, c1): hi then lo fragments per (block, K-step), and
  // the blocks' norms in accumulator order
  auto load_chunk = [&](int c0, int c1) {
    const f32x4 *hs = (const f32x4 *)(v.b1frag + (int64_t)c0 * NK * 512);
    const f32x4 *ls = (const f32x4 *)(v.b1frag_lo + (int64_t)c0 * NK * 512);
    f32x4 *dst = (f32x4 *)frag;
    for (int e = threadIdx.x; e < (c1 - c0) * NK * 64; e += SB32C) {
      const int blk = e >> 6, w = e & 63;
      dst[blk * 128 + w] = hs[e];
      dst[blk * 128 + 64 + w] = ls[e];
    }
    for (int e = threadIdx.x; e < (c1 - c0) * 32; e += SB32C)
      cnl[e] = v.cn32f[c0 * 32 + e];
  };
  // this lane's piece of its sample's row: features 16ks + 8h + j
  double raw[NK][8];
  auto load_row = [&](int64_t s0) {
    const int64_t si = s0 + r;
    const bool ok = si < n;
    const TX *xr = X + (ok ? si : 0) * ldx;
#pragma unroll
    for (int ks = 0; ks < NK; ++ks) {
      const int t0 = 16 * ks + 8 * h;
      if (ok && t0 + 8 <= d) {
        if constexpr (sizeof(TX) == 8) {
          const double2 *p = (const double2 *)(xr + t0);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const double2 u = p[q];
            raw[ks][2 * q] = u.x;
            raw[ks][2 * q + 1] = u.y;
          }
        } else {
          const float4 *p = (const float4 *)(xr + t0);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const float4 u = p[q];
            raw[ks][4 * q] = u.x;
            raw[ks][4 * q + 1] = u.y;
            raw[ks][4 * q + 2] = u.z;
            raw[ks][4 * q + 3] = u.w;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) raw[ks][j] = 0.0;
      }
    }
  };
  // the block-uniform step loop (every wave reaches the chunk barriers)
  const int64_t wofs = (int64_t)wid * 32;
  int64_t s0 = base + seg * 32;
  for (; s0 - wofs < n; s0 += step) {
    load_row(s0);
    bf16x8 xh[NK], xl[NK];
    float xx = 0.f;
#pragma unroll
    for (int ks = 0; ks < NK; ++ks)
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const float x0 = (float)raw[ks][j], x1 = (float)raw[ks][j + 1];
        xx = fmaf(x0, x0, xx);
        xx = fmaf(x1, x1, xx);
        const bf16x2 h2 = __builtin_convertvector(f32x2{x0, x1}, bf16x2);
        const uint32_t hu = __builtin_bit_cast(uint32_t, h2);
        const bf16x2 l2 = __builtin_convertvector(
            f32x2{x0 - __uint_as_float(hu << 16),
                  x1 - __uint_as_float(hu & 0xffff0000u)},
            bf16x2);
        xh[ks][j] = h2[0];
        xh[ks][j + 1] = h2[1];
        xl[ks][j] = l2[0];
        xl[ks][j + 1] = l2[1];
      }
    {
      float xa, xb;
      pair_xor<32>(xx, xa, xb);
      xx = xa + xb;
    }
    float r1 = INFINITY, r2 = INFINITY;
    int ri = 0;
    int cbase = 0;
    auto chain = [&](int cb, f32x16 &accv) {
      const f32x4 *c4p = (const f32x4 *)(cnl + (cb - cbase) * 32 + 16 * h);
      const f32x4 c0 = c4p[0], c1 = c4p[1], c2 = c4p[2], c3 = c4p[3];
      accv = f32x16{c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                    c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
#pragma unroll
      for (int ks = 0; ks < NK; ++ks) {
        const char *blk = frag + ((int64_t)(cb - cbase) * NK + ks) * 2048;
        const bf16x8 ah = *(const bf16x8 *)(blk + lane * 16);
        const bf16x8 al = *(const bf16x8 *)(blk + 1024 + lane * 16);
        accv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xh[ks], accv, 0, 0,
                                                       0);
        accv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xl[ks], accv, 0, 0,
                                                       0);
        accv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, xh[ks], accv, 0, 0,
                                                       0);
      }
    };
    for (int c0 = 0; c0 < nkb; c0 += CB) {
      const int c1 = min(nkb, c0 + CB);
      __syncthreads();  // every wave is done with the previous chunk
      load_chunk(c0, c1);
      __syncthreads();
      cbase = c0;
      for (int g0 = c0; g0 < c1; g0 += GB) {
        const int g1 = min(c1, g0 + GB);
        float b1 = INFINITY, b2 = INFINITY;
        auto score = [&](int cb, const f32x16 &accv) {
          const uint32_t t0 = opaque_s32((uint32_t)((cb - g0) * 16));
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const float sp = __uint_as_float(
                (__float_as_uint(accv[g]) & vmask) | (t0 + g));
            b2 = __builtin_amdgcn_fmed3f(b1, b2, sp);
            b1 = min_nc(b1, sp, ninf);
          }
        };
        f32x16 acc_a, acc_b;
        chain(g0, acc_a);
        int cb = g0;
        for (; cb + 2 <= g1; cb += 2) {
          chain(cb + 1, acc_b);
          score(cb, acc_a);
          if (cb + 2 < g1) chain(cb + 2, acc_a);
          score(cb + 1, acc_b);
        }
        if (cb < g1) score(cb, acc_a);
        const uint32_t tg = __float_as_uint(b1) & PACK_MASK;
        const int g = (int)(tg & 15);
        const int gi =
            (g0 + (int)(tg >> 4)) * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
        const bool nw = b1 < r1;
        r2 = nw ? min_nc(r1, b2, ninf) : min_nc(r2, b1, ninf);
        ri = nw ? gi : ri;
        r1 = nw ? b1 : r1;
      }
    }
    {  // merge the two lanes of a sample (symmetric in the pair)
      float a1, c1, a2, c2;
      int ai, ci;
      pair_xor<32>(r1, a1, c1);
      pair_xor<32>(r2, a2, c2);
      pair_xor<32>(ri, ai, ci);
      const bool tc = (c1 < a1) | ((c1 == a1) & (ci < ai));
      r1 = tc ? c1 : a1;
      ri = tc ? ci : ai;
      r2 = tc ? min_nc(a1, c2, ninf) : min_nc(a2, c1, ninf);
    }
    float xn;
    const float B2 = bound2_fast(bk, xx, xn);
    const int64_t si = s0 + r;
    const bool sane = (xn < 1e18f) & (xn * cm < 1e30f) & (r1 < 1e30f);
    const bool unique = sane & (r2 - r1 > B2);
    const bool und = si < n && !unique;
    const uint64_t um = __ballot(h == 0 && und);
    const int add = __popcll(um);
    if (listing && tl_cnt + add <= TL_CAP) {
      if (h == 0 && und)
        wl[tl_cnt + lane_prefix(um)] = make_int2((int)(si - base), -1);
      tl_cnt += add;
    } else {
      tl_over += add;
    }
    if (h == 0 && si < n) lab_out[si] = unique ? ri : -1;
  }
  if (lane == 0) {
    if (listing) v.tcount[seg] = tl_cnt;
    if (tl_over) atomicAdd(&v.hdr->qcount, (uint32_t)tl_over);
  }
}

template <class TX>
static int launch_screen_c32(const TX *X, int64_t end, int d, int64_t ldx,
                             int k, const WsView &v, int32_t *lab_out,
                             int64_t base, int use_list, hipStream_t s,
                             int *nseg) {
  const int nk = (int)(dpad16(d) / 16);
  if (!v.b1frag || !v.b1frag_lo || nk < 3 || nk > 4) return 1;
  const void *kf = nk == 3 ? (const void *)k_screen_c32<TX, 3>
                           : (const void *)k_screen_c32<TX, 4>;
  const size_t lds = nk == 3 ? (size_t)c32_cb<3>() * (3 * 2048 + 128)
                             : (size_t)c32_cb<4>() * (4 * 2048 + 128);
  if (hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return fail(DKM_E_LAUNCH, "screen_c32: LDS attribute");
  const int64_t cap = (int64_t)dev_info().cus * resident_blocks(kf, SB32C, lds);
  const int64_t per_block = 32 * (SB32C / 64);
  const int64_t need = (end - base + per_block - 1) / per_block;
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min(need, cap));
  *nseg = (int)std::min<int64_t>((int64_t)g * (SB32C / 64), TL_SEGS);
  if (nk == 3)
    k_screen_c32<TX, 3><<<g, SB32C, lds, s>>>(X, end, d, ldx, k, v, lab_out,
                                              base, use_list);
  else
    k_screen_c32<TX, 4><<<g, SB32C, lds, s>>>(X, end, d, ldx, k, v, lab_out,
                                              base, use_list);
  return check_launch("screen assignment (chunked 32x32)");
}

// ---------------------------------------------------------------------------
// Single-product screen (P_B1) for k x d beyond the LDS sums budget with the
// bf16 centres resident in LDS (b1_ok: C3's k = 1000, d = 64).  One product
// per term -- xh.ch on v_mfma_f32_32x32x16_bf16 -- a third of bf16x3's
// matrix work, with its own bound:
//   x -> fl32 -> bf16 and -2c -> fl32 -> bf16 (round to nearest) lose
//   <= 2^-8 each (unit roundoff of an 8-bit significand), a product
//   <= (2^-7 + 2^-16) |x (-2c)|; B = 2 (1.02 2^-8 + (16 NKS + 2) 2^-23) mag
//   covers that, the fp32 chain of dpad products + |c|^2, packing 2^PACK1
//   ulp and numpy's rounding (screen_bound's terms).  Unlike bf16x3's, this
//   B is not doubled beyond the rigorous value: the slack is the 1.02.
// The looser bound leaves ~5% of converged C3 samples undecided, nearly all
// with exactly two candidates, so each lane keeps a packed top-3 (4 VALU
// ops per score: pack, 2 x med3, min) and the decision is three-way:
//   s2 - s1 > 2B            -> the label;
//   s3 - s1 > 2B (else)     -> candidates {c1, c2}: the per-wave candidate
//                              list (k_cand2: reference arithmetic on both);
//   otherwise               -> the re-check list (k_recheck_list).
// Labels only (amode none): the sums of these shapes come from
// k_label_sums.  Lane l = (r = l & 31, h = l >> 5) holds features
// 16ks + 8h .. +7 of sample r for every K-step ks; accumulator register g
// = centre cb*32 + (g & 3) + 8 (g >> 2) + 4h, tag = (block in group) x 16 + g
// in PACK1 = 9 bits (groups of 32 blocks = 1024 centres).
// ---------------------------------------------------------------------------
// 16 waves per CU (one block: the centres fill the LDS), <= 128 VGPRs: no
// register prefetch of the next tile -- the CU's other waves cover a
// wave's load (at 2 waves per SIMD with a prefetched tile the kernel waited
// 48% of its cycles: PMC r02a)
#ifndef DKM_AB_SBB
#define DKM_AB_SBB 768
#endif
constexpr int SBB = DKM_AB_SBB;
constexpr uint32_t PACK1 = 9, PACK1_MASK = (1u << PACK1) - 1;
// threshold pass: at most this many of a wave's 32 samples may end with an
// over-full (or unusable) candidate list before the wave redoes the tile
// with the top-3 pass
constexpr int B1_RTHR = 4;

template <class TX, int NKS>
__global__ void __launch_bounds__(SBB)
    k_screen_b1(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                int k, WsView v, int32_t *__restrict__ lab_out, int64_t base,
                int delta, int hint) {
  constexpr int GB = 1 << (PACK1 - 4);  // 32-centre blocks per group
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nkb = (int)(kpad32(k) / 32);
  char *frag = (char *)smem;                                // nkb x NKS KB
  float *cn = (float *)(frag + (int64_t)nkb * NKS * 1024);  // nkb x 32
  {
    const f32x4 *src = (const f32x4 *)v.b1frag;
    f32x4 *dst = (f32x4 *)frag;
    for (int e = threadIdx.x; e < nkb * NKS * 64; e += SBB) dst[e] = src[e];
    for (int e = threadIdx.x; e < nkb * 32; e += SBB) cn[e] = v.cn32f[e];
    // hint == 2: the norm chunks with one slot poisoned (+inf), chunk
    // (block, half, 4-slot group j, slot t) at ((cb * 2 + h) * 4 + j) * 4 + t
    if (hint == 2)
      for (int e = threadIdx.x; e < nkb * 32; e += SBB) {
        const f32x4 c = ((const f32x4 *)v.cn32f)[e >> 2];
        f32x4 *dst = (f32x4 *)(cn + nkb * 32) + e;
        (*dst) = c;
        (*dst)[e & 3] = INFINITY;
      }
  }
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  // bound constants (screen_bound's terms with the single-product split)
  const float rel = 1.02f * 0x1.0p-8f + (16.0f * NKS + 2.0f) * 0x1.0p-23f;
  BoundK bk = bound_consts<P_F32>(d, cm);
  bk.k_mag = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(
      2.0f * (2.0f * rel + 0x1.0p-23f * (float)(1u << PACK1)) * 1.0001f)));
  const float ninf = __uint_as_float(opaque_u32(0xff800000u));
  const uint32_t vmask = opaque_u32(~PACK1_MASK);
  __syncthreads();

  const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t wv = (int64_t)blockIdx.x * (SBB / 64) + wid;
  const int64_t step = (int64_t)gridDim.x * (SBB / 64) * 32;
  int2 *wl = v.tlist + wv * TL_CAP;  // >= 3 candidates
  int2 *cl = v.clist + wv * B1_CAP;  // 2 candidates
  int4 *nl = v.nlist + wv * B1_NCAP; // 3..6 candidates
  int nl_cnt = 0;
  const bool listing = wv < TL_SEGS && wv < B1_SEGS;
  int tl_cnt = 0, cl_cnt = 0, tl_over = 0;
  uint32_t t_tiles = 0, t_done = 0;  // threshold passes run / accepted


  double tile[NKS][8];
  int pv = -1;
  const uint32_t lane_off = (uint32_t)(r * ldx * (int64_t)sizeof(TX)) +
                            (uint32_t)(8 * h * sizeof(TX));
  auto load_tile = [&](int64_t s0) {
    const int64_t rows = std::max<int64_t>(0, n - s0);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(X + std::min(s0, n) * ldx), 0,
        (int)std::min<int64_t>(rows * ldx * (int64_t)sizeof(TX), 0x7fffffff),
        0x00020000);
    if (delta || hint) {
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(lab_out + std::min(s0, n)), 0,
          (int)std::min<int64_t>(rows * 4, 0x7fffffff), 0x00020000);
      pv = (int)__builtin_amdgcn_raw_buffer_load_b32(rl, r * 4, 0, 0);
    }
    // every load of the tile is issued unconditionally, so one wait covers
    // them all (loads under a lane-dependent `16 ks + 8 h < d` branch each
    // waited inside their branch: NKS serial HBM round trips per tile).
    // Loads past the last row read 0 (num_records); features past d of a
    // row read its successor and are zeroed below.
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int o = 16 * ks * (int)sizeof(TX);
      if constexpr (sizeof(TX) == 8) {
#pragma unroll
        for (int p4 = 0; p4 < 4; ++p4) {
          const double2 v2 = __builtin_bit_cast(
              double2, __builtin_amdgcn_raw_buffer_load_b128(
                           rx, lane_off, o + 16 * p4, 0));
          tile[ks][2 * p4] = v2.x;
          tile[ks][2 * p4 + 1] = v2.y;
        }
      } else {
#pragma unroll
        for (int p4 = 0; p4 < 2; ++p4) {
          const float4 v4 = __builtin_bit_cast(
              float4, __builtin_amdgcn_raw_buffer_load_b128(
                          rx, lane_off, o + 16 * p4, 0));
          tile[ks][4 * p4] = v4.x;
          tile[ks][4 * p4 + 1] = v4.y;
          tile[ks][4 * p4 + 2] = v4.z;
          tile[ks][4 * p4 + 3] = v4.w;
        }
      }
    }
    if (d != 16 * NKS) {  // wave-uniform
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int m = 0; m < 8; ++m)
          tile[ks][m] = 16 * ks + 8 * h + m < d ? tile[ks][m] : 0.0;
    }
  };

  typedef float f32x16 __attribute__((ext_vector_type(16)));
#ifndef DKM_AB_B1_PREFETCH
#define DKM_AB_B1_PREFETCH 0
#endif
  // A/B: prefetch the next tile (and its labels) into the tile registers
  // as soon as the current one is converted (needs ~64 more VGPRs: pair
  // with a smaller block, -DDKM_AB_SBB=512)
  if (DKM_AB_B1_PREFETCH && base + wv * 32 < n) load_tile(base + wv * 32);
  for (int64_t s0 = base + wv * 32; s0 < n; s0 += step) {
    if (!DKM_AB_B1_PREFETCH) load_tile(s0);
    float xx = 0.f;
    bf16x8 xh[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int m = 0; m < 8; m += 2) {
        const float x0 = (float)tile[ks][m];
        const float x1 = (float)tile[ks][m + 1];
        xx = fmaf(x0, x0, xx);
        xx = fmaf(x1, x1, xx);
        const bf16x2 h2 = __builtin_convertvector(f32x2{x0, x1}, bf16x2);
        xh[ks][m] = h2[0];
        xh[ks][m + 1] = h2[1];
      }
    {
      float xa, xb;
      pair_xor<32>(xx, xa, xb);
      xx = xa + xb;
    }
    const int prv = pv;
    if (DKM_AB_B1_PREFETCH && s0 + step < n) load_tile(s0 + step);
    const int64_t si = s0 + r;
    float xn;
    const float B2 = bound2_fast(bk, xx, xn);
    const bool sane0 = (xn < 1e18f) & (xn * cm < 1e30f);
    bool unique = false, two = false, many = false;
    int i1 = 0, i2 = 0;
    uint32_t mpk0 = 0, mpk1 = 0, mpk2 = 0;  // many: the candidate set
    bool need3 = true;
    auto chain = [&](int cb, f32x16 &accv) {
      const f32x4 *c4p = (const f32x4 *)(cn + cb * 32 + 16 * h);
      const f32x4 c0 = c4p[0], c1 = c4p[1], c2 = c4p[2], c3 = c4p[3];
      accv = f32x16{c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                    c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 ah =
            *(const bf16x8 *)(frag + ((int64_t)cb * NKS + ks) * 1024 +
                              lane * 16);
        accv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xh[ks], accv, 0, 0,
                                                       0);
      }
    };
    if (hint) {
      // ---- threshold pass (label hint p = the sample's incoming label) ----
      // s_hat_p: this sample's score against centre p from the same bf16
      // operands (exact bf16 products, fp32 sums: within the single-product
      // bound B = B2 / 2 of the reference distance, like every MFMA score).
      // T = s_hat_p + B2: a centre j with s_j > T has D_j > D_p, so it is
      // neither the reference winner nor tied with it.  Only the scores
      // <= T are kept (the hint's own centre always is), so a lane spends
      // one compare per score instead of the top-3's four ops.
      const bool pok = prv >= 0 && prv < k;
      const uint64_t bad = __ballot(!pok && s0 + r < n);
      if (__popcll(bad) <= 2 * B1_RTHR) {
        const int p = pok ? prv : 0;
        const int pcb = p >> 5, pw = p & 31;
        float dot = 0.f;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8 cp = *(const bf16x8 *)(frag + ((int64_t)pcb * NKS + ks) *
                                                         1024 + (pw + 32 * h) * 16);
#pragma unroll
          for (int m = 0; m < 8; ++m)
            dot = fmaf((float)xh[ks][m], (float)cp[m], dot);
        }
        {
          float da, db;
          pair_xor<32>(dot, da, db);
          dot = da + db;
        }
        const float sp =
            cn[pcb * 32 + 16 * ((pw >> 2) & 1) + (pw & 3) + 4 * (pw >> 3)] + dot;
        const float T = pok ? sp + B2 : -INFINITY;
        // hint == 2: the lane holding centre p's score (half (p >> 2) & 1)
        // reads p's norm as +inf in block p >> 5, so its MFMA score for p
        // never passes the test, and starts its kept list with (s_hat_p, p)
        // instead: s_hat_p is a score of p from the same bf16 operands,
        // within the same bound.  Without it every sample's own group took
        // the append branches once per tile.
        const bool own_l = hint == 2 && pok && h == ((pw >> 2) & 1);
        const int own_cb = own_l ? pcb : -1, own_j = pw >> 3;
        const f32x4 *own_p = (const f32x4 *)(cn + nkb * 32) +
                             ((pcb * 2 + h) * 4 + own_j) * 4 + (pw & 3);
        // up to 3 kept (score, centre) per lane, in scan order; cnt counts all
        float q0 = own_l ? sp : INFINITY, q1 = INFINITY, q2 = INFINITY;
        int j0 = own_l ? p : 0, j1 = 0, j2 = 0, cnt = own_l ? 1 : 0;
        // each block is tested whole, interleaved with the next block's MFMA
        // chain: 8 v_med3 pair minima, a v_min3 tree and one compare (13
        // VALU) and a single branch; the 4-register group tests and the
        // per-register appends run only inside a taken block, which with the
        // own centre poisoned means an ambiguous sample (rare).  Per-group
        // branches (16 VALU, 4 branches a block) ran 28.3 against 26.6 ms
        // per C3 step (profiles/r02/ab_m3/).
#ifndef DKM_AB_B1_PROBE
#define DKM_AB_B1_PROBE 0
#endif
        float probe = 0.f;  // A/B timing probes only (results invalid)
        auto test_blk = [&](const f32x16 &accv, float (&m)[8], bool &any) {
          if (DKM_AB_B1_PROBE == 2) {
            probe = fmaxf(probe, accv[0]);
            any = false;
            return;
          }
#pragma unroll
          for (int i = 0; i < 8; ++i)
            m[i] = __builtin_amdgcn_fmed3f(accv[2 * i], accv[2 * i + 1], ninf);
          const float a = fminf(fminf(m[0], m[1]), m[2]);
          const float b = fminf(fminf(m[3], m[4]), m[5]);
          const float c = fminf(fminf(m[6], m[7]), a);
          any = fminf(b, c) <= T;
        };
        auto append = [&](int cb, const f32x16 &accv, const bool (&gh)[4]) {
          if (DKM_AB_B1_PROBE) {
            probe += (gh[0] | gh[1] | gh[2] | gh[3]) ? 1.f : 0.f;
            return;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (gh[q]) {
#pragma unroll
              for (int g = 4 * q; g < 4 * q + 4; ++g) {
                const float sc = accv[g];
                if (sc <= T) {
                  const int ci = cb * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
                  q2 = cnt == 2 ? sc : q2;
                  j2 = cnt == 2 ? ci : j2;
                  q1 = cnt == 1 ? sc : q1;
                  j1 = cnt == 1 ? ci : j1;
                  q0 = cnt == 0 ? sc : q0;
                  j0 = cnt == 0 ? ci : j0;
                  ++cnt;
                }
              }
            }
          }
        };
        // two-stage pipeline over the centre blocks: the LDS reads of block
        // cb + 1 (norms into its accumulator, fragments into registers) are
        // issued before block cb is scored, and its MFMA chain after, so
        // no MFMA waits on an LDS read issued just before it
        auto rd = [&](int cb, bf16x8 (&f)[NKS], f32x16 &accv) {
          const f32x4 *c4p = (const f32x4 *)(cn + cb * 32 + 16 * h);
          const bool own = cb == own_cb;
          const f32x4 c0 = *(own && own_j == 0 ? own_p : c4p),
                      c1 = *(own && own_j == 1 ? own_p : c4p + 1),
                      c2 = *(own && own_j == 2 ? own_p : c4p + 2),
                      c3 = *(own && own_j == 3 ? own_p : c4p + 3);
          accv = f32x16{c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                        c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks)
            f[ks] = *(const bf16x8 *)(frag + ((int64_t)cb * NKS + ks) * 1024 +
                                      lane * 16);
        };
        auto mm = [&](const bf16x8 (&f)[NKS], f32x16 &accv) {
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks)
            accv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[ks], xh[ks], accv,
                                                           0, 0, 0);
        };
        auto append_blk = [&](int cb, const f32x16 &accv, const float (&m)[8],
                              bool any) {
          if (any) {
            bool gh[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
              gh[q] = __builtin_amdgcn_fmed3f(m[2 * q], m[2 * q + 1], ninf) <= T;
            append(cb, accv, gh);
          }
        };
        {
          f32x16 acc_a, acc_b;
          bf16x8 fa[NKS], fb[NKS];
          float ma[8], mb[8];
          bool ga, gb;
          auto interleave = [&]() {
            __builtin_amdgcn_sched_group_barrier(0x100, 4 + NKS, 0);  // DS rd
#pragma unroll
            for (int i = 0; i < NKS; ++i) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
              __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU
            }
          };
          rd(0, fa, acc_a);
          mm(fa, acc_a);
          int cb = 0;
          for (; cb + 2 < nkb; cb += 2) {
            rd(cb + 1, fb, acc_b);
            test_blk(acc_a, ma, ga);
            mm(fb, acc_b);
            interleave();
            append_blk(cb, acc_a, ma, ga);
            rd(cb + 2, fa, acc_a);
            test_blk(acc_b, mb, gb);
            mm(fa, acc_a);
            interleave();
            append_blk(cb + 1, acc_b, mb, gb);
          }
          if (cb + 1 < nkb) {
            rd(cb + 1, fb, acc_b);
            test_blk(acc_a, ma, ga);
            mm(fb, acc_b);
            interleave();
            append_blk(cb, acc_a, ma, ga);
            test_blk(acc_b, mb, gb);
            append_blk(cb + 1, acc_b, mb, gb);
          } else {
            test_blk(acc_a, ma, ga);
            append_blk(cb, acc_a, ma, ga);
          }
        }
        if (DKM_AB_B1_PROBE) {  // keep the hint as the only candidate
          cnt = (probe == 12345.f || h != ((pw >> 2) & 1)) ? 0 : 1;
          q0 = sp;
          j0 = p;
        }
        // the sample's two lanes: union of their kept lists
        int ocnt, oj0, oj1, oj2;
        float oq0, oq1, oq2;
        ocnt = __shfl_xor(cnt, 32, 64);
        oq0 = __shfl_xor(q0, 32, 64);
        oq1 = __shfl_xor(q1, 32, 64);
        oq2 = __shfl_xor(q2, 32, 64);
        oj0 = __shfl_xor(j0, 32, 64);
        oj1 = __shfl_xor(j1, 32, 64);
        oj2 = __shfl_xor(j2, 32, 64);
        const bool over = cnt > 3 || ocnt > 3 || cnt + ocnt == 0 || !pok ||
                          !sane0 || !(T < 1e30f);
        // best by (score, centre) over the <= 6 kept, then how many lie
        // within B2 of it (the reference winner is among those)
        float sv[6] = {q0, q1, q2, oq0, oq1, oq2};
        int cv[6] = {j0, j1, j2, oj0, oj1, oj2};
        bool ok[6] = {cnt > 0, cnt > 1, cnt > 2, ocnt > 0, ocnt > 1, ocnt > 2};
        float bs = INFINITY;
        int bc = 0x7fffffff;
#pragma unroll
        for (int e = 0; e < 6; ++e)
          if (ok[e] && (sv[e] < bs || (sv[e] == bs && cv[e] < bc))) {
            bs = sv[e];
            bc = cv[e];
          }
        int namb = 0, other = 0;
        uint32_t pk[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu};
#pragma unroll
        for (int e = 0; e < 6; ++e)
          if (ok[e] && !(sv[e] - bs > B2)) {
            // the ambiguous members, packed 16 bits each in kept order
#pragma unroll
            for (int w = 0; w < 6; ++w)
              if (w == namb)
                pk[w >> 1] = (w & 1) ? (pk[w >> 1] & 0xffffu) |
                                           ((uint32_t)cv[e] << 16)
                                     : (pk[w >> 1] & 0xffff0000u) |
                                           (uint32_t)cv[e];
            ++namb;
            other = cv[e] != bc ? cv[e] : other;
          }
        const uint64_t mo = __ballot(over && s0 + r < n && h == 0);
        ++t_tiles;
        if (__popcll(mo) <= B1_RTHR) {
          ++t_done;
          need3 = false;
          unique = !over && namb == 1;
          two = !over && namb == 2;
          many = !over && namb >= 3;
          i1 = bc;
          i2 = other;
          mpk0 = pk[0];
          mpk1 = pk[1];
          mpk2 = pk[2];
        }

      }
    }
    if (need3) {
      // running (value, centre) top-3 of this lane over all groups
      float r1 = INFINITY, r2 = INFINITY, r3 = INFINITY;
      int ii1 = 0, ii2 = 0, ii3 = 0;
      for (int g0 = 0; g0 < nkb; g0 += GB) {
        const int g1 = min(nkb, g0 + GB);
        // two independent packed top-3 chains (even / odd registers): half
        // the dependency depth of one chain; merged at the group fold
        float b1 = INFINITY, b2 = INFINITY, b3 = INFINITY;
        float e1 = INFINITY, e2 = INFINITY, e3 = INFINITY;
        auto score = [&](int cb, const f32x16 &accv) {
          const uint32_t t0 = opaque_s32((uint32_t)((cb - g0) * 16));
  #pragma unroll
          for (int g = 0; g < 16; g += 2) {
            const float sp =
                __uint_as_float((__float_as_uint(accv[g]) & vmask) | (t0 + g));
            const float sq = __uint_as_float(
                (__float_as_uint(accv[g + 1]) & vmask) | (t0 + g + 1));
            b3 = __builtin_amdgcn_fmed3f(b2, b3, sp);
            b2 = __builtin_amdgcn_fmed3f(b1, b2, sp);
            b1 = min_nc(b1, sp, ninf);
            e3 = __builtin_amdgcn_fmed3f(e2, e3, sq);
            e2 = __builtin_amdgcn_fmed3f(e1, e2, sq);
            e1 = min_nc(e1, sq, ninf);
          }
        };
        f32x16 acc_a, acc_b;
        chain(g0, acc_a);
        int cb = g0;
        for (; cb + 2 <= g1; cb += 2) {  // ping-pong: no runtime-indexed arrays
          chain(cb + 1, acc_b);
          score(cb, acc_a);
          if (cb + 2 < g1) chain(cb + 2, acc_a);
          score(cb + 1, acc_b);
        }
        if (cb < g1) score(cb, acc_a);
        // fold the group's packed top-3 into the running (value, index) top-3
        auto gidx = [&](float p) {
          const uint32_t tg = __float_as_uint(p) & PACK1_MASK;
          const int g = (int)(tg & 15);
          return (g0 + (int)(tg >> 4)) * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
        };
        auto ins = [&](float p) {
          const int pi = gidx(p);
          const bool c1 = p < r1, c2 = p < r2, c3 = p < r3;
          r3 = c2 ? r2 : (c3 ? p : r3);
          ii3 = c2 ? ii2 : (c3 ? pi : ii3);
          r2 = c1 ? r1 : (c2 ? p : r2);
          ii2 = c1 ? ii1 : (c2 ? pi : ii2);
          r1 = c1 ? p : r1;
          ii1 = c1 ? pi : ii1;
        };
        ins(b1);
        ins(b2);
        ins(b3);
        ins(e1);
        ins(e2);
        ins(e3);
      }
      {  // merge the two lanes of a sample: the top-3 of both triples under
         // the (value, index) order, so both lanes build the same triple
        const float o1 = __shfl_xor(r1, 32, 64), o2 = __shfl_xor(r2, 32, 64),
                    o3 = __shfl_xor(r3, 32, 64);
        const int j1 = __shfl_xor(ii1, 32, 64), j2 = __shfl_xor(ii2, 32, 64),
                  j3 = __shfl_xor(ii3, 32, 64);
        auto lt = [](float a, int ia, float b, int ib) {
          return a < b || (a == b && ia < ib);
        };
        auto ins3 = [&](float p, int pi) {
          const bool c1 = lt(p, pi, r1, ii1), c2 = lt(p, pi, r2, ii2),
                     c3 = lt(p, pi, r3, ii3);
          r3 = c2 ? r2 : (c3 ? p : r3);
          ii3 = c2 ? ii2 : (c3 ? pi : ii3);
          r2 = c1 ? r1 : (c2 ? p : r2);
          ii2 = c1 ? ii1 : (c2 ? pi : ii2);
          r1 = c1 ? p : r1;
          ii1 = c1 ? pi : ii1;
        };
        ins3(o1, j1);
        ins3(o2, j2);
        ins3(o3, j3);
      }
      const bool sane = sane0 & (r1 < 1e30f);
      unique = sane & (r2 - r1 > B2);
      two = sane & !unique & (r3 - r1 > B2);
      i1 = ii1;
      i2 = ii2;
    }
    const bool valid = si < n && h == 0;
    const int prev = delta ? prv : -1;
    // 3..6 candidates of the threshold pass -> the N-candidate list
    bool nlisted = false;
    {
      const uint64_t mn = __ballot(valid && many);
      const int addn = __popcll(mn);
      if (addn && listing && nl_cnt + addn <= B1_NCAP) {
        if (valid && many)
          nl[nl_cnt + lane_prefix(mn)] =
              make_int4((int)(si - base), (int)mpk0, (int)mpk1, (int)mpk2);
        nl_cnt += addn;
        nlisted = many;
      }
    }
    // two candidates -> candidate list, more -> re-check list
    const uint64_t mc = __ballot(valid && two);
    const uint64_t mt = __ballot(valid && !unique && !two && !nlisted);
    const int addc = __popcll(mc), addt = __popcll(mt);
    bool spill = false;  // list full: the label scan finds the sample
    if (listing && cl_cnt + addc <= B1_CAP) {
      if (valid && two)
        cl[cl_cnt + lane_prefix(mc)] =
            make_int2((int)(si - base), i1 | (i2 << 16));
      cl_cnt += addc;
    } else {
      spill = valid && two;
      tl_over += addc;
    }
    if (listing && tl_cnt + addt <= TL_CAP) {
      if (valid && !unique && !two && !nlisted)
        wl[tl_cnt + lane_prefix(mt)] = make_int2((int)(si - base), prev);
      tl_cnt += addt;
    } else {
      spill |= valid && !unique && !two && !nlisted;
      tl_over += addt;
    }
    (void)spill;
    // a label equal to the incoming one (the hint) needs no store; an
    // N-listed sample keeps it until k_candn writes the winner
    if (valid && !nlisted && !(unique && i1 == (hint ? prv : prev)))
      lab_out[si] = unique ? i1 : -(prev + 2);
  }
  if (lane == 0 && listing) {
    v.tcount[wv] = tl_cnt;
    v.ccount[wv] = cl_cnt;
    v.ncount[wv] = nl_cnt;
  }
  if (lane == 0 && t_tiles) {  // diagnostics (dkm_screen_counters)
    atomicAdd((unsigned long long *)&v.hdr->reserved[0],
              (unsigned long long)t_tiles);
    atomicAdd((unsigned long long *)&v.hdr->reserved[1],
              (unsigned long long)t_done);
  }

  if (lane == 0 && tl_over) atomicAdd(&v.hdr->qcount, (uint32_t)tl_over);
}

// One 8-lane share of numpy's pairwise leaf: r_j = sum_i (x[j+8i]-c[j+8i])^2
// for i < nst (nst <= 16).  Every load is issued before the first use, so an
// entry costs one memory round trip instead of nst dependent ones.
template <class TX>
__device__ __forceinline__ void leaf8_load_x(const TX *xr, int nst,
                                             double (&xv)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < nst) xv[i] = (double)xr[8 * i];
}

__device__ __forceinline__ double leaf8_share(const double (&xv)[16],
                                              const double *cr, int nst) {
  double cv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < nst) cv[i] = cr[8 * i];
  double r = 0.0;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < nst) {
      const double df = xv[i] - cv[i];
      r = i ? r + df * df : df * df;
    }
  return r;
}

// 3..6-candidate samples of k_screen_b1's threshold pass: the reference
// arithmetic on exactly those centres (every other centre is strictly
// farther), best by (distance, index).  8 lanes per distance in numpy's
// leaf order as k_cand2 (d % 8 == 0, d <= 128); 8 entries per wave pass.
template <class TX>
__global__ void __launch_bounds__(BLOCK)
    k_candn(const TX *__restrict__ X, int d, int64_t ldx,
            const double *__restrict__ C, WsView v,
            int32_t *__restrict__ lab_out, int64_t base, int nseg) {
  const int64_t wv = (int64_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
  const int64_t nwv = (int64_t)gridDim.x * (BLOCK / 64);
  const int lane = threadIdx.x & 63;
  const int e = lane >> 3, j = lane & 7;
  const int nst = d >> 3;
  unsigned long long mine = 0;
  for (int64_t L = wv; L < (int64_t)nseg * (B1_NCAP / 64); L += nwv) {
    const int64_t sg = L % nseg;
    const int t0 = (int)(L / nseg) * 64;
    const int cnt = v.ncount[sg];
    if (t0 == 0 && lane == 0) mine += cnt;
    if (t0 >= cnt) continue;  // wave-uniform
    const int4 *list = v.nlist + sg * B1_NCAP + t0;
    const int m = min(64, cnt - t0);
    const int4 own = list[min(lane, m - 1)];  // the batch, one entry a lane
    for (int q = 0; q < m; q += 8) {
      const bool live = q + e < m;
      const int src = min(q + e, m - 1);
      const int4 it = make_int4(__shfl(own.x, src, 64), __shfl(own.y, src, 64),
                                __shfl(own.z, src, 64), __shfl(own.w, src, 64));
      const int64_t si = base + it.x;
      const TX *xr = X + si * ldx + j;
      const uint32_t pk[3] = {(uint32_t)it.y, (uint32_t)it.z, (uint32_t)it.w};
      double xv[16];
      leaf8_load_x(xr, nst, xv);
      double best = INFINITY;
      int bi = -1;
      for (int w = 0; w < 6; ++w) {
        const int c = (int)((pk[w >> 1] >> (16 * (w & 1))) & 0xffffu);
        if (c == 0xffff) break;
        double r = leaf8_share(xv, C + (int64_t)c * d + j, nst);
        r = r + __shfl_xor(r, 1, 64);
        r = r + __shfl_xor(r, 2, 64);
        r = r + __shfl_xor(r, 4, 64);
        const double dc = argmin_key(sqrt(r));
        if (dc < best || (dc == best && c < bi) || bi < 0) {
          best = dc;
          bi = c;
        }
      }
      if (live && j == 0) lab_out[si] = bi;
    }
  }
  if (mine) atomicAdd((unsigned long long *)&v.hdr->rechecked_total, mine);
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

// resolve_lane's two stages for ONE sample i with the whole wave: lanes
// over centres (jc = lane, lane + 64, ...), the same fp32 scores and bound
// (stage 1), then the reference arithmetic on the centres within the bound
// (stage 2; every centre when the scores are not sane), reduced over the
// wave by (distance, index).  The re-check list's stage-2 samples go here:
// lane per sample, a sample with many candidates (a near-tie among many
// centres) held its whole wave for k sequential exact distances.
template <int MAXD, class TX>
__device__ __forceinline__ void resolve_wave(
    const TX *__restrict__ X, int64_t ldx, int d, int k, int64_t i, int prev,
    const float *cl, const float *cnl, int dp, float cm, const double *ct64,
    int32_t *lab_out, int amode, const AccTarget &at) {
  const int lane = threadIdx.x & 63;
  const TX *xr = X + i * ldx;
  float xf[MAXD];
  float xx = 0.f;
#pragma unroll
  for (int t = 0; t < MAXD; ++t) {      // the same fp32 chain as resolve_lane
    xf[t] = t < d ? (float)ld_x(xr + t) : 0.f;
    xx = fmaf(xf[t], xf[t], xx);
  }
  // the centre's fp32 row (dp floats, 16-B aligned) by 16-B loads, all
  // issued before the fma chain (the same chain order as resolve_lane)
  auto score = [&](int jc) {
    const f32x4 *cr = (const f32x4 *)(cl + (int64_t)jc * dp);
    f32x4 c4[MAXD / 4];
#pragma unroll
    for (int t4 = 0; t4 < MAXD / 4; ++t4)
      if (4 * t4 < dp) c4[t4] = cr[t4];
    float dot = 0.f;
#pragma unroll
    for (int t4 = 0; t4 < MAXD / 4; ++t4)
      if (4 * t4 < dp) {
        dot = fmaf(xf[4 * t4 + 0], c4[t4].x, dot);
        dot = fmaf(xf[4 * t4 + 1], c4[t4].y, dot);
        dot = fmaf(xf[4 * t4 + 2], c4[t4].z, dot);
        dot = fmaf(xf[4 * t4 + 3], c4[t4].w, dot);
      }
    return fmaf(-2.f, dot, cnl[jc]);
  };
  float b1 = INFINITY, b2 = INFINITY;
  int i1 = INT32_MAX;
#pragma unroll 2
  for (int jc = lane; jc < k; jc += 64) {
    const float sc = score(jc);
    i1 = sc < b1 ? jc : i1;
    b2 = __builtin_amdgcn_fmed3f(b1, b2, sc);
    b1 = fminf(b1, sc);
  }
  // wave top-2 (NaN scores never win: fminf / med3 drop them, and the sane
  // test below sends such a sample to stage 2 over every centre)
  for (int off = 1; off < 64; off <<= 1) {
    const float o1 = __shfl_xor(b1, off, 64), o2 = __shfl_xor(b2, off, 64);
    const int oi = __shfl_xor(i1, off, 64);
    const bool tk = (o1 < b1) | ((o1 == b1) & (oi < i1));
    b2 = tk ? fminf(b1, o2) : fminf(b2, o1);
    i1 = tk ? oi : i1;
    b1 = tk ? o1 : b1;
  }
  const float xn = sqrtf(xx) * (1.0f + (d + 4) * 0x1.0p-24f);
  const float B = screen_bound<P_F32>(d, xn, cm, false);
  const bool sane = (xn < 1e18f) && (xn * cm < 1e30f) && (b1 < 1e30f);
  int bi = i1;
  if (!(sane && b2 - b1 > 2.0f * B)) {
    const float lim = b1 + 2.0f * B;
    double best = INFINITY;
    bi = INT32_MAX;
    for (int jc = lane; jc < k; jc += 64) {
      if (sane && !(score(jc) <= lim)) continue;
      const SqDiffT<TX> f{xr, ct64 + jc, ct_ld(k)};
      const double dist = argmin_key(sqrt(pw_leaf(f, 0, d)));
      if (dist < best || bi == INT32_MAX) {
        best = dist;
        bi = jc;
      }
    }
    for (int off = 1; off < 64; off <<= 1) {
      const double ob = __shfl_xor(best, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      const bool tk = (ob < best) | ((ob == best) & (oi < bi));
      best = tk ? ob : best;
      bi = tk ? oi : bi;
    }
  }
  if (lane == 0) lab_out[i] = bi;
  recheck_accumulate(amode, at, xr, d, bi, prev, lane);
}

constexpr int RL_CAP = 128;  // per-wave list: a full batch + one chunk

static size_t recheck_lane_lds(int64_t, int64_t) {
  return (size_t)(BLOCK / 64) * RL_CAP * 8;
}

template <int MAXD, bool VEC, class TX>
__global__ void __launch_bounds__(BLOCK)
    k_recheck_lane(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                   int k, WsView v, int32_t *__restrict__ lab_out,
                   double *acc, int amode, int64_t base) {
  if (v.hdr->qcount == 0) return;  // the screen resolved everything
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int dp = (int)round_up(d, 4);  // c32 row stride (dkm_util)
  // (fp32 centres: global, scalar loads in resolve_lane)
  int64_t *lists = (int64_t *)smem;
  double *lds_acc = (double *)(lists + (BLOCK / 64) * RL_CAP);
  __shared__ unsigned long long blk_count;
  if (threadIdx.x == 0) blk_count = 0;
  if (amode & AM_INLDS) zero_lds_acc(lds_acc, k, d);
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  const AccTarget at = acc_target(amode, lds_acc, acc, k, d);
  __syncthreads();

  const int lane = threadIdx.x & 63;
  int64_t *wl = lists + (threadIdx.x >> 6) * RL_CAP;

  auto resolve = [&](int64_t i) {
    resolve_lane<MAXD, VEC, TX>(X, ldx, d, k, i, -lab_out[i] - 2, v.c32,
                                v.cn32, dp,
                                cm, v.ct64, lab_out, amode, at);
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

#ifndef DKM_LIST_SPREAD
#define DKM_LIST_SPREAD 1
#endif
// The screen's per-wave lists (WsView::tlist/tcount, nseg segments): lane
// per listed sample (resolve_lane), fp32 centres in LDS.  No label scan:
// the work is proportional to the undecided samples only.
template <int MAXD, bool VEC, class TX>
__global__ void __launch_bounds__(BLOCK)
    k_recheck_list(const TX *__restrict__ X, int d, int64_t ldx, int k,
                   WsView v, int32_t *__restrict__ lab_out, double *acc,
                   int amode, int64_t base, int nseg, int wave_all) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int dp = (int)round_up(d, 4);
  // (fp32 centres: global, scalar loads in resolve_lane)
  double *lds_acc = (double *)smem;
  __shared__ unsigned long long blk_count;
  // per wave: samples stage 1 left undecided, resolved 64 at a time (a
  // lone stage-2 lane would otherwise hold its whole wave for a second pass)
  __shared__ int2 dlist[BLOCK / 64][128];
  if (threadIdx.x == 0) blk_count = 0;
  if (amode & AM_INLDS) zero_lds_acc(lds_acc, k, d);
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  const AccTarget at = acc_target(amode, lds_acc, acc, k, d);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wv = (int64_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
  const int64_t nwv = (int64_t)gridDim.x * (BLOCK / 64);
  unsigned long long mine = 0;
  int2 *dl = dlist[threadIdx.x >> 6];
  int dcnt = 0;  // wave-uniform
  auto stage2 = [&](int2 it) {
    resolve_lane<MAXD, VEC, TX>(X, ldx, d, k, base + it.x, it.y, v.c32,
                                v.cn32, dp,
                                cm, v.ct64, lab_out, amode, at);
  };
  // wave_all: the samples go to the global list that k_recheck_wave
  // resolves a wave per sample (v.smoved as (offset, prev) pairs; the
  // per-wave LDS list only takes what overflows it).  Otherwise stage 1 runs
  // here lane per sample and its leftovers are resolved 64 at a time (a long
  // list holds many of them: a wave per sample cost 0.7 ms per C2 iteration)
  int2 *s2l = (int2 *)v.smoved;
  const uint32_t s2cap = (uint32_t)std::min<int64_t>(v.nq / 2, INT32_MAX);
#if DKM_LIST_SPREAD
  // (segment, 64-sample batch) pairs dealt round-robin over all waves, batch
  // index major: every resident wave gets work and the segments' row loads
  // overlap across waves.  Wave-uniform loop; empty batches are skipped.
  for (int64_t L = wv; L < (int64_t)nseg * (TL_CAP / 64); L += nwv) {
    const int64_t sg = L % nseg;
    const int t0 = (int)(L / nseg) * 64;
    const int cnt = v.tcount[sg];
    if (t0 == 0) mine += cnt;
    if (t0 >= cnt) continue;
    const int2 *e = v.tlist + sg * TL_CAP;
    {
#else
  for (int64_t sg = wv; sg < nseg; sg += nwv) {
    const int cnt = v.tcount[sg];
    mine += cnt;
    const int2 *e = v.tlist + sg * TL_CAP;
    for (int t0 = 0; t0 < cnt; t0 += 64) {
#endif
      int2 it = make_int2(0, 0);
      bool ok = true;
      if (t0 + lane < cnt) {
        it = e[t0 + lane];
        // wave_all (short lists): every sample straight to k_recheck_wave
        ok = !wave_all &&
             resolve_lane<MAXD, VEC, TX, true>(X, ldx, d, k, base + it.x,
                                               it.y, v.c32, v.cn32, dp, cm,
                                               v.ct64, lab_out, amode, at);
      }
      unsigned long long m = __ballot(!ok);
      if (m && wave_all) {
        uint32_t pos = 0;
        if (lane == 0) pos = atomicAdd(&v.hdr->s2count, (uint32_t)__popcll(m));
        pos = (uint32_t)__shfl((int)pos, 0, 64);
        const uint32_t p = pos + (uint32_t)__popcll(m & ((1ull << lane) - 1));
        if (!ok && p < s2cap) s2l[p] = it;
        m = __ballot(!ok && p >= s2cap);   // the rest: this wave, stage 2
        ok = ok || p < s2cap;
      }
      if (!ok) dl[dcnt + __popcll(m & ((1ull << lane) - 1))] = it;
      dcnt += __popcll(m);
      if (dcnt >= 64) {
        wave_lds_sync();
        stage2(dl[lane]);
        const int rem = dcnt - 64;
        const int2 tail = lane < rem ? dl[64 + lane] : make_int2(0, 0);
        wave_lds_sync();
        if (lane < rem) dl[lane] = tail;
        dcnt = rem;
      }
    }
  }
  wave_lds_sync();
  if (lane < dcnt) stage2(dl[lane]);
  recheck_finish_count(mine, &blk_count, v);
  if (amode & AM_INLDS) flush_lds_acc(lds_acc, acc, k, d);
}

// k_recheck_list's stage-2 samples (fp32 stage 1 could not decide them),
// one wave per sample: lanes over centres (resolve_wave), so a sample with
// many candidates no longer holds a lane -- and its wave -- for a walk over
// every centre with one exact distance after another (the 1-4 ms spikes of
// the steady C3 iterations).  Sums by global fp64 atomics (rare samples).
template <int MAXD, class TX>
__global__ void __launch_bounds__(BLOCK)
    k_recheck_wave(const TX *__restrict__ X, int d, int64_t ldx, int k,
                   WsView v, int32_t *__restrict__ lab_out, double *acc,
                   int amode, int64_t base) {
  const uint32_t cap = (uint32_t)std::min<int64_t>(v.nq / 2, INT32_MAX);
  const uint32_t cnt = min(v.hdr->s2count, cap);
  const int64_t wv = (int64_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
  const int64_t nwv = (int64_t)gridDim.x * (BLOCK / 64);
  if (wv >= cnt) return;
  const int dp = (int)round_up(d, 4);
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  const int am = amode & ~AM_INLDS;
  const AccTarget at = acc_target(am, nullptr, acc, k, d);
  const int2 *s2l = (const int2 *)v.smoved;
  for (int64_t r = wv; r < cnt; r += nwv) {
    const int2 it = s2l[r];
    resolve_wave<MAXD, TX>(X, ldx, d, k, base + it.x, it.y, v.c32, v.cn32,
                           dp, cm, v.ct64, lab_out, am, at);
  }
}

template <bool SMALL, class TX>
__global__ void __launch_bounds__(BLOCK)
    k_recheck_exact(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                    int k, WsView v, int32_t *__restrict__ lab_out,
                    double *acc, int amode, int64_t base) {
  if (v.hdr->qcount == 0) return;  // the screen resolved everything
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
        const SqDiffT<TX> f{xr, v.ct64 + jc, ct_ld(k)};
        const double dist =
            argmin_key(sqrt(SMALL ? pw_leaf(f, 0, d) : pw_sum(f, d)));
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
                      int64_t n, int32_t *nz) {
  bool any = false;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const double v = x[e];
    y[e] += v;
    any |= v != 0.0;
  }
  // one store per wave that saw a nonzero (the flag was zeroed before)
  if (nz && __ballot(any) && (threadIdx.x & 63) == 0) nz[0] = 1;
}

// (hi, lo) += x, compensated: TwoSum of hi + x, the error into lo, then
// renormalised so that hi = fl(hi + lo) (the running sums the centre update
// reads) and |lo| <= ulp(hi) / 2.  Built with -ffp-contract=off: every
// operation rounds on its own, which TwoSum needs.
__global__ void k_add_dd(double *__restrict__ hi, double *__restrict__ lo,
                         const double *__restrict__ x, int64_t n, int32_t *nz) {
  bool any = false;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const double v = x[e];
    any |= v != 0.0;
    const double a = hi[e];
    const double s = a + v;
    const double bb = s - a;
    const double err = (a - (s - bb)) + (v - bb);
    const double t = lo[e] + err;
    const double h2 = s + t;
    lo[e] = t - (h2 - s);
    hi[e] = h2;
  }
  if (nz && __ballot(any) && (threadIdx.x & 63) == 0) nz[0] = 1;
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
  const int64_t cap =
      (int64_t)dev_info().cus * resident_blocks(kern, block, lds);
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

// Larger k x d runs the CHUNK screen (fragments staged through LDS).
static bool screen_ok(int64_t k, int64_t d) {
  return k >= 2 && k <= 32767 && d <= 128;
}

// 16-centre blocks resident in LDS per chunk (CHUNK screen), 0 = all fit
static int screen_chunk_blocks(int64_t k, int64_t d) {
  if (screen_lds_fixed(k, d) <= LDS_BUDGET) return 0;
  const int64_t per = (dpad32(d) / 32) * 2048 + 64;
  return (int)std::max<int64_t>(1, (int64_t)LDS_BUDGET / per);
}

template <int PREC, int NKS, int NB, bool VEC, class TX, bool CHUNK,
          bool T3P = false>
static int launch_screen_t(const TX *X, int64_t end, int d, int64_t ldx,
                           int k, const WsView &v, int32_t *lab_out,
                           double *acc, int amode, int64_t base, size_t lds,
                           int use_list, int chb, hipStream_t s, int *nseg) {
  const void *kf = (const void *)k_screen<PREC, NKS, NB, VEC, TX, CHUNK, T3P>;
  const int64_t cap = (int64_t)dev_info().cus * resident_blocks(kf, SB, lds);
  const int64_t per_block = 16 * NB * (SB / 64);
  const int64_t need = (end - base + per_block - 1) / per_block;
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min(need, cap));
  *nseg = (int)std::min<int64_t>((int64_t)g * (SB / 64), TL_SEGS);
  k_screen<PREC, NKS, NB, VEC, TX, CHUNK, T3P><<<g, SB, lds, s>>>(
      X, end, d, ldx, k, v, lab_out, acc, amode, base, use_list, chb);
  return check_launch("screen assignment");
}

// The rows an AM_MLIST screen moved (v.smoved, *cnt of them; new label in
// lab, previous in prevs[row]): +x to the new cluster, -x to the previous
// one, into block-private LDS sums flushed once per block.  Lanes over
// features (d <= 32: two rows per wave instruction), MV_U row pairs in
// flight per wave; the list order is free, so no sort (the sorted segment
// sums walked 4.7 M listed rows at 0.55 TB/s, 4.4 ms, at C2's iteration 2).
constexpr int MV_U = 8;
template <class TX>
__global__ void __launch_bounds__(256)
    k_moved_sums(const TX *__restrict__ X, int64_t ldx, int d,
                 const int32_t *__restrict__ list, const int32_t *cnt,
                 const int32_t *__restrict__ lab,
                 const int32_t *__restrict__ prevs, int k, double *acc) {
  extern __shared__ double lds_acc[];
  zero_lds_acc(lds_acc, k, d);
  __syncthreads();
  const int ds = lds_stride(d);
  const int lane = threadIdx.x & 63, g = lane >> 5, f = lane & 31;
  const int64_t m = *cnt;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  for (int64_t p0 = w * 2 * MV_U; p0 < m; p0 += nw * 2 * MV_U) {
    int64_t row[MV_U];
#pragma unroll
    for (int u = 0; u < MV_U; ++u) {
      const int64_t p = p0 + 2 * u + g;
      row[u] = p < m ? (int64_t)list[p] : -1;
    }
    int lb[MV_U], pv[MV_U];
    double x[MV_U];
#pragma unroll
    for (int u = 0; u < MV_U; ++u) {
      const bool ok = row[u] >= 0;
      lb[u] = ok ? lab[row[u]] : -1;
      pv[u] = ok ? prevs[row[u]] : -1;
      x[u] = ok && f < d ? (double)X[row[u] * ldx + f] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < MV_U; ++u) {
      if (lb[u] < 0) continue;
      if (f < d) {
        lds_add(lds_acc + (int64_t)lb[u] * ds + f, x[u]);
        if (pv[u] >= 0) lds_add(lds_acc + (int64_t)pv[u] * ds + f, -x[u]);
      }
      if (f == 0) {
        lds_add(lds_acc + (int64_t)k * ds + lb[u], 1.0);
        if (pv[u] >= 0) lds_add(lds_acc + (int64_t)k * ds + pv[u], -1.0);
      }
    }
  }
  __syncthreads();
  flush_lds_acc(lds_acc, acc, k, d);
}

template <class TX>
static int launch_moved_sums(const TX *X, int64_t ldx, int d, int k,
                             const int32_t *lab, double *acc, const WsView &v,
                             hipStream_t s) {
  const size_t lds = (size_t)lds_acc_len(k, d) * 8;
  if (d > 32 || lds > 64 * 1024) return 1;
  k_moved_sums<TX><<<(unsigned)dev_info().cus, 256, lds, s>>>(
      X, ldx, d, v.smoved, &v.hdr->nmoved, lab, v.queue, k, acc);
  return check_launch("moved-row sums");
}

template <class TX>
static int launch_screen_w32(const TX *X, int64_t end, int d, int64_t ldx,
                             int k, const WsView &v, int32_t *lab_out,
                             double *acc, int amode, int64_t base, size_t lds,
                             int use_list, hipStream_t s, int *nseg,
                             XImage img, bool build = false) {
  // the image serves launches that need no sums from the raw rows; a build
  // launch (full sums, base 0) writes it instead
  const bool im = !build && img.tiles && img.kind == IMG_SPLIT &&
                  !am_full(amode) && base % 32 == 0;
  // the waves' transpose scratch: the X-converting launches only (three
  // blocks per CU need <= 53 KB each)
  if (!im) lds += (size_t)(SBW / 64) * W32_SCR;
  // the threshold pass: image delta launches (incoming labels = hints)
  const size_t pcn_bytes = (size_t)kpad32(k) * 16 * 4;
  const bool hint = im && (amode & AM_DELTA) && k <= W32_HINT_KMAX &&
                    lds + pcn_bytes <= LDS_BUDGET;
  if (hint) lds += pcn_bytes;
  // AM_MLIST: the moved-row staging after them (the kernel's layout)
  if (amode & AM_MLIST) {
    if (!(im && hint)) return 1;  // the image threshold pass only
    lds += (size_t)(SBW / 64) * W32_MLB * 4;
  }
  const void *kf = hint ? (const void *)k_screen_w32<TX, true, true>
                   : im ? (const void *)k_screen_w32<TX, true>
                        : (const void *)k_screen_w32<TX, false>;
  const int64_t cap = (int64_t)dev_info().cus * resident_blocks(kf, SBW, lds);
  const int64_t per_block = 32 * (SBW / 64);
  const int64_t need = (end - base + per_block - 1) / per_block;
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min(need, cap));
  *nseg = (int)std::min<int64_t>((int64_t)g * (SBW / 64), TL_SEGS);
  if (hint)
    k_screen_w32<TX, true, true><<<g, SBW, lds, s>>>(
        X, end, d, ldx, k, v, lab_out, acc, amode, base, use_list, img, 0);
  else if (im)
    k_screen_w32<TX, true><<<g, SBW, lds, s>>>(X, end, d, ldx, k, v, lab_out,
                                               acc, amode, base, use_list, img,
                                               0);
  else
    k_screen_w32<TX, false><<<g, SBW, lds, s>>>(
        X, end, d, ldx, k, v, lab_out, acc, amode, base, use_list,
        build ? img : XImage{nullptr, nullptr, IMG_NONE}, build ? 1 : 0);
  return check_launch("screen assignment (32x32)");
}

template <int PREC, bool VEC, class TX>
static int launch_screen_nks(const TX *X, int64_t end, int d, int64_t ldx,
                             int k, const WsView &v, int32_t *lab_out,
                             double *acc, int amode, int64_t base, size_t lds,
                             int use_list, int chb, hipStream_t s,
                             int *nseg) {
#define DKM_SCREEN_CASE(NKS, NB)                                             \
  case NKS:                                                                  \
    return chb ? ((use_list & 2)                                             \
                      ? launch_screen_t<PREC, NKS, DKM_NB_CHUNK, VEC, TX,    \
                                        true, true>(                         \
                            X, end, d, ldx, k, v, lab_out, acc, amode, base, \
                            lds, use_list, chb, s, nseg)                     \
                      : launch_screen_t<PREC, NKS, DKM_NB_CHUNK, VEC, TX,    \
                                        true>(                               \
                            X, end, d, ldx, k, v, lab_out, acc, amode, base, \
                            lds, use_list, chb, s, nseg))                    \
               : launch_screen_t<PREC, NKS, NB, VEC, TX, false>(             \
                     X, end, d, ldx, k, v, lab_out, acc, amode, base, lds,   \
                     use_list, chb, s, nseg);
  switch (dpad32(d) / 32) {
    DKM_SCREEN_CASE(1, DKM_NB1)
    DKM_SCREEN_CASE(2, 1)
    DKM_SCREEN_CASE(3, 1)
    DKM_SCREEN_CASE(4, 1)
  }
#undef DKM_SCREEN_CASE
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
  const int per_cu = resident_blocks(kf, BLOCK, lds);
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

template <int MAXD, bool VEC, class TX>
static int launch_list_t(const TX *X, int d, int64_t ldx, int k,
                         const WsView &v, int32_t *lab_out, double *acc,
                         int amode, int64_t base, int nseg, size_t lds,
                         hipStream_t s, bool wave_all) {
  const void *kf = (const void *)k_recheck_list<MAXD, VEC, TX>;
  const int per_cu = resident_blocks(kf, BLOCK, lds);
  const int64_t units = DKM_LIST_SPREAD ? (int64_t)nseg * (TL_CAP / 64) : nseg;
  const int64_t g = std::max<int64_t>(
      1, std::min<int64_t>((int64_t)dev_info().cus * per_cu,
                           (units + BLOCK / 64 - 1) / (BLOCK / 64)));
  if (hipMemsetAsync(&v.hdr->s2count, 0, 4, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "list re-check: counter reset");
  k_recheck_list<MAXD, VEC, TX><<<(unsigned)g, BLOCK, lds, s>>>(
      X, d, ldx, k, v, lab_out, acc, amode, base, nseg, wave_all ? 1 : 0);
  if (int r = check_launch("list re-check")) return r;
  if (!wave_all) return 0;
  k_recheck_wave<MAXD, TX><<<(unsigned)(dev_info().cus * 4), BLOCK, 0, s>>>(
      X, d, ldx, k, v, lab_out, acc, amode, base);
  return check_launch("list re-check (wave per sample)");
}

// Can the listed samples be resolved lane-per-sample (k_recheck_list)?
static bool list_ok(int64_t k, int64_t d) {
  return d <= 128 && recheck_lane_lds(k, d) <= LDS_BUDGET;
}

// wave_all: the list is short (a re-screen's leftovers): every sample goes
// to k_recheck_wave (a wave per sample, its latency spread over the chip)
// instead of lane-per-sample stage 1, whose per-wave walk over all k centres
// costs ~1 ms whatever the list's length.
template <class TX>
static int launch_list(const TX *X, int d, int64_t ldx, int k,
                       const WsView &v, int32_t *lab_out, double *acc,
                       int acc_kind, bool vec, int64_t base, int nseg,
                       hipStream_t s, bool wave_all = false) {
  const size_t fb = 0;  // centres are read from global (scalar loads)
  const size_t a_bytes = (size_t)lds_acc_len(k, d) * 8;
  const int amode = acc_mode(acc_kind, fb + a_bytes <= LDS_BUDGET);
  const size_t lds = fb + ((amode & AM_INLDS) ? a_bytes : 0);
  const int maxd = d <= 32 ? 32 : d <= 64 ? 64 : 128;
#define DKM_LL(M)                                                            \
  (vec ? launch_list_t<M, true, TX>(X, d, ldx, k, v, lab_out, acc, amode,    \
                                    base, nseg, lds, s, wave_all)            \
       : launch_list_t<M, false, TX>(X, d, ldx, k, v, lab_out, acc, amode,   \
                                     base, nseg, lds, s, wave_all))
  const int r = maxd == 32 ? DKM_LL(32) : maxd == 64 ? DKM_LL(64) : DKM_LL(128);
#undef DKM_LL
  return r;
}


// ---------------------------------------------------------------------------
// Label-partitioned sums (k x d sums too large for block-private LDS, e.g.
// k = 1000, d = 64: 512 KB).  Instead of d fp64 global atomics per sample
// (8e9 of them at 125M x 64: ~0.5 s), block (x, y) owns the clusters
// [y*kr, y*kr + kr) -- their sums fit in LDS -- and the sample range of its
// waves; every row is read (coalesced, lanes over features) only by the
// blocks whose cluster range holds its label, so X is read once in all.
// Labels are read gridDim.y times (4 B each).  Delta (prev != null): only
// samples whose label changed, +x to the new cluster and -x from the old.
// The block's LDS sums are flushed once with fp64 atomics.
// ---------------------------------------------------------------------------
template <class TX>
__global__ void __launch_bounds__(BLOCK)
    k_label_sums(const TX *__restrict__ X, int64_t lo, int64_t hi, int d,
                 int64_t ldx, const int32_t *__restrict__ lab,
                 const int32_t *__restrict__ prev, int k, int kr,
                 double *acc) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int c0 = blockIdx.y * kr, c1 = min(k, c0 + kr), nc = c1 - c0;
  const int ds = lds_stride(d);
  double *rows = smem;
  double *cnt = smem + (int64_t)nc * ds;
  for (int64_t e = threadIdx.x; e < (int64_t)nc * ds + nc; e += BLOCK)
    smem[e] = 0.0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wv = (int64_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
  const int64_t nwv = (int64_t)gridDim.x * (BLOCK / 64);
  for (int64_t i0 = lo + wv * 64; i0 < hi; i0 += nwv * 64) {
    const int64_t i = i0 + lane;
    int a = -1, p = -1;
    if (i < hi) {
      a = lab[i];
      if (prev) {
        p = prev[i];
        if (p == a) a = p = -1;
      }
    }
    const bool ina = a >= c0 && a < c1, inp = p >= c0 && p < c1;
    uint64_t m = __ballot(ina || inp);
    while (m) {  // wave-uniform: 4 rows per pass, loads issued together
      int bl[4], ua[4], up[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        bl[u] = m ? __builtin_ctzll(m) : -1;
        if (m) m &= m - 1;
        ua[u] = bl[u] >= 0 ? __builtin_amdgcn_readlane(a, bl[u]) : -1;
        up[u] = bl[u] >= 0 ? __builtin_amdgcn_readlane(p, bl[u]) : -1;
      }
      for (int t = lane; t < d; t += 64) {
        double x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          x[u] = bl[u] >= 0 ? ld_x(X + (i0 + bl[u]) * ldx + t) : 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (ua[u] >= c0 && ua[u] < c1)
            lds_add(rows + (int64_t)(ua[u] - c0) * ds + t, x[u]);
          if (up[u] >= c0 && up[u] < c1)
            lds_add(rows + (int64_t)(up[u] - c0) * ds + t, -x[u]);
        }
      }
      if (lane == 0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (ua[u] >= c0 && ua[u] < c1) lds_add(cnt + (ua[u] - c0), 1.0);
          if (up[u] >= c0 && up[u] < c1) lds_add(cnt + (up[u] - c0), -1.0);
        }
      }
    }
  }
  __syncthreads();
  const int64_t nd = (int64_t)nc * d;
  for (int64_t e = threadIdx.x; e < nd + nc; e += BLOCK) {
    const double v = e < nd ? rows[(e / d) * ds + (e % d)] : cnt[e - nd];
    if (v != 0.0)
      atomic_add_f64(e < nd ? acc + (int64_t)c0 * d + e
                            : acc + (int64_t)k * d + c0 + (e - nd),
                     v);
  }
}

// Clusters per k_label_sums range: their LDS sums within LDS_BUDGET.
static int label_sums_kr(int64_t k, int d) {
  const int64_t per = ((int64_t)lds_stride(d) + 1) * 8;
  return (int)std::max<int64_t>(1, std::min<int64_t>(k, LDS_BUDGET / per));
}

template <class TX>
static int launch_label_sums(const TX *X, int64_t lo, int64_t hi, int d,
                             int64_t ldx, const int32_t *lab,
                             const int32_t *prev, int k, double *acc,
                             hipStream_t s) {
  if (hi <= lo) return 0;
  const int kr = label_sums_kr(k, d);
  const int ny = (k + kr - 1) / kr;
  const size_t lds = (size_t)(((int64_t)lds_stride(d) + 1) * kr) * 8;
  const void *kf = (const void *)k_label_sums<TX>;
  const int64_t cap = (int64_t)dev_info().cus * resident_blocks(kf, BLOCK, lds);
  const int64_t waves = (hi - lo + 63) / 64;
  const int64_t gx = std::max<int64_t>(
      1, std::min<int64_t>((cap + ny - 1) / ny * 2,
                           (waves + BLOCK / 64 - 1) / (BLOCK / 64)));
  k_label_sums<TX><<<dim3((unsigned)gx, (unsigned)ny), BLOCK, lds, s>>>(
      X, lo, hi, d, ldx, lab, prev, k, kr, acc);
  return check_launch("label sums");
}

// Sums from finished labels: the counting sort + segmented sums of
// dkm_sums.hip when its scratch holds the range (k <= SORT_KMAX), else
// k_label_sums.  AB_LABEL_SUMS (A/B builds) forces k_label_sums.
template <class TX>
static int launch_post_sums(const TX *X, int64_t lo, int64_t hi, int d,
                            int64_t ldx, const int32_t *lab,
                            const int32_t *prev, int k, double *acc,
                            const WsView &v, hipStream_t s) {
  if (!AB_LABEL_SUMS && sorted_sums_ok(k, hi - lo, v))
    return sorted_sums<TX>(X, lo, hi, d, ldx, lab, prev, k, acc, v, s);
  return launch_label_sums<TX>(X, lo, hi, d, ldx, lab, prev, k, acc, s);
}

// Do the [sums | counts] of k x d fit block-private LDS beside the screen's
// fragments (else the screens write labels and k_label_sums sums)?
static bool sums_fit_lds(int64_t k, int64_t d) {
  const size_t a = (size_t)lds_acc_len(k, (int)d) * 8;
  const size_t f = d <= 32 ? (size_t)(kpad32(k) / 32) * (4096 + 128)
                           : screen_lds_fixed(k, d);
  return f + a <= LDS_BUDGET;
}

template <class TX>
static int launch_screen_b1(const TX *X, int64_t end, int d, int64_t ldx,
                            int k, const WsView &v, int32_t *lab_out,
                            int64_t base, int hint, hipStream_t s, int *nseg) {
  size_t lds = b1_frag_bytes(k, d);
  // hint 2: the poisoned norm table (kpad32 x 16 B) fits beside the centres
  if (hint && lds + (size_t)kpad32(k) * 16 <= B1_LDS_POISON_MAX) {
    lds += (size_t)kpad32(k) * 16;
    hint = 2;
  }
  const int nks = (int)(dpad16(d) / 16);
  const void *kf = nullptr;
#define DKM_B1(N)                                            \
  case N:                                                    \
    kf = (const void *)k_screen_b1<TX, N>;                   \
    break;
  switch (nks) {
    DKM_B1(1) DKM_B1(2) DKM_B1(3) DKM_B1(4)
    DKM_B1(5) DKM_B1(6) DKM_B1(7) DKM_B1(8)
    default:
      return fail(DKM_E_ARG, "screen_b1: d too large");
  }
#undef DKM_B1
  if (hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return fail(DKM_E_LAUNCH, "screen_b1: LDS attribute");
  const int64_t need = (end - base + 32 * (SBB / 64) - 1) / (32 * (SBB / 64));
  const unsigned g = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>(need, (int64_t)dev_info().cus));
  *nseg = (int)std::min<int64_t>((int64_t)g * (SBB / 64),
                                 std::min(TL_SEGS, B1_SEGS));
  const int delta = 0;  // labels only (amode none): no previous label
  switch (nks) {
#define DKM_B1L(N)                                                          \
  case N:                                                                   \
    k_screen_b1<TX, N><<<g, SBB, lds, s>>>(X, end, d, ldx, k, v, lab_out,   \
                                           base, delta, hint);              \
    break;
    DKM_B1L(1) DKM_B1L(2) DKM_B1L(3) DKM_B1L(4)
    DKM_B1L(5) DKM_B1L(6) DKM_B1L(7) DKM_B1L(8)
#undef DKM_B1L
  }
  return check_launch("screen assignment (single product)");
}

template <class TX>
static int launch_cand2(const TX *X, int d, int64_t ldx, const double *C,
                        const WsView &v, int32_t *lab_out, int64_t base,
                        int nseg, hipStream_t s) {
  // dkm_cand.hip (the screens list two-candidate samples only for
  // d % 8 == 0, d <= 128)
  const int r = launch_cand2_leaf<TX>(X, d, ldx, C, v, lab_out, base, nseg,
                                      dev_info().cus, s);
  return r == 1 ? fail(DKM_E_ARG, "two-candidate re-check: d % 8 != 0") : r;
}

template <class TX>
static int launch_candn(const TX *X, int d, int64_t ldx, const double *C,
                        const WsView &v, int32_t *lab_out, int64_t base,
                        int nseg, hipStream_t s) {
  const int64_t units = (int64_t)nseg * (B1_NCAP / 64);
  const int64_t g = std::max<int64_t>(
      1, std::min<int64_t>((int64_t)dev_info().cus * 8,
                           (units + BLOCK / 64 - 1) / (BLOCK / 64)));
  k_candn<TX><<<(unsigned)g, BLOCK, 0, s>>>(X, d, ldx, C, v, lab_out, base,
                                            nseg);
  return check_launch("N-candidate re-check");
}

// ---- the re-screen of a screen's re-check list ---------------------------
// Per-segment offsets of the list (exclusive prefix of tcount) and its total
// (one block, nseg <= TL_SEGS).
__global__ void __launch_bounds__(1024)
    k_list_scan(const int32_t *__restrict__ tcount, int nseg,
                int32_t *__restrict__ prefix, uint32_t *total) {
  __shared__ int32_t part[1024];
  const int t = threadIdx.x;
  const int per = (nseg + 1023) / 1024;
  const int a = min(nseg, t * per), b = min(nseg, a + per);
  int sum = 0;
  for (int i = a; i < b; ++i) sum += min(max(tcount[i], 0), TL_CAP);
  part[t] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - sum;
  for (int i = a; i < b; ++i) {
    prefix[i] = run;
    run += min(max(tcount[i], 0), TL_CAP);
  }
  if (t == 1023) *total = (uint32_t)part[1023];
}

// The list compacted: a wave per segment.
__global__ void __launch_bounds__(256)
    k_list_compact(const int2 *__restrict__ tlist,
                   const int32_t *__restrict__ tcount,
                   const int32_t *__restrict__ prefix, int nseg,
                   int2 *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  for (int64_t sg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); sg < nseg;
       sg += (int64_t)gridDim.x * 4) {
    const int cnt = min(max(tcount[sg], 0), TL_CAP);
    const int2 *src = tlist + sg * TL_CAP;
    int2 *dst = out + prefix[sg];
    for (int i = lane; i < cnt; i += 64) dst[i] = src[i];
  }
}

// rows base + list[r].x of X -> out (m x d, packed)
template <class TX>
__global__ void __launch_bounds__(256)
    k_gather_rows(const TX *__restrict__ X, int64_t ldx, int d,
                  const int2 *__restrict__ list, int m, int64_t base,
                  TX *__restrict__ out) {
  const int64_t tot = (int64_t)m * d;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / d;
    const int t = (int)(e - r * d);
    out[e] = X[(base + list[r].x) * ldx + t];
  }
}

__global__ void __launch_bounds__(256)
    k_scatter_labels(const int32_t *__restrict__ lab,
                     const int2 *__restrict__ list, int m,
                     int32_t *__restrict__ lab_out) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < m;
       r += (int64_t)gridDim.x * 256)
    lab_out[list[r].x] = lab[r];
}

template <class TX>
static int launch_screen(int prec, const TX *X, int64_t n, int d,
                         int64_t ldx, const double *C, int k, const WsView &v,
                         size_t wsb, int32_t *labels, double *acc,
                         int acc_kind, hipStream_t s, XImage img,
                         bool nohint = false, bool force_b1 = false,
                         void *build_img = nullptr, bool sub = false,
                         bool transl = false);

// The samples a screen left to the exact re-check (its per-wave lists) are
// gathered, RS_ROWS at a time, and screened again by the chunked bf16x3
// screen with the two-candidate list (k_screen T3 + k_cand2), the list's
// leftovers by its own re-check; their labels are scattered back.  A single-
// product screen's list (~2^-8 bound) mostly resolves to one or two
// candidates under bf16x3 (~2^-16), so those samples skip the re-check's
// fp32 scan of all k centres (lane per sample, latency-bound: 6-7 ms for
// C3 iteration 1's 1.15M listed rows, 1-4 ms spikes for a few hundred rows
// in steady iterations); the bf16x3 screen's own list (C3 iteration 0,
// ~2 % of the rows against the initial centres) gains the two-candidate
// path, at the top-3 cost on those rows only.  One 4-byte device -> host
// read per call (the list's length sizes the gathered chunks).
template <class TX>
static int rescreen_list(const TX *X, int d, int64_t ldx, const double *C,
                         int k, const WsView &v, size_t wsb, int32_t *lab_out,
                         int64_t base, int nseg, hipStream_t s) {
  nseg = std::min(nseg, TL_SEGS);
  if (nseg <= 0) return 0;
  k_list_scan<<<1, 1024, 0, s>>>(v.tcount, nseg, v.rprefix, &v.hdr->rtotal);
  if (int r = check_launch("re-screen: list scan")) return r;
  // the length through pinned host memory (a pageable read stalled the
  // stream for ~3 ms once per process in the C3 trace)
  static thread_local uint32_t *pinned = nullptr;
  if (!pinned && hipHostMalloc((void **)&pinned, 64, hipHostMallocDefault) !=
                     hipSuccess)
    return fail(DKM_E_LAUNCH, "re-screen: pinned buffer");
  if (hipMemcpyAsync(pinned, &v.hdr->rtotal, 4, hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "re-screen: list length");
  const uint32_t tot = *pinned;
  if (tot == 0) return 0;
  const int cus = dev_info().cus;
  k_list_compact<<<(unsigned)std::min<int64_t>((nseg + 3) / 4, cus * 8), 256,
                   0, s>>>(v.tlist, v.tcount, v.rprefix, nseg, v.rlist);
  if (int r = check_launch("re-screen: compact")) return r;
  for (int64_t c0 = 0; c0 < (int64_t)tot; c0 += RS_ROWS) {
    const int m = (int)std::min<int64_t>(RS_ROWS, (int64_t)tot - c0);
    const unsigned g = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>(((int64_t)m * d + 255) / 256, (int64_t)cus * 16));
    k_gather_rows<TX><<<g, 256, 0, s>>>(X, ldx, d, v.rlist + c0, m, base,
                                        (TX *)v.rx);
    if (int r = check_launch("re-screen: gather")) return r;
    if (int r = launch_screen<TX>(P_B3, (const TX *)v.rx, m, d, d, C, k, v,
                                  wsb, v.rlab, nullptr, 0, s,
                                  XImage{nullptr, nullptr, IMG_NONE, nullptr,
                                         nullptr},
                                  false, false, nullptr, true))
      return r;
    k_scatter_labels<<<(unsigned)std::max(1, std::min((m + 255) / 256,
                                                      cus * 8)),
                       256, 0, s>>>(v.rlab, v.rlist + c0, m, lab_out + base);
    if (int r = check_launch("re-screen: scatter")) return r;
  }
  // the screen's lists are done: the caller's list pass finds nothing
  if (hipMemsetAsync(v.tcount, 0, (size_t)TL_SEGS * 4, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "re-screen: list reset");
  return 0;
}

// Screen + exact re-check over [0, n).  Labels go to `labels` when given,
// else to the workspace scratch (queue region), in chunks of its capacity.
template <class TX>
static int launch_screen(int prec, const TX *X, int64_t n, int d,
                         int64_t ldx, const double *C, int k, const WsView &v,
                         size_t wsb, int32_t *labels, double *acc,
                         int acc_kind, hipStream_t s, XImage img,
                         bool nohint, bool force_b1, void *build_img,
                         bool sub, bool transl) {
  (void)wsb;
  const int64_t nq = std::min<int64_t>(v.nq, INT32_MAX);
  if (!labels && nq < 1)
    return fail(DKM_E_WORKSPACE, "screen: no label scratch");
  // DKM_MODE_TRANSLATE (a fit's first assignment against crowded initial
  // centres): many samples keep two or more candidates, so the call runs in
  // row chunks that keep the per-wave lists within their capacity
  const int64_t chunk =
      labels ? (transl ? std::min<int64_t>(n, TRANSL_CHUNK) : n) : nq;
  const bool vec = (d % 8 == 0) && (ldx % (16 / (int64_t)sizeof(TX)) == 0) &&
                   (((uintptr_t)X % 16) == 0);
  // single-product screen: labels only, so the sums must come from
  // k_label_sums (full sums, or delta against a copy of the old labels)
  const bool b1 = prec == P_B1 && v.b1frag && vec &&
                  (int64_t)32 * ldx * (int64_t)sizeof(TX) < (1ll << 31) &&
                  (acc_kind == 0 || acc_kind == 1 || (labels && nq >= n));
  if (prec == P_B1 && !b1) prec = P_B3;
  if (img.kind == IMG_SORTED && !b1)
    return fail(DKM_E_ARG, "screen: the sorted image needs the single-product "
                           "screen (16-B aligned rows)");
  // d <= 32 bf16x3 with the 32x32x16 fragments resident: k_screen_w32
  const size_t fb32 = (size_t)(kpad32(k) / 32) * (4096 + 128);
  const bool w32 = prec == P_B3 && d <= 32 && vec && fb32 <= LDS_BUDGET &&
                   (int64_t)32 * ldx * (int64_t)sizeof(TX) < (1ll << 31) &&
                   !AB_NO_W32;
  const int chb = w32 ? 0 : screen_chunk_blocks(k, d);
  const size_t fb = w32 ? fb32
                    : chb ? (size_t)chb * ((dpad32(d) / 32) * 2048 + 64)
                          : screen_lds_fixed(k, d);
  const size_t a_bytes = (size_t)lds_acc_len(k, d) * 8;
  // sums that do not fit block-private LDS: the screen writes labels only
  // and k_label_sums accumulates from them (delta: against a copy of the
  // previous labels in the label scratch)
  const bool lds_fits = fb + a_bytes <= LDS_BUDGET;
  // AB_DELTA_POST: delta sums from k_label_sums even when they fit LDS
  // (the screen then needs only the fragments' LDS: more blocks per CU)
  const bool force_post = acc_kind == 2 && AB_DELTA_POST;
  const bool post = acc_kind != 0 && (!lds_fits || force_post || b1) &&
                    !AB_NO_POST &&
                    (acc_kind == 1 || (labels && nq >= n));
  // the sorted image's incremental sums: the label sync lists the moved
  // rows with their previous labels (in the queue scratch), so neither a
  // copy of the labels nor a scan for changes is needed
  const bool premoved = post && acc_kind == 2 && b1 &&
                        img.kind == IMG_SORTED && chunk >= n &&
                        !AB_LABEL_SUMS && sorted_sums_ok(k, n, v);
  const int32_t *prevbuf = nullptr;
  if (post && acc_kind == 2 && !premoved) {
    if (hipMemcpyAsync(v.queue, labels, (size_t)n * 4,
                       hipMemcpyDeviceToDevice, s) != hipSuccess)
      return fail(DKM_E_LAUNCH, "screen: label copy");
    prevbuf = v.queue;
  }
  const int skind = post ? 0 : acc_kind;
  const int amode = acc_mode(skind, lds_fits);
  const size_t lds = fb + ((amode & AM_INLDS) ? a_bytes : 0);
  const int use_list = list_ok(k, d) && !AB_NO_LIST ? 1 : 0;
  // the chunked bf16x3 screen's two-candidate list (T3 in k_screen): labels-
  // only launches whose rows k_cand2 can take (d % 8 == 0, d <= 128)
  // (sub: this call is a re-screen's, on gathered rows)
  const bool c2 = sub && !b1 && !w32 && chb && prec == P_B3 &&
                  amode == AM_NONE && v.clist && vec && d % 8 == 0 &&
                  d >= 8 && d <= 128;
  // the re-screen of this call's re-check list: labels-only screens whose
  // gathered rows the chunked bf16x3 screen with its two-candidate list
  // takes (c2's conditions on the gathered, packed rows)
  const bool rescreen = !sub && v.rlist && amode == AM_NONE && use_list &&
                        screen_chunk_blocks(k, d) > 0 &&
                        (b1 || (prec == P_B3 && chb && !w32)) &&
                        d % 8 == 0 && d >= 8 && d <= 128;
  // DKM_IMAGE_BUILD: the split image written by this call's full-sums w32
  // pass over X (one launch from row 0), else built first
  bool fuse_build = false;
  if (build_img) {
    fuse_build = w32 && am_full(amode) && img.kind == IMG_SPLIT && chunk >= n;
    if (!fuse_build) {
      if (int r = launch_x_image<TX>(X, n, d, ldx, img.kind, build_img,
                                     dev_info().cus, s))
        return r;
    }
  }
  // the d <= 32 image threshold pass of a delta call: the rows it moves
  // are listed and summed by sorted_sums_moved after the re-checks (a
  // moved row's fp64 load and +-x adds inside the screen stalled its wave:
  // C2's iteration 2, 4.7 % of the rows moving, took 7.2 ms against 3.7)
  bool mlist = w32 && acc_kind == 2 && !post && labels && chunk >= n &&
               img.tiles && img.kind == IMG_SPLIT && !build_img &&
               (int64_t)n <= nq && sorted_sums_ok(k, n, v) && !AB_NO_MLIST;
  if (mlist && hipMemsetAsync(&v.hdr->nmoved, 0, 4, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "screen: memset");
  for (int64_t base = 0; base < n; base += chunk) {
    const int64_t end = std::min(n, base + chunk);
    int32_t *lab_out = labels ? labels : v.queue - base;
    int r, nseg = 0;
    if (b1) {
      // the incoming labels (previous iteration) seed the threshold pass
      // (NOHINT: the caller knows them to be poor, e.g. labels of the
      // initial centres -- the top-3 pass runs directly)
      const int hint = labels && acc_kind != 0 && !nohint ? 1 : 0;
      r = force_b1 ? 1
                   : launch_screen_b2<TX>(X, end, d, ldx, k, v, lab_out, base,
                                          hint, dev_info().cus, s, &nseg, img,
                                          transl);
      if (r == 1 && img.kind == IMG_SORTED)
        return fail(DKM_E_ARG, "screen: the sorted image needs k_screen_b2");
      if (r == 1)
        r = launch_screen_b1<TX>(X, end, d, ldx, k, v, lab_out, base, hint, s,
                                 &nseg);
      if (r) return r;
      r = launch_cand2<TX>(X, d, ldx, C, v, lab_out, base, nseg, s);
      if (!r && hint) r = launch_candn<TX>(X, d, ldx, C, v, lab_out, base,
                                           nseg, s);
    } else if (w32) {
      r = mlist ? launch_screen_w32<TX>(X, end, d, ldx, k, v, lab_out, acc,
                                        AM_DELTA | AM_MLIST, base, fb,
                                        use_list, s, &nseg, img)
                : 1;
      if (r == 1) {
        mlist = false;
        r = launch_screen_w32<TX>(X, end, d, ldx, k, v, lab_out, acc, amode,
                                  base, lds, use_list, s, &nseg, img,
                                  fuse_build);
      }
    }
    else if (prec == P_F32)
      r = vec ? launch_screen_nks<P_F32, true, TX>(X, end, d, ldx, k, v,
                                                   lab_out, acc, amode, base,
                                                   lds, use_list, chb, s, &nseg)
              : launch_screen_nks<P_F32, false, TX>(X, end, d, ldx, k, v,
                                                    lab_out, acc, amode, base,
                                                    lds, use_list, chb, s, &nseg);
    else {
      // the chunked labels-only bf16x3 screen in 32x32x16 form (32 < d <= 64)
      const bool c32 = chb && vec && amode == AM_NONE && !sub && d > 32 &&
                       d <= 64 && !AB_NO_C32;
      r = c32 ? launch_screen_c32<TX>(X, end, d, ldx, k, v, lab_out, base,
                                      use_list, s, &nseg)
              : 1;
      if (r == 1)
        r = vec ? launch_screen_nks<P_B3, true, TX>(
                      X, end, d, ldx, k, v, lab_out, acc, amode, base, lds,
                      use_list | (c2 ? 2 : 0), chb, s, &nseg)
                : launch_screen_nks<P_B3, false, TX>(X, end, d, ldx, k, v,
                                                     lab_out, acc, amode,
                                                     base, lds, use_list, chb,
                                                     s, &nseg);
    }
    if (r) return r;
    if (c2 && (r = launch_cand2<TX>(X, d, ldx, C, v, lab_out, base,
                                    std::min(nseg, B1_SEGS), s)))
      return r;
    if (rescreen && (r = rescreen_list<TX>(X, d, ldx, C, k, v, wsb, lab_out,
                                           base, nseg, s)))
      return r;
    if ((use_list || b1) && (r = launch_list<TX>(X, d, ldx, k, v, lab_out,
                                                  acc, skind, vec, base,
                                                  nseg, s, sub)))
      return r;
    if ((r = launch_recheck<TX>(X, end, d, ldx, k, v, lab_out, acc,
                                skind, vec, base, s)))
      return r;
    // the sorted image's label copy: the rows the re-checks decided (and,
    // premoved, the list of rows that moved)
    if (b1 && (r = launch_plab_sync(img, n, k, labels, dev_info().cus, s,
                                    premoved ? v.smoved : nullptr,
                                    premoved ? &v.hdr->nmoved : nullptr,
                                    premoved ? v.queue : nullptr)))
      return r;
    if (mlist) {
      r = launch_moved_sums<TX>(X, ldx, d, k, lab_out, acc, v, s);
      if (r == 1)
        r = sorted_sums_moved<TX>(X, n, d, ldx, lab_out, v.queue, k, acc, v,
                                  s);
      if (r) return r;
    } else if (premoved) {
      if ((r = sorted_sums_moved<TX>(X, n, d, ldx, lab_out, v.queue, k, acc,
                                     v, s)))
        return r;
    } else if (post && (r = launch_post_sums<TX>(X, base, end, d, ldx,
                                                 lab_out, prevbuf, k, acc, v,
                                                 s)))
      return r;
  }
  return 0;
}

// d > 128: the bf16x3 GEMM screen (dkm_gemm.hip), which also resolves the
// samples it leaves open with the reference arithmetic.  Sums come from k_label_sums (X is read once more,
// lanes over features) unless the previous labels cannot be kept for a
// delta pass (label scratch smaller than n): then the merge step adds the
// changed rows itself with fp64 atomics.
template <class TX>
static int launch_gemm(const TX *X, int64_t n, int d, int64_t ldx,
                       const double *C, int k, const WsView &v, size_t wsb,
                       int32_t *labels, double *acc, int acc_kind,
                       bool one, const XImage *img, hipStream_t s,
                       const XImage *bimg = nullptr) {
  (void)wsb;
  const int64_t nq = std::min<int64_t>(v.nq, INT32_MAX);
  if (!labels && nq < 1)
    return fail(DKM_E_WORKSPACE, "gemm: no label scratch");
  if (bimg && !labels)
    return fail(DKM_E_ARG, "gemm: image build needs the labels");
  const int64_t chunk = labels ? n : nq;
  const bool post =
      acc_kind != 0 && (acc_kind == 1 || (labels && nq >= n));
  const int32_t *prevbuf = nullptr;
  if (post && acc_kind == 2) {
    if (hipMemcpyAsync(v.queue, labels, (size_t)n * 4,
                       hipMemcpyDeviceToDevice, s) != hipSuccess)
      return fail(DKM_E_LAUNCH, "gemm: label copy");
    prevbuf = v.queue;
  }
  const int skind = post ? 0 : acc_kind;
  for (int64_t base = 0; base < n; base += chunk) {
    const int64_t end = std::min(n, base + chunk);
    int32_t *lab_out = labels ? labels : v.queue - base;
    int r = gemm_screen<TX>(X, base, end, d, ldx, C, k, v, lab_out,
                            skind ? acc : nullptr, skind == 2, one, img, s,
                            bimg);
    if (r) return r;
    if (post && (r = launch_post_sums<TX>(X, base, end, d, ldx, lab_out,
                                          prevbuf, k, acc, v, s)))
      return r;
  }
  return 0;
}

template <class TX>
static int x_image(const TX *X, int64_t n, int64_t d, int64_t ldx, int kind,
                   void *image, size_t image_bytes, void *stream,
                   const char *who);

template <class TX>
static int assign(const TX *X, int64_t n, int64_t d, int64_t ldx,
                  const double *C, int64_t k, const void *ws, size_t wsb,
                  int32_t *labels, double *acc, int acc_kind, int mode,
                  void *stream, const char *who, const void *image = nullptr,
                  int image_kind = 0) {
  if (n < 0 || d <= 0 || k <= 0 || ldx < d)
    return fail(DKM_E_ARG, std::string(who) + ": bad n/d/k/ldx");
  if (d > INT32_MAX || k > INT32_MAX)
    return fail(DKM_E_ARG, std::string(who) + ": d/k too large");
  if (n == 0) return 0;
  if (!X || !C) return fail(DKM_E_ARG, std::string(who) + ": NULL X/C");
  if (!labels && !acc)
    return fail(DKM_E_ARG, std::string(who) + ": nothing to write");
  hipStream_t s = (hipStream_t)stream;
  if (mode & ~(DKM_MODE_MASK | DKM_MODE_NOHINT | DKM_MODE_B1 |
               DKM_MODE_TRANSLATE))
    return fail(DKM_E_ARG, std::string(who) + ": unknown mode flags");
  // DKM_IMAGE_BUILD: build the (allocated, unbuilt) image during this call
  const bool build = image && (image_kind & DKM_IMAGE_BUILD);
  image_kind &= ~DKM_IMAGE_BUILD;
  if (build && image_kind == IMG_SORTED)
    return fail(DKM_E_ARG, std::string(who) +
                               ": the sorted image is built by "
                               "dkm_x_image_sorted_*");
  const bool nohint = mode & DKM_MODE_NOHINT, force_b1 = mode & DKM_MODE_B1;
  bool transl = mode & DKM_MODE_TRANSLATE;
  mode &= DKM_MODE_MASK;
  if (mode == DKM_MODE_AUTO)
    mode = !screen_ok(k, d) && !gemm_path(k, d) ? DKM_MODE_EXACT
           // the GEMM screen (d > 128) and sums beyond LDS with the bf16
           // centres resident: the single product
           : gemm_path(k, d) ||
                   (screen_ok(k, d) && b1_ok(k, d) &&
                    !sums_fit_lds(k, d))
               ? DKM_MODE_SCREEN_BF16
               : DKM_MODE_SCREEN_BF16X3;
  if (image && (image_kind < IMG_SINGLE || image_kind > IMG_GEMM ||
                (image_kind == IMG_GEMM) != gemm_path(k, d)))
    return fail(DKM_E_ARG, std::string(who) +
                               ": image kind does not fit (k, d)");
  // the sorted image keeps a copy of the labels that only k_screen_b2
  // maintains: any other arithmetic would leave it stale
  if (image && image_kind == IMG_SORTED &&
      (mode != DKM_MODE_SCREEN_BF16 || !screen_ok(k, d) || !labels || force_b1))
    return fail(DKM_E_ARG, std::string(who) +
                               ": the sorted image needs the single-product "
                               "screen (MODE_SCREEN_BF16 or AUTO) and labels");
  const bool split_w32 = image_kind == IMG_SPLIT && mode ==
      DKM_MODE_SCREEN_BF16X3 && screen_ok(k, d) && d <= 32;
  // the bf16x3 GEMM screen's chunk splits write the single-product image's
  // hi tiles as they convert X (the fit's first iteration; no image pass)
  const bool split_gemm = build && image_kind == IMG_GEMM && labels &&
      mode == DKM_MODE_SCREEN_BF16X3 && gemm_path(k, d) && !AB_NO_GEMM_BUILD;
  if (build && !split_w32 && !split_gemm) {
    // no screen writes this kind in its pass: build it first
    if (int r = x_image<TX>(X, n, d, ldx, image_kind, (void *)image,
                            x_image_bytes(n, d, image_kind), stream, who))
      return r;
  }
  if (mode == DKM_MODE_EXACT)
    return launch_exact<TX>(X, n, (int)d, ldx, C, (int)k, labels, acc,
                            acc_kind, s);
  if ((mode == DKM_MODE_SCREEN_BF16X3 || mode == DKM_MODE_SCREEN_BF16) &&
      gemm_path(k, d)) {
    WsView v;
    if (int r = ws_view(ws, wsb, k, d, &v)) return r;
    // the resident sample tiles serve the single-product screen only
    XImage gimg;
    const bool use_img = image && image_kind == IMG_GEMM &&
                         mode == DKM_MODE_SCREEN_BF16;
    if (use_img) gimg = x_image_view(image, n, d, IMG_GEMM);
    XImage bimg;
    if (split_gemm) bimg = x_image_view(image, n, d, IMG_GEMM);
    return launch_gemm<TX>(X, n, (int)d, ldx, C, (int)k, v, wsb, labels, acc,
                           acc_kind, mode == DKM_MODE_SCREEN_BF16,
                           use_img ? &gimg : nullptr, s,
                           split_gemm ? &bimg : nullptr);
  }
  if (mode == DKM_MODE_SCREEN32 || mode == DKM_MODE_SCREEN_BF16X3 ||
      mode == DKM_MODE_SCREEN_BF16) {
    if (!screen_ok(k, d))
      return launch_exact<TX>(X, n, (int)d, ldx, C, (int)k, labels, acc,
                              acc_kind, s);
    WsView v;
    if (int r = ws_view(ws, wsb, k, d, &v)) return r;
    const int prec = mode == DKM_MODE_SCREEN32 ? P_F32
                     : mode == DKM_MODE_SCREEN_BF16 ? P_B1
                                                    : P_B3;
    const XImage img = image ? x_image_view(image, n, d, image_kind)
                             : XImage{nullptr, nullptr, IMG_NONE, nullptr,
                                      nullptr};
    // the translated centres serve the single-product screen without the
    // sorted image (its block skipping reads absolute scores)
    if (image_kind == IMG_SORTED || prec != P_B1) transl = false;
    return launch_screen<TX>(prec, X, n, (int)d, ldx, C, (int)k, v, wsb,
                             labels, acc, acc_kind, s, img, nohint, force_b1,
                             build && split_w32 ? (void *)image : nullptr,
                             false, transl);
  }
  return fail(DKM_E_ARG, std::string(who) + ": bad mode");
}

template <class TX>
static int x_image(const TX *X, int64_t n, int64_t d, int64_t ldx, int kind,
                   void *image, size_t image_bytes, void *stream,
                   const char *who) {
  if (n < 0 || d <= 0 || ldx < d || d > INT32_MAX)
    return fail(DKM_E_ARG, std::string(who) + ": bad n/d/ldx");
  if (kind == IMG_GEMM ? d <= 128 : d > 128)
    return fail(DKM_E_ARG, std::string(who) +
                               ": the GEMM image needs d > 128, the others "
                               "d <= 128");
  if (n == 0) return 0;
  if (!X || !image) return fail(DKM_E_ARG, std::string(who) + ": NULL");
  if (kind != IMG_SINGLE && kind != IMG_SPLIT && kind != IMG_GEMM)
    return fail(DKM_E_ARG, std::string(who) + ": bad image kind");
  if (image_bytes < x_image_bytes(n, d, kind))
    return fail(DKM_E_WORKSPACE, std::string(who) + ": image too small");
  if (kind == IMG_GEMM)
    return gemm_image<TX>(X, n, (int)d, ldx, x_image_view(image, n, d, kind),
                          (hipStream_t)stream);
  return launch_x_image<TX>(X, n, (int)d, ldx, kind, image, dev_info().cus,
                            (hipStream_t)stream);
}

template <class TX>
static int x_image_sorted(const TX *X, int64_t n, int64_t d, int64_t ldx,
                          const int32_t *labels, int64_t k, const void *ws,
                          size_t wsb, void *image, size_t image_bytes,
                          double *acc, void *stream, const char *who) {
  const std::string w(who);
  if (n < 0 || d <= 0 || ldx < d || k <= 1 || k > INT32_MAX)
    return fail(DKM_E_ARG, w + ": bad n/d/k/ldx");
  if (n > INT32_MAX) return fail(DKM_E_ARG, w + ": n > 2^31 - 1");
  if (n == 0) return 0;
  if (!X || !labels || !image) return fail(DKM_E_ARG, w + ": NULL");
  if (!dkm_x_image_sorted_ok(k, d))
    return fail(DKM_E_ARG, w + ": (k, d) does not take the sorted image");
  if (image_bytes < x_image_bytes(n, d, IMG_SORTED))
    return fail(DKM_E_WORKSPACE, w + ": image too small");
  WsView v;
  if (int r = ws_view(ws, wsb, k, d, &v)) return r;
  if (!sorted_sums_ok(k, n, v))
    return fail(DKM_E_WORKSPACE, w + ": workspace label scratch < n");
  hipStream_t s = (hipStream_t)stream;
  const bool fused = acc && x_image_sums_fused(d);
  if (int r = launch_x_image_sorted<TX>(X, n, (int)d, ldx, labels, (int)k, v,
                                        image, dev_info().cus, s,
                                        fused ? acc : nullptr))
    return r;
  if (acc && !fused)
    return launch_post_sums<TX>(X, 0, n, (int)d, ldx, labels, nullptr,
                                (int)k, acc, v, s);
  return 0;
}

template <class TX>
static int label_sums_abi(const TX *X, int64_t n, int64_t d, int64_t ldx,
                          const int32_t *labels, int64_t k, const void *ws,
                          size_t wsb, double *acc, void *stream) {
  if (n < 0 || d <= 0 || k <= 0 || ldx < d || d > INT32_MAX || k > INT32_MAX)
    return fail(DKM_E_ARG, "label_sums: bad n/d/k/ldx");
  if (n == 0) return 0;
  if (!X || !labels || !acc) return fail(DKM_E_ARG, "label_sums: NULL");
  WsView v;
  if (int r = ws_view(ws, wsb, k, d, &v)) return r;
  return launch_post_sums<TX>(X, 0, n, (int)d, ldx, labels, nullptr, (int)k,
                              acc, v, (hipStream_t)stream);
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

int dkm_x_image_kind(int64_t k, int64_t d, int mode) {
  if (k <= 0 || d <= 0 || k > INT32_MAX || d > INT32_MAX) return IMG_NONE;
  mode &= DKM_MODE_MASK;
  if (gemm_path(k, d))  // AUTO picks the single-product GEMM screen
    return mode == DKM_MODE_AUTO || mode == DKM_MODE_SCREEN_BF16 ? IMG_GEMM
                                                                 : IMG_NONE;
  if (d > 128 || !screen_ok(k, d)) return IMG_NONE;
  if (mode == DKM_MODE_AUTO)
    mode = b1_ok(k, d) && !sums_fit_lds(k, d) ? DKM_MODE_SCREEN_BF16
                                              : DKM_MODE_SCREEN_BF16X3;
  if (mode == DKM_MODE_SCREEN_BF16)
    return b1_ok(k, d) && b2_lds_bytes(k, d) <= 160 * 1024
               ? IMG_SINGLE
               : IMG_NONE;
  if (mode == DKM_MODE_SCREEN_BF16X3)
    return d <= 32 && (size_t)(kpad32(k) / 32) * (4096 + 128) <= LDS_BUDGET &&
                   !AB_NO_W32
               ? IMG_SPLIT
               : IMG_NONE;
  return IMG_NONE;
}

size_t dkm_x_image_bytes(int64_t n, int64_t d, int kind) {
  if (n < 0 || d <= 0 || d > INT32_MAX) return 0;
  if (kind == IMG_GEMM) return d > 128 ? x_image_bytes(n, d, kind) : 0;
  if (d > 128) return 0;
  if (kind == IMG_SPLIT && d > 32) return 0;
  if (kind != IMG_SINGLE && kind != IMG_SPLIT && kind != IMG_SORTED) return 0;
  return x_image_bytes(n, d, kind);
}

int dkm_x_image_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                    int kind, void *image, size_t image_bytes, void *stream) {
  return x_image<double>(X, n, d, ldx, kind, image, image_bytes, stream,
                         "dkm_x_image_f64");
}

int dkm_x_image_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                    int kind, void *image, size_t image_bytes, void *stream) {
  return x_image<float>(X, n, d, ldx, kind, image, image_bytes, stream,
                        "dkm_x_image_f32");
}

int dkm_x_image_sorted_ok(int64_t k, int64_t d) {
  // the single-product screen that keeps the image's label copy needs
  // 16-B sample rows (launch_screen's `vec`; the caller checks the row
  // stride and alignment of X)
  return k > 1 && k <= INT32_MAX && d > 0 && d <= 128 && d % 8 == 0 &&
                 dkm_x_image_kind(k, d, DKM_MODE_SCREEN_BF16) == IMG_SINGLE &&
                 mind_ok(k, d)
             ? 1
             : 0;
}

int dkm_x_image_sorted_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                           const int32_t *labels, int64_t k, const void *ws,
                           size_t ws_bytes, void *image, size_t image_bytes,
                           void *stream) {
  return x_image_sorted<double>(X, n, d, ldx, labels, k, ws, ws_bytes, image,
                                image_bytes, nullptr, stream,
                                "dkm_x_image_sorted_f64");
}

int dkm_x_image_sorted_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                           const int32_t *labels, int64_t k, const void *ws,
                           size_t ws_bytes, void *image, size_t image_bytes,
                           void *stream) {
  return x_image_sorted<float>(X, n, d, ldx, labels, k, ws, ws_bytes, image,
                               image_bytes, nullptr, stream,
                               "dkm_x_image_sorted_f32");
}

int dkm_x_image_sorted_sums_f64(const double *X, int64_t n, int64_t d,
                                int64_t ldx, const int32_t *labels, int64_t k,
                                const void *ws, size_t ws_bytes, void *image,
                                size_t image_bytes, double *acc,
                                void *stream) {
  if (!acc) return fail(DKM_E_ARG, "x_image_sorted_sums: acc is NULL");
  return x_image_sorted<double>(X, n, d, ldx, labels, k, ws, ws_bytes, image,
                                image_bytes, acc, stream,
                                "dkm_x_image_sorted_sums_f64");
}

int dkm_x_image_sorted_sums_f32(const float *X, int64_t n, int64_t d,
                                int64_t ldx, const int32_t *labels, int64_t k,
                                const void *ws, size_t ws_bytes, void *image,
                                size_t image_bytes, double *acc,
                                void *stream) {
  if (!acc) return fail(DKM_E_ARG, "x_image_sorted_sums: acc is NULL");
  return x_image_sorted<float>(X, n, d, ldx, labels, k, ws, ws_bytes, image,
                               image_bytes, acc, stream,
                               "dkm_x_image_sorted_sums_f32");
}

#define DKM_IMG_CHECK(who)                                                  \
  if (image && image_bytes < dkm_x_image_bytes(                             \
                                 n, d, image_kind & ~DKM_IMAGE_BUILD))      \
    return fail(DKM_E_ARG, std::string(who) +                               \
                               ": image_bytes does not match n, d and kind");

int dkm_partial_sum_img_f64(const double *X, const void *image, int image_kind,
                            size_t image_bytes, int64_t n, int64_t d,
                            int64_t ldx, const double *C, int64_t k,
                            const void *ws, size_t ws_bytes, int32_t *labels,
                            double *acc, int mode, void *stream) {
  if (!acc) return fail(DKM_E_ARG, "partial_sum: acc is NULL");
  DKM_IMG_CHECK("dkm_partial_sum_img_f64")
  return assign<double>(X, n, d, ldx, C, k, ws, ws_bytes, labels, acc, 1,
                        mode, stream, "dkm_partial_sum_img_f64", image,
                        image_kind);
}

int dkm_partial_sum_img_f32(const float *X, const void *image, int image_kind,
                            size_t image_bytes, int64_t n, int64_t d,
                            int64_t ldx, const double *C, int64_t k,
                            const void *ws, size_t ws_bytes, int32_t *labels,
                            double *acc, int mode, void *stream) {
  if (!acc) return fail(DKM_E_ARG, "partial_sum: acc is NULL");
  DKM_IMG_CHECK("dkm_partial_sum_img_f32")
  return assign<float>(X, n, d, ldx, C, k, ws, ws_bytes, labels, acc, 1,
                       mode, stream, "dkm_partial_sum_img_f32", image,
                       image_kind);
}

int dkm_assign_delta_img_f64(const double *X, const void *image,
                             int image_kind, size_t image_bytes, int64_t n,
                             int64_t d, int64_t ldx, const double *C,
                             int64_t k, const void *ws, size_t ws_bytes,
                             int32_t *labels, double *delta, int mode,
                             void *stream) {
  if (!labels || !delta)
    return fail(DKM_E_ARG, "assign_delta: labels and delta are required");
  DKM_IMG_CHECK("dkm_assign_delta_img_f64")
  return assign<double>(X, n, d, ldx, C, k, ws, ws_bytes, labels, delta, 2,
                        mode, stream, "dkm_assign_delta_img_f64", image,
                        image_kind);
}

int dkm_assign_delta_img_f32(const float *X, const void *image, int image_kind,
                             size_t image_bytes, int64_t n, int64_t d,
                             int64_t ldx, const double *C, int64_t k,
                             const void *ws, size_t ws_bytes, int32_t *labels,
                             double *delta, int mode, void *stream) {
  if (!labels || !delta)
    return fail(DKM_E_ARG, "assign_delta: labels and delta are required");
  DKM_IMG_CHECK("dkm_assign_delta_img_f32")
  return assign<float>(X, n, d, ldx, C, k, ws, ws_bytes, labels, delta, 2,
                       mode, stream, "dkm_assign_delta_img_f32", image,
                       image_kind);
}
#undef DKM_IMG_CHECK

int dkm_label_sums_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                       const int32_t *labels, int64_t k, const void *ws,
                       size_t ws_bytes, double *acc, void *stream) {
  return label_sums_abi<double>(X, n, d, ldx, labels, k, ws, ws_bytes, acc,
                                stream);
}

int dkm_label_sums_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                       const int32_t *labels, int64_t k, const void *ws,
                       size_t ws_bytes, double *acc, void *stream) {
  return label_sums_abi<float>(X, n, d, ldx, labels, k, ws, ws_bytes, acc,
                               stream);
}

int dkm_add_f64(double *y, const double *x, int64_t n, void *stream) {
  if ((!y || !x) && n > 0) return fail(DKM_E_ARG, "add: NULL");
  if (n <= 0) return 0;
  const int64_t g = std::min<int64_t>((n + 255) / 256, 4096);
  k_add<<<(unsigned)g, 256, 0, (hipStream_t)stream>>>(y, x, n, nullptr);
  return check_launch("dkm_add_f64");
}

int dkm_add_f64_nz(double *y, const double *x, int64_t n, int32_t *nonzero,
                   void *stream) {
  if ((!y || !x) && n > 0) return fail(DKM_E_ARG, "add_nz: NULL");
  if (!nonzero) return fail(DKM_E_ARG, "add_nz: NULL flag");
  if (hipMemsetAsync(nonzero, 0, 4, (hipStream_t)stream) != hipSuccess)
    return fail(DKM_E_LAUNCH, "add_nz: flag reset");
  if (n <= 0) return 0;
  const int64_t g = std::min<int64_t>((n + 255) / 256, 4096);
  k_add<<<(unsigned)g, 256, 0, (hipStream_t)stream>>>(y, x, n, nonzero);
  return check_launch("dkm_add_f64_nz");
}

int dkm_add_f64_dd(double *hi, double *lo, const double *x, int64_t n,
                   int32_t *nonzero, void *stream) {
  if ((!hi || !lo || !x) && n > 0) return fail(DKM_E_ARG, "add_dd: NULL");
  if (nonzero &&
      hipMemsetAsync(nonzero, 0, 4, (hipStream_t)stream) != hipSuccess)
    return fail(DKM_E_LAUNCH, "add_dd: flag reset");
  if (n <= 0) return 0;
  const int64_t g = std::min<int64_t>((n + 255) / 256, 4096);
  k_add_dd<<<(unsigned)g, 256, 0, (hipStream_t)stream>>>(hi, lo, x, n,
                                                          nonzero);
  return check_launch("dkm_add_f64_dd");
}

// Result-invalidating A/B timing probes and A/B variant objects
// (variants.sh / variants_b2.sh builds only): the library reports them,
// and tests/test_isa_guard.py requires 0 of the in-tree product build.
int dkm_build_flags(void) {
  return tu_flags_util() | tu_flags_dense() | tu_flags_b2() |
         tu_flags_sorted() | tu_flags_cand() | tu_flags_sparse() |
         tu_flags_gemm() | tu_flags_sums() | tu_flags_neighbors();
}

}  // extern "C"

// Code-object preload (dkm_preload): the runtime loads this file's kernels
// on first use of any of them; an attribute query here does it up front.
namespace dkm {
#if DKM_AB_B1_PROBE || defined(DKM_DBG_NOCOMPUTE) || defined(DKM_DBG_NOLOAD)
#define DKM_DENSE_PROBE 1
#else
#define DKM_DENSE_PROBE 0
#endif
DKM_TU_FLAGS(dense, DKM_DENSE_PROBE)
__global__ void k_tu_dense() {}
int preload_dense() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void *)k_tu_dense) == hipSuccess ? 0
                                                                       : 1;
}
}  // namespace dkm
