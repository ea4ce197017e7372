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
//   k_exact_reg<MAXD>  lane = sample, x in VGPRs, centres (fp64) in LDS,
//                      the exact numpy-order distance to every centre.
//   k_exact_gen        lane = sample, any d, x/centres through the caches.
//   k_screen<MAXD>     lane = sample, fp32 score s_j = |c_j|^2 - 2 x.c_j
//                      against fp32 centres in LDS; a rigorous error bound
//                      decides whether the fp32 winner is the exact winner.
//                      Ambiguous samples are queued for ...
//   k_recheck          wave = one queued sample, lanes = centres, exact
//                      arithmetic, wave-wide (dist, index) argmin.
// Sums/counts go to acc = [sums k*d | counts k] (fp64) through LDS-private
// accumulators flushed once per block, or global fp64 atomics when they do
// not fit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "dkm_internal.h"

namespace dkm {

constexpr int BLOCK = 256;
constexpr size_t LDS_BUDGET = 80 * 1024;  // per block -> >= 2 blocks / CU

enum AccMode { ACC_NONE = 0, ACC_LDS = 1, ACC_GLOBAL = 2 };

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

// Add a sample row to its cluster's sum (and count) -- lane-per-sample form.
template <class TX>
__device__ __forceinline__ void acc_row_lane(int amode, double *lds_acc,
                                             double *acc, int64_t k, int d,
                                             int label, const TX *xrow) {
  if (amode == ACC_LDS) {
    const int ds = lds_stride(d);
    double *srow = lds_acc + (int64_t)label * ds;
    for (int t = 0; t < d; ++t)
      __hip_atomic_fetch_add(srow + t, ld_x(xrow + t), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(lds_acc + k * ds + label, 1.0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
  } else if (amode == ACC_GLOBAL) {
    double *srow = acc + (int64_t)label * d;
    for (int t = 0; t < d; ++t) atomic_add_f64(srow + t, ld_x(xrow + t));
    atomic_add_f64(acc + k * d + label, 1.0);
  }
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
  double *lds_acc = smem + (int64_t)k * d;   // k*(d+1) accumulators
  const int64_t kd = (int64_t)k * d;
  for (int64_t e = threadIdx.x; e < kd; e += blockDim.x) cl[e] = C[e];
  if (amode == ACC_LDS) zero_lds_acc(lds_acc, k, d);
  __syncthreads();

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
    if (labels) labels[i] = bi;
    acc_row_lane(amode, lds_acc, acc, k, d, bi, xr);
  }
  if (amode == ACC_LDS) {
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
  const int64_t kd = (int64_t)k * d;
  if (amode == ACC_LDS) {
    zero_lds_acc(lds_acc, k, d);
    __syncthreads();
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += stride) {
    const TX *xr = X + i * ldx;
    const int bi = exact_label_lane(xr, d, C, k);
    if (labels) labels[i] = bi;
    acc_row_lane(amode, lds_acc, acc, k, d, bi, xr);
  }
  if (amode == ACC_LDS) {
    __syncthreads();
    flush_lds_acc(lds_acc, acc, k, d);
  }
}

// ---------------------------------------------------------------------------
// fp32 screen + rigorous bound; ambiguous samples -> exact re-check queue
// ---------------------------------------------------------------------------
// Bound on |(s_j + |x|^2) - numpy_dist_j^2| for the fp32 score
// s_j = fl32(fmaf(-2, dot32(x32, c32_j), fl32(|c_j|^2))):
//   conversions x->x32, c->c32 (2u|x.c|), the d-term fp32 dot (d*u*sum|x c|),
//   the fp32 norm rounding (u|c|^2) and the final fma (u|s|), all bounded by
//   |x.c| <= |x||c|, |c| <= cmax; plus numpy's own fp64 rounding (relative
//   2^-52 scale) and fp32 underflow (absolute).  Doubled for safety.
__device__ __forceinline__ double screen_bound(int d, double xn, double cm) {
  const double u = 0x1.0p-24;
  double b = 2.0 * (d + 6) * u * (2.0 * xn * cm + cm * cm);
  b += 16.0 * 0x1.0p-52 * (xn + cm) * (xn + cm);
  b += 8.0 * sqrt((double)d) * 0x1.0p-149 * (xn + cm + 1.0) + d * 0x1.0p-147;
  return b;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Four consecutive features t0..t0+3 of one sample as fp64 (zero past d).
template <class TX>
__device__ __forceinline__ void load4(const TX *xr, int t0, int d, bool ok,
                                      bool vec, double (&o)[4]) {
  if (ok && vec && t0 + 3 < d) {
    if constexpr (sizeof(TX) == 8) {
      const double2 a = *(const double2 *)(xr + t0);
      const double2 b = *(const double2 *)(xr + t0 + 2);
      o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
    } else {
      const float4 a = *(const float4 *)(xr + t0);
      o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    }
  } else {
#pragma unroll
    for (int m = 0; m < 4; ++m)
      o[m] = (ok && t0 + m < d) ? (double)xr[t0 + m] : 0.0;
  }
}

// fp32 MFMA screen (v_mfma_f32_16x16x4_f32, exact fp32 fma chains).
// A wave handles 16 samples per step: lane l = (q = l >> 4, j = l & 15)
// holds features db*16 + 4q + m (m = 0..3, every 16-feature block db) of
// sample j -- 16 rows x 128 contiguous bytes per load pair, kept in VGPRs as
// fp64 for the accumulation and as fp32 B-fragments for the MFMAs.  The A
// operand (centres) comes from LDS in fragment order (k_frag).  The MFMA
// output puts the dots of centres cb*16 + 4q + i (i = 0..3) for sample j in
// lane (q, j); each lane keeps a top-2 of its centres, two xor-shuffles merge
// the four lanes of a sample.
template <int NDB, class TX>
__global__ void __launch_bounds__(BLOCK)
    k_screen_mfma(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                  int k, WsView v, int32_t *labels, double *acc, int amode,
                  int64_t base, int vec) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nkb = (int)(kpad16(k) / 16);
  float *cf = (float *)smem;                       // nkb*NDB*256
  float *cn = cf + (int64_t)nkb * NDB * 256;       // nkb*16
  double *lds_acc = smem + ((int64_t)nkb * NDB * 256 + nkb * 16) / 2;
  const int64_t kd = (int64_t)k * d;
  {
    const f32x4 *src = (const f32x4 *)v.cfrag;
    f32x4 *dst = (f32x4 *)cf;
    for (int e = threadIdx.x; e < nkb * NDB * 64; e += BLOCK) dst[e] = src[e];
    for (int e = threadIdx.x; e < nkb * 16; e += BLOCK) cn[e] = v.cnpad[e];
    if (amode == ACC_LDS) zero_lds_acc(lds_acc, k, d);
  }
  const double cm = __longlong_as_double((long long)v.hdr->cmax_bits);
  const int64_t nq = v.hdr->n_queue;
  __syncthreads();

  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & 15;
  const int64_t wv = (int64_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
  const int64_t nwv = (int64_t)gridDim.x * (BLOCK / 64);
  for (int64_t s0 = base + wv * 16; s0 < n; s0 += nwv * 16) {
    const int64_t si = s0 + j;
    const bool valid = si < n;
    const TX *xr = X + (valid ? si : s0) * ldx;
    double xv[NDB][4];
    float xb[NDB][4];
    double xx = 0.0;
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      load4(xr, db * 16 + 4 * q, d, valid, vec != 0, xv[db]);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        xx = fma(xv[db][m], xv[db][m], xx);
        xb[db][m] = (float)xv[db][m];
      }
    }
    xx += __shfl_xor(xx, 16, WAVE);
    xx += __shfl_xor(xx, 32, WAVE);

    float b1 = INFINITY, b2 = INFINITY;
    int i1 = 0;
    for (int cb = 0; cb < nkb; ++cb) {
      f32x4 accv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        const f32x4 a = *(const f32x4 *)(cf + (((int64_t)cb * NDB + db) * 64 +
                                               lane) * 4);
        accv = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, xb[db][0], accv, 0,
                                                    0, 0);
        accv = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, xb[db][1], accv, 0,
                                                    0, 0);
        accv = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, xb[db][2], accv, 0,
                                                    0, 0);
        accv = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, xb[db][3], accv, 0,
                                                    0, 0);
      }
      const float4 cn4 = *(const float4 *)(cn + cb * 16 + 4 * q);
      const float cnv[4] = {cn4.x, cn4.y, cn4.z, cn4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float sc = fmaf(-2.f, accv[i], cnv[i]);
        if (sc < b1) {
          b2 = b1;
          b1 = sc;
          i1 = cb * 16 + 4 * q + i;
        } else if (sc < b2) {
          b2 = sc;
        }
      }
    }
    // merge the top-2 of the four lanes of sample j (first index on ties)
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float ob1 = __shfl_xor(b1, off, WAVE);
      const float ob2 = __shfl_xor(b2, off, WAVE);
      const int oi1 = __shfl_xor(i1, off, WAVE);
      if (ob1 < b1 || (ob1 == b1 && oi1 < i1)) {
        b2 = fminf(b1, ob2);
        b1 = ob1;
        i1 = oi1;
      } else {
        b2 = fminf(b2, ob1);
      }
    }
    const double xn = sqrt(xx);
    const double B = screen_bound(d, xn, cm);
    const bool sane = (xn < 1e18) && (xn * cm < 1e30);
    const bool unique = sane && ((double)b2 - (double)b1 > 2.0 * B);
    if (!valid) continue;
    if (!unique) {
      if (q == 0) {
        const uint32_t pos = atomicAdd(&v.hdr->qcount, 1u);
        if ((int64_t)pos < nq) v.queue[pos] = (int32_t)(si - base);
      }
      continue;  // label + sums by k_recheck
    }
    if (q == 0 && labels) labels[si] = i1;
    if (amode == ACC_LDS) {
      double *srow = lds_acc + (int64_t)i1 * lds_stride(d);
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int t = db * 16 + 4 * q + m;
          if (t < d)
            __hip_atomic_fetch_add(srow + t, xv[db][m], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      if (q == 0)
        __hip_atomic_fetch_add(lds_acc + (int64_t)k * lds_stride(d) + i1, 1.0,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (amode == ACC_GLOBAL) {
      double *srow = acc + (int64_t)i1 * d;
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int t = db * 16 + 4 * q + m;
          if (t < d) atomic_add_f64(srow + t, xv[db][m]);
        }
      if (q == 0) atomic_add_f64(acc + kd + i1, 1.0);
    }
  }
  if (amode == ACC_LDS) {
    __syncthreads();
    flush_lds_acc(lds_acc, acc, k, d);
  }
}

// ---------------------------------------------------------------------------
// bf16x3 MFMA screen (v_mfma_f32_16x16x32_bf16).  x = xh + xl + O(2^-16|x|),
// c likewise; x.c ~ xh.ch + xh.cl + xl.ch, products exact in fp32, fp32
// accumulation.  Bound on |(s_j + |x|^2) - numpy_dist_j^2| (doubled):
//   split remainder 3.1 * 2^-16 * sum|x c|, fp32 accumulation of 3d terms
//   (3d + 6) * 2^-23 * sum|x c|, fp32 |c|^2 and final fma 2^-24 (|c|^2 +
//   2|x.c|), numpy's fp64 rounding, bf16 underflow (absolute).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double screen_bound_b3(int d, double xn,
                                                  double cm) {
  const double rel = 3.1 * 0x1.0p-16 + (3.0 * d + 6.0) * 0x1.0p-23;
  double b = 2.0 * rel * (2.0 * xn * cm + cm * cm);
  b += 16.0 * 0x1.0p-52 * (xn + cm) * (xn + cm);
  b += 8.0 * d * 0x1.0p-120 * (xn + cm + 1.0);
  return b;
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Eight consecutive features t0..t0+7 as fp64 (zero past d / invalid).
template <class TX>
__device__ __forceinline__ void load8(const TX *xr, int t0, int d, bool ok,
                                      bool vec, double (&o)[8]) {
  if (ok && vec && t0 + 7 < d) {
    if constexpr (sizeof(TX) == 8) {
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const double2 a = *(const double2 *)(xr + t0 + 2 * h);
        o[2 * h] = a.x;
        o[2 * h + 1] = a.y;
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 a = *(const float4 *)(xr + t0 + 4 * h);
        o[4 * h] = a.x; o[4 * h + 1] = a.y; o[4 * h + 2] = a.z;
        o[4 * h + 3] = a.w;
      }
    }
  } else {
#pragma unroll
    for (int m = 0; m < 8; ++m)
      o[m] = (ok && t0 + m < d) ? (double)xr[t0 + m] : 0.0;
  }
}

constexpr int SBLOCK = 512;

// A wave handles NB blocks of 16 samples per step; lane l = (q = l >> 4,
// j = l & 15) holds features ks*32 + 8q + jj (jj < 8) of sample j of each
// block: 16 rows x 256 contiguous bytes per 4 load instructions.  Centres:
// bf16 hi/lo fragments in LDS (k_frag).  The MFMA output gives lane (q, j)
// the dots of centres cb*16 + 4q + i (i < 4) with sample j; top-2 per lane,
// two xor-shuffles merge the four lanes of a sample.
template <int NKS, int NB, class TX>
__global__ void __launch_bounds__(SBLOCK)
    k_screen_b3(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                int k, WsView v, int32_t *labels, double *acc, int amode,
                int64_t base, int vec) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nkb = (int)(kpad16(k) / 16);
  bf16x8 *cf = (bf16x8 *)smem;                        // nkb*NKS*128 vecs
  float *cn = (float *)(cf + (int64_t)nkb * NKS * 128);  // nkb*16
  double *lds_acc = (double *)(cn + nkb * 16);
  const int64_t kd = (int64_t)k * d;
  {
    const bf16x8 *src = (const bf16x8 *)v.bfrag;
    for (int e = threadIdx.x; e < nkb * NKS * 128; e += SBLOCK) cf[e] = src[e];
    for (int e = threadIdx.x; e < nkb * 16; e += SBLOCK) cn[e] = v.cnpad[e];
    if (amode == ACC_LDS) zero_lds_acc(lds_acc, k, d);
  }
  const double cm = __longlong_as_double((long long)v.hdr->cmax_bits);
  const int64_t nq = v.hdr->n_queue;
  __syncthreads();

  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & 15;
  const int64_t wv = (int64_t)blockIdx.x * (SBLOCK / 64) + (threadIdx.x >> 6);
  const int64_t nwv = (int64_t)gridDim.x * (SBLOCK / 64);
  for (int64_t s0 = base + wv * 16 * NB; s0 < n; s0 += nwv * 16 * NB) {
    double xv[NB][NKS][8];
    bf16x8 xh[NB][NKS], xl[NB][NKS];
    double xx[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int64_t si = s0 + 16 * b + j;
      const bool valid = si < n;
      const TX *xr = X + (valid ? si : s0) * ldx;
      xx[b] = 0.0;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        load8(xr, ks * 32 + 8 * q, d, valid, vec != 0, xv[b][ks]);
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const double x = xv[b][ks][m];
          xx[b] = fma(x, x, xx[b]);
          const __bf16 h = (__bf16)(float)x;
          xh[b][ks][m] = h;
          xl[b][ks][m] = (__bf16)(float)(x - (double)(float)h);
        }
      }
      xx[b] += __shfl_xor(xx[b], 16, WAVE);
      xx[b] += __shfl_xor(xx[b], 32, WAVE);
    }
    float b1[NB], b2[NB];
    int i1[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      b1[b] = INFINITY;
      b2[b] = INFINITY;
      i1[b] = 0;
    }
    for (int cb = 0; cb < nkb; ++cb) {
      f32x4 accv[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) accv[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 ah = cf[((cb * NKS + ks) * 2 + 0) * 64 + lane];
        const bf16x8 al = cf[((cb * NKS + ks) * 2 + 1) * 64 + lane];
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
      const float4 cn4 = *(const float4 *)(cn + cb * 16 + 4 * q);
      const float cnv[4] = {cn4.x, cn4.y, cn4.z, cn4.w};
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float sc = fmaf(-2.f, accv[b][i], cnv[i]);
          const bool lt = sc < b1[b];
          b2[b] = lt ? b1[b] : fminf(b2[b], sc);
          i1[b] = lt ? cb * 16 + 4 * q + i : i1[b];
          b1[b] = lt ? sc : b1[b];
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int off = 16; off <= 32; off <<= 1) {
        const float ob1 = __shfl_xor(b1[b], off, WAVE);
        const float ob2 = __shfl_xor(b2[b], off, WAVE);
        const int oi1 = __shfl_xor(i1[b], off, WAVE);
        if (ob1 < b1[b] || (ob1 == b1[b] && oi1 < i1[b])) {
          b2[b] = fminf(b1[b], ob2);
          b1[b] = ob1;
          i1[b] = oi1;
        } else {
          b2[b] = fminf(b2[b], ob1);
        }
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int64_t si = s0 + 16 * b + j;
      if (si >= n) continue;
      const double xn = sqrt(xx[b]);
      const double B = screen_bound_b3(d, xn, cm);
      const bool sane = (xn < 1e18) && (xn * cm < 1e30);
      const bool unique = sane && ((double)b2[b] - (double)b1[b] > 2.0 * B);
      if (!unique) {
        if (q == 0) {
          const uint32_t pos = atomicAdd(&v.hdr->qcount, 1u);
          if ((int64_t)pos < nq) v.queue[pos] = (int32_t)(si - base);
        }
        continue;  // label + sums by k_recheck
      }
      const int lab = i1[b];
      if (q == 0 && labels) labels[si] = lab;
      if (amode == ACC_LDS) {
        double *srow = lds_acc + (int64_t)lab * lds_stride(d);
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
          for (int m = 0; m < 8; ++m) {
            const int t = ks * 32 + 8 * q + m;
            if (t < d)
              __hip_atomic_fetch_add(srow + t, xv[b][ks][m], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        if (q == 0)
          __hip_atomic_fetch_add(lds_acc + (int64_t)k * lds_stride(d) + lab,
                                 1.0, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (amode == ACC_GLOBAL) {
        double *srow = acc + (int64_t)lab * d;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
          for (int m = 0; m < 8; ++m) {
            const int t = ks * 32 + 8 * q + m;
            if (t < d) atomic_add_f64(srow + t, xv[b][ks][m]);
          }
        if (q == 0) atomic_add_f64(acc + kd + lab, 1.0);
      }
    }
  }
  if (amode == ACC_LDS) {
    __syncthreads();
    flush_lds_acc(lds_acc, acc, k, d);
  }
}

// Exact re-check for d <= 128: numpy's pairwise order is a single leaf, so
// no recursion stack (low VGPR use, high occupancy).
template <class TX>
__global__ void __launch_bounds__(BLOCK)
    k_recheck_small(const TX *__restrict__ X, int d, int64_t ldx,
                    const double *__restrict__ C, int k, WsView v,
                    int32_t *labels, double *acc, int64_t base) {
  const uint32_t qc = v.hdr->qcount;
  const int64_t total = std::min<int64_t>((int64_t)qc, v.hdr->n_queue);
  if (blockIdx.x == 0 && threadIdx.x == 0)
    atomicAdd((unsigned long long *)&v.hdr->rechecked_total,
              (unsigned long long)qc);
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t qi = wave; qi < total; qi += nwaves) {
    const int64_t i =
        base + __builtin_amdgcn_readfirstlane(v.queue[qi]);  // wave-uniform
    const TX *xr = X + i * ldx;
    double best = INFINITY;
    int bi = 0x7fffffff;
    for (int jc = lane; jc < k; jc += 64) {
      const double dist =
          sqrt(pw_leaf(SqDiffT<TX>{xr, v.ct64 + jc, (int64_t)k}, 0, d));
      if (dist < best || bi == 0x7fffffff) {
        best = dist;
        bi = jc;
      }
    }
    wave_argmin(best, bi);
    if (lane == 0 && labels) labels[i] = bi;
    if (acc) {
      for (int t = lane; t < d; t += 64)
        atomic_add_f64(acc + (int64_t)bi * d + t, ld_x(xr + t));
      if (lane == 0) atomic_add_f64(acc + (int64_t)k * d + bi, 1.0);
    }
  }
}

// wave per queued sample; lanes own centres j = lane, lane+64, ...
template <class TX>
__global__ void __launch_bounds__(BLOCK)
    k_recheck(const TX *__restrict__ X, int d, int64_t ldx,
              const double *__restrict__ C, int k, WsView v, int32_t *labels,
              double *acc, int64_t base) {
  const uint32_t qc = v.hdr->qcount;
  const int64_t total = std::min<int64_t>((int64_t)qc, v.hdr->n_queue);
  if (blockIdx.x == 0 && threadIdx.x == 0)
    atomicAdd((unsigned long long *)&v.hdr->rechecked_total,
              (unsigned long long)qc);
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t q = wave; q < total; q += nwaves) {
    const int64_t i = base + v.queue[q];
    const TX *xr = X + i * ldx;
    double best = INFINITY;
    int bi = 0x7fffffff;  // lanes without a centre never win
    for (int j = lane; j < k; j += 64) {
      const double dist = sqrt(pw_sum(SqDiff<TX>{xr, C + (int64_t)j * d}, d));
      if (dist < best || bi == 0x7fffffff) {
        best = dist;
        bi = j;
      }
    }
    wave_argmin(best, bi);
    if (lane == 0 && labels) labels[i] = bi;
    if (acc) {
      for (int t = lane; t < d; t += 64)
        atomic_add_f64(acc + (int64_t)bi * d + t, ld_x(xr + t));
      if (lane == 0) atomic_add_f64(acc + (int64_t)k * d + bi, 1.0);
    }
  }
}

// ---------------------------------------------------------------------------
// host dispatch
// ---------------------------------------------------------------------------
static int pick_maxd(int d) {
  if (d <= 8) return 8;
  if (d <= 16) return 16;
  if (d <= 32) return 32;
  if (d <= 64) return 64;
  if (d <= 128) return 128;
  return 0;
}

static unsigned grid_for(int64_t n, const void *kern, size_t lds) {
  int per_cu = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, BLOCK,
                                                   lds) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int64_t cap = (int64_t)dev_info().cus * per_cu;
  const int64_t need = (n + BLOCK - 1) / BLOCK;
  return (unsigned)std::max<int64_t>(1, std::min(need, cap));
}

template <class TX>
static int launch_exact(const TX *X, int64_t n, int d, int64_t ldx,
                        const double *C, int k, int32_t *labels, double *acc,
                        hipStream_t s) {
  const int64_t kd = (int64_t)k * d;
  const size_t c_bytes = (size_t)kd * 8;
  const size_t a_bytes = (size_t)lds_acc_len(k, d) * 8;
  const int maxd = pick_maxd(d);
  const bool creg = maxd > 0 && maxd <= 64 && c_bytes <= LDS_BUDGET;
  int amode = ACC_NONE;
  if (acc) {
    const size_t base = creg ? c_bytes : 0;
    amode = (base + a_bytes <= LDS_BUDGET) ? ACC_LDS : ACC_GLOBAL;
  }
  const size_t lds =
      (creg ? c_bytes : 0) + (amode == ACC_LDS ? a_bytes : 0);
  if (creg) {
#define DKM_EXACT_CASE(M)                                                   \
  case M: {                                                                 \
    const void *kf = (const void *)k_exact_reg<M, TX>;                      \
    unsigned g = grid_for(n, kf, lds);                                      \
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
    unsigned g = grid_for(n, kf, lds);
    k_exact_gen<TX><<<g, BLOCK, lds, s>>>(X, n, d, ldx, C, k, labels, acc,
                                          amode);
  }
  return check_launch("exact assignment");
}

template <class TX>
static int launch_recheck(const TX *X, int d, int64_t ldx, const double *C,
                          int k, const WsView &v, int32_t *labels,
                          double *acc, int64_t base, int64_t count,
                          hipStream_t s);

static size_t screen_lds_fixed(int64_t k, int64_t d) {
  return (size_t)(kpad16(k) * dpad16(d) + kpad16(k)) * 4;
}

template <class TX>
static bool screen_ok(int64_t k, int d) {
  return k >= 2 && d <= 128 && screen_lds_fixed(k, d) <= LDS_BUDGET;
}

template <class TX>
static int launch_screen(const TX *X, int64_t n, int d, int64_t ldx,
                         const double *C, int k, const WsView &v, size_t wsb,
                         int32_t *labels, double *acc, hipStream_t s) {
  const int64_t kd = (int64_t)k * d;
  const size_t cb = screen_lds_fixed(k, d);
  const size_t a_bytes = (size_t)lds_acc_len(k, d) * 8;
  int amode = ACC_NONE;
  if (acc) amode = (cb + a_bytes <= LDS_BUDGET) ? ACC_LDS : ACC_GLOBAL;
  const size_t lds = cb + (amode == ACC_LDS ? a_bytes : 0);
  const size_t fixed = (size_t)((const char *)v.queue - (const char *)v.hdr);
  const int64_t nq = std::min<int64_t>((int64_t)((wsb - fixed) / 4), INT32_MAX);
  if (nq < 1) return fail(DKM_E_WORKSPACE, "screen: no re-check slots");
  const int vec = ((ldx % (16 / (int64_t)sizeof(TX))) == 0 &&
                   ((uintptr_t)X % 16) == 0) ? 1 : 0;
  const int ndb = (int)(dpad16(d) / 16);
  // Chunks of at most n_queue samples: every ambiguous sample gets a slot.
  for (int64_t base = 0; base < n; base += nq) {
    const int64_t end = std::min(n, base + nq);
    hipError_t e = hipMemsetAsync(&v.hdr->qcount, 0, 4, s);
    if (e != hipSuccess)
      return fail((int)e, std::string("screen: reset queue: ") +
                              hipGetErrorString(e));
    const int64_t tiles = (end - base + 15) / 16;
    switch (ndb) {
#define DKM_SCREEN_CASE(M)                                                  \
  case M: {                                                                 \
    const void *kf = (const void *)k_screen_mfma<M, TX>;                    \
    unsigned g = grid_for(tiles * 64, kf, lds);                             \
    k_screen_mfma<M, TX><<<g, BLOCK, lds, s>>>(X, end, d, ldx, k, v,        \
                                               labels, acc, amode, base,    \
                                               vec);                        \
    break;                                                                  \
  }
      DKM_SCREEN_CASE(1)
      DKM_SCREEN_CASE(2)
      DKM_SCREEN_CASE(3)
      DKM_SCREEN_CASE(4)
      DKM_SCREEN_CASE(5)
      DKM_SCREEN_CASE(6)
      DKM_SCREEN_CASE(7)
      DKM_SCREEN_CASE(8)
#undef DKM_SCREEN_CASE
      default:
        return fail(DKM_E_ARG, "screen: d too large");
    }
    if (int r = check_launch("screen assignment")) return r;
    // exact re-check of the queued samples: grid sized for the worst case,
    // the kernel reads the true count from the workspace header.
    if (int r = launch_recheck<TX>(X, d, ldx, C, k, v, labels, acc, base,
                                   end - base, s))
      return r;
  }
  return 0;
}

static size_t b3_lds_fixed(int64_t k, int64_t d) {
  return (size_t)(kpad16(k) * dpad32(d) * 4 + kpad16(k) * 4);
}

template <class TX>
static bool b3_ok(int64_t k, int d) {
  return k >= 2 && d <= 128 && b3_lds_fixed(k, d) <= LDS_BUDGET;
}

template <class TX>
static int launch_recheck(const TX *X, int d, int64_t ldx, const double *C,
                          int k, const WsView &v, int32_t *labels,
                          double *acc, int64_t base, int64_t count,
                          hipStream_t s) {
  const int64_t waves_per_block = BLOCK / 64;
  const unsigned rg = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>((int64_t)dev_info().cus * 16,
                           (count + waves_per_block - 1) / waves_per_block));
  if (d <= 128)
    k_recheck_small<TX><<<rg, BLOCK, 0, s>>>(X, d, ldx, C, k, v, labels, acc,
                                             base);
  else
    k_recheck<TX><<<rg, BLOCK, 0, s>>>(X, d, ldx, C, k, v, labels, acc, base);
  return check_launch("exact re-check");
}

template <int NKS, int NB, class TX>
static unsigned b3_grid(int64_t nsamp, size_t lds) {
  const void *kf = (const void *)k_screen_b3<NKS, NB, TX>;
  int per_cu = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, SBLOCK,
                                                   lds) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int64_t cap = (int64_t)dev_info().cus * per_cu;
  const int64_t need = (nsamp + 16 * NB * (SBLOCK / 64) - 1) /
                       (16 * NB * (SBLOCK / 64));
  return (unsigned)std::max<int64_t>(1, std::min(need, cap));
}

template <class TX>
static int launch_screen_b3(const TX *X, int64_t n, int d, int64_t ldx,
                            const double *C, int k, const WsView &v,
                            size_t wsb, int32_t *labels, double *acc,
                            hipStream_t s) {
  const int64_t kd = (int64_t)k * d;
  const size_t cb = b3_lds_fixed(k, d);
  const size_t a_bytes = (size_t)lds_acc_len(k, d) * 8;
  int amode = ACC_NONE;
  if (acc) amode = (cb + a_bytes <= LDS_BUDGET) ? ACC_LDS : ACC_GLOBAL;
  const size_t lds = cb + (amode == ACC_LDS ? a_bytes : 0);
  const size_t fixed = (size_t)((const char *)v.queue - (const char *)v.hdr);
  const int64_t nq = std::min<int64_t>((int64_t)((wsb - fixed) / 4), INT32_MAX);
  if (nq < 1) return fail(DKM_E_WORKSPACE, "screen: no re-check slots");
  const int vec = ((ldx % (16 / (int64_t)sizeof(TX))) == 0 &&
                   ((uintptr_t)X % 16) == 0) ? 1 : 0;
  const int nks = (int)(dpad32(d) / 32);
  for (int64_t base = 0; base < n; base += nq) {
    const int64_t end = std::min(n, base + nq);
    hipError_t e = hipMemsetAsync(&v.hdr->qcount, 0, 4, s);
    if (e != hipSuccess)
      return fail((int)e, std::string("screen: reset queue: ") +
                              hipGetErrorString(e));
    switch (nks) {
#define DKM_B3_CASE(KS, NBV)                                                \
  case KS: {                                                                \
    unsigned g = b3_grid<KS, NBV, TX>(end - base, lds);                     \
    k_screen_b3<KS, NBV, TX><<<g, SBLOCK, lds, s>>>(                        \
        X, end, d, ldx, k, v, labels, acc, amode, base, vec);               \
    break;                                                                  \
  }
      DKM_B3_CASE(1, 2)
      DKM_B3_CASE(2, 2)
      DKM_B3_CASE(3, 1)
      DKM_B3_CASE(4, 1)
#undef DKM_B3_CASE
      default:
        return fail(DKM_E_ARG, "screen_bf16x3: d too large");
    }
    if (int r = check_launch("bf16x3 screen assignment")) return r;
    if (int r = launch_recheck<TX>(X, d, ldx, C, k, v, labels, acc, base,
                                   end - base, s))
      return r;
  }
  return 0;
}

template <class TX>
static int assign(const TX *X, int64_t n, int64_t d, int64_t ldx,
                  const double *C, int64_t k, const void *ws, size_t wsb,
                  int32_t *labels, double *acc, int mode, void *stream,
                  const char *who) {
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
    mode = b3_ok<TX>(k, (int)d)       ? DKM_MODE_SCREEN_BF16X3
           : screen_ok<TX>(k, (int)d) ? DKM_MODE_SCREEN32
                                      : DKM_MODE_EXACT;
  if (mode == DKM_MODE_EXACT)
    return launch_exact<TX>(X, n, (int)d, ldx, C, (int)k, labels, acc, s);
  if (mode == DKM_MODE_SCREEN_BF16X3) {
    if (!b3_ok<TX>(k, (int)d))
      return launch_exact<TX>(X, n, (int)d, ldx, C, (int)k, labels, acc, s);
    WsView v;
    if (int r = ws_view(ws, wsb, k, d, &v)) return r;
    return launch_screen_b3<TX>(X, n, (int)d, ldx, C, (int)k, v, wsb, labels,
                                acc, s);
  }
  if (mode == DKM_MODE_SCREEN32) {
    if (!screen_ok<TX>(k, (int)d))
      return launch_exact<TX>(X, n, (int)d, ldx, C, (int)k, labels, acc, s);
    WsView v;
    if (int r = ws_view(ws, wsb, k, d, &v)) return r;
    return launch_screen<TX>(X, n, (int)d, ldx, C, (int)k, v, wsb, labels, acc,
                             s);
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
  return assign<double>(X, n, d, ldx, C, k, ws, ws_bytes, labels, acc, mode,
                        stream, "dkm_partial_sum_f64");
}

int dkm_partial_sum_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                        const double *C, int64_t k, const void *ws,
                        size_t ws_bytes, int32_t *labels, double *acc,
                        int mode, void *stream) {
  if (!acc) return fail(DKM_E_ARG, "partial_sum: acc is NULL");
  return assign<float>(X, n, d, ldx, C, k, ws, ws_bytes, labels, acc, mode,
                       stream, "dkm_partial_sum_f32");
}

int dkm_predict_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                    const double *C, int64_t k, const void *ws,
                    size_t ws_bytes, int32_t *labels, int mode, void *stream) {
  if (!labels) return fail(DKM_E_ARG, "predict: labels is NULL");
  return assign<double>(X, n, d, ldx, C, k, ws, ws_bytes, labels, nullptr,
                        mode, stream, "dkm_predict_f64");
}

int dkm_predict_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                    const double *C, int64_t k, const void *ws,
                    size_t ws_bytes, int32_t *labels, int mode, void *stream) {
  if (!labels) return fail(DKM_E_ARG, "predict: labels is NULL");
  return assign<float>(X, n, d, ldx, C, k, ws, ws_bytes, labels, nullptr,
                       mode, stream, "dkm_predict_f32");
}

}  // extern "C"
