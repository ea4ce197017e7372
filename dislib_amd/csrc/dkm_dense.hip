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

// Add a sample row to its cluster's sum (and count) -- lane-per-sample form.
template <class TX>
__device__ __forceinline__ void acc_row_lane(int amode, double *lds_acc,
                                             double *acc, int64_t k, int d,
                                             int label, const TX *xrow) {
  if (amode == ACC_LDS) {
    double *srow = lds_acc + (int64_t)label * d;
    for (int t = 0; t < d; ++t)
      __hip_atomic_fetch_add(srow + t, ld_x(xrow + t), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(lds_acc + k * d + label, 1.0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
  } else if (amode == ACC_GLOBAL) {
    double *srow = acc + (int64_t)label * d;
    for (int t = 0; t < d; ++t) atomic_add_f64(srow + t, ld_x(xrow + t));
    atomic_add_f64(acc + k * d + label, 1.0);
  }
}

__device__ __forceinline__ void flush_lds_acc(const double *lds_acc,
                                              double *acc, int64_t len) {
  for (int64_t e = threadIdx.x; e < len; e += blockDim.x) {
    const double v = lds_acc[e];
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
  if (amode == ACC_LDS)
    for (int64_t e = threadIdx.x; e < kd + k; e += blockDim.x)
      lds_acc[e] = 0.0;
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
    flush_lds_acc(lds_acc, acc, kd + k);
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
    for (int64_t e = threadIdx.x; e < kd + k; e += blockDim.x)
      lds_acc[e] = 0.0;
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
    flush_lds_acc(lds_acc, acc, kd + k);
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

template <int MAXD, class TX>
__global__ void __launch_bounds__(BLOCK)
    k_screen(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
             const double *__restrict__ C, int k, int dpad, WsView v,
             int32_t *labels, double *acc, int amode, int64_t base) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  float *c32 = (float *)smem;                       // k*dpad
  float *cn = c32 + (int64_t)k * dpad;              // k
  double *lds_acc =
      smem + round_up((int64_t)k * dpad + k, 4) / 2;  // 16-B aligned
  const int64_t kd = (int64_t)k * d;
  for (int64_t e = threadIdx.x; e < (int64_t)k * dpad; e += blockDim.x)
    c32[e] = v.c32[e];
  for (int64_t e = threadIdx.x; e < k; e += blockDim.x) cn[e] = v.cn32[e];
  if (amode == ACC_LDS)
    for (int64_t e = threadIdx.x; e < kd + k; e += blockDim.x)
      lds_acc[e] = 0.0;
  const double cm = __longlong_as_double((long long)v.hdr->cmax_bits);
  const int64_t nq = v.hdr->n_queue;
  __syncthreads();

  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = base + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       i < n; i += stride) {
    const TX *xr = X + i * ldx;
    float x32[MAXD];
    double xx = 0.0;
#pragma unroll
    for (int t = 0; t < MAXD; ++t) {
      const double xv = t < d ? ld_x(xr + t) : 0.0;
      xx = fma(xv, xv, xx);
      x32[t] = (float)xv;
    }
    float b1 = INFINITY, b2 = INFINITY;
    int i1 = 0;
    for (int j = 0; j < k; ++j) {
      const float *cj = c32 + (int64_t)j * dpad;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
      for (int t = 0; t < MAXD; t += 4) {
        if (t < dpad) {
          const float4 cv = *(const float4 *)(cj + t);
          a0 = fmaf(x32[t + 0], cv.x, a0);
          a1 = fmaf(x32[t + 1], cv.y, a1);
          a2 = fmaf(x32[t + 2], cv.z, a2);
          a3 = fmaf(x32[t + 3], cv.w, a3);
        }
      }
      const float dot = (a0 + a1) + (a2 + a3);
      const float s = fmaf(-2.f, dot, cn[j]);
      if (s < b1) {
        b2 = b1;
        b1 = s;
        i1 = j;
      } else if (s < b2) {
        b2 = s;
      }
    }
    const double xn = sqrt(xx);
    const double B = screen_bound(d, xn, cm);
    const bool sane = (xn < 1e18) && (xn * cm < 1e30);
    const bool unique = sane && ((double)b2 - (double)b1 > 2.0 * B);
    if (!unique) {
      // the host splits calls so that n <= n_queue: pos < nq always
      const uint32_t pos = atomicAdd(&v.hdr->qcount, 1u);
      if ((int64_t)pos < nq) v.queue[pos] = (int32_t)(i - base);
      continue;  // label + sums by k_recheck
    }
    if (labels) labels[i] = i1;
    acc_row_lane(amode, lds_acc, acc, k, d, i1, xr);
  }
  if (amode == ACC_LDS) {
    __syncthreads();
    flush_lds_acc(lds_acc, acc, kd + k);
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
  const size_t a_bytes = (size_t)(kd + k) * 8;
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
static bool screen_ok(int64_t k, int d) {
  const int64_t dpad = round_up(d, 4);
  const size_t cb = (size_t)(round_up(k * dpad + k, 4)) * 4;
  return k >= 2 && pick_maxd(d) > 0 && d <= 128 && cb <= LDS_BUDGET;
}

template <class TX>
static int launch_screen(const TX *X, int64_t n, int d, int64_t ldx,
                         const double *C, int k, const WsView &v, size_t wsb,
                         int32_t *labels, double *acc, hipStream_t s) {
  const int64_t kd = (int64_t)k * d;
  const int dpad = (int)round_up(d, 4);
  const size_t cb = (size_t)(round_up((int64_t)k * dpad + k, 4)) * 4;
  const size_t a_bytes = (size_t)(kd + k) * 8;
  int amode = ACC_NONE;
  if (acc) amode = (cb + a_bytes <= LDS_BUDGET) ? ACC_LDS : ACC_GLOBAL;
  const size_t lds = cb + (amode == ACC_LDS ? a_bytes : 0);
  const size_t fixed = (size_t)((const char *)v.queue - (const char *)v.hdr);
  const int64_t nq = std::min<int64_t>((int64_t)((wsb - fixed) / 4), INT32_MAX);
  if (nq < 1) return fail(DKM_E_WORKSPACE, "screen: no re-check slots");
  const int64_t waves_per_block = BLOCK / 64;
  // Chunks of at most n_queue samples: every ambiguous sample gets a slot.
  for (int64_t base = 0; base < n; base += nq) {
    const int64_t end = std::min(n, base + nq);
    hipError_t e = hipMemsetAsync(&v.hdr->qcount, 0, 4, s);
    if (e != hipSuccess)
      return fail((int)e, std::string("screen: reset queue: ") +
                              hipGetErrorString(e));
    switch (pick_maxd(d)) {
#define DKM_SCREEN_CASE(M)                                                  \
  case M: {                                                                 \
    const void *kf = (const void *)k_screen<M, TX>;                         \
    unsigned g = grid_for(end - base, kf, lds);                             \
    k_screen<M, TX><<<g, BLOCK, lds, s>>>(X, end, d, ldx, C, k, dpad, v,    \
                                          labels, acc, amode, base);        \
    break;                                                                  \
  }
      DKM_SCREEN_CASE(8)
      DKM_SCREEN_CASE(16)
      DKM_SCREEN_CASE(32)
      DKM_SCREEN_CASE(64)
      DKM_SCREEN_CASE(128)
#undef DKM_SCREEN_CASE
      default:
        return fail(DKM_E_ARG, "screen: d too large");
    }
    if (int r = check_launch("screen assignment")) return r;
    // exact re-check of the queued samples: grid sized for the worst case,
    // the kernel reads the true count from the workspace header.
    const unsigned rg = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>((int64_t)dev_info().cus * 8,
                             (end - base + waves_per_block - 1) /
                                 waves_per_block));
    k_recheck<TX><<<rg, BLOCK, 0, s>>>(X, d, ldx, C, k, v, labels, acc, base);
    if (int r = check_launch("exact re-check")) return r;
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
    mode = screen_ok<TX>(k, (int)d) ? DKM_MODE_SCREEN32 : DKM_MODE_EXACT;
  if (mode == DKM_MODE_EXACT)
    return launch_exact<TX>(X, n, (int)d, ldx, C, (int)k, labels, acc, s);
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
