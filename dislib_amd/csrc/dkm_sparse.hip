// dkm_sparse.hip -- CSR Subset path.
//
// Replaces the sparse branch of `_partial_sum` / `_predict`
// (cluster/kmeans/base.py:169,196), where the reference calls
// sklearn.metrics.pairwise_distances(sample_csr, centres_csr) per sample.
// sklearn 1.7.2 `_euclidean_distances` (metrics/pairwise.py:391-442) for
// fp64 CSR inputs computes, per centre j,
//   dot_j = scipy csr_matmat: sequential over the sample's stored entries,
//           sums[j] += x_v * C[j][col_v]   (product then add, no FMA)
//   xx    = sequential sum of x_v^2 over stored entries
//   yy_j  = sequential sum of C[j][t]^2 over t (stored entries; exact zeros
//           add nothing)
//   dist_j = sqrt(max(0, ((-2 * dot_j) + xx) + yy_j))
// followed by np.argmin (first index).  This kernel reproduces that
// arithmetic bit-for-bit.
//
// Layout: one wave per sample, lanes over centres j = lane, lane+64, ...;
// the centres are read transposed (C^T, d x k, built by dkm_prepare_centers
// with DKM_PREP_CSR) so that the 64 lanes of a stored column read 512
// contiguous bytes.  Sums are added with fp64 atomics (lanes over the
// sample's stored entries).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "dkm_internal.h"

// A/B switch (variants.sh): the per-centre-group kernel for every k
#ifndef DKM_AB_CSR_OLD
#define DKM_AB_CSR_OLD 0
#endif

namespace dkm {

__global__ void __launch_bounds__(256)
    k_csr_assign(const int64_t *__restrict__ indptr,
                 const int32_t *__restrict__ indices,
                 const double *__restrict__ data, int64_t n, int d,
                 const double *__restrict__ CT, const double *__restrict__ yy,
                 int k, int32_t *labels, double *acc) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < n; i += nwaves) {
    const int64_t a = indptr[i], b = indptr[i + 1];
    double xx = 0.0;  // identical in every lane (broadcast loads)
    for (int64_t v = a; v < b; ++v) xx = xx + data[v] * data[v];
    double best = INFINITY;
    int bi = 0x7fffffff;
    for (int j = lane; j < k; j += 64) {
      double dot = 0.0;
      for (int64_t v = a; v < b; ++v)
        dot = dot + data[v] * CT[(int64_t)indices[v] * k + j];
      double dd = -2.0 * dot;
      dd = dd + xx;
      dd = dd + yy[j];
      const double dist = sqrt(dd > 0.0 ? dd : 0.0);
      if (dist < best || bi == 0x7fffffff) {
        best = dist;
        bi = j;
      }
    }
    wave_argmin(best, bi);
    if (lane == 0 && labels) labels[i] = bi;
    if (acc) {
      for (int64_t v = a + lane; v < b; v += 64)
        atomic_add_f64(acc + (int64_t)bi * d + indices[v], data[v]);
      if (lane == 0) atomic_add_f64(acc + (int64_t)k * d + bi, 1.0);
    }
  }
}

// Centres per lane known at compile time (k <= 64 * KPL): the row's stored
// entries are loaded once, 64 at a time (lane e holds entry e), and walked
// in order by readlane, so each entry's C^T row loads (512 B per 64
// centres) issue back to back instead of behind an index load per centre
// group.  Every centre's dot still runs over the entries in stored order
// (product, then add), exactly as above.
template <int KPL>
__global__ void __launch_bounds__(256)
    k_csr_assign_r(const int64_t *__restrict__ indptr,
                   const int32_t *__restrict__ indices,
                   const double *__restrict__ data, int64_t n, int d,
                   const double *__restrict__ CT, const double *__restrict__ yy,
                   int k, int32_t *labels, double *acc) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < n; i += nwaves) {
    const int64_t a = indptr[i], b = indptr[i + 1];
    double xx = 0.0;
    double dot[KPL];
#pragma unroll
    for (int g = 0; g < KPL; ++g) dot[g] = 0.0;
    for (int64_t c0 = a; c0 < b; c0 += 64) {
      const int cnt = (int)std::min<int64_t>(64, b - c0);
      int myi = 0;
      double myv = 0.0;
      if (lane < cnt) {
        myi = indices[c0 + lane];
        myv = data[c0 + lane];
      }
      const int64_t mv = __double_as_longlong(myv);
#pragma unroll 4
      for (int e = 0; e < cnt; ++e) {
        const int idx = __builtin_amdgcn_readlane(myi, e);
        const int lo = __builtin_amdgcn_readlane((int)(mv & 0xffffffff), e);
        const int hi = __builtin_amdgcn_readlane((int)(mv >> 32), e);
        const double val = __longlong_as_double(
            ((int64_t)(uint32_t)hi << 32) | (uint32_t)lo);
        xx = xx + val * val;
        const double *row = CT + (int64_t)idx * k;
#pragma unroll
        for (int g = 0; g < KPL; ++g) {
          const int j = lane + 64 * g;
          if (j < k) dot[g] = dot[g] + val * row[j];
        }
      }
    }
    double best = INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int g = 0; g < KPL; ++g) {
      const int j = lane + 64 * g;
      if (j < k) {
        double dd = -2.0 * dot[g];
        dd = dd + xx;
        dd = dd + yy[j];
        const double dist = sqrt(dd > 0.0 ? dd : 0.0);
        if (dist < best || bi == 0x7fffffff) {
          best = dist;
          bi = j;
        }
      }
    }
    wave_argmin(best, bi);
    if (lane == 0 && labels) labels[i] = bi;
    if (acc) {
      for (int64_t v = a + lane; v < b; v += 64)
        atomic_add_f64(acc + (int64_t)bi * d + indices[v], data[v]);
      if (lane == 0) atomic_add_f64(acc + (int64_t)k * d + bi, 1.0);
    }
  }
}

static int csr_assign(const int64_t *indptr, const int32_t *indices,
                      const double *data, int64_t n, int64_t d,
                      const double *C, int64_t k, const void *ws, size_t wsb,
                      int32_t *labels, double *acc, void *stream,
                      const char *who) {
  if (n < 0 || d <= 0 || k <= 0 || d > INT32_MAX || k > INT32_MAX)
    return fail(DKM_E_ARG, std::string(who) + ": bad n/d/k");
  if (n == 0) return 0;
  if (!indptr || !C || (!indices && !data))
    return fail(DKM_E_ARG, std::string(who) + ": NULL input");
  (void)C;  // the kernel reads C^T and |c|^2 prepared in the workspace
  WsView v;
  if (int r = ws_view(ws, wsb, k, d, &v)) return r;
  int dev = 0, cus = 256;
  hipDeviceProp_t p;
  if (hipGetDevice(&dev) == hipSuccess &&
      hipGetDeviceProperties(&p, dev) == hipSuccess)
    cus = p.multiProcessorCount;
  const int64_t blocks = std::min<int64_t>((n + 3) / 4, (int64_t)cus * 16);
  const unsigned g = (unsigned)std::max<int64_t>(1, blocks);
  hipStream_t s = (hipStream_t)stream;
#define DKM_CSR_R(KPL)                                                       \
  k_csr_assign_r<KPL><<<g, 256, 0, s>>>(indptr, indices, data, n, (int)d,     \
                                        v.ct64, v.cn64, (int)k, labels, acc)
  if (DKM_AB_CSR_OLD || k > 512)
    k_csr_assign<<<g, 256, 0, s>>>(indptr, indices, data, n, (int)d, v.ct64,
                                   v.cn64, (int)k, labels, acc);
  else if (k <= 64)
    DKM_CSR_R(1);
  else if (k <= 128)
    DKM_CSR_R(2);
  else if (k <= 256)
    DKM_CSR_R(4);
  else
    DKM_CSR_R(8);
#undef DKM_CSR_R
  return check_launch(who);
}

}  // namespace dkm

using namespace dkm;

extern "C" {

int dkm_partial_sum_csr_f64(const int64_t *indptr, const int32_t *indices,
                            const double *data, int64_t n, int64_t d,
                            const double *C, int64_t k, const void *ws,
                            size_t ws_bytes, int32_t *labels, double *acc,
                            void *stream) {
  if (!acc) return fail(DKM_E_ARG, "partial_sum_csr: acc is NULL");
  return csr_assign(indptr, indices, data, n, d, C, k, ws, ws_bytes, labels,
                    acc, stream, "dkm_partial_sum_csr_f64");
}

int dkm_predict_csr_f64(const int64_t *indptr, const int32_t *indices,
                        const double *data, int64_t n, int64_t d,
                        const double *C, int64_t k, const void *ws,
                        size_t ws_bytes, int32_t *labels, void *stream) {
  if (!labels) return fail(DKM_E_ARG, "predict_csr: labels is NULL");
  return csr_assign(indptr, indices, data, n, d, C, k, ws, ws_bytes, labels,
                    nullptr, stream, "dkm_predict_csr_f64");
}

}  // extern "C"
