// dkm_cand.hip -- exact resolution of the single-product screens'
// two-candidate samples (k_cand2): the reference arithmetic of
// `_vec_matrix_euclid` (dislib cluster/kmeans/base.py:204-205, numpy's
// pairwise sum of (x - c)^2, correctly rounded sqrt) on the two centres the
// screen left, first index among equal distances (np.argmin, base.py:173).
//
// The screens only list a sample here for 8 <= d <= 128 with d % 8 == 0,
// where numpy's sum is one pairwise leaf: 8 accumulators r_j = sum_i
// (x[j + 8 i] - c[j + 8 i])^2, combined as ((r0+r1)+(r2+r3))+((r4+r5)+
// (r6+r7)).  Lane (e, j) = (lane >> 3, lane & 7) keeps r_j of BOTH
// candidates of entry e: 8 entries per wave step, the sample's row read
// once (the earlier form gave each candidate its own 8 lanes and read the
// row twice, 4 entries a step), every load of a step issued before the
// first use.  The combine tree is three xor shuffles (IEEE addition is
// commutative, so both partners of a pair hold the same bits).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dkm_internal.h"

namespace dkm {

constexpr int CBLOCK = 256;

template <class TX, int NST>
__global__ void __launch_bounds__(CBLOCK)
    k_cand2(const TX *__restrict__ X, int d, int64_t ldx,
            const double *__restrict__ C, WsView v,
            int32_t *__restrict__ lab_out, int64_t base, int nseg) {
  const int64_t wv = (int64_t)blockIdx.x * (CBLOCK / 64) + (threadIdx.x >> 6);
  const int64_t nwv = (int64_t)gridDim.x * (CBLOCK / 64);
  const int lane = threadIdx.x & 63;
  const int e = lane >> 3, j = lane & 7;
  unsigned long long mine = 0;
  // (segment, 64-entry batch) pairs over all waves, batch index major
  for (int64_t L = wv; L < (int64_t)nseg * (B1_CAP / 64); L += nwv) {
    const int64_t sg = L % nseg;
    const int t0 = (int)(L / nseg) * 64;
    const int cnt = v.ccount[sg];
    if (t0 == 0 && lane == 0) mine += cnt;
    if (t0 >= cnt) continue;  // wave-uniform
    const int2 *list = v.clist + sg * B1_CAP + t0;
    const int m = min(64, cnt - t0);
    const int2 own = list[min(lane, m - 1)];  // the batch, one entry a lane
    // two 8-entry steps per pass, every load of both issued before the
    // first use (one step in flight per wave read the rows at 0.31 of HBM)
    for (int p = 0; p < m; p += 16) {
      double xv[2][NST], a[2][NST], b[2][NST];
      int64_t si[2];
      int c1[2], c2[2];
      bool live[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        live[h] = p + 8 * h + e < m;
        const int src = min(p + 8 * h + e, m - 1);
        const int sx = __shfl(own.x, src, 64), sy = __shfl(own.y, src, 64);
        c1[h] = sy & 0xffff;
        c2[h] = (int)((unsigned)sy >> 16);
        si[h] = base + sx;
        const TX *xr = X + si[h] * ldx + j;
        const double *cr1 = C + (int64_t)c1[h] * d + j;
        const double *cr2 = C + (int64_t)c2[h] * d + j;
#pragma unroll
        for (int i = 0; i < NST; ++i) {
          xv[h][i] = (double)xr[8 * i];
          a[h][i] = cr1[8 * i];
          b[h][i] = cr2[8 * i];
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double r1 = 0.0, r2 = 0.0;
#pragma unroll
        for (int i = 0; i < NST; ++i) {
          const double d1 = xv[h][i] - a[h][i], d2 = xv[h][i] - b[h][i];
          r1 = i ? r1 + d1 * d1 : d1 * d1;
          r2 = i ? r2 + d2 * d2 : d2 * d2;
        }
#pragma unroll
        for (int off = 1; off < 8; off <<= 1) {
          r1 = r1 + __shfl_xor(r1, off, 64);
          r2 = r2 + __shfl_xor(r2, off, 64);
        }
        const double q1 = argmin_key(sqrt(r1)), q2 = argmin_key(sqrt(r2));
        if (live[h] && j == 0)
          lab_out[si[h]] =
              (q2 < q1 || (q2 == q1 && c2[h] < c1[h])) ? c2[h] : c1[h];
      }
    }
  }
  if (mine) atomicAdd((unsigned long long *)&v.hdr->rechecked_total, mine);
}

template <class TX>
int launch_cand2_leaf(const TX *X, int d, int64_t ldx, const double *C,
                      const WsView &v, int32_t *lab_out, int64_t base,
                      int nseg, int cus, hipStream_t s) {
  if (d % 8 != 0 || d < 8 || d > 128) return 1;
  const int64_t units = (int64_t)nseg * (B1_CAP / 64);
  const unsigned g = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>((int64_t)cus * 8,
                           (units + CBLOCK / 64 - 1) / (CBLOCK / 64)));
  switch (d / 8) {
#define DKM_C2(N)                                                          \
  case N:                                                                  \
    k_cand2<TX, N><<<g, CBLOCK, 0, s>>>(X, d, ldx, C, v, lab_out, base,    \
                                        nseg);                             \
    break;
    DKM_C2(1) DKM_C2(2) DKM_C2(3) DKM_C2(4) DKM_C2(5) DKM_C2(6) DKM_C2(7)
    DKM_C2(8) DKM_C2(9) DKM_C2(10) DKM_C2(11) DKM_C2(12) DKM_C2(13)
    DKM_C2(14) DKM_C2(15) DKM_C2(16)
#undef DKM_C2
    default:
      return 1;
  }
  return check_launch("two-candidate re-check");
}

template int launch_cand2_leaf<double>(const double *, int, int64_t,
                                       const double *, const WsView &,
                                       int32_t *, int64_t, int, int,
                                       hipStream_t);
template int launch_cand2_leaf<float>(const float *, int, int64_t,
                                      const double *, const WsView &,
                                      int32_t *, int64_t, int, int,
                                      hipStream_t);

}  // namespace dkm

// Code-object preload (dkm_preload): the runtime loads this file's kernels
// on first use of any of them; an attribute query here does it up front.
namespace dkm {
DKM_TU_FLAGS(cand, 0)
__global__ void k_tu_cand() {}
int preload_cand() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void *)k_tu_cand) == hipSuccess ? 0
                                                                       : 1;
}
}  // namespace dkm
