// dkm_neighbors.hip -- the distance primitive reused outside the Lloyd loop
// (SURVEY.md 8 f4).
//
// * kNN: NearestNeighbors.kneighbors (reference neighbors/base.py:40-87).
//   The reference fits sklearn NearestNeighbors on every fit Subset, queries
//   it with every query Subset and merges the per-pair k-lists by sort.
//   sklearn's kd_tree (its choice for d <= 15) ranks by the sequential
//   squared sum  r = 0; r += (q_t - x_t)^2  (EuclideanDistance.rdist, no
//   FMA) and reports sqrt(r).  Here one brute-force pass over the whole fit
//   set computes that same r for every (query, fit row) pair and keeps the
//   k smallest by (r, index):
//     k_knn_part   lane = query (its row in VGPRs), wave-uniform fit row j
//                  read by scalar loads (constant address space: SGPRs, no
//                  LDS broadcast), fit rows cut into P partitions so that
//                  (queries / 64) x P waves fill the chip; a per-lane sorted
//                  top-K (K = 1..32, registers, unrolled insertion network
//                  entered only by lanes whose r beats their K-th).
//     k_knn_merge  lane = query: the P partial lists merged by (r, index),
//                  sqrt, int64 indices.
//   n_neighbors > 32: passes of up to 32 columns; pass c starts strictly
//   after the (r, index) where pass c - 1 ended (a per-query floor), so the
//   passes enumerate the same (r, index) order, 32 entries at a time.
//   Roofline: VALU fp64 -- 3 d ops (sub, mul, add) per pair.
//   CSR Subsets: k_knn_csr_part, the same partitions and merge over the
//   k_radius_csr intersection arithmetic (sklearn's brute force on CSR).
//
// * Epsilon query: DBSCAN _compute_neighbours (reference
//   cluster/dbscan/classes.py:124-141): for each query row, every row with
//   _vec_matrix_euclid distance < eps (numpy's pairwise order, the k-means
//   exact arithmetic of dkm_internal.h), sorted by distance.
//     k_radius<PASS> lane = query, fit rows partitioned over waves; pass 0
//                  counts (int64 atomics per lane-partition), pass 1 writes
//                  (index, distance) at an atomically advanced cursor;
//     k_seg_sort   block per query list: (distance, index) ascending --
//                  bitonic in LDS up to 4096 entries; beyond, sorted runs
//                  of 4096 merged pairwise through workspace scratch.
#include "dkm_internal.h"

#include <algorithm>
#include <cmath>

namespace dkm {

namespace {

constexpr int NB = 256;  // threads per block (4 waves)
typedef const __attribute__((address_space(4))) double cdouble;

// ---------------------------------------------------------------------------
// kNN
// ---------------------------------------------------------------------------
// Ranking key of a squared distance r >= 0: its bit pattern (monotonic for
// non-negative doubles; -0.0 folded onto +0.0), NaN after +inf as sklearn's
// argpartition ranks it (data overflowing to inf - inf), and the empty slot
// after every real row, so every list fills with real rows.
constexpr uint64_t KEY_NAN = 0x7ff8000000000000ull;
constexpr uint64_t KEY_EMPTY = ~0ull;
__device__ __forceinline__ uint64_t rkey(double r) {
  return r != r ? KEY_NAN : (uint64_t)__double_as_longlong(r + 0.0);
}
__device__ __forceinline__ double key_r(uint64_t key) {
  return key == KEY_EMPTY ? INFINITY : __longlong_as_double((long long)key);
}

template <int K>
struct TopK {
  uint64_t r[K];
  int i[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int s = 0; s < K; ++s) {
      r[s] = KEY_EMPTY;
      i[s] = INT32_MAX;
    }
  }
  // (v, j) by lexicographic (key, index).  The comparison stays
  // lexicographic for the entry carried down the list after a swap: a
  // displaced (r, i) must still go ahead of a held (r, i') with i < i' (a
  // "strict <, empty slots take ties" rule for scan-order pushes drops it
  // instead).
  __device__ __forceinline__ bool before_last(uint64_t v, int j) const {
    return v < r[K - 1] || (v == r[K - 1] && j < i[K - 1]);
  }
  __device__ __forceinline__ void push(uint64_t v, int j) {
    if (before_last(v, j)) {
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const bool lt = v < r[s] || (v == r[s] && j < i[s]);
        const uint64_t tr = r[s];
        const int ti = i[s];
        r[s] = lt ? v : tr;
        i[s] = lt ? j : ti;
        v = lt ? tr : v;
        j = lt ? ti : j;
      }
    }
  }
};

// Sequential squared distance of a register-resident query to fit row xr
// (wave-uniform: scalar loads).  MAXD = 0: the query is read from global.
template <int MAXD>
__device__ __forceinline__ double seq_r(const double (&q)[MAXD > 0 ? MAXD : 1],
                                        const double *qg, cdouble *xr, int d) {
  double r = 0.0;
  if constexpr (MAXD > 0) {
#pragma unroll
    for (int t = 0; t < MAXD; ++t)
      if (t < d) {
        const double df = q[t] - xr[t];
        r = r + df * df;
      }
  } else {
    for (int t = 0; t < d; ++t) {
      const double df = qg[t] - xr[t];
      r = r + df * df;
    }
  }
  return r;
}

template <int MAXD, int K>
__global__ void __launch_bounds__(NB)
    k_knn_part(const double *__restrict__ Q, int64_t nq, int64_t ldq,
               const double *__restrict__ X, int64_t nx, int64_t ldx, int d,
               int64_t plen, int P, double *__restrict__ pr,
               int *__restrict__ pi, const double *__restrict__ flr,
               const int *__restrict__ fli) {
  const int lane = threadIdx.x & 63;
  const int64_t qg = (int64_t)blockIdx.x * (NB / 64) +
                     __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = blockIdx.y;
  const int64_t q = qg * 64 + lane;
  if (qg * 64 >= nq) return;  // wave-uniform
  const bool live = q < nq;
  const double *qrow = Q + (live ? q : 0) * ldq;
  double qv[MAXD > 0 ? MAXD : 1];
  if constexpr (MAXD > 0) {
#pragma unroll
    for (int t = 0; t < MAXD; ++t) qv[t] = t < d ? qrow[t] : 0.0;
  }
  TopK<K> top;
  top.init();
  const int64_t j0 = (int64_t)p * plen;
  const int64_t j1 = std::min<int64_t>(nx, j0 + plen);
  cdouble *xc = (cdouble *)X;
  if (flr) {
    // a later pass: only (r, j) strictly after the previous pass's last
    const uint64_t fr = live ? (uint64_t)__double_as_longlong(flr[q])
                             : KEY_EMPTY;
    const int fi = live ? fli[q] : INT32_MAX;
    for (int64_t j = j0; j < j1; ++j) {
      const uint64_t r = rkey(seq_r<MAXD>(qv, qrow, xc + j * ldx, d));
      if (r > fr || (r == fr && (int)j > fi)) top.push(r, (int)j);
    }
  } else {
    for (int64_t j = j0; j < j1; ++j)
      top.push(rkey(seq_r<MAXD>(qv, qrow, xc + j * ldx, d)), (int)j);
  }
  if (!live) return;
  double *po = pr + (q * P + p) * K;
  int *io = pi + (q * P + p) * K;
#pragma unroll
  for (int s = 0; s < K; ++s) {  // keys, as bits in the partial buffer
    po[s] = __longlong_as_double((long long)top.r[s]);
    io[s] = top.i[s];
  }
}

// sklearn's squared CSR distance of query row [qa, qb) (|q|^2 = xx) to fit
// row j, clamped at 0 (the arithmetic of the comment below).
__device__ __forceinline__ double csr_pair_r(
    int64_t qa, int64_t qb, const int32_t *__restrict__ qi,
    const double *__restrict__ qd, double xx, const int64_t *__restrict__ xp,
    const int32_t *__restrict__ xi, const double *__restrict__ xd, int64_t j,
    int f32) {
  const int64_t a = xp[j], b = xp[j + 1];
  double yy = 0.0, dot = 0.0;
  int64_t t = qa;
  int32_t qc = t < qb ? qi[t] : INT32_MAX;
  for (int64_t u = a; u < b; ++u) {
    const int32_t c = xi[u];
    const double v = xd[u];
    yy += v * v;
    while (qc < c) {
      ++t;
      qc = t < qb ? qi[t] : INT32_MAX;
    }
    if (qc == c) dot += qd[t] * v;
  }
  double r = -2.0 * dot;
  r += xx;
  r += yy;
  if (f32) {  // float32 Subsets: the squares rounded to float32 first
    const float r32 = (float)r;
    return r32 < 0.f ? 0.0 : (double)r32;
  }
  return r < 0.0 ? 0.0 : r;
}

// Sparse kNN partial lists.  sklearn picks brute force for CSR fit data and,
// its ArgKmin reduction refusing sparse-sparse pairs, ranks by
// pairwise_distances_chunked(squared=True): r = max(((-2 q.x) + ||q||^2) +
// ||x||^2, 0) in the arithmetic of k_radius_csr below (row norms summed in
// stored order, q.x in the query's stored = increasing-column order), then
// sqrt(r).  The self pair is exactly 0 (q.q and ||q||^2 are the same sum).
// lane = query row (its merge cursor), wave-uniform fit row j (scalar
// loads), fit rows partitioned over blockIdx.y like k_knn_part.
template <int K>
__global__ void __launch_bounds__(NB)
    k_knn_csr_part(const int64_t *__restrict__ qp,
                   const int32_t *__restrict__ qi,
                   const double *__restrict__ qd, int64_t nq,
                   const int64_t *__restrict__ xp,
                   const int32_t *__restrict__ xi,
                   const double *__restrict__ xd, int64_t nx, int64_t plen,
                   int P, int f32, double *__restrict__ pr,
                   int *__restrict__ pi, const double *__restrict__ flr,
                   const int *__restrict__ fli) {
  const int lane = threadIdx.x & 63;
  const int64_t qg = (int64_t)blockIdx.x * (NB / 64) +
                     __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = blockIdx.y;
  const int64_t q = qg * 64 + lane;
  if (qg * 64 >= nq) return;  // wave-uniform
  const bool live = q < nq;
  const int64_t qa = live ? qp[q] : 0;
  const int64_t qb = live ? qp[q + 1] : 0;
  double xx = 0.0;
  for (int64_t t = qa; t < qb; ++t) {
    const double v = qd[t];
    xx += v * v;
  }
  const uint64_t fr =
      (live && flr) ? (uint64_t)__double_as_longlong(flr[q]) : 0;
  const int fi = (live && fli) ? fli[q] : -1;
  TopK<K> top;
  top.init();
  const int64_t j0 = (int64_t)p * plen;
  const int64_t j1 = std::min<int64_t>(nx, j0 + plen);
  for (int64_t j = j0; j < j1; ++j) {
    // (finite data whose squares overflow: inf - inf = NaN, ranked after
    // +inf).  A later pass: only (r, j) strictly after the previous pass's
    // last.
    const uint64_t rk = rkey(csr_pair_r(qa, qb, qi, qd, xx, xp, xi, xd, j,
                                        f32));
    if (rk > fr || (rk == fr && (int)j > fi)) top.push(rk, (int)j);
  }
  if (!live) return;
  double *po = pr + (q * P + p) * K;
  int *io = pi + (q * P + p) * K;
#pragma unroll
  for (int s = 0; s < K; ++s) {
    po[s] = __longlong_as_double((long long)top.r[s]);
    io[s] = top.i[s];
  }
}

template <int K>
__global__ void __launch_bounds__(NB)
    k_knn_merge(const double *__restrict__ pr, const int *__restrict__ pi,
                int64_t nq, int P, int kn, double *__restrict__ out_d,
                int64_t *__restrict__ out_i, int64_t ldo,
                double *__restrict__ flr, int *__restrict__ fli, int f32) {
  const int64_t q = (int64_t)blockIdx.x * NB + threadIdx.x;
  if (q >= nq) return;
  TopK<K> top;
  top.init();
  for (int p = 0; p < P; ++p) {
    const double *a = pr + (q * P + p) * K;
    const int *b = pi + (q * P + p) * K;
    for (int s = 0; s < kn; ++s) {
      const uint64_t v = (uint64_t)__double_as_longlong(a[s]);
      if (!top.before_last(v, b[s]))
        break;  // the partition's list is sorted: nothing further enters
      top.push(v, b[s]);
    }
  }
#pragma unroll
  for (int s = 0; s < K; ++s)
    if (s < kn) {
      const double r = key_r(top.r[s]);
      // f32: r is a float32 value; the fp64 sqrt rounds to float32's own
      out_d[q * ldo + s] = f32 ? (double)(float)sqrt(r) : sqrt(r);
      out_i[q * ldo + s] = (int64_t)top.i[s];
      if (s == kn - 1) {  // where the next pass starts (a key)
        flr[q] = __longlong_as_double((long long)top.r[s]);
        fli[q] = top.i[s];
      }
    }
}

// ---------------------------------------------------------------------------
// kNN beyond 32 neighbours in two scans (32 < kn <= KB_KN_MAX).
//   scan 1  k_knn_part / k_knn_csr_part with K = 32 over Pb >= kn/32 + 1
//           partitions: per query, Pb sorted lists of 32.
//   k_knn_thresh  block per query: the kn-th smallest (key, index) of the
//           union of those lists.  The union is a subset of the fit rows, so
//           this is an upper bound (tk, ti) of the true kn-th pair.
//   scan 2  k_knn_cand / k_knn_csr_cand: the same pair arithmetic; every
//           (key, j) <= (tk, ti) is appended to the query's candidate list
//           (per-lane atomics on the lane's own counter: about kn appends per
//           query over the whole scan).
//   k_knn_final  block per query: bitonic sort of the candidates in LDS by
//           (key, index), the first kn written out.  A list longer than
//           KB_CAP raises a flag and the host reruns the call in passes of 32.
// Two scans of nq x nx pairs instead of ceil(kn / 32) (kn = 1000: 32).
// ---------------------------------------------------------------------------
constexpr int KB_CAP = 4096;      // candidates per query (LDS sort)
constexpr int KB_KN_MAX = 2048;   // kn this path takes
constexpr int KB_P_MAX = KB_CAP / 32;
constexpr int64_t KB_QC = 8192;   // queries per chunk (workspace bound)

__device__ __forceinline__ bool key_le(uint64_t a, int ia, uint64_t b,
                                       int ib) {
  return a < b || (a == b && ia <= ib);
}

// Bitonic sort of n <= KB_CAP (key, index) pairs in LDS, ascending.
__device__ void lds_sort_keys(uint64_t *sk, int *si, int n) {
  int p2 = 2;
  while (p2 < n) p2 <<= 1;
  for (int e = n + threadIdx.x; e < p2; e += NB) {
    sk[e] = KEY_EMPTY;
    si[e] = INT32_MAX;
  }
  __syncthreads();
  for (int size = 2; size <= p2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int e = threadIdx.x; e < p2; e += NB) {
        const int f = e ^ stride;
        if (f > e) {
          const bool up = (e & size) == 0;
          const bool gt = !key_le(sk[e], si[e], sk[f], si[f]);
          if (gt == up) {
            const uint64_t tk = sk[e];
            sk[e] = sk[f];
            sk[f] = tk;
            const int ti = si[e];
            si[e] = si[f];
            si[f] = ti;
          }
        }
      }
      __syncthreads();
    }
}

__global__ void __launch_bounds__(NB)
    k_knn_thresh(const double *__restrict__ pr, const int *__restrict__ pi,
                 int64_t nq, int P, int kn, uint64_t *__restrict__ thk,
                 int *__restrict__ thi, unsigned *__restrict__ cc) {
  __shared__ uint64_t sk[KB_CAP];
  __shared__ int si[KB_CAP];
  const int64_t q = blockIdx.x;
  if (q >= nq) return;
  const int m = P * 32;
  for (int e = threadIdx.x; e < m; e += NB) {
    sk[e] = (uint64_t)__double_as_longlong(pr[q * m + e]);
    si[e] = pi[q * m + e];
  }
  lds_sort_keys(sk, si, m);
  if (threadIdx.x == 0) {
    thk[q] = sk[kn - 1];
    thi[q] = si[kn - 1];
    cc[q] = 0;
  }
}

template <int MAXD>
__global__ void __launch_bounds__(NB)
    k_knn_cand(const double *__restrict__ Q, int64_t nq, int64_t ldq,
               const double *__restrict__ X, int64_t nx, int64_t ldx, int d,
               int64_t plen, const uint64_t *__restrict__ thk,
               const int *__restrict__ thi, unsigned *__restrict__ cc,
               uint64_t *__restrict__ ck, int *__restrict__ ci) {
  const int lane = threadIdx.x & 63;
  const int64_t qg = (int64_t)blockIdx.x * (NB / 64) +
                     __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t q = qg * 64 + lane;
  if (qg * 64 >= nq) return;  // wave-uniform
  const bool live = q < nq;
  const double *qrow = Q + (live ? q : 0) * ldq;
  double qv[MAXD > 0 ? MAXD : 1];
  if constexpr (MAXD > 0) {
#pragma unroll
    for (int t = 0; t < MAXD; ++t) qv[t] = t < d ? qrow[t] : 0.0;
  }
  const uint64_t tk = live ? thk[q] : 0;
  const int ti = live ? thi[q] : -1;
  const int64_t j0 = (int64_t)blockIdx.y * plen;
  const int64_t j1 = std::min<int64_t>(nx, j0 + plen);
  cdouble *xc = (cdouble *)X;
  for (int64_t j = j0; j < j1; ++j) {
    const uint64_t r = rkey(seq_r<MAXD>(qv, qrow, xc + j * ldx, d));
    if (live && key_le(r, (int)j, tk, ti)) {
      const unsigned pos = atomicAdd(cc + q, 1u);
      if (pos < (unsigned)KB_CAP) {
        ck[q * KB_CAP + pos] = r;
        ci[q * KB_CAP + pos] = (int)j;
      }
    }
  }
}

__global__ void __launch_bounds__(NB)
    k_knn_csr_cand(const int64_t *__restrict__ qp,
                   const int32_t *__restrict__ qi,
                   const double *__restrict__ qd, int64_t nq,
                   const int64_t *__restrict__ xp,
                   const int32_t *__restrict__ xi,
                   const double *__restrict__ xd, int64_t nx, int64_t plen,
                   int f32, const uint64_t *__restrict__ thk,
                   const int *__restrict__ thi, unsigned *__restrict__ cc,
                   uint64_t *__restrict__ ck, int *__restrict__ ci) {
  const int lane = threadIdx.x & 63;
  const int64_t qg = (int64_t)blockIdx.x * (NB / 64) +
                     __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t q = qg * 64 + lane;
  if (qg * 64 >= nq) return;  // wave-uniform
  const bool live = q < nq;
  const int64_t qa = live ? qp[q] : 0;
  const int64_t qb = live ? qp[q + 1] : 0;
  double xx = 0.0;
  for (int64_t t = qa; t < qb; ++t) {
    const double v = qd[t];
    xx += v * v;
  }
  const uint64_t tk = live ? thk[q] : 0;
  const int ti = live ? thi[q] : -1;
  const int64_t j0 = (int64_t)blockIdx.y * plen;
  const int64_t j1 = std::min<int64_t>(nx, j0 + plen);
  for (int64_t j = j0; j < j1; ++j) {
    const uint64_t r =
        rkey(csr_pair_r(qa, qb, qi, qd, xx, xp, xi, xd, j, f32));
    if (live && key_le(r, (int)j, tk, ti)) {
      const unsigned pos = atomicAdd(cc + q, 1u);
      if (pos < (unsigned)KB_CAP) {
        ck[q * KB_CAP + pos] = r;
        ci[q * KB_CAP + pos] = (int)j;
      }
    }
  }
}

__global__ void __launch_bounds__(NB)
    k_knn_final(const unsigned *__restrict__ cc,
                const uint64_t *__restrict__ ck, const int *__restrict__ ci,
                int64_t nq, int kn, double *__restrict__ out_d,
                int64_t *__restrict__ out_i, int64_t ldo, int f32,
                unsigned *__restrict__ overflow) {
  __shared__ uint64_t sk[KB_CAP];
  __shared__ int si[KB_CAP];
  const int64_t q = blockIdx.x;
  if (q >= nq) return;
  const unsigned c = cc[q];
  if (c > (unsigned)KB_CAP) {  // block-uniform
    if (threadIdx.x == 0) atomicOr(overflow, 1u);
    return;
  }
  const int m = (int)c;  // >= kn: the threshold pair and all before it
  for (int e = threadIdx.x; e < m; e += NB) {
    sk[e] = ck[q * KB_CAP + e];
    si[e] = ci[q * KB_CAP + e];
  }
  lds_sort_keys(sk, si, m);
  for (int e = threadIdx.x; e < kn; e += NB) {
    const double r = key_r(sk[e]);
    out_d[q * ldo + e] = f32 ? (double)(float)sqrt(r) : sqrt(r);
    out_i[q * ldo + e] = (int64_t)si[e];
  }
}

// ---------------------------------------------------------------------------
// epsilon query
// ---------------------------------------------------------------------------
template <int MAXD, int PASS>
__global__ void __launch_bounds__(NB)
    k_radius(const double *__restrict__ Q, int64_t nq, int64_t ldq,
             const double *__restrict__ X, int64_t nx, int64_t ldx, int d,
             double eps, int64_t plen, unsigned long long *__restrict__ cnt,
             int64_t *__restrict__ out_i, double *__restrict__ out_d) {
  const int lane = threadIdx.x & 63;
  const int64_t qg = (int64_t)blockIdx.x * (NB / 64) +
                     __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = blockIdx.y;
  const int64_t q = qg * 64 + lane;
  if (qg * 64 >= nq) return;
  const bool live = q < nq;
  const double *qrow = Q + (live ? q : 0) * ldq;
  double qv[MAXD > 0 ? MAXD : 8];
  if constexpr (MAXD > 0) {
#pragma unroll
    for (int t = 0; t < MAXD; ++t) qv[t] = t < d ? qrow[t] : 0.0;
  }
  const int64_t j0 = (int64_t)p * plen;
  const int64_t j1 = std::min<int64_t>(nx, j0 + plen);
  cdouble *xc = (cdouble *)X;
  const double e2 = eps * eps;
  // eps <= 0: sqrt(r) >= 0 is never below it (and eps^2 would be > 0)
  const double e2lo = eps > 0 ? e2 * (1.0 - 0x1.0p-48) : -1.0;
  const double e2hi = eps > 0 ? e2 * (1.0 + 0x1.0p-48) : -1.0;
  unsigned long long mine = 0;
  for (int64_t j = j0; j < j1; ++j) {
    double r;
    if constexpr (MAXD > 0)
      r = exact_sqdist_reg<MAXD>(qv, xc + j * ldx, d);
    else
      r = pw_sum(SqDiff<double>{qrow, X + j * ldx}, d);
    // _vec_matrix_euclid computes row - sample; (a - b)^2 == (b - a)^2.
    // sqrt(r) < eps is decided on r where r is clear of eps^2 by a relative
    // 2^-48 (far beyond the rounding of eps^2 and of the correctly rounded
    // sqrt); the band between takes the reference's sqrt and compare.
    const bool in = r < e2lo || (r <= e2hi && sqrt(r) < eps);
    if (live && in) {
      const double dist = sqrt(r);
      if constexpr (PASS == 0) {
        ++mine;
      } else {
        const unsigned long long at = atomicAdd(cnt + q, 1ull);
        out_i[at] = j;
        out_d[at] = dist;
      }
      (void)dist;
    }
  }
  if constexpr (PASS == 0)
    if (live && mine) atomicAdd(cnt + q, mine);
}

// Sparse epsilon query (the reference's `pairwise_distances` branch of
// _compute_neighbours, cluster/dbscan/classes.py:130).  sklearn 1.7's
// _euclidean_distances for fp64 CSR computes
//   r = ((-2 * q.x) + ||q||^2) + ||x||^2,  max(r, 0),  sqrt
// with the row norms summed in stored order (_sqeuclidean_row_norms_sparse)
// and q.x by scipy's csr_matmat: products q_c * x_c accumulated from 0 in
// the order of q's stored entries.  With sorted indices that is the
// increasing-column order of the intersection, which a merge of the two
// sorted rows visits.  One lane per query row; the fit row is wave-uniform
// (scalar loads), the lane's merge cursor walks its own query row.
template <int PASS>
__global__ void __launch_bounds__(NB)
    k_radius_csr(const int64_t *__restrict__ indptr,
                 const int32_t *__restrict__ indices,
                 const double *__restrict__ data, int64_t q0, int64_t nq,
                 int64_t nx, double eps, int64_t plen, int f32,
                 unsigned long long *__restrict__ cnt,
                 int64_t *__restrict__ out_i, double *__restrict__ out_d) {
  const int lane = threadIdx.x & 63;
  const int64_t qg = (int64_t)blockIdx.x * (NB / 64) +
                     __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = blockIdx.y;
  const int64_t q = qg * 64 + lane;
  if (qg * 64 >= nq) return;
  const bool live = q < nq;
  const float eps32 = (float)eps;  // numpy compares float32 in float32
  const int64_t qa = live ? indptr[q0 + q] : 0;
  const int64_t qb = live ? indptr[q0 + q + 1] : 0;
  double xx = 0.0;
  for (int64_t t = qa; t < qb; ++t) {
    const double v = data[t];
    xx += v * v;
  }
  const int64_t j0 = (int64_t)p * plen;
  const int64_t j1 = std::min<int64_t>(nx, j0 + plen);
  const double e2 = eps * eps;
  const double e2lo = eps > 0 ? e2 * (1.0 - 0x1.0p-48) : -1.0;
  const double e2hi = eps > 0 ? e2 * (1.0 + 0x1.0p-48) : -1.0;
  unsigned long long mine = 0;
  for (int64_t j = j0; j < j1; ++j) {
    const int64_t a = indptr[j], b = indptr[j + 1];
    double yy = 0.0, dot = 0.0;
    int64_t t = qa;
    int32_t qc = t < qb ? indices[t] : INT32_MAX;
    for (int64_t u = a; u < b; ++u) {
      const int32_t c = indices[u];
      const double v = data[u];
      yy += v * v;
      while (qc < c) {
        ++t;
        qc = t < qb ? indices[t] : INT32_MAX;
      }
      if (qc == c) dot += data[t] * v;
    }
    double r = -2.0 * dot;
    r += xx;
    r += yy;
    double dist;
    bool in;
    if (f32) {
      // float32 Subsets: sklearn's upcast path rounds the fp64 squares to
      // float32, then max and sqrt in float32 (correctly rounded: the fp64
      // sqrt of a float rounds to the float32 sqrt)
      float r32 = (float)r;
      r32 = r32 < 0.f ? 0.f : r32;
      const float d32 = (float)sqrt((double)r32);
      dist = d32;
      in = d32 < eps32;
    } else {
      r = r < 0.0 ? 0.0 : r;  // np.maximum(r, 0): NaN stays NaN
      dist = sqrt(r);
      in = r < e2lo || (r <= e2hi && dist < eps);
    }
    if (live && in) {
      if constexpr (PASS == 0) {
        ++mine;
      } else {
        const unsigned long long at = atomicAdd(cnt + q, 1ull);
        out_i[at] = j;
        out_d[at] = dist;
      }
    }
  }
  if constexpr (PASS == 0)
    if (live && mine) atomicAdd(cnt + q, mine);
}

constexpr int SORT_CAP = 4096;

__device__ __forceinline__ bool key_lt(double da, int64_t ia, double db,
                                       int64_t ib) {
  return da < db || (da == db && ia < ib);
}

__global__ void __launch_bounds__(NB)
    k_seg_sort(const int64_t *__restrict__ offsets, int64_t nq,
               int64_t *__restrict__ idx, double *__restrict__ dist,
               int64_t *__restrict__ sidx, double *__restrict__ sdist) {
  __shared__ double sd[SORT_CAP];
  __shared__ int64_t si[SORT_CAP];
  const int64_t q = blockIdx.x;
  if (q >= nq) return;
  const int64_t o = offsets[q];
  const int64_t m = offsets[q + 1] - o;
  if (m <= 1) return;
  if (m <= SORT_CAP) {
    int p2 = 2;
    while (p2 < m) p2 <<= 1;
    for (int e = threadIdx.x; e < p2; e += NB) {
      sd[e] = e < m ? dist[o + e] : INFINITY;
      si[e] = e < m ? idx[o + e] : INT64_MAX;
    }
    __syncthreads();
    for (int size = 2; size <= p2; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int e = threadIdx.x; e < p2; e += NB) {
          const int f = e ^ stride;
          if (f > e) {
            const bool up = (e & size) == 0;
            const bool gt = key_lt(sd[f], si[f], sd[e], si[e]);
            if (gt == up) {
              const double td = sd[e];
              sd[e] = sd[f];
              sd[f] = td;
              const int64_t ti = si[e];
              si[e] = si[f];
              si[f] = ti;
            }
          }
        }
        __syncthreads();
      }
    for (int e = threadIdx.x; e < m; e += NB) {
      dist[o + e] = sd[e];
      idx[o + e] = si[e];
    }
    return;
  }
  // beyond LDS: sort runs of SORT_CAP in LDS (bitonic, written back in
  // place), then merge run pairs through the scratch copy: an entry's
  // place in the merged run = its place in its own run + the count of the
  // other run's keys below it (binary search; keys are distinct since the
  // indices are).  O(m log^2 m) per list instead of the rank sort's O(m^2)
  // (a dense epsilon-ball of 1e5 neighbours was 1e10 comparisons).
  for (int64_t c0 = 0; c0 < m; c0 += SORT_CAP) {
    const int mc = (int)std::min<int64_t>(SORT_CAP, m - c0);
    int p2 = 2;
    while (p2 < mc) p2 <<= 1;
    __syncthreads();
    for (int e = threadIdx.x; e < p2; e += NB) {
      sd[e] = e < mc ? dist[o + c0 + e] : INFINITY;
      si[e] = e < mc ? idx[o + c0 + e] : INT64_MAX;
    }
    __syncthreads();
    for (int size = 2; size <= p2; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int e = threadIdx.x; e < p2; e += NB) {
          const int f = e ^ stride;
          if (f > e) {
            const bool up = (e & size) == 0;
            const bool gt = key_lt(sd[f], si[f], sd[e], si[e]);
            if (gt == up) {
              const double td = sd[e];
              sd[e] = sd[f];
              sd[f] = td;
              const int64_t ti = si[e];
              si[e] = si[f];
              si[f] = ti;
            }
          }
        }
        __syncthreads();
      }
    for (int e = threadIdx.x; e < mc; e += NB) {
      dist[o + c0 + e] = sd[e];
      idx[o + c0 + e] = si[e];
    }
  }
  __syncthreads();
  double *sdd = dist + o, *ddd = sdist + o;
  int64_t *sii = idx + o, *dii = sidx + o;
  for (int64_t run = SORT_CAP; run < m; run <<= 1) {
    for (int64_t e = threadIdx.x; e < m; e += NB) {
      const int64_t lo = e / (2 * run) * (2 * run);
      const int64_t mid = std::min(lo + run, m), hi = std::min(lo + 2 * run, m);
      const double de = sdd[e];
      const int64_t ie = sii[e];
      // the other run of the pair, and the count of its keys below (e)
      const bool first = e < mid;
      int64_t a = first ? mid : lo, b = first ? hi : mid;
      while (a < b) {
        const int64_t c = (a + b) >> 1;
        if (key_lt(sdd[c], sii[c], de, ie))
          a = c + 1;
        else
          b = c;
      }
      const int64_t pos = first ? e + (a - mid) : (e - mid) + lo + (a - lo);
      ddd[pos] = de;
      dii[pos] = ie;
    }
    __syncthreads();
    double *td = sdd;
    sdd = ddd;
    ddd = td;
    int64_t *ti = sii;
    sii = dii;
    dii = ti;
  }
  if (sdd != dist + o) {  // the sorted list ended in the scratch copy
    for (int64_t e = threadIdx.x; e < m; e += NB) {
      dist[o + e] = sdd[e];
      idx[o + e] = sii[e];
    }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
int knn_k(int64_t kn) {
  int K = 1;
  while (K < kn) K <<= 1;
  return K;
}

int maxd_of(int64_t d) {
  return d <= 8 ? 8 : d <= 16 ? 16 : d <= 32 ? 32 : d <= 64 ? 64 : 0;
}

// waves = groups x P >= 4096 (16 per CU of 256; a fixed target, so the
// workspace size does not depend on the device); partitions no shorter than
// 256 rows
void knn_grid(int64_t nq, int64_t nx, int64_t *plen, int *P) {
  const int64_t groups = (nq + 63) / 64;
  const int64_t want = 4096;
  int64_t p = std::max<int64_t>(1, (want + groups - 1) / groups);
  p = std::min<int64_t>(p, std::max<int64_t>(1, nx / 256));
  p = std::min<int64_t>(p, 65535);
  *plen = (nx + p - 1) / p;
  *P = (int)((nx + *plen - 1) / *plen);
}

template <int MAXD, int K>
void launch_knn_part(dim3 g, hipStream_t s, const double *Q, int64_t nq,
                     int64_t ldq, const double *X, int64_t nx, int64_t ldx,
                     int d, int64_t plen, int P, double *pr, int *pi,
                     const double *flr, const int *fli) {
  k_knn_part<MAXD, K><<<g, NB, 0, s>>>(Q, nq, ldq, X, nx, ldx, d, plen, P, pr,
                                       pi, flr, fli);
}

template <int K>
int knn_dispatch(int maxd, dim3 g, hipStream_t s, const double *Q, int64_t nq,
                 int64_t ldq, const double *X, int64_t nx, int64_t ldx, int d,
                 int64_t plen, int P, double *pr, int *pi, const double *flr,
                 const int *fli) {
  switch (maxd) {
    case 8: launch_knn_part<8, K>(g, s, Q, nq, ldq, X, nx, ldx, d, plen, P, pr, pi, flr, fli); break;
    case 16: launch_knn_part<16, K>(g, s, Q, nq, ldq, X, nx, ldx, d, plen, P, pr, pi, flr, fli); break;
    case 32: launch_knn_part<32, K>(g, s, Q, nq, ldq, X, nx, ldx, d, plen, P, pr, pi, flr, fli); break;
    case 64: launch_knn_part<64, K>(g, s, Q, nq, ldq, X, nx, ldx, d, plen, P, pr, pi, flr, fli); break;
    default: launch_knn_part<0, K>(g, s, Q, nq, ldq, X, nx, ldx, d, plen, P, pr, pi, flr, fli); break;
  }
  return check_launch("knn partial lists");
}

template <int K>
int knn_csr_launch(dim3 g, hipStream_t s, const int64_t *qp,
                   const int32_t *qi, const double *qd, int64_t nq,
                   const int64_t *xp, const int32_t *xi, const double *xd,
                   int64_t nx, int64_t plen, int P, int f32, double *pr,
                   int *pi, const double *flr, const int *fli) {
  k_knn_csr_part<K><<<g, NB, 0, s>>>(qp, qi, qd, nq, xp, xi, xd, nx, plen, P,
                                     f32, pr, pi, flr, fli);
  return check_launch("knn csr partial lists");
}

// the merge of one pass (K = slots of the partial lists, kk <= K columns
// of out starting at c0)
int knn_merge_launch(int K, hipStream_t s, const double *pr, const int *pi,
                     int64_t nq, int P, int kk, double *od, int64_t *oi,
                     int64_t ldo, double *flr, int *fli, int f32) {
  const unsigned gm = (unsigned)((nq + NB - 1) / NB);
  switch (K) {
    case 1: k_knn_merge<1><<<gm, NB, 0, s>>>(pr, pi, nq, P, kk, od, oi, ldo, flr, fli, f32); break;
    case 2: k_knn_merge<2><<<gm, NB, 0, s>>>(pr, pi, nq, P, kk, od, oi, ldo, flr, fli, f32); break;
    case 4: k_knn_merge<4><<<gm, NB, 0, s>>>(pr, pi, nq, P, kk, od, oi, ldo, flr, fli, f32); break;
    case 8: k_knn_merge<8><<<gm, NB, 0, s>>>(pr, pi, nq, P, kk, od, oi, ldo, flr, fli, f32); break;
    case 16: k_knn_merge<16><<<gm, NB, 0, s>>>(pr, pi, nq, P, kk, od, oi, ldo, flr, fli, f32); break;
    default: k_knn_merge<32><<<gm, NB, 0, s>>>(pr, pi, nq, P, kk, od, oi, ldo, flr, fli, f32); break;
  }
  return check_launch("knn merge");
}

int knn_args(const double *Q, int64_t nq, int64_t ldq, const double *X,
             int64_t nx, int64_t ldx, int64_t d, int64_t kn) {
  if (nq < 0 || nx < 1 || d < 1 || ldq < d || ldx < d)
    return fail(DKM_E_ARG, "knn: bad nq/nx/d/ld");
  if (kn < 1 || kn > nx)
    return fail(DKM_E_ARG, "knn: n_neighbors must be in [1, nx]");
  if (nx > INT32_MAX || d > INT32_MAX)
    return fail(DKM_E_ARG, "knn: nx/d too large");
  if (nq > 0 && (!Q || !X)) return fail(DKM_E_ARG, "knn: NULL Q/X");
  return 0;
}

template <int MAXD, int PASS>
void launch_radius(dim3 g, hipStream_t s, const double *Q, int64_t nq,
                   int64_t ldq, const double *X, int64_t nx, int64_t ldx,
                   int d, double eps, int64_t plen, unsigned long long *cnt,
                   int64_t *oi, double *od) {
  k_radius<MAXD, PASS><<<g, NB, 0, s>>>(Q, nq, ldq, X, nx, ldx, d, eps, plen,
                                        cnt, oi, od);
}

template <int PASS>
int radius_dispatch(int64_t d, dim3 g, hipStream_t s, const double *Q,
                    int64_t nq, int64_t ldq, const double *X, int64_t nx,
                    int64_t ldx, double eps, int64_t plen,
                    unsigned long long *cnt, int64_t *oi, double *od) {
  const int di = (int)d;
  // d <= 64: the query row in VGPRs (exact_sqdist_reg, one pairwise leaf)
  const int maxd = maxd_of(d);
  switch (maxd) {
    case 8: launch_radius<8, PASS>(g, s, Q, nq, ldq, X, nx, ldx, di, eps, plen, cnt, oi, od); break;
    case 16: launch_radius<16, PASS>(g, s, Q, nq, ldq, X, nx, ldx, di, eps, plen, cnt, oi, od); break;
    case 32: launch_radius<32, PASS>(g, s, Q, nq, ldq, X, nx, ldx, di, eps, plen, cnt, oi, od); break;
    case 64: launch_radius<64, PASS>(g, s, Q, nq, ldq, X, nx, ldx, di, eps, plen, cnt, oi, od); break;
    default: launch_radius<0, PASS>(g, s, Q, nq, ldq, X, nx, ldx, di, eps, plen, cnt, oi, od); break;
  }
  return check_launch(PASS == 0 ? "radius count" : "radius fill");
}

int radius_args(const double *Q, int64_t nq, int64_t ldq, const double *X,
                int64_t nx, int64_t ldx, int64_t d, double eps) {
  if (nq < 0 || nx < 0 || d < 1 || ldq < d || ldx < d)
    return fail(DKM_E_ARG, "radius: bad nq/nx/d/ld");
  if (d > INT32_MAX) return fail(DKM_E_ARG, "radius: d too large");
  if (std::isnan(eps)) return fail(DKM_E_ARG, "radius: eps is NaN");
  if (nq > 0 && nx > 0 && (!Q || !X)) return fail(DKM_E_ARG, "radius: NULL Q/X");
  return 0;
}

int radius_csr_args(const int64_t *indptr, const int32_t *indices,
                    const double *data, int64_t n, int64_t d, int64_t q0,
                    int64_t nq, double eps) {
  if (n < 0 || d < 1 || d > INT32_MAX || nq < 0 || q0 < 0 || q0 + nq > n)
    return fail(DKM_E_ARG, "radius csr: bad n/d/q0/nq");
  if (std::isnan(eps)) return fail(DKM_E_ARG, "radius csr: eps is NaN");
  if (n > 0 && (!indptr || (!indices && nq) || (!data && nq)))
    return fail(DKM_E_ARG, "radius csr: NULL indptr/indices/data");
  return 0;
}

// The two-scan path (kn in (32, KB_KN_MAX]): partitions and workspace.
// Pb >= kn / 32 + 1 partitions such that the union of their top-32 lists
// holds >= kn rows (every row when partitions are shorter than 32).
bool kb_applies(int64_t kn) { return kn > 32 && kn <= KB_KN_MAX; }

void kb_grid(int64_t nq, int64_t nx, int64_t kn, int64_t *plen, int *P) {
  int64_t pl0;
  int P0;
  knn_grid(nq, nx, &pl0, &P0);
  for (int64_t want = std::max<int64_t>(P0, kn / 32 + 1);; ++want) {
    const int64_t w = std::min<int64_t>({want, (int64_t)KB_P_MAX, nx});
    const int64_t pl = (nx + w - 1) / w;
    const int64_t np = (nx + pl - 1) / pl;
    int64_t uni = 0;
    for (int64_t p = 0; p < np; ++p)
      uni += std::min<int64_t>(32, std::min(nx, (p + 1) * pl) - p * pl);
    if (uni >= kn || w >= KB_P_MAX || w >= nx) {
      *plen = pl;
      *P = (int)np;
      return;
    }
  }
}

struct KbWs {
  double *pr;
  int *pi;
  uint64_t *thk;
  int *thi;
  unsigned *cc;
  uint64_t *ck;
  int *ci;
  unsigned *flag;
};

size_t kb_layout(int64_t qc, int P, char *base, KbWs *w) {
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 255) & ~(size_t)255;
    return base ? base + at : nullptr;
  };
  const size_t m = (size_t)qc * P * 32;
  char *a = take(m * 8), *b = take(m * 4), *c = take((size_t)qc * 8),
       *d = take((size_t)qc * 4), *e = take((size_t)qc * 4),
       *f = take((size_t)qc * KB_CAP * 8), *g = take((size_t)qc * KB_CAP * 4),
       *h = take(4);
  if (w) *w = KbWs{(double *)a, (int *)b, (uint64_t *)c, (int *)d,
                   (unsigned *)e, (uint64_t *)f, (int *)g, (unsigned *)h};
  return o;
}

size_t kb_bytes(int64_t nq, int64_t nx, int64_t kn) {
  int64_t plen;
  int P;
  kb_grid(nq, nx, kn, &plen, &P);
  return kb_layout(std::min<int64_t>(std::max<int64_t>(nq, 1), KB_QC), P,
                   nullptr, nullptr);
}

// One chunk-looped two-scan call.  scan(q0, qc, g, plen, P, pr, pi) and
// cand(q0, qc, g, plen, thk, thi, cc, ck, ci) launch the dense or CSR
// kernels; *overflow = 1 when a candidate list outgrew KB_CAP (the caller
// reruns in passes).
template <class Scan, class Cand>
int kb_run(int64_t nq, int64_t nx, int64_t kn, void *ws, int f32,
           double *out_dist, int64_t *out_idx, hipStream_t s, Scan scan,
           Cand cand, bool *overflow) {
  int64_t plen;
  int P;
  kb_grid(nq, nx, kn, &plen, &P);
  KbWs w;
  kb_layout(std::min<int64_t>(nq, KB_QC), P, (char *)ws, &w);
  if (hipMemsetAsync(w.flag, 0, 4, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "knn: memset");
  for (int64_t q0 = 0; q0 < nq; q0 += KB_QC) {
    const int64_t qc = std::min<int64_t>(KB_QC, nq - q0);
    const dim3 g((unsigned)((qc + 255) / 256), (unsigned)P);
    if (int r = scan(q0, qc, g, plen, P, w.pr, w.pi)) return r;
    k_knn_thresh<<<(unsigned)qc, NB, 0, s>>>(w.pr, w.pi, qc, P, (int)kn,
                                             w.thk, w.thi, w.cc);
    if (int r = check_launch("knn threshold")) return r;
    if (int r = cand(q0, qc, g, plen, w.thk, w.thi, w.cc, w.ck, w.ci))
      return r;
    k_knn_final<<<(unsigned)qc, NB, 0, s>>>(w.cc, w.ck, w.ci, qc, (int)kn,
                                            out_dist + q0 * kn,
                                            out_idx + q0 * kn, kn, f32,
                                            w.flag);
    if (int r = check_launch("knn final sort")) return r;
  }
  unsigned fl = 0;
  if (hipMemcpyAsync(&fl, w.flag, 4, hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "knn: reading the overflow flag");
  *overflow = fl != 0;
  return 0;
}

}  // namespace
}  // namespace dkm

using namespace dkm;

extern "C" {

size_t dkm_knn_workspace_bytes(int64_t nq, int64_t nx, int64_t kn) {
  if (nq < 0 || nx < 1 || kn < 1 || kn > nx) return 0;
  int64_t plen;
  int P;
  knn_grid(std::max<int64_t>(nq, 1), nx, &plen, &P);
  const int K = knn_k(std::min<int64_t>(kn, 32));
  const int64_t q = std::max<int64_t>(nq, 1);
  // partial lists of one pass, then the per-query floor (r, index); the
  // two-scan path's chunk when it applies (its fallback is the passes)
  const size_t passes = (size_t)q * P * K * (8 + 4) + (size_t)q * (8 + 4) + 512;
  return kb_applies(kn) ? std::max(passes, kb_bytes(nq, nx, kn)) : passes;
}

int dkm_knn_f64(const double *Q, int64_t nq, int64_t ldq, const double *X,
                int64_t nx, int64_t ldx, int64_t d, int64_t kn, void *ws,
                size_t ws_bytes, double *out_dist, int64_t *out_idx,
                void *stream) {
  if (int r = knn_args(Q, nq, ldq, X, nx, ldx, d, kn)) return r;
  if (nq == 0) return 0;
  if (!out_dist || !out_idx) return fail(DKM_E_ARG, "knn: NULL outputs");
  const size_t need = dkm_knn_workspace_bytes(nq, nx, kn);
  if (!ws || ws_bytes < need)
    return fail(DKM_E_WORKSPACE, "knn: workspace smaller than "
                                 "dkm_knn_workspace_bytes()");
  hipStream_t s = (hipStream_t)stream;
  const int maxd = maxd_of(d);
  if (kb_applies(kn)) {
    bool over = false;
    auto scan = [&](int64_t q0, int64_t qc, dim3 g, int64_t pl, int P,
                    double *pr, int *pi) {
      return knn_dispatch<32>(maxd, g, s, Q + q0 * ldq, qc, ldq, X, nx, ldx,
                              (int)d, pl, P, pr, pi, nullptr, nullptr);
    };
    auto cand = [&](int64_t q0, int64_t qc, dim3 g, int64_t pl,
                    const uint64_t *thk, const int *thi, unsigned *cc,
                    uint64_t *ck, int *ci) {
      const double *Qc = Q + q0 * ldq;
      switch (maxd) {
        case 8: k_knn_cand<8><<<g, NB, 0, s>>>(Qc, qc, ldq, X, nx, ldx, (int)d, pl, thk, thi, cc, ck, ci); break;
        case 16: k_knn_cand<16><<<g, NB, 0, s>>>(Qc, qc, ldq, X, nx, ldx, (int)d, pl, thk, thi, cc, ck, ci); break;
        case 32: k_knn_cand<32><<<g, NB, 0, s>>>(Qc, qc, ldq, X, nx, ldx, (int)d, pl, thk, thi, cc, ck, ci); break;
        case 64: k_knn_cand<64><<<g, NB, 0, s>>>(Qc, qc, ldq, X, nx, ldx, (int)d, pl, thk, thi, cc, ck, ci); break;
        default: k_knn_cand<0><<<g, NB, 0, s>>>(Qc, qc, ldq, X, nx, ldx, (int)d, pl, thk, thi, cc, ck, ci); break;
      }
      return check_launch("knn candidates");
    };
    if (int r = kb_run(nq, nx, kn, ws, 0, out_dist, out_idx, s, scan, cand,
                       &over))
      return r;
    if (!over) return 0;
  }
  int64_t plen;
  int P;
  knn_grid(nq, nx, &plen, &P);
  const int KP = knn_k(std::min<int64_t>(kn, 32));
  double *pr = (double *)ws;
  int *pi = (int *)(pr + (size_t)nq * P * KP);
  double *flr = (double *)(((uintptr_t)(pi + (size_t)nq * P * KP) + 255) &
                           ~(uintptr_t)255);
  int *fli = (int *)(flr + nq);
  const dim3 g((unsigned)((nq + 255) / 256), (unsigned)P);
  for (int64_t c0 = 0; c0 < kn; c0 += 32) {
    const int kk = (int)std::min<int64_t>(32, kn - c0);
    const int K = knn_k(kk);
    const double *fr = c0 ? flr : nullptr;
    const int *fi = c0 ? fli : nullptr;
    int r;
    switch (K) {
      case 1: r = knn_dispatch<1>(maxd, g, s, Q, nq, ldq, X, nx, ldx, (int)d, plen, P, pr, pi, fr, fi); break;
      case 2: r = knn_dispatch<2>(maxd, g, s, Q, nq, ldq, X, nx, ldx, (int)d, plen, P, pr, pi, fr, fi); break;
      case 4: r = knn_dispatch<4>(maxd, g, s, Q, nq, ldq, X, nx, ldx, (int)d, plen, P, pr, pi, fr, fi); break;
      case 8: r = knn_dispatch<8>(maxd, g, s, Q, nq, ldq, X, nx, ldx, (int)d, plen, P, pr, pi, fr, fi); break;
      case 16: r = knn_dispatch<16>(maxd, g, s, Q, nq, ldq, X, nx, ldx, (int)d, plen, P, pr, pi, fr, fi); break;
      default: r = knn_dispatch<32>(maxd, g, s, Q, nq, ldq, X, nx, ldx, (int)d, plen, P, pr, pi, fr, fi); break;
    }
    if (r) return r;
    if (int e = knn_merge_launch(K, s, pr, pi, nq, P, kk, out_dist + c0,
                                 out_idx + c0, kn, flr, fli, 0))
      return e;
  }
  return 0;
}

int dkm_knn_csr_f64(const int64_t *q_indptr, const int32_t *q_indices,
                    const double *q_data, int64_t nq, const int64_t *x_indptr,
                    const int32_t *x_indices, const double *x_data,
                    int64_t nx, int64_t d, int64_t kn, int out_f32, void *ws,
                    size_t ws_bytes, double *out_dist, int64_t *out_idx,
                    void *stream) {
  if (nq < 0 || nx < 1 || d < 1 || d > INT32_MAX || nx > INT32_MAX)
    return fail(DKM_E_ARG, "knn csr: bad nq/nx/d");
  if (kn < 1 || kn > nx)
    return fail(DKM_E_ARG, "knn csr: n_neighbors must be in [1, nx]");
  if (nq == 0) return 0;
  if (!q_indptr || !q_indices || !q_data || !x_indptr || !x_indices ||
      !x_data)
    return fail(DKM_E_ARG, "knn csr: NULL indptr/indices/data");
  if (!out_dist || !out_idx) return fail(DKM_E_ARG, "knn csr: NULL outputs");
  const size_t need = dkm_knn_workspace_bytes(nq, nx, kn);
  if (!ws || ws_bytes < need)
    return fail(DKM_E_WORKSPACE, "knn csr: workspace smaller than "
                                 "dkm_knn_workspace_bytes()");
  hipStream_t s = (hipStream_t)stream;
  const int f32 = out_f32 ? 1 : 0;
  if (kb_applies(kn)) {
    bool over = false;
    auto scan = [&](int64_t q0, int64_t qc, dim3 g, int64_t pl, int P,
                    double *pr, int *pi) {
      return knn_csr_launch<32>(g, s, q_indptr + q0, q_indices, q_data, qc,
                                x_indptr, x_indices, x_data, nx, pl, P, f32,
                                pr, pi, nullptr, nullptr);
    };
    auto cand = [&](int64_t q0, int64_t qc, dim3 g, int64_t pl,
                    const uint64_t *thk, const int *thi, unsigned *cc,
                    uint64_t *ck, int *ci) {
      k_knn_csr_cand<<<g, NB, 0, s>>>(q_indptr + q0, q_indices, q_data, qc,
                                      x_indptr, x_indices, x_data, nx, pl,
                                      f32, thk, thi, cc, ck, ci);
      return check_launch("knn csr candidates");
    };
    if (int r = kb_run(nq, nx, kn, ws, f32, out_dist, out_idx, s, scan, cand,
                       &over))
      return r;
    if (!over) return 0;
  }
  int64_t plen;
  int P;
  knn_grid(nq, nx, &plen, &P);
  const int KP = knn_k(std::min<int64_t>(kn, 32));
  double *pr = (double *)ws;
  int *pi = (int *)(pr + (size_t)nq * P * KP);
  double *flr = (double *)(((uintptr_t)(pi + (size_t)nq * P * KP) + 255) &
                           ~(uintptr_t)255);
  int *fli = (int *)(flr + nq);
  const dim3 g((unsigned)((nq + 255) / 256), (unsigned)P);
  for (int64_t c0 = 0; c0 < kn; c0 += 32) {
    const int kk = (int)std::min<int64_t>(32, kn - c0);
    const int K = knn_k(kk);
    const double *fr = c0 ? flr : nullptr;
    const int *fi = c0 ? fli : nullptr;
    int r;
    switch (K) {
      case 1: r = knn_csr_launch<1>(g, s, q_indptr, q_indices, q_data, nq, x_indptr, x_indices, x_data, nx, plen, P, out_f32 ? 1 : 0, pr, pi, fr, fi); break;
      case 2: r = knn_csr_launch<2>(g, s, q_indptr, q_indices, q_data, nq, x_indptr, x_indices, x_data, nx, plen, P, out_f32 ? 1 : 0, pr, pi, fr, fi); break;
      case 4: r = knn_csr_launch<4>(g, s, q_indptr, q_indices, q_data, nq, x_indptr, x_indices, x_data, nx, plen, P, out_f32 ? 1 : 0, pr, pi, fr, fi); break;
      case 8: r = knn_csr_launch<8>(g, s, q_indptr, q_indices, q_data, nq, x_indptr, x_indices, x_data, nx, plen, P, out_f32 ? 1 : 0, pr, pi, fr, fi); break;
      case 16: r = knn_csr_launch<16>(g, s, q_indptr, q_indices, q_data, nq, x_indptr, x_indices, x_data, nx, plen, P, out_f32 ? 1 : 0, pr, pi, fr, fi); break;
      default: r = knn_csr_launch<32>(g, s, q_indptr, q_indices, q_data, nq, x_indptr, x_indices, x_data, nx, plen, P, out_f32 ? 1 : 0, pr, pi, fr, fi); break;
    }
    if (r) return r;
    if (int e = knn_merge_launch(K, s, pr, pi, nq, P, kk, out_dist + c0,
                                 out_idx + c0, kn, flr, fli, out_f32 ? 1 : 0))
      return e;
  }
  return 0;
}

int dkm_radius_count_f64(const double *Q, int64_t nq, int64_t ldq,
                         const double *X, int64_t nx, int64_t ldx, int64_t d,
                         double eps, int64_t *counts, void *stream) {
  if (int r = radius_args(Q, nq, ldq, X, nx, ldx, d, eps)) return r;
  if (nq == 0) return 0;
  if (!counts) return fail(DKM_E_ARG, "radius: NULL counts");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(counts, 0, (size_t)nq * 8, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "radius: memset");
  if (nx == 0) return 0;
  int64_t plen;
  int P;
  knn_grid(nq, nx, &plen, &P);
  const dim3 g((unsigned)((nq + 255) / 256), (unsigned)P);
  return radius_dispatch<0>(d, g, s, Q, nq, ldq, X, nx, ldx, eps, plen,
                            (unsigned long long *)counts, nullptr, nullptr);
}

size_t dkm_radius_workspace_bytes(int64_t nq, int64_t total) {
  if (nq < 0 || total < 0) return 0;
  return (size_t)nq * 8 + (size_t)total * 16 + 256;
}

int dkm_radius_fill_f64(const double *Q, int64_t nq, int64_t ldq,
                        const double *X, int64_t nx, int64_t ldx, int64_t d,
                        double eps, const int64_t *offsets, void *ws,
                        size_t ws_bytes, int64_t *out_idx, double *out_dist,
                        void *stream) {
  if (int r = radius_args(Q, nq, ldq, X, nx, ldx, d, eps)) return r;
  if (nq == 0 || nx == 0) return 0;
  if (!offsets || !out_idx || !out_dist)
    return fail(DKM_E_ARG, "radius: NULL offsets/outputs");
  hipStream_t s = (hipStream_t)stream;
  int64_t total = 0;
  if (hipMemcpyAsync(&total, offsets + nq, 8, hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "radius: reading offsets[nq]");
  if (total < 0) return fail(DKM_E_ARG, "radius: offsets[nq] < 0");
  if (!ws || ws_bytes < dkm_radius_workspace_bytes(nq, total))
    return fail(DKM_E_WORKSPACE, "radius: workspace smaller than "
                                 "dkm_radius_workspace_bytes()");
  // cursors = offsets[0..nq)
  unsigned long long *cur = (unsigned long long *)ws;
  int64_t *sidx = (int64_t *)((char *)ws + (size_t)nq * 8);
  double *sdist = (double *)(sidx + total);
  if (hipMemcpyAsync(cur, offsets, (size_t)nq * 8, hipMemcpyDeviceToDevice,
                     s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "radius: cursor copy");
  int64_t plen;
  int P;
  knn_grid(nq, nx, &plen, &P);
  const dim3 g((unsigned)((nq + 255) / 256), (unsigned)P);
  if (int r = radius_dispatch<1>(d, g, s, Q, nq, ldq, X, nx, ldx, eps, plen,
                                 cur, out_idx, out_dist))
    return r;
  if (total == 0) return 0;
  k_seg_sort<<<(unsigned)nq, NB, 0, s>>>(offsets, nq, out_idx, out_dist, sidx,
                                         sdist);
  return check_launch("radius sort");
}

int dkm_radius_count_csr_f64(const int64_t *indptr, const int32_t *indices,
                             const double *data, int64_t n, int64_t d,
                             int64_t q0, int64_t nq, double eps, int out_f32,
                             int64_t *counts, void *stream) {
  if (int r = radius_csr_args(indptr, indices, data, n, d, q0, nq, eps))
    return r;
  if (nq == 0) return 0;
  if (!counts) return fail(DKM_E_ARG, "radius csr: NULL counts");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(counts, 0, (size_t)nq * 8, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "radius csr: memset");
  int64_t plen;
  int P;
  knn_grid(nq, n, &plen, &P);
  const dim3 g((unsigned)((nq + 255) / 256), (unsigned)P);
  k_radius_csr<0><<<g, NB, 0, s>>>(indptr, indices, data, q0, nq, n, eps,
                                   plen, out_f32 ? 1 : 0,
                                   (unsigned long long *)counts, nullptr,
                                   nullptr);
  return check_launch("radius csr count");
}

int dkm_radius_fill_csr_f64(const int64_t *indptr, const int32_t *indices,
                            const double *data, int64_t n, int64_t d,
                            int64_t q0, int64_t nq, double eps, int out_f32,
                            const int64_t *offsets, void *ws, size_t ws_bytes,
                            int64_t *out_idx, double *out_dist,
                            void *stream) {
  if (int r = radius_csr_args(indptr, indices, data, n, d, q0, nq, eps))
    return r;
  if (nq == 0) return 0;
  if (!offsets || !out_idx || !out_dist)
    return fail(DKM_E_ARG, "radius csr: NULL offsets/outputs");
  hipStream_t s = (hipStream_t)stream;
  int64_t total = 0;
  if (hipMemcpyAsync(&total, offsets + nq, 8, hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "radius csr: reading offsets[nq]");
  if (total < 0) return fail(DKM_E_ARG, "radius csr: offsets[nq] < 0");
  if (total == 0) return 0;
  if (!ws || ws_bytes < dkm_radius_workspace_bytes(nq, total))
    return fail(DKM_E_WORKSPACE, "radius csr: workspace smaller than "
                                 "dkm_radius_workspace_bytes()");
  unsigned long long *cur = (unsigned long long *)ws;
  int64_t *sidx = (int64_t *)((char *)ws + (size_t)nq * 8);
  double *sdist = (double *)(sidx + total);
  if (hipMemcpyAsync(cur, offsets, (size_t)nq * 8, hipMemcpyDeviceToDevice,
                     s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "radius csr: cursor copy");
  int64_t plen;
  int P;
  knn_grid(nq, n, &plen, &P);
  const dim3 g((unsigned)((nq + 255) / 256), (unsigned)P);
  k_radius_csr<1><<<g, NB, 0, s>>>(indptr, indices, data, q0, nq, n, eps,
                                   plen, out_f32 ? 1 : 0, cur, out_idx,
                                   out_dist);
  if (int e = check_launch("radius csr fill")) return e;
  k_seg_sort<<<(unsigned)nq, NB, 0, s>>>(offsets, nq, out_idx, out_dist, sidx,
                                         sdist);
  return check_launch("radius csr sort");
}

}  // extern "C"

// Code-object preload (dkm_preload): the runtime loads this file's kernels
// on first use of any of them; an attribute query here does it up front.
namespace dkm {
DKM_TU_FLAGS(neighbors, 0)
__global__ void k_tu_neighbors() {}
int preload_neighbors() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void *)k_tu_neighbors) == hipSuccess ? 0
                                                                       : 1;
}
}  // namespace dkm
