// dkm_sums.hip -- per-cluster [sums | counts] from finished labels, for the
// shapes whose k x d fp64 sums do not fit a block's LDS (the screens then
// write labels only): the second half of dislib's `_partial_sum`
// (cluster/kmeans/base.py:174-181: `partials[label] += row` and the counts).
//
// Counting sort of the sample indices by label, then segmented row sums:
//   k_sort_count    per-block LDS histogram of the keys, one global atomic
//                   per (block, non-empty cluster);
//   k_sort_scan     exclusive scan of the k counts -> cluster offsets;
//   k_sort_scatter  per-block ranges reserved with one atomic per (block,
//                   cluster), ranks from LDS atomics -> indices grouped by
//                   cluster (order inside a cluster is free: fp64 sums);
//   k_seg_sums      a wave walks SEG consecutive sorted indices, lanes over
//                   features (or sub-groups of G lanes over rows for d <= 32),
//                   keeps the running sum of the current cluster in VGPRs and
//                   adds it to acc with fp64 atomics when the cluster changes.
// X is read once, row by row (each row contiguous: full 128-B lines), the
// labels three times (4 B each), and acc sees ~d atomics per (wave chunk,
// cluster) instead of per sample.
//
// Delta (prev != NULL): only samples whose label changed contribute; they
// are compacted first (k_moved), sorted by the new label (+x) and again by
// the previous label (-x).
//
// Replaces k_label_sums (dkm_dense.hip), which read the labels once per
// LDS-sized cluster range (k / 18 times at d = 1024).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "dkm_internal.h"

namespace dkm {

namespace {

constexpr int SBLK = 1024;    // threads per sort block
constexpr int SRANGE = 16384; // sort positions per block
constexpr int SEG = 1024;     // sorted positions per k_seg_sums wave chunk
constexpr int SEG_LIST = 64;  // the same for moved-sample lists
constexpr int SUMB = 256;     // threads per k_seg_sums block

int cus() {
  static thread_local int cached_dev = -1, n = 256;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return n;
  if (dev != cached_dev) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess) n = p.multiProcessorCount;
    cached_dev = dev;
  }
  return n;
}

__device__ __forceinline__ int64_t n_items(const int32_t *ndev, int64_t nh) {
  return ndev ? (int64_t)*ndev : nh;
}

// sample index at sorted-input position p: an explicit list or lo + p
__device__ __forceinline__ int32_t item_at(const int32_t *items, int64_t lo,
                                           int64_t p) {
  return items ? items[p] : (int32_t)(lo + p);
}

}  // namespace

// Samples whose label changed (lab != prev) over [lo, hi), compacted into
// `out` (order free); the count accumulates in *count.  One global atomic
// per block: waves count their ballots, the block reserves, waves write.
__global__ void __launch_bounds__(SBLK)
    k_moved(const int32_t *__restrict__ lab, const int32_t *__restrict__ prev,
            int64_t lo, int64_t hi, int32_t *__restrict__ out,
            int32_t *count) {
  __shared__ int wcount[SBLK / 64];
  __shared__ int bbase;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r0 = lo + (int64_t)blockIdx.x * SRANGE;
  const int64_t r1 = std::min(hi, r0 + SRANGE);
  constexpr int PER = SRANGE / (SBLK / 64);  // positions per wave
  const int64_t w0 = r0 + (int64_t)w * PER, w1 = std::min(r1, w0 + PER);
  int c = 0;
  for (int64_t i0 = w0; i0 < w1; i0 += 64) {
    const int64_t i = i0 + lane;
    const bool mv = i < w1 && lab[i] != prev[i];
    c += __popcll(__ballot(mv));
  }
  if (lane == 0) wcount[w] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int j = 0; j < SBLK / 64; ++j) {
      const int x = wcount[j];
      wcount[j] = t;
      t += x;
    }
    bbase = t ? atomicAdd(count, t) : 0;
  }
  __syncthreads();
  int pos = bbase + wcount[w];
  for (int64_t i0 = w0; i0 < w1; i0 += 64) {
    const int64_t i = i0 + lane;
    const bool mv = i < w1 && lab[i] != prev[i];
    const uint64_t m = __ballot(mv);
    if (mv) {
      const int r = __builtin_amdgcn_mbcnt_hi(
          (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      out[pos + r] = (int32_t)i;
    }
    pos += __popcll(m);
  }
}

// Histogram of key[item] over the sorted-input positions of this block.
__global__ void __launch_bounds__(SBLK)
    k_sort_count(const int32_t *__restrict__ key,
                 const int32_t *__restrict__ items, const int32_t *ndev,
                 int64_t nh, int64_t lo, int k, int32_t *__restrict__ cnt) {
  extern __shared__ int hist[];
  const int64_t n = n_items(ndev, nh);
  // block-stride over SRANGE chunks: an explicit list (delta path) is
  // launched on a fixed grid and is usually short or empty
  for (int64_t p0 = (int64_t)blockIdx.x * SRANGE; p0 < n;
       p0 += (int64_t)gridDim.x * SRANGE) {
    const int64_t p1 = std::min(n, p0 + SRANGE);
    __syncthreads();
    for (int c = threadIdx.x; c < k; c += SBLK) hist[c] = 0;
    __syncthreads();
    for (int64_t p = p0 + threadIdx.x; p < p1; p += SBLK) {
      const int c = key[item_at(items, lo, p)];
      if ((unsigned)c < (unsigned)k) atomicAdd(&hist[c], 1);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < k; c += SBLK)
      if (hist[c]) atomicAdd(&cnt[c], hist[c]);
  }
}

// Exclusive scan of cnt[0..k) -> off[0..k], cur = off (one block).
__global__ void __launch_bounds__(SBLK)
    k_sort_scan(const int32_t *__restrict__ cnt, int k,
                int32_t *__restrict__ off, int32_t *__restrict__ cur) {
  __shared__ int part[SBLK];
  const int per = (k + SBLK - 1) / SBLK;
  const int c0 = threadIdx.x * per, c1 = std::min(k, c0 + per);
  int s = 0;
  for (int c = c0; c < c1; ++c) s += cnt[c];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int st = 1; st < SBLK; st <<= 1) {  // Hillis-Steele inclusive scan
    const int v = threadIdx.x >= st ? part[threadIdx.x - st] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = part[threadIdx.x] - s;
  for (int c = c0; c < c1; ++c) {
    off[c] = run;
    cur[c] = run;
    run += cnt[c];
  }
  if (threadIdx.x == SBLK - 1) off[k] = part[SBLK - 1];
}

// Scatter the items of this block's positions to their cluster's range.
__global__ void __launch_bounds__(SBLK)
    k_sort_scatter(const int32_t *__restrict__ key,
                   const int32_t *__restrict__ items, const int32_t *ndev,
                   int64_t nh, int64_t lo, int k, int32_t *__restrict__ cur,
                   int32_t *__restrict__ out) {
  extern __shared__ int hist[];  // [k] counts, then ranks; [k] bases
  int *base = hist + k;
  const int64_t n = n_items(ndev, nh);
  for (int64_t p0 = (int64_t)blockIdx.x * SRANGE; p0 < n;
       p0 += (int64_t)gridDim.x * SRANGE) {
    const int64_t p1 = std::min(n, p0 + SRANGE);
    __syncthreads();
    for (int c = threadIdx.x; c < k; c += SBLK) hist[c] = 0;
    __syncthreads();
    for (int64_t p = p0 + threadIdx.x; p < p1; p += SBLK) {
      const int c = key[item_at(items, lo, p)];
      if ((unsigned)c < (unsigned)k) atomicAdd(&hist[c], 1);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < k; c += SBLK) {
      const int h = hist[c];
      base[c] = h ? atomicAdd(&cur[c], h) : 0;
      hist[c] = 0;
    }
    __syncthreads();
    for (int64_t p = p0 + threadIdx.x; p < p1; p += SBLK) {
      const int32_t it = item_at(items, lo, p);
      const int c = key[it];
      if ((unsigned)c < (unsigned)k) out[base[c] + atomicAdd(&hist[c], 1)] = it;
    }
  }
}

// Segmented sums over the grouped indices.  G lanes per row (G = 64 with
// NJ features per lane, or G = 8/16/32 lanes and 64/G rows at a time for
// small d); blockIdx.y picks the column block of G*NJ features.
template <class TX, int G, int NJ>
__global__ void __launch_bounds__(SUMB)
    k_seg_sums(const TX *__restrict__ X, int64_t ldx, int d,
               const int32_t *__restrict__ sorted,
               const int32_t *__restrict__ off, int k, double sign,
               double *__restrict__ acc, int seg) {
  constexpr int R = 64 / G;                 // rows in flight per step
  // steps issued together: >= 8 loads per lane in flight, and fp32 rows
  // twice as many (the same bytes in flight as fp64)
  constexpr int U = (NJ >= 8 ? 1 : 8 / NJ) * (sizeof(TX) == 4 ? 2 : 1);
  const int64_t n = off[k];  // sorted entries (keys outside [0, k) dropped)
  const int lane = threadIdx.x & 63, sg = lane / G, gl = lane % G;
  const int col0 = blockIdx.y * (G * NJ);
  const int64_t wv = (int64_t)blockIdx.x * (SUMB / 64) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (SUMB / 64);
  for (int64_t p0 = wv * seg; p0 < n; p0 += nw * seg) {
    const int64_t p1 = std::min(n, p0 + seg);
    // cluster of position p0 + sg: largest c with off[c] <= p0 + sg
    const int64_t q0 = p0 + sg;
    int lo_c = 0, hi_c = k;  // off[lo_c] <= q0 < off[hi_c]
    while (hi_c - lo_c > 1) {
      const int mid = (lo_c + hi_c) >> 1;
      if (off[mid] <= q0) lo_c = mid;
      else hi_c = mid;
    }
    int c = lo_c;
    int64_t nxt = off[c + 1];
    double a[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) a[j] = 0.0;
    int cnt = 0;
    auto flush = [&]() {
      if (cnt) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int t = col0 + gl + G * j;
          if (t < d) atomic_add_f64(acc + (int64_t)c * d + t, sign * a[j]);
          a[j] = 0.0;
        }
        if (blockIdx.y == 0 && gl == 0)
          atomic_add_f64(acc + (int64_t)k * d + c, sign * (double)cnt);
        cnt = 0;
      }
    };
    for (int64_t q = q0; q < p1; q += R * U) {
      double x[U][NJ];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t pos = q + (int64_t)u * R;
        const int32_t it = sorted[pos < p1 ? pos : p1 - 1];
        const TX *row = X + (int64_t)it * ldx;
        // Unconditional loads from a clamped position / column and no select: a
        // select of a load lets hipcc branch around each load with a
        // vmcnt(0) inside (16 serialised loads per row; it did so for fp32,
        // 1.4 TB/s against 6.0 for fp64, tools/bench_sums.py r05o, and for
        // fp64 once the address was clamped).  The values of rows past the
        // chunk and columns past d are never added (pos < p1 below) or
        // flushed (t < d).
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int t = col0 + gl + G * j;
          x[u][j] = (double)row[t < d ? t : d - 1];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t pos = q + (int64_t)u * R;
        if (pos < p1) {
          while (pos >= nxt) {  // skips empty clusters
            flush();
            ++c;
            nxt = off[c + 1];
          }
#pragma unroll
          for (int j = 0; j < NJ; ++j) a[j] += x[u][j];
          ++cnt;
        }
      }
    }
    flush();
  }
}

bool sorted_sums_ok(int64_t k, int64_t n, const WsView &v) {
  return v.soff && k <= SORT_KMAX && n <= v.nq && n <= INT32_MAX;
}

template <class TX>
static int launch_seg(const TX *X, int64_t ldx, int d, const int32_t *sorted,
                      int64_t nh, const int32_t *off, int k, double sign,
                      double *acc, hipStream_t s, bool list = false) {
  // explicit (moved-sample) lists: a smaller grid, grid-striding, and short
  // wave chunks -- the list is usually far shorter than its bound nh, and a
  // 1024-position chunk per wave left a 100k-row list to ~100 waves, each
  // with two dependent loads per step (1 ms per C3 delta pass)
  const int seg = list ? SEG_LIST : SEG;
  const int64_t chunks = (nh + seg - 1) / seg;
  const int64_t g = std::max<int64_t>(
      1, std::min<int64_t>((int64_t)cus() * (list ? 2 : 8),
                           (chunks + SUMB / 64 - 1) / (SUMB / 64)));
#define DKM_SEG(GG, NN)                                                       \
  {                                                                           \
    const unsigned gy = (unsigned)((d + GG * NN - 1) / (GG * NN));            \
    k_seg_sums<TX, GG, NN><<<dim3((unsigned)g, gy), SUMB, 0, s>>>(            \
        X, ldx, d, sorted, off, k, sign, acc, seg);                           \
  }
  if (d <= 8) DKM_SEG(8, 1)
  else if (d <= 16) DKM_SEG(16, 1)
  else if (d <= 32) DKM_SEG(32, 1)
  else if (d <= 64) DKM_SEG(64, 1)
  else if (d <= 128) DKM_SEG(64, 2)
  else if (d <= 256) DKM_SEG(64, 4)
  else if (d <= 512) DKM_SEG(64, 8)
  else DKM_SEG(64, 16)
#undef DKM_SEG
  return check_launch("segmented sums");
}

static int set_sort_lds() {
  if (hipFuncSetAttribute((const void *)k_sort_scatter,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          SORT_KMAX * 8) != hipSuccess ||
      hipFuncSetAttribute((const void *)k_sort_count,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          SORT_KMAX * 4) != hipSuccess)
    return fail(DKM_E_LAUNCH, "sorted sums: LDS attribute");
  return 0;
}

// Counting sort of the items (explicit list of *ndev <= nh entries, or
// [lo, lo + nh)) by key into v.sitems, cluster c at [v.soff[c],
// v.soff[c+1]); keys outside [0, k) (a previous label -1) are dropped.
static int sort_items(const int32_t *key, const int32_t *items,
                      const int32_t *ndev, int64_t nh, int64_t lo, int k,
                      const WsView &v, hipStream_t s) {
  // an explicit list has *ndev <= nh entries, usually few: a fixed grid of
  // a block per CU strides over whatever it holds (0.06 + 0.56 ms of empty
  // sort + sum launches per converged C3 iteration on the n-sized grids)
  const int64_t chunks = (nh + SRANGE - 1) / SRANGE;
  const unsigned nb = (unsigned)std::max<int64_t>(
      1, ndev ? std::min<int64_t>(chunks, cus()) : chunks);
  if (hipMemsetAsync(v.scnt, 0, (size_t)k * 4, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "sorted sums: memset");
  k_sort_count<<<nb, SBLK, (size_t)k * 4, s>>>(key, items, ndev, nh, lo, k,
                                               v.scnt);
  k_sort_scan<<<1, SBLK, 0, s>>>(v.scnt, k, v.soff, v.scur);
  k_sort_scatter<<<nb, SBLK, (size_t)k * 8, s>>>(key, items, ndev, nh, lo, k,
                                                 v.scur, v.sitems);
  return check_launch("label sort");
}

int sort_by_label(const int32_t *lab, int64_t lo, int64_t hi, int k,
                  const WsView &v, hipStream_t s) {
  if (!sorted_sums_ok(k, hi - lo, v))
    return fail(DKM_E_WORKSPACE, "label sort: scratch too small");
  if (int r = set_sort_lds()) return r;
  return sort_items(lab, nullptr, nullptr, hi - lo, lo, k, v, s);
}

// Sort the items by key, then add sign * row to acc[key] for each.
template <class TX>
static int sort_and_sum(const TX *X, int64_t ldx, int d, const int32_t *key,
                        const int32_t *items, const int32_t *ndev, int64_t nh,
                        int64_t lo, int k, double sign, double *acc,
                        const WsView &v, hipStream_t s) {
  if (int r = sort_items(key, items, ndev, nh, lo, k, v, s)) return r;
  return launch_seg<TX>(X, ldx, d, v.sitems, nh, v.soff, k, sign, acc, s,
                        ndev != nullptr);
}

template <class TX>
int sorted_sums(const TX *X, int64_t lo, int64_t hi, int d, int64_t ldx,
                const int32_t *lab, const int32_t *prev, int k, double *acc,
                const WsView &v, hipStream_t s) {
  if (hi <= lo) return 0;
  const int64_t n = hi - lo;
  if (!sorted_sums_ok(k, n, v))
    return fail(DKM_E_WORKSPACE, "sorted sums: scratch too small");
  if (int r = set_sort_lds()) return r;
  if (!prev)
    return sort_and_sum<TX>(X, ldx, d, lab, nullptr, nullptr, n, lo, k, 1.0,
                            acc, v, s);
  int32_t *nmv = &v.hdr->nmoved;
  if (hipMemsetAsync(nmv, 0, 4, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "sorted sums: memset");
  k_moved<<<(unsigned)((n + SRANGE - 1) / SRANGE), SBLK, 0, s>>>(
      lab, prev, lo, hi, v.smoved, nmv);
  if (int r = check_launch("moved samples")) return r;
  if (int r = sort_and_sum<TX>(X, ldx, d, lab, v.smoved, nmv, n, 0, k, 1.0,
                               acc, v, s))
    return r;
  return sort_and_sum<TX>(X, ldx, d, prev, v.smoved, nmv, n, 0, k, -1.0, acc,
                          v, s);
}

template <class TX>
int sorted_sums_moved(const TX *X, int64_t n, int d, int64_t ldx,
                      const int32_t *lab, const int32_t *prevs, int k,
                      double *acc, const WsView &v, hipStream_t s) {
  if (n <= 0) return 0;
  if (!sorted_sums_ok(k, n, v))
    return fail(DKM_E_WORKSPACE, "sorted sums: scratch too small");
  if (int r = set_sort_lds()) return r;
  int32_t *nmv = &v.hdr->nmoved;
  if (int r = sort_and_sum<TX>(X, ldx, d, lab, v.smoved, nmv, n, 0, k, 1.0,
                               acc, v, s))
    return r;
  return sort_and_sum<TX>(X, ldx, d, prevs, v.smoved, nmv, n, 0, k, -1.0, acc,
                          v, s);
}

template int sorted_sums_moved<float>(const float *, int64_t, int, int64_t,
                                      const int32_t *, const int32_t *, int,
                                      double *, const WsView &, hipStream_t);
template int sorted_sums_moved<double>(const double *, int64_t, int, int64_t,
                                       const int32_t *, const int32_t *, int,
                                       double *, const WsView &, hipStream_t);

template int sorted_sums<float>(const float *, int64_t, int64_t, int, int64_t,
                                const int32_t *, const int32_t *, int,
                                double *, const WsView &, hipStream_t);
template int sorted_sums<double>(const double *, int64_t, int64_t, int,
                                 int64_t, const int32_t *, const int32_t *,
                                 int, double *, const WsView &, hipStream_t);

}  // namespace dkm

// Code-object preload (dkm_preload): the runtime loads this file's kernels
// on first use of any of them; an attribute query here does it up front.
namespace dkm {
DKM_TU_FLAGS(sums, 0)
__global__ void k_tu_sums() {}
int preload_sums() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void *)k_tu_sums) == hipSuccess ? 0
                                                                       : 1;
}
}  // namespace dkm
