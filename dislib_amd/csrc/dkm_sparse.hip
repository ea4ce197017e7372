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
// followed by np.argmin (first index).  Labels are bit-exact: a sample is
// labelled by the screen below only when a rigorous bound proves the
// reference arithmetic picks the same centre, otherwise by that arithmetic.
//
// The time goes into gathering nnz rows of C^T per sample (k values each),
// an L2-bandwidth-bound walk: at C5 (k = 256, 10 nnz) the fp32 table was
// 10 KB per sample from a 10.24 MB table that overflows an XCD's 4 MB L2
// (16 TB/s of L2 gathers, 3.4 KB/sample of fabric traffic, round 4).  The
// screen table is therefore bf16 (round to nearest from fp64; the bound
// below widens by the rounding): half the bytes per gather and a 5.12 MB
// table whose L2 share doubles.  Large tables are cut into S slices (S = 1,
// 2, 4 or 8; CSR_SLICE_BYTES) and block b works on slice b % S, so blocks b
// and b + 8 share an XCD and gather from one slice (a speed assumption,
// never a correctness one).  Every slice costs a walk over the sample's
// entries, a reduction and a state per sample, and that costs more than the
// L2 locality gains (fp32 C5: S = 1 7.0 ms per step; S = 2: 7.3, S = 4: 7.6,
// S = 8: 8.8; profiles/r04/c5ab).
//   k_csr_screen   8 lanes per sample (8 samples per wave), 8 centres per
//                  lane per 64-centre pass, 16-B loads of the bf16 C^T; the
//                  row's entries staged 8 at a time in the group's lanes and
//                  walked by ds_bpermute.  Per centre j only s_j = |c_j|^2 -
//                  2 x.c_j (one fp32 fma per stored entry); the slice's
//                  state is its two smallest scores and the index of the
//                  first; the bound B (below) is one per sample.
//   k_csr_merge    one lane per sample: the slices' states merged (ascending
//                  centre ranges: a strict < keeps the first index); decided
//                  when s1 + B < s2 - B for the best s1 and the next s2 --
//                  then the reference's fp64 distances order the same way,
//                  strictly, also after sqrt -- else listed for
//                  k_csr_resolve.  Writes the label and, on the incremental
//                  path, moves the rows whose label changed (+x new,
//                  -x previous; fp64 atomics).
//   k_csr_resolve  a wave per listed sample: the reference arithmetic over
//                  all k centres (fp64 C^T), first-index argmin.
//   k_csr_seg_sums the full [sums | counts]: samples counting-sorted by
//                  label (dkm_sums.hip), a block per 4096 sorted positions
//                  adds rows into an LDS copy of the cluster's sum (fp64 LDS
//                  atomics) and flushes it once per cluster segment.
// Samples are processed in chunks so that the S slice states fit the
// workspace tail (20 bytes per slice and sample).
//
// The bound.  With u = 2^-24 (fp32), w = 2^-53 (fp64) and b = 2^-8 (bf16:
// round to nearest to an 8-bit significand, unit roundoff 2^-8), n stored
// entries, A_j >= sum |x_v c_jv| and M_j = xx +
// |c_j|^2 + 2 A_j + |s_j| >= the magnitude of every partial result:
//   bf16 table vs exact        2 b (1 + 2^-14) A_j (c_jv rounded to bf16,
//                                                in the -2 x.c term)
//   fp32 dot vs exact          (n + 2) u A_j     (x rounded, fma chain)
//   sklearn's fp64 dot         n w A_j
//   s_j rounding, |c|^2 -> fp32  u |s_j| + u |c_j|^2
//   sklearn's two additions    2 w M_j;  sqrt strictly monotone: 4 w M_j
// B_j = 2 x their sum (+ 2^-100 absolute, for underflow): s1 + B1 < s_j - B_j
// implies S_1 < S_j with a margin that survives sqrt, where S = sklearn's
// squared distances.  The screen uses one B >= every B_j per sample, from
// A_j <= ||x|| ||c_j|| (Cauchy-Schwarz), ||c_j|| <= cmax = max_j ||c_j|| and
// |s_j| <= |c_j|^2 + 2 A_j: no per-centre |x||c| sums, which doubled the
// screen's VALU work (C5: 11.7 -> 10.4 ms per step, every sample still
// decided), at a bound a few times looser than the per-centre one.  NaN /
// inf anywhere (a centre norm, an overflowing score) makes B or the scores
// non-finite: undecided.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <type_traits>

#include "dkm_internal.h"

namespace dkm {

namespace {

constexpr int CSR_BLOCK = 256;
constexpr int CSR_G = 8;                   // lanes per sample
constexpr int CSR_SPW = WAVE / CSR_G;      // samples per wave
constexpr int CSR_W = 8;                   // centres per lane and pass
static_assert(CSR_PASS == CSR_W * CSR_G, "a pass is 8 centres per lane");
constexpr int CSR_SEGP = 4096;             // sorted positions per sums block
constexpr int CSR_TD = 16384;              // sums columns per LDS tile
constexpr int CSR_SUMB = 1024;

enum { OP_PREDICT = 0, OP_FULL = 1, OP_DELTA = 2, OP_FULL_ATOMIC = 3 };

struct SliceState {
  float s1, s2;  // the slice's smallest score and the next one
};

__device__ __forceinline__ int lane_prefix64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

__device__ __forceinline__ void add_row(const int64_t *indptr,
                                        const int32_t *indices,
                                        const double *data, int64_t i, int c,
                                        int d, int k, double sign,
                                        double *acc) {
  const int64_t a = indptr[i], b = indptr[i + 1];
  for (int64_t v = a; v < b; ++v)
    atomic_add_f64(acc + (int64_t)c * d + indices[v], sign * data[v]);
  atomic_add_f64(acc + (int64_t)k * d + c, sign);
}

}  // namespace

// NP passes of 64 centres per walk over the entries (a slice wider than
// 64 * NP centres is walked again).  Slice s covers centres
// [s * ks, min(k, (s + 1) * ks)), ks a multiple of 64.  Per centre only the
// fp32 score s_j = |c_j|^2 - 2 x.c_j (one fma per stored entry); the bound
// B is one per sample (the header comment), so a lane keeps its two
// smallest scores and the index of the smallest.
template <int NP>
__global__ void __launch_bounds__(CSR_BLOCK)
    k_csr_screen(const int64_t *__restrict__ indptr,
                 const int32_t *__restrict__ indices,
                 const double *__restrict__ data, int64_t i0, int64_t m,
                 const uint16_t *__restrict__ CT, int64_t dct,
                 const float *__restrict__ cn, int k, int S, int ks,
                 const WsHeader *__restrict__ hdr,
                 SliceState *__restrict__ pst, int32_t *__restrict__ pidx,
                 float *__restrict__ pxx, float *__restrict__ pb) {
  const int lane = threadIdx.x & 63, sg = lane / CSR_G, gl = lane % CSR_G;
  const int gbase = sg * CSR_G;
  const int s = blockIdx.x % S;
  const int64_t stream = blockIdx.x / S, nstream = gridDim.x / S;
  const int64_t wv = stream * (CSR_BLOCK / 64) + (threadIdx.x >> 6);
  const int64_t nwv = nstream * (CSR_BLOCK / 64);
  const int j_lo = s * ks, j_hi = min(k, j_lo + ks);
  // this slice's d x ks block of the sliced bf16 C^T
  const uint16_t *CTs = CT + (int64_t)s * dct * ks - j_lo;
  // max_j ||c_j|| (fp64, ordered bits), rounded up to fp32
  const float cmax =
      (float)__longlong_as_double((long long)hdr->cmax_bits) * 1.000001f;
  // Software pipeline over the wave's 8-sample groups: the next group's row
  // bounds load at the start of a group, its first 2 x 8 (index, value)
  // pairs at the end, so a group's gathers wait on no other load.
  int64_t a_nx = 0, b_nx = 0;
  int pi[2] = {0, 0};
  float pv[2] = {0.f, 0.f};
  auto load_pairs = [&](int64_t a0, int64_t b0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t t = a0 + CSR_G * u + gl;
      pi[u] = t < b0 ? indices[t] : 0;
      pv[u] = t < b0 ? (float)data[t] : 0.f;
    }
  };
  {
    const int64_t q = wv * CSR_SPW + sg;
    if (q < m) {
      a_nx = indptr[i0 + q];
      b_nx = indptr[i0 + q + 1];
    }
    load_pairs(a_nx, b_nx);
  }
  for (int64_t q0 = wv * CSR_SPW; q0 < m; q0 += nwv * CSR_SPW) {
    const int64_t q = q0 + sg;
    const bool live = q < m;
    const int64_t a = a_nx, b = b_nx;
    const int ci[2] = {pi[0], pi[1]};
    const float cvv[2] = {pv[0], pv[1]};
    {
      const int64_t qn = q + nwv * CSR_SPW;
      a_nx = qn < m ? indptr[i0 + qn] : 0;
      b_nx = qn < m ? indptr[i0 + qn + 1] : 0;
    }
    const float nf = (float)(b - a);
    float s1 = INFINITY, s2 = INFINITY;
    int i1 = 0x7fffffff;
    float xx = 0.f;
    for (int jp = j_lo; jp < j_hi; jp += CSR_PASS * NP) {
      float dot[NP][CSR_W];
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int h = 0; h < CSR_W; ++h) dot[p][h] = 0.f;
      const bool first = jp == j_lo;
      for (int64_t c0 = a; c0 < b; c0 += CSR_G) {
        const int cnt = (int)min<int64_t>(CSR_G, b - c0);
        const int64_t u = (c0 - a) / CSR_G;
        int myi = 0;
        float myv = 0.f;
        if (u < 2) {  // group-uniform: the pipelined pairs
          myi = u ? ci[1] : ci[0];
          myv = u ? cvv[1] : cvv[0];
        } else if (gl < cnt) {
          myi = indices[c0 + gl];
          myv = (float)data[c0 + gl];
        }
        // the chunk's C^T row loads first, then the fmas, E entries at a
        // time from entry h (E = EM, or 2 when no group of the wave has more
        // left; EM x NP <= 16 loads in flight): lanes past a group's entries
        // hold (0, 0.0), so a shorter group's extra entries load row 0 and
        // add +-0 (a non-finite centre value leaves every sample undecided
        // anyway, through B).  No exec masks; pass blocks past the slice are
        // wave-uniform skips.
        constexpr int EM = NP >= 4 ? 2 : CSR_G;
        auto chunk = [&](auto e_tag, int h) {
          constexpr int E = decltype(e_tag)::value;
          uint4 cv[E][NP];
          float vv[E];
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const int idx = __shfl(myi, gbase + h + e, WAVE);
            vv[e] = __shfl(myv, gbase + h + e, WAVE);
            // byte offset < 2^32: d x ks bf16 per slice (csr_run checks)
            const uint16_t *row = (const uint16_t *)(
                (const char *)CTs +
                2u * (uint32_t)(idx * ks + jp + CSR_W * gl));
#pragma unroll
            for (int p = 0; p < NP; ++p) {
              const bool blk = p == 0 || jp + CSR_PASS * p < j_hi;
              cv[e][p] = blk ? *(const uint4 *)(row + CSR_PASS * p)
                             : make_uint4(0u, 0u, 0u, 0u);
            }
          }
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const float v = vv[e];
            if (first) xx = fmaf(v, v, xx);
#pragma unroll
            for (int p = 0; p < NP; ++p) {
              const uint32_t w4[4] = {cv[e][p].x, cv[e][p].y, cv[e][p].z,
                                      cv[e][p].w};
#pragma unroll
              for (int t = 0; t < 4; ++t) {  // bf16 pair -> two fp32
                dot[p][2 * t] =
                    fmaf(v, __uint_as_float(w4[t] << 16), dot[p][2 * t]);
                dot[p][2 * t + 1] = fmaf(
                    v, __uint_as_float(w4[t] & 0xffff0000u), dot[p][2 * t + 1]);
              }
            }
          }
        };
#pragma unroll
        for (int h = 0; h < CSR_G; h += EM) {
          if (h && !__any(cnt > h)) break;
          if (__any(cnt - h > 2))
            chunk(std::integral_constant<int, EM>{}, h);
          else
            chunk(std::integral_constant<int, 2>{}, h);
        }
      }
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int h = 0; h < CSR_W; ++h) {
          const int j = jp + CSR_PASS * p + CSR_W * gl + h;
          if (j < j_hi) {  // centres ascending per lane: strict < = first
            // |c_j|^2 loaded here, not before the walk: 32 VGPRs held over
            // the gathers cost a wave per SIMD
            const float sj = fmaf(-2.f, dot[p][h], cn[j]);
            if (sj < s1) {
              s2 = s1;
              s1 = sj;
              i1 = j;
            } else {
              s2 = fminf(s2, sj);
            }
          }
        }
      }
    }
    load_pairs(a_nx, b_nx);  // the next group's first 16 pairs
#pragma unroll
    for (int off = CSR_G / 2; off >= 1; off >>= 1) {
      const float o1 = __shfl_xor(s1, off, WAVE);
      const float o2 = __shfl_xor(s2, off, WAVE);
      const int oi = __shfl_xor(i1, off, WAVE);
      const bool take = o1 < s1 || (o1 == s1 && oi < i1);
      s2 = fminf(fminf(s2, o2), take ? s1 : o1);
      if (take) {
        s1 = o1;
        i1 = oi;
      }
    }
    if (live && gl == 0) {
      pst[(int64_t)s * m + q] = SliceState{s1, s2};
      pidx[(int64_t)s * m + q] = i1;
      if (s == 0) {
        // the bound of every centre of the sample (header comment): A >=
        // sum |x_v c_jv| by Cauchy-Schwarz, |c_j|^2 <= cmax^2, |s_j| <=
        // |c_j|^2 + 2A; doubled, + 2^-100 for underflow; NaN / inf: no
        // decision.  The bf16 table: 2 x (2 x b A) = 2^-6 A (1 + 2^-14)
        // with b = 2^-8 (the fp64 -> fp32 -> bf16 double rounding is in
        // the 1 + 2^-14).
        const float xx_up = xx * (1.f + (nf + 4.f) * 0x1.0p-23f);
        const float A = sqrtf(xx_up) * cmax * (1.f + 0x1.0p-20f);
        const float c2 = cmax * cmax * (1.f + 0x1.0p-22f);
        const float M = xx_up + 2.f * c2 + 4.f * A;
        const float B = (0x1.0p-6f * (1.f + 0x1.0p-14f) * A +
                         0x1.0p-23f * (2.f * c2 + 2.f * A +
                                       2.f * (nf + 2.f) * A) +
                         (2.f * nf + 6.f) * 0x1.0p-52f * M + 0x1.0p-100f) *
                        (1.f + 0x1.0p-20f);
        pxx[q] = xx * (1.f - (nf + 4.f) * 0x1.0p-23f);
        pb[q] = B;
      }
    }
  }
}

// One lane per sample: merge the slices, decide, write the label, list the
// undecided, move the rows.
__global__ void __launch_bounds__(256)
    k_csr_merge(const int64_t *__restrict__ indptr,
                const int32_t *__restrict__ indices,
                const double *__restrict__ data, int64_t i0, int64_t m, int d,
                int k, int S, const SliceState *__restrict__ pst,
                const int32_t *__restrict__ pidx,
                const float *__restrict__ pxx, const float *__restrict__ pb,
                int32_t *labels, double *acc, int op,
                int32_t *__restrict__ list, uint32_t *nlist) {
  const int lane = threadIdx.x & 63;
  for (int64_t q0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63);
       q0 < m; q0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = q0 + lane;
    bool und = false;
    if (q < m) {
      SliceState w = pst[q];
      int wi = pidx[q];
      float s2 = w.s2;  // the smallest score but the best, over the slices
      for (int sl = 1; sl < S; ++sl) {
        const SliceState t = pst[(int64_t)sl * m + q];
        const int ti = pidx[(int64_t)sl * m + q];
        if (ti != 0x7fffffff &&
            (wi == 0x7fffffff || t.s1 < w.s1 || (t.s1 == w.s1 && ti < wi))) {
          s2 = fminf(fminf(s2, w.s1), t.s2);
          w = t;
          wi = ti;
        } else {
          s2 = fminf(fminf(s2, t.s1), t.s2);
        }
      }
      const float B = pb[q];
      const float L = s2 - B;
      // every other centre's fp64 distance^2 provably exceeds the best's
      // (strictly, also after sqrt), and the clamp at 0 cannot tie them
      const bool decided =
          wi != 0x7fffffff && w.s1 + B < L && pxx[q] + L > 0.f;
      const int64_t i = i0 + q;
      const int prev = (op == OP_DELTA) ? labels[i] : -1;
      if (decided) {
        if (labels && !(op == OP_DELTA && prev == wi)) labels[i] = wi;
        if (op == OP_FULL_ATOMIC || (op == OP_DELTA && prev != wi)) {
          add_row(indptr, indices, data, i, wi, d, k, 1.0, acc);
          if (op == OP_DELTA && prev >= 0 && prev < k)
            add_row(indptr, indices, data, i, prev, d, k, -1.0, acc);
        }
      } else {
        und = true;
        if (labels) labels[i] = -(prev + 2);
      }
    }
    const uint64_t mu = __ballot(und);
    if (mu) {
      int base = 0;
      if (lane == 0) base = (int)atomicAdd(nlist, (uint32_t)__popcll(mu));
      base = __shfl(base, 0, WAVE);
      if (und) list[base + lane_prefix64(mu)] = (int32_t)q;
    }
  }
}

// A wave per undecided sample: the reference arithmetic over every centre.
__global__ void __launch_bounds__(256)
    k_csr_resolve(const int64_t *__restrict__ indptr,
                  const int32_t *__restrict__ indices,
                  const double *__restrict__ data, int64_t i0, int d,
                  const double *__restrict__ CT, int64_t ldct,
                  const double *__restrict__ yy, int k, int32_t *labels,
                  double *acc, int op, const int32_t *__restrict__ list,
                  const uint32_t *nlist, unsigned long long *total) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const uint32_t cnt = *nlist;
  if (wave == 0 && lane == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
  for (int64_t e = wave; e < (int64_t)cnt; e += nwaves) {
    const int64_t i = i0 + list[e];
    const int64_t a = indptr[i], b = indptr[i + 1];
    double xx = 0.0;
    for (int64_t v = a; v < b; ++v) xx = xx + data[v] * data[v];
    double best = INFINITY;
    int bi = 0x7fffffff;
    for (int j = lane; j < k; j += 64) {
      double dot = 0.0;
      for (int64_t v = a; v < b; ++v)
        dot = dot + data[v] * CT[(int64_t)indices[v] * ldct + j];
      double dd = -2.0 * dot;
      dd = dd + xx;
      dd = dd + yy[j];
      // np.maximum(dd, 0) keeps a NaN (sklearn's clamp), then the argmin
      // key ranks it first (np.argmin)
      const double dist = argmin_key(sqrt(dd > 0.0 || dd != dd ? dd : 0.0));
      if (dist < best || bi == 0x7fffffff) {
        best = dist;
        bi = j;
      }
    }
    wave_argmin(best, bi);
    if (bi == 0x7fffffff) bi = 0;  // k >= 1: unreachable
    const int prev = (op == OP_DELTA) ? -labels[i] - 2 : -1;
    if (lane == 0 && labels) labels[i] = bi;
    const bool add = op == OP_FULL_ATOMIC || (op == OP_DELTA && prev != bi);
    if (add) {
      for (int64_t v = a + lane; v < b; v += 64) {
        atomic_add_f64(acc + (int64_t)bi * d + indices[v], data[v]);
        if (op == OP_DELTA && prev >= 0 && prev < k)
          atomic_add_f64(acc + (int64_t)prev * d + indices[v], -data[v]);
      }
      if (lane == 0) {
        atomic_add_f64(acc + (int64_t)k * d + bi, 1.0);
        if (op == OP_DELTA && prev >= 0 && prev < k)
          atomic_add_f64(acc + (int64_t)k * d + prev, -1.0);
      }
    }
  }
}

// Full sums over label-sorted samples: a block per CSR_SEGP positions and
// column tile (blockIdx.y); 16 lanes per row add the row's entries into the
// LDS copy of the current cluster's sum, flushed at each cluster change.
__global__ void __launch_bounds__(CSR_SUMB)
    k_csr_seg_sums(const int64_t *__restrict__ indptr,
                   const int32_t *__restrict__ indices,
                   const double *__restrict__ data,
                   const int32_t *__restrict__ sorted,
                   const int32_t *__restrict__ off, int k, int d, int td,
                   double *__restrict__ acc) {
  extern __shared__ double lsum[];
  const int64_t n = off[k];
  const int64_t p0 = (int64_t)blockIdx.x * CSR_SEGP;
  if (p0 >= n) return;
  const int64_t p1 = std::min<int64_t>(n, p0 + CSR_SEGP);
  const int col0 = blockIdx.y * td;
  const int tw = min(td, d - col0);
  for (int t = threadIdx.x; t < tw; t += CSR_SUMB) lsum[t] = 0.0;
  int lo_c = 0, hi_c = k;  // off[lo_c] <= p0 < off[hi_c]
  while (hi_c - lo_c > 1) {
    const int mid = (lo_c + hi_c) >> 1;
    if (off[mid] <= p0) lo_c = mid;
    else hi_c = mid;
  }
  int c = lo_c;
  const int sub = threadIdx.x & 15, row0 = threadIdx.x >> 4;
  for (int64_t p = p0; p < p1;) {
    while (off[c + 1] <= p) ++c;  // empty clusters
    const int64_t e = std::min<int64_t>(p1, off[c + 1]);
    __syncthreads();
    for (int64_t r = p + row0; r < e; r += CSR_SUMB / 16) {
      const int64_t i = sorted[r];
      const int64_t a = indptr[i], b = indptr[i + 1];
      for (int64_t v = a + sub; v < b; v += 16) {
        const int t = indices[v] - col0;
        if (t >= 0 && t < tw)
          __hip_atomic_fetch_add(&lsum[t], data[v], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < tw; t += CSR_SUMB) {
      const double x = lsum[t];
      if (x != 0.0) {
        atomic_add_f64(acc + (int64_t)c * d + col0 + t, x);
        lsum[t] = 0.0;
      }
    }
    if (threadIdx.x == 0 && blockIdx.y == 0)
      atomic_add_f64(acc + (int64_t)k * d + c, (double)(e - p));
    p = e;
  }
}

static int csr_cus() {
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


static int csr_full_sums(const int64_t *indptr, const int32_t *indices,
                         const double *data, int64_t n, int d, int k,
                         const int32_t *labels, double *acc, const WsView &v,
                         hipStream_t st) {
  const int td = (int)std::min<int64_t>(round_up(d, 64), CSR_TD);
  const unsigned ny = (unsigned)((d + td - 1) / td);
  if (hipFuncSetAttribute((const void *)k_csr_seg_sums,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          CSR_TD * 8) != hipSuccess)
    return fail(DKM_E_LAUNCH, "csr sums: LDS attribute");
  const int64_t span = std::min<int64_t>(v.nq, INT32_MAX);
  for (int64_t lo = 0; lo < n; lo += span) {
    const int64_t hi = std::min(n, lo + span);
    if (int r = sort_by_label(labels, lo, hi, k, v, st)) return r;
    const unsigned nb =
        (unsigned)std::max<int64_t>(1, (hi - lo + CSR_SEGP - 1) / CSR_SEGP);
    k_csr_seg_sums<<<dim3(nb, ny), CSR_SUMB, (size_t)td * 8, st>>>(
        indptr, indices, data, v.sitems, v.soff, k, d, td, acc);
    if (int r = check_launch("csr sums")) return r;
  }
  return 0;
}

static int csr_run(const int64_t *indptr, const int32_t *indices,
                   const double *data, int64_t n, int64_t d, const double *C,
                   int64_t k, const void *ws, size_t wsb, int32_t *labels,
                   double *acc, int op, void *stream, const char *who) {
  if (n < 0 || d <= 0 || k <= 0 || d > INT32_MAX || k > INT32_MAX)
    return fail(DKM_E_ARG, std::string(who) + ": bad n/d/k");
  if (n == 0) return 0;
  if (!indptr || !C || (!indices && !data))
    return fail(DKM_E_ARG, std::string(who) + ": NULL input");
  (void)C;  // the kernels read C^T and |c|^2 prepared in the workspace
  WsView v;
  if (int r = ws_view(ws, wsb, k, d, &v)) return r;
  if (op == OP_FULL && (!labels || !sorted_sums_ok(k, 1, v)))
    op = OP_FULL_ATOMIC;  // no label array to sort (or k beyond the sort)
  const int S = csr_slices(k, d);
  const int ks = (int)csr_slice_width(k, d);
  if ((uint64_t)d * (uint64_t)ks * 2 > 0xffffffffull)  // 32-bit gather offsets
    return fail(DKM_E_ARG, std::string(who) + ": d x slice width beyond 4 GiB");
  // per chunk sample: S slice states (12 B), x.x and B bounds (8 B), list
  // slot (4 B)
  const int64_t chunk =
      std::min<int64_t>(n, v.nq * 12 / (12 * S + 12));
  if (chunk <= 0)
    return fail(DKM_E_WORKSPACE, std::string(who) + ": workspace too small");
  char *tail = (char *)v.queue;
  SliceState *pst = (SliceState *)tail;
  int32_t *pidx = (int32_t *)(pst + (int64_t)S * chunk);
  float *pxx = (float *)(pidx + (int64_t)S * chunk);
  float *pb = pxx + chunk;
  int32_t *list = (int32_t *)(pb + chunk);
  uint32_t *nlist = &v.hdr->csr_nund;
  hipStream_t st = (hipStream_t)stream;
  const int cu = csr_cus();
  const int npass = (ks + CSR_PASS - 1) / CSR_PASS;
  for (int64_t i0 = 0; i0 < n; i0 += chunk) {
    const int64_t m = std::min(chunk, n - i0);
    const int64_t groups = (m + CSR_SPW - 1) / CSR_SPW;
    const int64_t per_slice = std::max<int64_t>(
        1, std::min<int64_t>((int64_t)cu * 8 / S,
                             (groups + CSR_BLOCK / 64 - 1) / (CSR_BLOCK / 64)));
    const unsigned g = (unsigned)(per_slice * S);
#define DKM_SCREEN(NP)                                                       \
  k_csr_screen<NP><<<g, CSR_BLOCK, 0, st>>>(indptr, indices, data, i0, m,   \
                                            v.ctb, d,                       \
                                            v.cn32,                         \
                                            (int)k, S, ks, v.hdr, pst,      \
                                            pidx, pxx, pb)
    if (npass >= 4)
      DKM_SCREEN(4);
    else if (npass >= 2)
      DKM_SCREEN(2);
    else
      DKM_SCREEN(1);
#undef DKM_SCREEN
    if (hipMemsetAsync(nlist, 0, 4, st) != hipSuccess)
      return fail(DKM_E_LAUNCH, std::string(who) + ": memset");
    const unsigned gm = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>((m + 255) / 256, (int64_t)cu * 16));
    k_csr_merge<<<gm, 256, 0, st>>>(indptr, indices, data, i0, m, (int)d,
                                    (int)k, S, pst, pidx, pxx, pb, labels,
                                    acc, op, list, nlist);
    k_csr_resolve<<<(unsigned)cu * 4, 256, 0, st>>>(
        indptr, indices, data, i0, (int)d, v.ct64, ct_ld(k), v.cn64, (int)k,
        labels, acc, op, list, nlist,
        (unsigned long long *)&v.hdr->rechecked_total);
    if (int r = check_launch(who)) return r;
  }
  if (op == OP_FULL)
    return csr_full_sums(indptr, indices, data, n, (int)d, (int)k, labels,
                         acc, v, st);
  return 0;
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
  return csr_run(indptr, indices, data, n, d, C, k, ws, ws_bytes, labels, acc,
                 OP_FULL, stream, "dkm_partial_sum_csr_f64");
}

int dkm_assign_delta_csr_f64(const int64_t *indptr, const int32_t *indices,
                             const double *data, int64_t n, int64_t d,
                             const double *C, int64_t k, const void *ws,
                             size_t ws_bytes, int32_t *labels, double *delta,
                             void *stream) {
  if (!labels || !delta)
    return fail(DKM_E_ARG, "assign_delta_csr: labels/delta is NULL");
  return csr_run(indptr, indices, data, n, d, C, k, ws, ws_bytes, labels,
                 delta, OP_DELTA, stream, "dkm_assign_delta_csr_f64");
}

int dkm_predict_csr_f64(const int64_t *indptr, const int32_t *indices,
                        const double *data, int64_t n, int64_t d,
                        const double *C, int64_t k, const void *ws,
                        size_t ws_bytes, int32_t *labels, void *stream) {
  if (!labels) return fail(DKM_E_ARG, "predict_csr: labels is NULL");
  return csr_run(indptr, indices, data, n, d, C, k, ws, ws_bytes, labels,
                 nullptr, OP_PREDICT, stream, "dkm_predict_csr_f64");
}

}  // extern "C"

// Code-object preload (dkm_preload): the runtime loads this file's kernels
// on first use of any of them; an attribute query here does it up front.
namespace dkm {
DKM_TU_FLAGS(sparse, 0)
__global__ void k_tu_sparse() {}
int preload_sparse() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void *)k_tu_sparse) == hipSuccess ? 0
                                                                       : 1;
}
}  // namespace dkm
