// dkm_prune.hip -- samples whose label provably cannot change are not
// screened again (dkm_assign_pruned_*).
//
// The reference assigns every sample to its nearest centre every iteration
// (dislib cluster/kmeans/base.py:171-173).  Late in a fit almost no label
// changes, and the triangle inequality proves most of them in advance
// (the per-sample bounds of Hamerly, "Making k-means even faster", SDM 2010):
//   u >= d(x, c_a)            (a = the sample's label)
//   l <= d(x, c_j), j != a
// After the centres move by delta_j = |c_j' - c_j|,
//   u' = u + delta_a,  l' = l - max_{j != a} delta_j
// stay bounds, and u' < l' proves that a is still the unique nearest centre
// -- with margins that cover the reference's own fp64 rounding of the
// distances, so its argmin (first index on ties) is a as well.  Only the
// other samples ("active") are gathered into a compact block and screened
// by k_screen_b2 in bounds mode, which also returns fresh bounds for them
// (dkm_b2.hip: the hinted threshold pass raised by a margin M per row gives
// the lower bound; the kept set and the own score give the upper one).
//
// Layout of the caller's state buffer (dkm_prune_state_bytes):
//   ul    float2[n]  (u, l) per sample
//   act   int32[n]   active sample indices, ascending
//   mask  uint64[ceil(n / 64)] active bits
//   bcnt  int64[nb + 1] per-range active counts -> exclusive offsets
//   drift float[kpad32] + stats (max, second max, argmax)
//   xa    TX[cap x d] gathered rows, la int32[cap], bnd float4[cap]
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dkm_internal.h"

namespace dkm {

constexpr int PR_BLOCK = 256;
constexpr int64_t PR_RANGE = 16384;  // rows per compaction range (one block)

static int prune_cus() {
  int dev = 0, n = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
          hipSuccess)
    n = 256;
  return n;
}

static int64_t prune_cap(int64_t n) {
  // gathered rows per chunk: an eighth of the data, at least 1M (or n)
  int64_t c = std::max<int64_t>((int64_t)1 << 20, n / 8);
  c = std::min<int64_t>(c, n);
  return std::max<int64_t>(32, round_up(c, 32));
}

size_t prune_state_bytes(int64_t n, int64_t k, int64_t d) {
  const int64_t nb = (n + PR_RANGE - 1) / PR_RANGE;
  const int64_t cap = prune_cap(n);
  size_t b = 0;
  b += round_up(n * 8, 256);                    // ul
  b += round_up(n * 4, 256);                    // act
  b += round_up((n + 63) / 64 * 8, 256);        // mask
  b += round_up((nb + 1) * 8, 256);             // bcnt
  b += round_up(round_up(k, 32) * 4 + 64, 256); // drift + stats
  b += round_up(cap * d * 8, 256);              // xa (fp64 worst case)
  b += round_up(cap * 4, 256);                  // la
  b += round_up(cap * 16, 256);                 // bnd
  return b;
}

PruneView prune_view(void *state, int64_t n, int64_t k, int64_t d) {
  PruneView p;
  char *q = (char *)state;
  const int64_t nb = (n + PR_RANGE - 1) / PR_RANGE;
  p.n = n;
  p.nb = nb;
  p.cap = prune_cap(n);
  p.ul = (float2 *)q;
  q += round_up(n * 8, 256);
  p.act = (int32_t *)q;
  q += round_up(n * 4, 256);
  p.mask = (uint64_t *)q;
  q += round_up((n + 63) / 64 * 8, 256);
  p.bcnt = (int64_t *)q;
  q += round_up((nb + 1) * 8, 256);
  p.drift = (float *)q;
  p.dstat = p.drift + round_up(k, 32);
  q += round_up(round_up(k, 32) * 4 + 64, 256);
  p.xa = q;
  q += round_up(p.cap * d * 8, 256);
  p.la = (int32_t *)q;
  q += round_up(p.cap * 4, 256);
  p.bnd = (float4 *)q;
  return p;
}

// an fp32 value >= x (round to nearest, then one ulp up when below)
__device__ __forceinline__ float f32_up(double x) {
  const float f = (float)x;  // x >= 0 here
  return (double)f >= x ? f : __uint_as_float(__float_as_uint(f) + 1u);
}

// delta_j = |C_j - Cp_j| (fp64, then rounded up with a 2^-20 margin); the
// largest two and the argmax.  One block: k x d is small.
__global__ void __launch_bounds__(1024)
    k_drift(const double *__restrict__ C, const double *__restrict__ Cp,
            int64_t k, int64_t d, float *__restrict__ drift,
            float *__restrict__ dstat) {
  __shared__ float s1[1024], s2[1024];
  __shared__ int sj[1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float m1 = 0.f, m2 = 0.f;
  int j1 = -1;
  for (int64_t c = w; c < k; c += 16) {
    double a = 0.0;
    for (int64_t f = lane; f < d; f += 64) {
      const double t = C[c * d + f] - Cp[c * d + f];
      a = fma(t, t, a);
    }
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    float dl = f32_up(sqrt(a));
    dl = dl + dl * 0x1.0p-20f;
    if (!(dl < INFINITY)) dl = INFINITY;  // NaN centres: nothing prunes
    if (lane == 0) drift[c] = dl;
    if (dl > m1) {
      m2 = m1;
      m1 = dl;
      j1 = (int)c;
    } else if (dl > m2) {
      m2 = dl;
    }
  }
  s1[threadIdx.x] = m1;
  s2[threadIdx.x] = m2;
  sj[threadIdx.x] = j1;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b1 = 0.f, b2 = 0.f;
    int bj = -1;
    for (int t = 0; t < 1024; t += 64) {  // one entry per wave (lane 0)
      const float a1 = s1[t], a2 = s2[t];
      if (a1 > b1) {
        b2 = fmaxf(b1, a2);
        b1 = a1;
        bj = sj[t];
      } else {
        b2 = fmaxf(b2, a1);
      }
    }
    dstat[0] = b1;
    dstat[1] = b2;
    dstat[2] = __int_as_float(bj);
  }
}

__device__ __forceinline__ float up_m(float x) { return x + fabsf(x) * 0x1.0p-20f; }
__device__ __forceinline__ float dn_m(float x) { return x - fabsf(x) * 0x1.0p-20f; }

// Bounds after the centre move, and the active bits: block b owns rows
// [b PR_RANGE, (b + 1) PR_RANGE); bcnt[b] = its active count.  Two tiers:
// (1) u + delta_a < l - max_{j != a} delta_j; (2) for the rows that fail
// it, the exact distance to the current c_a (fp64, 8 lanes per row)
// replaces u -- the screen's u carries the bf16 bound, the exact one does
// not, and once stored it keeps most rows in tier 1.
template <class TX>
__global__ void __launch_bounds__(PR_BLOCK)
    k_prune(const TX *__restrict__ X, int64_t ldx, int d,
            const double *__restrict__ C, const int32_t *__restrict__ lab,
            int64_t n, int64_t k, const float *__restrict__ drift,
            const float *__restrict__ dstat, float2 *__restrict__ ul,
            uint64_t *__restrict__ mask, int64_t *__restrict__ bcnt) {
  __shared__ int cnt;
  __shared__ int2 fl[PR_BLOCK / 64][64];    // (row, label) of tier-1 fails
  __shared__ float flo[PR_BLOCK / 64][64];  // their moved lower bound
  __shared__ int fok[PR_BLOCK / 64][64];    // tier 2 passed
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float dmax = dstat[0], d2 = dstat[1];
  const int jmax = __float_as_int(dstat[2]);
  const int64_t r0 = (int64_t)blockIdx.x * PR_RANGE;
  const int64_t r1 = std::min<int64_t>(n, r0 + PR_RANGE);
  int mine = 0;
  for (int64_t i0 = r0; i0 < r1; i0 += PR_BLOCK) {
    const int64_t i = i0 + threadIdx.x;
    bool valid = false, pass = false;
    int a = -1;
    float l = 0.f;
    if (i < r1) {
      a = lab[i];
      if (a >= 0 && a < k) {
        valid = true;
        const float2 b = ul[i];
        const float u = up_m(b.x + drift[a]);
        l = dn_m(b.y - (a == jmax ? d2 : dmax));
        // strict, with one more margin each side; NaN fails
        pass = up_m(u) < dn_m(l);
        ul[i] = make_float2(u, l);
      }
    }
    const bool fail = valid && !pass;
    const uint64_t fm = __ballot(fail);
    const int nf = __popcll(fm);
    const int pos = __popcll(fm & ((1ull << lane) - 1ull));
    if (fail) {
      fl[w][pos] = make_int2((int)(i - r0), a);
      flo[w][pos] = l;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int g = lane >> 3, sub = lane & 7;
    for (int q = 0; q < nf; q += 8) {
      const int e = q + g;
      double acc = 0.0;
      int2 ra = make_int2(0, 0);
      if (e < nf) {
        ra = fl[w][e];
        const TX *xr = X + (r0 + ra.x) * ldx;
        const double *cr = C + (int64_t)ra.y * d;
#pragma unroll 4
        for (int f = sub; f < d; f += 8) {
          const double t = (double)xr[f] - cr[f];
          acc = fma(t, t, acc);
        }
      }
      acc += __shfl_xor(acc, 1, 64);
      acc += __shfl_xor(acc, 2, 64);
      acc += __shfl_xor(acc, 4, 64);
      if (e < nf && sub == 0) {
        // sum of d squares in fp64: within (d + 2) 2^-53 of the exact one
        float ue = f32_up(sqrt(acc * (1.0 + 0x1.0p-40)));
        ue = ue + ue * 0x1.0p-20f;
        const float lp = flo[w][e];
        const bool ok = up_m(ue) < dn_m(lp);
        fok[w][e] = ok;
        if (ok) ul[r0 + ra.x] = make_float2(ue, lp);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool active = i < r1 && (!valid || (fail && !fok[w][pos]));
    const uint64_t m = __ballot(active);
    if (lane == 0 && i0 + 64 * w < r1) mask[(i0 + 64 * w) >> 6] = m;
    mine += active;
  }
  atomicAdd(&cnt, mine);
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = cnt;
}

// exclusive scan of the nb range counts (one block); bcnt[nb] = total
__global__ void __launch_bounds__(1024)
    k_prune_scan(int64_t *__restrict__ bcnt, int64_t nb) {
  __shared__ int64_t part[1024];
  const int64_t per = (nb + 1023) / 1024;
  const int64_t a = (int64_t)threadIdx.x * per, b = std::min(nb, a + per);
  int64_t s = 0;
  for (int64_t i = a; i < b; ++i) s += bcnt[i];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int i = 0; i < 1024; ++i) {
      const int64_t v = part[i];
      part[i] = t;
      t += v;
    }
    bcnt[nb] = t;
  }
  __syncthreads();
  int64_t o = part[threadIdx.x];
  for (int64_t i = a; i < b; ++i) {
    const int64_t v = bcnt[i];
    bcnt[i] = o;
    o += v;
  }
}

// active indices in ascending order: range b writes from offset bcnt[b]
__global__ void __launch_bounds__(PR_BLOCK)
    k_prune_compact(int64_t n, const uint64_t *__restrict__ mask,
                    const int64_t *__restrict__ bcnt, int32_t *__restrict__ act) {
  __shared__ int wc[PR_BLOCK / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * PR_RANGE;
  const int64_t r1 = std::min<int64_t>(n, r0 + PR_RANGE);
  int64_t off = bcnt[blockIdx.x];
  for (int64_t i0 = r0; i0 < r1; i0 += PR_BLOCK) {
    const int64_t iw = i0 + 64 * w;
    const uint64_t m = iw < r1 ? mask[iw >> 6] : 0ull;
    if (lane == 0) wc[w] = __popcll(m);
    __syncthreads();
    int before = 0, tot = 0;
    for (int t = 0; t < PR_BLOCK / 64; ++t) {
      before += t < w ? wc[t] : 0;
      tot += wc[t];
    }
    if ((m >> lane) & 1ull)
      act[off + before + __popcll(m & ((1ull << lane) - 1ull))] =
          (int32_t)(iw + lane);
    off += tot;
    __syncthreads();
  }
}

// gathered rows: xa[j] = X[act[j]] (d elements), la[j] = lab[act[j]]
template <class TX>
__global__ void __launch_bounds__(PR_BLOCK)
    k_prune_gather(const TX *__restrict__ X, int64_t ldx, int d,
                   const int32_t *__restrict__ act, int64_t m,
                   TX *__restrict__ xa, const int32_t *__restrict__ lab,
                   int32_t *__restrict__ la) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * (PR_BLOCK / 64) + (threadIdx.x >> 6);
  const int64_t step = (int64_t)gridDim.x * (PR_BLOCK / 64);
  for (int64_t j = w0; j < m; j += step) {
    const int64_t i = act[j];
    const TX *src = X + i * ldx;
    TX *dst = xa + j * d;
    for (int f = lane; f < d; f += 64) dst[f] = src[f];
    if (lane == 0) la[j] = lab[i];
  }
}

// fresh bounds (and, gathered, the labels) back to the samples
__global__ void __launch_bounds__(PR_BLOCK)
    k_prune_final(const int32_t *__restrict__ act, int64_t j0, int64_t m,
                  const int32_t *__restrict__ la, const float4 *__restrict__ bnd,
                  int32_t *__restrict__ lab, float2 *__restrict__ ul) {
  const int64_t j = (int64_t)blockIdx.x * PR_BLOCK + threadIdx.x;
  if (j >= m) return;
  const int64_t i = act ? act[j0 + j] : j0 + j;
  const int w = la[j];
  const float4 b = bnd[j];
  const float l = w == __float_as_int(b.w) ? b.y : b.z;
  ul[i] = make_float2(b.x, l);
  if (act) lab[i] = w;
}

template <class TX>
int launch_prune(const TX *X, int64_t ldx, const double *C, const double *Cp,
                 int64_t k, int64_t d, const int32_t *lab, const PruneView &p,
                 hipStream_t s) {
  k_drift<<<1, 1024, 0, s>>>(C, Cp, k, d, p.drift, p.dstat);
  k_prune<TX><<<(unsigned)p.nb, PR_BLOCK, 0, s>>>(X, ldx, (int)d, C, lab, p.n,
                                                  k, p.drift, p.dstat, p.ul,
                                                  p.mask, p.bcnt);
  k_prune_scan<<<1, 1024, 0, s>>>(p.bcnt, p.nb);
  k_prune_compact<<<(unsigned)p.nb, PR_BLOCK, 0, s>>>(p.n, p.mask, p.bcnt,
                                                      p.act);
  return check_launch("prune");
}

template <class TX>
int launch_prune_gather(const TX *X, int64_t ldx, int d, const PruneView &p,
                        int64_t j0, int64_t m, const int32_t *lab,
                        hipStream_t s) {
  const int64_t g = std::max<int64_t>(
      1, std::min<int64_t>((m + 3) / 4, (int64_t)prune_cus() * 16));
  k_prune_gather<TX><<<(unsigned)g, PR_BLOCK, 0, s>>>(
      X, ldx, d, p.act + j0, m, (TX *)p.xa, lab, p.la);
  return check_launch("prune gather");
}

int launch_prune_final(bool gathered, const PruneView &p, int64_t j0,
                       int64_t m, const int32_t *la, int32_t *lab,
                       hipStream_t s) {
  k_prune_final<<<(unsigned)((m + PR_BLOCK - 1) / PR_BLOCK), PR_BLOCK, 0, s>>>(
      gathered ? p.act : nullptr, j0, m, la, p.bnd, lab, p.ul);
  return check_launch("prune bounds");
}

template int launch_prune<double>(const double *, int64_t, const double *,
                                  const double *, int64_t, int64_t,
                                  const int32_t *, const PruneView &,
                                  hipStream_t);
template int launch_prune<float>(const float *, int64_t, const double *,
                                 const double *, int64_t, int64_t,
                                 const int32_t *, const PruneView &,
                                 hipStream_t);
template int launch_prune_gather<double>(const double *, int64_t, int,
                                         const PruneView &, int64_t, int64_t,
                                         const int32_t *, hipStream_t);
template int launch_prune_gather<float>(const float *, int64_t, int,
                                        const PruneView &, int64_t, int64_t,
                                        const int32_t *, hipStream_t);

}  // namespace dkm
