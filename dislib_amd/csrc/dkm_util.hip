// dkm_util.hip -- error plumbing, workspace, centre preparation, centre
// update + convergence criterion, synthetic blob generator.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "dkm_internal.h"

namespace dkm {

static thread_local std::string g_err;

void set_error(const std::string &msg) { g_err = msg; }

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

int check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return fail((int)e, std::string(what) + ": " + hipGetErrorString(e));
  return 0;
}

int64_t default_queue(int64_t k, int64_t d) {
  (void)k;
  (void)d;
  return int64_t(1) << 22;  // 4M re-check slots (16 MB); overflow -> inline
}

// GEMM screen regions (gemm_path only)
static size_t gemm_bytes(int64_t k, int64_t d) {
  if (!gemm_path(k, d)) return 0;
  const int64_t kp = kpad256(k), dp = dpad32(d), m = gemm_chunk(d);
  size_t b = 0;
  b += round_up(kp * dp * 4, 256);              // gfrag
  b += round_up(kp * dp * 2, 256);              // gfrag1
  b += round_up(kp * 4, 256);                   // gcn
  b += 2 * round_up(m * dp * 4, 256);           // gxs (two chunks)
  b += 2 * round_up(m * 4, 256);                // gxn (two chunks)
  b += round_up(m * (kp / GT) * GTOP * 8, 256); // gpart
  return b;
}

size_t ws_bytes(int64_t k, int64_t d, int64_t n_queue) {
  if (n_queue <= 0) n_queue = default_queue(k, d);
  const int64_t dpad = round_up(d, 4);
  size_t b = WS_HDR;
  b += round_up(k * dpad * 4, 256);   // c32
  b += round_up(k * 4, 256);          // cn32
  b += round_up(k * 8, 256);          // cn64
  b += round_up(ct_ld(k) * d * 8, 256);  // ct64 (d x ct_ld(k))
  b += round_up(csr_ctb_len(k, d) * 2, 256);  // ctb (sliced bf16)
  b += round_up(kpad16(k) * dpad32(d) * 4, 256);  // cfrag
  b += round_up(kpad16(k) * 4, 256);  // cnpad
  b += round_up(kpad16(k) * dpad32(d) * 4, 256);  // bfrag (hi + lo bf16)
  b += round_up(kpad32(k) * 32 * 4, 256);         // b32frag
  b += round_up(kpad32(k) * 4, 256);              // cn32f
  b += (size_t)TL_SEGS * TL_CAP * 8;  // tlist
  b += (size_t)TL_SEGS * 4;           // tcount
  if (mind_ok(k, d)) b += round_up(k * MIND_LD * 4, 256);  // mind
  b += gemm_bytes(k, d);
  if (b1_ok(k, d)) {
    b += round_up(kpad32(k) * dpad16(d) * 2, 256);  // b1frag
    b += round_up(kpad32(k) * dpad16(d) * 2, 256);  // b1frag_t
    b += round_up(kpad32(k) * dpad16(d) * 2, 256);  // b1frag_lo
    b += round_up(d * 4, 256);                      // mvec
    b += (size_t)B1_SEGS * B1_CAP * 8;              // clist
    b += (size_t)B1_SEGS * 4;                       // ccount
    b += (size_t)B1_SEGS * B1_NCAP * 16;            // nlist
    b += (size_t)B1_SEGS * 4;                       // ncount
  }
  if (rescreen_ok(k, d)) {
    b += (size_t)TL_SEGS * TL_CAP * 8;              // rlist
    b += (size_t)TL_SEGS * 4;                       // rprefix
    b += (size_t)RS_ROWS * 4;                       // rlab
    b += (size_t)RS_ROWS * d * 8;                   // rx
  }
  if (k <= SORT_KMAX) b += round_up((k + 1) * 4, 256) + 2 * round_up(k * 4, 256);
  b += 3 * round_up(n_queue * 4, 256);  // queue, sitems, smoved
  return b;
}

int ws_view(const void *ws, size_t bytes, int64_t k, int64_t d, WsView *v) {
  if (!ws) return fail(DKM_E_ARG, "workspace is NULL");
  const int64_t dpad = round_up(d, 4);
  char *p = (char *)ws;
  v->hdr = (WsHeader *)p;
  p += WS_HDR;
  v->c32 = (float *)p;
  p += round_up(k * dpad * 4, 256);
  v->cn32 = (float *)p;
  p += round_up(k * 4, 256);
  v->cn64 = (double *)p;
  p += round_up(k * 8, 256);
  v->ct64 = (double *)p;
  p += round_up(ct_ld(k) * d * 8, 256);
  v->ctb = (uint16_t *)p;
  p += round_up(csr_ctb_len(k, d) * 2, 256);
  v->cfrag = (float *)p;
  p += round_up(kpad16(k) * dpad32(d) * 4, 256);
  v->cnpad = (float *)p;
  p += round_up(kpad16(k) * 4, 256);
  v->bfrag = (uint16_t *)p;
  p += round_up(kpad16(k) * dpad32(d) * 4, 256);
  v->b32frag = (uint16_t *)p;
  p += round_up(kpad32(k) * 32 * 4, 256);
  v->cn32f = (float *)p;
  p += round_up(kpad32(k) * 4, 256);
  v->tlist = (int2 *)p;
  p += (size_t)TL_SEGS * TL_CAP * 8;
  v->tcount = (int32_t *)p;
  p += (size_t)TL_SEGS * 4;
  v->mind = nullptr;
  if (mind_ok(k, d)) {
    v->mind = (float *)p;
    p += round_up(k * MIND_LD * 4, 256);
  }
  v->gfrag = nullptr;
  v->gfrag1 = nullptr;
  v->gcn = nullptr;
  v->gxs = nullptr;
  v->gxn = nullptr;
  v->gxs1 = nullptr;
  v->gxn1 = nullptr;
  v->gpart = nullptr;
  v->gchunk = 0;
  v->b1frag = nullptr;
  v->b1frag_t = nullptr;
  v->b1frag_lo = nullptr;
  v->mvec = nullptr;
  v->clist = nullptr;
  v->ccount = nullptr;
  v->nlist = nullptr;
  v->ncount = nullptr;
  if (gemm_path(k, d)) {
    const int64_t kp = kpad256(k), dp = dpad32(d), m = gemm_chunk(d);
    v->gchunk = m;
    v->gfrag = p;
    p += round_up(kp * dp * 4, 256);
    v->gfrag1 = p;
    p += round_up(kp * dp * 2, 256);
    v->gcn = (float *)p;
    p += round_up(kp * 4, 256);
    v->gxs = p;
    p += round_up(m * dp * 4, 256);
    v->gxs1 = p;
    p += round_up(m * dp * 4, 256);
    v->gxn = (float *)p;
    p += round_up(m * 4, 256);
    v->gxn1 = (float *)p;
    p += round_up(m * 4, 256);
    v->gpart = (int2 *)p;
    p += round_up(m * (kp / GT) * GTOP * 8, 256);
  }
  if (b1_ok(k, d)) {
    v->b1frag = (uint16_t *)p;
    p += round_up(kpad32(k) * dpad16(d) * 2, 256);
    v->b1frag_t = (uint16_t *)p;
    p += round_up(kpad32(k) * dpad16(d) * 2, 256);
    v->b1frag_lo = (uint16_t *)p;
    p += round_up(kpad32(k) * dpad16(d) * 2, 256);
    v->mvec = (float *)p;
    p += round_up(d * 4, 256);
    v->clist = (int2 *)p;
    p += (size_t)B1_SEGS * B1_CAP * 8;
    v->ccount = (int32_t *)p;
    p += (size_t)B1_SEGS * 4;
    v->nlist = (int4 *)p;
    p += (size_t)B1_SEGS * B1_NCAP * 16;
    v->ncount = (int32_t *)p;
    p += (size_t)B1_SEGS * 4;
  }
  v->rlist = nullptr;
  v->rprefix = nullptr;
  v->rlab = nullptr;
  v->rx = nullptr;
  if (rescreen_ok(k, d)) {
    v->rlist = (int2 *)p;
    p += (size_t)TL_SEGS * TL_CAP * 8;
    v->rprefix = (int32_t *)p;
    p += (size_t)TL_SEGS * 4;
    v->rlab = (int32_t *)p;
    p += (size_t)RS_ROWS * 4;
    v->rx = (void *)p;
    p += (size_t)RS_ROWS * d * 8;
  }
  v->soff = v->scur = v->scnt = nullptr;
  if (k <= SORT_KMAX) {
    v->soff = (int32_t *)p;
    p += round_up((k + 1) * 4, 256);
    v->scur = (int32_t *)p;
    p += round_up(k * 4, 256);
    v->scnt = (int32_t *)p;
    p += round_up(k * 4, 256);
  }
  const size_t fixed = (size_t)(p - (char *)ws);
  if (bytes < fixed + 768)
    return fail(DKM_E_WORKSPACE, "workspace too small for k/d");
  v->nq = (int64_t)((bytes - fixed) / 12) / 64 * 64;
  v->queue = (int32_t *)p;
  v->sitems = v->queue + v->nq;
  v->smoved = v->sitems + v->nq;
  return 0;
}

// ---------------------------------------------------------------------------
// prepare: header + fp32 centres + norms + cmax
// ---------------------------------------------------------------------------
__global__ void k_ws_header(WsHeader *h, int64_t k, int64_t d, int64_t dpad,
                            int64_t n_queue) {
  if (threadIdx.x == 0) {
    h->magic = WS_MAGIC;
    h->k = k;
    h->d = d;
    h->dpad = dpad;
    h->n_queue = n_queue;
    h->cmax_bits = 0;
    h->umax_bits = 0;
    h->qcount = 0;  // rechecked_total accumulates over the workspace life
  }
}

// one 256-thread block per centre
constexpr int SEQ_CHUNK = 2048;  // row values staged in LDS per sequential pass
__global__ void __launch_bounds__(256) k_prepare(const double *__restrict__ C,
                                                 int64_t k, int64_t d,
                                                 int64_t dpad, int flags,
                                                 WsView v) {
  __shared__ double srow[SEQ_CHUNK];
  const int64_t c = blockIdx.x;
  const double *row = C + c * d;
  const int64_t ld = ct_ld(k);
  // the CSR screen's sliced bf16 C^T: slice c / w, column c % w; round to
  // nearest (fp64 -> fp32 -> bf16: within 2^-8 (1 + 2^-14) relative, the
  // bound's term)
  const int64_t w = csr_slice_width(k, d);
  uint16_t *ctbs = v.ctb + (c / w) * d * w + (c % w);
  for (int64_t t = threadIdx.x; t < dpad; t += blockDim.x) {
    const double val = t < d ? row[t] : 0.0;
    v.c32[c * dpad + t] = (float)val;
    if (t < d) {
      v.ct64[t * ld + c] = val;  // C^T: re-check, CSR
      ctbs[t * w] = __builtin_bit_cast(uint16_t, (__bf16)(float)val);
    }
  }
  // sequential over t: sklearn row_norms(squared=True) order
  // (utils/sparsefuncs_fast.pyx:26-44); exact zeros change nothing.  The
  // row goes through LDS in chunks so that the one summing lane reads it
  // at LDS latency, not HBM latency.
  double n2 = 0.0;
  for (int64_t t0 = 0; t0 < d; t0 += SEQ_CHUNK) {
    const int m = (int)(d - t0 < SEQ_CHUNK ? d - t0 : SEQ_CHUNK);
    __syncthreads();
    for (int t = threadIdx.x; t < m; t += blockDim.x) srow[t] = row[t0 + t];
    __syncthreads();
    if (threadIdx.x == 0)
      for (int t = 0; t < m; ++t) n2 = n2 + srow[t] * srow[t];
  }
  if (threadIdx.x == 0) {
    v.cn64[c] = n2;
    v.cn32[c] = (float)n2;
    const double nrm = sqrt(n2);
    // non-negative doubles order like their bit patterns
    atomicMax((unsigned long long *)&v.hdr->cmax_bits,
              (unsigned long long)__double_as_longlong(nrm));
  }
  if (v.mvec) {
    // ||c - m|| for DKM_MODE_TRANSLATE's bound (any order: it bounds the
    // bf16 operands' magnitudes, rounded up by the kernels' 1.000001)
    __syncthreads();
    double u2 = 0.0;
    for (int64_t t = threadIdx.x; t < d; t += blockDim.x) {
      const double u = row[t] - (double)v.mvec[t];
      u2 += u * u;
    }
    srow[threadIdx.x] = u2;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
      if (threadIdx.x < off) srow[threadIdx.x] += srow[threadIdx.x + off];
      __syncthreads();
    }
    if (threadIdx.x == 0)
      atomicMax((unsigned long long *)&v.hdr->umax_bits,
                (unsigned long long)__double_as_longlong(
                    sqrt(srow[0]) * (1.0 + 0x1.0p-40)));
  }
}

// DKM_MODE_TRANSLATE's m: the centres' mean per feature, rounded to fp32
// (any m keeps the screen exact; the mean makes max ||c - m|| small)
// A block per group of 32 features, its 8 waves' lanes over the centres
// (one feature a lane group of 8 rows: a lane per feature walking all k
// centres took 0.24 ms per C3 iteration, latency-bound).
__global__ void __launch_bounds__(256) k_mvec(const double *__restrict__ C,
                                              int64_t k, int64_t d,
                                              float *__restrict__ m) {
  __shared__ double part[8][32];
  const int f = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t t = (int64_t)blockIdx.x * 32 + f;
  double a = 0.0;
  if (t < d)
    for (int64_t c0 = g; c0 < k; c0 += 64) {  // 8 loads in flight a lane
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t c = c0 + 8 * u;
        x[u] = c < k ? C[c * d + t] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) a += x[u];
    }
  part[g][f] = a;
  __syncthreads();
  if (g == 0 && t < d) {
    double s = 0.0;
    for (int i = 0; i < 8; ++i) s += part[i][f];
    m[t] = (float)(s / (double)k);
  }
}

// Centres in MFMA A-fragment order (dkm_dense k_screen), pre-scaled by -2
// (exact) so that the MFMA chain started from |c|^2 yields the score
// |c|^2 - 2 x.c directly.  Block (cb, ks) = 16 centres x 32 features = 2 KB.
// Lane l of a wave stands for centre cb*16 + (l & 15) and features
// ks*32 + 8*(l >> 4) + m, m = 0..7:
//  cfrag: 8 fp32 at l*32 B (v_mfma_f32_16x16x4_f32, k-step m);
//  bfrag: 8 bf16 hi at l*16 B, 8 bf16 lo at 1024 + l*16 B
//         (v_mfma_f32_16x16x32_bf16).
// Zero padded; cnpad = 2^100 for padding centres (finite: the screen packs
// centre indices into the low mantissa bits of the scores).
__global__ void __launch_bounds__(256) k_frag(const double *__restrict__ C,
                                              int64_t k, int64_t d, WsView v) {
  const int64_t nkb = kpad16(k) / 16, nks = dpad32(d) / 32;
  const int64_t total = nkb * nks * 512;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t blk = e >> 9, w = e & 511;
    const int64_t cb = blk / nks, ks = blk - cb * nks;
    const int l = (int)(w >> 3), m = (int)(w & 7);
    const int64_t c = cb * 16 + (l & 15);
    const int64_t t = ks * 32 + 8 * (l >> 4) + m;
    const double x = (c < k && t < d) ? -2.0 * C[c * d + t] : 0.0;
    v.cfrag[blk * 512 + l * 8 + m] = (float)x;
    // bf16x3 split of x = -2c: x = hi + lo + O(2^-16 |x|), hi = bf16(x),
    // lo = bf16(x - hi)
    const __bf16 hi = (__bf16)(float)x;
    const __bf16 lo = (__bf16)(float)(x - (double)(float)hi);
    uint16_t *dst = v.bfrag + blk * 1024;
    dst[l * 8 + m] = __builtin_bit_cast(uint16_t, hi);
    dst[512 + l * 8 + m] = __builtin_bit_cast(uint16_t, lo);
  }
  const int64_t kp = kpad16(k);
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < kp;
       c += (int64_t)gridDim.x * blockDim.x)
    v.cnpad[c] = c < k ? v.cn32[c] : 0x1.0p100f;
  const int64_t nb32 = kpad32(k) / 32;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       e < nb32 * 32; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cb = e >> 5;
    const int hh = (int)((e >> 4) & 1), g = (int)(e & 15);
    const int64_t c = cb * 32 + (g & 3) + 8 * (g >> 2) + 4 * hh;
    v.cn32f[e] = c < k ? v.cn32[c] : 0x1.0p100f;
  }
  if (v.b1frag) {
    // k_screen_b1: block cb, K-step ks (16 features), lane l = (r, h),
    // element j <- bf16(-2 c[cb*32 + r][16 ks + 8 h + j]); 1 KB per (cb, ks)
    const int64_t nk16 = dpad16(d) / 16;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
         e < nb32 * nk16 * 512; e += (int64_t)gridDim.x * blockDim.x) {
      const int64_t blk = e >> 9;
      const int w = (int)(e & 511), l = w >> 3, j = w & 7;
      const int64_t cb = blk / nk16, ks = blk - cb * nk16;
      const int64_t c = cb * 32 + (l & 31);
      const int64_t t = 16 * ks + 8 * (l >> 5) + j;
      const double x = (c < k && t < d) ? -2.0 * C[c * d + t] : 0.0;
      const __bf16 hi = (__bf16)(float)x;
      v.b1frag[blk * 512 + l * 8 + j] = __builtin_bit_cast(uint16_t, hi);
      // the bf16x3 low part in the same order (k_screen_c32)
      v.b1frag_lo[blk * 512 + l * 8 + j] = __builtin_bit_cast(
          uint16_t, (__bf16)(float)(x - (double)(float)hi));
      // the translated centres: -2 (c - m) rounded the same way
      const double xt =
          (c < k && t < d) ? -2.0 * (C[c * d + t] - (double)v.mvec[t]) : 0.0;
      v.b1frag_t[blk * 512 + l * 8 + j] =
          __builtin_bit_cast(uint16_t, (__bf16)(float)xt);
    }
  }
  if (d > 32) return;
  // 32x32x16 order (k_screen_w32): block cb, K-slice ks, lane l = (r, h),
  // element j <- -2 c[cb*32 + r][16h + 8ks + j]; |c|^2 of accumulator
  // register g of lane half h = centre cb*32 + (g & 3) + 8 (g >> 2) + 4h
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       e < nb32 * 1024; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cb = e >> 10, w = e & 1023;
    const int ks = (int)(w >> 9), l = (int)((w >> 3) & 63), j = (int)(w & 7);
    const int64_t c = cb * 32 + (l & 31);
    const int64_t t = 16 * (l >> 5) + 8 * ks + j;
    const double x = (c < k && t < d) ? -2.0 * C[c * d + t] : 0.0;
    const __bf16 hi = (__bf16)(float)x;
    const __bf16 lo = (__bf16)(float)(x - (double)(float)hi);
    uint16_t *dst = v.b32frag + (cb * 2 + ks) * 1024;
    dst[l * 8 + j] = __builtin_bit_cast(uint16_t, hi);
    dst[512 + l * 8 + j] = __builtin_bit_cast(uint16_t, lo);
  }
}

// Block-skip table of k_screen_b2 (IMG_SORTED): one block per centre p,
// mind[p][cb] = a lower bound on min_{j in block cb, j != p, j < k}
// |c_p - c_j|.  The fp64 distance is within (d + 4) 2^-53 of the true one
// (d <= 128); 2^-40 and the fp32 round-down keep the stored value below it.
// A NaN centre gives NaN entries, which never clear a block.
__global__ void __launch_bounds__(256) k_mind(const double *__restrict__ C,
                                              int64_t k, int64_t d,
                                              float *__restrict__ mind) {
  const int64_t p = blockIdx.x;
  const int64_t nkb = (k + 31) / 32;
  for (int64_t j0 = 0; j0 < nkb * 32; j0 += 256) {
    const int64_t j = j0 + threadIdx.x;
    double dist = INFINITY;
    if (j < k && j != p) {
      double a = 0.0;
      for (int64_t t = 0; t < d; ++t) {
        const double df = C[p * d + t] - C[j * d + t];
        a = fma(df, df, a);
      }
      dist = sqrt(a) * (1.0 - 0x1.0p-40);
    }
    // min over the 32 lanes of the block (NaN-propagating)
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) {
      const double o = __shfl_xor(dist, off, 32);
      dist = (o != o || o < dist) ? o : dist;
    }
    if ((threadIdx.x & 31) == 0 && j < nkb * 32)
      mind[p * MIND_LD + (j >> 5)] = __double2float_rd(dist);
  }
  for (int64_t cb = nkb + threadIdx.x; cb < MIND_LD; cb += 256)
    mind[p * MIND_LD + cb] = INFINITY;
}

// ---------------------------------------------------------------------------
// update: C[c] = sums/counts (counts != 0), per-centre shift, criterion
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_update(const double *__restrict__ acc,
                                                double *__restrict__ C,
                                                int64_t k, int64_t d, int mode,
                                                double *__restrict__ shift) {
  const int64_t c = blockIdx.x;
  const double cnt = acc[k * d + c];
  __shared__ double red[256];
  double ss = 0.0;
  if (mode == DKM_SUMS_RECIP) {
    // sparse criterion (sklearn euclidean_distances, sequential sums):
    // computed from old and new rows before the new row is stored; the
    // rows go through LDS in chunks (one lane sums, at LDS latency).
    __shared__ double sold[SEQ_CHUNK], snew[SEQ_CHUNK];
    double dot = 0.0, aa = 0.0, bb = 0.0;
    const double inv = cnt != 0.0 ? 1.0 / cnt : 0.0;
    for (int64_t t0 = 0; t0 < d; t0 += SEQ_CHUNK) {
      const int m = (int)(d - t0 < SEQ_CHUNK ? d - t0 : SEQ_CHUNK);
      __syncthreads();
      for (int t = threadIdx.x; t < m; t += blockDim.x) {
        const double old = C[c * d + t0 + t];
        sold[t] = old;
        snew[t] = cnt != 0.0 ? acc[c * d + t0 + t] * inv : old;
      }
      __syncthreads();
      if (threadIdx.x == 0)
        for (int t = 0; t < m; ++t) {
          dot = dot + snew[t] * sold[t];
          aa = aa + snew[t] * snew[t];
          bb = bb + sold[t] * sold[t];
        }
    }
    if (threadIdx.x == 0) {
      double dd = -2.0 * dot;
      dd = dd + aa;
      dd = dd + bb;
      shift[1 + c] = sqrt(dd > 0.0 ? dd : 0.0);
    }
    __syncthreads();
    if (cnt != 0.0) {
      const double inv = 1.0 / cnt;
      for (int64_t t = threadIdx.x; t < d; t += blockDim.x)
        C[c * d + t] = acc[c * d + t] * inv;
    }
    return;
  }
  if (cnt != 0.0) {
    for (int64_t t = threadIdx.x; t < d; t += blockDim.x) {
      const double s = acc[c * d + t];
      double nv;
      if (mode == DKM_SUMS_F32)
        nv = (double)((float)s / (float)cnt);
      else
        nv = s / cnt;
      const double old = C[c * d + t];
      const double df = nv - old;
      ss = fma(df, df, ss);
      C[c * d + t] = nv;
    }
  }
  red[threadIdx.x] = ss;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) shift[1 + c] = sqrt(red[0]);
}

// sequential sum over centres in index order (base.py:128-129), one lane
__global__ void k_criterion(double *shift, int64_t k, double tol2,
                            int32_t *flag) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double diff = 0.0;
    for (int64_t c = 0; c < k; ++c) diff = diff + shift[1 + c];
    shift[0] = diff;
    if (flag) *flag = (diff < tol2) ? 1 : 0;
  }
}

// ---------------------------------------------------------------------------
// synthetic make_blobs (counter-based; mirrors oracle.make_blobs_rows)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) k_blobs(double *__restrict__ X,
                                               int64_t row0, int64_t n,
                                               int64_t d, int64_t n_blobs,
                                               uint64_t seed, double box,
                                               double stdv,
                                               int32_t *__restrict__ blob) {
  const uint64_t sm = seed << 40;
  const int64_t total = n * d;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / d, t = e - (e / d) * d;
    const uint64_t row = (uint64_t)(row0 + i);
    const uint64_t b = splitmix64(row ^ sm ^ 0xB10Bull) % (uint64_t)n_blobs;
    const uint64_t cc = (b * (uint64_t)d + (uint64_t)t) + seed * 0x100000000ull;
    const double u0 = (double)(splitmix64(cc ^ 0xC0FFEEull) >> 11) * 0x1.0p-53;
    const double cen = (2.0 * u0 - 1.0) * box;
    const uint64_t ctr = (row * (uint64_t)d + (uint64_t)t) ^ sm;
    const uint64_t h1 = splitmix64(ctr * 2ull);
    const uint64_t h2 = splitmix64(ctr * 2ull + 1ull);
    const double u1 = ((double)(h1 >> 11) + 1.0) * 0x1.0p-53;
    const double u2 = (double)(h2 >> 11) * 0x1.0p-53;
    const double z = sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2);
    X[i * d + t] = cen + stdv * z;
    if (blob && t == 0) blob[i] = (int32_t)b;
  }
}

DKM_TU_FLAGS(util, 0)

}  // namespace dkm

using namespace dkm;

extern "C" {

int dkm_abi_version(void) { return DKM_ABI_VERSION; }

const char *dkm_last_error(void) { return g_err.c_str(); }

int dkm_preload(void) {
  hipFuncAttributes a;
  int bad = hipFuncGetAttributes(&a, (const void *)k_prepare) != hipSuccess;
  bad += preload_dense() + preload_b2() + preload_sorted() + preload_cand() +
         preload_sparse() + preload_gemm() + preload_sums() +
         preload_neighbors();
  return bad ? fail(DKM_E_LAUNCH, "preload: kernel attribute query") : 0;
}

size_t dkm_workspace_bytes(int64_t k, int64_t d, int64_t n_queue) {
  if (k <= 0 || d <= 0) return 0;
  return ws_bytes(k, d, n_queue);
}

int dkm_prepare_centers(const double *C, int64_t k, int64_t d, int flags,
                        void *ws, size_t ws_b, double *acc, void *stream) {
  if (!C || k <= 0 || d <= 0) return fail(DKM_E_ARG, "prepare: bad C/k/d");
  if (k > INT32_MAX) return fail(DKM_E_ARG, "prepare: k too large");
  WsView v;
  if (int r = ws_view(ws, ws_b, k, d, &v)) return r;
  hipStream_t s = (hipStream_t)stream;
  const int64_t dpad = round_up(d, 4);
  k_ws_header<<<1, 64, 0, s>>>(v.hdr, k, d, dpad, v.nq);
  if (v.mvec && !(flags & DKM_PREP_CSR))
    k_mvec<<<(unsigned)std::max<int64_t>(1, (d + 31) / 32), 256, 0, s>>>(
        C, k, d, v.mvec);
  else
    v.mvec = nullptr;   // (a local copy: k_prepare skips ||c - m||)
  k_prepare<<<(unsigned)k, 256, 0, s>>>(C, k, d, dpad, flags, v);
  if (!(flags & DKM_PREP_CSR)) {  // the dense screens' centre tiles
    const int64_t tot = (kpad16(k) / 16) * (dpad32(d) / 32) * 512;
    const int64_t g = std::max<int64_t>(1, std::min<int64_t>((tot + 255) / 256,
                                                            4096));
    k_frag<<<(unsigned)g, 256, 0, s>>>(C, k, d, v);
    if (v.mind) k_mind<<<(unsigned)k, 256, 0, s>>>(C, k, d, v.mind);
  }
  if (int r = check_launch("dkm_prepare_centers")) return r;
  if (gemm_path(k, d) && !(flags & DKM_PREP_CSR))
    if (int r = gemm_prepare(C, k, d, v, s)) return r;
  if (acc) {
    hipError_t e = hipMemsetAsync(acc, 0, (size_t)(k * (d + 1)) * 8, s);
    if (e != hipSuccess)
      return fail((int)e, std::string("prepare: memset acc: ") +
                              hipGetErrorString(e));
  }
  return 0;
}

int dkm_update_centers(const double *acc, double *C, int64_t k, int64_t d,
                       int sums_mode, double tol, double *diff, int32_t *flag,
                       void *stream) {
  if (!acc || !C || !diff || k <= 0 || d <= 0)
    return fail(DKM_E_ARG, "update: bad arguments");
  if (sums_mode < DKM_SUMS_F64 || sums_mode > DKM_SUMS_RECIP)
    return fail(DKM_E_ARG, "update: bad sums_mode");
  hipStream_t s = (hipStream_t)stream;
  k_update<<<(unsigned)k, 256, 0, s>>>(acc, C, k, d, sums_mode, diff);
  k_criterion<<<1, 64, 0, s>>>(diff, k, tol * tol, flag);
  return check_launch("dkm_update_centers");
}

int dkm_make_blobs_f64(double *X, int64_t row0, int64_t n, int64_t d,
                       int64_t n_blobs, uint64_t seed, double box, double std,
                       int32_t *blob, void *stream) {
  if (!X || n < 0 || d <= 0 || n_blobs <= 0 || row0 < 0)
    return fail(DKM_E_ARG, "make_blobs: bad arguments");
  if (n == 0) return 0;
  const int64_t total = n * d;
  int64_t grid = (total + 255) / 256;
  if (grid > 65536) grid = 65536;
  k_blobs<<<(unsigned)grid, 256, 0, (hipStream_t)stream>>>(
      X, row0, n, d, n_blobs, seed, box, std, blob);
  return check_launch("dkm_make_blobs_f64");
}

int dkm_screen_stats(const void *ws, int64_t *n_rechecked, void *stream) {
  if (!ws || !n_rechecked) return fail(DKM_E_ARG, "screen_stats: NULL");
  WsHeader h;
  hipError_t e = hipMemcpyAsync(&h, ws, sizeof(h), hipMemcpyDeviceToHost,
                                (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess)
    return fail((int)e, std::string("screen_stats: ") + hipGetErrorString(e));
  if (h.magic != WS_MAGIC) return fail(DKM_E_ARG, "screen_stats: bad ws");
  *n_rechecked = (int64_t)h.rechecked_total;
  return 0;
}

int dkm_screen_counters(const void *ws, int64_t *out, void *stream) {
  if (!ws || !out) return fail(DKM_E_ARG, "screen_counters: NULL");
  WsHeader h;
  hipError_t e = hipMemcpyAsync(&h, ws, sizeof(h), hipMemcpyDeviceToHost,
                                (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess)
    return fail((int)e, std::string("screen_counters: ") +
                            hipGetErrorString(e));
  if (h.magic != WS_MAGIC) return fail(DKM_E_ARG, "screen_counters: bad ws");
  for (int i = 0; i < 3; ++i) out[i] = (int64_t)h.reserved[i];
  out[3] = (int64_t)h.sfall_total;
  return 0;
}

int dkm_screen_lists(const void *ws, size_t ws_bytes, int64_t *out,
                     void *stream) {
  if (!ws || !out) return fail(DKM_E_ARG, "screen_lists: NULL");
  hipStream_t s = (hipStream_t)stream;
  WsHeader h;
  hipError_t e = hipMemcpyAsync(&h, ws, sizeof(h), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess)
    return fail((int)e, std::string("screen_lists: ") + hipGetErrorString(e));
  if (h.magic != WS_MAGIC) return fail(DKM_E_ARG, "screen_lists: bad ws");
  WsView v;
  if (int r = ws_view(ws, ws_bytes, h.k, h.d, &v)) return r;
  for (int i = 0; i < 4; ++i) out[i] = 0;
  out[3] = (int64_t)h.qcount;
  const int nseg = std::max(0, std::min(h.lseg, TL_SEGS));
  if (nseg == 0) return 0;
  std::vector<int32_t> c(nseg);
  int32_t *src[3] = {v.tcount, v.ccount, v.ncount};
  for (int a = 0; a < 3; ++a) {
    if (!src[a] || (a > 0 && nseg > B1_SEGS)) continue;
    e = hipMemcpyAsync(c.data(), src[a], (size_t)nseg * 4,
                       hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess)
      return fail((int)e, std::string("screen_lists: ") +
                              hipGetErrorString(e));
    for (int i = 0; i < nseg; ++i) out[a] += c[i];
  }
  return 0;
}

}  // extern "C"
