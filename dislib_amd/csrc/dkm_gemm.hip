// dkm_gemm.hip -- assignment screen for large d (d > 128) as a bf16x3 MFMA
// GEMM: the dense contraction X . C^T of `_vec_matrix_euclid`
// (cluster/kmeans/base.py:171-173, 204-205) at C4 scale (10M x 1024,
// k = 4096), where the register-tile screen of dkm_dense.hip cannot hold a
// sample's row.
//
// Per chunk of gemm_chunk(d) samples:
//   k_gemm_split   samples (fp64 or fp32 rows) -> fp32 -> bf16 hi + lo, in
//                  the tile layout below, and an upper bound of ||x||.
//   k_gemm_screen  one 512-thread workgroup per (256-sample tile, 256-centre
//                  tile): scores s = |c|^2 - 2 x.c accumulated over d on
//                  v_mfma_f32_32x32x16_bf16 as xh.ch + xl.ch + xh.cl (the
//                  centre operand holds -2c, so the chain IS the score), both
//                  operands staged HBM/L2 -> LDS by global_load_lds
//                  (double-buffered 32-feature stages), then each sample's
//                  4 smallest scores of the tile -> gpart.
//   k_gemm_merge   per sample: the smallest scores over all centre tiles, a
//                  rigorous error bound 2B, and the decision: one score
//                  within 2B of the best -> label; a few -> the reference
//                  arithmetic on exactly those candidates (k_gemm_cand);
//                  more within 2B in a tile than it kept -> k_gemm_full,
//                  which scans those tiles whole.
//
// Tile layout (centres and samples alike): tile t, stage ks = 256 rows x
// 128 B; a row holds features 32ks..32ks+31 as bf16 hi (chunks 0-3) and lo
// (chunks 4-7), 16-B chunk c stored at slot c ^ ((row >> 1) & 7).  An MFMA
// operand read (ds_read_b128 of 8 consecutive features) then spreads every
// 16-lane group over 16 distinct slots of the 256-B bank row: no conflicts.
// The swizzle lives in the global layout, so the LDS copy is a plain linear
// global_load_lds (MI355X guide, "Swizzle must be BOTH-sides-or-neither").
//
// Error bound (B bounds |(p_j + |x|^2) - numpy's fl64 distance^2| for every
// centre j, p_j = the packed fp32 score; the decision uses 2B with B twice
// the rigorous value, so that any excluded centre is farther by >= 32 ulp
// of the distance^2 and cannot tie after sqrt -- DESIGN.md 3.7):
//   split:     x -> fl32 -> bf16 hi + bf16 lo (round to nearest), the lo*lo
//              product dropped: <= 0.76 * 2^-16 sum|x (-2c)|  (1.0 used)
//   chain:     3 dpad products + |c|^2, each addition rounded (<= 2^-23
//              relative, no assumption on the MFMA adder): (3 dpad + 2) 2^-23
//              of sum|terms| + |c|^2, sum|terms| <= 2|x||c|(1 + 2^-7)
//   packing:   6 tag bits in the mantissa: 2^-17 |s|
//   numpy:     fp64 (x - c)^2 terms + pairwise sum: 2^-48 (|x| + |c|)^2
//   underflow: 8 dpad 2^-120 (|x| + |c| + 1)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "dkm_internal.h"

namespace dkm {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GTHREADS = 512;          // 8 waves: 2 (centres) x 4 (samples)
constexpr int GLDS = 2 * 2 * GSTAGE;   // two stages of (centre + sample) tiles
constexpr uint32_t GTAG = 63;          // 6 tag bits: (centre block, register)
// second half of WsView::tlist: the full-scan list (first half: candidates)
constexpr int64_t GLIST2 = (int64_t)TL_SEGS * TL_CAP / 2;

__host__ __device__ __forceinline__ int gslot(int row, int c) {
  return c ^ ((row >> 1) & 7);
}
// hi-only 64-B rows (4 chunks): chunk c of row r at slot c ^ ((r >> 2) & 3)
__host__ __device__ __forceinline__ int gslot1(int row, int c) {
  return c ^ ((row >> 2) & 3);
}

// v_med3 against an opaque -inf: a min without fminf's NaN canonicalisation
__device__ __forceinline__ float g_opaque_ninf() {
  uint32_t r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(0xff800000u));
  return __uint_as_float(r);
}

// (value, centre) lexicographic insertion into an ascending top-4 list,
// branchless (c0 => c1 => c2 => c3 on a sorted list; no runtime indices)
__device__ __forceinline__ bool vi_less(float a, int ia, float b, int ib) {
  return (a < b) | ((a == b) & (ia < ib));  // bitwise: no branches
}
__device__ __forceinline__ void top_insert(float v, int i, float (&V)[GTOP],
                                           int (&I)[GTOP]) {
  static_assert(GTOP == 4, "top_insert is written for 4 entries");
  const bool c0 = vi_less(v, i, V[0], I[0]), c1 = vi_less(v, i, V[1], I[1]);
  const bool c2 = vi_less(v, i, V[2], I[2]), c3 = vi_less(v, i, V[3], I[3]);
  V[3] = c2 ? V[2] : (c3 ? v : V[3]);
  I[3] = c2 ? I[2] : (c3 ? i : I[3]);
  V[2] = c1 ? V[1] : (c2 ? v : V[2]);
  I[2] = c1 ? I[1] : (c2 ? i : I[2]);
  V[1] = c0 ? V[0] : (c1 ? v : V[1]);
  I[1] = c0 ? I[0] : (c1 ? i : I[1]);
  V[0] = c0 ? v : V[0];
  I[0] = c0 ? i : I[0];
}

// ---------------------------------------------------------------------------
// split: rows [row0, row0 + nrows) of X (scaled by `scale`, exact for +-2)
// into mrows/GT tiles; rows past nrows and features past d are zero.  One
// wave = 8 rows, lane (row rr = l >> 3, group f = l & 7): 8 lanes read 512
// contiguous bytes of a row per step.  xn (nullable): fp32 upper bound of
// the row's Euclidean norm.  out1 / xn1 (hi + lo splits only, nullable): the
// same rows' hi-only tiles and norms in the resident IMG_GEMM image as well
// (DKM_IMAGE_BUILD during the bf16x3 iteration: no separate image pass).
// ---------------------------------------------------------------------------
template <bool VEC, class TX>
__global__ void __launch_bounds__(256)
    k_gemm_split(const TX *__restrict__ X, int64_t row0, int64_t nrows,
                 int64_t mrows, int d, int64_t ldx, int nks, double scale,
                 char *__restrict__ out, float *__restrict__ xn, int one,
                 char *__restrict__ out1, float *__restrict__ xn1) {
  const int lane = threadIdx.x & 63, rr = lane >> 3, f = lane & 7;
  const int64_t wv = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nw = (int64_t)gridDim.x * 4;
  // 8-feature groups: 4 per 32-feature stage (hi/lo, or hi only: one)
  const int ngrp = nks * 4;
  for (int64_t rb = wv * 8; rb < mrows; rb += nw * 8) {
    const int64_t row = rb + rr;
    const bool valid = row < nrows;
    const TX *xr = X + (row0 + (valid ? row : 0)) * ldx;
    const int64_t st = row / GT;
    const int r = (int)(row - st * GT);
    double ss = 0.0;
    for (int g = f; g < ngrp; g += 8) {
      const int t0 = 8 * g;
      double xv[8];
      if (VEC && valid && t0 < d) {
        if constexpr (sizeof(TX) == 8) {
          const double2 *p = (const double2 *)(xr + t0);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const double2 u = p[q];
            xv[2 * q] = u.x;
            xv[2 * q + 1] = u.y;
          }
        } else {
          const float4 *p = (const float4 *)(xr + t0);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const float4 u = p[q];
            xv[4 * q] = u.x;
            xv[4 * q + 1] = u.y;
            xv[4 * q + 2] = u.z;
            xv[4 * q + 3] = u.w;
          }
        }
      } else {
#pragma unroll
        for (int m = 0; m < 8; ++m)
          xv[m] = (valid && t0 + m < d) ? (double)xr[t0 + m] : 0.0;
      }
      uint32_t hw[4], lw[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double a = xv[2 * q] * scale, b = xv[2 * q + 1] * scale;
        ss = ss + a * a;
        ss = ss + b * b;
        const float x0 = (float)a, x1 = (float)b;
        // scalar ops only (no v_pk_*_f32: see dkm_dense.hip's header note)
        const bf16x2 h2 = __builtin_convertvector(f32x2{x0, x1}, bf16x2);
        const uint32_t hu = __builtin_bit_cast(uint32_t, h2);
        const float h0 = __uint_as_float(hu << 16);
        const float h1 = __uint_as_float(hu & 0xffff0000u);
        const bf16x2 l2 =
            __builtin_convertvector(f32x2{x0 - h0, x1 - h1}, bf16x2);
        hw[q] = hu;
        lw[q] = __builtin_bit_cast(uint32_t, l2);
      }
      if (one) {
        const int ks = g >> 2, c = g & 3;
        char *tile = out + (st * nks + ks) * (int64_t)GSTAGE1 + r * 64;
        *(uint4 *)(tile + 16 * gslot1(r, c)) =
            make_uint4(hw[0], hw[1], hw[2], hw[3]);
      } else {
        const int ks = g >> 2, c = g & 3;
        char *tile = out + (st * nks + ks) * (int64_t)GSTAGE + r * 128;
        *(uint4 *)(tile + 16 * gslot(r, c)) =
            make_uint4(hw[0], hw[1], hw[2], hw[3]);
        *(uint4 *)(tile + 16 * gslot(r, 4 + c)) =
            make_uint4(lw[0], lw[1], lw[2], lw[3]);
        if (out1) {
          char *t1 = out1 + (st * nks + ks) * (int64_t)GSTAGE1 + r * 64;
          *(uint4 *)(t1 + 16 * gslot1(r, c)) =
              make_uint4(hw[0], hw[1], hw[2], hw[3]);
        }
      }
    }
    ss += __shfl_xor(ss, 1, 64);
    ss += __shfl_xor(ss, 2, 64);
    ss += __shfl_xor(ss, 4, 64);
    // fl32 of sqrt may round down by 2^-24: inflate (NaN / Inf stay so)
    const float nr = valid ? (float)sqrt(ss) * (1.0f + 0x1.0p-20f) : 0.0f;
    if (xn && f == 0) xn[row] = nr;
    if (xn1 && f == 0) xn1[row] = nr;
  }
}

__global__ void k_gemm_cnorm(const float *__restrict__ cn32, int64_t k,
                             int64_t kp, float *__restrict__ gcn) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < kp;
       c += (int64_t)gridDim.x * blockDim.x)
    gcn[c] = c < k ? cn32[c] : 0x1.0p100f;
}

// ---------------------------------------------------------------------------
// bf16x3 screen: one workgroup = centre tile ct x sample tile st, full K.
// Wave w: wm = w & 1 -> centres wm*128 .. +127 (4 blocks of 32 = A rows),
// wn = w >> 1 -> samples wn*64 .. +63 (2 blocks of 32 = B columns).
// 32x32x16 accumulator register g of lane (r, h): centre row
// (g & 3) + 8 (g >> 2) + 4h of the block, sample column r.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(GTHREADS)
    k_gemm_screen3(const char *__restrict__ afrag, const float *__restrict__ gcn,
                  const char *__restrict__ xs, int nst, int nct, int nks,
                  int2 *__restrict__ part, uint32_t *__restrict__ gcount) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // the merge's candidate-list counter, reset for this chunk (the previous
  // chunk's readers ran before this launch on the stream; a memset launch
  // per chunk cost 0.8 ms per C4 iteration)
  if (blockIdx.x == 0 && threadIdx.x == 0) *gcount = 0;
  typedef __attribute__((address_space(3))) void lds_void;
  // XCD-aware bijective remap (blocks b and b + 8 share an XCD): the nct
  // centre tiles of one sample tile run on one XCD, so its split rows are
  // read from HBM once and from that XCD's L2 afterwards
  const int G = nst * nct;
  const int b = blockIdx.x, xcd = b & 7, jx = b >> 3;
  const int q8 = G >> 3, r8 = G & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + jx;
  const int st = wg / nct, ct = wg - st * nct;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5, wm = w & 1, wn = w >> 1;
  const char *abase = afrag + (int64_t)ct * nks * GSTAGE;
  const char *bbase = xs + (int64_t)st * nks * GSTAGE;

  // stage ks -> buffer: each wave copies 4 x 1 KB of each operand (a linear
  // copy: the swizzle is already in the global layout)
  auto stage_load = [&](int ks, int buf) {
    char *la = lds + buf * (2 * GSTAGE);
    const char *ga = abase + (int64_t)ks * GSTAGE + w * 1024 + lane * 16;
    const char *gb = bbase + (int64_t)ks * GSTAGE + w * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_global_load_lds((const void *)(ga + i * 8192),
                                       (lds_void *)(la + i * 8192 + w * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds(
          (const void *)(gb + i * 8192),
          (lds_void *)(la + GSTAGE + i * 8192 + w * 1024), 16, 0, 0);
    }
  };

  // accumulators start from |c|^2 of their centre rows
  f32x16 acc[4][2];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const float *cp = gcn + (int64_t)ct * GT + wm * 128 + mb * 32 + 4 * h;
    f32x16 init;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const f32x4 c4 = *(const f32x4 *)(cp + 8 * qq);
      init[4 * qq + 0] = c4.x;
      init[4 * qq + 1] = c4.y;
      init[4 * qq + 2] = c4.z;
      init[4 * qq + 3] = c4.w;
    }
    acc[mb][0] = init;
    acc[mb][1] = init;
  }

  // lane's chunk offsets inside a row: K-substep s reads features
  // 16s + 8h .. +7, i.e. hi chunk 2s + h and lo chunk 4 + 2s + h
  const int sw = (r >> 1) & 7;
  const int oh0 = 16 * ((0 + h) ^ sw), oh1 = 16 * ((2 + h) ^ sw);
  const int ol0 = 16 * ((4 + h) ^ sw), ol1 = 16 * ((6 + h) ^ sw);
  const int arow = (wm * 128 + r) * 128, brow = (wn * 64 + r) * 128;

  stage_load(0, 0);
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) {
      stage_load(ks + 1, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // stage ks landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // ... for every wave
    asm volatile("" ::: "memory");
    const char *la = lds + buf * (2 * GSTAGE);
    const char *lb = la + GSTAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int oh = s ? oh1 : oh0;
      const int ol = s ? ol1 : ol0;
      bf16x8 ah[4], al[4], bh[2], bl[2];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const char *p = la + arow + mb * 32 * 128;
        ah[mb] = *(const bf16x8 *)(p + oh);
        al[mb] = *(const bf16x8 *)(p + ol);
      }
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const char *p = lb + brow + nb * 32 * 128;
        bh[nb] = *(const bf16x8 *)(p + oh);
        bl[nb] = *(const bf16x8 *)(p + ol);
      }
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              ah[mb], bh[nb], acc[mb][nb], 0, 0, 0);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              ah[mb], bl[nb], acc[mb][nb], 0, 0, 0);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              al[mb], bh[nb], acc[mb][nb], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // buffer `buf` is free for stage ks + 2
    asm volatile("" ::: "memory");
  }

  // ---- epilogue: each lane's top-4 per sample column, packed tags ----
  const float ninf = g_opaque_ninf();
  int2 *mrg = (int2 *)lds;  // [256 samples][4 sources][GTOP]
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    float v[GTOP];
#pragma unroll
    for (int e = 0; e < GTOP; ++e) v[e] = INFINITY;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float p = __uint_as_float(
            (__float_as_uint(acc[mb][nb][g]) & ~GTAG) | (uint32_t)(mb * 16 + g));
        v[3] = __builtin_amdgcn_fmed3f(v[2], v[3], p);
        v[2] = __builtin_amdgcn_fmed3f(v[1], v[2], p);
        v[1] = __builtin_amdgcn_fmed3f(v[0], v[1], p);
        v[0] = __builtin_amdgcn_fmed3f(v[0], p, ninf);
      }
    const int sample = wn * 64 + nb * 32 + r, src = wm * 2 + h;
#pragma unroll
    for (int e = 0; e < GTOP; ++e) {
      const uint32_t tg = __float_as_uint(v[e]) & GTAG;
      const int mb = (int)(tg >> 4), g = (int)(tg & 15);
      const int local = wm * 128 + mb * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
      mrg[(sample * 4 + src) * GTOP + e] =
          make_int2(__float_as_int(v[e]), ct * GT + local);
    }
  }
  __syncthreads();
  if (tid < GT) {
    float V[GTOP];
    int I[GTOP];
#pragma unroll
    for (int e = 0; e < GTOP; ++e) {
      V[e] = INFINITY;
      I[e] = 0x7fffffff;
    }
    const int2 *mp = mrg + tid * 4 * GTOP;
#pragma unroll
    for (int e = 0; e < 4 * GTOP; ++e) {
      const int2 q = mp[e];
      top_insert(__int_as_float(q.x), q.y, V, I);
    }
    int2 *out = part + ((int64_t)(st * GT + tid) * nct + ct) * GTOP;
#pragma unroll
    for (int e = 0; e < GTOP; ++e) out[e] = make_int2(__float_as_int(V[e]), I[e]);
  }
}

// ---------------------------------------------------------------------------
// single-product screen (hi x hi), persistent: one 512-thread workgroup per
// CU walks its share of the (sample tile, centre tile) pairs as one stream
// of 32-feature stages, so the loads of the next tile's first stages fly
// while the current tile finishes and its epilogue runs.
//   * XCD-aware split: workgroup b runs on XCD b & 7; XCD x owns a
//     contiguous range of the pairs (centre tile fastest) and its workgroups
//     take them round-robin, so at any time one XCD's CUs work on a few
//     sample tiles against all centre tiles (the sample tile is read from
//     HBM once, then from that XCD's L2).
//   * a 4-stage LDS ring (4 x 32 KB), 3 stages in flight, ONE barrier per
//     stage: the barrier of stage q also proves every wave is done with
//     stage q - 1, whose buffer (q + 3) & 3 then takes stage q + 3.
//   * global_load_lds (asm: see glds16) with the stage base in SGPRs and
//     the per-lane offset a constant VGPR (no address arithmetic per load).
//   * rows of 64 B (32 features) with 16-B chunk c at c ^ ((row >> 2) & 3):
//     every 16-lane group of a ds_read_b128 hits 16 distinct slots.
//   * epilogue: each lane keeps the GTOP smallest packed scores of its 64
//     (a med3 chain, the tag by one and-or), written to LDS as bare floats,
//     sample-minor (conflict-free; the tag names the centre), then thread =
//     sample merges the 4 sources into the tile's sorted top-GTOP.  (Keeping
//     only 2 or 3 per lane is cheaper but sends every sample with that many
//     candidates in one source to the full scan: measured slower per fit.)
// Wave w: wm = w & 1 -> centres wm*128 .. +127, wn = w >> 1 -> samples
// wn*64 .. +63, accumulator layout as k_gemm_screen3.
// ---------------------------------------------------------------------------
constexpr int G1RING = 4;

// 16 B per lane from gbase + voff (gbase wave-uniform) into LDS at
// lds_addr + 16 lane (wave-uniform; M0 written in the same statement).  An
// asm statement, so hipcc adds no vmcnt wait of its own before LDS accesses
// it cannot prove disjoint (it would drain the ring on every stage): the
// kernel counts these copies itself.
__device__ __forceinline__ void glds16(const char *gbase, uint32_t voff,
                                       uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gbase), "s"(lds_addr)
      : "memory");
}
constexpr int G1STAGE = 2 * GSTAGE1;             // A + B bytes of one stage
constexpr int G1MRG = G1RING * G1STAGE;    // epilogue [GTOP][4][GT] floats
constexpr int G1NRM = G1MRG + 4 * 4 * GT * 4;  // |c|^2 of 2 tiles
constexpr int G1LDS = G1NRM + 2 * GT * 4;

__global__ void __launch_bounds__(GTHREADS)
    k_gemm_screen1(const char *__restrict__ afrag,
                   const float *__restrict__ gcn, const char *__restrict__ xs,
                   int nst, int nct, int nks, int2 *__restrict__ part,
                   uint32_t *__restrict__ gcount) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  typedef __attribute__((address_space(3))) void lds_void;
  if (blockIdx.x == 0 && threadIdx.x == 0) *gcount = 0;  // as k_gemm_screen3
  const int G = nst * nct;
  const int per = (int)(gridDim.x >> 3);  // workgroups per XCD
  const int xcd = (int)(blockIdx.x & 7), j = (int)(blockIdx.x >> 3);
  const int q8 = G >> 3, r8 = G & 7;
  const int lo = xcd * q8 + (xcd < r8 ? xcd : r8);
  const int cnt = q8 + (xcd < r8 ? 1 : 0);
  const int ntile = j < cnt ? (cnt - j + per - 1) / per : 0;
  if (ntile == 0) return;  // workgroup-uniform
  const int Q = ntile * nks;
  // pair order (L2 reuse): blocks of SB sample tiles; inside a block, groups
  // of CG centre tiles, sample tile, centre tile.  A time step of one XCD
  // (its `per` workgroups, consecutive pairs) then covers SB sample tiles x
  // CG centre tiles (4 x 8 at k = 4096): each centre tile's stage is read
  // once per SB sample tiles, each sample tile's once per CG centre tiles
  // (C4: 13.6 KB read per sample and iteration, against 19.8 KB with all 16
  // centre tiles of 2 sample tiles per step; the same time).
  const int CG = nct < 8 ? nct : 8;
  const int SB = per / CG > 1 ? per / CG : 1;
  auto pair_of = [&](int p, int &st, int &ct) {
    const int b = p / (SB * nct);
    const int sb = nst - SB * b < SB ? nst - SB * b : SB;
    const int r0 = p - b * SB * nct;
    const int g = r0 / (sb * CG);
    const int cgw = nct - g * CG < CG ? nct - g * CG : CG;
    const int rr = r0 - g * sb * CG;
    st = SB * b + rr / cgw;
    ct = g * CG + rr % cgw;
  };
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5, wm = w & 1, wn = w >> 1;
  const uint32_t voff = (uint32_t)(w * 1024 + lane * 16), voff2 = voff + 8192;
  const uint32_t voffn = (uint32_t)(lane * 16);
  // this wave's 1-KB piece of each 8-KB half of an operand stage
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_void *)lds;
  const uint32_t lds_base =
      __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)w * 1024u);
  const uint32_t nrm_base =
      __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(G1NRM + w * 128));
  const int64_t tbytes = (int64_t)nks * GSTAGE1;  // one tile, every stage

  // The stage stream is issued in order: the tile of the next stage to
  // issue and its operand bases are kept (wave-uniform, SGPRs) and advanced
  // per stage, so pair_of's divisions run once per tile, not per stage (as
  // q / nks plus pair_of per stage they were ~10 SALU per MFMA, C4 PMC).
  int im = 0, iks = 0, ict = 0;
  const char *iga = nullptr, *igb = nullptr;
  auto issue_tile = [&](int m) {
    int st, ct;
    pair_of(lo + j + m * per, st, ct);
    st = __builtin_amdgcn_readfirstlane(st);
    ct = __builtin_amdgcn_readfirstlane(ct);
    ict = ct;
    iga = afrag + ct * tbytes;
    igb = xs + st * tbytes;
  };
  issue_tile(0);
  auto uni = [](const char *p) {  // the compiler cannot prove these uniform
    const uint64_t a = (uint64_t)p;
    return (const char *)(((uint64_t)__builtin_amdgcn_readfirstlane(
                               (uint32_t)(a >> 32))
                           << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a));
  };
  auto issue = [&](int q) {  // stage q (= im nks + iks) -> ring buffer q & 3
    const char *ga = uni(iga + (int64_t)iks * GSTAGE1);
    const char *gb = uni(igb + (int64_t)iks * GSTAGE1);
    const uint32_t la = __builtin_amdgcn_readfirstlane(
        lds_base + (uint32_t)((q & (G1RING - 1)) * G1STAGE));
    glds16(ga, voff, la);
    glds16(ga, voff2, la + 8192);
    glds16(gb, voff, la + GSTAGE1);
    glds16(gb, voff2, la + GSTAGE1 + 8192);
    if (iks == 0 && lane < 8)  // the tile's 256 |c|^2: 128 B per wave
      glds16(uni((const char *)(gcn + (int64_t)ict * GT + w * 32)), voffn,
             (uint32_t)__builtin_amdgcn_readfirstlane(
                 nrm_base + (uint32_t)((im & 1) * GT * 4)));
    // (readfirstlane: the lane < 8 branch above otherwise makes hipcc keep
    // the stage counters in VGPRs and the pointers in VGPR pairs)
    iks = __builtin_amdgcn_readfirstlane(iks + 1);
    if (iks == nks) {
      iks = 0;
      im = __builtin_amdgcn_readfirstlane(im + 1);
      if (im < ntile) issue_tile(im);
    }
  };

  // accumulators start from |c|^2 of their centre rows (LDS: copied with
  // the tile's first stage, so no global load waits behind the ring)
  f32x16 acc[4][2];
  auto init_acc = [&](int m) {
    const float *nl = (const float *)(lds + G1NRM) + (m & 1) * GT;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const float *cp = nl + wm * 128 + mb * 32 + 4 * h;
      f32x16 init;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const f32x4 c4 = *(const f32x4 *)(cp + 8 * qq);
        init[4 * qq + 0] = c4.x;
        init[4 * qq + 1] = c4.y;
        init[4 * qq + 2] = c4.z;
        init[4 * qq + 3] = c4.w;
      }
      acc[mb][0] = init;
      acc[mb][1] = init;
    }
  };

  const float ninf = g_opaque_ninf();
  float *mrg = (float *)(lds + G1MRG);  // [GTOP e][4 src][GT samples]
  auto epilogue = [&](int st, int ct) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      float v[GTOP];
#pragma unroll
      for (int e = 0; e < GTOP; ++e) v[e] = INFINITY;
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const float p = __uint_as_float(
              (__float_as_uint(acc[mb][nb][g]) & ~GTAG) |
              (uint32_t)(mb * 16 + g));
#pragma unroll
          for (int e = GTOP - 1; e > 0; --e)
            v[e] = __builtin_amdgcn_fmed3f(v[e - 1], v[e], p);
          v[0] = __builtin_amdgcn_fmed3f(v[0], p, ninf);
        }
      const int sample = wn * 64 + nb * 32 + r, src = wm * 2 + h;
#pragma unroll
      for (int e = 0; e < GTOP; ++e) mrg[(e * 4 + src) * GT + sample] = v[e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (tid < GT) {
      float V[GTOP];
      int I[GTOP];
#pragma unroll
      for (int e = 0; e < GTOP; ++e) {
        V[e] = INFINITY;
        I[e] = 0x7fffffff;
      }
#pragma unroll
      for (int e = 0; e < GTOP; ++e)
#pragma unroll
        for (int src = 0; src < 4; ++src) {
          const float qv = mrg[(e * 4 + src) * GT + tid];
          // the centre from the tag: source (wm', h') = (src >> 1, src & 1)
          const uint32_t tg = __float_as_uint(qv) & GTAG;
          const int mb = (int)(tg >> 4), g = (int)(tg & 15);
          const int qi = ct * GT + (src >> 1) * 128 + mb * 32 + (g & 3) +
                         8 * (g >> 2) + 4 * (src & 1);
          top_insert(qv, qi, V, I);
        }
      int2 *out = part + ((int64_t)(st * GT + tid) * nct + ct) * GTOP;
#pragma unroll
      for (int e = 0; e < GTOP; ++e)
        out[e] = make_int2(__float_as_int(V[e]), I[e]);
    }
  };

  // lane's chunk offsets in a 64-B row: K-substep s reads features
  // 16s + 8h .. +7, chunk 2s + h
  const int sw = (r >> 2) & 3;
  const int o0 = 16 * ((0 + h) ^ sw), o1 = 16 * ((2 + h) ^ sw);
  const int arow = (wm * 128 + r) * 64, brow = (wn * 64 + r) * 64;

  // stage q: its copies landed (this wave: later stages may stay in
  // flight; every wave: the barrier), this wave's LDS reads of stage q - 1
  // done (its buffer takes stage q + 3 after the barrier)
  auto sync_issue = [&](int q) {
    const int ahead = Q - 1 - q;
    if (ahead >= 2)
      asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    else if (ahead == 1)
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (q + 3 < Q) issue(q + 3);
  };
  // K-substep s of stage q into registers.  Per stage, after its barrier:
  // read substep 0, MFMAs of the previous stage's substep 1, read substep 1,
  // MFMAs of substep 0 -- every LDS read hides under 8 MFMAs.
  auto load_sub = [&](int q, int s, bf16x8 (&A)[4], bf16x8 (&B)[2]) {
    const char *la = lds + (q & (G1RING - 1)) * G1STAGE;
    const char *lb = la + GSTAGE1;
    const int oh = s ? o1 : o0;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      A[mb] = *(const bf16x8 *)(la + arow + mb * 32 * 64 + oh);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
      B[nb] = *(const bf16x8 *)(lb + brow + nb * 32 * 64 + oh);
  };
  auto mfmas = [&](const bf16x8 (&A)[4], const bf16x8 (&B)[2]) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            A[mb], B[nb], acc[mb][nb], 0, 0, 0);
  };

  for (int q = 0; q < 3 && q < Q; ++q) issue(q);
  bf16x8 A0[4], A1[4], B0[2], B1[2];
  for (int m = 0; m < ntile; ++m) {  // workgroup-uniform
    int st, ct;
    pair_of(lo + j + m * per, st, ct);
    const int q0 = m * nks;
    sync_issue(q0);
    init_acc(m);
    load_sub(q0, 0, A0, B0);
    load_sub(q0, 1, A1, B1);
    mfmas(A0, B0);
    // (Pinning this order with sched_barrier -- reads strictly before the
    // MFMAs that cover them -- made the bare loop 3 % faster but the whole
    // kernel 6-9 % slower on one box, A/B r05n: hipcc's interleaving of the
    // ring copies and reads with the MFMAs is kept.)
    for (int ks = 1; ks < nks; ++ks) {
      sync_issue(q0 + ks);
      load_sub(q0 + ks, 0, A0, B0);
      mfmas(A1, B1);
      load_sub(q0 + ks, 1, A1, B1);
      mfmas(A0, B0);
    }
    mfmas(A1, B1);
    epilogue(st, ct);
  }
}

// 2B of the decision test (B = twice the rigorous bound; header comment).
// one: the single-product screen (hi x hi): x and -2c rounded to bf16 lose
// <= 2^-8 each, a product <= (2^-7 + 2^-16) |x (-2c)| (1.02 2^-7 used),
// the fp32 chain has dpad products.
__device__ __forceinline__ float gemm_bound2(int dpad, float xn, float cm,
                                            bool one) {
  const float rel =
      one ? 1.02f * 0x1.0p-7f +
                (dpad + 2.0f) * 0x1.0p-23f * (1.0f + 0x1.0p-7f) + 0x1.0p-17f
          : 0x1.0p-16f +
                (3.0f * dpad + 2.0f) * 0x1.0p-23f * (1.0f + 0x1.0p-7f) +
                0x1.0p-17f;
  const float s = xn + cm;
  const float mag = 2.0f * xn * cm + cm * cm;
  const float b = rel * mag + 0x1.0p-48f * s * s +
                  (8.0f * dpad) * 0x1.0p-120f * (s + 1.0f);
  return 4.0f * b * 1.0001f;  // 1.0001: the fp32 evaluation of this bound
}

// Best kept score of sample i (tile minima are entry 0 of each tile), the
// limit best + 2B, and whether the kept scores hold every candidate.
struct GDecision {
  float lim;
  int best, ncand;
  bool complete;
};
__device__ __forceinline__ GDecision gemm_decide(const int2 *pp, int nct,
                                                 int dpad, float xn,
                                                 float cm, bool one) {
  float p1 = INFINITY;
  int i1 = 0x7fffffff;
  for (int e = 0; e < nct * GTOP; e += GTOP) {
    const int2 q = pp[e];
    const float pv = __int_as_float(q.x);
    if (vi_less(pv, q.y, p1, i1)) {
      p1 = pv;
      i1 = q.y;
    }
  }
  GDecision g;
  g.best = i1;
  g.lim = p1 + gemm_bound2(dpad, xn, cm, one);
  g.ncand = 0;
  // NaN / overflow: no bound holds -> incomplete (exact path)
  g.complete = (xn < 1e18f) & (xn * cm < 1e30f) & (p1 < 1e30f);
  for (int t = 0; t < nct; ++t) {
    const int2 *tp = pp + t * GTOP;
#pragma unroll
    for (int e = 0; e < GTOP; ++e)
      g.ncand += __int_as_float(tp[e].x) <= g.lim;
    // a tile whose 4th kept score is within the limit may hide more
    g.complete &= !(__int_as_float(tp[GTOP - 1].x) <= g.lim);
  }
  return g;
}

// +x to `lab` (and -x from `prev` in delta mode) with fp64 atomics: the
// fallback when no k_label_sums pass follows (flags & 1)
template <class TX>
__device__ void gemm_acc_row(const TX *xr, int d, int k, int lab, int prev,
                             int flags, double *acc) {
  if (!(flags & 1) || ((flags & 2) && lab == prev)) return;
  const bool sub = (flags & 2) && prev >= 0;
  double *cnt = acc + (int64_t)k * d;
  for (int t = 0; t < d; ++t) {
    const double x = (double)xr[t];
    atomic_add_f64(acc + (int64_t)lab * d + t, x);
    if (sub) atomic_add_f64(acc + (int64_t)prev * d + t, -x);
  }
  atomic_add_f64(cnt + lab, 1.0);
  if (sub) atomic_add_f64(cnt + prev, -1.0);
}
template <class TX>
__device__ void gemm_acc_wave(const TX *xr, int d, int k, int lab, int prev,
                              int flags, double *acc, int lane) {
  if (!(flags & 1) || ((flags & 2) && lab == prev)) return;
  const bool sub = (flags & 2) && prev >= 0;
  for (int t = lane; t < d; t += 64) {
    const double x = (double)xr[t];
    atomic_add_f64(acc + (int64_t)lab * d + t, x);
    if (sub) atomic_add_f64(acc + (int64_t)prev * d + t, -x);
  }
  if (lane == 0) {
    atomic_add_f64(acc + (int64_t)k * d + lab, 1.0);
    if (sub) atomic_add_f64(acc + (int64_t)k * d + prev, -1.0);
  }
}

// numpy's pairwise-sum leaves of a d-element row (128 < d <= 8192: one
// iterator buffer, every leaf 64..128 elements), left to right; built once
// per workgroup by one thread
constexpr int GMAXLEAF = 128;
struct LeafTab {
  int n;
  int lo[GMAXLEAF];
  int len[GMAXLEAF];
};
__device__ void build_leaves(int d, LeafTab &t) {
  int c = 0;
  pw_tree(
      [&](int64_t a, int64_t m) -> double {
        t.lo[c] = (int)a;
        t.len[c] = (int)m;
        ++c;
        return 0.0;
      },
      0, d);
  t.n = c;
}

// numpy's fl64 ||x - c||^2 (np.linalg.norm before the sqrt) by one wave:
// leaf l's 8 accumulator chains on lanes 8 (l % 8) .. + 7 (leaves over the
// 8-lane groups, 8 per pass), the leaf's ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
// by xor shuffles (fp addition commutes, so every lane of the group holds
// the same bits), the tail sequentially, then the halving tree over the
// leaf totals (tot: this wave's LDS row) in pw_tree's own order.
template <class TX>
__device__ double wave_sqdist(const TX *__restrict__ x,
                              const double *__restrict__ c, int d,
                              const LeafTab &t, double *tot, int lane) {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();  // the previous call's walk is done
  for (int base = 0; base < t.n * 8; base += 64) {
    const int ci = base + lane, l = ci >> 3, j = ci & 7;
    if (l < t.n) {  // uniform over each 8-lane group
      const int lo = t.lo[l], len = t.len[l], full = len & ~7;
      double df, r;
      if (len == 128) {
        // numpy's full 128-element leaf: every load issued before the
        // first add (the loop form waited one L2 / MALL round trip per 8
        // elements of the centre row); the same additions in the same order
        double xv[16], cv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          xv[u] = (double)x[lo + 8 * u + j];
          cv[u] = c[lo + 8 * u + j];
        }
        df = xv[0] - cv[0];
        r = df * df;
#pragma unroll
        for (int u = 1; u < 16; ++u) {
          df = xv[u] - cv[u];
          r = r + df * df;
        }
      } else {
        df = (double)x[lo + j] - c[lo + j];
        r = df * df;
        for (int i = 8; i < full; i += 8) {
          df = (double)x[lo + i + j] - c[lo + i + j];
          r = r + df * df;
        }
      }
      r = r + __shfl_xor(r, 1, 64);
      r = r + __shfl_xor(r, 2, 64);
      r = r + __shfl_xor(r, 4, 64);
      for (int i = full; i < len; ++i) {
        df = (double)x[lo + i] - c[lo + i];
        r = r + df * df;
      }
      if (j == 0) tot[l] = r;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  int cnt = 0;
  const double s =
      pw_tree([&](int64_t, int64_t) -> double { return tot[cnt++]; }, 0, d);
  return 0.0 + s;  // pw_sum's buffer loop: res = 0.0 + block
}

// np.argmin order: a NaN before any number (the first NaN wins), then the
// smaller value, then the smaller index
__device__ __forceinline__ bool nan_first_less(double a, int ia, double b,
                                               int ib) {
  const bool na = a != a, nb = b != b;
  if (na != nb) return na;
  if (!na && a != b) return a < b;
  return ia < ib;
}

// ---------------------------------------------------------------------------
// merge: thread per sample of the chunk.  gpart holds, per centre tile, the
// tile's 4 smallest packed scores (ascending).  Candidates = every kept
// score <= best + 2B; the set is complete unless some tile's 4th score is
// also within the limit.  One candidate: the label.  A complete set of
// several: listed for k_gemm_cand.  Incomplete: left for k_recheck_exact.
// flags: 1 = accumulate into acc with fp64 atomics, 2 = delta (labels hold
// the previous assignment).
// ---------------------------------------------------------------------------
template <class TX>
__global__ void __launch_bounds__(256)
    k_gemm_merge(const TX *__restrict__ X, int64_t row0, int64_t nrows, int d,
                 int64_t ldx, int k, int nct, int dpad,
                 const int2 *__restrict__ part, const float *__restrict__ xnv,
                 WsView v, int32_t *__restrict__ lab_out, double *acc,
                 int flags, int64_t lofs) {
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  const int lane = threadIdx.x & 63;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x; i0 < nrows;
       i0 += (int64_t)gridDim.x * blockDim.x) {  // block-uniform trip count
    const int64_t i = i0 + threadIdx.x;
    int list = -1;  // 0: candidate list, 1: full-scan list
    int prev = -1;
    if (i < nrows) {
      const GDecision g =
          gemm_decide(part + i * (int64_t)nct * GTOP, nct, dpad, xnv[i], cm,
                      flags & 4);
      const int64_t si = row0 + i;
      prev = (flags & 2) ? lab_out[si] : -1;
      if (g.complete && g.ncand == 1) {
        if (!(flags & 2) || g.best != prev) lab_out[si] = g.best;
        gemm_acc_row(X + si * ldx, d, k, g.best, prev, flags, acc);
      } else {
        list = g.complete ? 0 : 1;
      }
    }
#pragma unroll
    for (int L = 0; L < 2; ++L) {  // wave-aggregated appends
      const uint64_t m = __ballot(list == L);
      if (!m) continue;
      uint32_t slot = 0;
      if (lane == 0)
        slot = atomicAdd(L ? &v.hdr->gcount2 : &v.hdr->gcount,
                         (uint32_t)__popcll(m));
      slot = __shfl(slot, 0, 64);
      // the overflow list spans the call (deferred): rows from its base
      if (list == L)
        v.tlist[(L ? GLIST2 : 0) + slot + __popcll(m & ((1ull << lane) - 1))] =
            make_int2((int)(L ? lofs + i : i), prev);
    }
  }
}

// ---------------------------------------------------------------------------
// candidates: one wave per listed sample, one lane per kept score within the
// limit: the reference arithmetic (numpy's pairwise order, correctly
// rounded sqrt) on that centre, then the wave's first-index argmin.
// ---------------------------------------------------------------------------
template <bool COOP, class TX>
__global__ void __launch_bounds__(256)
    k_gemm_cand(const TX *__restrict__ X, int64_t row0, int d, int64_t ldx,
                const double *__restrict__ C, int k, int nct, int dpad,
                const int2 *__restrict__ part, const float *__restrict__ xnv,
                WsView v, int32_t *__restrict__ lab_out, double *acc,
                int flags) {
  __shared__ LeafTab tab;
  __shared__ double tots[4][GMAXLEAF];
  const uint32_t cnt = v.hdr->gcount;
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && threadIdx.x == 0 && cnt)  // diagnostics
    atomicAdd((unsigned long long *)&v.hdr->rechecked_total,
              (unsigned long long)cnt);
  if (blockIdx.x * (blockDim.x / 64) >= cnt) return;  // no listed sample
  const bool coop = COOP;  // d <= 8192: one numpy iterator buffer per row
  if (coop && threadIdx.x == 0) build_leaves(d, tab);
  __syncthreads();
  double *tot = tots[threadIdx.x >> 6];
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  for (uint32_t e = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
       e < cnt; e += nw) {  // wave-uniform
    const int2 it = v.tlist[e];
    const int64_t i = it.x, si = row0 + i;
    const int2 *pp = part + i * (int64_t)nct * GTOP;
    // best kept score (wave min over the entries), then the limit
    float p1 = INFINITY;
    int i1 = 0x7fffffff;
    for (int q = lane; q < nct * GTOP; q += 64) {
      const int2 c = pp[q];
      if (vi_less(__int_as_float(c.x), c.y, p1, i1)) {
        p1 = __int_as_float(c.x);
        i1 = c.y;
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float op = __shfl_xor(p1, off, 64);
      const int oi = __shfl_xor(i1, off, 64);
      if (vi_less(op, oi, p1, i1)) {
        p1 = op;
        i1 = oi;
      }
    }
    const float lim = p1 + gemm_bound2(dpad, xnv[i], cm, flags & 4);
    const TX *xr = X + si * ldx;
    double best = INFINITY;
    int lab = 0x7fffffff;  // lanes without a candidate never win
    if constexpr (COOP) {
      // candidates one at a time (wave-uniform), each distance by the wave
      for (int q = 0; q < nct * GTOP; ++q) {
        const int2 c = pp[q];
        if (!(__int_as_float(c.x) <= lim)) continue;
        const double dist =
            argmin_key(sqrt(wave_sqdist(xr, C + (int64_t)c.y * d, d, tab, tot,
                                        lane)));
        if (lab == 0x7fffffff || dist < best || (dist == best && c.y < lab)) {
          best = dist;
          lab = c.y;
        }
      }
    } else {
      // one candidate per lane, the row's pairwise sum sequentially
      for (int q = lane; q < nct * GTOP; q += 64) {
        const int2 c = pp[q];
        if (!(__int_as_float(c.x) <= lim)) continue;
        const double dist =
            argmin_key(sqrt(pw_sum(SqDiff<TX>{xr, C + (int64_t)c.y * d}, d)));
        if (lab == 0x7fffffff || dist < best || (dist == best && c.y < lab)) {
          best = dist;
          lab = c.y;
        }
      }
      wave_argmin(best, lab);
    }
    if (lane == 0) lab_out[si] = lab;
    gemm_acc_wave(xr, d, k, lab, it.y, flags, acc, lane);
  }
}

// ---------------------------------------------------------------------------
// overflow scan: the samples whose kept scores cannot bound the candidates
// (some centre tile holds more than GTOP scores within the limit; or the
// bound does not hold: NaN, overflow), deferred over the chunks of a call
// (a few hundred per 10M rows on the first iterations, none later) and
// scanned here in one launch: one 1024-thread workgroup per sample, every
// centre by the reference arithmetic (lanes over centres: coalesced C^T
// reads), then the workgroup's argmin in np.argmin's order (first NaN, else
// the smallest value, then index).
// ---------------------------------------------------------------------------
template <class TX>
__global__ void __launch_bounds__(1024)
    k_gemm_full(const TX *__restrict__ X, int64_t row0, int d, int64_t ldx,
                int k, WsView v, int32_t *__restrict__ lab_out, double *acc,
                int flags) {
  __shared__ double bd[16];
  __shared__ int bi[16];
  const uint32_t cnt = v.hdr->gcount2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (blockIdx.x == 0 && threadIdx.x == 0 && cnt) {  // diagnostics
    atomicAdd((unsigned long long *)&v.hdr->rechecked_total,
              (unsigned long long)cnt);
    atomicAdd((unsigned long long *)&v.hdr->reserved[4],
              (unsigned long long)cnt);
  }
  const int64_t ldc = ct_ld(k);
  for (uint32_t e = blockIdx.x; e < cnt; e += gridDim.x) {
    const int2 it = v.tlist[GLIST2 + e];
    const int64_t si = row0 + it.x;
    const TX *xr = X + si * ldx;
    double best = INFINITY;
    int lab = 0x7fffffff;  // lanes without a centre never win
    for (int jc = threadIdx.x; jc < k; jc += 1024) {
      const double dist =
          sqrt(pw_sum(SqDiffT<TX>{xr, v.ct64 + jc, ldc}, d));
      if (nan_first_less(dist, jc, best, lab)) {
        best = dist;
        lab = jc;
      }
    }
    auto wave_min = [&]() {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const double od = __shfl_xor(best, off, 64);
        const int oi = __shfl_xor(lab, off, 64);
        if (nan_first_less(od, oi, best, lab)) {
          best = od;
          lab = oi;
        }
      }
    };
    wave_min();
    if (lane == 0) {
      bd[w] = best;
      bi[w] = lab;
    }
    __syncthreads();
    if (w == 0) {
      best = lane < 16 ? bd[lane] : INFINITY;
      lab = lane < 16 ? bi[lane] : 0x7fffffff;
      wave_min();
      if (lane == 0) bi[0] = lab;
    }
    __syncthreads();
    lab = bi[0];
    if (threadIdx.x == 0) lab_out[si] = lab;
    if (w == 0) gemm_acc_wave(xr, d, k, lab, it.y, flags, acc, lane);
    __syncthreads();  // bd / bi reused by the next sample
  }
}

template <class TX>
int launch_split(const TX *X, int64_t row0, int64_t nrows, int64_t mrows,
                 int d, int64_t ldx, double scale, char *out, float *xn,
                 int one, hipStream_t s, char *out1 = nullptr,
                 float *xn1 = nullptr) {
  const int nks = (int)(dpad32(d) / GBK);
  const bool vec = (d % 8 == 0) && ((ldx * (int64_t)sizeof(TX)) % 16 == 0) &&
                   ((uintptr_t)X % 16 == 0);
  const int64_t blocks = std::min<int64_t>((mrows + 31) / 32, 16384);
  if (vec)
    k_gemm_split<true, TX><<<(unsigned)blocks, 256, 0, s>>>(
        X, row0, nrows, mrows, d, ldx, nks, scale, out, xn, one, out1, xn1);
  else
    k_gemm_split<false, TX><<<(unsigned)blocks, 256, 0, s>>>(
        X, row0, nrows, mrows, d, ldx, nks, scale, out, xn, one, out1, xn1);
  return check_launch("gemm split");
}

}  // namespace

int gemm_prepare(const double *C, int64_t k, int64_t d, const WsView &v,
                 hipStream_t s) {
  if (!v.gfrag) return fail(DKM_E_WORKSPACE, "gemm_prepare: no GEMM region");
  const int64_t kp = kpad256(k);
  if (int r = launch_split<double>(C, 0, k, kp, (int)d, d, -2.0, v.gfrag,
                                   nullptr, 0, s))
    return r;
  if (int r = launch_split<double>(C, 0, k, kp, (int)d, d, -2.0, v.gfrag1,
                                   nullptr, 1, s))
    return r;
  k_gemm_cnorm<<<(unsigned)((kp + 255) / 256), 256, 0, s>>>(v.cn32, k, kp,
                                                            v.gcn);
  return check_launch("gemm_prepare");
}

// the second stream of gemm_screen and its events, one set per device and
// host thread (created at first use, kept for the process)
struct SplitStream {
  hipStream_t s = nullptr;
  int cus = 256;  // compute units of the device
  hipEvent_t split_ev[2] = {nullptr, nullptr}, free_ev[2] = {nullptr, nullptr};
  bool ok = false;
};
static SplitStream &split_stream() {
  static thread_local SplitStream st[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  SplitStream &x = st[dev];
  if (!x.ok) {
    bool good =
        hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking) == hipSuccess;
    for (int i = 0; i < 2 && good; ++i)
      good = hipEventCreateWithFlags(&x.split_ev[i],
                                     hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&x.free_ev[i],
                                     hipEventDisableTiming) == hipSuccess;
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount,
                              dev) == hipSuccess &&
        cu >= 8)
      x.cus = cu;
    x.ok = good;
  }
  return x;
}

template <class TX>
int gemm_screen(const TX *X, int64_t base, int64_t end, int d, int64_t ldx,
                const double *C, int k, const WsView &v, int32_t *lab_out,
                double *acc, bool delta, bool one, const XImage *img,
                hipStream_t s, const XImage *bimg) {
  if (!v.gfrag) return fail(DKM_E_WORKSPACE, "gemm_screen: no GEMM region");
  // bimg: the IMG_GEMM image the bf16x3 splits also write (whole tiles from
  // row 0 of the image)
  if (bimg && (one || base % GT || v.gchunk % GT))
    return fail(DKM_E_ARG, "gemm_screen: image build needs the bf16x3 "
                           "splits on whole tiles");
  const void *kf = one ? (const void *)k_gemm_screen1
                       : (const void *)k_gemm_screen3;
  if (hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize,
                          one ? G1LDS : GLDS) != hipSuccess)
    return fail(DKM_E_LAUNCH, "gemm_screen: LDS attribute");
  const int nks = (int)(dpad32(d) / GBK);
  const int nct = (int)(kpad256(k) / GT);
  const int dpad = (int)dpad32(d);
  // bit 2: the single-product bound in the merge and candidate steps
  const int flags = (acc ? 1 : 0) | (delta ? 2 : 0) | (one ? 4 : 0);
  // a chunk on a whole sample tile reads the resident image instead
  const bool have_img = img && img->kind == IMG_GEMM && one;
  auto from_img = [&](int64_t c0) { return have_img && c0 % GT == 0; };
  // The split of chunk c + 1 (HBM-bound) runs on a second stream while
  // chunk c is screened (MFMA-bound): split buffers alternate, chunk c's
  // screen waits for its split, and split c + 2 waits until chunk c's
  // screen, merge and candidates (the readers of its buffer) are done.
  SplitStream &ss = split_stream();
  if (!ss.ok) return fail(DKM_E_LAUNCH, "gemm: second stream");
  char *xs_b[2] = {v.gxs, v.gxs1};
  float *xn_b[2] = {v.gxn, v.gxn1};
  // the split reads X: after everything already queued on the caller's
  // stream; both buffers start free
  if (hipEventRecord(ss.free_ev[0], s) != hipSuccess ||
      hipEventRecord(ss.free_ev[1], s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "gemm: event");
  auto split = [&](int64_t c0, int b) -> int {
    if (from_img(c0)) return 0;
    const int64_t rows = std::min<int64_t>(v.gchunk, end - c0);
    if (hipStreamWaitEvent(ss.s, ss.free_ev[b], 0) != hipSuccess)
      return fail(DKM_E_LAUNCH, "gemm: stream wait");
    if (int r = launch_split<TX>(
            X, c0, rows, round_up(rows, GT), d, ldx, 1.0, xs_b[b], xn_b[b],
            one ? 1 : 0, ss.s,
            bimg ? (char *)bimg->tiles + (c0 / GT) * (int64_t)nks * GSTAGE1
                 : nullptr,
            bimg ? (float *)bimg->xx + c0 : nullptr))
      return r;
    if (hipEventRecord(ss.split_ev[b], ss.s) != hipSuccess)
      return fail(DKM_E_LAUNCH, "gemm: event");
    return 0;
  };
  if (end - base > INT32_MAX)
    return fail(DKM_E_ARG, "gemm_screen: more than 2^31 - 1 rows per call");
  if (base < end) {
    if (int r = split(base, 0)) return r;
    if (hipMemsetAsync(&v.hdr->gcount2, 0, 4, s) != hipSuccess)
      return fail(DKM_E_LAUNCH, "gemm: list reset");
  }
  int64_t pending = 0;  // rows merged since the overflow list was scanned
  int b = 0;
  for (int64_t c0 = base; c0 < end; c0 += v.gchunk, b ^= 1) {
    const int64_t rows = std::min<int64_t>(v.gchunk, end - c0);
    const int64_t mrows = round_up(rows, GT);
    const int nst = (int)(mrows / GT);
    if (c0 + v.gchunk < end)
      if (int r = split(c0 + v.gchunk, b ^ 1)) return r;
    const char *xs = xs_b[b];
    const float *xn = xn_b[b];
    if (from_img(c0)) {
      xs = (const char *)img->tiles + (c0 / GT) * (int64_t)nks * GSTAGE1;
      xn = img->xx + c0;
    } else if (hipStreamWaitEvent(s, ss.split_ev[b], 0) != hipSuccess) {
      return fail(DKM_E_LAUNCH, "gemm: stream wait");
    }
    WsView vb = v;  // the merge and candidate steps read this chunk's xn
    vb.gxn = (float *)xn;
    if (one) {
      // persistent: one workgroup per CU (G1LDS of LDS each), a multiple
      // of the 8 XCDs
      const int64_t G = (int64_t)nst * nct;
      const int64_t nwg = 8 * std::min<int64_t>(ss.cus / 8, (G + 7) / 8);
      k_gemm_screen1<<<(unsigned)nwg, GTHREADS, G1LDS, s>>>(
          v.gfrag1, v.gcn, xs, nst, nct, nks, v.gpart, &v.hdr->gcount);
    } else {
      k_gemm_screen3<<<(unsigned)(nst * nct), GTHREADS, GLDS, s>>>(
          v.gfrag, v.gcn, xs, nst, nct, nks, v.gpart, &v.hdr->gcount);
    }
    if (int r = check_launch("gemm screen")) return r;
    const unsigned mb = (unsigned)std::min<int64_t>((rows + 255) / 256, 8192);
    k_gemm_merge<TX><<<mb, 256, 0, s>>>(X, c0, rows, d, ldx, k, nct, dpad,
                                        v.gpart, xn, vb, lab_out, acc, flags,
                                        c0 - base);
    if (int r = check_launch("gemm merge")) return r;
    // a wave per listed sample, up to 8 workgroups of 4 waves per CU (the
    // list length is known on the device only; idle waves exit at once)
    const unsigned cb = (unsigned)std::min<int64_t>((rows + 3) / 4,
                                                    (int64_t)ss.cus * 8);
    if (d <= 8192)
      k_gemm_cand<true, TX><<<cb, 256, 0, s>>>(X, c0, d, ldx, C, k, nct, dpad,
                                               v.gpart, xn, vb, lab_out, acc,
                                               flags);
    else
      k_gemm_cand<false, TX><<<cb, 256, 0, s>>>(X, c0, d, ldx, C, k, nct,
                                                dpad, v.gpart, xn, vb,
                                                lab_out, acc, flags);
    if (int r = check_launch("gemm candidates")) return r;
    if (hipEventRecord(ss.free_ev[b], s) != hipSuccess)
      return fail(DKM_E_LAUNCH, "gemm: event");
    // the deferred overflow list: scanned before it could outgrow its half
    // of tlist, and at the end
    pending += rows;
    if (c0 + v.gchunk >= end || pending + v.gchunk > GLIST2) {
      k_gemm_full<TX><<<(unsigned)ss.cus, 1024, 0, s>>>(X, base, d, ldx, k, v,
                                                       lab_out, acc, flags);
      if (int r = check_launch("gemm overflow scan")) return r;
      if (hipMemsetAsync(&v.hdr->gcount2, 0, 4, s) != hipSuccess)
        return fail(DKM_E_LAUNCH, "gemm: list reset");
      pending = 0;
    }
  }
  return 0;
}

template <class TX>
int gemm_image(const TX *X, int64_t n, int d, int64_t ldx, const XImage &img,
               hipStream_t s) {
  if (n == 0) return 0;
  return launch_split<TX>(X, 0, n, round_up(n, GT), d, ldx, 1.0,
                          (char *)img.tiles, (float *)img.xx, 1, s);
}

template int gemm_screen<double>(const double *, int64_t, int64_t, int,
                                 int64_t, const double *, int, const WsView &,
                                 int32_t *, double *, bool, bool,
                                 const XImage *, hipStream_t, const XImage *);
template int gemm_screen<float>(const float *, int64_t, int64_t, int, int64_t,
                                const double *, int, const WsView &,
                                int32_t *, double *, bool, bool,
                                const XImage *, hipStream_t, const XImage *);
template int gemm_image<double>(const double *, int64_t, int, int64_t,
                                const XImage &, hipStream_t);
template int gemm_image<float>(const float *, int64_t, int, int64_t,
                               const XImage &, hipStream_t);

}  // namespace dkm

// Code-object preload (dkm_preload): the runtime loads this file's kernels
// on first use of any of them; an attribute query here does it up front.
namespace dkm {
DKM_TU_FLAGS(gemm, 0)
__global__ void k_tu_gemm() {}
int preload_gemm() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void *)k_tu_gemm) == hipSuccess ? 0
                                                                       : 1;
}
}  // namespace dkm
