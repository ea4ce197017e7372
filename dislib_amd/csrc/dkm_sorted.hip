// dkm_sorted.hip -- the steady-state threshold pass over the label-sorted
// sample image (k_screen_sorted): the hot kernel of the C3 fit (125M x 64,
// k = 1000 per GPU) once labels have settled.
//
// Reference step: `_partial_sum`'s distance + argmin (dislib
// cluster/kmeans/base.py:171-173, `_vec_matrix_euclid` :204-205).  Labels
// stay bit-exact: a sample is decided here only when the rigorous bf16
// bound proves its winner; the rest go to the same candidate / re-check
// lists as k_screen_b2 (dkm_b2.hip), whose arithmetic this kernel shares.
//
// What it does differently from k_screen_b2's IMG_SORTED path (which stays
// as the fallback for the tiles listed here):
//
// * One reference centre per tile.  The threshold of row x may come from
//   ANY centre q: with T = s_hat_q + 2B, every centre whose score exceeds T
//   is strictly farther than q, and the winner w has s_w <= D_w + B <= D_q +
//   B <= T, so it is always kept.  The hint of the tile's first row, p0,
//   serves every row: no per-row hints, no own-block MFMA, no own-mask
//   words.  A row whose incoming label is another centre q (a sample that
//   moved since the image was sorted) simply keeps q among its entries.
// * The block mask is wave-uniform by construction (one ballot), so the
//   block loop pops it in SALU and the only VALU per block is the 16-row
//   minimum, one select (p0's own column) and the compare.
// * Kept pairs are not appended inside the loop: the loop records which
//   blocks passed (one SGPR bit each) and, after it, those blocks are
//   re-run and their (row, score, centre) pairs listed.  The loop body
//   carries no append code and no registers for it.
// * Chunk-cyclic tile order: a wave walks SCH consecutive image tiles (one
//   cluster, nearly always), so p0's block-bound row (mind) is re-read only
//   when p0 changes.
// * u (the bound on |x - c_p0| that clears blocks) is reduced over the rows
//   with DPP before a single square root.
//
// A tile is handed to k_screen_b2 (tile-list mode) when no row carries a
// valid label, when a row is not finite / too large for the fp32 bound, or
// when more than B2_RTHR rows keep more than SENT entries (b2's top-3
// pass).  Nothing of such a tile is written here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <type_traits>

#include "dkm_b2.h"

namespace dkm {

#ifndef DKM_AB_SBS
#define DKM_AB_SBS 768
#endif
constexpr int SBS = DKM_AB_SBS;  // threads per block (12 waves: 3 per SIMD)
// debug / A/B: 1 = hand every tile to k_screen_b2, 2 = screen every block
#ifndef DKM_AB_SORTED_DBG
#define DKM_AB_SORTED_DBG 0
#endif
// timing probe (results INVALID): the bound divided by this factor, to
// measure the work a tighter bound would leave
#ifndef DKM_AB_SORTED_BSCALE
#define DKM_AB_SORTED_BSCALE 1
#endif
constexpr int SCH = 16;          // consecutive image tiles per chunk
// kept (score, centre) entries per row besides its hint: up to 1 + SENT
// candidates go to k_candn's 6-centre list instead of the exhaustive
// re-check (k_screen_b2 keeps 3)
constexpr int SENT = 5;
// per-wave LDS scratch: -T[32], count[32], s_hat_p[32], 2B[32], hint[32],
// then the kept entries [32][SENT] (score bits, centre)
constexpr int SS_BYTES = 5 * 128 + 32 * SENT * 8;

// max of a float over the 32 lanes of each half-wave (both halves hold the
// same rows): DPP within 16-lane rows, then a 16-lane swap.  The values are
// >= 0 or -0.0 and never NaN, so their bits order as signed integers
// (-0.0 is the smallest): v_max_i32, no NaN canonicalisation.
template <int CTRL>
__device__ __forceinline__ int dpp_max_i32(int v) {
  const int o = __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
  return v > o ? v : o;
}
__device__ __forceinline__ float rows_max32(float x) {
  int v = __float_as_int(x);
  v = dpp_max_i32<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v = dpp_max_i32<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v = dpp_max_i32<0x124>(v);  // row_ror 4
  v = dpp_max_i32<0x128>(v);  // row_ror 8
  int a, b;
  pair_xor<16>(v, a, b);
  return __int_as_float(a > b ? a : b);
}

// Work distribution: chunks of SCH consecutive image tiles (one cluster,
// nearly always) handed out by a global counter (hdr->qhead) -- a static
// chunk-cyclic order left the waves that drew the crowded clusters running
// long after the rest (waves alive 53 % of the launch at C3).  The next
// chunk is claimed when a chunk starts, so its atomic has long returned when
// its first tile is prefetched.  Tiles handed to k_screen_b2 go to fall[]
// (count *nfall; rare: an atomic each).
// W1: the block mask fits 32 bits (nkb <= 32).
template <int NKS, bool W1>
__global__ void __launch_bounds__(SBS)
    k_screen_sorted(int64_t n, int d, int k, B2View v,
                    int32_t *__restrict__ lab_out, XImage img,
                    int32_t *__restrict__ fall, uint32_t *nfall) {
  typedef typename std::conditional<W1, uint32_t, uint64_t>::type bmask_t;
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nkb = (int)(kpad32(k) / 32);
  char *frag = (char *)smem;                                // nkb x NKS KB
  float *ncn = (float *)(frag + (int64_t)nkb * NKS * 1024);  // -|c|^2
  char *scr0 = (char *)(ncn + nkb * 32);
  {
    const f32x4 *src = (const f32x4 *)v.b1frag;
    f32x4 *dst = (f32x4 *)frag;
    for (int e = threadIdx.x; e < nkb * NKS * 64; e += SBS) dst[e] = src[e];
    for (int e = threadIdx.x; e < nkb * 32; e += SBS)
      ncn[e] = e < k ? -v.cn32[e] : -0x1.0p100f;  // padding: never passes
  }
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  // the threshold bound of k_screen_b2 (see dkm_b2.hip's header)
  const float relt = 1.02f * 0x1.0p-8f + (48.0f * NKS + 32.0f) * 0x1.0p-23f;
  BoundK bkt = bound_consts<P_F32>(d, cm);
  bkt.k_mag = __int_as_float(__builtin_amdgcn_readfirstlane(
      __float_as_int(2.0f * (2.0f * relt) * 1.0001f)));
  const float ninf = __uint_as_float(opaque_u32(0xff800000u));
  __syncthreads();

  const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int NW = SBS / 64;
  const int64_t wv = (int64_t)blockIdx.x * NW + wid;
  const int64_t nwv = (int64_t)gridDim.x * NW;
  const int64_t nt = (n + 31) / 32;  // image tiles (whole: perm -1 past n)
  char *scr = scr0 + (int64_t)wid * SS_BYTES;
  float *s_tn = (float *)scr;           // -T per row
  int *s_cnt = (int *)(scr + 128);      // kept entries appended
  float *s_sp = (float *)(scr + 256);   // s_hat_p per row (its own hint p)
  float *s_bt = (float *)(scr + 384);   // 2B per row
  int *s_hp = (int *)(scr + 512);       // hint p per row (mixed tiles)
  int2 *s_ent = (int2 *)(scr + 640);    // (score bits, centre)
  int2 *wl = v.tlist + wv * TL_CAP;     // >= 3 candidates / undecided
  int2 *cl = v.clist + wv * B1_CAP;     // 2 candidates
  int4 *nl = v.nlist + wv * B1_NCAP;    // 3..6 candidates
  const bool listing = wv < TL_SEGS && wv < B1_SEGS;
  int tl_cnt = 0, cl_cnt = 0, nl_cnt = 0, tl_over = 0;
  uint32_t t_tiles = 0, t_done = 0, t_blocks = 0;

  auto load_img = [&](int64_t t, bf16x8 (&dst)[NKS], float &xxd, int &pvd,
                      int &sidd) {
    const bf16x8 *src = (const bf16x8 *)(img.tiles + t * (NKS * 512)) + lane;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      dst[ks] = __builtin_nontemporal_load(src + 64 * ks);
    xxd = __builtin_nontemporal_load(img.xx + t * 32 + r);
    sidd = __builtin_nontemporal_load(img.perm + t * 32 + r);
    pvd = img.plab[t * 32 + r];
  };
  auto to_fallback = [&](int64_t t) {
    if (lane == 0) fall[atomicAdd(nfall, 1u)] = (int32_t)t;
  };
  // s_hat_q = |c_q|^2 + x.(-2 c_q)h for this lane's row and its centre q:
  // VALU dot products of the lane's own operand registers with c_q's (exact
  // bf16 products, an fp32 chain within the bound's chain term)
  auto s_hat = [&](const bf16x8 (&xh)[NKS], int q) {
    bf16x8 of[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      of[ks] = *(const bf16x8 *)(frag + ((int64_t)(q >> 5) * NKS + ks) * 1024 +
                                 ((q & 31) + 32 * h) * 16);
    float dg = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; j += 2)
        dg = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{xh[ks][j], xh[ks][j + 1]},
                                             bf16x2{of[ks][j], of[ks][j + 1]},
                                             dg, false);
    float da, db;
    pair_xor<32>(dg, da, db);
    return (da + db) - ncn[q];
  };

  int pc = -1;            // the centre whose mind row mnd holds
  float mnd = INFINITY;   // lane cb: mind[pc][cb]

  // ---- one tile ------------------------------------------------------------
  // p0 = the tile's reference centre (its first labelled row's label, >= 0)
  auto process = [&](int64_t t, const bf16x8 (&xh)[NKS], float xx, int prv,
                     int sid, int p0) {
    const int64_t s0 = t * 32;
    const bool valid = sid >= 0;
    // the row's own hint (its label when in [0, k), else p0)
    const int pr = valid && (unsigned)prv < (unsigned)k ? prv : p0;
    const bool minor = valid && pr != p0;
    const bool mixed = __ballot(minor) != 0;
    const float sp0 = s_hat(xh, p0);
    const float sp = mixed ? s_hat(xh, pr) : sp0;
    float xn;
    const float B2t = bound2_fast(bkt, xx, xn) / DKM_AB_SORTED_BSCALE;
    const bool rowok = (xn < 1e18f) & (xn * cm < 1e30f) &
                       (sp + B2t < 1e30f) & (sp0 + B2t < 1e30f);
    if (__ballot(valid && !rowok)) {  // non-finite / huge rows: b2 lists them
      to_fallback(t);
      return;
    }
    // T from the row's own hint: any centre whose score exceeds it is
    // strictly farther than the hint, the winner's score never does
    const float T = sp + B2t;
    // u >= |x - c_p0| (reference arithmetic) for every row: D^2 <= |x|^2 +
    // s_hat_p0 + B2t / 2, with 2^-16 on the fp32 |x|^2 and 2^-19 on the root
    // (v_sqrt_f32 is within 1 ulp).  A block whose centres are all farther
    // than 2u from c_p0 (mind) holds only centres strictly farther than
    // c_p0 from every row (triangle inequality): they can neither win nor
    // tie, whatever the row's threshold.
    const float u2 =
        valid ? fmaxf(fmaf(xx, 1.0f + 0x1.0p-16f, sp0 + B2t), 0.f) : 0.f;
    const float U = __builtin_amdgcn_sqrtf(rows_max32(u2)) *
                    (1.0f + 0x1.0p-19f);
    const float U2 = __int_as_float(
        __builtin_amdgcn_readfirstlane(__float_as_int(2.0f * U)));
    const bmask_t bmask = (bmask_t)__ballot(
        lane < nkb && (DKM_AB_SORTED_DBG == 2 || !(mnd > U2)));

    // ---- per-wave scratch: -T per row -> the chains' initial accumulator
    wave_sync();  // the previous tile's scratch reads are done
    if (h == 0) {
      s_tn[r] = valid ? -T : INFINITY;
      s_sp[r] = sp;
      s_bt[r] = B2t;
      // a minority row keeps p0 when p0 can still win: p0's column is
      // skipped in the block tests of every row (below)
      const bool seed = minor && sp0 <= T;
      s_cnt[r] = seed ? 1 : 0;
      if (seed) s_ent[r * SENT] = make_int2(__float_as_int(sp0), p0);
      if (mixed) s_hp[r] = valid ? pr : -1;
    }
    wave_sync();
    f32x16 cin;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 t4 = *(const f32x4 *)(s_tn + 8 * q + 4 * h);
      cin[4 * q] = t4.x;
      cin[4 * q + 1] = t4.y;
      cin[4 * q + 2] = t4.z;
      cin[4 * q + 3] = t4.w;
    }
    // p0's column: its score is entry 0 (or a seeded entry) of every row,
    // so the block test skips it (a NaN threshold never passes)
    const int pb = p0 >> 5;
    const bool ownl = r == (p0 & 31);
    auto rd_f = [&](int cb, bf16x8 (&f)[NKS]) {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
        f[ks] = *(const bf16x8 *)(frag + ((int64_t)cb * NKS + ks) * 1024 +
                                  lane * 16);
    };
    const float *ncn_r = ncn + r;
    auto rd_n = [&](int cb) { return ncn_r[cb * 32]; };
    auto mm = [&](const bf16x8 (&f)[NKS], f32x16 &acc) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[0], f[0], cin, 0, 0, 0);
#pragma unroll
      for (int ks = 1; ks < NKS; ++ks)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[ks], f[ks], acc, 0, 0,
                                                      0);
    };
    auto thr_of = [&](int cb, float nc) {
      return (cb == pb && ownl) ? __uint_as_float(0x7fc00000u) : nc;
    };
    bmask_t passed = 0;  // blocks holding a kept (row, centre) pair
    auto test = [&](int cb, const f32x16 &acc, float nc) {
      if (__ballot(min16(acc, ninf) <= thr_of(cb, nc)))
        passed |= (bmask_t)1 << cb;
    };
    // the blocks of bmask, software-pipelined one block deep: chain c1 is
    // issued before block c0 is tested, the fragments of c2 read meanwhile
    {
      f32x16 acc_a, acc_b;
      bf16x8 fa[NKS], fb[NKS];
      float na = 0.f, nb = 0.f;
      bmask_t m = bmask;
      auto pop = [&]() -> int {
        const int c = m ? (int)__builtin_ctzll((uint64_t)m) : 0;
        m &= m - 1;
        return c;
      };
      int left = __popcll((uint64_t)bmask);
      if (left > 0) {
        int c0 = pop(), c1 = pop(), c2 = pop(), c3 = pop();
        rd_f(c0, fa);
        na = rd_n(c0);
        mm(fa, acc_a);  // chain c0
        if (left > 1) {
          rd_f(c1, fb);
          nb = rd_n(c1);
        }
        for (; left > 3; left -= 2) {
          mm(fb, acc_b);  // chain c1
          rd_f(c2, fa);
          test(c0, acc_a, na);
          na = rd_n(c2);
          mm(fa, acc_a);  // chain c2
          rd_f(c3, fb);
          test(c1, acc_b, nb);
          nb = rd_n(c3);
          c0 = c2;
          c1 = c3;
          c2 = pop();
          c3 = pop();
        }
        // tail: 1, 2 or 3 blocks left (chain c0 issued, c1 read)
        if (left > 1) {
          mm(fb, acc_b);  // chain c1
          if (left > 2) rd_f(c2, fa);
          test(c0, acc_a, na);
          if (left > 2) {
            na = rd_n(c2);
            mm(fa, acc_a);  // chain c2
          }
          test(c1, acc_b, nb);
          if (left > 2) test(c2, acc_a, na);
        } else {
          test(c0, acc_a, na);
        }
      }
    }
    // ---- the passed blocks again: list their kept (row, score, centre) ----
    // (a minority row's own hint passes its test: it is entry 0, not listed)
    if (passed) {
      auto push = [&](int row, float s, int j) {
        const int slot = atomicAdd(&s_cnt[row], 1);
        if (slot < SENT)
          s_ent[row * SENT + slot] = make_int2(__float_as_int(s), j);
      };
      int pg[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        int4 p4 = make_int4(-1, -1, -1, -1);
        if (mixed) p4 = *(const int4 *)(s_hp + 8 * q + 4 * h);
        pg[4 * q] = p4.x;
        pg[4 * q + 1] = p4.y;
        pg[4 * q + 2] = p4.z;
        pg[4 * q + 3] = p4.w;
      }
      for (bmask_t pm = passed; pm; pm &= pm - 1) {
        const int cb = (int)__builtin_ctzll((uint64_t)pm);
        bf16x8 f[NKS];
        rd_f(cb, f);
        const float nc = rd_n(cb);
        f32x16 acc;
        mm(f, acc);
        const float thr = thr_of(cb, nc);
        const int j = cb * 32 + r;
#pragma unroll
        for (int g = 0; g < 16; ++g)
          if (acc[g] <= thr && j != pg[g]) {
            const int row = (g & 3) + 8 * (g >> 2) + 4 * h;
            push(row, (acc[g] - cin[g]) - nc, j);
          }
      }
    }
    // ---- decision ------------------------------------------------------------
    // steady state: no pair kept and every row already labelled p0
    if (!passed && __ballot(valid && h == 0 && prv != p0) == 0) {
      ++t_tiles;
      ++t_done;
      t_blocks += (uint32_t)__popcll((uint64_t)bmask);
      if (DKM_AB_SORTED_DBG == 3 && valid && h == 0)
        lab_out[sid] = 1000000 + __popcll(bmask) * 10000;
      return;
    }
    wave_sync();
    const int cnt = s_cnt[r];
    if (DKM_AB_SORTED_DBG == 4 || DKM_AB_SORTED_DBG == 5) {
      if (valid && h == 0)
        lab_out[sid] = 0x40000000 |
                       (int)((DKM_AB_SORTED_DBG == 4 ? passed : bmask) &
                             0x3fffffff);
      return;
    }
    if (DKM_AB_SORTED_DBG == 3) {
      if (valid && h == 0)
        lab_out[sid] = 10000000 + p0 * 1000 + __popcll(passed) * 100 +
                       cnt * 10 + (mixed ? 1 : 0);
      return;
    }
    const float spr = s_sp[r], btr = s_bt[r];
    float sv[SENT + 1];
    int cv[SENT + 1];
    bool ok[SENT + 1];
    sv[0] = spr;
    cv[0] = pr;
    ok[0] = true;
#pragma unroll
    for (int e = 0; e < SENT; ++e) {
      const int2 en = s_ent[r * SENT + e];
      sv[e + 1] = __int_as_float(en.x);
      cv[e + 1] = en.y;
      ok[e + 1] = e < cnt && (unsigned)en.y < (unsigned)k;
    }
    const bool over = cnt > SENT;
    const uint64_t mo = __ballot(over && valid && h == 0);
    if (__popcll(mo) > B2_RTHR) {  // b2's top-3 pass takes the tile
      to_fallback(t);
      return;
    }
    ++t_tiles;
    ++t_done;
    t_blocks += (uint32_t)__popcll((uint64_t)bmask);
    float bs = INFINITY;
    int bc = 0x7fffffff;
#pragma unroll
    for (int e = 0; e <= SENT; ++e)
      if (ok[e] && (sv[e] < bs || (sv[e] == bs && cv[e] < bc))) {
        bs = sv[e];
        bc = cv[e];
      }
    int namb = 0, other = 0;
    uint32_t pk[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu};
#pragma unroll
    for (int e = 0; e <= SENT; ++e)
      if (ok[e] && !(sv[e] - bs > btr)) {
#pragma unroll
        for (int w = 0; w < 6; ++w)
          if (w == namb)
            pk[w >> 1] = (w & 1) ? (pk[w >> 1] & 0xffffu) |
                                       ((uint32_t)cv[e] << 16)
                                 : (pk[w >> 1] & 0xffff0000u) |
                                       (uint32_t)cv[e];
        ++namb;
        other = cv[e] != bc ? cv[e] : other;
      }
    const bool unique = !over && namb == 1;
    const bool two = !over && namb == 2;
    const bool many = !over && namb >= 3;
    const bool vrow = valid && h == 0;
    bool nlisted = false;
    {
      const uint64_t mn = __ballot(vrow && many);
      const int addn = __popcll(mn);
      if (addn && listing && nl_cnt + addn <= B1_NCAP) {
        if (vrow && many)
          nl[nl_cnt + lane_prefix(mn)] =
              make_int4(sid, (int)pk[0], (int)pk[1], (int)pk[2]);
        nl_cnt += addn;
        nlisted = many;
      }
    }
    const uint64_t mc = __ballot(vrow && two);
    const uint64_t mt = __ballot(vrow && !unique && !two && !nlisted);
    const int addc = __popcll(mc), addt = __popcll(mt);
    if (listing && cl_cnt + addc <= B1_CAP) {
      if (vrow && two)
        cl[cl_cnt + lane_prefix(mc)] = make_int2(sid, bc | (other << 16));
      cl_cnt += addc;
    } else {
      tl_over += addc;
    }
    if (listing && tl_cnt + addt <= TL_CAP) {
      if (vrow && !unique && !two && !nlisted)
        wl[tl_cnt + lane_prefix(mt)] = make_int2(sid, -1);
      tl_cnt += addt;
    } else {
      tl_over += addt;
    }
    // a label equal to the incoming one needs no store; an N-listed sample
    // keeps it until k_candn writes the winner; a sample that overflowed a
    // list keeps -1 and the label scan finds it.  Every row whose label
    // changes or goes to a re-check gets -(previous + 2) in the image's
    // label copy (previous outside [0, k): -1), which k_plab syncs.
    if (vrow) {
      const bool same = unique && bc == prv;
      if (!nlisted && !same) lab_out[sid] = unique ? bc : -1;
      if (!same) {
        const int pm = (unsigned)prv < (unsigned)k ? prv : -1;
        img.plab[s0 + r] = -(pm + 2);
      }
    }
  };

  // ---- chunks from the global counter; the next one claimed early --------
  uint32_t *qhead = &v.hdr->qhead;
  const int64_t nch = (nt + SCH - 1) / SCH;
  // the atomic's value stays in lane 0's register until the chunk switch
  // that uses it (a chunk later: long returned, so no wait on it there)
  auto claim = [&]() -> uint32_t {
    uint32_t q = 0;
    if (lane == 0) q = atomicAdd(qhead, 1u);
    return q;
  };
  auto value = [&](uint32_t q) -> int64_t {
    return (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)q);
  };
  int64_t c = value(claim());
  uint32_t qnext = c < nch ? claim() : (uint32_t)nch;
  int64_t t = c * SCH;
  int ci = 0;
  bf16x8 xq[NKS];
  float xxq = 0.f;
  int pq = -1, sq = -1;
  if (c < nch) load_img(t, xq, xxq, pq, sq);
  while (c < nch) {
    bf16x8 xh[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) xh[ks] = xq[ks];
    const float xx = xxq;
    const int prv = pq, sid = sq;
    // the tile's reference centre, and its block-bound row when it changed:
    // loaded BEFORE the next tile's prefetch, so that waiting for it leaves
    // the prefetch in flight (vmcnt counts in issue order)
    const uint64_t bh =
        __ballot(sid >= 0 && (unsigned)prv < (unsigned)k) & 0xffffffffull;
    const int p0 =
        bh ? __builtin_amdgcn_readlane(prv, (int)__builtin_ctzll(bh)) : -1;
    if (p0 >= 0 && p0 != pc) {
      pc = p0;
      mnd = lane < nkb ? v.mind[(int64_t)p0 * MIND_LD + lane] : INFINITY;
      // waited for here, before the prefetch is issued (about once per
      // chunk): the compiler's own wait at the use, after the join, would
      // be a vmcnt(0) that also waits for the prefetch on every tile
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    }
    const int64_t tcur = t;
    if (++ci < SCH && t + 1 < nt) {
      ++t;
    } else {
      // the next chunk (claimed a chunk ago), and the one after it
      c = value(qnext);
      if (c < nch) qnext = claim();
      ci = 0;
      t = c * SCH;
    }
    if (c < nch) load_img(t, xq, xxq, pq, sq);  // in flight meanwhile
    if (p0 >= 0 && DKM_AB_SORTED_DBG != 1)
      process(tcur, xh, xx, prv, sid, p0);
    else if (__ballot(sid >= 0))
      to_fallback(tcur);  // no usable label: b2's top-3 pass
  }
  if (wv == 0 && lane == 0) v.hdr->lseg = (int32_t)nwv;
  if (lane == 0 && listing) {
    v.tcount[wv] = tl_cnt;
    v.ccount[wv] = cl_cnt;
    v.ncount[wv] = nl_cnt;
  }
  if (lane == 0 && t_tiles) {  // diagnostics (dkm_screen_counters)
    atomicAdd((unsigned long long *)&v.hdr->reserved[0],
              (unsigned long long)t_tiles);
    atomicAdd((unsigned long long *)&v.hdr->reserved[1],
              (unsigned long long)t_done);
  }
  if (lane == 0 && t_blocks)
    atomicAdd((unsigned long long *)&v.hdr->reserved[2],
              (unsigned long long)t_blocks);
  if (lane == 0 && tl_over) atomicAdd(&v.hdr->qcount, (uint32_t)tl_over);
}

static size_t sorted_lds_bytes(int64_t k, int64_t d) {
  const int64_t nkb = kpad32(k) / 32;
  return (size_t)nkb * (dpad16(d) / 16) * 1024 + (size_t)nkb * 128 +
         (size_t)(SBS / 64) * SS_BYTES;
}

static unsigned sorted_grid(int64_t nt, int cus) {
  constexpr int nw = SBS / 64;
  const int64_t need = (nt + (int64_t)nw * SCH - 1) / ((int64_t)nw * SCH);
  return (unsigned)std::max<int64_t>(
      1, std::min<int64_t>({need, (int64_t)cus,
                            (int64_t)std::min(TL_SEGS, B1_SEGS) / nw}));
}

int launch_screen_sorted(int64_t n, int d, int k, const WsView &v,
                         int32_t *lab_out, XImage img, int cus, hipStream_t s,
                         int *nseg, int32_t *fall, uint32_t *nfall) {
  if (img.kind != IMG_SORTED || !v.mind || !v.b1frag || d > 128 ||
      kpad32(k) / 32 > 64)
    return 1;
  const size_t lds = sorted_lds_bytes(k, d);
  if (lds > 160 * 1024) return 1;
  const int64_t nt = (n + 31) / 32;
  const unsigned g = sorted_grid(nt, cus);
  constexpr int nw = SBS / 64;
  const int64_t nwv = (int64_t)g * nw;
  if (nt > v.nq) return 1;  // the fallback list must fit
  const bool w1 = kpad32(k) <= 1024;
  const void *kf = nullptr;
  switch ((int)(dpad16(d) / 16)) {
#define DKM_SS(N)                                                       \
  case N:                                                               \
    kf = w1 ? (const void *)k_screen_sorted<N, true>                    \
            : (const void *)k_screen_sorted<N, false>;                  \
    break;
    DKM_SS(1) DKM_SS(2) DKM_SS(3) DKM_SS(4)
    DKM_SS(5) DKM_SS(6) DKM_SS(7) DKM_SS(8)
#undef DKM_SS
    default:
      return 1;
  }
  if (hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return fail(DKM_E_LAUNCH, "screen_sorted: LDS attribute");
  // sfall (nfall) and qhead, adjacent in the header
  static_assert(offsetof(WsHeader, qhead) == offsetof(WsHeader, sfall) + 4,
                "sfall, qhead adjacent");
  if (hipMemsetAsync(nfall, 0, 8, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "screen_sorted: memset");
  *nseg = (int)nwv;
  const B2View bv = b2_view(v, true);
  hipLaunchKernelGGL((void (*)(int64_t, int, int, B2View, int32_t *, XImage,
                               int32_t *, uint32_t *))kf,
                     dim3(g), dim3(SBS), lds, s, n, d, k, bv, lab_out, img,
                     fall, nfall);
  return check_launch("screen assignment (label-sorted image)");
}

}  // namespace dkm

// Code-object preload (dkm_preload): the runtime loads this file's kernels
// on first use of any of them; an attribute query here does it up front.
namespace dkm {
DKM_TU_FLAGS(sorted, DKM_AB_SORTED_BSCALE != 1 || DKM_AB_SORTED_DBG != 0)
__global__ void k_tu_sorted() {}
int preload_sorted() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void *)k_tu_sorted) == hipSuccess ? 0
                                                                       : 1;
}
}  // namespace dkm
