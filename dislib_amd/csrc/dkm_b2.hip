// dkm_b2.hip -- single-product screen with the centres on the lanes
// (k_screen_b2): the threshold pass of the k x d > LDS-sums shapes (C3:
// 125M x 64, k = 1000 per GPU), replacing k_screen_b1's (dkm_dense.hip).
//
// The reference step it serves is `_partial_sum`'s distance + argmin
// (dislib cluster/kmeans/base.py:171-173, `_vec_matrix_euclid` :204-205).
// Labels stay bit-exact: the screen only decides a sample when the bound
// proves the winner; everything else goes to the exact re-check kernels.
//
// Why the transpose.  k_screen_b1 multiplies A = centres (rows) by B =
// samples (columns), so a lane holds one sample and 16 centres, and every
// 32-centre block needs 16 norms per lane from LDS (4 ds_read_b128, as many
// LDS cycles as the block's 4 fragment reads).  At 3 waves per SIMD that is
// 2 ds_read_b128 per MFMA: the LDS array (256 B/clk/CU) is saturated at the
// MFMA rate.  Here A = samples and B = centres: lane l holds centre
// cb*32 + (l & 31) and 16 samples (rows (g & 3) + 8 (g >> 2) + 4h).  The
// accumulator starts from -T (T = the sample's threshold, a per-tile
// constant block), so the block test is
//     min_g (dot_gj - T_g) <= -|c_j|^2
// with one per-lane norm (ds_read_b32): 18 LDS cycles per block instead
// of 32, no per-block address selects.
//
// Threshold (label hint p = the sample's incoming label, as in b1):
//   s_hat_p = |c_p|^2 + x.(-2c_p)h from the same bf16 operands (an MFMA
//   "own block" whose columns are the tile's hinted centres: its diagonal),
//   T = s_hat_p + 2B.  A centre with s_j > T cannot win or tie.
// Own exclusion: the hinted centres P = {p_i} always pass.  A column whose
// centre is in P is masked (per-column bit mask over blocks, one v_bfe +
// one v_and_or per block) for every row of the tile, and the pairs
// (i, p_c), p_c in P, p_c != p_i, are tested once in the own block instead
// (duplicate hints: only the first column of a centre is tested).  So every
// (sample, centre) pair is tested exactly once, p_i itself by s_hat_p.
// Kept pairs (rare) go to a per-wave LDS list of B2_ENT entries per sample;
// the decision (unique / two / many / re-check) is b1's.
//
// Bound: B2t = 2 (1.02 2^-8 + (32 NKS + 16) 2^-23) mag: bf16 rounding of x
// and -2c, the fp32 MFMA chain (now over |T| + sum |x c|, <= 2.04 mag), the
// ŝ_p chain, and the few roundings of (acc + T) + |c|^2 -- each <= 2^-23 of
// a magnitude <= 2.04 mag.  The top-3 fallback keeps b1's packed bound.
//
// Block skipping (the label-sorted image, IMG_SORTED).  The fit builds the
// image once with its rows grouped by label (dkm_x_image_sorted_*), so a
// 32-row tile almost always carries one hint p for all its rows.  With
// u >= every row's reference distance to c_p (from s_hat_p and the bound)
// and mind[p][cb] <= the distance from c_p to the nearest other centre of
// block cb, a block with mind > 2u holds only centres strictly farther from
// every row than c_p (triangle inequality, Elkan): it is not screened.  At
// C3 most tiles then screen a third of the blocks.  The
// labels never depend on the grouping, only the speed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "dkm_b2.h"

namespace dkm {

#ifndef DKM_AB_SB2
#define DKM_AB_SB2 768
#endif
// A/B timing probes (results invalid; dkm_build_flags reports them):
// 1 = no centre-block loop, 2 = the loop's chains and reads without tests
#ifndef DKM_AB_B2_PROBE
#define DKM_AB_B2_PROBE 0
#endif
constexpr int SB2 = DKM_AB_SB2;
// A/B: the sorted image's steady state on this kernel alone (no
// k_screen_sorted)
#ifndef DKM_AB_NO_SORTED_FAST
#define DKM_AB_NO_SORTED_FAST 0
#endif
// per-wave LDS scratch: -T[32], hint[32], count[32], |x|^2[32], the tile
// transpose (32 rows x 16 bf16 features, 1 KB; the kept entries
// [32][B2_ENT] reuse it after the tile's conversion), then 32 x nkw
// own-mask words
constexpr int B2_SCR_FIXED = 4 * 128 + 1024;
static_assert(32 * B2_ENT * 8 + 128 <= 1024,
              "kept entries and s_hat_p fit the transpose");

// IMG: IMG_NONE (X converted in the kernel), IMG_SINGLE (the resident bf16
// image, sample order) or IMG_SORTED (the same image with its rows grouped
// by label: tile rows are samples perm[32 t + r], hints come from the image's
// own label copy plab, and centre blocks are skipped by the triangle bound)
template <class TX, int NKS, bool W1, int IMG>
__global__ void __launch_bounds__(SB2)
    k_screen_b2(const TX *__restrict__ X, int64_t n, int d, int64_t ldx, int k,
                B2View v, int32_t *__restrict__ lab_out, int64_t base,
                int hint, XImage img, const int32_t *__restrict__ tlst,
                const uint32_t *tlst_n) {
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  constexpr bool SORTED = IMG == IMG_SORTED;
  // tile-list mode (the tiles k_screen_sorted handed over): nothing to do
  // unless it listed some
  if (tlst && *tlst_n == 0) return;
  constexpr int GB = 1 << (PACK2 - 4);  // 32-centre blocks per top-3 group
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nkb = (int)(kpad32(k) / 32);
  // W1: one own-mask word per column (k <= 1024), held in a register
  const int nkw = W1 ? 1 : (nkb + 31) >> 5;
  char *frag = (char *)smem;                                // nkb x NKS KB
  float *cn = (float *)(frag + (int64_t)nkb * NKS * 1024);  // b1 order norms
  float *ncn = cn + nkb * 32;                               // -|c|^2, plain
  char *scr0 = (char *)(ncn + nkb * 32);
  {
    const f32x4 *src = (const f32x4 *)v.b1frag;
    f32x4 *dst = (f32x4 *)frag;
    for (int e = threadIdx.x; e < nkb * NKS * 64; e += SB2) dst[e] = src[e];
    for (int e = threadIdx.x; e < nkb * 32; e += SB2) {
      cn[e] = v.cn32f[e];
      // padding centres: -2^100 (never passes a sane threshold)
      ncn[e] = e < k ? -v.cn32[e] : -0x1.0p100f;
    }
  }
  const float cm =
      (float)__longlong_as_double((long long)v.hdr->cmax_bits) * 1.000001f;
  // top-3 fallback: b1's packed single-product bound
  const float rel = 1.02f * 0x1.0p-8f + (16.0f * NKS + 2.0f) * 0x1.0p-23f;
  BoundK bk = bound_consts<P_F32>(d, cm);
  if (v.transl) {
    // the products are x . (-2 (c - m)): their magnitude term takes
    // max ||c - m||; |c|^2 and the reference's rounding keep cm
    const float um =
        (float)__longlong_as_double((long long)v.hdr->umax_bits) * 1.000001f;
    bk.two_cm = __int_as_float(
        __builtin_amdgcn_readfirstlane(__float_as_int(2.0f * um)));
  }
  bk.k_mag = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(
      2.0f * (2.0f * rel + 0x1.0p-23f * (float)(1u << PACK2)) * 1.0001f)));
  // threshold pass: no packing, the chain over |T| + sum |x c| (see top)
  // (the chain's magnitudes stay <= 3.04 mag: the bound keeps the margin of
  // the earlier raised-threshold form)
  const float relt = 1.02f * 0x1.0p-8f + (48.0f * NKS + 32.0f) * 0x1.0p-23f;
  BoundK bkt = bk;
  bkt.k_mag = __int_as_float(__builtin_amdgcn_readfirstlane(
      __float_as_int(2.0f * (2.0f * relt) * 1.0001f)));
  const float ninf = __uint_as_float(opaque_u32(0xff800000u));
  const uint32_t vmask = opaque_u32(~PACK2_MASK);
  __syncthreads();

  const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int NW = SB2 / 64;  // screening waves per block
  const int64_t wv = (int64_t)blockIdx.x * NW + wid;
  const int64_t step = (int64_t)gridDim.x * NW * 32;
  char *scr = scr0 + (int64_t)wid * (B2_SCR_FIXED + 128 * nkw);
  float *s_tn = (float *)scr;              // -T per sample
  int *s_hp = (int *)(scr + 128);          // hint per sample (-1: none)
  int *s_cnt = (int *)(scr + 256);         // kept entries appended
  float *s_xx = (float *)(scr + 384);      // |x|^2 per sample
  // s_hat_p per sample, through the block loop (in registers it was one
  // VGPR too many: a spill reload whose vmcnt(0) waited for the prefetch);
  // the free tail of the transpose area, past the kept entries
  float *s_sp = (float *)(scr + 512 + 32 * B2_ENT * 8);
  char *s_tx = scr + 512;                   // one K-step of the tile, bf16
  int2 *s_ent = (int2 *)(scr + 512);       // (score bits, centre), later
  uint32_t *s_om = (uint32_t *)(scr + B2_SCR_FIXED);  // [word][column]
  int2 *wl = v.tlist + wv * TL_CAP;  // >= 3 candidates
  int2 *cl = v.clist + wv * B1_CAP;  // 2 candidates
  int4 *nl = v.nlist + wv * B1_NCAP; // 3..6 candidates
  int nl_cnt = 0;
  const bool listing = wv < TL_SEGS && wv < B1_SEGS;
  int tl_cnt = 0, cl_cnt = 0, tl_over = 0;
  uint32_t t_tiles = 0, t_done = 0;  // threshold passes run / accepted
  uint32_t t_blocks = 0;             // centre blocks screened (SORTED)

  // ---- tile loads: whole 128-B lines per wave-instruction ----------------
  // A lane's MFMA operand is 8 features of ITS sample, so loading it
  // directly touches 32 rows (64 lines) per wave-instruction: that pattern
  // streamed X at 3.4 TB/s (d = 64) against 6.0 TB/s for whole lines
  // (tools/membench.hip, profiles/r03/membench.txt).  Here K-step ks of
  // the tile (16 features = one 128-B line per fp64 row) is read by lanes
  // l = (row RI i + l / LR, 16-B piece l % LR): RI rows per instruction, every
  // line whole.  Each lane converts its piece to bf16 and the K-step goes
  // through a 1 KB LDS transpose into the operand layout; |x|^2 is summed
  // by the loading lanes (same rows for every K-step) and handed over the
  // same way.
  constexpr int EPL = 16 / (int)sizeof(TX);  // elements per 16-B piece
  constexpr int LR = 16 / EPL;                // lanes per row line (8 | 4)
  constexpr int RI = 64 / LR;                 // rows per instruction (8 | 16)
  constexpr int IC = 32 / RI;                 // instructions per K-step (4 | 2)
  typedef TX tx4 __attribute__((ext_vector_type(EPL)));
  tx4 raw[NKS][IC];
  int pv = -1;
  const int lrow = lane / LR, lpos = lane % LR;
  // per-instruction lane offsets (VGPRs; the K-step offset rides in the
  // instruction's immediate): as SGPR soffsets they were 4 NKS live SGPRs
  uint32_t lane_off[IC];
#pragma unroll
  for (int i = 0; i < IC; ++i)
    lane_off[i] = (uint32_t)((RI * i + lrow) * ldx * (int64_t)sizeof(TX)) +
                  (uint32_t)(16 * lpos);
  auto load_into = [&](int64_t s0, tx4 (&dst)[NKS][IC], int &pvd) {
    const int64_t rows = std::max<int64_t>(0, n - s0);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(X + std::min(s0, n) * ldx), 0,
        (int)std::min<int64_t>(rows * ldx * (int64_t)sizeof(TX), 0x7fffffff),
        0x00020000);
    if (hint) {
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(lab_out + std::min(s0, n)), 0,
          (int)std::min<int64_t>(rows * 4, 0x7fffffff), 0x00020000);
      pvd = (int)__builtin_amdgcn_raw_buffer_load_b32(rl, r * 4, 0, 0);
    }
    // every load issued before the first use; rows past n read 0
    // (num_records), features past d are zeroed at conversion
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int i = 0; i < IC; ++i)
        dst[ks][i] = __builtin_bit_cast(
            tx4, __builtin_amdgcn_raw_buffer_load_b128(
                     rx, lane_off[i] + 16 * ks * (int)sizeof(TX), 0, 0));
  };
  auto load_tile = [&](int64_t s0) { load_into(s0, raw, pv); };
  // operand half of row `row` in the transpose: swizzled by (row >> 3) & 1
  // so that the ds_read_b128 lane groups hit 64 distinct banks
  auto tx_addr = [](int row, int half) {
    return 32 * row + 16 * (half ^ ((row >> 3) & 1));
  };
  // a loading lane's piece of row RI i + lrow: tx_addr(row, half) + within
  // = RI 32 i + wofs[i & 1] (fp64: (row >> 3) & 1 = i & 1; fp32: RI = 16,
  // (row >> 3) & 1 = (lrow >> 3) & 1), two per-lane VGPRs and immediates
  uint32_t wofs[2];
  {
    const int half = EPL == 2 ? lpos >> 2 : lpos >> 1;
    const int within = EPL == 2 ? 4 * (lpos & 3) : 8 * (lpos & 1);
#pragma unroll
    for (int par = 0; par < 2; ++par)
      wofs[par] = (uint32_t)(tx_addr(RI * par + lrow, half) - 32 * RI * par +
                             within);
  }
  auto wofs_at = [&](int i) { return 32 * RI * i + wofs[EPL == 2 ? i & 1 : 0]; };

  // The image paths issue the next tile's loads after the block loop, not
  // before the tile: its 20 registers are then not live across the loop,
  // which kept the label-sorted variant from spilling (a spill reload's
  // vmcnt wait also waited for the prefetch).  C3: 13.3 against 13.6 ms
  // per step (profiles/r04/ab_latepf.txt); -DDKM_AB_B2_LATEPF=0 for A/B.
#ifndef DKM_AB_B2_LATEPF
#define DKM_AB_B2_LATEPF 1
#endif
  constexpr bool LATEPF = DKM_AB_B2_LATEPF && IMG != IMG_NONE;
  int64_t pf_s0 = 0;     // LATEPF: the next tile to prefetch (>= n: none)
  bool pf_done = true;
  // the image paths' tile loads: each lane's operand is one 16-B piece of
  // a 1 KB K-step block (whole lines), |x|^2 precomputed
  auto load_img = [&](int64_t s0, bf16x8 (&dst)[NKS], float &xxd, int &pvd,
                      int &sidd) {
    const bf16x8 *src =
        (const bf16x8 *)(img.tiles + (s0 >> 5) * (NKS * 512)) + lane;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      dst[ks] = __builtin_nontemporal_load(src + 64 * ks);
    xxd = __builtin_nontemporal_load(img.xx + s0 + r);
    if constexpr (SORTED) {
      // the image holds whole tiles: rows past n carry perm = -1
      sidd = __builtin_nontemporal_load(img.perm + s0 + r);
      pvd = img.plab[s0 + r];
    } else {
      sidd = s0 + r < n ? (int)(s0 + r) : -1;
      if (hint) {
        const int64_t rows = std::max<int64_t>(0, n - s0);
        const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(lab_out + std::min(s0, n)), 0,
            (int)std::min<int64_t>(rows * 4, 0x7fffffff), 0x00020000);
        pvd = (int)__builtin_amdgcn_raw_buffer_load_b32(rl, r * 4, 0, 0);
      }
    }
  };
  bf16x8 xq[NKS];        // the next tile (image paths)
  float xxq = 0.f;
  int pq = -1, sq = -1;
  auto late_prefetch = [&]() {
    if (LATEPF && !pf_done) {
      pf_done = true;
      if (pf_s0 < n) load_img(pf_s0, xq, xxq, pq, sq);
    }
  };

  // ---- one tile: threshold pass (or top-3), decision, lists, labels ----
  // s0 = the tile's first row (image row for SORTED), sid = this lane's
  // sample index (-1: a row past the data)
  auto process = [&](int64_t s0, const bf16x8 (&xh)[NKS], float xx, int prv,
                     int sid) {
    // (prv, p, pok and sid are re-read from the wave's LDS scratch after
    // the block loop: live across it they cost the registers that made the
    // kernel spill)
    float xn;
    const float B2t = bound2_fast(bkt, xx, xn);
    const bool sane0 = (xn < 1e18f) & (xn * cm < 1e30f);
    bool unique = false, two = false, many = false;
    int i1 = 0, i2 = 0;
    uint32_t mpk0 = 0, mpk1 = 0, mpk2 = 0;  // many: the candidate set
    bool need3 = true;
    if (hint) {
      const bool pok = prv >= 0 && prv < k && sid >= 0;
      const uint64_t bad = __ballot(!pok && sid >= 0);
      if (__popcll(bad) <= 2 * B2_RTHR) {
        const int p = pok ? prv : 0;
        // SORTED: a tile whose rows all carry one hint p0 (most of them:
        // the rows are grouped by label) skips every centre block the
        // triangle inequality clears (below); its own block is empty
        int p0 = 0;
        bool uni = false;
        float mnd = INFINITY;
        if (SORTED && v.mind) {
          p0 = __builtin_amdgcn_readfirstlane(prv);
          uni = __ballot(sid >= 0 && prv != p0) == 0 && p0 >= 0 && p0 < k;
          if (uni && lane < nkb) mnd = v.mind[(int64_t)p0 * MIND_LD + lane];
        }
        // ---- own block: columns = the tile's hinted centres p_c ----------
        f32x16 dn = f32x16{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f,
                           0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        float dg = 0.f;
        {
          bf16x8 of[NKS];
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks)
            of[ks] = *(const bf16x8 *)(frag + ((int64_t)(p >> 5) * NKS + ks) *
                                                  1024 +
                                       ((p & 31) + 32 * h) * 16);
          if (!uni) {
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks)
              dn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[ks], of[ks], dn,
                                                           0, 0, 0);
          }
          // s_hat_p's product x_r . (-2 c_p) by VALU dot products: lane
          // (r, h) holds x_r's and c_p's features 16 ks + 8h .. + 7 (xh and
          // of), so 4 NKS v_dot2c_f32_bf16 and one cross-half add (exact
          // bf16 products, an fp32 chain within the bound's chain term).
          // Selecting the MFMA's diagonal instead (one of 16 registers by a
          // per-lane index) compiled to ~100 VALU with a hazard nop each.
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
            for (int j = 0; j < 8; j += 2)
              dg = __builtin_amdgcn_fdot2_f32_bf16(
                  bf16x2{xh[ks][j], xh[ks][j + 1]},
                  bf16x2{of[ks][j], of[ks][j + 1]}, dg, false);
        }
        {
          float da, db;
          pair_xor<32>(dg, da, db);
          dg = da + db;
        }
        const float ncp = ncn[p];
        const float sp = dg - ncp;  // s_hat_p = |c_p|^2 + x.(-2 c_p)
        const float T = pok ? sp + B2t : -INFINITY;
        // ---- SORTED: the centre blocks this tile must screen -------------
        // Every row r has hint p0.  u_r bounds the reference distance
        // |x_r - c_p0| from above: D^2 <= |x|^2 + s_hat_p + B2t / 2 (the
        // screen bound), with 2^-16 on the fp32 |x|^2 and 2^-20 on the
        // root.  A block cb with mind[p0][cb] > 2 max_r u_r holds only
        // centres j with |x_r - c_j| >= |c_p0 - c_j| - |x_r - c_p0| >
        // |x_r - c_p0| for every row -- strictly farther than the hint, so
        // they can neither win nor tie (the margins cover the reference's
        // own fp64 rounding of both distances).  Rows that are not sane go
        // to the exact re-check whatever the blocks, so they do not count.
        // A tile with a few hints (a label boundary of the sorted order, a
        // sample that moved since the sort) takes the union over its hints
        // q of the blocks that q's rows need: up to 4 hints, two at a time
        // (lanes of half h test hint q_h, lane r block r) when nkb <= 32;
        // with more hints every block is screened.
        uint64_t bmask = 0;
        if (SORTED) {
          const bool rowok = sid >= 0 && sane0 && pok;
          float u = 0.f;
          if (rowok) {
            const float u2 = fmaf(xx, 1.0f + 0x1.0p-16f, sp + B2t);
            u = __builtin_sqrtf(fmaxf(u2, 0.f)) * (1.0f + 0x1.0p-20f);
          }
          if (uni) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1)
              u = fmaxf(u, __shfl_xor(u, off, 64));
            bmask = __ballot(lane < nkb && !(mnd > 2.0f * u));
          } else if (v.mind) {
            const int lpr = nkb <= 32 ? 2 : 1;  // hints per round
            // rows still to cover (lanes 0..31 = rows; half 1 duplicates)
            uint64_t todo = __ballot(h == 0 && rowok);
            for (int rd = 0; rd < 4 && todo; rd += lpr) {
              const int qa = __builtin_amdgcn_readlane(
                  prv, (int)__builtin_ctzll(todo));
              const uint64_t ma = __ballot(h == 0 && rowok && prv == qa);
              todo &= ~ma;
              int qb = qa;
              uint64_t mb = 0;
              if (lpr == 2 && todo) {
                qb = __builtin_amdgcn_readlane(prv,
                                               (int)__builtin_ctzll(todo));
                mb = __ballot(h == 0 && rowok && prv == qb);
                todo &= ~mb;
              }
              float ua = (ma >> r) & 1 ? u : 0.f;
              float ub = (mb >> r) & 1 ? u : 0.f;
#pragma unroll
              for (int off = 16; off >= 1; off >>= 1) {
                ua = fmaxf(ua, __shfl_xor(ua, off, 64));
                ub = fmaxf(ub, __shfl_xor(ub, off, 64));
              }
              const bool second = lpr == 2 && h == 1;
              const int q = second ? qb : qa;
              const float U = second ? ub : ua;
              const int cb = lpr == 2 ? r : lane;
              const bool live = cb < nkb && (!second || mb != 0);
              const float mn =
                  live ? v.mind[(int64_t)q * MIND_LD + cb] : INFINITY;
              const uint64_t nd = __ballot(live && !(mn > 2.0f * U));
              bmask |= lpr == 2 ? ((nd & 0xffffffffull) | (nd >> 32)) : nd;
            }
            if (todo) bmask = nkb >= 64 ? ~0ull : ((1ull << nkb) - 1);
          } else {
            bmask = nkb >= 64 ? ~0ull : ((1ull << nkb) - 1);
          }
        }
        // ---- per-wave scratch: -T, hints, counts, own masks --------------
        // (a uniform tile with one own-mask word per column needs no LDS
        // mask: its only hinted centre is p0, column p0 & 31 of block
        // p0 >> 5; nor the hints, nor the own block)
        const bool fast_om = uni && W1;
        wave_sync();
        if (h == 0) {
          s_tn[r] = -T;
          if (!uni) s_hp[r] = pok ? p : -1;
          s_cnt[r] = 0;
          s_sp[r] = sp;
        }
        uint32_t dup = 0;
        if (!fast_om) {
          for (int w = lane; w < 32 * nkw; w += 64) s_om[w] = 0u;
          wave_sync();
          if (h == 0 && pok) {
            const uint32_t bit = 1u << ((p >> 5) & 31);
            dup = atomicOr(&s_om[(p >> 10) * 32 + (p & 31)], bit) & bit;
          }
          int da, db;
          pair_xor<32>((int)dup, da, db);
          dup = (uint32_t)(da | db);
        }
        wave_sync();
        f32x16 cin;
        int pg[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 t4 = *(const f32x4 *)(s_tn + 8 * q + 4 * h);
          cin[4 * q] = t4.x;
          cin[4 * q + 1] = t4.y;
          cin[4 * q + 2] = t4.z;
          cin[4 * q + 3] = t4.w;
        }
        if (!uni) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int4 p4 = *(const int4 *)(s_hp + 8 * q + 4 * h);
            pg[4 * q] = p4.x;
            pg[4 * q + 1] = p4.y;
            pg[4 * q + 2] = p4.z;
            pg[4 * q + 3] = p4.w;
          }
        }
        const uint32_t om0 =
            fast_om ? (r == (p0 & 31) ? 1u << ((p0 >> 5) & 31) : 0u)
                    : s_om[r];
        auto push = [&](int row, float s, int j) {
          const int slot = atomicAdd(&s_cnt[row], 1);
          if (slot < B2_ENT)
            s_ent[row * B2_ENT + slot] = make_int2(__float_as_int(s), j);
        };
        // own block: pairs (row, p) with p != p_row; the column of a centre
        // hinted by several samples is tested once (dup)
        if (!uni) {
          float m = INFINITY;
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const float vg = pg[g] == p ? INFINITY : dn[g] + cin[g];
            m = fminf(m, vg);
          }
          if (pok && !dup && m <= ncp) {
#pragma unroll
            for (int g = 0; g < 16; ++g)
              if (pg[g] != p && dn[g] + cin[g] <= ncp) {
                const int row = (g & 3) + 8 * (g >> 2) + 4 * h;
                push(row, dn[g] - ncp, p);
              }
          }
        }
        // ---- centre blocks: lane = centre, registers = samples -----------
        auto rd_f = [&](int cb, bf16x8 (&f)[NKS]) {
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks)
            f[ks] = *(const bf16x8 *)(frag + ((int64_t)cb * NKS + ks) * 1024 +
                                      lane * 16);
        };
        // (this lane's norm column re-derived per tile: hoisted, it lived
        // across tiles and was the register the allocator spilled)
        const float *ncn_r = ncn + (int)opaque_u32((uint32_t)r);
        auto rd_n = [&](int cb) { return ncn_r[cb * 32]; };
        auto mm = [&](const bf16x8 (&f)[NKS], f32x16 &acc) {
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[0], f[0], cin, 0, 0,
                                                        0);
#pragma unroll
          for (int ks = 1; ks < NKS; ++ks)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh[ks], f[ks], acc, 0,
                                                          0, 0);
        };
        // whole-block test: the 16 rows' min against -|c_j|^2, or against a
        // NaN (never passes) where centre j is a hinted one (own block)
        auto test = [&](int cb, const f32x16 &acc, float nc, float &thr,
                        bool &any) {
          const uint32_t w = W1 ? om0 : s_om[(cb >> 5) * 32 + r];
          const int own = (int)(w << (31 - (cb & 31))) >> 31;
          thr = __uint_as_float(((uint32_t)own & 0xff800000u) |
                                __float_as_uint(nc));
          // 7 v_min3 + 1 v_min on the raw MFMA results (no NaN
          // canonicalisation: a NaN score comes with a NaN threshold, and
          // its sample is rejected by the `sane` test)
          any = min16(acc, ninf) <= thr;
          if (DKM_AB_B2_PROBE == 2) any = acc[0] == 12345.f;  // (invalid)
        };
        auto append = [&](int cb, const f32x16 &acc, float thr, float nc,
                          bool any) {
          if (any) {
            const int j = cb * 32 + r;
#pragma unroll
            for (int g = 0; g < 16; ++g)
              if (acc[g] <= thr) {
                const int row = (g & 3) + 8 * (g >> 2) + 4 * h;
                push(row, (acc[g] - cin[g]) - nc, j);
              }
          }
        };
        if (SORTED && DKM_AB_B2_PROBE != 1) {
          // the blocks of bmask (wave-uniform), in the dense loop's
          // software pipeline with c0..c3 = the next set bits in place of
          // cb .. cb + 3
          f32x16 acc_a, acc_b;
          bf16x8 fa[NKS], fb[NKS];
          float na, nb = 0.f, ta, tb;
          bool ga, gb;
          uint64_t m = bmask;
          auto pop = [&]() -> int {
            const int c = m ? __builtin_ctzll(m) : 0;
            m &= m - 1;
            return c;
          };
          int left = __popcll(bmask);
          t_blocks += (uint32_t)left;
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
              test(c0, acc_a, na, ta, ga);
              append(c0, acc_a, ta, na, ga);
              na = rd_n(c2);
              mm(fa, acc_a);  // chain c2
              rd_f(c3, fb);
              test(c1, acc_b, nb, tb, gb);
              append(c1, acc_b, tb, nb, gb);
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
              test(c0, acc_a, na, ta, ga);
              append(c0, acc_a, ta, na, ga);
              if (left > 2) {
                na = rd_n(c2);
                mm(fa, acc_a);  // chain c2
              }
              test(c1, acc_b, nb, tb, gb);
              append(c1, acc_b, tb, nb, gb);
              if (left > 2) {
                test(c2, acc_a, na, ta, ga);
                append(c2, acc_a, ta, na, ga);
              }
            } else {
              test(c0, acc_a, na, ta, ga);
              append(c0, acc_a, ta, na, ga);
            }
          }
        } else if (DKM_AB_B2_PROBE != 1) {
          // software pipeline, one block deep: block t's chain is issued
          // before block t - 1 is tested (the test VALU overlaps the MFMA
          // chain instead of waiting for its own block's results), and the
          // fragments of t + 1 are read while t's chain runs
          f32x16 acc_a, acc_b;
          bf16x8 fa[NKS], fb[NKS];
          float na, nb, ta, tb;
          bool ga, gb;
          rd_f(0, fa);
          na = rd_n(0);
          mm(fa, acc_a);  // chain 0
          if (nkb > 1) {
            rd_f(1, fb);
            nb = rd_n(1);
          }
          int cb = 0;
          // steady state: chains cb + 1, cb + 2 and reads cb + 2, cb + 3
          for (; cb + 3 < nkb; cb += 2) {
            mm(fb, acc_b);  // chain cb + 1
            rd_f(cb + 2, fa);
            test(cb, acc_a, na, ta, ga);
            append(cb, acc_a, ta, na, ga);
            na = rd_n(cb + 2);
            mm(fa, acc_a);  // chain cb + 2
            rd_f(cb + 3, fb);
            test(cb + 1, acc_b, nb, tb, gb);
            append(cb + 1, acc_b, tb, nb, gb);
            nb = rd_n(cb + 3);
          }
          // tail: 1, 2 or 3 blocks left (chain cb issued, reads cb + 1 done)
          if (cb + 1 < nkb) {
            mm(fb, acc_b);  // chain cb + 1
            if (cb + 2 < nkb) rd_f(cb + 2, fa);
            test(cb, acc_a, na, ta, ga);
            append(cb, acc_a, ta, na, ga);
            if (cb + 2 < nkb) {
              na = rd_n(cb + 2);
              mm(fa, acc_a);  // chain cb + 2
            }
            test(cb + 1, acc_b, nb, tb, gb);
            append(cb + 1, acc_b, tb, nb, gb);
            if (cb + 2 < nkb) {
              test(cb + 2, acc_a, na, ta, ga);
              append(cb + 2, acc_a, ta, na, ga);
            }
          } else {
            test(cb, acc_a, na, ta, ga);
            append(cb, acc_a, ta, na, ga);
          }
        }
        late_prefetch();
        // ---- decision over the hint and the kept entries ------------------
        wave_sync();
        const int cnt = s_cnt[r];
        // the hint as the scratch holds it: p when usable, else -1 (a row
        // without a usable hint is `over`, so nothing below needs its
        // incoming label); a uniform tile's is p0
        prv = uni ? p0 : s_hp[(int)opaque_u32((uint32_t)r)];
        const bool pokd = prv >= 0;
        const int pd = pokd ? prv : 0;
        // steady state: no row kept a centre besides its hint, and every row
        // is sane -- every label stays the hint: nothing to store or list
        {
          const float spq = s_sp[r];
          const bool quick = pokd && sane0 && spq + B2t < 1e30f && cnt == 0;
          if (__ballot(sid >= 0 && h == 0 && !quick) == 0) {
            ++t_tiles;
            ++t_done;
            return;
          }
        }
        float sv[B2_ENT + 1];
        int cv[B2_ENT + 1];
        bool ok[B2_ENT + 1];
        // s_hat_p and T again (the same fp32 operation: the same bits)
        const float sp2 = s_sp[r];
        const float T2 = pokd ? sp2 + B2t : -INFINITY;
        sv[0] = sp2;
        cv[0] = pd;
        ok[0] = true;
#pragma unroll
        for (int e = 0; e < B2_ENT; ++e) {
          const int2 en = s_ent[r * B2_ENT + e];
          sv[e + 1] = __int_as_float(en.x);
          cv[e + 1] = en.y;
          // (an index outside [0, k) never reaches the candidate kernels)
          ok[e + 1] = e < cnt && (unsigned)en.y < (unsigned)k;
        }
        const bool over = cnt > B2_ENT || !pokd || !sane0 || !(T2 < 1e30f);
        float bs = INFINITY;
        int bc = 0x7fffffff;
#pragma unroll
        for (int e = 0; e <= B2_ENT; ++e)
          if (ok[e] && (sv[e] < bs || (sv[e] == bs && cv[e] < bc))) {
            bs = sv[e];
            bc = cv[e];
          }
        int namb = 0, other = 0;
        uint32_t pk[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu};
#pragma unroll
        for (int e = 0; e <= B2_ENT; ++e)
          if (ok[e] && !(sv[e] - bs > B2t)) {
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
        const uint64_t mo = __ballot(over && sid >= 0 && h == 0);
        ++t_tiles;
        if (__popcll(mo) <= B2_RTHR) {
          ++t_done;
          need3 = false;
          unique = !over && namb == 1;
          two = !over && namb == 2;
          many = !over && namb >= 3;
          i1 = bc;
          i2 = other;
          mpk0 = pk[0];
          mpk1 = pk[1];
          mpk2 = pk[2];
        }
      }
    }
    if (need3) {
      late_prefetch();
      // ---- top-3 pass (no usable hint): b1's layout, centres on the rows --
      auto chain = [&](int cb, f32x16 &accv) {
        const f32x4 *c4p = (const f32x4 *)(cn + cb * 32 + 16 * h);
        const f32x4 c0 = c4p[0], c1 = c4p[1], c2 = c4p[2], c3 = c4p[3];
        accv = f32x16{c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                      c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8 ah =
              *(const bf16x8 *)(frag + ((int64_t)cb * NKS + ks) * 1024 +
                                lane * 16);
          accv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xh[ks], accv, 0,
                                                         0, 0);
        }
      };
      float r1 = INFINITY, r2 = INFINITY, r3 = INFINITY;
      int ii1 = 0, ii2 = 0, ii3 = 0;
      for (int g0 = 0; g0 < nkb; g0 += GB) {
        const int g1 = min(nkb, g0 + GB);
        float b1 = INFINITY, b2 = INFINITY, b3 = INFINITY;
        float e1 = INFINITY, e2 = INFINITY, e3 = INFINITY;
        auto score = [&](int cb, const f32x16 &accv) {
          const uint32_t t0 = opaque_s32((uint32_t)((cb - g0) * 16));
#pragma unroll
          for (int g = 0; g < 16; g += 2) {
            const float sa =
                __uint_as_float((__float_as_uint(accv[g]) & vmask) | (t0 + g));
            const float sb = __uint_as_float(
                (__float_as_uint(accv[g + 1]) & vmask) | (t0 + g + 1));
            b3 = __builtin_amdgcn_fmed3f(b2, b3, sa);
            b2 = __builtin_amdgcn_fmed3f(b1, b2, sa);
            b1 = min_nc(b1, sa, ninf);
            e3 = __builtin_amdgcn_fmed3f(e2, e3, sb);
            e2 = __builtin_amdgcn_fmed3f(e1, e2, sb);
            e1 = min_nc(e1, sb, ninf);
          }
        };
        f32x16 acc_a, acc_b;
        chain(g0, acc_a);
        int cb = g0;
        for (; cb + 2 <= g1; cb += 2) {
          chain(cb + 1, acc_b);
          score(cb, acc_a);
          if (cb + 2 < g1) chain(cb + 2, acc_a);
          score(cb + 1, acc_b);
        }
        if (cb < g1) score(cb, acc_a);
        auto gidx = [&](float q) {
          const uint32_t tg = __float_as_uint(q) & PACK2_MASK;
          const int g = (int)(tg & 15);
          return (g0 + (int)(tg >> 4)) * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
        };
        auto ins = [&](float q) {
          const int qi = gidx(q);
          const bool c1 = q < r1, c2 = q < r2, c3 = q < r3;
          r3 = c2 ? r2 : (c3 ? q : r3);
          ii3 = c2 ? ii2 : (c3 ? qi : ii3);
          r2 = c1 ? r1 : (c2 ? q : r2);
          ii2 = c1 ? ii1 : (c2 ? qi : ii2);
          r1 = c1 ? q : r1;
          ii1 = c1 ? qi : ii1;
        };
        ins(b1);
        ins(b2);
        ins(b3);
        ins(e1);
        ins(e2);
        ins(e3);
      }
      {  // merge the sample's two lanes (same triple on both)
        const float o1 = __shfl_xor(r1, 32, 64), o2 = __shfl_xor(r2, 32, 64),
                    o3 = __shfl_xor(r3, 32, 64);
        const int j1 = __shfl_xor(ii1, 32, 64), j2 = __shfl_xor(ii2, 32, 64),
                  j3 = __shfl_xor(ii3, 32, 64);
        auto lt = [](float a, int ia, float b, int ib) {
          return a < b || (a == b && ia < ib);
        };
        auto ins3 = [&](float q, int qi) {
          const bool c1 = lt(q, qi, r1, ii1), c2 = lt(q, qi, r2, ii2),
                     c3 = lt(q, qi, r3, ii3);
          r3 = c2 ? r2 : (c3 ? q : r3);
          ii3 = c2 ? ii2 : (c3 ? qi : ii3);
          r2 = c1 ? r1 : (c2 ? q : r2);
          ii2 = c1 ? ii1 : (c2 ? qi : ii2);
          r1 = c1 ? q : r1;
          ii1 = c1 ? qi : ii1;
        };
        ins3(o1, j1);
        ins3(o2, j2);
        ins3(o3, j3);
      }
      const bool sane = sane0 & (r1 < 1e30f);
      const float B2 = bound2_fast(bk, xx, xn);
      unique = sane & (r2 - r1 > B2);
      two = sane & !unique & (r3 - r1 > B2);
      i1 = ii1;
      i2 = ii2;
    }
    const bool valid = sid >= 0 && h == 0;
    // 3..6 candidates of the threshold pass -> the N-candidate list
    bool nlisted = false;
    {
      const uint64_t mn = __ballot(valid && many);
      const int addn = __popcll(mn);
      if (addn && listing && nl_cnt + addn <= B1_NCAP) {
        if (valid && many)
          nl[nl_cnt + lane_prefix(mn)] =
              make_int4((int)(sid - base), (int)mpk0, (int)mpk1, (int)mpk2);
        nl_cnt += addn;
        nlisted = many;
      }
    }
    // two candidates -> candidate list, more -> re-check list
    const uint64_t mc = __ballot(valid && two);
    const uint64_t mt = __ballot(valid && !unique && !two && !nlisted);
    const int addc = __popcll(mc), addt = __popcll(mt);
    if (listing && cl_cnt + addc <= B1_CAP) {
      if (valid && two)
        cl[cl_cnt + lane_prefix(mc)] =
            make_int2((int)(sid - base), i1 | (i2 << 16));
      cl_cnt += addc;
    } else {
      tl_over += addc;
    }
    if (listing && tl_cnt + addt <= TL_CAP) {
      if (valid && !unique && !two && !nlisted)
        wl[tl_cnt + lane_prefix(mt)] = make_int2((int)(sid - base), -1);
      tl_cnt += addt;
    } else {
      tl_over += addt;
    }
    // a label equal to the incoming one (the hint) needs no store; an
    // N-listed sample keeps it until k_candn writes the winner.  A sample
    // that overflowed a list keeps -1 (-(prev + 2), no previous label in
    // this labels-only pass): the label scan finds it.  SORTED: every row
    // whose label changes or goes to a re-check gets the marker
    // -(previous + 2) in the image's label copy; k_plab_sync fetches the
    // final label afterwards and, on the incremental path, lists the rows
    // that moved with their previous label.
    if (valid) {
      const bool same = unique && i1 == prv && (hint || SORTED);
      if (!nlisted && !same) lab_out[sid] = unique ? i1 : -1;
      // (a previous label outside [0, k) is marked as -1: -(prv + 2) of
      // such a label could fall on a label or past INT32_MIN)
      if (SORTED && !same)
        img.plab[s0 + r] = -(((unsigned)prv < (unsigned)k ? prv : -1) + 2);
    }
  };

  if constexpr (IMG != IMG_NONE) {
   if (tlst) {
    // ---- tile-list mode: the listed image tiles, appended to the lists
    // k_screen_sorted left (same segments)
    if (listing) {
      tl_cnt = v.tcount[wv];
      cl_cnt = v.ccount[wv];
      nl_cnt = v.ncount[wv];
    }
    const int64_t nls = *tlst_n;
    if (blockIdx.x == 0 && threadIdx.x == 0)
      atomicAdd((unsigned long long *)&v.hdr->sfall_total,
                (unsigned long long)nls);
    for (int64_t i = wv; i < nls; i += (int64_t)gridDim.x * NW) {
      const int64_t s0 = (int64_t)tlst[i] * 32;
      load_img(s0, xq, xxq, pq, sq);
      bf16x8 xh[NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) xh[ks] = xq[ks];
      process(s0, xh, xxq, pq, sq);
    }
   } else {
    // ---- sample image: the next tile's loads are in flight while this one
    // is screened (LATEPF: issued from process() after the block loop)
    int64_t s0 = base + wv * 32;
    if (s0 < n) load_img(s0, xq, xxq, pq, sq);
    for (; s0 < n; s0 += step) {
      bf16x8 xh[NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) xh[ks] = xq[ks];
      const float xx = xxq;
      const int prv = pq, sid = sq;
      if (LATEPF) {
        pf_s0 = s0 + step;
        pf_done = false;
      } else if (s0 + step < n) {
        load_img(s0 + step, xq, xxq, pq, sq);
      }
      process(s0, xh, xx, prv, sid);
      late_prefetch();
    }
   }
  } else {
  for (int64_t s0 = base + wv * 32; s0 < n; s0 += step) {
    load_tile(s0);
    bf16x8 xh[NKS];
    float xp[IC];  // |x|^2 partials of rows RI i + lrow
#pragma unroll
    for (int i = 0; i < IC; ++i) xp[i] = 0.f;
    // features past d (d % 16 != 0): lim recomputed per tile (opaque), or
    // the lane masks are hoisted into long-lived SGPR pairs
    const int lim = d == 16 * NKS ? 0x7fffffff
                                  : (int)opaque_u32((uint32_t)(d - EPL * lpos));
    wave_sync();  // the previous tile's kept entries were read
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
      for (int i = 0; i < IC; ++i) {
        float xf[EPL];
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const float x = (float)raw[ks][i][e];
          xf[e] = 16 * ks + e < lim ? x : 0.f;
          xp[i] = fmaf(xf[e], xf[e], xp[i]);
        }
        if constexpr (EPL == 2) {
          const bf16x2 b2 = __builtin_convertvector(f32x2{xf[0], xf[1]}, bf16x2);
          *(bf16x2 *)(s_tx + wofs_at(i)) = b2;
        } else {
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          const bf16x2 a2 = __builtin_convertvector(f32x2{xf[0], xf[1]}, bf16x2);
          const bf16x2 b2 = __builtin_convertvector(f32x2{xf[2], xf[3]}, bf16x2);
          *(bf16x4 *)(s_tx + wofs_at(i)) = bf16x4{a2[0], a2[1], b2[0], b2[1]};
        }
      }
      wave_sync();
      xh[ks] = *(const bf16x8 *)(s_tx + tx_addr(r, h));
      wave_sync();
    }
    // |x|^2: the LR lanes of a row line hold its partials
#pragma unroll
    for (int i = 0; i < IC; ++i) {
#pragma unroll
      for (int m = 1; m < LR; m <<= 1) xp[i] += __shfl_xor(xp[i], m, 64);
      if (lpos == 0) s_xx[RI * i + lrow] = xp[i];
    }
    wave_sync();
    const float xx = s_xx[r];
    process(s0, xh, xx, pv, s0 + r < n ? (int)(s0 + r) : -1);
  }
  }  // IMG_NONE
  if (!tlst && wv == 0 && lane == 0)
    v.hdr->lseg = (int32_t)std::min<int64_t>((int64_t)gridDim.x * NW,
                                             std::min(TL_SEGS, B1_SEGS));
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
    if (SORTED)
      atomicAdd((unsigned long long *)&v.hdr->reserved[2],
                (unsigned long long)t_blocks);
  }
  if (lane == 0 && tl_over) atomicAdd(&v.hdr->qcount, (uint32_t)tl_over);
}

size_t b2_lds_bytes(int64_t k, int64_t d) {
  const int64_t nkb = kpad32(k) / 32, nkw = (nkb + 31) / 32;
  return (size_t)nkb * (dpad16(d) / 16) * 1024 + (size_t)nkb * 256 +
         (size_t)(SB2 / 64) * (B2_SCR_FIXED + 128 * nkw);
}

// A/B timing probe builds (variants_b2.sh) report themselves
int b2_probe() { return DKM_AB_B2_PROBE; }

// ---- the sample image (dkm_x_image_*) ----------------------------------
static int64_t img_tile_bytes(int64_t d, int kind) {
  return kind == IMG_SPLIT ? 4096 : (dpad16(d) / 16) * 1024;
}

size_t x_image_bytes(int64_t n, int64_t d, int kind) {
  if (kind == IMG_GEMM) {
    const int64_t ntg = (n + GT - 1) / GT;
    return (size_t)ntg * (dpad32(d) / GBK) * GSTAGE1 + (size_t)ntg * GT * 4;
  }
  const int64_t nt = (n + 31) / 32;
  return (size_t)nt * img_tile_bytes(d, kind) + (size_t)nt * 128 +
         (kind == IMG_SORTED ? (size_t)nt * 256 : 0);
}

XImage x_image_view(const void *image, int64_t n, int64_t d, int kind) {
  const int64_t nt = (n + 31) / 32;
  XImage im;
  if (kind == IMG_GEMM) {
    const int64_t ntg = (n + GT - 1) / GT;
    im.tiles = (const uint16_t *)image;
    im.xx = (const float *)((const char *)image +
                            (size_t)ntg * (dpad32(d) / GBK) * GSTAGE1);
    im.kind = kind;
    im.perm = nullptr;
    im.plab = nullptr;
    return im;
  }
  im.tiles = (const uint16_t *)image;
  im.xx = (const float *)((const char *)image +
                          (size_t)nt * img_tile_bytes(d, kind));
  im.kind = kind;
  im.perm = nullptr;
  im.plab = nullptr;
  if (kind == IMG_SORTED) {
    im.perm = (const int32_t *)(im.xx + nt * 32);
    im.plab = (int32_t *)(im.perm + nt * 32);
  }
  return im;
}

// One workgroup per 32-row tile (grid-stride): the tile's rows are read
// with consecutive lanes on consecutive features (whole lines), staged as
// fp32 in LDS, then written in operand order with the same fp64 -> fp32 ->
// bf16 roundings the converting screens apply.  |x|^2 is summed in fp64
// over the fp32 values and rounded once.  perm != nullptr (IMG_SORTED):
// image row i holds sample perm[i] (-1: a zero row past the data).
template <class TX, int NKS>
__global__ void __launch_bounds__(256)
    k_x_image(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
              const int32_t *__restrict__ perm, uint16_t *__restrict__ tiles,
              float *__restrict__ xx) {
  constexpr int DP = 16 * NKS, LD = DP + 4;
  __shared__ float s[32 * LD];
  __shared__ int64_t srow[32];
  const int64_t nt = (n + 31) / 32;
  for (int64_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int64_t r0 = t * 32;
    __syncthreads();  // the previous tile's reads are done
    if (threadIdx.x < 32) {
      const int64_t i = r0 + threadIdx.x;
      srow[threadIdx.x] = perm ? (int64_t)perm[i] : (i < n ? i : -1);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 32 * DP; e += 256) {
      const int row = e / DP, col = e % DP;
      const int64_t src = srow[row];
      float v = 0.f;
      if (src >= 0 && col < d) v = (float)X[src * ldx + col];
      s[row * LD + col] = v;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
      double a = 0.0;
      for (int c = 0; c < DP; ++c) {
        const double v = s[threadIdx.x * LD + c];
        a = fma(v, v, a);
      }
      xx[r0 + threadIdx.x] = (float)a;
    }
    for (int e = threadIdx.x; e < NKS * 64; e += 256) {
      const int ks = e >> 6, l = e & 63;
      const float *src = s + (l & 31) * LD + 16 * ks + 8 * (l >> 5);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const bf16x2 b = __builtin_convertvector(f32x2{src[j], src[j + 1]},
                                                 bf16x2);
        o[j] = b[0];
        o[j + 1] = b[1];
      }
      *((bf16x8 *)(tiles + t * (NKS * 512)) + e) = o;
    }
  }
}

// IMG_SPLIT (d <= 32): hi and lo parts in k_screen_w32's B-operand order
template <class TX>
__global__ void __launch_bounds__(256)
    k_x_image_split(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                    uint16_t *__restrict__ tiles, float *__restrict__ xx) {
  constexpr int LD = 33;
  __shared__ float s[32 * LD];
  const int64_t nt = (n + 31) / 32;
  for (int64_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int64_t r0 = t * 32;
    __syncthreads();
    for (int e = threadIdx.x; e < 32 * 32; e += 256) {
      const int row = e >> 5, col = e & 31;
      float v = 0.f;
      if (r0 + row < n && col < d) v = (float)X[(r0 + row) * ldx + col];
      s[row * LD + col] = v;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
      double a = 0.0;
      for (int c = 0; c < 32; ++c) {
        const double v = s[threadIdx.x * LD + c];
        a = fma(v, v, a);
      }
      xx[r0 + threadIdx.x] = (float)a;
    }
    {
      const int e = threadIdx.x;  // 256 = 4 blocks x 64 lanes
      const int blk = e >> 6, l = e & 63, ks = blk & 1, lo = blk >> 1;
      const float *src = s + (l & 31) * LD + 16 * (l >> 5) + 8 * ks;
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const bf16x2 h2 = __builtin_convertvector(f32x2{src[j], src[j + 1]},
                                                  bf16x2);
        const uint32_t hu = __builtin_bit_cast(uint32_t, h2);
        const bf16x2 l2 = __builtin_convertvector(
            f32x2{src[j] - __uint_as_float(hu << 16),
                  src[j + 1] - __uint_as_float(hu & 0xffff0000u)},
            bf16x2);
        o[j] = lo ? l2[0] : h2[0];
        o[j + 1] = lo ? l2[1] : h2[1];
      }
      *((bf16x8 *)(tiles + t * 2048) + e) = o;
    }
  }
}

template <class TX>
static int launch_image_tiles(const TX *X, int64_t n, int d, int64_t ldx,
                              const int32_t *perm, const XImage &im, int cus,
                              hipStream_t s) {
  const int64_t nt = (n + 31) / 32;
  const unsigned g =
      (unsigned)std::max<int64_t>(1, std::min<int64_t>(nt, (int64_t)cus * 8));
  uint16_t *tiles = (uint16_t *)im.tiles;
  float *xx = (float *)im.xx;
  switch ((int)(dpad16(d) / 16)) {
#define DKM_XI(N)                                                         \
  case N:                                                                 \
    k_x_image<TX, N><<<g, 256, 0, s>>>(X, n, d, ldx, perm, tiles, xx);    \
    break;
    DKM_XI(1) DKM_XI(2) DKM_XI(3) DKM_XI(4)
    DKM_XI(5) DKM_XI(6) DKM_XI(7) DKM_XI(8)
#undef DKM_XI
    default:
      return fail(DKM_E_ARG, "x_image: d > 128");
  }
  return check_launch("sample image");
}

// The label-sorted image AND the full sums in one pass over X (the fit's
// first sorted iteration would otherwise read X once for the sums and once
// for the image).  Block b takes a contiguous range of 32-row tiles of the
// sorted order; a tile's rows are staged in LDS as fp64: the image tile and
// |x|^2 come from them exactly as k_x_image writes them, and the sums from
// the fp64 values, one running sum per (row group, feature) of the current
// cluster (positions < m are labelled and ascending by label), added to acc
// with fp64 atomics when the cluster changes and at the end of the range.
template <class TX, int NKS>
__global__ void __launch_bounds__(256)
    k_x_image_sums(const TX *__restrict__ X, int64_t n, int d, int64_t ldx,
                   const int32_t *__restrict__ perm,
                   const int32_t *__restrict__ off, int k,
                   uint16_t *__restrict__ tiles, float *__restrict__ xx,
                   double *__restrict__ acc) {
  constexpr int DP = 16 * NKS, LD = DP + 1, RG = 256 / DP;
  static_assert(256 % DP == 0, "DP divides the block");
  __shared__ double s[32 * LD];
  __shared__ int64_t srow[32];
  const int64_t nt = (n + 31) / 32;
  const int64_t per = (nt + gridDim.x - 1) / gridDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * per;
  const int64_t t1 = t0 + per < nt ? t0 + per : nt;
  if (t0 >= t1) return;
  const int64_t m = off[k];  // labelled positions
  const int f = threadIdx.x % DP, g = threadIdx.x / DP;
  // the cluster of the range's first position: largest c, off[c] <= p
  int c = 0;
  {
    const int64_t p0 = t0 * 32;
    int lo = 0, hi = k;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (off[mid] <= p0) lo = mid;
      else hi = mid;
    }
    c = lo;
  }
  int64_t nxt = off[c + 1];
  double a = 0.0;
  int cnt = 0;
  auto flush = [&]() {
    if (cnt) {
      if (f < d) atomic_add_f64(acc + (int64_t)c * d + f, a);
      if (f == 0) atomic_add_f64(acc + (int64_t)k * d + c, (double)cnt);
    }
    a = 0.0;
    cnt = 0;
  };
  // the next tile's row indices are loaded while this tile is processed
  // (a perm load, then the dependent row loads, cost two round trips a
  // tile: 17.5 -> 16.0 ms at C3; the next tile's rows in registers as well,
  // a two-stage pipeline, measured 17.4)
  int32_t pnext = threadIdx.x < 32 ? perm[t0 * 32 + threadIdx.x] : 0;
  for (int64_t t = t0; t < t1; ++t) {
    const int64_t r0 = t * 32;
    __syncthreads();  // the previous tile's reads are done
    if (threadIdx.x < 32) srow[threadIdx.x] = (int64_t)pnext;
    __syncthreads();
    double xv[32 * DP / 256];
#pragma unroll
    for (int u = 0; u < 32 * DP / 256; ++u) {
      const int e = threadIdx.x + 256 * u;
      const int row = e / DP, col = e % DP;
      const int64_t src = srow[row];
      xv[u] = src >= 0 && col < d ? (double)X[src * ldx + col] : 0.0;
    }
    if (threadIdx.x < 32 && t + 1 < t1) pnext = perm[r0 + 32 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < 32 * DP / 256; ++u) {
      const int e = threadIdx.x + 256 * u;
      s[(e / DP) * LD + e % DP] = xv[u];
    }
    __syncthreads();
    if (threadIdx.x < 32) {  // |x|^2 as k_x_image: fp64 fma of the fp32s
      double q = 0.0;
      for (int col = 0; col < DP; ++col) {
        const double v = (double)(float)s[threadIdx.x * LD + col];
        q = fma(v, v, q);
      }
      xx[r0 + threadIdx.x] = (float)q;
    }
    for (int e = threadIdx.x; e < NKS * 64; e += 256) {
      const int ks = e >> 6, l = e & 63;
      const double *src = s + (l & 31) * LD + 16 * ks + 8 * (l >> 5);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const bf16x2 b = __builtin_convertvector(
            f32x2{(float)src[j], (float)src[j + 1]}, bf16x2);
        o[j] = b[0];
        o[j + 1] = b[1];
      }
      *((bf16x8 *)(tiles + t * (NKS * 512)) + e) = o;
    }
    // sums: row group g takes rows g, g + RG, ... of the tile
    for (int r = g; r < 32; r += RG) {
      const int64_t p = r0 + r;
      if (p >= m) break;  // unlabelled / padding rows: no sums
      if (p >= nxt) {
        flush();
        while (off[c + 1] <= p) ++c;
        nxt = off[c + 1];
      }
      a += s[r * LD + f];
      ++cnt;
    }
  }
  flush();
}

template <class TX>
int launch_x_image(const TX *X, int64_t n, int d, int64_t ldx, int kind,
                   void *image, int cus, hipStream_t s) {
  const XImage im = x_image_view(image, n, d, kind);
  if (kind == IMG_SPLIT) {
    if (d > 32) return fail(DKM_E_ARG, "x_image: split image needs d <= 32");
    const int64_t nt = (n + 31) / 32;
    const unsigned g = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>(nt, (int64_t)cus * 8));
    k_x_image_split<TX><<<g, 256, 0, s>>>(X, n, d, ldx, (uint16_t *)image,
                                          (float *)im.xx);
    return check_launch("sample image (split)");
  }
  if (kind != IMG_SINGLE) return fail(DKM_E_ARG, "x_image: bad kind");
  return launch_image_tiles<TX>(X, n, d, ldx, nullptr, im, cus, s);
}

template int launch_x_image<double>(const double *, int64_t, int, int64_t,
                                    int, void *, int, hipStream_t);
template int launch_x_image<float>(const float *, int64_t, int, int64_t, int,
                                   void *, int, hipStream_t);

// ---- IMG_SORTED: the image with its rows grouped by label ----------------
// perm[i] for i in [0, ntot): the sorted indices (labels in [0, k)), then
// the samples whose label is outside [0, k) (appended by
// k_perm_unlabelled), then -1 for the padding rows past n.
__global__ void k_perm_sorted(const int32_t *__restrict__ sitems,
                              const int32_t *__restrict__ nsorted, int64_t n,
                              int64_t ntot, int32_t *__restrict__ perm) {
  const int64_t m = *nsorted;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < ntot;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < m) perm[i] = sitems[i];
    else if (i >= n) perm[i] = -1;
  }
}

// The image's initial label copy straight from the sort's cluster offsets:
// row i of the label-sorted image carries cluster c for soff[c] <= i <
// soff[c + 1], and -1 past soff[k] (unlabelled rows, padding) -- what k_plab's
// full pass (plab[i] = lab[perm[i]], a random 4-B gather per row: 3 ms at
// C3) computes, from a binary search per 4 rows and coalesced stores.
__global__ void k_plab_offsets(const int32_t *__restrict__ soff, int k,
                               int64_t ntot, int32_t *__restrict__ plab) {
  const int64_t m = soff[k];
  for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 4;
       i < ntot; i += (int64_t)gridDim.x * blockDim.x * 4) {
    int lo = 0, hi = k;  // soff[lo] <= i < soff[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (soff[mid] <= i) lo = mid;
      else hi = mid;
    }
    int32_t o[4];
    int c = lo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t r = i + e;
      while (c < k && soff[c + 1] <= r) ++c;  // empty clusters
      o[e] = r < m ? c : -1;
    }
    *(int4 *)(plab + i) = make_int4(o[0], o[1], o[2], o[3]);
  }
}

__global__ void k_perm_unlabelled(const int32_t *__restrict__ lab, int64_t n,
                                  int k, const int32_t *__restrict__ nsorted,
                                  unsigned long long *count,
                                  int32_t *__restrict__ perm) {
  const int lane = threadIdx.x & 63;
  const int64_t m = *nsorted;
  for (int64_t i0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) & ~63ll;
       i0 < n; i0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = i0 + lane;
    const bool un = i < n && (unsigned)lab[i] >= (unsigned)k;
    const uint64_t b = __ballot(un);
    if (!b) continue;
    unsigned long long at = 0;
    if (lane == 0) at = atomicAdd(count, (unsigned long long)__popcll(b));
    at = __shfl(at, 0, 64);
    if (un) perm[m + (int64_t)at + lane_prefix(b)] = (int32_t)i;
  }
}

// plab[i] = lab[perm[i]] (init), or only where plab[i] < 0 (sync: the rows
// the screen marked -(previous + 2)).  moved != NULL (incremental sums):
// a synced row whose label differs from its previous one is listed in
// moved[] (order free; *nmoved counts) and prevs[sample] = previous label.
// Each lane takes 4 consecutive rows with one 16-B load of plab (4-B loads
// kept too few bytes in flight: 0.41 ms per C3 sync, 1.2 TB/s).
__global__ void __launch_bounds__(256)
    k_plab(const int32_t *__restrict__ perm, const int32_t *__restrict__ lab,
           int64_t ntot, int k, int32_t *__restrict__ plab, int only_marked,
           int32_t *__restrict__ moved, int32_t *nmoved,
           int32_t *__restrict__ prevs) {
  // moved rows are staged per wave in LDS and reserved with one global
  // atomic per PLAB_BUF entries (the rows are spread over every wave: an
  // atomic per wave and step serialised on *nmoved)
  constexpr int PLAB_BUF = 512;
  __shared__ int32_t buf[4][PLAB_BUF];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t *wb = buf[w];
  int cnt = 0;  // wave-uniform
  auto flush = [&]() {
    int at = 0;
    if (lane == 0) at = atomicAdd(nmoved, cnt);
    at = __shfl(at, 0, 64);
    for (int e = lane; e < cnt; e += 64) moved[at + e] = wb[e];
    wave_sync();
    cnt = 0;
  };
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  // whole waves walk the range together (the ballots below); ntot is a
  // multiple of 32, so a lane's 4 rows are all in range or all out
  for (int64_t i0 = ((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) & ~63ll) * 4;
       i0 < ntot; i0 += stride) {
    const int64_t i = i0 + 4 * lane;
    int4 cur4 = make_int4(0, 0, 0, 0);
    if (i < ntot) cur4 = *(const int4 *)(plab + i);
    const int32_t cv[4] = {cur4.x, cur4.y, cur4.z, cur4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bool mv = false;
      int32_t p = -1, old = 0;
      if (i < ntot && (!only_marked || cv[e] < 0)) {
        p = perm[i + e];
        const int32_t nw = p >= 0 ? lab[p] : -1;
        // a label outside [0, k) is kept as -1: a negative copy is read as
        // the marker -(previous + 2), and -1 means "no previous label"
        plab[i + e] = (unsigned)nw < (unsigned)k ? nw : -1;
        old = -(cv[e] + 2);
        mv = moved && only_marked && p >= 0 && nw != old;
      }
      if (!moved) continue;  // kernel-uniform
      const uint64_t b = __ballot(mv);
      if (!b) continue;
      const int c = __popcll(b);
      if (cnt + c > PLAB_BUF) flush();
      if (mv) {
        wb[cnt + lane_prefix(b)] = p;
        prevs[p] = old;
      }
      wave_sync();
      cnt += c;
    }
  }
  if (moved && cnt) flush();
}

static unsigned flat_grid(int64_t n, int cus) {
  return (unsigned)std::max<int64_t>(
      1, std::min<int64_t>((n + 255) / 256, (int64_t)cus * 16));
}

template <class TX>
int launch_x_image_sorted(const TX *X, int64_t n, int d, int64_t ldx,
                          const int32_t *labels, int k, const WsView &v,
                          void *image, int cus, hipStream_t s, double *acc) {
  const XImage im = x_image_view(image, n, d, IMG_SORTED);
  const int64_t ntot = (n + 31) / 32 * 32;
  int32_t *perm = (int32_t *)im.perm;
  if (int r = sort_by_label(labels, 0, n, k, v, s)) return r;
  unsigned long long *cnt = (unsigned long long *)&v.hdr->reserved[3];
  if (hipMemsetAsync(cnt, 0, 8, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "sorted image: memset");
  const unsigned g = flat_grid(ntot, cus);
  k_perm_sorted<<<g, 256, 0, s>>>(v.sitems, v.soff + k, n, ntot, perm);
  k_perm_unlabelled<<<g, 256, 0, s>>>(labels, n, k, v.soff + k, cnt, perm);
  k_plab_offsets<<<flat_grid((ntot + 3) / 4, cus), 256, 0, s>>>(
      v.soff, k, ntot, im.plab);
  if (int r = check_launch("sorted image: permutation")) return r;
  if (!acc) return launch_image_tiles<TX>(X, n, d, ldx, perm, im, cus, s);
  const int64_t nt = (n + 31) / 32;
  const unsigned gs =
      (unsigned)std::max<int64_t>(1, std::min<int64_t>(nt, (int64_t)cus * 8));
  uint16_t *tiles = (uint16_t *)im.tiles;
  float *xx = (float *)im.xx;
  switch ((int)(dpad16(d) / 16)) {
#define DKM_XS(N)                                                           \
  case N:                                                                   \
    k_x_image_sums<TX, N><<<gs, 256, 0, s>>>(X, n, d, ldx, perm, v.soff, k, \
                                             tiles, xx, acc);               \
    break;
    DKM_XS(1) DKM_XS(2) DKM_XS(4) DKM_XS(8)
#undef DKM_XS
    default:  // the caller checks x_image_sums_fused(d)
      return fail(DKM_E_ARG, "sorted image + sums: dpad16(d) / 16 not 1, 2, "
                             "4 or 8");
  }
  return check_launch("sorted image + sums");
}

template int launch_x_image_sorted<double>(const double *, int64_t, int,
                                           int64_t, const int32_t *, int,
                                           const WsView &, void *, int,
                                           hipStream_t, double *);
template int launch_x_image_sorted<float>(const float *, int64_t, int,
                                          int64_t, const int32_t *, int,
                                          const WsView &, void *, int,
                                          hipStream_t, double *);

int launch_plab_sync(const XImage &img, int64_t n, int k, const int32_t *lab,
                     int cus, hipStream_t s, int32_t *moved, int32_t *nmoved,
                     int32_t *prevs) {
  if (img.kind != IMG_SORTED) return 0;
  const int64_t ntot = (n + 31) / 32 * 32;
  if (moved && hipMemsetAsync(nmoved, 0, 4, s) != hipSuccess)
    return fail(DKM_E_LAUNCH, "sorted image: memset");
  k_plab<<<flat_grid((ntot + 3) / 4, cus), 256, 0, s>>>(img.perm, lab, ntot, k,
                                              img.plab, 1, moved, nmoved,
                                              prevs);
  return check_launch("sorted image: label sync");
}

template <class TX>
int launch_screen_b2(const TX *X, int64_t end, int d, int64_t ldx, int k,
                     const WsView &v, int32_t *lab_out, int64_t base, int hint,
                     int cus, hipStream_t s, int *nseg, XImage img,
                     bool transl) {
  const size_t lds = b2_lds_bytes(k, d);
  if (lds > 160 * 1024) return 1;  // caller uses k_screen_b1
  // the image paths read whole tiles: the range must start on one (the
  // sorted image covers the whole range: its rows are not sample rows)
  int ik = img.tiles ? img.kind : IMG_NONE;
  if (ik == IMG_SORTED && base != 0)
    return fail(DKM_E_ARG, "screen_b2: the sorted image needs the whole range");
  if (ik == IMG_SORTED && transl)
    return fail(DKM_E_ARG, "screen_b2: no translation over the sorted image");
  if (transl && !v.b1frag_t) transl = false;
  if (ik == IMG_SINGLE && base % 32 != 0) ik = IMG_NONE;
  if (ik != IMG_SINGLE && ik != IMG_SORTED) ik = IMG_NONE;
  // the steady state over the sorted image: k_screen_sorted, then this
  // kernel over the tiles it listed (the fit's moved-list scratch holds the
  // list: it is filled only after the screen, by the label sync)
  const int32_t *tlst = nullptr;
  const uint32_t *tlst_n = nullptr;
  if (ik == IMG_SORTED && hint == 1 && !DKM_AB_NO_SORTED_FAST) {
    const int r = launch_screen_sorted(end, d, k, v, lab_out, img, cus, s,
                                       nseg, v.smoved, &v.hdr->sfall);
    if (r > 1 || r < 0) return r;
    if (r == 0) {
      tlst = v.smoved;
      tlst_n = &v.hdr->sfall;
    }
  }
  const int nks = (int)(dpad16(d) / 16);
  const bool w1 = kpad32(k) <= 1024;
  const void *kf = nullptr;
#define DKM_B2K(N, W, I) (const void *)k_screen_b2<TX, N, W, I>
#define DKM_B2W(N, I) (w1 ? DKM_B2K(N, true, I) : DKM_B2K(N, false, I))
  switch (nks) {
#define DKM_B2(N)                                                          \
  case N:                                                                  \
    kf = ik == IMG_SORTED   ? DKM_B2W(N, IMG_SORTED)                       \
         : ik == IMG_SINGLE ? DKM_B2W(N, IMG_SINGLE)                       \
                            : DKM_B2W(N, IMG_NONE);                        \
    break;
    DKM_B2(1) DKM_B2(2) DKM_B2(3) DKM_B2(4)
    DKM_B2(5) DKM_B2(6) DKM_B2(7) DKM_B2(8)
#undef DKM_B2
    default:
      return fail(DKM_E_ARG, "screen_b2: d too large");
  }
#undef DKM_B2W
#undef DKM_B2K
  if (hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return fail(DKM_E_LAUNCH, "screen_b2: LDS attribute");
  const int nw = SB2 / 64;  // screening waves
  unsigned g;
  if (tlst) {
    // tile-list mode: the waves append to k_screen_sorted's list segments
    // (no more waves than it had)
    g = (unsigned)std::max(1, *nseg / nw);
  } else {
    const int64_t need = (end - base + 32 * nw - 1) / (32 * nw);
    g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(need, (int64_t)cus));
    *nseg =
        (int)std::min<int64_t>((int64_t)g * nw, std::min(TL_SEGS, B1_SEGS));
  }
  const B2View bv = b2_view(v, ik == IMG_SORTED, transl);
  hipLaunchKernelGGL((void (*)(const TX *, int64_t, int, int64_t, int, B2View,
                               int32_t *, int64_t, int, XImage,
                               const int32_t *, const uint32_t *))kf,
                     dim3(g), dim3(SB2), lds, s, X, end, d, ldx, k, bv,
                     lab_out, base, hint, img, tlst, tlst_n);
  return check_launch("screen assignment (single product, centres on lanes)");
}

template int launch_screen_b2<double>(const double *, int64_t, int, int64_t,
                                      int, const WsView &, int32_t *, int64_t,
                                      int, int, hipStream_t, int *, XImage,
                                      bool);
template int launch_screen_b2<float>(const float *, int64_t, int, int64_t, int,
                                     const WsView &, int32_t *, int64_t, int,
                                     int, hipStream_t, int *, XImage, bool);

}  // namespace dkm

// Code-object preload (dkm_preload): the runtime loads this file's kernels
// on first use of any of them; an attribute query here does it up front.
namespace dkm {
DKM_TU_FLAGS(b2, DKM_AB_B2_PROBE)
__global__ void k_tu_b2() {}
int preload_b2() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void *)k_tu_b2) == hipSuccess ? 0
                                                                       : 1;
}
}  // namespace dkm
