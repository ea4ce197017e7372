// dkm_internal.h -- shared device helpers for libdkm (gfx950 / CDNA4 only).
//
// Compiled with -ffp-contract=off: the exact-arithmetic paths below must
// round every product and sum separately, exactly like numpy on the host.
// Where a fused multiply-add is wanted it is written explicitly (fma/fmaf).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/dkm.h"

namespace dkm {

constexpr int WAVE = 64;

// ---------------------------------------------------------------------------
// Error plumbing: a thread-local message, int return codes, no exceptions.
// ---------------------------------------------------------------------------
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
// Per-file code-object preload (each .hip file's kernels load on first use).
int preload_dense();
int preload_b2();
int preload_sorted();
int preload_cand();
int preload_sparse();
int preload_gemm();
int preload_sums();
int preload_neighbors();
int check_launch(const char *what);
// Build flags per translation unit (dkm_build_flags ORs them):
// DKM_BUILD_AB_VARIANT when the file was compiled as an A/B variant
// (variants.sh / variants_b2.sh define DKM_AB_VARIANT=1 on every object
// they compile with knobs), DKM_BUILD_TIMING_ONLY when one of the file's
// result-invalidating probe knobs is set.
#ifndef DKM_AB_VARIANT
#define DKM_AB_VARIANT 0
#endif
#define DKM_TU_FLAGS(name, probe)                                  \
  int tu_flags_##name() {                                          \
    return (DKM_AB_VARIANT ? DKM_BUILD_AB_VARIANT : 0) |           \
           ((probe) ? DKM_BUILD_TIMING_ONLY : 0);                  \
  }
int tu_flags_util();
int tu_flags_dense();
int tu_flags_b2();
int tu_flags_sorted();
int tu_flags_cand();
int tu_flags_sparse();
int tu_flags_gemm();
int tu_flags_sums();
int tu_flags_neighbors();

// ---------------------------------------------------------------------------
// Workspace layout (caller-allocated device memory, carved here).
// ---------------------------------------------------------------------------
struct WsHeader {
  uint64_t magic;
  int64_t k, d, dpad, n_queue;
  uint64_t cmax_bits;       // max_c ||c||_2 as ordered bits (non-negative)
  uint32_t qcount;          // samples queued for exact re-check this call
  uint32_t s2count;         // k_recheck_list's stage-2 samples (global list)
  uint64_t rechecked_total; // diagnostics
  uint32_t gcount;          // GEMM screen: candidate-list entries (per chunk)
  uint32_t gcount2;         // GEMM screen: full-scan entries (per chunk)
  int32_t nmoved;           // sorted sums: samples whose label changed
  uint32_t rtotal;          // re-screen: entries of the screen's re-check list
  uint32_t csr_nund;        // CSR screen: undecided samples of this chunk
  uint32_t pad2;
  uint64_t reserved[5];
  // k_screen_sorted: tiles handed to k_screen_b2 this call / in all calls
  uint32_t sfall;
  uint32_t qhead;  // k_screen_sorted: next chunk of image tiles (zeroed
                   // with sfall before each launch)
  int32_t lseg;    // list segments of the last single-product screen launch
  int32_t pad3;
  uint64_t sfall_total;
  uint64_t umax_bits;  // max_c ||c - m||_2 (m: b1frag_t's translation)
};
constexpr uint64_t WS_MAGIC = 0x444b4d5753303035ull;  // "DKMWS005"
constexpr size_t WS_HDR = 256;
static_assert(sizeof(WsHeader) <= WS_HDR, "the header fits WS_HDR");

__host__ __device__ inline int64_t round_up(int64_t a, int64_t b) {
  return (a + b - 1) / b * b;
}

// ---------------------------------------------------------------------------
// Large-d GEMM screen (dkm_gemm.hip, d > 128): tiles of GT rows x GBK
// features, bf16 hi/lo split, 128-B rows with XOR-swizzled 16-B chunks.
// ---------------------------------------------------------------------------
constexpr int GT = 256;                 // rows per tile (centres or samples)
constexpr int GBK = 32;                 // features per K-stage
constexpr int GSTAGE = GT * GBK * 4;    // bytes per operand tile per stage
// single-product (hi only) tiles: 32-feature stages of 64-B rows
constexpr int GSTAGE1 = GT * GBK * 2;
constexpr int GTOP = 4;                 // (score, centre) pairs kept per sample

__host__ __device__ inline int64_t kpad256(int64_t k) { return (k + 255) / 256 * 256; }

// Row stride (elements) of the transposed centres C^T (d x ct_ld(k)): 128-B
// aligned rows, so the CSR kernels' 32-centre slices are whole lines and
// their 16-B loads aligned.  Padding columns are never read into a result.
__host__ __device__ inline int64_t ct_ld(int64_t k) { return (k + 15) / 16 * 16; }

// ---------------------------------------------------------------------------
// Single-product screen (k_screen_b1, dkm_dense.hip): bf16 hi of x and -2c
// on v_mfma_f32_32x32x16_bf16, every centre resident in LDS (32-centre
// blocks x 16-feature K-steps, 1 KB each), a packed top-3 per sample; two
// candidates within the bound go to a per-wave candidate list (B1_CAP
// entries of (offset, c1 | c2 << 16)), three or more to the re-check lists.
// ---------------------------------------------------------------------------
constexpr int B1_SEGS = 4096;          // >= 256 CUs x 8 waves
constexpr int B1_CAP = 8192;           // candidate entries per screen wave
constexpr int B1_NCAP = 2048;          // 3..6-candidate entries per wave
constexpr size_t B1_LDS_MAX = 150 * 1024;
constexpr size_t B1_LDS_POISON_MAX = 160 * 1024;  // with the poisoned norms

__host__ __device__ inline int64_t dpad16(int64_t d);
inline size_t b1_frag_bytes(int64_t k, int64_t d) {
  return (size_t)(((k + 31) / 32 * 32) * ((d + 15) / 16 * 16) * 2 +
                  ((k + 31) / 32 * 32) * 4);
}
inline bool b1_ok(int64_t k, int64_t d) {
  return d <= 128 && k >= 2 && k <= 32767 && b1_frag_bytes(k, d) <= B1_LDS_MAX;
}
// The re-screen (dkm_dense.hip rescreen_list): the samples a screen leaves
// to the exact re-check are gathered and screened again by the chunked
// bf16x3 screen with its two-candidate list.  Shapes of the single-product
// screens with rows k_cand2 takes; RS_ROWS rows per gathered chunk.
constexpr int64_t RS_ROWS = 262144;
// DKM_MODE_TRANSLATE calls run in chunks of this many rows (the per-wave
// two-candidate and re-check lists of k_screen_b2: ~18 % and ~5 % of the
// rows against the reference's U[0, 1) initial centres at C3's shape)
constexpr int64_t TRANSL_CHUNK = 1ll << 25;
inline bool rescreen_ok(int64_t k, int64_t d) {
  return b1_ok(k, d) && d % 8 == 0 && d >= 8;
}

// GEMM screen eligibility: the register-tile screen takes d <= 128
inline bool gemm_path(int64_t k, int64_t d) {
  return d > 128 && k >= 2 && k <= 32767;
}
// samples per split chunk: <= 256 MB of split rows, a multiple of GT
inline int64_t gemm_chunk(int64_t d) {
  const int64_t per = ((d + 31) / 32 * 32) * 4;
  int64_t m = ((int64_t)1 << 28) / per / GT * GT;
  if (m > 65536) m = 65536;
  if (m < GT) m = GT;
  return m;
}

struct WsView {
  WsHeader *hdr;
  float *c32;     // k x dpad fp32 centres (zero padded)
  float *cn32;    // k fp32 ||c||^2 (computed in fp64, rounded once)
  double *cn64;   // k fp64 ||c||^2, sequential over t (sklearn row_norms)
  double *ct64;   // d x ct_ld(k) transposed centres (exact re-checks, CSR)
  uint16_t *ctb;  // bf16 transposed centres of the CSR screen, sliced:
                  // slice s = d rows of csr_slice_width(k, d) centres,
                  // contiguous (csr_ctb_len values in all)
  float *cfrag;   // fp32 -2*centres in MFMA A-fragment order (dkm_dense)
  float *cnpad;   // kpad16 fp32 ||c||^2, 2^100 for padding centres
  uint16_t *bfrag; // bf16 hi/lo of -2*centres, 16x16x32 fragment order
  uint16_t *b32frag; // d <= 32: bf16 hi/lo, 32x32x16 order (k_screen_w32)
  // b1_ok: b1frag of the translated centres -2 (c - m), m = mvec (fp32, the
  // centres' mean per feature; DKM_MODE_TRANSLATE)
  uint16_t *b1frag_t;
  // b1_ok: the bf16 low parts of -2c in b1frag's order (hi = b1frag): the
  // chunked bf16x3 screen in 32x32x16 form (k_screen_c32)
  uint16_t *b1frag_lo;
  float *mvec;
  float *cn32f;   // kpad32 ||c||^2 in 32x32 accumulator order
  uint16_t *b1frag; // b1_ok: bf16 hi of -2c, 32x32x16 order, dpad16 / 16
                    // K-steps per 32-centre block (k_screen_b1)
  int2 *clist;     // b1_ok: B1_SEGS x B1_CAP (offset, c1 | c2 << 16)
  int32_t *ccount; // b1_ok: entries used per screen wave
  int4 *nlist;     // b1_ok: B1_SEGS x B1_NCAP (offset, 6 centres as 16-bit
                   // pairs, 0xffff = none): 3..6-candidate samples
  int32_t *ncount; // b1_ok: entries used per screen wave
  int2 *tlist;    // TL_SEGS x TL_CAP undecided (offset, prev) per screen wave
  int32_t *tcount; // TL_SEGS entries used per screen wave
  // re-screen of the re-check list (rescreen_ok shapes, else nullptr): the
  // list compacted (TL_SEGS x TL_CAP entries), its per-segment offsets, and
  // a chunk of RS_ROWS gathered rows (fp64 or fp32) with their labels
  int2 *rlist;
  int32_t *rprefix;
  int32_t *rlab;
  void *rx;
  // block skipping of k_screen_b2 (mind_ok(k, d), else NULL): k x MIND_LD
  // lower bounds of the distance from centre p to the nearest other centre
  // of each 32-centre block (+inf past the last block)
  float *mind;
  // GEMM screen (gemm_path only; else NULL)
  char *gfrag;     // kpad256 x dpad32 centre tiles (-2c, bf16 hi/lo)
  char *gfrag1;    // kpad256 x dpad32 centre tiles (-2c, bf16 hi only:
                   // 32 features per 64-B row, the single-product screen)
  float *gcn;      // kpad256 fp32 ||c||^2, 2^100 for padding centres
  char *gxs;       // gemm_chunk samples: split tiles of the current chunk
  float *gxn;      // gemm_chunk fp32 upper bounds of ||x||
  char *gxs1;      // the same for the next chunk (split while the current
  float *gxn1;     // chunk is screened, on a second stream)
  int2 *gpart;     // gemm_chunk x kpad256/GT x GTOP (score bits, centre)
  int64_t gchunk;  // samples per split chunk
  // sorted sums (dkm_sums.hip; k <= SORT_KMAX, else NULL)
  int32_t *soff;   // k + 1 cluster offsets into sitems
  int32_t *scur;   // k scatter cursors
  int32_t *scnt;   // k counts
  // the tail: three arrays of nq entries
  int64_t nq;
  int32_t *queue; // label scratch / previous labels / re-check indices
  int32_t *sitems; // sample indices grouped by cluster
  int32_t *smoved; // samples whose label changed (delta sums)
};

// Single-product screen with the centres on the lanes (dkm_b2.hip): the
// threshold pass without per-block norm reads.  Returns 1 (nothing
// launched) when its LDS image does not fit; the caller runs k_screen_b1.
int b2_probe();  // != 0: a result-invalidating timing probe build
size_t b2_lds_bytes(int64_t k, int64_t d);
// the block-skip table (WsView::mind): 32-centre blocks per row
constexpr int MIND_LD = 64;
inline bool mind_ok(int64_t k, int64_t d) {
  return b1_ok(k, d) && (k + 31) / 32 <= MIND_LD;
}
// The sample image (dkm_x_image_*): a resident bf16 copy of X in the
// operand order of the screen that reads it, then fp32 |x|^2 per row
// (rows and features past n, d zero).  Kinds:
//  IMG_SINGLE (k_screen_b2): 32-row tiles of dpad16(d) / 16 K-steps x 1 KB,
//    lane l of K-step s = row l & 31, features 16 s + 8 (l >> 5) .. + 7;
//  IMG_SPLIT (k_screen_w32, d <= 32): 32-row tiles of 4 x 1 KB (hi K-slice
//    0, hi 1, lo 0, lo 1), lane l of slice s = row l & 31, features
//    16 (l >> 5) + 8 s .. + 7, hi = bf16(fl32(x)), lo = bf16(fl32(x) - hi).
//  IMG_SORTED (k_screen_b2 with block skipping): the IMG_SINGLE layout over
//    the rows perm[0 .. nt*32) -- the samples grouped by a label vector --
//    then int32 perm (sample of each image row, -1 past n) and int32 plab
//    (the current label of each image row: the screen's hints, kept equal
//    to labels[perm[i]] by the screen and k_plab sync).
//  IMG_GEMM (k_gemm_screen1, d > 128): the single-product GEMM screen's
//    sample tiles (dkm_gemm.hip layout: 256-row tiles of dpad32(d) / 32
//    stages x 16 KB, bf16 hi of fl32(x), 64-B rows) over every row, then
//    fp32 upper bounds of ||x|| (not |x|^2) per row, padding rows 0.
constexpr int IMG_NONE = 0, IMG_SINGLE = 1, IMG_SPLIT = 2, IMG_SORTED = 3,
              IMG_GEMM = 4;
struct XImage {
  const uint16_t *tiles;
  const float *xx;  // IMG_GEMM: ||x|| bounds
  int kind;
  const int32_t *perm;  // IMG_SORTED only
  int32_t *plab;        // IMG_SORTED only
};
size_t x_image_bytes(int64_t n, int64_t d, int kind);
XImage x_image_view(const void *image, int64_t n, int64_t d, int kind);
template <class TX>
int launch_x_image(const TX *X, int64_t n, int d, int64_t ldx, int kind,
                   void *image, int cus, hipStream_t s);
// acc != NULL: also acc += the full [sums | counts] of X by labels, in the
// same pass over X (x_image_sums_fused(d) must hold)
template <class TX>
int launch_x_image_sorted(const TX *X, int64_t n, int d, int64_t ldx,
                          const int32_t *labels, int k, const WsView &v,
                          void *image, int cus, hipStream_t s,
                          double *acc = nullptr);
inline bool x_image_sums_fused(int64_t d) {
  const int64_t nks = (d + 15) / 16;
  return nks == 1 || nks == 2 || nks == 4 || nks == 8;
}
// IMG_SORTED: plab <- labels[perm] where the screen marked it
// (-(previous + 2)); with `moved`: the rows whose label changed are listed in
// moved[] (count in *nmoved, zeroed here) and prevs[sample] = their previous
// label (the incremental sums' input, sorted_sums_moved).  No-op for the
// other kinds.
int launch_plab_sync(const XImage &img, int64_t n, int k, const int32_t *lab,
                     int cus, hipStream_t s, int32_t *moved = nullptr,
                     int32_t *nmoved = nullptr, int32_t *prevs = nullptr);
template <class TX>
int launch_screen_b2(const TX *X, int64_t end, int d, int64_t ldx, int k,
                     const WsView &v, int32_t *lab_out, int64_t base,
                     int hint, int cus, hipStream_t s, int *nseg,
                     XImage img, bool transl = false);

// Two-candidate samples of the single-product screens (dkm_cand.hip):
// the reference arithmetic on both listed centres.  1 = not launched
// (d % 8 != 0 or d > 128: the screens never list such samples).
template <class TX>
int launch_cand2_leaf(const TX *X, int d, int64_t ldx, const double *C,
                      const WsView &v, int32_t *lab_out, int64_t base,
                      int nseg, int cus, hipStream_t s);

// Sorted sums: counting sort of the sample indices by label (LDS histograms
// of k bins: k <= SORT_KMAX), then segmented row sums.
constexpr int SORT_KMAX = 16384;
bool sorted_sums_ok(int64_t k, int64_t n, const WsView &v);
template <class TX>
int sorted_sums(const TX *X, int64_t lo, int64_t hi, int d, int64_t ldx,
                const int32_t *lab, const int32_t *prev, int k, double *acc,
                const WsView &v, hipStream_t s);
// Incremental sums from a moved list already built (launch_plab_sync with
// moved = v.smoved, nmoved = &v.hdr->nmoved): +x by lab, -x by prevs.
template <class TX>
int sorted_sums_moved(const TX *X, int64_t n, int d, int64_t ldx,
                      const int32_t *lab, const int32_t *prevs, int k,
                      double *acc, const WsView &v, hipStream_t s);

// Sample indices [lo, hi) grouped by lab[i] (counting sort) into v.sitems,
// cluster c at [v.soff[c], v.soff[c + 1]) (the CSR sums, dkm_sparse.hip).
int sort_by_label(const int32_t *lab, int64_t lo, int64_t hi, int k,
                  const WsView &v, hipStream_t s);

// Per-wave lists of the screen's undecided samples (resolved by
// k_recheck_list without scanning the labels): one segment of TL_CAP
// entries per screen wave, TL_SEGS >= 256 CUs x 32 waves.
constexpr int TL_CAP = 2048;
constexpr int TL_SEGS = 8192;

// CSR screen (dkm_sparse.hip): the centres are cut into S slices (a power
// of two <= 8) whose bf16 C^T fits CSR_SLICE_BYTES, never narrower than one
// 64-centre pass; slice s is stored as its own contiguous d x width block,
// so that the lines of a slice spread over every set of an XCD's L2 (rows
// of the full d x k transpose, 1 KB apart at k = 256, fell into one set in
// eight: 10 % L2 misses at C5, profiles/r04/pmc/c5_csr_pmc_summary_4M.txt).
// 16 MB: every slice costs a walk over the entries, which outweighs the L2
// locality of smaller slices (C5's 10 MB table: one slice is fastest).
constexpr size_t CSR_SLICE_BYTES = 16u << 20;
constexpr int CSR_PASS = 64;
__host__ __device__ inline int csr_slices(int64_t k, int64_t d) {
  int S = 1;
  while (S < 8 && (k + S - 1) / S > CSR_PASS &&
         (size_t)(((k + S - 1) / S + CSR_PASS - 1) / CSR_PASS * CSR_PASS * d *
                  2) > CSR_SLICE_BYTES)
    S *= 2;
  return S;
}
__host__ __device__ inline int64_t csr_slice_width(int64_t k, int64_t d) {
  const int S = csr_slices(k, d);
  return ((k + S - 1) / S + CSR_PASS - 1) / CSR_PASS * CSR_PASS;
}
__host__ __device__ inline int64_t csr_ctb_len(int64_t k, int64_t d) {
  return (int64_t)csr_slices(k, d) * csr_slice_width(k, d) * d;
}

// MFMA fragment tiling of the centres: 16 centres x 16 dims per 1 KB block.
__host__ __device__ inline int64_t kpad16(int64_t k) { return (k + 15) / 16 * 16; }
__host__ __device__ inline int64_t kpad32(int64_t k) { return (k + 31) / 32 * 32; }
__host__ __device__ inline int64_t dpad16(int64_t d) { return (d + 15) / 16 * 16; }
__host__ __device__ inline int64_t dpad32(int64_t d) { return (d + 31) / 32 * 32; }
__host__ __device__ inline int64_t dpad64(int64_t d) { return (d + 63) / 64 * 64; }

size_t ws_bytes(int64_t k, int64_t d, int64_t n_queue);
int64_t default_queue(int64_t k, int64_t d);
int ws_view(const void *ws, size_t bytes, int64_t k, int64_t d, WsView *v);

// ---------------------------------------------------------------------------
// numpy add.reduce order (loops_utils.h pairwise sum, 8192-element buffers).
// `F` returns the t-th term.  Used on the exact paths only.
// ---------------------------------------------------------------------------
template <class F>
__device__ __forceinline__ double pw_leaf(const F &f, int64_t lo, int64_t n) {
  if (n < 8) {
    double r = -0.0;
    for (int64_t i = 0; i < n; ++i) r = r + f(lo + i);
    return r;
  }
  double r0 = f(lo + 0), r1 = f(lo + 1), r2 = f(lo + 2), r3 = f(lo + 3);
  double r4 = f(lo + 4), r5 = f(lo + 5), r6 = f(lo + 6), r7 = f(lo + 7);
  const int64_t stop = n - (n & 7);
  int64_t i = 8;
  for (; i < stop; i += 8) {
    r0 = r0 + f(lo + i + 0);
    r1 = r1 + f(lo + i + 1);
    r2 = r2 + f(lo + i + 2);
    r3 = r3 + f(lo + i + 3);
    r4 = r4 + f(lo + i + 4);
    r5 = r5 + f(lo + i + 5);
    r6 = r6 + f(lo + i + 6);
    r7 = r7 + f(lo + i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res = res + f(lo + i);
  return res;
}

// Recursive halving above 128 elements, as an explicit post-order walk.
// n <= 8192 (one iterator buffer): at most 6 halvings, so 8 stack levels.
// `leaf(lo, n)` returns the value of a leaf block (n <= 128); leaves are
// visited left to right.
template <class LEAF>
__device__ double pw_tree(LEAF &&leaf, int64_t lo, int64_t n) {
  if (n <= 128) return leaf(lo, n);
  int64_t flo[8];
  int fn[8];
  double fleft[8];
  int fstate[8];
  int sp = 0;
  flo[0] = lo;
  fn[0] = n;
  double val = 0.0;
  bool have = false;
  for (;;) {
    if (!have) {
      if (fn[sp] <= 128) {
        val = leaf(flo[sp], (int64_t)fn[sp]);
        have = true;
      } else {
        int64_t n2 = fn[sp] / 2;
        n2 -= n2 % 8;
        fstate[sp] = 0;
        flo[sp + 1] = flo[sp];
        fn[sp + 1] = n2;
        ++sp;
        continue;
      }
    }
    if (sp == 0) return val;
    --sp;
    int64_t n2 = fn[sp] / 2;
    n2 -= n2 % 8;
    if (fstate[sp] == 0) {
      fleft[sp] = val;
      fstate[sp] = 1;
      flo[sp + 1] = flo[sp] + n2;
      fn[sp + 1] = fn[sp] - n2;
      ++sp;
      have = false;
    } else {
      val = fleft[sp] + val;
    }
  }
}

template <class F>
__device__ double pw_block(const F &f, int64_t lo, int64_t n) {
  return pw_tree(
      [&](int64_t a, int64_t m) -> double { return pw_leaf(f, a, m); }, lo,
      n);
}

template <class F>
__device__ double pw_sum(const F &f, int64_t n) {
  double res = 0.0;
  for (int64_t s = 0; s < n; s += 8192) {
    const int64_t m = (n - s) < 8192 ? (n - s) : 8192;
    res = res + pw_block(f, s, m);
  }
  return res;
}

// Squared-difference term (x_t - c_t)^2, rounded exactly like numpy:
// the difference, then the product, each correctly rounded (no FMA).
template <class TX>
struct SqDiff {
  const TX *x;
  const double *c;
  __device__ __forceinline__ double operator()(int64_t t) const {
    const double df = (double)x[t] - c[t];
    return df * df;
  }
};

// Same term against transposed centres C^T (d x k): lane-coalesced reads.
template <class TX>
struct SqDiffT {
  const TX *x;
  const double *ct;  // &C^T[0][j]
  int64_t k;
  __device__ __forceinline__ double operator()(int64_t t) const {
    const double df = (double)x[t] - ct[t * k];
    return df * df;
  }
};

// Register-resident exact distance for d <= MAXD (MAXD multiple of 8):
// numpy's pairwise order specialised to n <= 128.  c may point to LDS.
template <int MAXD, class CPTR>
__device__ __forceinline__ double exact_sqdist_reg(const double (&x)[MAXD],
                                                   CPTR c, int d) {
  static_assert(MAXD % 8 == 0 && MAXD <= 128, "MAXD");
  if (d < 8) {
    double r = -0.0;
#pragma unroll
    for (int t = 0; t < 8 && t < MAXD; ++t)
      if (t < d) {
        const double df = x[t] - c[t];
        r = r + df * df;
      }
    return r;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const double df = x[j] - c[j];
    r[j] = df * df;
  }
  const int full = d - (d & 7);
#pragma unroll
  for (int b = 1; b < MAXD / 8; ++b) {
    if (8 * b < full) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const double df = x[8 * b + j] - c[8 * b + j];
        r[j] = r[j] + df * df;
      }
    }
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
  for (int t = 8; t < MAXD; ++t)
    if (t >= full && t < d) {
      const double df = x[t] - c[t];
      res = res + df * df;
    }
  return res;
}

// np.argmin's order on distances (base.py:173,200): a NaN ranks before every
// number (the FIRST NaN wins), otherwise first index of the minimum.  The
// distances are sqrt'd sums of squares, so every non-NaN one is >= 0 and
// mapping NaN to -1 gives that order under plain (value, index) compares.
__device__ __forceinline__ double argmin_key(double v) {
  return v != v ? -1.0 : v;
}

// (dist, idx) lexicographic minimum across a wave: first index wins ties.
__device__ __forceinline__ void wave_argmin(double &dist, int &idx) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double od = __shfl_xor(dist, off, WAVE);
    const int oi = __shfl_xor(idx, off, WAVE);
    if (od < dist || (od == dist && oi < idx)) {
      dist = od;
      idx = oi;
    }
  }
}

__device__ __forceinline__ void atomic_add_f64(double *p, double v) {
  unsafeAtomicAdd(p, v);  // global_atomic_add_f64 (no CAS loop on gfx950)
}

// ---------------------------------------------------------------------------
// dkm_gemm.hip entry points (host side)
// ---------------------------------------------------------------------------
// centre tiles + padded norms for the GEMM screen (after k_prepare)
int gemm_prepare(const double *C, int64_t k, int64_t d, const WsView &v,
                 hipStream_t s);
// Screen samples [base, end): labels (or -(prev + 2) for the exact re-check,
// counted in hdr->qcount).  acc != NULL: the merge step also moves rows
// between the sums with fp64 atomics (delta = true: only changed labels).
// img (IMG_GEMM, or NULL): the resident sample tiles the single-product
// screen reads instead of splitting X (chunks starting on a 256-row tile).
// bimg (bf16x3 only, or NULL): the IMG_GEMM image the chunk splits write too.
template <class TX>
int gemm_screen(const TX *X, int64_t base, int64_t end, int d, int64_t ldx,
                const double *C, int k, const WsView &v, int32_t *lab_out,
                double *acc, bool delta, bool one, const XImage *img,
                hipStream_t s, const XImage *bimg = nullptr);
// the IMG_GEMM image of X (x_image_view layout)
template <class TX>
int gemm_image(const TX *X, int64_t n, int d, int64_t ldx, const XImage &img,
               hipStream_t s);

}  // namespace dkm
