/*
 * dkm.h -- C ABI of libdkm.so, the MI355X (gfx950) k-means Lloyd hot path.
 *
 * Drop-in boundary for dislib's k-means (reference: /root/reference,
 * dislib v0.2.0).  The reference is pure Python over PyCOMPSs tasks; the
 * functions below replace its per-Subset task bodies and its reduction tree.
 * Each entry cites the reference function it replaces.
 *
 * Conventions
 *  - All array pointers are DEVICE pointers (hipMalloc / torch CUDA tensors)
 *    unless documented otherwise.  The caller owns every buffer; the library
 *    never allocates or frees caller memory.  A scratch area ("workspace") of
 *    dkm_workspace_bytes() bytes is provided by the caller.
 *  - Every call is asynchronous and stream-ordered on `stream` (a
 *    hipStream_t passed as void*; NULL = the legacy default stream).
 *  - Every call returns 0 on success, or a nonzero DKM_E_* / hipError_t code;
 *    dkm_last_error() returns a thread-local message for the last failure.
 *    No C++ exception ever crosses this boundary.
 *  - Matrices are row-major with a leading dimension (elements) `ld`.
 */
#ifndef DKM_H
#define DKM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DKM_ABI_VERSION 3

/* error codes (besides hipError_t values passed through) */
#define DKM_OK 0
#define DKM_E_ARG 10001       /* invalid argument / shape                    */
#define DKM_E_WORKSPACE 10002 /* workspace too small                         */
#define DKM_E_LAUNCH 10003    /* kernel launch failed                        */
#define DKM_E_PARSE 10004     /* malformed input text (loaders)              */
#define DKM_E_COMM 10005      /* RCCL missing or an RCCL call failed         */

/* assignment modes (flags) */
#define DKM_MODE_AUTO 0     /* library picks: SCREEN32 when profitable       */
#define DKM_MODE_EXACT 1    /* direct ||x-c||^2 in numpy's pairwise order for
                               every (sample, centre): reference arithmetic   */
#define DKM_MODE_SCREEN32 2 /* fp32 ||c||^2-2x.c screen with a rigorous error
                               bound; ambiguous samples re-checked with the
                               EXACT arithmetic.  Labels identical to EXACT. */
#define DKM_MODE_SCREEN_BF16X3 3 /* same, x.c from bf16 hi/lo splits on the
                               bf16 MFMA (hi*hi + hi*lo + lo*hi); its own
                               bound; labels identical to EXACT.            */
#define DKM_MODE_SCREEN_BF16 4 /* same, one bf16 product per term (hi*hi):
                               a third of the matrix work, a looser bound;
                               the candidates it leaves are re-checked with
                               the EXACT arithmetic.  Labels identical.     */
#define DKM_MODE_MASK 0xff  /* the arithmetic; flags may be OR'ed above it:  */
#define DKM_MODE_NOHINT 0x100 /* the incoming labels of dkm_partial_sum /
                               dkm_assign_delta are not used as hints (the
                               caller knows them to be poor, e.g. labels of
                               the initial centres): no threshold pass    */
#define DKM_MODE_B1 0x200   /* the single-product screen in its
                               centres-on-rows form (k_screen_b1, the
                               fallback when k_screen_b2's LDS image does
                               not fit) for every shape; identical labels */
#define DKM_MODE_TRANSLATE 0x400 /* with DKM_MODE_SCREEN_BF16 (or the AUTO
                               choice of it), no sorted image: the centres-
                               on-lanes screen scores ||c||^2 - 2 x.(c - m)
                               with m the centres' mean (the same order of
                               the centres for every sample; x.m is common to
                               all of them), so its bf16 rounding error
                               scales with max ||c - m|| instead of
                               max ||c||: crowded centres (the reference's
                               U[0, 1) initial centres) leave far fewer
                               samples to the re-checks.  Labels identical */

/* sum-dtype flags for dkm_update_centers (reference keeps X's dtype for the
 * partial sums; base.py:178 and :147) */
#define DKM_SUMS_F64 0
#define DKM_SUMS_F32 1  /* fp32 samples: centre = fl32(fl32(sum)/fl32(count)) */
#define DKM_SUMS_RECIP 2 /* sparse: centre = sum * (1.0/count) (scipy divide) */

int dkm_abi_version(void);

/* Load every kernel's code object now instead of at its first launch (the
 * runtime loads a source file's kernels lazily, several ms per file: the
 * first Lloyd iterations paid it inside the fit).  Optional; idempotent.
 * Replaces nothing in the reference (PyCOMPSs workers import their
 * libraries before the first task). */
int dkm_preload(void);
const char *dkm_last_error(void);

/* Workspace needed for k centres of d features and up to n_queue re-check
 * slots (n_queue = 0 lets the library pick).  Host function. */
size_t dkm_workspace_bytes(int64_t k, int64_t d, int64_t n_queue);

/* prepare flags */
#define DKM_PREP_CSR 1 /* prepare for the CSR kernels only: the transposed
                          centres C^T (fp64 and fp32, d rows, stride k
                          rounded up to 16) and |c|^2, without the dense
                          screens' centre tiles                            */

/* Derive per-iteration centre data (fp32 copy, |c|^2 in sklearn's sequential
 * order, error-bound scalars, optionally C^T) into the workspace and ZERO the
 * accumulator acc[k*(d+1)] ([sums | counts]) when acc != NULL.  Replaces the
 * implicit per-task centre broadcast of base.py:110,114 (and sklearn's
 * row_norms of the centres, recomputed per sample by the reference).      */
int dkm_prepare_centers(const double *C, int64_t k, int64_t d, int flags,
                        void *ws, size_t ws_bytes, double *acc, void *stream);

/* Fused assignment + per-cluster sum/count for dense samples.
 * Replaces `_partial_sum` (cluster/kmeans/base.py:166-181), including
 * `_vec_matrix_euclid` (:204-205), `np.argmin` (:173) and `set_label` (:176).
 * Accumulates into acc = [sums k*d | counts k] (fp64, += semantics; call
 * dkm_prepare_centers first in an iteration).  labels (int32[n]) may be NULL
 * when not wanted.  X is fp64 (…_f64) or fp32 (…_f32); C is always fp64.  */
int dkm_partial_sum_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                        const double *C, int64_t k, const void *ws,
                        size_t ws_bytes, int32_t *labels, double *acc,
                        int mode, void *stream);
int dkm_partial_sum_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                        const double *C, int64_t k, const void *ws,
                        size_t ws_bytes, int32_t *labels, double *acc,
                        int mode, void *stream);

/* Incremental form of dkm_partial_sum for the Lloyd loop.  labels (int32[n],
 * in/out) holds each sample's previous label (-1 = none); on return it holds
 * the new labels (identical to dkm_partial_sum's) and delta (k*(d+1), +=)
 * has received +x / +1 for every sample that joined a cluster and -x / -1
 * for every sample that left one, so acc_new = acc_old + delta is the
 * [sums | counts] of the new assignment (up to fp64 rounding order).  After
 * the first iterations few labels change, so almost no sample is added
 * anywhere; the caller refreshes acc from scratch periodically.           */
int dkm_assign_delta_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                         const double *C, int64_t k, const void *ws,
                         size_t ws_bytes, int32_t *labels, double *delta,
                         int mode, void *stream);
int dkm_assign_delta_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                         const double *C, int64_t k, const void *ws,
                         size_t ws_bytes, int32_t *labels, double *delta,
                         int mode, void *stream);

/* The sample image: a resident bf16 copy of X in the operand order of the
 * screen that reads it, plus fp32 |x|^2 per row.  Built once per dataset
 * (it depends only on X): the screen then streams 2 or 4 B per feature
 * instead of sizeof(X) and skips the conversion.  Labels, sums and
 * re-checks still come from X itself, so results are identical with or
 * without it.  An image is valid only for the exact X, n and d (and kind)
 * it was built from; rebuild it if X changes.
 *   kind DKM_IMAGE_SINGLE: bf16(fl32(x)) for the label-hinted
 *     single-product screen (MODE_SCREEN_BF16 or the AUTO choice when the
 *     sums exceed LDS; d <= 128);
 *   kind DKM_IMAGE_SPLIT: bf16 hi and lo of fl32(x) for the d <= 32
 *     bf16x3 screen (MODE_SCREEN_BF16X3 or the AUTO choice), read by its
 *     delta / labels-only launches;
 *   kind DKM_IMAGE_GEMM: bf16(fl32(x)) in the 256-row tiles of the
 *     single-product GEMM screen (d > 128: MODE_SCREEN_BF16 or AUTO), plus
 *     an fp32 upper bound of ||x|| per row (2 B per feature + 4 B per row;
 *     10M x 1024: 20.5 GB).
 * dkm_x_image_kind(k, d, mode) says which kind the selected screen reads
 * (DKM_IMAGE_NONE: building one would be wasted).  The _img forms of
 * dkm_partial_sum / dkm_assign_delta take it (image NULL = none); every
 * other argument is theirs.  Same interface as base.py:166-181.
 * image_kind | DKM_IMAGE_BUILD: the image memory is allocated but not built
 * yet; the call builds it (the d <= 32 bf16x3 screen's full-sums pass writes
 * the split image while it converts X anyway -- no separate pass over X --
 * any other call builds it first with dkm_x_image_*), after which the
 * caller passes the kind without the flag.                                */
#define DKM_IMAGE_NONE 0
#define DKM_IMAGE_SINGLE 1
#define DKM_IMAGE_SPLIT 2
#define DKM_IMAGE_SORTED 3
#define DKM_IMAGE_GEMM 4
#define DKM_IMAGE_BUILD 0x100
int dkm_x_image_kind(int64_t k, int64_t d, int mode);
size_t dkm_x_image_bytes(int64_t n, int64_t d, int kind);
int dkm_x_image_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                    int kind, void *image, size_t image_bytes, void *stream);
int dkm_x_image_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                    int kind, void *image, size_t image_bytes, void *stream);
/* The label-sorted image (DKM_IMAGE_SORTED, dkm_x_image_bytes(n, d, 3)
 * bytes): the DKM_IMAGE_SINGLE image of X with its rows grouped by
 * `labels` (a counting sort in the workspace, which needs n label slots:
 * dkm_workspace_bytes(k, d, n_queue >= n)), plus the row order and a copy of
 * the labels in that order.  The single-product screen then screens 32-row
 * tiles of (mostly) one label and skips every 32-centre block the triangle
 * inequality proves farther than that label's centre.  The labels never
 * depend on the grouping.  The image's label copy is maintained by the
 * calls that take the image: once built, pass it to EVERY call that updates
 * those labels (MODE_SCREEN_BF16 or AUTO; other modes refuse it), or build
 * it again.  dkm_x_image_sorted_ok(k, d): whether (k, d) takes it.        */
int dkm_x_image_sorted_ok(int64_t k, int64_t d);
int dkm_x_image_sorted_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                           const int32_t *labels, int64_t k, const void *ws,
                           size_t ws_bytes, void *image, size_t image_bytes,
                           void *stream);
int dkm_x_image_sorted_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                           const int32_t *labels, int64_t k, const void *ws,
                           size_t ws_bytes, void *image, size_t image_bytes,
                           void *stream);
/* The same image, and acc += the full [sums | counts] of X by `labels` (the
 * dkm_label_sums_* result) in the same pass over X: a fit that builds the
 * image from an iteration's labels gets that iteration's sums without a
 * second read of X (predict, then this call, instead of partial_sum, then
 * dkm_x_image_sorted_*).  Sums are fp64 atomics: equal to dkm_label_sums_*
 * up to the order of the additions.                                        */
int dkm_x_image_sorted_sums_f64(const double *X, int64_t n, int64_t d,
                                int64_t ldx, const int32_t *labels, int64_t k,
                                const void *ws, size_t ws_bytes, void *image,
                                size_t image_bytes, double *acc, void *stream);
int dkm_x_image_sorted_sums_f32(const float *X, int64_t n, int64_t d,
                                int64_t ldx, const int32_t *labels, int64_t k,
                                const void *ws, size_t ws_bytes, void *image,
                                size_t image_bytes, double *acc, void *stream);
/* image_bytes: the image buffer's size, checked against
 * dkm_x_image_bytes(n, d, image_kind) (an image built for other n or d is
 * refused instead of read out of bounds).                                 */
int dkm_partial_sum_img_f64(const double *X, const void *image, int image_kind,
                            size_t image_bytes, int64_t n, int64_t d,
                            int64_t ldx, const double *C, int64_t k,
                            const void *ws, size_t ws_bytes, int32_t *labels,
                            double *acc, int mode, void *stream);
int dkm_partial_sum_img_f32(const float *X, const void *image, int image_kind,
                            size_t image_bytes, int64_t n, int64_t d,
                            int64_t ldx, const double *C, int64_t k,
                            const void *ws, size_t ws_bytes, int32_t *labels,
                            double *acc, int mode, void *stream);
int dkm_assign_delta_img_f64(const double *X, const void *image,
                             int image_kind, size_t image_bytes, int64_t n,
                             int64_t d, int64_t ldx, const double *C,
                             int64_t k, const void *ws, size_t ws_bytes,
                             int32_t *labels, double *delta, int mode,
                             void *stream);
int dkm_assign_delta_img_f32(const float *X, const void *image, int image_kind,
                             size_t image_bytes, int64_t n, int64_t d,
                             int64_t ldx, const double *C, int64_t k,
                             const void *ws, size_t ws_bytes, int32_t *labels,
                             double *delta, int mode, void *stream);

/* acc[k*(d+1)] += [sums | counts] of the rows of X by labels (label < 0 or
 * >= k: skipped): the sums half of dkm_partial_sum for known labels.       */
int dkm_label_sums_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                       const int32_t *labels, int64_t k, const void *ws,
                       size_t ws_bytes, double *acc, void *stream);
int dkm_label_sums_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                       const int32_t *labels, int64_t k, const void *ws,
                       size_t ws_bytes, double *acc, void *stream);

/* y[i] += x[i] (device, fp64): acc_new = acc_old + delta.                  */
int dkm_add_f64(double *y, const double *x, int64_t n, void *stream);
/* The same, and *nonzero (device int32) <- 1 if any x[i] != 0, else 0:
 * a delta of all zeros leaves acc bit-identical, so the caller knows that
 * no sample changed cluster since its last full recomputation (its
 * periodic refresh is then skipped: the sums are exactly those of the
 * current assignment).                                                   */
int dkm_add_f64_nz(double *y, const double *x, int64_t n, int32_t *nonzero,
                   void *stream);
/* The running sums kept compensated: (hi, lo) += x by TwoSum, renormalised
 * so that hi = fl(hi + lo) -- hi is what dkm_update_centers reads.  Each
 * add is exact to ~2^-106 |hi|, so the only drift of a delta-updated state
 * against a fresh recomputation is the rounding of the deltas themselves
 * (<= ~2^-52 of the moved rows' magnitude per iteration), not the
 * |sums| x iterations of a plain fp64 add.  nonzero: as dkm_add_f64_nz
 * (NULL = not wanted).                                                   */
int dkm_add_f64_dd(double *hi, double *lo, const double *x, int64_t n,
                   int32_t *nonzero, void *stream);

/* Assignment only.  Replaces `_predict` (base.py:194-201).  Needs a prepared
 * workspace (dkm_prepare_centers with acc = NULL is allowed).             */
int dkm_predict_f64(const double *X, int64_t n, int64_t d, int64_t ldx,
                    const double *C, int64_t k, const void *ws,
                    size_t ws_bytes, int32_t *labels, int mode, void *stream);
int dkm_predict_f32(const float *X, int64_t n, int64_t d, int64_t ldx,
                    const double *C, int64_t k, const void *ws,
                    size_t ws_bytes, int32_t *labels, int mode, void *stream);

/* Centre recomputation + convergence criterion.  Replaces
 * `_recompute_centers` (base.py:137-147, the division and empty-cluster
 * rule) and the criterion of `_converged` (:122-135):
 *   C[c] = sums[c] / counts[c] for counts[c] != 0 (else unchanged),
 *   diff[1+c] = ||C_new[c] - C_old[c]||_2, diff[0] = sum over c in index
 *   order (diff: device buffer of k+1 doubles), and
 *   *flag = (diff[0] < tol*tol) ? 1 : 0 (flag nullable).
 * For DKM_SUMS_RECIP (sparse input) the per-centre distance follows
 * sklearn's sqrt(max(0, (-2 a.b + |a|^2) + |b|^2)) with sequential sums, as
 * the reference's sparse criterion does (base.py:123 pairwise_distances).
 * acc is the (all-reduced) [sums | counts] buffer.  sums_mode: DKM_SUMS_*. */
int dkm_update_centers(const double *acc, double *C, int64_t k, int64_t d,
                       int sums_mode, double tol, double *diff,
                       int32_t *flag, void *stream);

/* CSR samples (int64 indptr[n+1], int32 indices, fp64 data; d columns).
 * Replaces the sparse branch of `_partial_sum`/`_predict` (base.py:169,196:
 * sklearn euclidean_distances = sqrt(max(0, (-2 x.c + |x|^2) + |c|^2))).  */
int dkm_partial_sum_csr_f64(const int64_t *indptr, const int32_t *indices,
                            const double *data, int64_t n, int64_t d,
                            const double *C, int64_t k, const void *ws,
                            size_t ws_bytes, int32_t *labels, double *acc,
                            void *stream);
/* Incremental CSR form (the fit loop), same contract as
 * dkm_assign_delta_f64: labels in/out (-1 = none), delta += the rows whose
 * label changed (+x to the new cluster, -x from the previous one).       */
int dkm_assign_delta_csr_f64(const int64_t *indptr, const int32_t *indices,
                             const double *data, int64_t n, int64_t d,
                             const double *C, int64_t k, const void *ws,
                             size_t ws_bytes, int32_t *labels, double *delta,
                             void *stream);
int dkm_predict_csr_f64(const int64_t *indptr, const int32_t *indices,
                        const double *data, int64_t n, int64_t d,
                        const double *C, int64_t k, const void *ws,
                        size_t ws_bytes, int32_t *labels, void *stream);

/* ------------------------------------------------------------------------
 * Multi-GPU: the one collective of a Lloyd iteration (SURVEY.md section
 * 8(b,e)).  Replaces the `_merge` arity tree and the `compss_wait_on` gather
 * (cluster/kmeans/base.py:137-143, 184-191): an in-place RCCL sum of every
 * GPU's [sums k*d | counts k] buffer; each rank then runs the same
 * dkm_update_centers.  librccl is loaded at the first call (the instance
 * already in the process if any).  Host functions.
 * --------------------------------------------------------------------- */
#define DKM_COMM_ID_BYTES 128

/* One process per GPU: rank 0 creates the id (DKM_COMM_ID_BYTES bytes),
 * the caller hands it to every rank, every rank joins with its device. */
int dkm_allreduce_unique_id(void *id);
int dkm_allreduce_init_rank(const void *id, int nranks, int rank, int device);
/* One process driving ndev GPUs (ncclCommInitAll over devs[]). */
int dkm_allreduce_init(int ndev, const int *devs);
/* buf[0..count) (device memory of `device`) <- sum over all ranks,
 * stream-ordered on `stream` (a hipStream_t of that device). */
int dkm_allreduce_sum_f64(double *buf, int64_t count, int device,
                          void *stream);
/* Destroy every communicator of this process. */
int dkm_allreduce_finalize(void);
/* Destroy the communicator of `device` only (0 when it has none). */
int dkm_allreduce_finalize_device(int device);
/* 0 when librccl loads and has every entry point used here: a cheap,
 * non-blocking check every rank makes before the collective
 * ncclCommInitRank, so that the ranks agree on a fallback up front. */
int dkm_allreduce_available(void);
/* The communicator of `device`: its rank count (ncclCommCount) and this
 * rank's index in it (ncclCommUserRank).  DKM_E_ARG if it has none. */
int dkm_allreduce_comm_info(int device, int *nranks, int *rank);

/* Synthetic make_blobs rows [row0, row0+n) into X (n x d, ld = d), blob ids
 * into blob (nullable).  Counter-based: any row range regenerates
 * identically.  Bench/test data generator, not part of the reference path. */
int dkm_make_blobs_f64(double *X, int64_t row0, int64_t n, int64_t d,
                       int64_t n_blobs, uint64_t seed, double box, double std,
                       int32_t *blob, void *stream);

/* Diagnostics of the last SCREEN32 call on this workspace (device -> host,
 * synchronous on `stream`): number of samples sent to the exact re-check.  */
int dkm_screen_stats(const void *ws, int64_t *n_rechecked, void *stream);
/* Single-product screen counters over the workspace's life (host, syncs
 * `stream`): out[0] tiles given the threshold pass, out[1] tiles it
 * decided (the rest took the top-3 pass), out[2] 32-centre blocks screened
 * by threshold passes over the label-sorted image (DKM_IMAGE_SORTED),
 * out[3] tiles of that image the steady-state pass handed to the general
 * one (out has 4 entries).                                                 */
int dkm_screen_counters(const void *ws, int64_t *out, void *stream);
/* The lists the last single-product screen launch left (host, syncs
 * `stream`; diagnostics): out[0] samples for the exact re-check list,
 * out[1] two-candidate entries, out[2] 3..6-candidate entries, out[3]
 * samples that overflowed a list (found by the label scan).               */
int dkm_screen_lists(const void *ws, size_t ws_bytes, int64_t *out,
                     void *stream);

/* Build flags of this library: 0 for a product build.  DKM_BUILD_TIMING_ONLY
 * when an object was compiled with an A/B timing probe that invalidates
 * results (DKM_AB_B1_PROBE, DKM_AB_B2_PROBE, DKM_AB_SORTED_BSCALE != 1,
 * DKM_AB_SORTED_DBG, DKM_DBG_NOCOMPUTE, ...); DKM_BUILD_AB_VARIANT when any
 * object comes from an A/B variant build (csrc/variants*.sh).  bench.py
 * records a non-zero value in its line, and tests/test_isa_guard.py checks
 * that the in-tree library reports 0. */
#define DKM_BUILD_TIMING_ONLY 1
#define DKM_BUILD_AB_VARIANT 2
int dkm_build_flags(void);

/* ------------------------------------------------------------------------
 * Distance-primitive reuse outside the Lloyd loop (SURVEY.md section 8
 * row f4).  fp64 rows, row-major with leading dimensions; device pointers;
 * stream-ordered.
 * --------------------------------------------------------------------- */

/* Workspace bytes of dkm_knn_f64 (0 for invalid sizes). */
size_t dkm_knn_workspace_bytes(int64_t nq, int64_t nx, int64_t kn);
/* For each query row of Q (nq x d): the kn (1..32, <= nx) rows of X
 * (nx x d) nearest by dist = sqrt(r), r = sum_t (q_t - x_t)^2 summed
 * sequentially from t = 0 (sklearn KD-tree EuclideanDistance.rdist, the
 * regime sklearn picks for d <= 15), ascending (r, index).  out_dist
 * nq x kn fp64, out_idx nq x kn int64 (row indices of X).
 * Replaces NearestNeighbors.kneighbors: _get_neighbors per Subset pair and
 * _merge_queries (dislib/neighbors/base.py:40-111). */
int dkm_knn_f64(const double *Q, int64_t nq, int64_t ldq, const double *X,
                int64_t nx, int64_t ldx, int64_t d, int64_t kn, void *ws,
                size_t ws_bytes, double *out_dist, int64_t *out_idx,
                void *stream);
/* Sparse kNN, replacing the same reference path on CSR Subsets (sklearn
 * fits brute force on CSR and ranks by pairwise_distances_chunked with
 * squared=True): query CSR (q_indptr[nq+1] int64, q_indices int32 sorted
 * and unique within each row, q_data fp64) against the fit CSR (nx rows),
 * both d columns.  r = max(((-2 q.x) + ||q||^2) + ||x||^2, 0) in the
 * arithmetic of dkm_radius_count_csr_f64; neighbours ascending (r, index),
 * out_dist = sqrt(r).  kn in [1, nx] (passes of 32 beyond 32); workspace =
 * dkm_knn_workspace_bytes(nq, nx, kn).  The query and fit matrices may be
 * the same arrays.  out_f32 != 0: the Subsets were float32 (data passed
 * upcast to fp64): sklearn's upcast path rounds r to float32 before the
 * max, ranks by it and takes the float32 sqrt; so do these. */
int dkm_knn_csr_f64(const int64_t *q_indptr, const int32_t *q_indices,
                    const double *q_data, int64_t nq, const int64_t *x_indptr,
                    const int32_t *x_indices, const double *x_data,
                    int64_t nx, int64_t d, int64_t kn, int out_f32, void *ws,
                    size_t ws_bytes, double *out_dist, int64_t *out_idx,
                    void *stream);

/* DBSCAN epsilon query, replacing _compute_neighbours (dense) of
 * dislib/cluster/dbscan/classes.py:124-141: for query row q, the rows j of
 * X with numpy's sqrt(pairwise-sum((q - x_j)^2)) < eps (_vec_matrix_euclid,
 * :153-154).  Step 1: counts[nq] (int64) <- neighbour counts. */
int dkm_radius_count_f64(const double *Q, int64_t nq, int64_t ldq,
                         const double *X, int64_t nx, int64_t ldx, int64_t d,
                         double eps, int64_t *counts, void *stream);
/* Workspace bytes of dkm_radius_fill_f64 for `total` neighbours. */
size_t dkm_radius_workspace_bytes(int64_t nq, int64_t total);
/* Step 2: offsets[nq+1] = exclusive prefix sum of the counts (device);
 * list q goes to out_idx/out_dist[offsets[q] .. offsets[q+1]), ascending
 * (distance, index).  Reads offsets[nq] to the host (synchronises
 * `stream`). */
int dkm_radius_fill_f64(const double *Q, int64_t nq, int64_t ldq,
                        const double *X, int64_t nx, int64_t ldx, int64_t d,
                        double eps, const int64_t *offsets, void *ws,
                        size_t ws_bytes, int64_t *out_idx, double *out_dist,
                        void *stream);
/* Sparse epsilon query, replacing the `pairwise_distances` branch of
 * _compute_neighbours (dislib/cluster/dbscan/classes.py:130, sparse=True):
 * query rows q0 .. q0+nq of the CSR matrix (indptr[n+1] int64, indices
 * int32 sorted within each row, data fp64, n rows, d columns) against all
 * n rows.  Distance = sklearn 1.7 euclidean_distances for fp64 CSR:
 * sqrt(max(((-2 q.x) + ||q||^2) + ||x||^2, 0)), row norms summed in stored
 * order, q.x by scipy csr_matmat order (increasing column of the
 * intersection).  Same two steps, offsets and workspace as the dense pair.
 * out_f32 != 0 (float32 Subsets, data passed upcast to fp64): r rounded to
 * float32, then max, the float32 sqrt and `dist < float32(eps)`, as
 * sklearn's upcast path and numpy's float32 comparison do. */
int dkm_radius_count_csr_f64(const int64_t *indptr, const int32_t *indices,
                             const double *data, int64_t n, int64_t d,
                             int64_t q0, int64_t nq, double eps, int out_f32,
                             int64_t *counts, void *stream);
int dkm_radius_fill_csr_f64(const int64_t *indptr, const int32_t *indices,
                            const double *data, int64_t n, int64_t d,
                            int64_t q0, int64_t nq, double eps, int out_f32,
                            const int64_t *offsets, void *ws, size_t ws_bytes,
                            int64_t *out_idx, double *out_dist, void *stream);

/* ------------------------------------------------------------------------
 * Dataset loaders.  HOST functions: `buf`
 * and every output are host pointers; no GPU is touched.  `buf` holds
 * the whole file (len bytes); lines end at "\n", "\r\n" or "\r" (Python
 * text mode).  nthreads <= 0 = all hardware threads.  Call *_count first
 * to size the outputs.  `row_line[r]` = 0-based raw line of row r, so the
 * caller can cut Subsets every `subset_size` raw lines exactly like
 * `_load_file` (dislib/data/base.py:145-164).
 * --------------------------------------------------------------------- */

/* counts[4] <- {raw lines, rows, stored entries, threads used}.
 * Replaces the tokenizer of sklearn's load_svmlight_file as called by
 * `_read_libsvm` / `_read_file` (dislib/data/base.py:200-238). */
int dkm_libsvm_count(const char *buf, int64_t len, int nthreads,
                     int64_t *counts);
/* indptr[rows+1], indices[nnz] (as written: the caller applies sklearn's
 * zero_based="auto" shift per chunk), data[nnz], y[rows] (targets),
 * row_line[rows].  DKM_E_PARSE with sklearn's message for a bad number,
 * a negative index or indices that are not strictly increasing. */
int dkm_libsvm_parse(const char *buf, int64_t len, int nthreads,
                     int64_t *indptr, int32_t *indices, double *data,
                     double *y, int64_t *row_line);
/* counts[4] <- {raw lines, rows, fields of the first row, threads used}.
 * delimiter: a byte, or 0 for whitespace runs (numpy's delimiter=None).
 * Replaces np.genfromtxt in `_read_lines` / `_read_file`
 * (dislib/data/base.py:188, :212). */
int dkm_txt_count(const char *buf, int64_t len, int delimiter, int nthreads,
                  int64_t *counts);
/* out[rows x n_cols] row-major fp64 (unconvertible/empty field = NaN),
 * row_line[rows].  DKM_E_PARSE if a row has another number of fields. */
int dkm_txt_parse(const char *buf, int64_t len, int delimiter, int64_t n_cols,
                  int nthreads, double *out, int64_t *row_line);

#ifdef __cplusplus
}
#endif
#endif /* DKM_H */
