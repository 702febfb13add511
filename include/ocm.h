/*
 * ocm.h — C ABI of libocm.so, the MI355X (gfx950) SIMCA / VAE-SIMCA engine.
 *
 * The reference (TEAM-AIOLY/OCM-VAE-SIMCA) is pure Python and has no native
 * boundary; the boundary its drivers use is the estimator API of
 * utils/SIMCA.py and utils/CVSIMCA.py.  This header is the
 * native layer UNDER that API: every entry point replaces one piece of
 * arithmetic the reference runs through NumPy/SciPy/scikit-learn, cited
 * per function.  The Python mirror (ocm-vae-simca_amd/utils/SIMCA.py,
 * .../ocm/_lib.py) binds these with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Arrays marked [dev] are device pointers
 *    (HBM, e.g. torch tensor data_ptr()); [host] are host pointers.
 *  - Row-major.  X is n×p float32 with leading dimension ldx (elements).
 *  - `rows` [dev, nullable]: optional int64 row-index list; when non-NULL
 *    the r-th processed row is X[rows[r]] (class subsets / CV test sets
 *    without a gather copy).
 *  - `stream` is a hipStream_t (NULL = default stream).  Every call is
 *    stream-ordered; calls that return host values synchronise that stream.
 *  - Return 0 on success, a negative OCM_ERR_* code on failure;
 *    ocm_last_error() gives the message (thread-local).
 */
#ifndef OCM_H_
#define OCM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCM_ABI_VERSION 12

#define OCM_OK 0
#define OCM_ERR_ARG (-1)         /* invalid argument (maps to ValueError) */
#define OCM_ERR_HIP (-2)         /* HIP runtime error */
#define OCM_ERR_NOMEM (-3)       /* device allocation failed */
#define OCM_ERR_NOCONV (-4)      /* eigensolver hit max_iter (results still written) */
#define OCM_ERR_UNSUPPORTED (-5) /* shape outside the supported envelope */

/* decision types (utils/SIMCA.py:131-144) */
#define OCM_TYPE_SIM 0 /* dred = max(t, q)       */
#define OCM_TYPE_ALT 1 /* dred = sqrt(t² + q²)   */
#define OCM_TYPE_CI 2  /* dred = t + q           */
#define OCM_TYPE_DD 3  /* dred = t + q (dof-scaled t, q) */

typedef struct ocm_ctx ocm_ctx;

/* t = T2 * t2_scale, q = Q * q_scale; accept = dred(t, q) < dlim.
 * Non-dd types: t2_scale = 1/T2_limit, q_scale = 1/Q_limit.
 * dd: t2_scale = t2dof/t2scfact, q_scale = qdof/qscfact (utils/SIMCA.py:76-81,141-144). */
typedef struct ocm_decision {
  int32_t type;
  int32_t pad_;
  double t2_scale;
  double q_scale;
  double dlim;
} ocm_decision;

int ocm_abi_version(void);
/* 16 hex digits: the first 64 bits of the SHA-256 of the library's build
 * inputs (the csrc .hip sources, its headers and Makefile, in the Makefile's
 * ID_INPUTS order).  The Python binding refuses a library whose id differs from the
 * hash of the sources beside it (a stale prebuilt libocm.so). */
const char* ocm_build_id(void);
const char* ocm_last_error(void);
int ocm_ctx_create(int device, ocm_ctx** out);
int ocm_ctx_destroy(ocm_ctx* ctx);
/* Pre-size the context workspace (bytes) so later calls never allocate
 * (lets a caller capture the launch sequence in a hipGraph). */
int ocm_ctx_reserve(ocm_ctx* ctx, size_t bytes);

/* Live kernel timing for benchmarks: while enabled, every launch of a timed
 * kernel is bracketed by a hipEvent pair on its stream (no synchronisation).
 * ocm_ctx_read_timing waits for the recorded events, returns the summed
 * duration (ms) and launch count of kernel `kernel_id`, and clears them. */
#define OCM_TIMED_KERNELS 3
#define OCM_KERNEL_GRAM 0  /* the Gram main kernel (k_gram8e / k_gram8d / k_gram3 / k_gram) */
#define OCM_KERNEL_SCORE 1 /* k_score: fused projection / Q / T² kernel */
#define OCM_KERNEL_QUANT 2 /* k_q8_quant: int8 digit split feeding k_gram8d */
int ocm_ctx_set_timing(ocm_ctx* ctx, int enable);
int ocm_ctx_read_timing(ocm_ctx* ctx, int kernel_id, double* total_ms, int64_t* count);

/* Column mean of the first n processed rows, fp64 accumulation.
 * Replaces sklearn PCA mean_ (sklearn/decomposition/_pca.py:560; called
 * from utils/SIMCA.py:64-66).  Used with n = a small sample as the Gram
 * shift, and as the exact mean when needed.  mean_out [dev] p doubles. */
int ocm_colmean_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                    double* mean_out, void* stream);

/* Per-segment shifted Gram (default mode OCM_GRAM_I8X3): y = x − shift is
 * split into three int8 digits per value (power-of-two scale per 1536-row
 * block and column) and the six digit products of weight ≥ 254⁻² are summed
 * exactly in int32 on integer MFMA (fp32-grade Gram: max relative error
 * ≈ 5e-8 on the bench data).  Outlier guard: values above 16× their column's
 * robust sample scale (2^e ≥ median|y| over the first ≤ 4096 rows) are
 * screened out of the digits of their 32-column group and
 * added back exactly (fp64 fix-up), so one extreme row does not coarsen the
 * other rows of its block; when more than n/8 rows are screened the call
 * recomputes the Gram on the bf16×3 split.  Workspace: ≈ 3 B per value for the digit
 * planes plus the chunk partials (≈ 8.4 GB at 1M × 2048).
 * Replaces the SVD of the centred class matrix (utils/SIMCA.py:64-66 ->
 * sklearn _pca.py:569-584 scipy.linalg.svd gesdd): the covariance
 * eigen-decomposition needs only Σ yᵀy and Σ y with y = x - shift.
 * Segment s covers processed rows [seg_offsets[s], seg_offsets[s+1]).
 * G_out [dev] nseg·p·p doubles (full symmetric), colsum_out [dev] nseg·p.
 * seg_offsets [host] nseg+1 ascending, seg_offsets[0] = 0, last = n.
 * shift [dev] p floats.  p ≤ 64 always takes an fp64-accumulated VALU Gram. */
int ocm_gram_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                 const float* shift, const int64_t* seg_offsets, int32_t nseg, double* G_out, double* colsum_out,
                 void* stream);

/* Same with an explicit arithmetic mode and row-chunk length (0 = automatic):
 *   OCM_GRAM_I8X3   the default above;
 *   OCM_GRAM_F32    FP32 MFMA (v_mfma_f32_32x32x2_f32), f32 chunk partials summed in f64;
 *   OCM_GRAM_BF16X3 exact three-level bf16 split on bf16 MFMA;
 *   OCM_GRAM_I8X3_K32 the i8×3 Gram on v_mfma_i32_32x32x32_i8 (round 2's
 *                   kernel) instead of the default's 16x16x64: bit-identical
 *                   result, kept for kernel A/B. */
#define OCM_GRAM_I8X3 0
#define OCM_GRAM_F32 1
#define OCM_GRAM_BF16X3 2
#define OCM_GRAM_I8X3_K32 3
int ocm_gram_f32_ex(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                    const float* shift, const int64_t* seg_offsets, int32_t nseg, int32_t mode, int64_t chunk_rows,
                    double* G_out, double* colsum_out, void* stream);

/* Outlier-guard marks ((row, 32-column group) pairs screened out) of the
 * context's last i8×3 Gram that synchronised (diagnostics / tests). */
int ocm_gram_last_marks(ocm_ctx* ctx, int64_t* marks_out);

/* Covariance from a signed combination of segment Grams (CV downdating):
 *   Gc = Σ_t coef[t]·G[t], sc = Σ_t coef[t]·colsum[t], d = sc/n,
 *   C = (Gc - n·d·dᵀ)/(n-1), mean = shift + d.
 * Replaces np.cov / explained_variance_ = S²/(n-1) (_pca.py:584).
 * G_list/colsum_list/coef [host] arrays of nterm pointers/values; C_out [dev]
 * p·p doubles; mean_out [dev] p doubles. */
int ocm_cov_from_gram(ocm_ctx* ctx, const double* const* G_list, const double* const* colsum_list,
                      const double* coef, int32_t nterm, const float* shift, int64_t n, int32_t p, double* C_out,
                      double* mean_out, void* stream);

/* Top-k eigenpairs of symmetric C (fp64 subspace iteration + Rayleigh-Ritz,
 * Jacobi on the projected block) and the tail moments
 *   theta[m-1] = Σ_{i>k} λ_i^m  (m = 1..3, utils/SIMCA.py:189-191, 203-204, 226-227)
 * computed from the deflated matrix (I-VVᵀ)C(I-VVᵀ) (traces, no full spectrum).
 * theta_mode: 0 none, 1 θ1..θ2, 2 θ1..θ3.
 * evals_out [dev] k (descending), evecs_out [dev] k×p rows = loadings with the
 * sklearn svd_flip sign (max-|entry| positive, extmath.py:895-953),
 * theta_out [dev] 3, iters_out [host, nullable].  Returns OCM_ERR_NOCONV if
 * the residual tolerance was not met within max_iter (outputs still valid).
 * Any 1 ≤ k ≤ p: the block is k plus oversampling; beyond 64 columns the
 * block's b×b Cholesky and Rayleigh–Ritz problems are solved on the host in
 * fp64 (the p×b products stay on the GPU). */
int ocm_eig_topk(ocm_ctx* ctx, const double* C, int32_t p, int32_t k, double tol, int32_t max_iter,
                 int32_t theta_mode, double* evals_out, double* evecs_out, double* theta_out, int32_t* iters_out,
                 void* stream);

/* Same, with the θ3 trace work split into `theta3_nslices` slices of which
 * this call computes slice `theta3_slice` only: theta_out[2] is then that
 * slice's partial sum and the caller sums the partials of every slice (the
 * ranks of a row-sharded fit each take one slice and all-reduce θ3;
 * SURVEY.md §8e).  theta_out[0..1] and all other outputs are complete on every
 * slice.  ocm_eig_topk is the call with (0, 1). */
int ocm_eig_topk_ex(ocm_ctx* ctx, const double* C, int32_t p, int32_t k, double tol, int32_t max_iter,
                    int32_t theta_mode, int32_t theta3_slice, int32_t theta3_nslices, double* evals_out,
                    double* evecs_out, double* theta_out, int32_t* iters_out, void* stream);
/* ocm_eig_topk_ex plus inv_out [dev] k = 1/λ with np.linalg.pinv's cutoff (|λ| ≤ rcond·max|λ| → 0), the
 * diagonal of pinv(cov(T)) that ocm_inv_evals_f64 forms (utils/SIMCA.py:69), queued inside the call so the
 * fit-set scoring can follow the eigensolve without another launch from the host. */
int ocm_eig_topk_ex2(ocm_ctx* ctx, const double* C, int32_t p, int32_t k, double tol, int32_t max_iter,
                     int32_t theta_mode, int32_t theta3_slice, int32_t theta3_nslices, double* evals_out,
                     double* evecs_out, double* theta_out, int32_t* iters_out, double rcond, double* inv_out,
                     void* stream);

/* ---- row-sharded fit: one all-reduce of packed moments ----
 * ocm_gram_pack turns a rank's shifted Gram (G, colsum about `shift`, n rows,
 * as ocm_gram_f32 returns them) into its moments about zero, packed
 *   packed_out[0 .. p(p+1)/2)      upper triangle (row-major) of
 *                                  G + s·csᵀ + cs·sᵀ + n·s·sᵀ  (Σ x xᵀ)
 *   packed_out[p(p+1)/2 .. +p)     cs + n·s                    (Σ x)
 *   packed_out[p(p+1)/2 + p]       n
 * so that a plain sum over ranks (one RCCL all-reduce of p(p+1)/2 + p + 1
 * doubles) gives the moments of all rows whatever shift each rank used.
 * ocm_cov_from_packed then forms μ = Σx/n and C = (Σ x xᵀ − n·μμᵀ)/(n−1)
 * (np.cov / sklearn explained_variance_, utils/SIMCA.py:64-66 →
 * _pca.py:584) with n read from the buffer on the device.  [dev] all. */
int ocm_gram_pack(ocm_ctx* ctx, const double* G, const double* colsum, const float* shift, int64_t n, int32_t p,
                  double* packed_out, void* stream);
int ocm_cov_from_packed(ocm_ctx* ctx, const double* packed, int32_t p, double* C_out, double* mean_out,
                        void* stream);

/* Symmetric pseudo-inverse (eigenvalue cutoff rcond·λmax) of a small d×d
 * fp64 matrix, d ≤ 64 (np.linalg.pinv(np.cov(...)) at utils/SIMCA.py:69,
 * VAE_SIMCA.py:247-248, utils/final_vaesimca.py:430-434).  [dev] in/out. */
int ocm_sym_pinv_f64(ocm_ctx* ctx, const double* A, int32_t d, double rcond, double* out, void* stream);

/* diag(pinv(cov(T))) on the eigenbasis, cov(T) = diag(λ): out_i = 1/λ_i
 * where |λ_i| > rcond·max|λ|, else 0 (np.linalg.pinv's cutoff, rcond 1e-15,
 * utils/SIMCA.py:69).  One launch in place of the host-issued elementwise
 * ops of the fit.  [dev] evals / out (k doubles, may alias).  ABI 9. */
int ocm_inv_evals_f64(ocm_ctx* ctx, const double* evals, int32_t k, double rcond, double* out, void* stream);

/* Fused scoring of float32 spectra (utils/SIMCA.py:65-71 fit, 104-107
 * transform, 127-130 predict):  y = x - mu; t = P·y (k); Q = ‖y − Pᵀt‖²;
 * T2 = tᵀ·A·t.  FP32 MFMA projection + explicit residual (first-order
 * insensitive to rounding in t).  P [dev] k×p float64 row-major with orthonormal rows
 * (ldp = p), mu [dev] p doubles, A [dev] k×k doubles.
 * Outputs (all nullable, [dev]): T_out m×k float32,
 * T2_out m doubles, Q_out m floats.  If dec != NULL [host] the decision is
 * fused: accept_out[r·accept_stride] = 1.0/0.0 (float64, the reference's
 * predictions[:, i] column).  stats_out [dev, nullable] 4 doubles
 * = {ΣT2, ΣT2², ΣQ, ΣQ²} (chi2pom moments).  k ≤ 64. */
int ocm_score_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                  const double* P, const double* mu, const double* A, int32_t k, float* T_out, double* T2_out,
                  float* Q_out, const ocm_decision* dec, double* accept_out, int64_t accept_stride,
                  double* stats_out, void* stream);

/* Same with A = diag(a_diag) (a_diag [dev] k doubles) — the SIMCA case: the
 * scores are on the eigenbasis, so invcovT = pinv(cov(T)) = diag(1/λ)
 * (utils/SIMCA.py:69).  For p ∈ {256, 512, 1024, 2048}, k ≤ 20 and 16-B
 * aligned X / ldx this runs k_score_1p, which reads every row of X from HBM
 * once (the row tile stays in registers between the projection and the
 * residual); other shapes take the two-sweep kernel of ocm_score_f32.
 * Arguments and outputs as ocm_score_f32. */
int ocm_score_f32_diag(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                       const double* P, const double* mu, const double* a_diag, int32_t k, float* T_out,
                       double* T2_out, float* Q_out, const ocm_decision* dec, double* accept_out,
                       int64_t accept_stride, double* stats_out, void* stream);

/* Reduced distances and decision from stored T2/Q (utils/SIMCA.py:76-81,
 * 109-114, 131-145).  Outputs nullable [dev]: t2red, qred, dred (m doubles),
 * accept (m doubles 0/1 at stride accept_stride). */
int ocm_decide(ocm_ctx* ctx, const double* T2, const float* Q, int64_t m, const ocm_decision* dec,
               double* t2red_out, double* qred_out, double* dred_out, double* accept_out, int64_t accept_stride,
               void* stream);

/* q_i = Σ_j (x_ij - xhat_ij)² (fp64 accumulation) for a VAE reconstruction
 * (vae_model.py:164, utils/final_vaesimca.py:425,492), the latent round-trip Q
 * (VAE_SIMCA.py:256-259, 365-366) and the Euclidean latent distance h about a
 * stored mean (utils/final_vaesimca.py:510-512: ldxh = 0 broadcasts one xhat
 * row).  x [dev] m×p float32 (ldx), xhat [dev] (ldxh), q_out [dev] m floats. */
int ocm_rowsq_residual_f32(ocm_ctx* ctx, const float* x, int64_t ldx, const float* xhat, int64_t ldxh, int64_t m,
                           int32_t p, float* q_out, void* stream);

/* q_i = Σ_j (s(x_ij) − s(xhat_ij))², s(v) = clamp((v − min_j x_ij)/(max_j x_ij − min_j x_ij + eps), 0, 1):
 * the per-sample min–max scaled reconstruction residual that
 * utils/final_vaesimca.py:417-423 (calibration Q threshold) and :484-490
 * (test Q) use for BCE-trained networks (eps = 1e-8 there).  Scaling in
 * float32 in the reference's order, f64 sum.  x, xhat [dev] m×p float32
 * (ldx, ldxh ≥ p), q_out [dev] m floats. */
int ocm_rowsq_minmax_f32(ocm_ctx* ctx, const float* x, int64_t ldx, const float* xhat, int64_t ldxh, int64_t m,
                         int32_t p, float eps, float* q_out, void* stream);

/* b[i] = (float)a[i] — loadings / mean handed to the float32 scoring kernel. */
int ocm_cast_f64_f32(ocm_ctx* ctx, const double* a, int64_t n, float* b, void* stream);

/* np.percentile(v, pct) with linear interpolation (utils/SIMCA.py:160,187;
 * VAE_SIMCA.py:285,305; utils/final_vaesimca.py:436-437) by radix select.
 * dtype: 0 = float64, 1 = float32.  v [dev] n values (no NaN);
 * out [host] 1 double. */
int ocm_percentile(ocm_ctx* ctx, const void* v, int32_t dtype, int64_t n, double pct, double* out, void* stream);

/* One radix-select pass (for multi-rank percentiles: callers all-reduce the
 * histogram between passes).  Counts values whose order key matches
 * `prefix` on the bits above `shift + 8`, binned by the 8 bits at `shift`.
 * hist_out [dev] 256 uint64 (overwritten). */
int ocm_radix_hist(ocm_ctx* ctx, const void* v, int32_t dtype, int64_t n, uint64_t prefix, int32_t shift,
                   uint64_t* hist_out, void* stream);

/* ---- class-wise cross-validation fold engine (utils/CVSIMCA.py:103-269) ----
 * One Gram pass gives every fold's Gram (segments), train Gram = total − fold;
 * one eigensolve per fold at LV_max; each LV ≤ LV_max reuses it through
 *   T²_LV = Σ_{j<LV} t_j²/λ_j,   Q_LV = Q_{LVmax} + Σ_{LV≤j<LVmax} t_j².   */

/* G_out = Σ_t coef[t]·G_list[t] (p×p), colsum_out = Σ_t coef[t]·colsum_list[t]
 * (either output nullable; colsum_list nullable).  G_out may alias G_list[0]
 * only.  G_list/colsum_list/coef [host] arrays of nterm device pointers/values. */
int ocm_gram_combine(ocm_ctx* ctx, const double* const* G_list, const double* const* colsum_list,
                     const double* coef, int32_t nterm, int32_t p, double* G_out, double* colsum_out, void* stream);

/* Per-LV T² and Q of m rows from their LV_max scores (training rows of a fold:
 * the perc / chi2pom limit statistics, utils/SIMCA.py:157-159, 172-181, 186-187,
 * 211-216).  T [dev] m×k float32 (from ocm_score_f32, k = LV_max), Q [dev] m
 * float32, inv_evals [dev] k doubles (diag of invcovT), lvs [host] nlv values
 * in [1, k].  Outputs nullable [dev]: T2_out nlv×m doubles, Q_out nlv×m floats,
 * stats_out nlv×4 doubles {ΣT², ΣT²², ΣQ, ΣQ²}.  k, nlv ≤ 64. */
int ocm_cv_prefix(ocm_ctx* ctx, const float* T, int64_t m, int32_t k, const float* Q, const double* inv_evals,
                  const int32_t* lvs, int32_t nlv, double* T2_out, float* Q_out, double* stats_out, void* stream);

/* One decision configuration of the CV sweep: LV components, a decision
 * type and its scales / critical distance (as ocm_decision). */
typedef struct ocm_cv_config {
  int32_t lv;
  int32_t type;
  double t2_scale;
  double q_scale;
  double dlim;
} ocm_cv_config;
#define OCM_CV_MAXCFG 1024

/* Confusion counts of every configuration over the test rows of a fold
 * (utils/CVSIMCA.py:186-199 → utils/SIMCA.py:238-266): rows < m_split are the
 * held-out target rows, the rest the other-class rows.  positive [dev] m
 * bytes (y_true == class_index).  counts_out [dev] ncfg×2×4 uint64
 * {TP, TN, FP, FN} per (config, part).  accept_out [dev, nullable] ncfg×m
 * doubles 0/1 (pooled predictions).  cfg [host]. */
int ocm_cv_counts(ocm_ctx* ctx, const float* T, int64_t m, int32_t k, const float* Q, const double* inv_evals,
                  const uint8_t* positive, int64_t m_split, const ocm_cv_config* cfg, int32_t ncfg,
                  uint64_t* counts_out, double* accept_out, void* stream);

/* Confusion counts of one class column of a prediction matrix
 * (utils/SIMCA.py:238-245, called from predict(X, y_true) at :146-152):
 * accept [dev] m doubles 0/1 at stride accept_stride (the column written by
 * ocm_score_f32*'s fused decision), positive [dev] m bytes (y_true == class).
 * counts_out [dev] 4 uint64 {TP, TN, FP, FN}. */
int ocm_confusion_counts(ocm_ctx* ctx, const double* accept, int64_t m, int64_t accept_stride,
                         const uint8_t* positive, uint64_t* counts_out, void* stream);

/* ---- spectral preprocessing ----
 * SNV x ← (x − mean_row)/(std_row + 1e-8) (np.std ddof 0; simca_nuts.py:47-49,
 * utils/data_utils.py:57) when snv != 0, then, when window > 0, the
 * Savitzky–Golay filter scipy.signal.savgol_filter(x, window, polyorder,
 * deriv, delta, axis=1, mode='interp') (simca_nuts.py:51,
 * simca_new_cheese.py:37-38) given as taps [host] (window + 2·(window/2)·window
 * doubles: interior correlation taps, then the left and right edge rows; see
 * ocm/preprocess.py savgol_taps).  One HBM pass per row.  X, out [dev] m×p
 * float32 (ldx, ldo; out may not alias X).  window odd ≤ 63, p ≤ 12288. */
int ocm_snv_savgol_f32(ocm_ctx* ctx, const float* X, int64_t ldx, int64_t m, int32_t p, int32_t snv,
                       int32_t window, const double* taps, float* out, int64_t ldo, void* stream);

/* ---- dense symmetric eigensolver (fp64) ----
 * evals_out [dev] all p eigenvalues of C (p×p fp64, symmetric) in descending order; when k > 0,
 * evecs_out [dev] k×p the leading k eigenvectors as rows (svd_flip sign: largest |entry| positive).
 * Householder tridiagonalisation on the GPU, QL eigenvalues and inverse-iteration vectors of the
 * tridiagonal on the host, back-transformation on the GPU.  Replaces the full spectrum of the
 * reference's SVD (utils/SIMCA.py:64-66,88 `eigs_all`; sklearn _pca.py:584-598) and is the fallback of
 * ocm_eig_topk when its subspace iteration does not converge.  Synchronises the stream.
 * Limits: 1 ≤ p ≤ 16384 for eigenvalues only (k = 0); p ≤ 12288 when k > 0 (checked before any
 * work).  OCM_ERR_NOCONV if the implicit QL of the tridiagonal does not converge. */
int ocm_eigh_f64(ocm_ctx* ctx, const double* C, int32_t p, double* evals_out, int32_t k, double* evecs_out,
                 void* stream);

/* ---- preprocessing in the load path (lazy view) ----
 * The drivers run SNV then Savitzky–Golay right before SIMCA
 * (simca_nuts.py:47-52, simca_new_cheese.py:37-38, utils/data_utils.py:57-61).
 * An ocm_prep describes that transform and the *_prep kernels apply it to each
 * row as they load it, so the preprocessed matrix X′ never exists in HBM.
 * Row r, column j, float32 arithmetic identical in every kernel (the Gram,
 * the scores and ocm_prep_apply_f32 see bit-identical values):
 *   u_c = x_c − m_r when snv and deriv == 0, else u_c = x_c
 *   window == 0:                 a = u_j
 *   interior, odd deriv:         a = Σ_{t=1..H} c_{H+t}·(u_{j+t} − u_{j−t})   (c antisymmetric)
 *   interior, deriv 0:           a = c_H·u_j + Σ_{t=1..H} c_{H+t}·(u_{j+t} + u_{j−t})
 *   interior, even deriv ≥ 2:    a = Σ_{t=1..H} c_{H+t}·((u_{j+t} − u_j) + (u_{j−t} − u_j))
 *   edges (j < H or j ≥ p − H):  a = Σ_t e_{j,t}·(u_{s+t} − [deriv ≥ 1]·u_j), s = 0 or p − window
 *   y_j = a·s_r when snv, else a
 * (fmaf chains in t order from 0; H = window/2; (m_r, s_r) = (mean_r,
 * 1/(std_r + 1e-8)) from ocm_prep_rowstats_f32).  Savitzky–Golay maps a
 * constant to 0 for deriv ≥ 1 and to itself for deriv 0, so y = SG(SNV(x))
 * up to float32 rounding, with the row mean cancelling exactly in the
 * drivers' deriv-1 filters; differences of neighbouring samples keep a large
 * baseline from costing precision. */
typedef struct ocm_prep {
  int32_t window;        /* 0 (SNV only) or odd 3..31 */
  int32_t deriv;         /* Savitzky–Golay derivative order (0 when window == 0) */
  int32_t snv;           /* 1: apply the SNV row statistics */
  int32_t pad_;
  const float* taps;     /* [dev] window + 2·H·window floats: interior c, left-edge rows, right-edge rows
                            (ocm/preprocess.py savgol_taps); NULL when window == 0 */
  const float* rowstat;  /* [dev] (m_r, s_r) per row of X, indexed like X (gather lists index it too);
                            NULL when snv == 0 */
} ocm_prep;

/* rowstat_out [dev] m×2 floats: m_r = mean (fp64, rounded), s_r = 1/(std_r + 1e-8) (np.std ddof 0)
 * of each row of X — the one read-only pre-pass the SNV needs. */
int ocm_prep_rowstats_f32(ocm_ctx* ctx, const float* X, int64_t ldx, int64_t m, int32_t p, float* rowstat_out,
                          void* stream);
/* out [dev] m×p (ldo) = the preprocessed rows X[rows[i]] (rows nullable): the materialised view, for
 * shapes and modes the fused kernels do not cover and for tests. */
int ocm_prep_apply_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                       const ocm_prep* prep, float* out, int64_t ldo, void* stream);
/* ocm_colmean_f32 / ocm_gram_f32_ex / ocm_score_f32_diag on the preprocessed rows, read raw from X.
 * The default i8×3 Gram applies the transform in its quantiser (halo columns staged through LDS) and
 * k_score_1p applies it to each row tile in registers as the tile arrives (p ∈ {256, 512, 1024, 2048},
 * window ∈ {0, 5, 15}, p % 4 == 0); other shapes, windows and Gram modes materialise the preprocessed
 * rows in a temporary device buffer first. */
int ocm_colmean_f32_prep(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                         const ocm_prep* prep, double* mean_out, void* stream);
int ocm_gram_f32_prep(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                      const float* shift, const int64_t* seg_offsets, int32_t nseg, int32_t mode,
                      int64_t chunk_rows, const ocm_prep* prep, double* G_out, double* colsum_out, void* stream);
/* Write-through (round 5): ocm_gram_f32_prep (i8×3, all n rows of X, no gather list) whose quantiser
 * also writes the preprocessed rows to xout [dev] n×p (ldo % 4 == 0, 16-B aligned) as it forms them:
 * the stencil runs once, in the Gram's read of X, and the consumers after the Gram (scoring of the fit
 * and predict sets) read X′ with the plain kernels.  The values are those of ocm_prep_apply_f32 bit for
 * bit.  Shapes and transforms the fused quantiser does not cover run the eager pass into xout, then the
 * Gram on it. */
int ocm_gram_f32_prep_write(ocm_ctx* ctx, const float* X, int64_t ldx, int64_t n, int32_t p, const float* shift,
                            const int64_t* seg_offsets, int32_t nseg, int64_t chunk_rows, const ocm_prep* prep,
                            double* G_out, double* colsum_out, float* xout, int64_t ldo, void* stream);
/* Number of times this context materialised a lazy view (the fallback paths above), for tests and
 * diagnostics: 0 after any call on the fused paths. */
int ocm_prep_materialised(ocm_ctx* ctx, int64_t* count_out);
/* How many Rayleigh–Ritz tests of ocm_eig_topk* this context ran twice: the
 * test fused into the Jacobi takes S from a side stream in flight and gives up
 * after ≈ 1 s (kernels serialised, or the side stream not scheduled); the host
 * then runs the Jacobi + test again behind S's event (a diagnostic counter). */
int ocm_eig_test_reruns(ocm_ctx* ctx, int64_t* count_out);
int ocm_score_f32_diag_prep(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                            const ocm_prep* prep, const double* P, const double* mu, const double* a_diag, int32_t k,
                            float* T_out, double* T2_out, float* Q_out, const ocm_decision* dec,
                            double* accept_out, int64_t accept_stride, double* stats_out, void* stream);

/* ---- float64 spectra: the PCA precision follows the input dtype ----
 * The reference's PCA runs in the input dtype (utils/SIMCA.py:64-66 →
 * sklearn _pca.py:544-584 on float64 X), and its scores, residuals and Q are
 * then float64 (utils/SIMCA.py:65-71, 104-107, 127-130).  X [dev] n×p float64
 * (ldx elements); rows as above.
 *
 * ocm_colmean_f64: column mean of the first n processed rows (fp64).
 * ocm_gram_f64: per-segment shifted Gram Σ (x − s)(x − s)ᵀ and Σ (x − s) on
 *   fp64 MFMA (v_mfma_f64_16x16x4f64), no digit split; arguments and outputs as
 *   ocm_gram_f32 (the float shift is exact in fp64), so ocm_cov_from_gram /
 *   ocm_gram_pack apply unchanged.
 * ocm_score_f64_diag: t = P·(x − μ), T² = Σ t²·a_diag, and Q = ‖(x − μ) − Pᵀt‖²
 *   as the explicit residual of the reconstruction X̂ = T·P + μ
 *   (utils/SIMCA.py:67-68, 71), fused decision and the moments, as
 *   ocm_score_f32_diag; T_out m×k float64 (nullable), Q_out m float64; any
 *   1 ≤ k ≤ p (component blocks of 64 beyond that).
 * ocm_decide_f64: ocm_decide with float64 Q. */
int ocm_colmean_f64(ocm_ctx* ctx, const double* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                    double* mean_out, void* stream);
int ocm_gram_f64(ocm_ctx* ctx, const double* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                 const float* shift, const int64_t* seg_offsets, int32_t nseg, double* G_out, double* colsum_out,
                 void* stream);
int ocm_score_f64_diag(ocm_ctx* ctx, const double* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                       const double* P, const double* mu, const double* a_diag, int32_t k, double* T_out,
                       double* T2_out, double* Q_out, const ocm_decision* dec, double* accept_out,
                       int64_t accept_stride, double* stats_out, void* stream);
int ocm_decide_f64(ocm_ctx* ctx, const double* T2, const double* Q, int64_t m, const ocm_decision* dec,
                   double* t2red_out, double* qred_out, double* dred_out, double* accept_out, int64_t accept_stride,
                   void* stream);

/* ---- VAE network support (vae_model.py:37-81, BatchNorm1d in train mode) ----
 * Training-mode batch norm over (N, C, L) contiguous activations, bf16 or f32,
 * statistics per channel over N·L < 2³¹ (torch.nn.functional.batch_norm semantics:
 * biased variance normalises, unbiased variance feeds running_var with
 * `momentum`).  Replaces the MIOpen spatial BN the reference's nn.BatchNorm1d
 * lowers to (vae_model.py:45-47, 75-77).  running_mean / running_var may both
 * be NULL (no update); gamma / beta may be NULL (affine=False); num_batches_tracked
 * [nullable] is incremented by one (nn.BatchNorm1d's counter).  scratch [dev]
 * ocm_bn_scratch_bytes(C) bytes of caller-owned memory that stays put while a
 * captured hipGraph replays the launches, ZERO-FILLED BEFORE ITS FIRST USE and
 * then reused by every call of that layer (forward and backward): it ends in
 * per-channel completion counters — the last of a channel's reduction
 * workgroups forms the statistics, one launch per direction fewer — which
 * every call leaves zero.  Calls sharing one scratch must be stream-ordered.
 * All work is stream-ordered (graph-capturable). */
#define OCM_DTYPE_F32 0
#define OCM_DTYPE_BF16 1
/* act: OCM_ACT_ELU fuses the ELU (α = 1) that follows every batch norm of the
 * VAE (vae_model.py:45-49, 75-79): y = ELU(BN(x)) forward; the backward takes
 * the gradient of the ELU output and that output y (dz = dy·(y > 0 ? 1 : y + 1)). */
#define OCM_ACT_NONE 0
#define OCM_ACT_ELU 1
size_t ocm_bn_scratch_bytes(int32_t C);
int ocm_bn_fwd_train(ocm_ctx* ctx, int32_t dtype, const void* x, int32_t N, int32_t C, int32_t L,
                     const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
                     float* running_var, int64_t* num_batches_tracked, int32_t act, void* y, float* save_mean,
                     float* save_invstd, void* scratch, void* stream);
/* Eval-mode BatchNorm1d (running statistics, vae_model.py:45-47 in model.eval(), the
 * latent encoding of utils/final_vaesimca.py:406-442): y = (x − rm)·γ/√(rv + ε) + β,
 * then the fused ELU with act = OCM_ACT_ELU; gamma / beta nullable.  No scratch,
 * any N (one flat grid).  ABI 9. */
int ocm_bn_fwd_eval(ocm_ctx* ctx, int32_t dtype, const void* x, int32_t N, int32_t C, int32_t L,
                    const float* running_mean, const float* running_var, float eps, const float* gamma,
                    const float* beta, int32_t act, void* y, void* stream);
/* dx = γ·invstd·(dz − mean(dz) − x̂·mean(dz·x̂)), dz = dy (act NONE) or the ELU's input gradient;
 * dgamma = Σ dz·x̂, dbeta = Σ dz (either may be NULL); y [act ELU] the forward's output. */
int ocm_bn_bwd(ocm_ctx* ctx, int32_t dtype, const void* x, const void* dy, int32_t N, int32_t C, int32_t L,
               const float* gamma, const float* save_mean, const float* save_invstd, int32_t act, const void* y,
               void* dx, float* dgamma, float* dbeta, void* scratch, void* stream);
/* ocm_bn_fused_timeouts (ABI 12): with OCM_BN_FUSED=1 in the environment (an experiment, off by default:
 * slower on the C4 step), training-mode ocm_bn_fwd_train / ocm_bn_bwd run as ONE launch where the
 * layout allows (L % 8 = 0, 16-byte aligned tensors, the grid co-resident on the device): each workgroup
 * keeps its share of the channel in registers while the channel's last workgroup forms the statistics,
 * the others waiting on an epoch word in the scratch.  A wait that exceeds ≈ 1 s gives up rather than
 * hang (its outputs are then wrong) and is counted (count_out: the process total). */
int ocm_bn_fused_timeouts(int64_t* count_out);

/* ---- VAE narrow convolutions (vae_model.py:37-81: Conv1d / ConvTranspose1d,
 * 1-12 channels, kernel 7, stride 1 or 2; the layers nn.Conv1d /
 * nn.ConvTranspose1d lower to MIOpen in the reference) ----
 * Activations (B, C, L) contiguous, float32 or bfloat16 (dtype_*: OCM_DTYPE_*);
 * weights, bias, gradients float32; float32 accumulation.  Stream-ordered,
 * graph-capturable (scratch is caller-owned).
 *
 * ocm_conv1d, mode OCM_CONV_DOWN:  y[b][o][l] = bias[o] + Σ_i Σ_t w[o][i][t]·x[b][i][l·s + t − pad]
 *   (Conv1d forward, w [O][I][K]; ConvTranspose1d input gradient with w its [I][O][K] weight, x = dy);
 * mode OCM_CONV_UP:  y[b][o][j] = bias[o] + Σ_i Σ_t w[i][o][t]·x[b][i][(j + pad − t)/s] over the
 *   terms where s divides j + pad − t (ConvTranspose1d forward, w [I][O][K]; Conv1d input gradient with
 *   w its [O][I][K] weight read as [I][O][K] of dy's channels).  bias nullable; I ≤ 64, K ≤ 15.
 * ocm_conv1d_wgrad: G[o][i][t] = Σ_b Σ_l P[b][o][l]·Q[b][i][l·s + t − pad], written [O][I][K]
 *   (Conv1d: P = dy, Q = x → its [O][I][K] weight gradient; ConvTranspose1d: P = x, Q = dy → its
 *   [I][O][K] weight gradient); psum_out [nullable] = Σ_b Σ_l P[b][o][l] (Conv1d's bias gradient).
 *   scratch ≥ ocm_conv1d_scratch_bytes(O, I, K), zero-filled before its first use and reused (it
 *   starts with completion counters that every call leaves zero: the last partial workgroup of
 *   an output group sums the partials — one launch); fixed-order two-stage sums (deterministic).
 * ocm_conv1d_wgrad_qsum (ABI 12): the same G, and qsum_out[i] = Σ_b Σ_j Q[b][i][j] (ConvTranspose1d's bias
 *   gradient, Q = dy) in the same launch when Lq = s·Lp and pad + s ≤ K (bf16 operands, the matrix-core
 *   path: a row of ones in P), else by ocm_chan_sum after it.  scratch as ocm_conv1d_wgrad's.
 * ocm_chan_sum: out[c] = Σ_b Σ_l v[b][c][l] (the bias gradient), C ≤ 284; scratch as above with
 *   O·I·K ≥ C (the same zero-filled, reused memory as the layer's wgrad may serve both). */
#define OCM_CONV_DOWN 0
#define OCM_CONV_UP 1
size_t ocm_conv1d_scratch_bytes(int32_t O, int32_t I, int32_t K);
int ocm_conv1d(ocm_ctx* ctx, int32_t mode, int32_t dtype_in, const void* x, int32_t B, int32_t I, int32_t Lin,
               const float* w, const float* bias, int32_t O, int32_t Lout, int32_t K, int32_t stride, int32_t pad,
               int32_t dtype_out, void* y, void* stream);
int ocm_conv1d_wgrad(ocm_ctx* ctx, int32_t dtype_p, const void* P, int32_t O, int32_t Lp, int32_t dtype_q,
                     const void* Q, int32_t I, int32_t Lq, int32_t B, int32_t K, int32_t stride, int32_t pad,
                     float* G_out, float* psum_out, void* scratch, void* stream);
int ocm_conv1d_wgrad_qsum(ocm_ctx* ctx, int32_t dtype_p, const void* P, int32_t O, int32_t Lp, int32_t dtype_q,
                          const void* Q, int32_t I, int32_t Lq, int32_t B, int32_t K, int32_t stride, int32_t pad,
                          float* G_out, float* qsum_out, void* scratch, void* stream);
int ocm_chan_sum(ocm_ctx* ctx, int32_t dtype, const void* v, int32_t B, int32_t C, int32_t L, float* out,
                 void* scratch, void* stream);

/* ---- the VAE training step's small tensors, fused (vae_model.py:136-158, vae_bce_nut.py:178-203,
 * utils/final_vaesimca.py:198-224): the graphed step is bound by its kernel count, so the
 * reparameterisation + KL, the de-standardisation + reconstruction term + total, their backward
 * passes and Adam each take one launch.  Activations in dtype (OCM_DTYPE_*), sums fp64 with
 * fixed-order partials, losses float32; graph-capturable (scratch caller-owned,
 * ocm_vae_scratch_bytes(B) bytes, zeroed once before first use).
 *
 * ocm_vae_bottleneck_fwd: z = μ + ε·exp(½·logσ²); kl_out = −½·mean_B Σ_d (1 + logσ² − μ² − exp(logσ²))
 *   (vae_model.py:150-152, reparameterize :124-126).  μ, logσ², ε, z [dev] B×d, B·d ≤ 2²⁰; scratch
 *   [dev] ocm_vae_bottleneck_scratch_bytes(), zero-filled once before first use (its counters are
 *   left zero).
 * ocm_vae_bottleneck_bwd: dμ = dz + dkl·μ/B, dlogσ² = dz·ε·½exp(½logσ²) − ½·dkl·(1 − exp(logσ²))/B
 *   (dz or dkl may be NULL: no gradient from that output).
 * ocm_vae_recon_fwd: x̂ = xs·std + mean (forward's de-standardisation, vae_model.py:130-134); kind
 *   OCM_VAE_LOSS_BCE: mean BCE-with-logits(x̂, clamp((x − min_x)/(max_x − min_x + eps), 0, 1)) per
 *   sample min / max (vae_model.py:153-156); OCM_VAE_LOSS_MSE: mean (x̂ − x)² (final_vaesimca.py:208);
 *   out2 [dev] {recon + β·kl, recon} (kl [dev] nullable: 0); gxs_out [dev] B×L f32 = d recon / d xs.
 * ocm_vae_recon_bwd: dxs = dtotal·gxs (n values, written in dtype), dkl_out = β·dtotal (nullable).
 * ocm_adam_step: torch.optim.Adam (L2 weight_decay, no amsgrad) over `ntensors` tensors of
 *   `table` [dev] (offsets: prefix of numel, total = Σ numel); step [dev] f32 counter, advanced by
 *   one per call (bias corrections 1 − βᵗ); scratch [dev] ocm_vae_scratch_bytes(4096) bytes,
 *   zero-filled once (completion counters, left zero). */
#define OCM_VAE_LOSS_BCE 0
#define OCM_VAE_LOSS_MSE 1
typedef struct ocm_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t offset;
  int64_t numel;
} ocm_adam_tensor;
size_t ocm_vae_scratch_bytes(int32_t B);
size_t ocm_vae_bottleneck_scratch_bytes(void);
int ocm_vae_bottleneck_fwd(ocm_ctx* ctx, int32_t dtype, const void* mu, const void* logvar, const void* eps, int32_t B,
                           int32_t d, void* z_out, float* kl_out, void* scratch, void* stream);
int ocm_vae_bottleneck_bwd(ocm_ctx* ctx, int32_t dtype, const void* dz, const float* dkl, const void* mu,
                           const void* logvar, const void* eps, int32_t B, int32_t d, void* dmu_out, void* dlogvar_out,
                           void* stream);
/* ocm_vae_bottleneck_fwd_ld / _bwd_ld (ABI 12): the same with μ, logσ² (and dμ, dlogσ²) as rows of stride
 * ld ≥ d — ld = 2d, logvar = mu + d: the packed B×2d output of one [fc_mu; fc_logvar] product
 * (vae_model.py:81-82), read and written in place; ε, z, dz stay B×d. */
int ocm_vae_bottleneck_fwd_ld(ocm_ctx* ctx, int32_t dtype, const void* mu, const void* logvar, int32_t ld,
                              const void* eps, int32_t B, int32_t d, void* z_out, float* kl_out, void* scratch,
                              void* stream);
int ocm_vae_bottleneck_bwd_ld(ocm_ctx* ctx, int32_t dtype, const void* dz, const float* dkl, const void* mu,
                              const void* logvar, int32_t ld, const void* eps, int32_t B, int32_t d, void* dmu_out,
                              void* dlogvar_out, void* stream);
int ocm_vae_recon_fwd(ocm_ctx* ctx, int32_t kind, const float* x, int32_t dtype, const void* xs, int32_t B, int32_t L,
                      const float* mean, const float* std, float eps, const float* kl, float beta, float* gxs_out,
                      float* out2, void* scratch, void* stream);
int ocm_vae_recon_bwd(ocm_ctx* ctx, const float* dtotal, const float* gxs, int64_t n, int32_t dtype, void* dxs_out,
                      float beta, float* dkl_out, void* stream);
int ocm_adam_step(ocm_ctx* ctx, const ocm_adam_tensor* table, int32_t ntensors, int64_t total, float* step, float lr,
                  float beta1, float beta2, float eps, float weight_decay, void* scratch, void* stream);
/* ocm_cast_multi: dst[k] = src[k] converted (float32 ↔ bfloat16, round to nearest even) for n ≤ 32
 *   tensors of numel[k] elements in one launch (src / dst / numel: HOST arrays of device pointers;
 *   the pointers travel as kernel arguments, so a captured graph replays them).  The VAE step casts
 *   its Linear weights to bf16 once per step, and their bf16 gradients back, in one launch each.
 * ocm_vae_standardise: out = (x − mean) / std per column of a B×L float32 batch, in dtype
 *   (vae_model.py:128-129 standardises the spectra before the encoder). */
int ocm_cast_multi(ocm_ctx* ctx, int32_t n, const void* const* src, int32_t src_dtype, void* const* dst,
                   int32_t dst_dtype, const int64_t* numel, void* stream);
int ocm_vae_standardise(ocm_ctx* ctx, const float* x, int32_t B, int32_t L, const float* mean, const float* std_,
                        int32_t dtype, void* out, void* stream);
/* ocm_vae_act_bias_bwd (ABI 11): the backward tail of a bf16 Linear layer (vae_model.py:80-84):
 *   act 1 (Linear → ELU): gy_out = g · elu'(y), y the pre-activation (torch's elu_backward, float32
 *   arithmetic rounded to bf16), and gbias_out[c] = Σ_r gy[r, c] (float32 over the rounded values,
 *   rounded to bf16); act 0 (Linear alone): gbias_out = Σ_r g[r, c], y / gy_out unused.
 *   g, y, gy_out [dev] B×N bf16 row-major, N a multiple of 8, 16-byte aligned; gbias_out [dev] N bf16.
 *   One launch instead of torch's elu_backward and sum-reduction kernels. */
int ocm_vae_act_bias_bwd(ocm_ctx* ctx, int32_t act, const void* g, const void* y, int32_t B, int32_t N, void* gy_out,
                         void* gbias_out, void* stream);
/* ocm_vae_linear_act (ABI 12): y = x·Wᵀ + b (bf16, float32 accumulation, rounded to bf16) and a = ELU(y) of
 * the rounded y (torch's expm1 form) in one launch, for the bottleneck's short-K Linear + ELU layers
 * (vae_model.py:83-84).  x M×K, W N×K, bias N (nullable), y_out / a_out M×N, all bf16 and row-major;
 * M, N multiples of 64, K ∈ {32, 64, 128, 256}; x and W 16-byte aligned. */
int ocm_vae_linear_act(ocm_ctx* ctx, const void* x, const void* W, const void* bias, int32_t M, int32_t N, int32_t K,
                       void* y_out, void* a_out, void* stream);
/* ocm_gemm_bf16_sk (ABI 11): C = A·B (+ bias) in bf16 with float32 accumulation, for the VAE bottleneck's
 *   long-K products (vae_model.py:80-84: fc[0]'s forward, fc_dec[3]'s input gradient), split over K in
 *   256-deep chunks: A [dev] M×K row-major; B [dev] N×K row-major when b_nk (a Linear weight, C = A·Bᵀ),
 *   else K×N row-major; bias [dev] N bf16 or NULL; C [dev] M×N row-major.  M, N multiples of 64, K of 256,
 *   16-byte aligned.  scratch [dev] ocm_gemm_bf16_sk_scratch_bytes(M, N, K) bytes (caller-owned, so a
 *   captured graph keeps it): float32 partial tiles, summed in chunk order by the second launch. */
size_t ocm_gemm_bf16_sk_scratch_bytes(int32_t M, int32_t N, int32_t K);
int ocm_gemm_bf16_sk(ocm_ctx* ctx, int32_t b_nk, const void* A, const void* B, const void* bias, int32_t M, int32_t N,
                     int32_t K, void* C, void* scratch, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OCM_H_ */
