/*
 * tpe_hip.h -- C ABI of the MI355X TPE suggest engine (libtpe_hip.so).
 *
 * The reference (hyperopt 0.2.4, /root/reference) is pure Python/numpy and
 * has no FFI of its own; its hot path is the per-label posterior evaluation
 * that `tpe.suggest` drives through `pyll.rec_eval` (hyperopt/tpe.py:942).
 * Each entry point below replaces one group of the numpy expressions on that
 * path and is what a binding of that path (ctypes / cffi / pybind) would
 * call.  The Python host layer `hyperopt_amd/_lib.py` binds these with
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - every pointer is a caller-owned DEVICE pointer unless marked "host";
 *   - `stream` is a hipStream_t passed as void* (0 = legacy default stream);
 *   - every call is asynchronous on `stream`, captures into a hipGraph,
 *     performs no allocation and no host synchronisation;
 *   - return value: 0 on success, a negative TPE_E* code otherwise; the text
 *     of the last error on the calling thread is tpe_last_error();
 *   - scores/log-densities are float64 on the ABI; `precision` (32 or 64)
 *     selects the arithmetic of the continuous scoring kernel only.
 */
#ifndef TPE_HIP_H
#define TPE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TPE_ABI_VERSION 22

enum {
  TPE_OK = 0,
  TPE_E_ARG = -1,        /* bad argument (null pointer, bad size/kind)      */
  TPE_E_LAUNCH = -2,     /* HIP launch / runtime error                      */
  TPE_E_UNSUPPORTED = -3 /* configuration outside what the kernels support  */
};

/* mixture families (hyperopt/tpe.py:79, 229; categorical tpe.py:60-73) */
enum { TPE_GMM1 = 0, TPE_LGMM1 = 1, TPE_CAT = 2 };

/* observation transform applied before the Parzen fit (tpe.py:506-572) */
enum { TPE_OBS_IDENTITY = 0, TPE_OBS_LOG = 1 };

/* job flags */
enum {
  TPE_F_LOW = 1,        /* lower bound present (tpe.py:93, 166)              */
  TPE_F_HIGH = 2,       /* upper bound present                               */
  TPE_F_QUANT = 4,      /* quantized (q is not None)                         */
  TPE_F_INJECTED = 8,   /* candidates read from `cand` instead of sampled    */
  TPE_F_DRAW32 = 16,    /* sampled quantized job: draw in fp32 (set only when
                           every lattice index |k| <= 2^12, so fp32 resolves a
                           slot to < 2^-11 of q)                              */
  TPE_F_LATTICE_READY = 32, /* lattice job: the caller has already set its
                           slot_first region [lat_off, lat_off + lat_n) to
                           all-ones and its `counts` entry to 0 (e.g. in the
                           level's upload); when every job of a
                           tpe_lattice_sample / tpe_lattice_compact call has
                           it, those calls skip their memsets               */
  /* (TPE_F_DRAW32 on an unquantized job: the fp32 candidate stream -- the
     table path's -- scored exactly by tpe_score_pruned64)                   */
};

/*
 * One Parzen-fit segment: the below- or above-set observations of one label.
 * Replaces `adaptive_parzen_normal` (tpe.py:399-467) and the observation
 * transforms of the ap_*_sampler functions (tpe.py:484-572).  Inputs are set
 * by the host; the kernel fills the outputs.  The fitted mixture has
 * n_obs + 1 components written at [comp_off, comp_off + n_obs + 1), sorted
 * by mean, exactly as the reference returns them.
 */
typedef struct tpe_seg {
  /* inputs */
  int64_t obs_off;      /* first observation in the obs pool                */
  int64_t comp_off;     /* first output component in the mixture pool       */
  int32_t n_obs;        /* observations in this segment (tid order)         */
  int32_t lf;           /* linear forgetting (tpe.py:380-392); 0 = off      */
  int32_t transform;    /* TPE_OBS_*                                         */
  int32_t family;       /* TPE_GMM1 / TPE_LGMM1 (coefficient layout)         */
  double floor;         /* log transform: log(max(obs, floor))              */
  double prior_weight, prior_mu, prior_sigma;
  double low, high;     /* truncation for p_accept (tpe.py:145-150)         */
  int32_t bounded;      /* 1 if low/high given                              */
  /* outputs */
  int32_t prior_pos;    /* index of the prior component in the sorted mix   */
  double p_accept;      /* sum w*(Phi(high)-Phi(low)), 1 if unbounded        */
  double cmax;          /* max_k log2-coefficient (fp32 scoring offset)      */
  double center;        /* fp32 scoring origin (float-rounded prior_mu)      */
  double lglob;         /* lower bound of log2(sum)-cmax over the support    */
  int32_t n_wide;       /* wide components (prior + sigma >= sigma_p/4)      */
  int32_t given;        /* 1: an explicit mixture (tpe_mixture_prepare): its
                           w / mu / sigma are the caller's, not fitted       */
} tpe_seg;

/*
 * One categorical segment (randint / pchoice / choice posterior,
 * tpe.py:578-615 with pyll/base.py:1053-1060).  counts are accumulated in
 * observation order, so they are bit-identical to np.bincount.
 */
typedef struct tpe_cat_seg {
  int64_t obs_off;      /* int64 observations (already offset-free)         */
  int64_t p_off;        /* first output probability                          */
  int32_t n_obs;
  int32_t n_cat;        /* K                                                 */
  int32_t lf;
  int32_t mode;         /* 0 randint: counts+pw ; 1 categorical: counts+K*pw*p */
  double prior_weight;
  int64_t prior_p_off;  /* mode 1: prior probabilities p in the p pool       */
} tpe_cat_seg;

/*
 * One label's scoring job.  For continuous labels below/above index two
 * tpe_seg entries; for categorical labels two tpe_cat_seg entries.
 * Candidates are either sampled in registers from the BELOW posterior with
 * Philox4x32-10 keyed by (key, global candidate index) -- so results do not
 * depend on how candidates are sharded over GPUs -- or injected (TPE_F_INJECTED).
 */
typedef struct tpe_job {
  int32_t family;       /* TPE_GMM1 / TPE_LGMM1 / TPE_CAT                    */
  int32_t flags;        /* TPE_F_*                                           */
  int32_t below, above; /* segment indices                                   */
  double low, high, q;  /* GMM1: x-space bounds; LGMM1: log-space bounds    */
  int64_t n_cand;       /* candidates scored by this call                   */
  int64_t cand_base;    /* global index of the first one (multi-GPU shard)  */
  int64_t cand_off;     /* TPE_F_INJECTED: first candidate in `cand`         */
  uint64_t key;         /* Philox key (seed mixed with label id)            */
  int64_t lat_off;      /* quantized: first lattice slot in the slot pool   */
  int64_t lat_kmin;     /* quantized: lattice index of slot 0               */
  int64_t lat_n;        /* quantized: number of slots; categorical: K (0 = unknown) */
  int64_t out_off;      /* optional per-candidate outputs: first element    */
  double bin_lo, bin_hi;/* sorted path: candidate coordinate range to bin    */
  int64_t sort_off;     /* sorted path: first slot in the sorted pool        */
  int64_t cnt_off;      /* sorted path: first element of the count matrix    */
  int64_t tbl_off;      /* table path: first cell of this job's cell table   */
  int64_t tbl_cap;      /* table path: cells allocated at tbl_off            */
} tpe_job;

/* best candidate of one label: np.argmax semantics (first max, NaN wins) */
typedef struct tpe_best {
  double score;         /* below_llik - above_llik of the winner            */
  int64_t index;        /* global candidate index of the winner (-1: none)  */
  double value;         /* candidate value (category index for TPE_CAT)     */
  int64_t n_scored;     /* candidates entered into the argmax               */
} tpe_best;

/* ---- Parzen posterior (adaptive_parzen_normal, tpe.py:399-467) ---------- */
/* obs: fp64 pool (n_obs_total); scratch: device workspace of
 * tpe_fit_scratch_bytes(n_seg, max_obs, n_obs_total) bytes;
 * w/mu/sigma: fp64 mixture pool (sorted components);
 * wcdf: fp64 cumulative weights (sampler); coef64: 4 doubles / component;
 * coef32: 4 floats / component.  max_obs = max n_obs over segs.
 * Pruning data for the sorted scoring path (per component, float; all four
 * NULL to skip): coef32n = coef32 with wide components masked (c = -inf),
 * wide32 = the wide components' coefficients compacted at comp_off, pm / sm
 * = prefix max of (mu + reach) / suffix min of (mu - reach) over narrow
 * components. */
int64_t tpe_fit_scratch_bytes(int n_seg, int max_obs, int64_t n_obs_total);
int tpe_parzen_fit(const double* obs, void* scratch, tpe_seg* segs, int n_seg, int max_obs,
                   int64_t n_obs_total, double* w, double* mu, double* sigma, double* wcdf,
                   double* coef64, float* coef32, float* coef32n, float* wide32, float* pm,
                   float* sm, void* stream);

/* ---- observation lists from an HBM-resident history ---------------------
 * Replaces the per-suggest rebuild of miscs_to_idxs_vals (base.py:200-214)
 * and the list comprehensions of ap_split_trials (tpe.py:623-646, tid order
 * kept).  vals / active: label-major matrices, element (col, row) at
 * col * ld + row; rows (nullable = identity): the n_rows history rows in tid
 * order; is_below: one flag per position of `rows` (1 = among the n_below
 * best losses).  Each descriptor compacts the rows active for `col` on its
 * side of the split into obs_f64 (Parzen fit pool) or, with to_int, into
 * obs_i64 as (int64)value - offset (categorical pool), writing at most
 * `count` elements; a different number of matches sets bit 4 of *err. */
typedef struct tpe_gather {
  int32_t col;          /* label column                                      */
  int32_t below;        /* 1: below rows, 0: above rows                      */
  int64_t dst_off;      /* first output element                              */
  int64_t offset;       /* to_int: subtracted (randint low)                  */
  int64_t count;        /* elements expected (the segment's n_obs)           */
  int32_t to_int;       /* 1: int64 output, 0: fp64 output                   */
  int32_t hist;         /* tpe_gather_obs_multi: index of the history (else 0) */
} tpe_gather;
/* Rows appended to an HBM-resident history: `stage` (device) holds the new
 * rows' values, label-major (n_labels x k fp64), then their active flags
 * (n_labels x k bytes); they are written to rows r0..r0+k-1 of vals / active
 * (label-major, leading dimension ld). */
int tpe_history_append(const void* stage, int n_labels, int64_t k, double* vals, uint8_t* active,
                       int64_t ld, int64_t r0, void* stream);
int tpe_gather_obs(const double* vals, const uint8_t* active, int64_t ld, const int32_t* rows,
                   int64_t n_rows, const uint8_t* is_below, const tpe_gather* gathers,
                   const tpe_gather* host_gathers, int n_gathers, double* obs_f64,
                   int64_t* obs_i64, int32_t* err, void* stream);

/* Many histories in one launch (batched independent studies, the C4 shape of
 * SURVEY §8(f) row 3): gather g reads history hists[g.hist].  A history's
 * row list (rows_off < 0: identity) and split flags live in the caller's
 * `aux` buffer at byte offsets rows_off / isb_off; n_cols bounds `col`. */
typedef struct tpe_history {
  const double* vals;     /* label-major values, (col, row) at col * ld + row    */
  const uint8_t* active;  /* same layout, 1 = label active in that row          */
  int64_t ld;
  int64_t n_cols;
  int64_t n_rows;         /* positions (length of the row list / flags)         */
  int64_t rows_off;       /* byte offset of int32 rows in aux, or -1 (identity) */
  int64_t isb_off;        /* byte offset of the uint8 split flags in aux        */
} tpe_history;
int tpe_gather_obs_multi(const tpe_history* hists, const tpe_history* host_hists, int n_hists,
                         const void* aux, const tpe_gather* gathers,
                         const tpe_gather* host_gathers, int n_gathers, double* obs_f64,
                         int64_t* obs_i64, int32_t* err, void* stream);

/* ---- sorted history: the Parzen fit without a per-suggest sort ------------
 * adaptive_parzen_normal (tpe.py:399-467) sorts each below / above set; both
 * are subsets of the label's history, and a stable sort of a subset is the
 * history's stable order with the other rows left out.  The history keeps,
 * for every fitted column, its rows sorted by (transformed value, row) in
 * `order` (label-major like vals: column col's order at order + col * ld);
 * tpe_history_order merges rows [n_old, n_old + n_new) (n_new <= 2048 per
 * call) into the order of rows [0, n_old) -- O(rows) per append.  The
 * transform is the fit's: log(max(v, floor)) for TPE_OBS_LOG (NaN last).
 * scratch: tpe_history_order_scratch_bytes(n_specs, n_old + n_new) bytes. */
typedef struct tpe_colspec {
  int32_t col;          /* history column                                    */
  int32_t transform;    /* TPE_OBS_*                                         */
  double floor;         /* TPE_OBS_LOG: log(max(v, floor))                   */
} tpe_colspec;
int64_t tpe_history_order_scratch_bytes(int n_specs, int64_t n_rows);
int tpe_history_order(const double* vals, int64_t ld, const tpe_colspec* specs,
                      const tpe_colspec* host_specs, int n_specs, int64_t n_old, int64_t n_new,
                      int32_t* order, void* scratch, void* stream);
/* The fit of segment i (segs[i]) from the sorted history: gathers[i] names its
 * column, side (below: 1) and observation count (identity row list: row r of
 * the history is position r, is_below[r] its split flag, n_rows of them).
 * One compaction block per segment: the segment's rows in tid order
 * (linear-forgetting positions, the prior's searchsorted slot), then the
 * column's order compacted to the segment (means and weights in sorted
 * order); then tpe_parzen_fit's own bandwidth / coefficient launches (same
 * bits).  A count other than gathers[i].count sets bit 4 of *err (the
 * segment's means are not written; the call's results are void).
 * Precondition: `order` holds, per column, a permutation of the rows
 * [0, n_rows) -- n_rows must be the history's row count (tpe_history_order's
 * n_rows), so is_below must hold exactly one flag per history row.
 * scratch: tpe_fit_sorted_scratch_bytes(n_seg, n_rows) bytes. */
int64_t tpe_fit_sorted_scratch_bytes(int n_seg, int64_t n_rows);
int tpe_fit_sorted(const double* vals, const uint8_t* active, int64_t ld, const int32_t* order,
                   int64_t n_rows, const uint8_t* is_below, const tpe_gather* gathers,
                   const tpe_gather* host_gathers, tpe_seg* segs, int n_seg, void* scratch,
                   double* w, double* mu, double* sigma, double* wcdf, double* coef64,
                   float* coef32, int32_t* err, void* stream);

/* ---- explicit mixtures (GMM1 / LGMM1 with given parameters) -------------
 * The reference's GMM1 / GMM1_lpdf / LGMM1 / LGMM1_lpdf (tpe.py:79-180,
 * 229-307) take the mixture directly (weights, mus, sigmas, low, high, q).
 * tpe_mixture_prepare readies such mixtures for tpe_sample and the scorers:
 * every segment (given = 1) holds its K = n_obs + 1 components at comp_off in
 * w (raw weights) / mu / sigma, prior_pos any component index, prior_mu a
 * point near the mixture (the fp32 coefficients' origin), low / high /
 * bounded its truncation.  Writes the normalised weights, p_accept (GMM1),
 * the cumulative weights and the fp64 / fp32 coefficients exactly as the fit
 * does for a fitted mixture (the sigmas are kept as given).
 * scratch: tpe_mixture_scratch_bytes(n_seg, max_comp) bytes. */
int64_t tpe_mixture_scratch_bytes(int n_seg, int max_comp);
int tpe_mixture_prepare(tpe_seg* segs, int n_seg, int max_comp, void* scratch, double* w,
                        const double* mu, double* sigma, double* wcdf, double* coef64,
                        float* coef32, void* stream);

/* ---- categorical posterior (tpe.py:578-615) ------------------------------ */
/* p_pool: probabilities (mode 1 also reads the prior p from it at
 * prior_p_off); logp_pool / cdf_pool: log p and cumulative p at p_off.
 * max_cat: the largest n_cat over segs (host value, sizes the grid). */
int tpe_cat_posterior(const int64_t* obs, const tpe_cat_seg* segs, int n_seg, int max_cat,
                      double* p_pool, double* logp_pool, double* cdf_pool, void* stream);

/* The same posteriors read straight from an HBM-resident history (the
 * arguments of tpe_gather_obs below): segment i's observations are the rows
 * of column gathers[i].col active there and on side gathers[i].below of the
 * split (is_below; rows: optional row list), in row order, their category
 * (int64)value - gathers[i].offset -- the lists tpe_gather_obs would write,
 * counted without writing them.  gathers: device array aligned with segs
 * (obs_off unused).  An observation count other than segs[i].n_obs sets bit
 * 4 of *err.  Replaces tpe_gather_obs + tpe_cat_posterior for the
 * categorical labels of a level (tpe.py:578-615, pyll/base.py:1053-1060).
 * work (device, nullable) of work_bytes >= tpe_cat_hist_scratch_bytes(n_seg,
 * max_cat, n_rows) > 0: a long history is counted in row chunks by many
 * blocks (the same bits); otherwise one block per (segment, category). */
int tpe_cat_posterior_hist(const double* vals, const uint8_t* active, int64_t ld,
                           const int32_t* rows, int64_t n_rows, const uint8_t* is_below,
                           const struct tpe_gather* gathers, const tpe_cat_seg* segs, int n_seg,
                           int max_cat, double* p_pool, double* logp_pool, double* cdf_pool,
                           void* work, int64_t work_bytes, int32_t* err, void* stream);
/* Work bytes of tpe_cat_posterior_hist's chunked path for these sizes (0:
 * the sizes take the single-block path; -1: bad arguments). */
int64_t tpe_cat_hist_scratch_bytes(int n_seg, int max_cat, int64_t n_rows);

/* ---- continuous candidates: sample (or read) + score + argmax ------------
 * Replaces GMM1/LGMM1 sampling (tpe.py:79-106, 229-257), GMM1_lpdf /
 * LGMM1_lpdf (tpe.py:117-180, 265-307) and broadcast_best (tpe.py:649-658)
 * for UNQUANTIZED labels.  partial: workspace of tpe_best, capacity
 * n_partial (query with tpe_score_partials()).  out_bl/out_al (nullable):
 * per-candidate log-likelihoods at job.out_off; out_x (nullable): the
 * candidates themselves.  best: one tpe_best per job. */
int64_t tpe_score_partials(const tpe_job* host_jobs, int n_jobs);
int tpe_score_continuous(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                         const tpe_seg* segs, const double* w, const double* mu,
                         const double* sigma, const double* wcdf, const double* coef64,
                         const float* coef32, const double* cand, int precision,
                         double* out_bl, double* out_al, double* out_x,
                         tpe_best* partial, int64_t n_partial, tpe_best* best,
                         void* stream);

/* ---- continuous candidates, sorted + pruned (fp32 throughput path) -------
 * Same results as tpe_score_continuous(precision=32) on sampled candidates
 * (same Philox draws, same winner up to fp32 rounding), but candidates are
 * first bucketed by value (count -> scan -> scatter, deterministic, no
 * global atomics) so each scoring block spans a narrow interval and only
 * components within reach -- those whose term can exceed 2^-40 of the
 * mixture sum -- plus the wide components are evaluated.
 * tpe_sort_layout: count-matrix elements and sorted-pool slots one job of
 * n_cand candidates needs.  pairs (nullable): u64 counter of evaluated
 * (candidate, component) pairs. */
int64_t tpe_sort_layout(int64_t n_cand, int64_t* sorted_slots);
/* draw the candidates (same Philox streams as tpe_score_continuous) into
 * gen (generation order) and bucket them by value into sorted_x / sorted_i
 * (candidate value, local index); gen/sorted at job.sort_off, counts: a
 * workspace of 2 x tpe_sort_layout() elements per job at 2 * job.cnt_off */
int tpe_sort_candidates(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                        const tpe_seg* segs, const double* mu, const double* sigma,
                        const double* wcdf, uint32_t* counts, float* gen,
                        float* sorted_x, uint32_t* sorted_i, void* stream);
/* score the bucketed candidates with component pruning + fused argmax */
int tpe_score_sorted(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                     const tpe_seg* segs, const float* coef32, const float* coef32n,
                     const float* wide32, const float* pm, const float* sm,
                     const float* sorted_x, const uint32_t* sorted_i,
                     tpe_best* partial, int64_t n_partial, tpe_best* best,
                     uint64_t* pairs, void* stream);

/* ---- continuous candidates, cell-table path (fp32 throughput path) -------
 * Same quantity as tpe_score_continuous(precision=32): per candidate the log
 * densities of both mixtures (GMM1_lpdf / LGMM1_lpdf, tpe.py:117-180,
 * 265-307) and the fused argmax (broadcast_best, tpe.py:649-658).  The
 * candidate coordinate range is cut into nb cells of half-width h.  On every
 * cell each mixture sum_j exp(l_j(y)) is expanded around the cell centre y0
 * as exp(m) * sum_{n<9} P_n u^n, u = (y - y0)/h: a degree-8 polynomial whose
 * P_0..P_5 are stored in fp32 and P_6..P_8 in fp16 (tpe_table_build).  Each
 * component's factor exp(A u + B u^2) is expanded only where 9|A| + 65|B| <=
 * 5.8 (series truncation <= 4.4e-7 relative on |u| <= 1.0501,
 * tools/table_bounds.py); the stored polynomial's whole error against its
 * mixture -- truncation, the build's fp32 terms, series, sums and merges,
 * fp32/fp16 storage -- is bounded per job from the build's worst case
 * (tpe_table.eps_mix); components whose largest term
 * on the whole range is below e^-25 / M of the prior component's smallest
 * term are left out (< 1.4e-11 of the sum).
 * From those two polynomials the build also fits, per cell, a cubic of the
 * score f(u) = (m_b - m_a) + log P_b(u) - log P_a(u) at four Chebyshev nodes
 * of [-1.05, 1.05], rounds it to fp32 and BOUNDS its error against f on
 * |u| <= 1.0501 (per sub-interval, the log series of both polynomials and a
 * majorant of its remainder): a cell whose bound exceeds 1e-6 is flagged;
 * the largest bound of the others (with the cubic's evaluation terms) is
 * tpe_table.eps_cubic.
 * A candidate whose cell fails the bound, or that lies outside the grid, is
 * scored by the exact fp32 log-sum-exp over all components instead.
 * tables: one tpe_table per job (device); cells: byte pool, 128 B per cell
 * slot: job j's region starts at 128 * job.tbl_off and holds tbl_cap 64-B
 * cells, then tbl_cap (m_below, m_above) fp32 pairs, then (at the next 16-B
 * boundary) tbl_cap 16-B score cubics {c0, c1, c2, c3} (c0 NaN: flagged);
 * reach_hi / reach_lo: fp64 per-component workspace (size of the mixture
 * pool); wide_idx: int32, same size.
 * stats (nullable, 3 x u64): [0] candidates scored by a fallback (exact
 * log-sum-exp; for tpe_score_table_fast also the two-polynomial cell),
 * [1] cells that failed the bound, [2] score cubics that failed their check. */
typedef struct tpe_table {
  double lo, hi;        /* candidate coordinate range (x, or log x for LGMM1) */
  double h_below, h_above; /* largest admissible half-width per mixture       */
  double origin;        /* left edge of cell 0 (cell c is centred at         */
                        /* origin + (2c+1) h)                                */
  double h;             /* cell half-width used                              */
  float inv_h, inv_w;   /* 1/h and 1/(2h)                                    */
  int32_t nb;           /* cells used (<= job.tbl_cap)                       */
  int32_t n_wide_below, n_wide_above;
  float slope;          /* max over unflagged cells of |c1| + 2.11|c2| + 3.31|c3|:
                           a bound of |df/du| on |u| <= 1.0501 (score cubics),
                           written by tpe_table_build                        */
  float eps_cubic;      /* max over unflagged cells of the proven bound of
                           |s32 - f^(u)| for a cubic-scored candidate, less its
                           2^-22 |s32| part: the cubic's fit to the stored
                           polynomials' score f^ (interval remainder, DESIGN.md
                           3.1), its fp32 evaluation and u's rounding, and the
                           fp32 score offset                                  */
  float eps_mix;        /* proven bound of the relative error of one stored
                           polynomial against its mixture on |u| <= 1.0501
                           (truncation, exclusion, the build's fp32 terms,
                           series, sums and merges, fp32/fp16 storage)       */
  int32_t build_items;  /* most components one cell's expansion summed       */
  float build_ab;       /* max over summed components of 1.0501|A| + 1.1028|B| */
  double T_below, T_above; /* log-term floor: components whose term stays
                              below it on a cell are left out               */
} tpe_table;

/* partial-workspace entries tpe_score_table needs */
int64_t tpe_table_partials(const tpe_job* host_jobs, int n_jobs);
/* scratch: tpe_table_scratch_bytes(n_jobs, max_comp) bytes; max_comp = the
 * largest component count (n_obs + 1) of the jobs' mixtures */
int64_t tpe_table_scratch_bytes(int n_jobs, int max_comp);
int tpe_table_build(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                    const tpe_seg* segs, const double* mu, const double* sigma,
                    const double* coef64, int max_comp, double* reach_hi, double* reach_lo,
                    int32_t* wide_idx, double* scratch, tpe_table* tables, float* cells,
                    uint64_t* stats, void* stream);
int tpe_score_table(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                    const tpe_seg* segs, const double* mu, const double* sigma,
                    const double* wcdf, const float* coef32, const tpe_table* tables,
                    const float* cells, const double* cand, double* out_bl, double* out_al,
                    double* out_x, tpe_best* partial, int64_t n_partial, tpe_best* best,
                    uint64_t* stats, void* stream);
/* The suggest path (sampled jobs only), in two calls.
 * tpe_score_table_fast: the same draws as tpe_score_table; each candidate is
 * scored by its cell's score cubic -- one 16-B load and three FMAs -- or, on a
 * flagged cubic, by the two-polynomial cell, then the exact fp32
 * log-sum-exp.  Writes the per-block fp32 winners to `partial` and the band
 * tiles.  tpe_band_rescore: the winner decided EXACTLY -- np.argmax
 * (tpe.py:649-658) over the fp64 scores of every candidate that can still be
 * the maximum.
 *
 * Band.  With eps(s) a proven bound of |s32 - s64| (for a
 * cubic-scored candidate eps = table.eps_cubic + 2.0001 table.eps_mix +
 * 2^-22 |s32|; a two-polynomial candidate carries its own; a log-sum-exp
 * candidate is always re-scored), candidate i can be the exact winner only if
 * s32_i + eps_i >= G := max_k (s32_k - eps_k).  Each scorer block (tile of
 * 8192 candidates) writes, without atomics, a header {lo = its best
 * s32 - eps, hi_max = its largest s32 + eps, n} (4 uint32 per tile in
 * band_ctl) and its candidates with s32 + eps >= lo (a superset: G >= lo)
 * into its own 256 entries of `band` (n = 0xFFFFFFFF: more than tile_cap,
 * <= 256, did not fit; tests shrink tile_cap to force the overflow path).
 * tpe_band_rescore (one launch, 4 blocks per job) takes G from the headers,
 * keeps the entries with s32 + eps >= G and re-scores them in fp64 -- per
 * table cell, a degree-20 expansion of both mixtures around the cell centre
 * over every component within e^-45 of the sum (components whose series
 * would converge slowly summed term by term) -- and takes the np.argmax
 * winner (largest score, then smallest index): best[j] = {fp64 score, index,
 * value (x, or exp(y) in fp64 for LGMM1), n_cand}.  A job with a full tile
 * that can still hold the winner (hi_max >= G) keeps the fp32 winner with
 * n_scored = -1: the caller re-scores it exactly (tpe_score_pruned64 with
 * TPE_F_DRAW32).
 * band / band_ctl / work: tpe_band_bytes(host_jobs, n_jobs, &ctl, &work),
 * ctl and work bytes (work: zeroed once before its first use; the rescore
 * leaves it zero).  No state carries from one call to the next in band or
 * band_ctl: every tile rewrites its header.  Both calls take the same job
 * list and partial workspace (tpe_table_partials()).
 * out_score / out_x / out_eps (nullable, tests): per candidate at
 * job.out_off, the fp32 score, the value and the bound eps used (+inf for
 * a log-sum-exp candidate). */
typedef struct tpe_band {
  int64_t index;        /* global candidate index                            */
  float y;              /* candidate in the scoring coordinate (fp32 draw)   */
  float hi;             /* s32 + eps: upper bound of its exact score          */
} tpe_band;
int64_t tpe_band_bytes(const tpe_job* host_jobs, int n_jobs, int64_t* ctl_bytes,
                       int64_t* work_bytes);
int tpe_score_table_fast(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                         const tpe_seg* segs, const double* mu, const double* sigma,
                         const double* wcdf, const float* coef32, const tpe_table* tables,
                         const float* cells, tpe_band* band, uint32_t* band_ctl,
                         double* out_score, double* out_x, double* out_eps, tpe_best* partial,
                         int64_t n_partial, int tile_cap, uint64_t* stats, void* stream);
int tpe_band_rescore(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                     const tpe_seg* segs, const double* coef64, const tpe_table* tables,
                     const tpe_band* band, const uint32_t* band_ctl, const tpe_best* partial,
                     int64_t n_partial, tpe_best* best, void* work, void* stream);

/* ---- continuous candidates, exact fp64 with pruning (parity mode) ----------
 * Same results as tpe_score_continuous(precision=64) up to fp64 rounding (a
 * sampled job with TPE_F_DRAW32 scores the fp32 stream of the table path
 * instead -- the exact re-score of a job whose band overflowed): the
 * plan of tpe_table_build (with an e^-40 exclusion margin and the fp64
 * sampler's |z| < 8.7 range) finds, per mixture, the components whose term
 * can reach e^-40 of the sum somewhere on the candidate range, with reach
 * windows over the sorted means; each candidate sums its window plus the
 * wide components in fp64 (every component when it lies off the range), so
 * the work per candidate follows the components near it, not M.  Workspaces
 * as tpe_table_build (reach_hi / reach_lo / wide_idx / scratch / tables);
 * partial: tpe_pruned64_partials() entries.  out_* as tpe_score_continuous. */
int64_t tpe_pruned64_partials(const tpe_job* host_jobs, int n_jobs);
int tpe_score_pruned64(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                       const tpe_seg* segs, const double* mu, const double* sigma,
                       const double* wcdf, const double* coef64, int max_comp,
                       double* reach_hi, double* reach_lo, int32_t* wide_idx, double* scratch,
                       tpe_table* tables, const double* cand, double* out_bl, double* out_al,
                       double* out_x, tpe_best* partial, int64_t n_partial, tpe_best* best,
                       void* stream);

/* ---- quantized labels: lattice path ---------------------------------------
 * Candidates of a quantized label take values k*q (np.round(x/q)*q,
 * tpe.py:106, 256); equal values have equal scores, so every distinct value
 * is scored once (fp64, the reference's erf-pair sum) and the argmax keeps the
 * first candidate index of the best value -- identical to np.argmax over all
 * candidates.  slot_first: uint64 pool of lattice slots (all jobs);
 * vals/firsts/scores: compacted present values (capacity n_cap per job at
 * job.lat_off); counts: int64 per job. */
int tpe_lattice_sample(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                       const tpe_seg* segs, const double* mu, const double* sigma,
                       const double* wcdf, uint64_t* slot_first, int32_t* err,
                       void* stream);
int tpe_lattice_compact(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                        const uint64_t* slot_first, double* vals, int64_t* firsts,
                        int64_t* counts, void* stream);
/* scores values (lattice values, or injected candidates when firsts==NULL
 * and counts==NULL: then job.n_cand values at job.cand_off of `vals`).
 * err: int32 flag set to 1 on a negative lognormal_cdf argument
 * (tpe.py:196-197). */
int64_t tpe_quantized_partials(const tpe_job* host_jobs, int n_jobs, int64_t max_vals);
/* reach_hi / reach_lo (nullable, both or neither): scratch of one double per
 * component of the pools (indexed by comp_off like the table path's): the
 * prefix max of mu + b / suffix min of mu - b, b = 6.5 max(sqrt2 sigma, EPS),
 * of every job's two mixtures (written here, k_qreach), so each value sums
 * only the window of components whose erf pair is not saturated -- the same
 * sums bit for bit as the full loop (NULL). */
int tpe_score_quantized(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                        const tpe_seg* segs, const double* w, const double* mu,
                        const double* sigma, const double* vals, const int64_t* firsts,
                        const int64_t* counts, int64_t max_vals, double* out_bl,
                        double* out_al, tpe_best* partial, int64_t n_partial,
                        tpe_best* best, int32_t* err, double* reach_hi, double* reach_lo,
                        void* stream);
/* The suggest path's lattice argmax, prefix first (replaces sample + compact
 * + score + reduce for sampled jobs without per-candidate outputs; the
 * result is the same tpe_best).  Draws the first `prefix` candidates of every
 * job (a positive multiple of 4096), scores every lattice slot, and takes the
 * best seen value at its first index; a job where a slot not yet seen scores
 * higher (or NaN) draws the rest of its stream and decides again.  A value
 * first seen after the prefix can only win by a strictly better score, so
 * the winner is np.argmax's over the whole stream either way.
 * partial: >= n_jobs * max(lat_n) tpe_best; need: int32 per job (written). */
int tpe_lattice_suggest(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                        const tpe_seg* segs, const double* w, const double* mu,
                        const double* sigma, const double* wcdf, uint64_t* slot_first,
                        int64_t prefix, tpe_best* partial, int64_t n_partial, int32_t* need,
                        tpe_best* best, int32_t* err, double* reach_hi, double* reach_lo,
                        void* stream);  /* reach_hi / reach_lo: as tpe_score_quantized */

/* ---- categorical labels: sample (or read) + score + argmax ---------------- */
int64_t tpe_categorical_partials(const tpe_job* host_jobs, int n_jobs);
int tpe_score_categorical(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                          const tpe_cat_seg* csegs, const double* logp_pool,
                          const double* cdf_pool, const double* cand, double* out_bl, double* out_al,
                          double* out_x, tpe_best* partial, int64_t n_partial,
                          tpe_best* best, void* stream);
/* The suggest path's categorical argmax, prefix first (sampled jobs without
 * per-candidate outputs; the same tpe_best as tpe_score_categorical).  Draws
 * the first `prefix` candidates of every job (a positive multiple of 4096);
 * a later candidate can only win with a strictly better-scoring category, all
 * of which are then absent from the prefix -- a job where one of them can be
 * drawn at all (non-empty inverse-CDF interval) draws the rest of its stream
 * and decides again.  partial: >= tpe_categorical_partials(); need: int32
 * per job (written: 1 = the rest was drawn). */
int tpe_categorical_suggest(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
                            const tpe_cat_seg* csegs, const double* logp_pool,
                            const double* cdf_pool, int64_t prefix, tpe_best* partial,
                            int64_t n_partial, int32_t* need, tpe_best* best, void* stream);

/* ---- sampler only (KS tests, debugging): n_cand draws of job.below ------- */
int tpe_sample(const tpe_job* jobs, const tpe_job* host_jobs, int n_jobs,
               const tpe_seg* segs, const double* mu, const double* sigma,
               const double* wcdf, int precision, double* out_x, void* stream);

/* ---- prior draws (startup phase: rand.suggest, hyperopt/rand.py:15-27) ----
 * Replaces the prior samplers of pyll/stochastic.py:36-158: n draws of every
 * prior, draw i of prior j at out[j * n + i], a function of (key, base + i)
 * only (Philox4x32-10).  kind: TPE_PRIOR_*; a, b = low, high (uniform,
 * loguniform in log space, randint: [low, high)) or mu, sigma (normal,
 * lognormal in log space); q > 0 quantizes as np.round(x / q) * q;
 * categorical: n_cat probabilities at p + p_off (need not be normalised).
 * Values are fp64 (category / randint values as whole numbers). */
enum {
  TPE_PRIOR_UNIFORM = 0, TPE_PRIOR_LOGUNIFORM = 1, TPE_PRIOR_NORMAL = 2,
  TPE_PRIOR_LOGNORMAL = 3, TPE_PRIOR_RANDINT = 4, TPE_PRIOR_CATEGORICAL = 5
};
typedef struct tpe_prior {
  int32_t kind;
  int32_t n_cat;        /* categorical: number of categories                 */
  double a, b, q;
  int64_t p_off;        /* categorical: first probability in `p`             */
  uint64_t key;         /* Philox key (seed mixed with the label)            */
} tpe_prior;
int tpe_prior_sample(const tpe_prior* priors, const tpe_prior* host_priors, int n_priors,
                     const double* p, int64_t n, int64_t base, double* out, void* stream);

/* ---- argmax combine: n_sets tpe_best arrays of n_labels each (e.g. one per
 * rank after an all-gather) -> n_labels winners, same tie rules. ------------ */
int tpe_best_combine(const tpe_best* sets, int n_sets, int n_labels, tpe_best* out,
                     void* stream);

/* ---- per-label records of one rank's level: slot s of `out` (n_slots
 * tpe_best, device) <- the records of the jobs j with slot[j] == s (device
 * int32 per job), folded in job order with the argmax rules; index -1 where
 * no job maps to s.  The input of tpe_maxloc_allreduce for a label-sharded
 * level. */
int tpe_best_scatter(const tpe_best* by_job, const int32_t* slot, int n_jobs, tpe_best* out,
                     int n_slots, void* stream);

/* ---- cross-GPU max-loc (replaces the argmax of tpe.py:650-658
 * across ranks): all-gather of every rank's n_labels records over the caller's
 * RCCL communicator `comm` (an ncclComm_t; librccl.so.1 is bound at the first
 * call), then tpe_best_combine of the world's sets into `out`.  `local`: this
 * rank's records (index -1 where it scored nothing); `gathered`: device
 * scratch of world * n_labels records.  Asynchronous on `stream`. */
int tpe_maxloc_allreduce(const tpe_best* local, tpe_best* gathered, tpe_best* out, int n_labels,
                         void* comm, void* stream);

/* ---- level launcher: a whole suggest level's stream work in one host call.
 * `ops` (host) is a list of records, each naming one of the entry points above
 * (or a runtime step) by `code` and carrying that call's arguments, in
 * declaration order, as 64-bit words (pointers and handles as addresses,
 * int / int64_t by value).  tpe_run_ops issues them in order and stops at the
 * first failing record (its index in *failed_op, -1 when all succeeded).  A
 * binding that replays the same level (same kernels, grids, workspace) keeps
 * its record array and re-issues it with one call: the per-call inputs live
 * in the device buffers the records point to (the level's upload), or captures
 * them once into a hipGraph and replays that (tpe_ops_capture below). ------ */
enum {
  TPE_OP_GATHER_OBS = 1,       /* tpe_gather_obs                             */
  TPE_OP_GATHER_OBS_MULTI,     /* tpe_gather_obs_multi                       */
  TPE_OP_PARZEN_FIT,           /* tpe_parzen_fit                             */
  TPE_OP_CAT_POSTERIOR,        /* tpe_cat_posterior                          */
  TPE_OP_TABLE_BUILD,          /* tpe_table_build                            */
  TPE_OP_SCORE_TABLE,          /* tpe_score_table                            */
  TPE_OP_SCORE_TABLE_FAST,     /* tpe_score_table_fast                       */
  TPE_OP_SCORE_PRUNED64,       /* tpe_score_pruned64                         */
  TPE_OP_SCORE_CONTINUOUS,     /* tpe_score_continuous                       */
  TPE_OP_SORT_CANDIDATES,      /* tpe_sort_candidates                        */
  TPE_OP_SCORE_SORTED,         /* tpe_score_sorted                           */
  TPE_OP_LATTICE_SAMPLE,       /* tpe_lattice_sample                         */
  TPE_OP_LATTICE_COMPACT,      /* tpe_lattice_compact                        */
  TPE_OP_SCORE_QUANTIZED,      /* tpe_score_quantized                        */
  TPE_OP_SCORE_CATEGORICAL,    /* tpe_score_categorical                      */
  TPE_OP_SAMPLE,               /* tpe_sample                                 */
  TPE_OP_EVENT_RECORD,         /* hipEventRecord(a[0] event, a[1] stream)    */
  TPE_OP_STREAM_WAIT,          /* hipStreamWaitEvent(a[0] stream, a[1] event) */
  TPE_OP_MEMCPY,               /* hipMemcpyAsync(a[0] dst, a[1] src, a[2] bytes,
                                  a[3] hipMemcpyKind, a[4] stream)           */
  TPE_OP_STREAM_SYNC,          /* hipStreamSynchronize(a[0] stream)          */
  TPE_OP_BEST_SCATTER,         /* tpe_best_scatter                           */
  TPE_OP_MAXLOC_ALLREDUCE,     /* tpe_maxloc_allreduce (RCCL, stream-ordered) */
  TPE_OP_LATTICE_SUGGEST,      /* tpe_lattice_suggest                        */
  TPE_OP_BAND_RESCORE,         /* tpe_band_rescore                           */
  TPE_OP_FIT_SORTED,           /* tpe_fit_sorted                             */
  TPE_OP_HISTORY_ORDER,        /* tpe_history_order                          */
  TPE_OP_CATEGORICAL_SUGGEST,  /* tpe_categorical_suggest                    */
  TPE_OP_CAT_POSTERIOR_HIST,   /* tpe_cat_posterior_hist                     */
  TPE_OP_COUNT
};
#define TPE_OP_ARGS 23
typedef struct tpe_op {
  int32_t code;
  int32_t n_args;               /* must equal the entry point's parameter count */
  int64_t a[TPE_OP_ARGS];
} tpe_op;                       /* 192 bytes */
int tpe_run_ops(const tpe_op* ops, int n_ops, int* failed_op);
/* Issuing threads of tpe_run_ops (1, the default, or 2); returns the previous
 * setting, TPE_E_ARG for another n.  With 2, a batch whose records use more
 * than one stream is issued by the caller (the records on the stream of the
 * first record that names one, and records without a stream) and a resident
 * worker thread of the library (every other stream's records), each in list
 * order; event records (TPE_OP_EVENT_RECORD / TPE_OP_STREAM_WAIT) are issued
 * in their global list order, so the streams' work and dependencies are those
 * of one-thread issue.  *failed_op names the first failing record in list
 * order.  A batch issued while another thread's batch holds the worker is
 * issued by the caller alone. */
int tpe_set_issue_threads(int n);
/* The same records as a hipGraph: tpe_ops_capture issues ops[0..n_ops) into a
 * stream capture of `capture_stream` (a stream of the caller's, not the null
 * stream), with every record's stream operand that names `from_stream` (the
 * records' main stream, possibly the null stream) pointed at
 * `capture_stream` instead; every stream the records fork to must be joined
 * back by an event wait among the records.  The graph is instantiated in
 * *graph_exec -- nothing runs.  Records that cannot be captured
 * (TPE_OP_STREAM_SYNC, TPE_OP_MAXLOC_ALLREDUCE) fail it with TPE_E_ARG at
 * *failed_op; a capture the runtime refuses fails it with TPE_E_LAUNCH.  The
 * graph holds every record's words as captured (pointers, sizes, grids): a
 * binding replays it with tpe_graph_launch only while re-issuing exactly those
 * records, the per-call inputs again in the device buffers they point to.
 * tpe_graph_destroy frees it. */
int tpe_ops_capture(const tpe_op* ops, int n_ops, void* from_stream, void* capture_stream,
                    void** graph_exec, int* failed_op);
int tpe_graph_launch(void* graph_exec, void* stream);
int tpe_graph_destroy(void* graph_exec);

/* host: rows of the k smallest losses in np.argsort(losses, kind="stable")
 * order (NaN after +inf, ties to the earlier row) -- the below split of
 * ap_split_trials (tpe.py:623-646) -- written to out (host) in ascending row
 * order; returns min(k, n), -1 on bad arguments. */
int64_t tpe_smallest_rows(const double* losses, int64_t n, int64_t k, int64_t* out);
/* host: tpe_smallest_rows plus the level inputs of the split in one pass:
 * isb[r] = 1 for the below rows (else 0), nb[j] = active below rows of label
 * j, na[j] = n_active[j] - nb[j] (a history without from_tid aliasing: every
 * row is below or above).  active: T x L bytes, row-major.  Returns the
 * number of below rows written to below_rows (ascending), -1 on bad
 * arguments (ap_split_trials, tpe.py:623-646). */
int64_t tpe_split_inputs(const double* losses, int64_t T, int64_t n_below, const uint8_t* active,
                         int64_t L, const int64_t* n_active, uint8_t* isb, int64_t* below_rows,
                         int64_t* nb, int64_t* na);

const char* tpe_last_error(void);
int tpe_abi_version(void);
/* Self-check of the hardware transcendentals the fp32 error bounds assume
 * (DESIGN.md 3.1): out[0] = max relative error of v_exp_f32 over every fp32
 * x in [-126, 12]; out[1] = max over positive normal fp32 p of
 * |v_log_f32(p) - log2 p| / max(1, |log2 p|).  Exhaustive (2^32 inputs, a
 * few ms); out: 2 doubles (device), asynchronous on `stream`. */
int tpe_check_transcendentals(double* out, void* stream);

/* host: writes sizeof(tpe_seg, tpe_cat_seg, tpe_job, tpe_best, tpe_table, tpe_gather,
 * tpe_history, tpe_prior, tpe_op, tpe_band, tpe_colspec) to out[0..n); returns 11 */
int tpe_struct_sizes(int32_t* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* TPE_HIP_H */
