/*
 * cbn_amd.h -- C ABI of the MI355X-native batched inference engine for
 * ContinuousBayesianNetwork (libcbn_amd.so).
 *
 * Plain C: pointers, sizes, int32/int64/float; device pointers are HIP device
 * addresses; `stream` is a hipStream_t passed as void* (NULL = default stream).
 * No torch types cross this boundary.  Every entry point returns 0 on success
 * and a negative CBN_E* code on failure; cbn_last_error() gives the message.
 *
 * Each entry point names the reference interface it replaces
 * (Giovannibriglia/ContinuousBayesianNetwork, file:line).
 */
#ifndef CBN_AMD_H
#define CBN_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CBN_AMD_ABI_VERSION 5

#define CBN_MAX_PARENTS 8    /* parents per node handled by one factor descriptor */
#define CBN_MAX_EVIDENCE 256 /* distinct evidence columns per query batch        */

#define CBN_OK 0
#define CBN_E_ARG -1
#define CBN_E_HIP -2
#define CBN_E_LIMIT -3
#define CBN_E_UNSUPPORTED -4  /* the plan cannot take this launch mode (caller picks another) */
#define CBN_E_TIMEOUT -5      /* an earlier single-launch call of this plan timed out in its grid barrier
                                 (not every block was resident): that call's rows are NaN; reported (and
                                 cleared) by the plan's next cbn_plan_run / cbn_plan_status */

/* Factor kinds of bayesian_network.py:271-294 (the per-node `x` multiplied
 * into out_pdf):
 *   SCALAR : root node, pdf [1, N]      -> x = mean over the N samples     [1]
 *   SHARED : parents, none observed     -> x = mean over N^k parent combos [1, N]
 *   QUERY  : >=1 parent observed        -> x = mean over free-parent combos,
 *            indexed per query by the observed parents' values          [Q, N] */
#define CBN_FACTOR_SCALAR 0
#define CBN_FACTOR_SHARED 1
#define CBN_FACTOR_QUERY 2

/* One node's factor on the inference path of BayesianNetwork.infer
 * (bayesian_network.py:241-255 builds one `pdfs` per ancestor via
 * Node.get_prob, node.py:115-204).  All pointers are device pointers. */
typedef struct cbn_factor_desc {
    int32_t kind;                                 /* CBN_FACTOR_*                        */
    int32_t n_parents;                            /* k (sorted parent order, node.py:65) */
    int32_t node_card;                            /* |domain(node)|                      */
    int32_t parent_card[CBN_MAX_PARENTS];         /* |domain(parent_i)|                  */
    int32_t parent_ev_slot[CBN_MAX_PARENTS];      /* -1: free parent; else evidence col  */
    const float* cpd;                             /* dense CPD [parent_card..., node_card]
                                                     (root: marginal [node_card]); every
                                                     entry finite and >= 0 (BruteForce's
                                                     joint / (marginal + 1e-10) always
                                                     is): the table kernels stop
                                                     multiplying a query's row once it
                                                     is all +0, which equals the
                                                     reference's product only when no
                                                     later factor is inf (0 x inf = NaN) */
    const int32_t* node_sample_idx;               /* [N] node sample -> domain idx or -1 */
    const int32_t* parent_sample_idx;             /* [k*N] free-parent sample idx or -1  */
    const float* parent_domain[CBN_MAX_PARENTS];  /* sorted domain values (observed parents) */
} cbn_factor_desc;

typedef struct cbn_plan cbn_plan;  /* opaque: device descriptors + factor tables */

/* ABI version / last error message of the calling thread. */
int cbn_abi_version(void);
const char* cbn_last_error(void);

/* Dense BruteForce CPD from the fitted maximum-likelihood rows.
 * Replaces brute_force.py:17-53 (_fit's mle_tensor) + the per-call equality
 * scans of brute_force.py:227-241 (joint / parent-marginal sums).
 *   cell[r]  : flat index of mle row r in [n_parent_cells, node_card]
 *   prob[r]  : its empirical probability (counts / total)
 *   normalize: 1 -> cpd = joint / (sum_v joint + 1e-10)  (conditional, :240-241)
 *              0 -> cpd = joint                          (root marginal, :192-201) */
int cbn_bf_cpd_build(const int32_t* cell, const float* prob, int64_t n_rows,
                     int64_t n_parent_cells, int32_t node_card, int32_t normalize,
                     float* cpd, void* stream);

/* Evaluate a dense BruteForce CPD at arbitrary float points.
 * Replaces BruteForce._get_prob (brute_force.py:172-244):
 *   points   : [n_points, n_cols] float32, columns = parents..., node
 *   domains  : per column, a sorted domain array (device) and its size
 *   out[i]   : cpd[idx(points[i])], 0 where any value is not in its domain
 *              (the reference's 0 / (0 + 1e-10)). */
int cbn_bf_cpd_eval(const float* cpd, int32_t n_cols, const float* const* domains,
                    const int32_t* domain_card, const float* points, int64_t n_points,
                    float* out, void* stream);

/* ---- CPDs beyond dense tables: sparse (hashed) BruteForce CPDs and nodes
 * with more than CBN_MAX_PARENTS parents.
 *
 * The reference answers BruteForce.get_prob for ANY fitted data with two
 * equality scans over the unique training rows (brute_force.py:228-237), so
 * continuous / high-cardinality columns work there at O(points x rows) per
 * call.  A dense table over the columns' domains would hold prod(cards)
 * cells; past a size limit the estimator keeps instead a hash table keyed by
 * the row's mixed-radix domain index (parents in sorted order, node last;
 * prod(cards) < 2^62) whose value is the row's conditional probability
 * joint / (parent marginal + 1e-10) -- rows absent from the table give 0,
 * exactly the reference's 0 / (0 + 1e-10).  Keys of empty slots are -1;
 * capacity is a power of two >= 2 x rows (linear probing). */
#define CBN_MAX_DIRECT_PARENTS 32

/* Insert n (key, value) pairs (keys unique, >= 0) into a hash table of
 * `capacity` slots (power of two); the table is cleared first. */
int cbn_hash_build(const int64_t* keys, const float* vals, int64_t n, int64_t* table_keys, float* table_vals,
                   int64_t capacity, void* stream);

/* A BruteForce CPD over n_cols columns (parents in sorted order, node last):
 * dense array [cards...] or hash table.  Host struct; pointers are device
 * pointers except `domains` / `cards` (host arrays of n_cols entries). */
typedef struct cbn_cpd_ref {
    int32_t n_cols;
    const float* const* domains;  /* sorted domain values of each column            */
    const int32_t* cards;         /* |domain| of each column                        */
    const float* dense;           /* dense CPD (NULL: sparse)                       */
    const int64_t* keys;          /* sparse: table keys (-1 empty)                  */
    const float* vals;            /* sparse: conditional probabilities              */
    int64_t capacity;             /* sparse: slots (power of two)                   */
} cbn_cpd_ref;

/* BruteForce._get_prob (brute_force.py:172-244) on a dense or hashed CPD:
 * out[i] = P(points[i]) -- points [n_points, n_cols] float32. */
int cbn_cpd_ref_eval(const cbn_cpd_ref* cpd, const float* points, int64_t n_points, float* out, void* stream);

/* One factor of a DIRECT plan: evaluated per (query, sample column) straight
 * from its CPD (no per-plan table: the tables of these factors would have
 * prod(observed cards) rows), any number of parents up to
 * CBN_MAX_DIRECT_PARENTS.  Same kinds and sample-index conventions as
 * cbn_factor_desc.  Root (SCALAR): cpd is the node marginal (n_cols = 1). */
typedef struct cbn_direct_factor {
    int32_t kind;                     /* CBN_FACTOR_*                                   */
    int32_t n_parents;                /* k <= CBN_MAX_DIRECT_PARENTS (sorted order)     */
    const int32_t* parent_ev_slot;    /* host [k]: evidence column or -1 (free)         */
    const int32_t* node_sample_idx;   /* device [N]: node sample -> domain idx or -1    */
    const int32_t* parent_sample_idx; /* device [k*N]: free-parent sample idx or -1     */
    cbn_cpd_ref cpd;                  /* columns: parents..., node                      */
    /* host [k] or NULL (all 1): the width of each observed parent's evidence
     * column -- 1, or N_max for a [n_queries, N_max] column that the node reads
     * through Node._setup_parents_query's .expand(-1, N) (node.py:246-248: a
     * node whose evidence keys are not all its parents) as N per-query sample
     * values of that parent; element (q, i) of such a column is value i of
     * query q, and the factor averages over them like a free parent's samples
     * (node.py:335-375).  Added in ABI 5 (round 6). */
    const int32_t* parent_ev_width;
} cbn_direct_factor;

/* A plan whose factors are evaluated directly (BayesianNetwork.infer,
 * bayesian_network.py:208-305, for networks whose dense factor tables do not
 * fit): cbn_plan_run computes every (query, column) product in the
 * reference's factor order, then the global-max division (raw + scale; the
 * CBN_RUN_RAW launch for the sharded path).  query_max / query_write /
 * the single-launch path are not available (CBN_E_UNSUPPORTED). */
int cbn_plan_create_direct(const cbn_direct_factor* factors, int32_t n_factors, int32_t n_samples,
                           cbn_plan** plan);

/* Build a plan for one (target node, observed-column set, N_max) of
 * BayesianNetwork.infer (bayesian_network.py:208-305).  Copies the
 * descriptors to the device and allocates the factor tables. */
int cbn_plan_create(const cbn_factor_desc* factors, int32_t n_factors, int32_t n_samples,
                    cbn_plan** plan);
int cbn_plan_destroy(cbn_plan* plan);
/* Bytes of factor tables / whether the query kernels stage them in LDS. */
int64_t cbn_plan_table_bytes(const cbn_plan* plan);
int cbn_plan_uses_lds(const cbn_plan* plan);

/* Marginalise the free parents of the factors whose tables cannot be filled
 * straight from their CPD (the torch.mean(pdf, dim=parent dims) of
 * bayesian_network.py:292).  One launch for all such factors; a no-op when
 * every factor is a root or has all parents observed. */
int cbn_plan_build_tables(cbn_plan* plan, void* stream);

/* Pass 1: *max_bits = max over (q, j) of prod_f x_f[q, j] (float bits; all
 * values are >= 0).  The word is overwritten (no zeroing needed); a plan is
 * used by one stream at a time.  evidence[c] is the [n_queries] float32
 * column for evidence slot c (node.py:230-256 reads them as float32). */
int cbn_plan_query_max(cbn_plan* plan, int64_t n_queries, const float* const* evidence,
                       int32_t n_evidence, uint32_t* max_bits, void* stream);

/* Pass 2: out[q, j] = prod_f x_f[q, j] / max  (bayesian_network.py:269-296),
 * out is [n_queries, N] row-major float32. */
int cbn_plan_query_write(cbn_plan* plan, int64_t n_queries, const float* const* evidence,
                         int32_t n_evidence, const uint32_t* max_bits, float* out,
                         void* stream);

/* build_tables + query_max + query_write on one stream (single GPU). */
int cbn_plan_infer(cbn_plan* plan, int64_t n_queries, const float* const* evidence,
                   int32_t n_evidence, uint32_t* max_bits, float* out, void* stream);

/* query_max + query_write, preceded by build_tables when flags has
 * CBN_RUN_BUILD_TABLES; CBN_RUN_TIMED records HIP events around the two
 * passes on `stream` (up to 512 calls, read back by cbn_plan_timing). */
#define CBN_RUN_BUILD_TABLES 1
#define CBN_RUN_TIMED 2
#define CBN_RUN_TWO_PASS 4  /* force max + write launches (no single-launch grid-barrier path) */
/* CBN_RUN_RAW: one launch that stores the UNnormalised products in out and
 * this batch's per-block maxima in max_bits[0, cbn_plan_max_words(plan))
 * (unused words 0).  The sharded path all-reduces those words (MAX) across
 * ranks, then cbn_scale divides in place by their max -- bayesian_network.py:296
 * over the whole, multi-rank batch.  CBN_E_UNSUPPORTED for plans off the fast
 * path (cbn_plan_max_words == 0; the caller then uses query_max / all-reduce /
 * query_write). */
#define CBN_RUN_RAW 8
int cbn_plan_run(cbn_plan* plan, int64_t n_queries, const float* const* evidence,
                 int32_t n_evidence, uint32_t* max_bits, float* out, int32_t flags, void* stream);

/* Largest batch the single-launch path takes (0: not available for this
 * plan); larger batches run as two launches.  Status: nonzero when a fused
 * launch's grid barrier timed out (a block never became resident) -- its
 * output is then invalid; reads device memory (synchronous). */
int64_t cbn_plan_fused_capacity(const cbn_plan* plan);

/* Words of per-block maxima a CBN_RUN_RAW launch writes (0: no raw launch). */
int32_t cbn_plan_max_words(const cbn_plan* plan);

/* out[i] /= float(max over max_bits[0, n_max)) for i < n (in place, on
 * `stream`): the global-max division of bayesian_network.py:296 after a
 * CBN_RUN_RAW launch and the cross-rank all-reduce of its words. */
int cbn_scale(float* out, int64_t n, const uint32_t* max_bits, int32_t n_max, void* stream);
/* cbn_scale for up to 8 batches in one launch: outs[b][0, n_elems[b]) /=
 * max over max_bits[b * n_max, (b + 1) * n_max) (outs / n_elems: host arrays
 * of device pointers / sizes).  The pipelined sharded step exchanges and
 * scales several raw launches at once (distributed.ShardedStepper). */
int cbn_scale_batch(float* const* outs, const int64_t* n_elems, int32_t n_batches, const uint32_t* max_bits,
                    int32_t n_max, void* stream);
/* A CBN_RUN_RAW launch that also finishes an EARLIER raw launch: divides
 * fold_rows[0, fold_n_elems) in place by float(max over fold_words[0,
 * fold_n_words)) -- that step's cbn_scale (bayesian_network.py:296), bit for
 * bit -- inside this launch, overlapping the products (the pipelined sharded
 * stepper scales step s in the launch of step s + 2G).  fold_rows NULL: a plain
 * raw launch.  Staged plans only (CBN_PLAN_STAGED), else CBN_E_UNSUPPORTED;
 * fold_n_elems % 4 == 0, fold_rows 16-B aligned, 1 <= fold_n_words <= 256.
 * Added in ABI 4. */
int cbn_plan_run_fold(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                      uint32_t* max_bits, float* out, float* fold_rows, int64_t fold_n_elems,
                      const uint32_t* fold_words, int32_t fold_n_words, int32_t flags, void* stream);
int cbn_plan_status(cbn_plan* plan, int32_t* status);

/* CBN_E_TIMEOUT (and clears the report) if a single-launch call of the plan
 * timed out in its grid barrier since the last report, else CBN_OK: a read of
 * the plan's host-mapped status word, no device round trip.  A caller that
 * synchronised the stream of its calls learns of such a call at that point
 * instead of on the plan's next cbn_plan_run.  Added in ABI 4 (round 3).
 * No reference counterpart (the reference's infer has no grid barrier). */
int cbn_plan_check(cbn_plan* plan);

/* Which kernels serve the plan (bit set): diagnostics / bench labels. */
#define CBN_PLAN_FAST 1        /* table fast path (k_query_fast / k_query_staged) */
#define CBN_PLAN_LDS 2         /* the table image is staged in LDS (else read from L2 / HBM) */
#define CBN_PLAN_PAIRED 4      /* N = 32 bank-half table layout */
#define CBN_PLAN_STAGED 8      /* k_query_staged (evidence staged by factor) */
#define CBN_PLAN_FUSED 16      /* single-launch (grid barrier) path available */
#define CBN_PLAN_PARAMETRIC 32 /* parametric CPDs (cbn_param.hip) */
#define CBN_PLAN_VPL2 64       /* 8 output columns per lane */
#define CBN_PLAN_DIRECT 128    /* direct plan (cbn_plan_create_direct) */
#define CBN_PLAN_COLS 256      /* k_query_cols (evidence indexed once per slot; non-paired table plans) */
#define CBN_PLAN_SLOTS 512     /* k_query_slots (slot-indexed evidence, global tables, >= 4 lanes per query; round 5) */
int32_t cbn_plan_flags(const cbn_plan* plan);

/* Test hook: mark the plan as if a single-launch call had timed out in its
 * grid barrier, so the next cbn_plan_run returns CBN_E_TIMEOUT (exercises the
 * reporting path without starving the GPU).  No reference counterpart. */
int cbn_debug_flag_timeout(cbn_plan* plan);

/* 1 when the library was loaded with CBN_DIAG=1: only then are the
 * diagnostic kernel-selection variables (CBN_NO_STAGED, CBN_FAST_VPL,
 * CBN_PARAM_GENERIC, ... -- same-box A/B builds) honoured, and each CBN_*
 * variable of the environment is listed on stderr at load.  Otherwise they
 * are ignored: a stray variable cannot swap the kernels of a serving process.
 * Added in round 5 (ABI 4, additive).  No reference counterpart. */
int32_t cbn_diag_enabled(void);

/* Average device time (ms) of the max and write passes over the timed calls
 * since the last read; waits for them; resets the ring. */
int cbn_plan_timing(cbn_plan* plan, int32_t* n_timed, float* avg_max_ms, float* avg_write_ms);

/* ------------------------------------------------ parametric CPDs ------
 * The reference's continuous estimators evaluate a density of the node at its
 * sample points given a location mu computed from the parents' values:
 *   GAUSS    : LinearRegression._get_prob (linear_regression.py:104-124)
 *              pdf = (1 / (sigma * sqrt(2 pi))) * exp(-0.5 * ((x - mu) / sigma)^2)
 *   LOGISTIC : LogisticRegression._get_prob (logistIc_regression.py:70-100) and
 *              NeuralNetwork._get_prob (neural_network.py:99-131)
 *              d = (x - mu) / s;  pdf = exp(-d) / (s * (1 + exp(-d))^2)
 * mu = an nn.Linear stack: y = W x + b per layer, the activation after every
 * layer but the last (neural_network.py:45-54); one layer = a linear model. */
#define CBN_MAX_LAYERS 4     /* layers of the fixed-size width[] form (deeper: widths) */
#define CBN_MAX_WIDTH 32     /* hidden units of the register-resident fast kernels: models
                                with one hidden layer of any width and <= CBN_MAX_PARENTS
                                inputs, or <= 4 layers of <= 32 units; larger models run
                                the generic kernel (activations in LDS)                 */
#define CBN_MAX_MODEL_LAYERS 64   /* generic kernel: nn.Linear layers                    */
#define CBN_MAX_MODEL_WIDTH 256   /* generic kernel: inputs / units of any layer         */
#define CBN_FAMILY_GAUSS 1
#define CBN_FAMILY_LOGISTIC 2
#define CBN_ACT_TANH 1       /* activation_map of neural_network.py:10-18 */
#define CBN_ACT_RELU 2
#define CBN_ACT_SIGMOID 3
#define CBN_ACT_LEAKYRELU 4  /* negative slope 0.01 (nn.LeakyReLU default) */
#define CBN_ACT_GELU 5       /* exact (erf) form, nn.GELU default         */
#define CBN_ACT_ELU 6        /* alpha 1 */
#define CBN_INPUT_FREE -1    /* input = a free parent: its N sample points (mean over combos) */
#define CBN_INPUT_ONE -2     /* input = constant 1 (root models: neural_network.py:117-119)  */

typedef struct cbn_param_model {
    int32_t family;                     /* CBN_FAMILY_*                                  */
    int32_t n_layers;                   /* 1..CBN_MAX_MODEL_LAYERS                       */
    int32_t width[CBN_MAX_LAYERS + 1];  /* width[0] = inputs, width[n_layers] = 1         */
    int32_t act;                        /* CBN_ACT_* (ignored when n_layers == 1)         */
    const float* weights;               /* device: per layer W[out][in] row-major, then b[out] */
    float scale;                        /* sigma = exp(log_sigma) / s = exp(log_scale), fp32 */
    float norm;                         /* GAUSS: 1 / (sigma * sqrt(2 pi)) as fp32 ops; else 0 */
    const int32_t* widths;              /* host [n_layers + 1] or NULL: replaces width[]
                                           (required when n_layers > CBN_MAX_LAYERS)      */
} cbn_param_model;

/* One ancestor's factor of BayesianNetwork.infer for a parametric estimator.
 *   SCALAR (root)      : x = mean_j pdf(s_j; mu(1))                         [1]
 *   SHARED (no parent observed): x[j] = mean over N^k parent-sample combos c
 *                        of pdf(s_j; mu(c))                                  [N]
 *   QUERY              : x[q, j] = mean over the free parents' combos c of
 *                        pdf(s_j; mu(observed values of query q, c))     [Q, N]
 * (node.py:115-204 with bayesian_network.py:271-294's mean over parent axes.) */
typedef struct cbn_param_factor {
    int32_t kind;                         /* CBN_FACTOR_*                            */
    int32_t input_slot[CBN_MAX_PARENTS];  /* per model input: evidence column >= 0,
                                             CBN_INPUT_FREE or CBN_INPUT_ONE          */
    const float* input_samples;           /* device [width[0]][N]: rows of FREE inputs */
    const float* node_samples;            /* device [N]: the node's evaluation points  */
    cbn_param_model model;
    const int32_t* input_slots;           /* host [width[0]] or NULL: replaces input_slot[]
                                             (required for > CBN_MAX_PARENTS inputs)   */
} cbn_param_factor;

/* Plan of one (target, observed set, N_max) over parametric factors, run by
 * cbn_plan_run (default: one raw launch + an in-place scale; CBN_RUN_RAW: the
 * raw launch alone, per-block maxima in max_bits[0, cbn_plan_max_words)) and
 * released by cbn_plan_destroy.  Query-independent factors (SCALAR / SHARED)
 * are evaluated once here. */
int cbn_plan_create_param(const cbn_param_factor* factors, int32_t n_factors, int32_t n_samples,
                          cbn_plan** plan);

/* Estimator get_prob: out[r, v] = pdf(points[r, v]; mu(query[r, :])) for
 * r < n_rows, v < n_points (query = NULL: the model input is the constant
 * CBN_INPUT_ONE vector, or -- root_bias_only -- mu = the last layer's bias,
 * LinearRegression's query-free mean, linear_regression.py:112-117).
 * points [n_rows, n_points], query [n_rows, width[0]], out [n_rows, n_points]:
 * float32 device, row-major. */
int cbn_param_eval(const cbn_param_model* model, const float* points, int64_t n_rows, int32_t n_points,
                   const float* query, int32_t root_bias_only, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CBN_AMD_H */
