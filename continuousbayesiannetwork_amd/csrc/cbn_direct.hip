// cbn_direct.hip -- direct-evaluation inference plans and hashed BruteForce
// CPDs (gfx950).
//
// Reference: BayesianNetwork.infer (cbn/base/bayesian_network.py:208-305) over
// factors from Node.get_prob (cbn/base/node.py:115-204) evaluated by
// BruteForce._get_prob (cbn/parameter_learning/brute_force.py:172-244), which
// answers ANY fitted data -- continuous or high-cardinality columns, any
// number of parents -- with equality scans over the unique training rows.
//
// The table path (cbn_infer.hip) tabulates every factor over its observed
// parents' domains: prod(observed cards) rows x N.  For ~1 000-value columns
// or nodes with many parents that is unbounded, so a DIRECT plan evaluates
// each factor per (query, sample column) from the CPD itself -- a dense array
// when it fits, else a hash table of the unique rows (key = mixed-radix domain
// index, value = joint / (parent marginal + 1e-10), built at fit):
//   x_f[q, j] = (1 / F) sum over free-parent sample combos c of
//               P(node = s_j | observed parents = e_q, free parents = c)
// with F = N^(free parents) (node.py:152-193 + torch.mean of
// bayesian_network.py:292), multiplied into the row in the reference's
// factor order; roots and no-observed-parent factors are query-independent
// constants computed once per plan (k_direct_const).  One raw launch (rows +
// one max word per block), then k_scale divides by the global max -- the same
// two steps the sharded path runs around its all-reduce.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "cbn_internal.h"

using namespace cbn;

namespace cbn {

constexpr int kMaxDP = CBN_MAX_DIRECT_PARENTS;

struct DevCpd {
    const float* dense;      // dense CPD (or nullptr)
    const long long* keys;   // hash table keys (-1: empty)
    const float* vals;
    long long mask;          // capacity - 1
};

struct DevDCol {             // one parent column of a direct factor
    const float* dom;        // sorted domain (observed parents)
    const int* sample_idx;   // [N] free-parent sample -> domain idx (-1: none)
    long long stride;        // mixed-radix weight of this column
    int card;
    int ev_slot;             // evidence column or -1 (free)
    int wide;                // observed through .expand(-1, N) from a [Q, N] column (node.py:246-248):
                             // value i of query q is column element q * N + i, averaged like a free
                             // parent's samples (ABI 5, cbn_direct_factor.parent_ev_width)
};

// a combo column of the free-parent mean: a free parent (its plan-time sample
// indices) or a wide observed parent (query q's own N values, looked up in the
// domain per combo)
__device__ __forceinline__ bool combo_col(const DevDCol& c) { return c.ev_slot < 0 || c.wide; }

struct DevDirect {
    int kind;
    int n_parents;
    int n_obs;
    int n_free;
    long long free_combos;   // N^n_free
    const int* node_sample_idx;
    DevCpd cpd;
    int cidx;                // constant factors: row of the plan's const buffer
    int qk;                  // QUERY factors: row of the per-call key buffer (k_direct_keys)
    DevDCol col[kMaxDP];
};

struct DirectPlan {
    int nf = 0;
    int ns = 0;
    int N = 0;
    DevDirect* d_fac = nullptr;
    float* d_const = nullptr;   // [n_const][N]: SCALAR (replicated) / SHARED rows
    int* d_cfac = nullptr;      // [n_const]: factor of each const row
    int n_const = 0;
    int max_slots = 0;
    int nq = 0;                 // QUERY factors
    int* d_qf = nullptr;        // [nq]: factor of each key row
    long long* d_keys = nullptr;  // [nq][Q] observed-parent key of each (factor, query), -1: off-domain
    long long keys_cap = 0;     // elements
    double query_combos = 0;    // sum over QUERY factors of their free-parent combos (per query and column)
};

// Work bounds: a direct factor's free-parent mean loops over
// its F = N^(free parents) combos serially per (query, column) -- the
// reference materialises Q x F x N pdf values for the same factor
// (node.py:335-375).  Two bounds keep every launch short:
// * per thread (plan time): the serial chain of one (query, column) thread --
//   the sum of the QUERY factors' F in k_query_direct, one factor's F in
//   k_direct_const -- is at most 2^26 CPD lookups (~1 s of one thread's
//   latency-bound loop), so even a one-query call cannot run for minutes;
// * per call: Q x N x (sum of the QUERY factors' F) <= 2^40 CPD lookups, and
//   per query-independent factor F x N <= 2^40: split the batch.
constexpr double kDirectCallLookups = 1099511627776.0;  // 2^40
constexpr long long kDirectThreadLookups = 1LL << 26;

}  // namespace cbn

namespace {

#define DHIP_TRY(expr)                                                                    \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return set_err(CBN_E_HIP, "%s failed: %s", #expr, hipGetErrorString(_e));     \
    } while (0)

constexpr int kDThreads = 256;

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebULL;
    x ^= x >> 31;
    return x;
}

__device__ __forceinline__ float hash_get(const long long* __restrict__ keys, const float* __restrict__ vals,
                                          long long mask, long long key) {
    long long h = (long long)(mix64((unsigned long long)key) & (unsigned long long)mask);
    for (long long probe = 0; probe <= mask; ++probe) {
        const long long k = keys[h];
        if (k == key) return vals[h];
        if (k < 0) return 0.f;
        h = (h + 1) & mask;
    }
    return 0.f;
}

__device__ __forceinline__ float cpd_get(const DevCpd& c, long long key) {
    return c.dense ? c.dense[key] : hash_get(c.keys, c.vals, c.mask, key);
}

__device__ __forceinline__ int bsearch_dom(const float* __restrict__ dom, int card, float x) {
    int lo = 0, hi = card;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (dom[mid] < x) lo = mid + 1; else hi = mid;
    }
    return (lo < card && dom[lo] == x) ? lo : -1;
}

__global__ void k_hash_clear(long long* __restrict__ keys, float* __restrict__ vals, long long cap) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < cap; i += (long long)gridDim.x * blockDim.x) {
        keys[i] = -1;
        vals[i] = 0.f;
    }
}

__global__ void k_hash_insert(const long long* __restrict__ in_keys, const float* __restrict__ in_vals, long long n,
                              long long* __restrict__ keys, float* __restrict__ vals, long long mask) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const long long key = in_keys[i];
        long long h = (long long)(mix64((unsigned long long)key) & (unsigned long long)mask);
        for (long long probe = 0; probe <= mask; ++probe) {
            const unsigned long long prev =
                atomicCAS(reinterpret_cast<unsigned long long*>(keys + h), ~0ULL, (unsigned long long)key);
            if (prev == ~0ULL || prev == (unsigned long long)key) {
                vals[h] = in_vals[i];
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

struct RefCols {
    const float* dom[kMaxDP + 1];
    int card[kMaxDP + 1];
    long long stride[kMaxDP + 1];
};

__global__ void k_cpd_ref_eval(DevCpd c, int n_cols, RefCols rc, const float* __restrict__ pts, long long n,
                               float* __restrict__ out) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        long long key = 0;
        bool ok = true;
        for (int k = 0; k < n_cols; ++k) {
            const int idx = bsearch_dom(rc.dom[k], rc.card[k], pts[i * n_cols + k]);
            ok &= idx >= 0;
            key += (long long)(idx < 0 ? 0 : idx) * rc.stride[k];
        }
        out[i] = ok ? cpd_get(c, key) : 0.f;
    }
}

struct DEv {
    const float* p[CBN_MAX_EVIDENCE];
};

// domain index of combo column c's sample i for query q (-1: none / off-domain)
__device__ __forceinline__ int combo_idx(const DevDCol& c, int i, const DEv* ev, long long q, int N) {
    return c.wide ? bsearch_dom(c.dom, c.card, ev->p[c.ev_slot][q * N + i]) : c.sample_idx[i];
}

// sum over a factor's free-parent (and wide-parent) sample combos of the CPD
// at key base + the combo's part (query-independent factors: SHARED = mean
// over the N^k parent sample combos; ev / q: the query, for wide parents)
__device__ double direct_free_mean(const DevDirect& d, long long base, int N, const DEv* ev = nullptr,
                                   long long q = 0) {
    // the combos in the reference's meshgrid order (c = 0 .. F-1, the last
    // free parent varying fastest): the outer loop forms the other free
    // parents' key part (one mixed-radix division chain per N combos), the
    // inner loop walks the last free parent's N samples -- the same terms in
    // the same order as one flat loop over c, so the same fp64 sum
    int pl = -1;
    for (int p = d.n_parents - 1; p >= 0 && pl < 0; --p)
        if (combo_col(d.col[p])) pl = p;
    if (pl < 0) return (double)cpd_get(d.cpd, base);  // F = 1
    const DevDCol& lc = d.col[pl];
    const long long ls = lc.stride;
    const long long outer = d.free_combos / N;
    double s = 0.0;  // fp64 sum, one rounding of the mean (see entry_partial, cbn_infer.hip)
    for (long long o = 0; o < outer; ++o) {
        long long key = base, cc = o;
        bool ok = true;
        for (int p = pl - 1; p >= 0; --p) {
            const DevDCol& col = d.col[p];
            if (combo_col(col)) {
                const long long qq = cc / N;
                const int pi = combo_idx(col, (int)(cc - qq * N), ev, q, N);
                cc = qq;
                ok &= pi >= 0;
                key += (long long)(pi < 0 ? 0 : pi) * col.stride;
            }
        }
        if (!ok) continue;  // N terms of +0.0: s is unchanged (s >= +0)
        for (int j = 0; j < N; ++j) {
            const int pi = combo_idx(lc, j, ev, q, N);
            s += pi >= 0 ? (double)cpd_get(d.cpd, key + (long long)pi * ls) : 0.0;
        }
    }
    return s;
}

__global__ void k_direct_const(const DevDirect* __restrict__ fac, const int* __restrict__ cfac, int n_const, int N,
                               float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_const * N) return;
    const int r = i / N, j = i - r * N;
    const DevDirect& d = fac[cfac[r]];
    float x;
    if (d.kind == CBN_FACTOR_SCALAR) {
        double s = 0.0;
        for (int jj = 0; jj < N; ++jj) {
            const int ni = d.node_sample_idx[jj];
            s += ni >= 0 ? (double)cpd_get(d.cpd, ni) : 0.0;
        }
        x = (float)(s / (double)N);
    } else {
        const int ni = d.node_sample_idx[j];
        x = ni < 0 ? 0.f : (float)(direct_free_mean(d, ni, N) / (double)d.free_combos);
    }
    out[i] = x;
}

// Observed-parent part of each QUERY factor's CPD key, once per (factor,
// query) instead of once per (query, sample column): thread per (k, q), q
// fastest (coalesced evidence reads, wave-uniform factor).  keys[k * Q + q] =
// sum over observed parents of domain index * stride, or -1 when a value is
// outside the fitted domain.
__global__ void __launch_bounds__(kDThreads) k_direct_keys(const DevDirect* __restrict__ fac,
                                                            const int* __restrict__ qf, int nq, DEv ev, long long Q,
                                                            long long* __restrict__ keys) {
    const long long n = (long long)nq * Q;
    for (long long it = blockIdx.x * (long long)blockDim.x + threadIdx.x; it < n;
         it += (long long)gridDim.x * blockDim.x) {
        const int k = (int)(it / Q);
        const long long q = it - (long long)k * Q;
        const DevDirect& d = fac[qf[k]];
        long long base = 0;
        bool ok = true;
        for (int p = 0; p < d.n_parents; ++p) {
            const DevDCol& col = d.col[p];
            if (col.ev_slot >= 0 && !col.wide) {
                const int idx = bsearch_dom(col.dom, col.card, ev.p[col.ev_slot][q]);
                ok &= idx >= 0;
                base += (long long)(idx < 0 ? 0 : idx) * col.stride;
            }
        }
        keys[it] = ok ? base : -1;
    }
}

// one thread per (query, sample column): the product over factors in the
// reference's order; unnormalised rows + one max word per block.  keys: the
// k_direct_keys rows (nullptr: the observed parents are looked up here)
__global__ void __launch_bounds__(kDThreads) k_query_direct(const DevDirect* __restrict__ fac, int nf, int N,
                                                             const float* __restrict__ cst, DEv ev, long long Q,
                                                             const long long* __restrict__ keys,
                                                             unsigned* __restrict__ words, int n_words,
                                                             float* __restrict__ out) {
    const long long n = Q * N;
    unsigned lmaxb = 0;
    for (long long it = blockIdx.x * (long long)blockDim.x + threadIdx.x; it < n;
         it += (long long)gridDim.x * blockDim.x) {
        const long long q = it / N;
        const int j = (int)(it - q * N);
        float acc = 1.f;  // out_pdf = ones (bayesian_network.py:269)
        for (int f = 0; f < nf; ++f) {
            const DevDirect& d = fac[f];
            float x;
            if (d.kind != CBN_FACTOR_QUERY) {
                x = cst[(long long)d.cidx * N + j];
            } else {
                const int ni = d.node_sample_idx[j];
                long long base = ni < 0 ? 0 : ni;
                bool ok = ni >= 0;
                if (keys) {
                    const long long kb = keys[(long long)d.qk * Q + q];
                    ok &= kb >= 0;
                    base += kb < 0 ? 0 : kb;
                } else {
                    for (int p = 0; p < d.n_parents; ++p) {
                        const DevDCol& col = d.col[p];
                        if (col.ev_slot >= 0 && !col.wide) {
                            const int idx = bsearch_dom(col.dom, col.card, ev.p[col.ev_slot][q]);
                            ok &= idx >= 0;
                            base += (long long)(idx < 0 ? 0 : idx) * col.stride;
                        }
                    }
                }
                x = ok ? (float)(direct_free_mean(d, base, N, &ev, q) / (double)d.free_combos) : 0.f;
            }
            acc = acc * x;
        }
        out[it] = acc;
        // non-negative floats: unsigned order == float order, and NaN bits sort
        // above +inf -- a NaN row makes the max NaN, as torch.max does
        lmaxb = max(lmaxb, __float_as_uint(acc));
    }
    // block max -> one word
    __shared__ unsigned wm[kDThreads / kWave];
    unsigned m = lmaxb;
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, kWave));
    if ((threadIdx.x & (kWave - 1)) == 0) wm[threadIdx.x / kWave] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned b = 0;
        for (int i = 0; i < kDThreads / kWave; ++i) b = max(b, wm[i]);
        words[blockIdx.x] = b;
    }
    if (blockIdx.x == 0)
        for (int i = (int)gridDim.x + threadIdx.x; i < n_words; i += blockDim.x) words[i] = 0u;
}

int fill_cols(const cbn_cpd_ref& r, long long* stride, const char* what, int f) {
    if (r.n_cols < 1 || r.n_cols > kMaxDP + 1 || !r.domains || !r.cards)
        return set_err(CBN_E_ARG, "%s %d: bad CPD columns", what, f);
    if (!r.dense && (!r.keys || !r.vals || r.capacity < 2 || (r.capacity & (r.capacity - 1))))
        return set_err(CBN_E_ARG, "%s %d: CPD is neither dense nor a power-of-two hash table", what, f);
    long long s = 1;
    for (int k = r.n_cols - 1; k >= 0; --k) {
        if (r.cards[k] <= 0 || !r.domains[k]) return set_err(CBN_E_ARG, "%s %d: column %d domain", what, f, k);
        stride[k] = s;
        if (s > (1LL << 62) / r.cards[k]) return set_err(CBN_E_LIMIT, "%s %d: prod(cards) >= 2^62", what, f);
        s *= r.cards[k];
    }
    return CBN_OK;
}

DevCpd dev_cpd(const cbn_cpd_ref& r) {
    DevCpd c;
    c.dense = r.dense;
    c.keys = reinterpret_cast<const long long*>(r.keys);
    c.vals = r.vals;
    c.mask = r.dense ? 0 : r.capacity - 1;
    return c;
}

}  // namespace

void cbn::direct_destroy(DirectPlan* dp) {
    if (!dp) return;
    if (dp->d_fac) (void)hipFree(dp->d_fac);
    if (dp->d_const) (void)hipFree(dp->d_const);
    if (dp->d_cfac) (void)hipFree(dp->d_cfac);
    if (dp->d_qf) (void)hipFree(dp->d_qf);
    if (dp->d_keys) (void)hipFree(dp->d_keys);
    delete dp;
}

int cbn::direct_max_words(const DirectPlan* dp) { return dp ? dp->max_slots : 0; }

int cbn::direct_build_consts(DirectPlan* dp, hipStream_t s) {
    if (!dp || dp->n_const == 0) return CBN_OK;
    const int n = dp->n_const * dp->N;
    hipLaunchKernelGGL(k_direct_const, dim3((n + 255) / 256), dim3(256), 0, s, dp->d_fac, dp->d_cfac, dp->n_const,
                       dp->N, dp->d_const);
    DHIP_TRY(hipGetLastError());
    return CBN_OK;
}

int cbn::direct_run(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                    uint32_t* max_bits, float* out, int32_t flags, hipStream_t s) {
    DirectPlan* dp = plan->direct;
    if (n_evidence != dp->ns) return set_err(CBN_E_ARG, "plan expects %d evidence columns, got %d", dp->ns, n_evidence);
    if (n_queries <= 0) return set_err(CBN_E_ARG, "cbn_plan_run: direct plans need >= 1 query");
    if ((double)n_queries * dp->N * dp->query_combos > kDirectCallLookups)
        return set_err(CBN_E_LIMIT,
                       "direct plan: %lld queries x %d columns x %.0f free-parent combos = %.3g CPD lookups > 2^40 in one "
                       "call; split the batch",
                       (long long)n_queries, dp->N, dp->query_combos, (double)n_queries * dp->N * dp->query_combos);
    if (!out || !max_bits) return set_err(CBN_E_ARG, "cbn_plan_run: null output");
    DEv ev;
    memset(&ev, 0, sizeof(ev));
    for (int i = 0; i < n_evidence; ++i) {
        if (!evidence[i]) return set_err(CBN_E_ARG, "null evidence column %d", i);
        ev.p[i] = evidence[i];
    }
    if (flags & CBN_RUN_BUILD_TABLES) {
        const int rc = direct_build_consts(dp, s);
        if (rc) return rc;
    }
    // observed-parent keys once per (factor, query) when N > 1 columns would
    // repeat the lookups (the buffer only grows; hipFree waits for the launches
    // still reading the old one; beyond 256 MiB the query kernel looks the
    // keys up itself)
    long long* keys = nullptr;
    const long long nkeys = (long long)dp->nq * n_queries;
    if (dp->nq > 0 && dp->N > 1 && nkeys * (long long)sizeof(long long) <= (256LL << 20)) {
        if (nkeys > dp->keys_cap) {
            if (dp->d_keys) DHIP_TRY(hipFree(dp->d_keys));
            dp->d_keys = nullptr;
            dp->keys_cap = 0;
            DHIP_TRY(hipMalloc(reinterpret_cast<void**>(&dp->d_keys), sizeof(long long) * nkeys));
            dp->keys_cap = nkeys;
        }
        keys = dp->d_keys;
        const long long kg = std::max(1LL, std::min((nkeys + kDThreads - 1) / kDThreads, 8LL * num_cu()));
        hipLaunchKernelGGL(k_direct_keys, dim3((unsigned)kg), dim3(kDThreads), 0, s, dp->d_fac, dp->d_qf, dp->nq, ev,
                           (long long)n_queries, keys);
        DHIP_TRY(hipGetLastError());
    }
    const long long n = n_queries * (long long)dp->N;
    long long grid = (n + kDThreads - 1) / kDThreads;
    grid = std::max(1LL, std::min(grid, (long long)dp->max_slots));
    const bool raw = (flags & CBN_RUN_RAW) != 0;
    unsigned* words = raw ? max_bits : plan->d_sync + kMaxWordOff;
    hipLaunchKernelGGL(k_query_direct, dim3((unsigned)grid), dim3(kDThreads), 0, s, dp->d_fac, dp->nf, dp->N,
                       dp->d_const, ev, (long long)n_queries, keys, words, dp->max_slots, out);
    DHIP_TRY(hipGetLastError());
    if (raw) return CBN_OK;
    if (reinterpret_cast<uintptr_t>(out) % 16) return set_err(CBN_E_ARG, "cbn_plan_run: out must be 16-B aligned");
    return launch_scale(out, n, words, dp->max_slots, max_bits, s);
}

extern "C" {

int cbn_hash_build(const int64_t* keys, const float* vals, int64_t n, int64_t* table_keys, float* table_vals,
                   int64_t capacity, void* stream) {
    if (n < 0 || capacity < 2 || (capacity & (capacity - 1)) || n > capacity / 2 || !table_keys || !table_vals ||
        (n > 0 && (!keys || !vals)))
        return set_err(CBN_E_ARG, "cbn_hash_build: bad arguments (capacity a power of two >= 2 n)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const long long gc = std::min<long long>((capacity + 255) / 256, 4LL * num_cu());
    hipLaunchKernelGGL(k_hash_clear, dim3((unsigned)gc), dim3(256), 0, s, reinterpret_cast<long long*>(table_keys),
                       table_vals, (long long)capacity);
    DHIP_TRY(hipGetLastError());
    if (n == 0) return CBN_OK;
    const long long gi = std::min<long long>((n + 255) / 256, 4LL * num_cu());
    hipLaunchKernelGGL(k_hash_insert, dim3((unsigned)gi), dim3(256), 0, s, reinterpret_cast<const long long*>(keys),
                       vals, (long long)n, reinterpret_cast<long long*>(table_keys), table_vals,
                       (long long)(capacity - 1));
    DHIP_TRY(hipGetLastError());
    return CBN_OK;
}

int cbn_cpd_ref_eval(const cbn_cpd_ref* cpd, const float* points, int64_t n_points, float* out, void* stream) {
    if (!cpd || n_points < 0 || (n_points > 0 && (!points || !out))) return set_err(CBN_E_ARG, "cbn_cpd_ref_eval: bad arguments");
    RefCols rc;
    memset(&rc, 0, sizeof(rc));
    int e = fill_cols(*cpd, rc.stride, "cpd", 0);
    if (e) return e;
    for (int k = 0; k < cpd->n_cols; ++k) {
        rc.dom[k] = cpd->domains[k];
        rc.card[k] = cpd->cards[k];
    }
    if (n_points == 0) return CBN_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const long long g = std::min<long long>((n_points + 255) / 256, 4LL * num_cu());
    hipLaunchKernelGGL(k_cpd_ref_eval, dim3((unsigned)g), dim3(256), 0, s, dev_cpd(*cpd), cpd->n_cols, rc, points,
                       (long long)n_points, out);
    DHIP_TRY(hipGetLastError());
    return CBN_OK;
}

int cbn_plan_create_direct(const cbn_direct_factor* factors, int32_t n_factors, int32_t n_samples, cbn_plan** plan) {
    if (!plan || !factors || n_factors <= 0 || n_samples <= 0)
        return set_err(CBN_E_ARG, "cbn_plan_create_direct: bad arguments");
    *plan = nullptr;
    const int N = n_samples;
    std::vector<DevDirect> host(n_factors);
    int ns = 0, n_const = 0;
    double query_combos = 0;
    for (int f = 0; f < n_factors; ++f) {
        const cbn_direct_factor& h = factors[f];
        DevDirect& d = host[f];
        memset(&d, 0, sizeof(d));
        if (h.kind < CBN_FACTOR_SCALAR || h.kind > CBN_FACTOR_QUERY)
            return set_err(CBN_E_ARG, "factor %d: bad kind %d", f, h.kind);
        if (h.n_parents < 0 || h.n_parents > kMaxDP)
            return set_err(CBN_E_LIMIT, "factor %d: %d parents > %d", f, h.n_parents, kMaxDP);
        if ((h.kind == CBN_FACTOR_SCALAR) != (h.n_parents == 0)) return set_err(CBN_E_ARG, "factor %d: SCALAR iff root", f);
        if (!h.node_sample_idx) return set_err(CBN_E_ARG, "factor %d: missing node samples", f);
        if (h.cpd.n_cols != h.n_parents + 1) return set_err(CBN_E_ARG, "factor %d: CPD has %d columns", f, h.cpd.n_cols);
        long long stride[kMaxDP + 1];
        int e = fill_cols(h.cpd, stride, "factor", f);
        if (e) return e;
        d.kind = h.kind;
        d.n_parents = h.n_parents;
        d.node_sample_idx = h.node_sample_idx;
        d.cpd = dev_cpd(h.cpd);
        long long F = 1;
        for (int p = 0; p < h.n_parents; ++p) {
            DevDCol& c = d.col[p];
            c.dom = h.cpd.domains[p];
            c.card = h.cpd.cards[p];
            c.stride = stride[p];
            c.ev_slot = h.parent_ev_slot ? h.parent_ev_slot[p] : -1;
            if (c.ev_slot >= CBN_MAX_EVIDENCE) return set_err(CBN_E_ARG, "factor %d: evidence slot %d", f, c.ev_slot);
            const int width = c.ev_slot >= 0 && h.parent_ev_width ? h.parent_ev_width[p] : 1;
            if (width != 1 && width != N)
                return set_err(CBN_E_ARG, "factor %d: parent %d evidence width %d (1 or N = %d)", f, p, width, N);
            c.wide = width != 1 ? 1 : 0;
            if (c.ev_slot >= 0) {
                ++d.n_obs;
                ns = std::max(ns, c.ev_slot + 1);
                if (c.wide) {  // N per-query values: N more combos, like a free parent
                    if (F > kDirectThreadLookups / N)
                        return set_err(CBN_E_LIMIT,
                                       "factor %d: more than 2^26 parent sample combos (one thread's serial loop)", f);
                    F *= N;
                }
            } else {
                if (!h.parent_sample_idx) return set_err(CBN_E_ARG, "factor %d: free parent without samples", f);
                c.sample_idx = h.parent_sample_idx + (long long)p * N;
                ++d.n_free;
                // each (query, column) thread loops over the F free-parent combos
                // serially (work bounds: kDirectThreadLookups / kDirectCallLookups)
                if (F > kDirectThreadLookups / N)
                    return set_err(CBN_E_LIMIT,
                                   "factor %d: more than 2^26 free-parent sample combos (one thread's serial loop)", f);
                F *= N;
            }
        }
        d.free_combos = F;
        if ((h.kind == CBN_FACTOR_QUERY) != (d.n_obs > 0)) return set_err(CBN_E_ARG, "factor %d: QUERY iff some parent observed", f);
        if (h.kind == CBN_FACTOR_QUERY) {
            query_combos += (double)F;
            if (query_combos > (double)kDirectThreadLookups)
                return set_err(CBN_E_LIMIT,
                               "factors up to %d: %.0f free-parent combos per (query, column) > 2^26 (one thread's "
                               "serial loop over every query factor)", f, query_combos);
        } else if ((double)F * N > kDirectCallLookups)
            return set_err(CBN_E_LIMIT, "factor %d: %lld free-parent combos x %d columns > 2^40 CPD lookups", f, F, N);
        if (h.kind != CBN_FACTOR_QUERY) d.cidx = n_const++;
    }
    std::vector<int> qf;
    for (int f = 0; f < n_factors; ++f)
        if (host[f].kind == CBN_FACTOR_QUERY) {
            host[f].qk = (int)qf.size();
            qf.push_back(f);
        }
    DirectPlan* dp = new DirectPlan();
    dp->nf = n_factors;
    dp->ns = ns;
    dp->N = N;
    dp->n_const = n_const;
    dp->max_slots = std::min(4 * num_cu(), kMaxSlots);
    dp->nq = (int)qf.size();
    dp->query_combos = query_combos;
    std::vector<int> cfac;
    for (int f = 0; f < n_factors; ++f)
        if (host[f].kind != CBN_FACTOR_QUERY) cfac.push_back(f);
    cbn_plan* P = new cbn_plan();
    P->nf = n_factors;
    P->ns = ns;
    P->N = N;
    P->direct = dp;
    bool ok = hipMalloc(&dp->d_fac, sizeof(DevDirect) * n_factors) == hipSuccess &&
              hipMalloc(&dp->d_const, sizeof(float) * std::max(1, n_const * N)) == hipSuccess &&
              hipMalloc(&dp->d_cfac, sizeof(int) * std::max(1, n_const)) == hipSuccess &&
              hipMalloc(&dp->d_qf, sizeof(int) * std::max<size_t>(1, qf.size())) == hipSuccess &&
              hipMalloc(&P->d_sync, sizeof(unsigned) * kSyncWords) == hipSuccess;
    ok = ok && hipMemcpy(dp->d_fac, host.data(), sizeof(DevDirect) * n_factors, hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && (cfac.empty() ||
                hipMemcpy(dp->d_cfac, cfac.data(), sizeof(int) * cfac.size(), hipMemcpyHostToDevice) == hipSuccess);
    ok = ok && (qf.empty() ||
                hipMemcpy(dp->d_qf, qf.data(), sizeof(int) * qf.size(), hipMemcpyHostToDevice) == hipSuccess);
    ok = ok && hipMemset(P->d_sync, 0, sizeof(unsigned) * kSyncWords) == hipSuccess;
    if (!ok) {
        cbn_plan_destroy(P);
        return set_err(CBN_E_HIP, "cbn_plan_create_direct: device allocation/upload failed");
    }
    int rc = direct_build_consts(dp, nullptr);
    if (!rc && hipDeviceSynchronize() != hipSuccess) rc = set_err(CBN_E_HIP, "cbn_plan_create_direct: const build failed");
    if (rc) {
        cbn_plan_destroy(P);
        return rc;
    }
    *plan = P;
    return CBN_OK;
}

}  // extern "C"
