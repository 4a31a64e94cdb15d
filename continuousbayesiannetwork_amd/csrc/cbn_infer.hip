// cbn_infer.hip -- MI355X (gfx950) kernels + C ABI for the batched inference
// path of ContinuousBayesianNetwork's BayesianNetwork.infer
// (reference: cbn/base/bayesian_network.py:208-305, cbn/base/node.py:115-375,
//  cbn/parameter_learning/brute_force.py:30-257).
//
// Design:
//   * fit:  the BruteForce maximum-likelihood rows become a dense CPD table per
//           node (k_cpd_scatter / k_cpd_normalize).  The reference instead scans
//           all rows with equality masks on every call (brute_force.py:240-254).
//   * plan: every ancestor factor of the target is marginalised over its free
//           parents ONCE per call into a small table (k_build_tables):
//             SCALAR [1], SHARED [N], QUERY [prod(card of observed parents), N].
//           This is bayesian_network.py:292's torch.mean over parent axes, done
//           on the table instead of on a [Q, N, ..., N] tensor per query.
//   * query: one thread owns VEC consecutive outputs of one query row; it maps
//           each observed value to a domain index by binary search in LDS,
//           gathers the factor rows from the LDS-staged table image and
//           multiplies them in the reference's factor order.  Pass 1 folds the
//           global max (bayesian_network.py:296) with one atomic per block;
//           pass 2 recomputes and writes out/max with 16-B stores.
//   Evidence columns are read straight from the caller's [Q,1] tensors
//   (coalesced along the query axis); nothing is staged through the host.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cbn_amd.h"

namespace {

thread_local std::string g_err;

int set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return set_err(CBN_E_HIP, "%s failed: %s", #expr, hipGetErrorString(_e));     \
    } while (0)

constexpr int kMaxP = CBN_MAX_PARENTS;
constexpr int kWave = 64;
constexpr int kQueryThreads = 1024;
constexpr int kBuildThreads = 256;
constexpr int kLdsBudget = 160 * 1024;
constexpr int kReduceLds = (kQueryThreads / kWave) * sizeof(float);

// Device-side factor descriptor (built once per plan, read with wave-uniform
// indices so the compiler keeps it on the scalar path).
struct DevFactor {
    int kind;
    int n_parents;
    int node_card;
    int n_free;
    int parent_card[kMaxP];
    int ev_slot[kMaxP];
    int cpd_stride[kMaxP];
    int dom_off[kMaxP];        // float offset of observed parent's domain in the image
    const float* cpd;
    const int* node_sample_idx;
    const int* parent_sample_idx;
    long long table_off;       // float offset of this factor's table in the image
    long long rows;            // prod(card of observed parents) (QUERY) or 1
    long long n_entries;       // table entries
    long long free_combos;     // N^n_free
    int wave_mode;             // 1: one wave per entry (many free combos)
    long long unit_begin;      // prefix of work units over factors
    long long n_units;
};

struct EvPtrs {
    const float* p[CBN_MAX_EVIDENCE];
};

struct ColPtrs {
    const float* dom[kMaxP + 1];
    int card[kMaxP + 1];
    int stride[kMaxP + 1];
};

__device__ __forceinline__ int bsearch_eq(const float* __restrict__ dom, int card, float x) {
    int lo = 0, hi = card;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (dom[mid] < x) lo = mid + 1; else hi = mid;
    }
    return (lo < card && dom[lo] == x) ? lo : -1;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    return v;
}

// ---------------------------------------------------------------- fit ------
__global__ void k_cpd_scatter(const int32_t* __restrict__ cell, const float* __restrict__ prob,
                              long long n_rows, float* __restrict__ cpd) {
    for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < n_rows;
         r += (long long)gridDim.x * blockDim.x)
        cpd[cell[r]] = prob[r];  // mle rows are unique -> one writer per cell
}

__global__ void k_cpd_normalize(float* __restrict__ cpd, long long n_pcells, int card) {
    for (long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x; c < n_pcells;
         c += (long long)gridDim.x * blockDim.x) {
        float* row = cpd + c * card;
        float s = 0.f;
        for (int v = 0; v < card; ++v) s += row[v];
        const float den = s + 1e-10f;  // brute_force.py:253-254
        for (int v = 0; v < card; ++v) row[v] = row[v] / den;
    }
}

__global__ void k_cpd_eval(const float* __restrict__ cpd, int n_cols, ColPtrs cols,
                           const float* __restrict__ pts, long long n_pts, float* __restrict__ out) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n_pts;
         i += (long long)gridDim.x * blockDim.x) {
        long long off = 0;
        bool ok = true;
        for (int c = 0; c < n_cols; ++c) {
            const int idx = bsearch_eq(cols.dom[c], cols.card[c], pts[i * n_cols + c]);
            ok &= idx >= 0;
            off += (long long)(idx < 0 ? 0 : idx) * cols.stride[c];
        }
        out[i] = ok ? cpd[off] : 0.f;
    }
}

// --------------------------------------------------------------- tables ----
// Value of one table entry restricted to the free-combo range [c0, c1) with
// step `cs`.  Table entry = (1/F) sum_{free combos} cpd[observed idx, free
// sample idx, node sample idx]; samples not in the domain contribute 0 but
// still count in F (node.py:291-333 pads with off-domain values).
__device__ float entry_partial(const DevFactor& d, long long entry, int N, long long c0,
                               long long c1, long long cs) {
    if (d.kind == CBN_FACTOR_SCALAR) {
        float s = 0.f;
        for (long long j = c0; j < c1; j += cs) {
            const int ni = d.node_sample_idx[j];
            s += ni >= 0 ? d.cpd[ni] : 0.f;
        }
        return s;
    }
    const long long row = entry / N;
    const int j = (int)(entry - row * N);
    const int ni = d.node_sample_idx[j];
    if (ni < 0) return 0.f;
    // observed-parent part of the CPD offset (last observed parent fastest)
    long long base = ni;
    long long r = row;
    for (int p = d.n_parents - 1; p >= 0; --p) {
        if (d.ev_slot[p] >= 0) {
            const int card = d.parent_card[p];
            const long long idx = r % card;
            r /= card;
            base += idx * d.cpd_stride[p];
        }
    }
    float s = 0.f;
    for (long long c = c0; c < c1; c += cs) {
        long long off = base;
        long long cc = c;
        bool ok = true;
        for (int p = d.n_parents - 1; p >= 0; --p) {
            if (d.ev_slot[p] < 0) {
                const int smp = (int)(cc % N);
                cc /= N;
                const int pi = d.parent_sample_idx[p * N + smp];
                ok &= pi >= 0;
                off += (long long)(pi < 0 ? 0 : pi) * d.cpd_stride[p];
            }
        }
        s += ok ? d.cpd[off] : 0.f;
    }
    return s;
}

__global__ void __launch_bounds__(kBuildThreads)
k_build_tables(const DevFactor* __restrict__ fac, int nf, long long total_units, int N,
               float* __restrict__ image, unsigned* __restrict__ max_bits) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && max_bits) *max_bits = 0u;
    const int lane = threadIdx.x & (kWave - 1);
    const long long wave = (blockIdx.x * (long long)blockDim.x + threadIdx.x) / kWave;
    const long long n_waves = (long long)gridDim.x * blockDim.x / kWave;
    for (long long u = wave; u < total_units; u += n_waves) {
        int lo = 0, hi = nf - 1;  // factor owning unit u (wave-uniform)
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (fac[mid].unit_begin <= u) lo = mid; else hi = mid - 1;
        }
        const DevFactor& d = fac[lo];
        const long long lu = u - d.unit_begin;
        const long long F = d.kind == CBN_FACTOR_SCALAR ? (long long)N : d.free_combos;
        if (d.wave_mode) {
            const float s = wave_sum(entry_partial(d, lu, N, lane, F, kWave));
            if (lane == 0) image[d.table_off + lu] = s / (float)F;
        } else {
            const long long e = lu * kWave + lane;
            if (e < d.n_entries) image[d.table_off + e] = entry_partial(d, e, N, 0, F, 1) / (float)F;
        }
    }
}

// ---------------------------------------------------------------- query ----
template <int VEC, bool USE_LDS, bool WRITE>
__global__ void __launch_bounds__(kQueryThreads)
k_query(const DevFactor* __restrict__ fac, int nf, const float* __restrict__ image,
        int image_floats, EvPtrs ev, long long Q, int N, int L,
        unsigned* __restrict__ max_bits, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float4 smem4[];
    const float* img = image;
    if (USE_LDS) {
        const float4* src = reinterpret_cast<const float4*>(image);
        for (int i = threadIdx.x; i < image_floats / 4; i += blockDim.x) smem4[i] = src[i];
        __syncthreads();
        img = reinterpret_cast<const float*>(smem4);
    }
    float maxv = 1.f;
    if (WRITE) maxv = __uint_as_float(*max_bits);
    float lmax = 0.f;
    const long long items = Q * L;
    for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < items;
         g += (long long)gridDim.x * blockDim.x) {
        const long long q = g / L;
        const int l = (int)(g - q * L);
        float acc[VEC];
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] = 1.f;  // out_pdf = ones (bayesian_network.py:269)
        for (int f = 0; f < nf; ++f) {
            const DevFactor& d = fac[f];
            const int kind = d.kind;
            if (kind == CBN_FACTOR_SCALAR) {
                const float v = img[d.table_off];
#pragma unroll
                for (int i = 0; i < VEC; ++i) acc[i] = acc[i] * v;
                continue;
            }
            long long base = d.table_off + (long long)l * VEC;
            bool ok = true;
            if (kind == CBN_FACTOR_QUERY) {
                long long row = 0;
                for (int p = 0; p < d.n_parents; ++p) {
                    const int slot = d.ev_slot[p];
                    if (slot < 0) continue;
                    const int card = d.parent_card[p];
                    const float x = ev.p[slot][q];
                    const int idx = bsearch_eq(img + d.dom_off[p], card, x);
                    ok &= idx >= 0;
                    row = row * card + (idx < 0 ? 0 : idx);
                }
                base += row * N;
            }
            if constexpr (VEC == 4) {
                const float4 t = *reinterpret_cast<const float4*>(img + base);
                const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
                for (int i = 0; i < VEC; ++i) acc[i] = acc[i] * (ok ? tv[i] : 0.f);
            } else {
#pragma unroll
                for (int i = 0; i < VEC; ++i) acc[i] = acc[i] * (ok ? img[base + i] : 0.f);
            }
        }
        if (WRITE) {
            float* o = out + q * N + (long long)l * VEC;
            if constexpr (VEC == 4) {
                *reinterpret_cast<float4*>(o) =
                    make_float4(acc[0] / maxv, acc[1] / maxv, acc[2] / maxv, acc[3] / maxv);
            } else {
#pragma unroll
                for (int i = 0; i < VEC; ++i) o[i] = acc[i] / maxv;
            }
        } else {
#pragma unroll
            for (int i = 0; i < VEC; ++i) lmax = fmaxf(lmax, acc[i]);
        }
    }
    if (!WRITE) {
        // per-wave maxima live after the (16-B padded) image in the dynamic LDS
        float* wmax = reinterpret_cast<float*>(smem4) + (USE_LDS ? image_floats : 0);
        lmax = wave_max(lmax);
        const int w = threadIdx.x / kWave;
        if ((threadIdx.x & (kWave - 1)) == 0) wmax[w] = lmax;
        __syncthreads();
        if (threadIdx.x == 0) {
            float m = 0.f;
            for (int i = 0; i < (int)(blockDim.x / kWave); ++i) m = fmaxf(m, wmax[i]);
            atomicMax(max_bits, __float_as_uint(m));  // values >= 0: uint order == float order
        }
    }
}

int g_num_cu = 0;

int num_cu() {
    if (g_num_cu == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
        g_num_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    }
    return g_num_cu;
}

}  // namespace

struct cbn_plan {
    int nf = 0;
    int N = 0;
    DevFactor* d_fac = nullptr;
    float* d_image = nullptr;     // [tables | observed-parent domains], float4 padded
    int image_floats = 0;
    long long table_floats = 0;
    long long total_units = 0;
    bool use_lds = false;
    int vec = 1;
    int blocks_per_cu = 1;
    std::vector<DevFactor> h_fac;
};

namespace {

template <int VEC, bool LDS, bool WRITE>
int launch_query(cbn_plan* p, long long Q, const EvPtrs& ev, unsigned* max_bits, float* out,
                 hipStream_t s) {
    const int L = p->N / VEC;
    const long long items = Q * (long long)L;
    if (items == 0) return CBN_OK;
    long long blocks = (items + kQueryThreads - 1) / kQueryThreads;
    const long long cap = (long long)num_cu() * p->blocks_per_cu;
    if (blocks > cap) blocks = cap;
    const size_t lds = (LDS ? (size_t)p->image_floats * sizeof(float) : 0) + kReduceLds;
    hipLaunchKernelGGL((k_query<VEC, LDS, WRITE>), dim3((unsigned)blocks), dim3(kQueryThreads), lds, s,
                       p->d_fac, p->nf, p->d_image, p->image_floats, ev, Q, p->N, L, max_bits, out);
    HIP_TRY(hipGetLastError());
    return CBN_OK;
}

template <bool WRITE>
int dispatch_query(cbn_plan* p, long long Q, const float* const* evidence, int n_ev,
                   unsigned* max_bits, float* out, hipStream_t s) {
    if (n_ev < 0 || n_ev > CBN_MAX_EVIDENCE) return set_err(CBN_E_LIMIT, "n_evidence %d out of range", n_ev);
    EvPtrs ev;
    memset(&ev, 0, sizeof(ev));
    for (int i = 0; i < n_ev; ++i) ev.p[i] = evidence[i];
    if (p->vec == 4) {
        return p->use_lds ? launch_query<4, true, WRITE>(p, Q, ev, max_bits, out, s)
                          : launch_query<4, false, WRITE>(p, Q, ev, max_bits, out, s);
    }
    return p->use_lds ? launch_query<1, true, WRITE>(p, Q, ev, max_bits, out, s)
                      : launch_query<1, false, WRITE>(p, Q, ev, max_bits, out, s);
}

template <int VEC, bool WRITE>
void allow_big_lds() {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_query<VEC, true, WRITE>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBudget);
}

}  // namespace

// ================================================================ C ABI ====
extern "C" {

int cbn_abi_version(void) { return CBN_AMD_ABI_VERSION; }

const char* cbn_last_error(void) { return g_err.c_str(); }

int cbn_bf_cpd_build(const int32_t* cell, const float* prob, int64_t n_rows, int64_t n_parent_cells,
                     int32_t node_card, int32_t normalize, float* cpd, void* stream) {
    if (!cpd || node_card <= 0 || n_parent_cells <= 0 || n_rows < 0 || (n_rows > 0 && (!cell || !prob)))
        return set_err(CBN_E_ARG, "cbn_bf_cpd_build: bad arguments");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    HIP_TRY(hipMemsetAsync(cpd, 0, sizeof(float) * (size_t)n_parent_cells * node_card, s));
    if (n_rows > 0) {
        const long long blocks = std::min<long long>((n_rows + 255) / 256, 4096);
        hipLaunchKernelGGL(k_cpd_scatter, dim3((unsigned)blocks), dim3(256), 0, s, cell, prob,
                           (long long)n_rows, cpd);
        HIP_TRY(hipGetLastError());
    }
    if (normalize) {
        const long long blocks = std::min<long long>((n_parent_cells + 255) / 256, 4096);
        hipLaunchKernelGGL(k_cpd_normalize, dim3((unsigned)blocks), dim3(256), 0, s, cpd,
                           (long long)n_parent_cells, (int)node_card);
        HIP_TRY(hipGetLastError());
    }
    return CBN_OK;
}

int cbn_bf_cpd_eval(const float* cpd, int32_t n_cols, const float* const* domains,
                    const int32_t* domain_card, const float* points, int64_t n_points, float* out,
                    void* stream) {
    if (n_cols <= 0 || n_cols > kMaxP + 1) return set_err(CBN_E_LIMIT, "cbn_bf_cpd_eval: n_cols %d", n_cols);
    if (!cpd || !domains || !domain_card || (n_points > 0 && (!points || !out)))
        return set_err(CBN_E_ARG, "cbn_bf_cpd_eval: null pointer");
    ColPtrs cols;
    memset(&cols, 0, sizeof(cols));
    int stride = 1;
    for (int c = n_cols - 1; c >= 0; --c) {
        if (domain_card[c] <= 0) return set_err(CBN_E_ARG, "cbn_bf_cpd_eval: empty domain");
        cols.dom[c] = domains[c];
        cols.card[c] = domain_card[c];
        cols.stride[c] = stride;
        stride *= domain_card[c];
    }
    if (n_points == 0) return CBN_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const long long blocks = std::min<long long>((n_points + 255) / 256, 8192);
    hipLaunchKernelGGL(k_cpd_eval, dim3((unsigned)blocks), dim3(256), 0, s, cpd, (int)n_cols, cols,
                       points, (long long)n_points, out);
    HIP_TRY(hipGetLastError());
    return CBN_OK;
}

int cbn_plan_create(const cbn_factor_desc* factors, int32_t n_factors, int32_t n_samples, cbn_plan** plan) {
    if (!plan || !factors || n_factors <= 0 || n_samples <= 0)
        return set_err(CBN_E_ARG, "cbn_plan_create: bad arguments");
    *plan = nullptr;
    const int N = n_samples;
    std::vector<DevFactor> fac(n_factors);
    long long off = 0, units = 0;
    for (int f = 0; f < n_factors; ++f) {
        const cbn_factor_desc& h = factors[f];
        DevFactor& d = fac[f];
        memset(&d, 0, sizeof(d));
        if (h.kind < CBN_FACTOR_SCALAR || h.kind > CBN_FACTOR_QUERY)
            return set_err(CBN_E_ARG, "factor %d: bad kind %d", f, h.kind);
        if (h.n_parents < 0 || h.n_parents > kMaxP)
            return set_err(CBN_E_LIMIT, "factor %d: %d parents > %d", f, h.n_parents, kMaxP);
        if ((h.kind == CBN_FACTOR_SCALAR) != (h.n_parents == 0))
            return set_err(CBN_E_ARG, "factor %d: SCALAR iff root", f);
        if (!h.cpd || !h.node_sample_idx || h.node_card <= 0)
            return set_err(CBN_E_ARG, "factor %d: missing cpd/node samples", f);
        d.kind = h.kind;
        d.n_parents = h.n_parents;
        d.node_card = h.node_card;
        d.cpd = h.cpd;
        d.node_sample_idx = h.node_sample_idx;
        d.parent_sample_idx = h.parent_sample_idx;
        long long stride = h.node_card;
        int n_ev = 0;
        long long rows = 1, F = 1;
        for (int p = h.n_parents - 1; p >= 0; --p) {
            if (h.parent_card[p] <= 0) return set_err(CBN_E_ARG, "factor %d: parent %d card", f, p);
            d.parent_card[p] = h.parent_card[p];
            d.ev_slot[p] = h.parent_ev_slot[p];
            d.cpd_stride[p] = (int)stride;
            stride *= h.parent_card[p];
            if (stride > (1LL << 31)) return set_err(CBN_E_LIMIT, "factor %d: CPD too large", f);
            if (h.parent_ev_slot[p] >= 0) {
                if (h.parent_ev_slot[p] >= CBN_MAX_EVIDENCE || !h.parent_domain[p])
                    return set_err(CBN_E_ARG, "factor %d: bad evidence slot/domain", f);
                ++n_ev;
                rows *= h.parent_card[p];
            } else {
                if (!h.parent_sample_idx) return set_err(CBN_E_ARG, "factor %d: free parent without samples", f);
                F *= N;
                if (F > (1LL << 40)) return set_err(CBN_E_LIMIT, "factor %d: too many free combos", f);
                d.n_free++;
            }
        }
        if ((h.kind == CBN_FACTOR_QUERY) != (n_ev > 0))
            return set_err(CBN_E_ARG, "factor %d: QUERY iff some parent observed", f);
        d.rows = rows;
        d.free_combos = F;
        d.n_entries = h.kind == CBN_FACTOR_SCALAR ? 1 : rows * N;
        const long long F_eff = h.kind == CBN_FACTOR_SCALAR ? N : F;
        d.wave_mode = F_eff >= kWave ? 1 : 0;
        d.n_units = d.wave_mode ? d.n_entries : (d.n_entries + kWave - 1) / kWave;
        d.unit_begin = units;
        units += d.n_units;
        d.table_off = off;
        off += (d.n_entries + 3) & ~3LL;
    }
    const long long table_floats = off;
    // observed-parent domains appended after the tables (one copy per use)
    std::vector<std::pair<const float*, int>> doms;
    for (int f = 0; f < n_factors; ++f) {
        for (int p = 0; p < fac[f].n_parents; ++p) {
            if (fac[f].ev_slot[p] >= 0) {
                fac[f].dom_off[p] = (int)off;
                doms.push_back({factors[f].parent_domain[p], fac[f].parent_card[p]});
                off += (fac[f].parent_card[p] + 3) & ~3LL;
            }
        }
    }
    if (off > (1LL << 30)) return set_err(CBN_E_LIMIT, "plan image too large");
    cbn_plan* P = new cbn_plan();
    P->nf = n_factors;
    P->N = N;
    P->image_floats = (int)off;
    P->table_floats = table_floats;
    P->total_units = units;
    P->vec = (N % 4 == 0) ? 4 : 1;
    const long long bytes = off * (long long)sizeof(float);
    P->use_lds = bytes + kReduceLds <= kLdsBudget;
    // 1024-thread blocks: at most 2 per CU (32 waves); LDS may allow only 1
    P->blocks_per_cu = P->use_lds ? (2 * (bytes + kReduceLds) <= kLdsBudget ? 2 : 1) : 2;
    P->h_fac = fac;
    if (hipMalloc(&P->d_fac, sizeof(DevFactor) * n_factors) != hipSuccess ||
        hipMalloc(&P->d_image, sizeof(float) * std::max<long long>(off, 4)) != hipSuccess) {
        cbn_plan_destroy(P);
        return set_err(CBN_E_HIP, "cbn_plan_create: hipMalloc failed");
    }
    if (hipMemcpy(P->d_fac, fac.data(), sizeof(DevFactor) * n_factors, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(P->d_image, 0, sizeof(float) * std::max<long long>(off, 4)) != hipSuccess) {
        cbn_plan_destroy(P);
        return set_err(CBN_E_HIP, "cbn_plan_create: upload failed");
    }
    long long pos = table_floats;
    for (auto& dm : doms) {
        if (hipMemcpy(P->d_image + pos, dm.first, sizeof(float) * dm.second, hipMemcpyDeviceToDevice) != hipSuccess) {
            cbn_plan_destroy(P);
            return set_err(CBN_E_HIP, "cbn_plan_create: domain copy failed");
        }
        pos += (dm.second + 3) & ~3LL;
    }
    if (P->use_lds) {
        allow_big_lds<4, false>(); allow_big_lds<4, true>();
        allow_big_lds<1, false>(); allow_big_lds<1, true>();
    }
    *plan = P;
    return CBN_OK;
}

int cbn_plan_destroy(cbn_plan* plan) {
    if (!plan) return CBN_OK;
    if (plan->d_fac) (void)hipFree(plan->d_fac);
    if (plan->d_image) (void)hipFree(plan->d_image);
    delete plan;
    return CBN_OK;
}

int64_t cbn_plan_table_bytes(const cbn_plan* plan) {
    return plan ? (int64_t)plan->image_floats * (int64_t)sizeof(float) : -1;
}

int cbn_plan_uses_lds(const cbn_plan* plan) { return plan && plan->use_lds ? 1 : 0; }

int cbn_plan_build_tables(cbn_plan* plan, uint32_t* max_bits, void* stream) {
    if (!plan) return set_err(CBN_E_ARG, "null plan");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    long long waves = plan->total_units;
    long long blocks = (waves * kWave + kBuildThreads - 1) / kBuildThreads;
    if (blocks > (long long)num_cu() * 8) blocks = (long long)num_cu() * 8;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_build_tables, dim3((unsigned)blocks), dim3(kBuildThreads), 0, s, plan->d_fac,
                       plan->nf, plan->total_units, plan->N, plan->d_image, max_bits);
    HIP_TRY(hipGetLastError());
    return CBN_OK;
}

int cbn_plan_query_max(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                       uint32_t* max_bits, void* stream) {
    if (!plan || !max_bits || n_queries < 0) return set_err(CBN_E_ARG, "cbn_plan_query_max: bad arguments");
    return dispatch_query<false>(plan, n_queries, evidence, n_evidence, max_bits, nullptr,
                                 reinterpret_cast<hipStream_t>(stream));
}

int cbn_plan_query_write(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                         const uint32_t* max_bits, float* out, void* stream) {
    if (!plan || !max_bits || n_queries < 0 || (n_queries > 0 && !out))
        return set_err(CBN_E_ARG, "cbn_plan_query_write: bad arguments");
    return dispatch_query<true>(plan, n_queries, evidence, n_evidence, const_cast<uint32_t*>(max_bits), out,
                                reinterpret_cast<hipStream_t>(stream));
}

int cbn_plan_infer(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                   uint32_t* max_bits, float* out, void* stream) {
    int rc = cbn_plan_build_tables(plan, max_bits, stream);
    if (rc) return rc;
    rc = cbn_plan_query_max(plan, n_queries, evidence, n_evidence, max_bits, stream);
    if (rc) return rc;
    return cbn_plan_query_write(plan, n_queries, evidence, n_evidence, max_bits, out, stream);
}

}  // extern "C"
