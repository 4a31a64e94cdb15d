// cbn_infer.hip -- MI355X (gfx950) kernels + C ABI for the batched inference
// path of ContinuousBayesianNetwork's BayesianNetwork.infer
// (reference: cbn/base/bayesian_network.py:208-305, cbn/base/node.py:115-375,
//  cbn/parameter_learning/brute_force.py:17-244).
//
// Design:
//   * fit:  the BruteForce maximum-likelihood rows become a dense CPD table per
//           node (k_cpd_scatter / k_cpd_normalize).  The reference instead scans
//           all rows with equality masks on every call (brute_force.py:227-241).
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
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include <unistd.h>  // environ

#include "cbn_internal.h"

using namespace cbn;

namespace {
thread_local std::string g_err;
}  // namespace

// Diagnostic switches (same-box A/B builds under tools/: CBN_NO_STAGED,
// CBN_FAST_VPL, CBN_PARAM_GENERIC, ...) are honoured only when CBN_DIAG=1 is
// set when the library is loaded, so a stray variable in a serving process
// cannot swap kernels; with CBN_DIAG=1 every CBN_* variable of the
// environment is listed on stderr at load (ADVICE / VERDICT r04).
namespace {
const bool g_diag = [] {
    const char* e = getenv("CBN_DIAG");
    const bool on = e && e[0] == '1' && e[1] == 0;
    if (on)
        for (char** v = environ; v && *v; ++v)
            if (!strncmp(*v, "CBN_", 4) && strncmp(*v, "CBN_DIAG=", 9))
                fprintf(stderr, "[libcbn_amd] CBN_DIAG=1: diagnostic override %s\n", *v);
    return on;
}();
}  // namespace

const char* cbn::diag_env(const char* name) { return g_diag ? getenv(name) : nullptr; }

int cbn::set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

namespace cbn {
// Device-side factor descriptor (built once per plan, read with wave-uniform
// indices so the compiler keeps it on the scalar path).
struct DevFactor {
    int kind;
    int n_parents;
    int node_card;
    int n_free;
    int parent_card[CBN_MAX_PARENTS];
    int ev_slot[CBN_MAX_PARENTS];
    int cpd_stride[CBN_MAX_PARENTS];
    const float* cpd;
    const int* node_sample_idx;
    const int* parent_sample_idx;
    int table_off;   // float offset of this factor's table ([rows][RS]) in the image
    int rows;        // prod(card of observed parents) (QUERY) or 1
    int n_entries;   // rows * N
    int free_combos; // N^n_free
    int wave_mode;   // build kernel: 1 = one wave per entry (many free combos)
};

struct QSlot {
    int dom_off;  // float offset of the sorted domain in the image
    int card;
    int dense;    // 1: domain is exactly {0, 1, ..., card-1} -> index = value
    int pad;
};

struct BuildItem {
    int factor;
    int unit_begin;
};
}  // namespace cbn

namespace {

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return set_err(CBN_E_HIP, "%s failed: %s", #expr, hipGetErrorString(_e));     \
    } while (0)

constexpr int kMaxP = CBN_MAX_PARENTS;
constexpr int kQueryThreads = 1024;
constexpr int kBuildThreads = 256;

struct EvPtrs {
    const float* p[CBN_MAX_EVIDENCE];
};

// Fast path: evidence column of observed parent p of factor f at [f * 4 + p]
// (nullptr: no such parent), built by the host per call and copied into LDS at
// kernel entry (during the table fill), so after the fill a lane reaches its
// evidence with one LDS read instead of record -> slot -> column-pointer hops.
// Entry [f * 4] is never null and carries tags in its low bits (columns are
// 4-B aligned): kTagMore = the factor has further observed parents,
// kTagNone = no observed parent (a valid dummy column, read at row 0), so the
// first-parent loads of all a lane's factors issue back to back, unbranched.
constexpr uintptr_t kTagMore = 1, kTagNone = 2;
// Kernel arguments are copied per launch: plans of <= 32 factors (configs[1],
// [2]) take a 1 KiB table (launch 3.2 us of host time instead of 4.9 us with
// the 3.3 KiB one, profiles/r01_launch_cost.txt).
constexpr int kFastPtrsSmall = 128;
template <int NP>
struct FPtrsT {
    const float* p[NP];
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

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    return v;
}

__device__ __forceinline__ unsigned wave_max_u(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (unsigned)__shfl_xor((int)v, o, kWave));
    return v;
}

// Diagnostic build only (-DCBN_STAMPS): per-wave s_memtime stamps of the query
// kernels' phases into a debug buffer (never read by the kernels themselves).
#ifdef CBN_STAMPS
__device__ unsigned long long* g_stamps = nullptr;
// the buffer pointer is read ONCE per wave (CBN_STAMP_INIT, after stamp 0's
// clock read); a stamp is then one s_memrealtime + one un-waited store
// Clock ring (round 5): per launch of k_query_staged,
// block 0 / thread 0 records {shader cycles (s_memtime), 100 MHz ticks
// (s_memrealtime)} at entry and after its final stores -- block 0 waits in the
// grid barrier for every other block, so its span is the launch's, and the
// ratio of the two is the shader clock the launch ran at.  Plain vector
// stores by one lane; launches on one stream run one after the other.
constexpr unsigned kClockRing = 4096;
__device__ unsigned long long* g_clock = nullptr;  // [launch][4]
__device__ unsigned g_clock_n = 0;
#define CBN_STAMP_INIT                                                                        \
    const unsigned long long _t0 = __builtin_amdgcn_s_memrealtime();                          \
    const unsigned long long _m0 = __builtin_amdgcn_s_memtime();                              \
    (void)_m0;                                                                                \
    unsigned long long* const _stp = g_stamps;                                                \
    if (_stp && (threadIdx.x & 63) == 0)                                                      \
        _stp[((size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 12] = _t0
#define CBN_STAMP(k)                                                                          \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        unsigned long long _t = __builtin_amdgcn_s_memrealtime(); /* 100 MHz, chip-wide */   \
        if (_stp && (threadIdx.x & 63) == 0)                                                  \
            _stp[((size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 12 + (k)] = _t; \
        __builtin_amdgcn_sched_barrier(0);                                                    \
    } while (0)
#define CBN_CLOCK_END                                                                         \
    do {                                                                                      \
        unsigned long long* const _ck = g_clock;                                              \
        if (_ck && blockIdx.x == 0 && threadIdx.x == 0) {                                     \
            const unsigned long long _m1 = __builtin_amdgcn_s_memtime();                      \
            const unsigned long long _r1 = __builtin_amdgcn_s_memrealtime();                  \
            const unsigned _i = g_clock_n;                                                    \
            if (_i < kClockRing) {                                                            \
                _ck[4 * _i] = _m0;                                                            \
                _ck[4 * _i + 1] = _t0;                                                        \
                _ck[4 * _i + 2] = _m1;                                                        \
                _ck[4 * _i + 3] = _r1;                                                        \
            }                                                                                 \
            g_clock_n = _i + 1;                                                               \
        }                                                                                     \
    } while (0)
#else
#define CBN_STAMP_INIT do {} while (0)
#define CBN_STAMP(k) do {} while (0)
#define CBN_CLOCK_END do {} while (0)
#endif

// Diagnostic build only (-DCBN_CHECKED): validate global addresses in the
// fast query kernel before use; a violation is recorded and the access skipped.
#ifdef CBN_CHECKED
__device__ unsigned* g_dbg = nullptr;
#define CBN_OK_OR(cond, code) ((cond) ? true : (g_dbg ? (atomicOr(g_dbg, 1u << (code)), atomicAdd(g_dbg + 1 + (code), 1u), false) : false))
#else
#define CBN_OK_OR(cond, code) true
#endif

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) float gfloat_t;

// Load through a pointer that came from LDS as a GLOBAL load: a generic
// pointer compiles to flat_load, which the compiler fences with vmcnt(0) +
// lgkmcnt(0) and so serialises a batch of evidence loads.
__device__ __forceinline__ float gload(const float* p, long long i) {
    return ((gfloat_t*)p)[i];
}
typedef const __attribute__((address_space(1))) void gbl_void_t;
typedef const __attribute__((address_space(4))) int cint_t;

// Output rows are stored WRITE-THROUGH (sc1: the line leaves the XCD's L2 at
// once instead of staying dirty): a launch that ends with 8 MB of plain stores
// makes the next dependent launch wait for their write-back (the price
// table's "boundary" row: + bytes / 6 TB/s).  rsrc = a buffer descriptor over
// this block's rows (wave-uniform base and size), off = byte offset in it.
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(float* base, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff), 0x00020000);
}
__device__ __forceinline__ void store_wt(__amdgpu_buffer_rsrc_t r, int off, float4 v) {
    u32x4_t x = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
#ifndef CBN_STORE_AUX
#define CBN_STORE_AUX 16
#endif
    __builtin_amdgcn_raw_buffer_store_b128(x, r, off, 0, CBN_STORE_AUX);  // aux 16 = sc1
}

// Four ints through the constant address space: at a wave-uniform address that
// is one s_load_dwordx4 (a generic load issued after LDS-DMA or other writes
// would be a vector load: the compiler cannot prove the memory unclobbered).
__device__ __forceinline__ int4 sload_int4(const void* p) {
    const cint_t* q = reinterpret_cast<const cint_t*>(reinterpret_cast<uintptr_t>(p));
    return make_int4(q[0], q[1], q[2], q[3]);
}

// Copy n4 float4 from global to LDS with LDS-DMA (global_load_lds_dwordx4: no
// VGPR staging; one wave-instruction moves 1 KiB).  Chunk order is rotated by
// block so the CUs do not all hit the same L2 channel at once.  Completion is
// awaited by the caller's __syncthreads() (it waits vmcnt(0)).
__device__ __forceinline__ void lds_dma_copy(const float* __restrict__ g, float4* lds, int n4,
                                             int nw = kQueryThreads / kWave) {
    // nw: waves per block (a compile-time default: reading blockDim costs a
    // kernel-argument line fetch on the launch's critical path)
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int nchunk = (n4 + kWave - 1) / kWave;
    for (int c0 = wave; c0 < nchunk; c0 += nw) {
        const int c = (c0 + (int)blockIdx.x) % nchunk;
        const int i = c * kWave + lane;
        if (i < n4 && CBN_OK_OR(i >= 0, 0))
            __builtin_amdgcn_global_load_lds((gbl_void_t*)(g + (size_t)i * 4), (lds_void_t*)(lds + c * kWave), 16,
                                             0, 0);
    }
}

// ---------------------------------------------------------------- fit ------
__global__ void k_cpd_scatter(const int32_t* __restrict__ cell, const float* __restrict__ prob,
                              long long n_rows, float* __restrict__ cpd) {
    for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < n_rows;
         r += (long long)gridDim.x * blockDim.x)
        cpd[cell[r]] = prob[r];  // mle rows are unique -> one writer per cell
}

// The parent marginal is summed in fp64 and rounded once (round 6): the
// reference's fp32 sum (torch's cascaded reduction over the unique rows,
// brute_force.py:236-238) is within a couple of ulp of the exact sum, while a
// sequential fp32 sum of a peaked row (one dominant joint among 64) drifts by
// several ulp in a consistent direction -- 3.5e-5 relative over the 100
// factors of the configs[4] grid at 400 000 training rows
// (tests/test_gpu_parity.py::test_grid_bench_batch_full_size).  Fit time only.
__global__ void k_cpd_normalize(float* __restrict__ cpd, long long n_pcells, int card) {
    for (long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x; c < n_pcells;
         c += (long long)gridDim.x * blockDim.x) {
        float* row = cpd + c * card;
        double s = 0.0;
        for (int v = 0; v < card; ++v) s += (double)row[v];
        const float den = (float)s + 1e-10f;  // brute_force.py:240-241 (fp32, as the reference)
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
// Table entry = (1/F) sum over free-parent sample combos of
// cpd[observed idx, free sample idx, node sample idx]; samples not in the
// domain contribute 0 but still count in F (node.py:291-333 pads with
// off-domain values).  SCALAR (root) tables hold the mean over the N node
// samples, replicated over the N columns.  int32 index math throughout
// (plan_create bounds every table and CPD below 2^31).  The sums run in fp64
// and the mean is rounded to fp32 once: the reference's torch.mean over the
// meshgrid axes (bayesian_network.py:271-293; node.py:206-284 repeats each
// observed value N times, so at d = N = 64 one free parent is 4 096 combos)
// is a cascaded fp32 reduction within a few ulp of the exact mean; a plain
// fp32 running sum over F terms drifts by up to F/2 ulp.
__device__ double entry_partial(const DevFactor& d, int entry, int N, int c0, int c1, int cs) {
    if (d.kind == CBN_FACTOR_SCALAR) {
        double s = 0.0;
        for (int j = c0; j < c1; j += cs) {
            const int ni = d.node_sample_idx[j];
            s += ni >= 0 ? (double)d.cpd[ni] : 0.0;
        }
        return s;
    }
    const int row = entry / N;
    const int j = entry - row * N;
    const int ni = d.node_sample_idx[j];
    if (ni < 0) return 0.0;
    int base = ni;  // observed-parent part of the CPD offset (last observed parent fastest)
    int r = row;
    for (int p = d.n_parents - 1; p >= 0; --p) {
        if (d.ev_slot[p] >= 0) {
            const int card = d.parent_card[p];
            const int q = r / card;
            base += (r - q * card) * d.cpd_stride[p];
            r = q;
        }
    }
    double s = 0.0;
    for (int c = c0; c < c1; c += cs) {
        int off = base;
        int cc = c;
        bool ok = true;
        for (int p = d.n_parents - 1; p >= 0; --p) {
            if (d.ev_slot[p] < 0) {
                const int q = cc / N;
                const int pi = d.parent_sample_idx[p * N + (cc - q * N)];
                cc = q;
                ok &= pi >= 0;
                off += (pi < 0 ? 0 : pi) * d.cpd_stride[p];
            }
        }
        s += ok ? (double)d.cpd[off] : 0.0;
    }
    return s;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

__global__ void __launch_bounds__(kBuildThreads)
k_build_tables(const DevFactor* __restrict__ fac, const BuildItem* __restrict__ items, int n_items,
               int total_units, int N, int RS, float* __restrict__ image) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    const int n_waves = gridDim.x * blockDim.x / kWave;
    for (int u = wave; u < total_units; u += n_waves) {
        int lo = 0, hi = n_items - 1;  // build item owning unit u (wave-uniform)
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (items[mid].unit_begin <= u) lo = mid; else hi = mid - 1;
        }
        const DevFactor& d = fac[items[lo].factor];
        const int lu = u - items[lo].unit_begin;
        const int F = d.kind == CBN_FACTOR_SCALAR ? N : (int)d.free_combos;
        float* tab = image + d.table_off;
        // table rows are RS >= N floats apart (padding spreads LDS banks)
        if (d.wave_mode) {
            const double s = wave_sum_d(entry_partial(d, lu, N, lane, F, kWave));
            if (lane == 0) tab[(lu / N) * RS + lu % N] = (float)(s / (double)F);
        } else {
            const int e = lu * kWave + lane;
            if (e < d.n_entries) tab[(e / N) * RS + e % N] = (float)(entry_partial(d, e, N, 0, F, 1) / (double)F);
        }
    }
}

// ---------------------------------------------------------------- query ----
// Per-factor record staged in LDS for the query prologue.
// Prefix merge (staged plans): the reference's product starts from ones, so
// 1 * x_0 = x_0 exactly and the first factors of a query-independent prefix
// (1-row tables: roots, unobserved-parent factors) fold EXACTLY into the first
// multi-row factor's table: T_k'[r][j] = (((x_0[j] * x_1[j]) ...) * T_k[r][j])
// in the reference's order -- the value the query kernel would hold after
// factor k.  The staged kernel then starts at factor k (fewer LDS row reads).
// offs: table offsets of factors 0..k (k <= 8).
struct PrefixOffs {
    int off[9];
};
__global__ void __launch_bounds__(256) k_merge_prefix(float* __restrict__ image, PrefixOffs po, int k, int rows, int N,
                                                        int RS) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= rows * N) return;
    const int r = e / N, j = e % N;
    float v = image[po.off[0] + j];
    for (int i = 1; i < k; ++i) v = v * image[po.off[i] + j];
    float* t = image + po.off[k] + (long long)r * RS + j;
    *t = v * *t;
}

constexpr int kFqInts = 4 + 2 * kMaxP;  // img_off, kind, n_obs, pad, obs_slot[], obs_card[]
constexpr int kUnroll = 4;

__device__ __forceinline__ int slot_index(const float* __restrict__ img, const QSlot& sl, float x) {
    if (sl.dense) {
        const int i = (int)x;
        return (x >= 0.f && x < (float)sl.card && (float)i == x) ? i : -1;
    }
    return bsearch_eq(img + sl.dom_off, sl.card, x);
}

// One launch = one pass over the queries.  Block b owns the contiguous query
// range [q0, q1); L lanes x VEC values cover one query row.
//   fill : LDS image <- table image built by k_build_tables (+ domains), one
//          flat float4 copy with kUnroll independent loads in flight per lane
//   A1   : sidx[q][s] = domain index of evidence column s for query q; the
//          evidence loads of a chunk are issued back-to-back (kUnroll per lane,
//          consecutive lanes -> consecutive queries of one column)
//   A2   : offs[q][f] = image offset of factor f's row for query q (-1: value
//          outside the fitted domain -> the reference's 0 factor)
//   B    : acc = prod_f table_f[offs[q][f] + lane cols] in the reference's
//          factor order (bayesian_network.py:271-294)
// WRITE=false publishes max(acc) (last block to arrive); WRITE=true stores acc/max.
template <int VEC, bool USE_LDS, bool WRITE>
__global__ void __launch_bounds__(kQueryThreads)
k_query(const DevFactor* __restrict__ fac, int nf, const QSlot* __restrict__ slots, int ns,
        const float* __restrict__ gimage, int image_floats, EvPtrs ev, long long Q, int N, int RS, int L, int CH,
        unsigned* __restrict__ sync, unsigned* __restrict__ max_bits, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float4 smem4[];
    float* simg = reinterpret_cast<float*>(smem4);
    int* fq = reinterpret_cast<int*>(simg + (USE_LDS ? image_floats : 0));  // nf * kFqInts
    QSlot* sslot = reinterpret_cast<QSlot*>(fq + nf * kFqInts);             // ns
    int* sidx = reinterpret_cast<int*>(sslot + ns);                         // CH * ns
    int* offs = sidx + CH * ns;                                              // CH * nf
    float* wmax = reinterpret_cast<float*>(offs + CH * nf);                 // 16
    const float** sev = reinterpret_cast<const float**>(wmax + 16);        // ns pointers
    const int tid = threadIdx.x;
    const int nthr = blockDim.x;
    if (tid < ns) sev[tid] = ev.p[tid];

    // ---- fill
    if (USE_LDS) lds_dma_copy(gimage, smem4, image_floats / 4);
    for (int f = tid; f < nf; f += nthr) {
        const DevFactor& d = fac[f];
        int* r = fq + f * kFqInts;
        r[0] = d.table_off;
        r[1] = d.kind;
        int n_obs = 0;
        for (int p = 0; p < d.n_parents; ++p) {
            if (d.ev_slot[p] >= 0) {
                r[4 + n_obs] = d.ev_slot[p];
                r[4 + kMaxP + n_obs] = d.parent_card[p];
                ++n_obs;
            }
        }
        r[2] = n_obs;
    }
    for (int s = tid; s < ns; s += nthr) sslot[s] = slots[s];
    __syncthreads();
    const float* img = USE_LDS ? simg : gimage;

    float maxv = 1.f;
    if (WRITE) maxv = __uint_as_float(*max_bits);
    float lmax = 0.f;
    const long long per = (Q + gridDim.x - 1) / gridDim.x;
    const long long q0 = (long long)blockIdx.x * per;
    const long long q1 = q0 + per < Q ? q0 + per : Q;
    for (long long base = q0; base < q1; base += CH) {
        const int cnt = (int)(q1 - base < CH ? q1 - base : CH);
        // A1
        const int pairs = cnt * ns;
        for (int t0 = tid; t0 < pairs; t0 += nthr * kUnroll) {
            float xv[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int t = t0 + u * nthr;
                if (t < pairs) {
                    const int s = t / cnt;
                    xv[u] = gload(sev[s], base + (t - s * cnt));
                }
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int t = t0 + u * nthr;
                if (t < pairs) {
                    const int s = t / cnt;
                    sidx[(t - s * cnt) * ns + s] = slot_index(img, sslot[s], xv[u]);
                }
            }
        }
        __syncthreads();
        // A2
        for (int t = tid; t < cnt * nf; t += nthr) {
            const int qi = t / nf;
            const int* r = fq + (t - qi * nf) * kFqInts;
            int off = r[0];
            if (r[1] == CBN_FACTOR_QUERY) {
                int row = 0;
                bool ok = true;
                for (int p = 0; p < r[2]; ++p) {
                    const int i = sidx[qi * ns + r[4 + p]];
                    ok &= i >= 0;
                    row = row * r[4 + kMaxP + p] + (i < 0 ? 0 : i);
                }
                off = ok ? off + row * RS : -1;
            }
            offs[t] = off;
        }
        __syncthreads();
        // B
        for (int it = tid; it < cnt * L; it += nthr) {
            const int qi = it / L;
            const int l = it - qi * L;
            float acc[VEC];
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[i] = 1.f;  // out_pdf = ones (bayesian_network.py:269)
            const int* oq = offs + qi * nf;
#pragma unroll 4
            for (int f = 0; f < nf; ++f) {
                const int o = oq[f];
                if constexpr (VEC == 4) {
                    const float4 t = o >= 0 ? *reinterpret_cast<const float4*>(img + o + l * 4)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
                    acc[0] = acc[0] * t.x;
                    acc[1] = acc[1] * t.y;
                    acc[2] = acc[2] * t.z;
                    acc[3] = acc[3] * t.w;
                } else {
                    acc[0] = acc[0] * (o >= 0 ? img[o + l] : 0.f);
                }
            }
            if (WRITE) {
                float* o = out + (base + qi) * N + (long long)l * VEC;
                if constexpr (VEC == 4) {
                    *reinterpret_cast<float4*>(o) =
                        make_float4(acc[0] / maxv, acc[1] / maxv, acc[2] / maxv, acc[3] / maxv);
                } else {
                    o[0] = acc[0] / maxv;
                }
            } else {
#pragma unroll
                for (int i = 0; i < VEC; ++i) lmax = fmaxf(lmax, acc[i]);
            }
        }
        __syncthreads();
    }
    if (!WRITE) {
        lmax = wave_max(lmax);
        const int w = tid / kWave;
        if ((tid & (kWave - 1)) == 0) wmax[w] = lmax;
        __syncthreads();
        if (tid == 0) {
            float m = 0.f;
            for (int i = 0; i < nthr / kWave; ++i) m = fmaxf(m, wmax[i]);
            // values >= 0: uint order == float order.  The last block to arrive
            // publishes the max and re-arms the plan's staging word + counter,
            // so no memset launch is needed between calls.
            // returning device-scope atomics (no fence, ~3.5 us each): this
            // block's max is performed before its arrival is counted, so the
            // last arriver's exchange returns every block's contribution
            if (atomicMax(&sync[4], __float_as_uint(m)) == 0xFFFFFFFFu) atomicOr(&sync[2], 2u);
            const unsigned prev = atomicAdd(&sync[5], 1u);
            if (prev == gridDim.x - 1) {
                const unsigned v = atomicExch(&sync[4], 0u);
                atomicExch(&sync[5], 0u);
                atomicExch(max_bits, v);
            }
        }
    }
}

constexpr int kFastObs = 4;  // fast path: observed parents per factor


// Per-factor static record, written into the plan image at plan creation and
// copied to LDS with the tables (one LDS-DMA stream, no per-call build).
struct alignas(16) FastRec {
    int table_off;
    int n_obs;
    int card[kFastObs];     // bit 30: domain is {0..card-1} (index = value)
    int dom_off[kFastObs];
    int slot[kFastObs];
    int pad[2];
};
constexpr int kDenseBit = 1 << 30;
constexpr int kRecFloats = sizeof(FastRec) / 4;

// Fast path: the L = N / (4 VPL) lanes of one query (a power of two dividing
// 64, so a query never straddles waves) split its factors: lane l loads the
// evidence of factors l, l+L, ... (all loads issued before any is used),
// maps them to domain indices and writes the factors' row offsets into the
// wave's private LDS slice; after a wave-local LDS fence every lane reads all
// offsets (4 per ds_read_b128) and multiplies its 4*VPL columns of each factor
// row in the reference's factor order.  No block barrier after the prologue.
constexpr int kLoc = 8;

// MODE 0: max pass, 1: write pass (two launches); 2: fused -- one launch, one
// round per wave, products kept in registers across an agent-scope grid
// barrier on the global max (all blocks co-resident: grid <= #CUs, 1 block/CU).
// MODE 3 (raw): one launch, no grid barrier -- stores the unnormalised
// products and publishes this launch's max like MODE 0 (the sharded path
// all-reduces that max across ranks, then k_scale divides in place: the same
// fp32 division acc / max as the single-launch path, so the rows are identical).
constexpr int kModeMax = 0, kModeWrite = 1, kModeFused = 2, kModeRaw = 3;
constexpr unsigned kSpinLimit = 1u << 22;  // bounded barrier spin (~0.3 s): never hang

// Fused grid barrier on the global max, called by ONE wave per block (all
// blocks co-resident).  Slot barrier: no counters, no re-arming.  One relaxed
// agent-scope 8-byte store publishes {epoch, block max} (single-copy atomic, so
// a reader sees the old epoch or the new pair, never a mix); the wave then
// polls every block's slot (lane i owns slots i, i+64, ...) until all carry
// this epoch -- one round trip after the last block arrives instead of a chain
// of fan-in atomics.  Returns the max word of all blocks.  Bounded spin: a
// block that never arrives sets sync[2] (the timeout flag) instead of hanging.
__device__ __forceinline__ unsigned slot_barrier_max(unsigned* __restrict__ sync, unsigned epoch, float bm) {
    const int lane = threadIdx.x & (kWave - 1);
    unsigned long long* slots = reinterpret_cast<unsigned long long*>(sync + kSlotWordOff);
    const unsigned long long tag = (unsigned long long)epoch << 32;
    if (lane == 0)
        __hip_atomic_store(&slots[blockIdx.x], tag | __float_as_uint(bm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int G = gridDim.x;
    constexpr int kPer = kMaxSlots / kWave;
    unsigned gm = 0;
    unsigned spins = 0;
    for (;;) {
        // all of this round's loads in flight before any is consumed (a
        // per-slot branch would serialise them: one round trip each)
        unsigned long long v[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k)
            if (k * kWave < G)  // wave-uniform
                v[k] = __hip_atomic_load(&slots[min(lane + k * kWave, G - 1)], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        bool done = true;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            if (k * kWave < G) {
                const bool here = (v[k] >> 32) == (unsigned long long)epoch;
                done &= here;
                const unsigned b = here ? (unsigned)v[k] : 0u;
                gm = gm > b ? gm : b;
            }
        }
        if (__builtin_amdgcn_ballot_w64(!done) == 0) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kSpinLimit) {
            // timed out: flag it on the device (cbn_plan_status) and in the plan's
            // host-mapped status word (the next cbn_plan_run reports it), and make
            // this block's rows NaN instead of dividing by a partial max
            if (lane == 0) {
                atomicOr(&sync[2], 1u);
                unsigned* hs = *reinterpret_cast<unsigned* const*>(sync + kHostStatusWordOff);
                if (hs) __hip_atomic_store(hs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            return 0x7fc00000u;  // NaN
        }
    }
    return wave_max_u(gm);  // non-negative floats: unsigned order == float order
}

#ifdef CBN_BAR2
// Diagnostic A/B (tools/ab_libs.sh): two-level form of slot_barrier_max.  The
// blocks of one group (blockIdx % 8: one XCD under the observed round-robin
// placement -- speed only, the protocol does not depend on it) reduce their
// 32 slots; each block of the group publishes the same group word {epoch,
// group max} once it saw all 32 (idempotent stores), and every block then
// polls the 8 group words: 40 polled words per wave per round instead of 256.
__device__ __forceinline__ unsigned slot_barrier_max2(unsigned* __restrict__ sync, unsigned epoch, float bm) {
    const int lane = threadIdx.x & (kWave - 1);
    unsigned long long* slots = reinterpret_cast<unsigned long long*>(sync + kSlotWordOff);
    unsigned long long* gslots = slots + kMaxSlots - 8;  // 8 group words: the last slots (fused grid <= #CUs)
    const unsigned long long tag = (unsigned long long)epoch << 32;
    if (lane == 0)
        __hip_atomic_store(&slots[blockIdx.x], tag | __float_as_uint(bm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int G = gridDim.x;
    const int grp = blockIdx.x & 7;
    unsigned spins = 0;
    auto timeout = [&]() {
        if (lane == 0) {
            atomicOr(&sync[2], 1u);
            unsigned* hs = *reinterpret_cast<unsigned* const*>(sync + kHostStatusWordOff);
            if (hs) __hip_atomic_store(hs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    };
    // level 1: this group's slots grp, grp + 8, ... (< G); lane i owns slot grp + 8 i
    unsigned gm = 0;
    for (;;) {
        const int s = grp + 8 * lane;
        unsigned long long v = s < G ? __hip_atomic_load(&slots[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tag;
        const bool here = (v >> 32) == (unsigned long long)epoch;
        if (__builtin_amdgcn_ballot_w64(!here) == 0) {
            gm = wave_max_u(s < G ? (unsigned)v : 0u);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kSpinLimit) {
            timeout();
            return 0x7fc00000u;
        }
    }
    if (lane == 0)
        __hip_atomic_store(&gslots[grp], tag | gm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // level 2: the 8 group words (groups with no block: G < 8)
    for (;;) {
        unsigned long long v = (lane < 8 && lane < G) ? __hip_atomic_load(&gslots[lane], __ATOMIC_RELAXED,
                                                                          __HIP_MEMORY_SCOPE_AGENT) : tag;
        const bool here = (v >> 32) == (unsigned long long)epoch;
        if (__builtin_amdgcn_ballot_w64(!here) == 0) return wave_max_u((lane < 8 && lane < G) ? (unsigned)v : 0u);
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kSpinLimit) {
            timeout();
            return 0x7fc00000u;
        }
    }
}
#define slot_barrier_max slot_barrier_max2
#endif

template <int VPL, bool USE_LDS, int MODE, int NP>
__global__ void __launch_bounds__(kQueryThreads)
k_query_fast(int rec_off, int nf, int ns, const float* __restrict__ gimage, int image_floats, FPtrsT<NP> fp,
             long long Q, long long per, int N, int RS, int L, int paired, unsigned* __restrict__ sync,
             unsigned epoch, const unsigned* __restrict__ max_in, int n_max, unsigned* __restrict__ max_out,
             float* __restrict__ out, int lds_tab, unsigned long long lmask0, unsigned long long lmask1) {
    CBN_STAMP_INIT;
    extern __shared__ __attribute__((aligned(16))) float4 smem4[];
    float* simg = reinterpret_cast<float*>(smem4);
    const int nf4 = (nf + 3) & ~3;
    // global-table plans: the small tables (image floats [0, lds_tab), factors
    // in lmask) are copied to LDS; the others are gathered from L2 / MALL
    // (and the factor records follow them in LDS: the index loop's record reads
    // are then LDS reads, which do not wait behind the evidence loads in flight)
    if (USE_LDS) lds_tab = 0;
    const float** ptab =
        reinterpret_cast<const float**>(simg + (USE_LDS ? image_floats : lds_tab + nf * kRecFloats));  // [nf4][4]
    int* woffs_all = reinterpret_cast<int*>(ptab + NP);  // per wave: (64 / L) queries x nf4
    const int tid = threadIdx.x;
    const int nthr = blockDim.x;
    const int lane = tid & (kWave - 1);
    const int wid = tid / kWave;
    const int qpw = kWave / L;  // queries per wave per round
    int* woffs = woffs_all + wid * qpw * nf4;
    float* wmax = reinterpret_cast<float*>(woffs_all + (nthr / kWave) * qpw * nf4);
    // per = ceil(Q / gridDim.x), from the host (a 64-bit division here is ~150
    // scalar instructions on the launch's critical path)
    const long long q0 = (long long)blockIdx.x * per;
    const long long q1 = q0 + per < Q ? q0 + per : Q;
    const long long i_end = q1 * L;
    if (USE_LDS) lds_dma_copy(gimage, smem4, image_floats / 4);  // tables + domains + records
    else {
        if (lds_tab > 0) lds_dma_copy(gimage, smem4, lds_tab / 4);  // the small tables
        lds_dma_copy(gimage + rec_off, smem4 + lds_tab / 4, nf * kRecFloats / 4);  // the records
    }
    if (tid < NP) ptab[tid] = fp.p[tid];
    (void)ns;
    CBN_STAMP(1);
    __syncthreads();  // LDS image (waits vmcnt(0)) + evidence column pointers ready
    CBN_STAMP(2);
    const float* img = USE_LDS ? simg : gimage;
    const FastRec* rec = reinterpret_cast<const FastRec*>(USE_LDS ? simg + rec_off : simg + lds_tab);
    const int lsh = __builtin_ctz(L);  // L: a power of two (query index = item >> lsh)

    float maxv = 1.f;
    if (MODE == kModeWrite) {
        // the max pass's per-block maxima (or one all-reduced word): every wave
        // reduces them itself (L2 hits, no block sync)
        unsigned m = 0;
        for (int i = lane; i < n_max; i += kWave) m = max(m, max_in[i]);
        m = wave_max_u(m);
        maxv = __uint_as_float(m);
        if (max_out && blockIdx.x == 0 && tid == 0) *max_out = m;
    }
    float lmax = 0.f;
    const int qi = lane / L;  // query slot of this lane within the wave
    const int l = lane - qi * L;
    int* my = woffs + qi * nf4;
    // Paired layout (VPL 2, L 4, N 32): ds_read_b128 serves a wave in four
    // 16-lane groups, each holding four queries with distinct qi & 3.  Slot g =
    // qi & 3 reads the odd factor of each pair first (g >= 2) and the upper
    // half of each row first (g odd), so the four queries of a group always read
    // four different 16-bank quarters (bank half = factor parity).  The lane's
    // outputs: cols [clo, clo + 4) in acc[0..3], [chi, chi + 4) in acc[4..7].
    const bool pr = VPL == 2 && USE_LDS && paired;
    const int g4 = qi & 3;
    const bool swp = pr && (g4 >> 1) != 0;
    const int h0 = pr ? (g4 & 1) : 0;
    int col[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) col[v] = pr ? (l + 4 * (v ^ h0)) * 4 : (l * VPL + v) * 4;
    bool first = true;
    constexpr int NV = 4 * VPL;  // outputs owned by this lane
    float acc[NV];
    long long fq = -1;  // fused: the one query this lane holds (-1: none)
    // wave-uniform round loop: a wave's 64 items are qpw whole queries
    float x[kLoc][kFastObs];
    // Evidence of slot j of chunk c0 of round wb into x[j]: every observed
    // parent of the lane's factor c0 + l + j L, always kFastObs loads (an absent
    // parent reads row 0 of the first column), so the number of loads in flight
    // is static and the compiler's waits count them.  The factors are taken in
    // chunks of kLoc * L, and slot j is refilled with the NEXT chunk's (or the
    // next round's first chunk's) evidence as soon as its domain index is done:
    // the evidence loads of a chunk fly while the previous chunk is indexed,
    // instead of one memory round trip per chunk.
    auto q_of = [&](long long wb) { return wb + lane < i_end ? (wb + lane) >> lsh : q0; };
    auto load_one = [&](long long q, int c0, int j) {
        const int f = c0 + l + j * L;
        const int fs = f < nf ? f : 0;
        const uintptr_t p0 = reinterpret_cast<uintptr_t>(ptab[fs * kFastObs]);
        const float* col = reinterpret_cast<const float*>(p0 & ~(kTagMore | kTagNone));
        x[j][0] = gload(col, (p0 & kTagNone) ? 0 : q);
#pragma unroll
        for (int p = 1; p < kFastObs; ++p) {
            const float* cp = (f < nf && (p0 & kTagMore)) ? ptab[fs * kFastObs + p] : nullptr;
            x[j][p] = gload(cp ? cp : col, cp ? q : 0);
        }
#ifdef CBN_CHECKED
        if (!CBN_OK_OR(q >= 0 && q < Q, 2)) x[j][0] = -1.f;
#endif
    };
    long long wbase = q0 * L + (long long)wid * kWave;
    if (wbase < i_end) {
        const long long qf = q_of(wbase);
#pragma unroll
        for (int j = 0; j < kLoc; ++j) load_one(qf, 0, j);
    }
    const int chunk = kLoc * L;
    for (; wbase < i_end; wbase += nthr) {
        const long long it = wbase + lane;
        const bool valid = it < i_end;
        const long long q = valid ? it >> lsh : q0;
        if (first) CBN_STAMP(3);
        for (int c0 = 0; c0 < nf; c0 += chunk) {  // wave-uniform
        const bool more = c0 + chunk < nf;  // refill target: this round's next chunk, else the next round's first
        const bool refill = more || wbase + nthr < i_end;
        const long long qn = q_of(more ? wbase : wbase + nthr);
        const int cn = more ? c0 + chunk : 0;
#pragma unroll
        for (int j = 0; j < kLoc; ++j) {
            const int f = c0 + l + j * L;
            if (f < nf) {
                const FastRec& r = rec[f];
                int o = r.table_off;
                if (r.n_obs > 0) {
                    int row = 0;
                    bool ok = true;
#pragma unroll
                    for (int p = 0; p < kFastObs; ++p) {
                        if (p < r.n_obs) {
                            const int card = r.card[p] & (kDenseBit - 1);
                            const float xv = x[j][p];
                            int i;
                            if (r.card[p] & kDenseBit) {
                                i = (int)xv;
                                i = (xv >= 0.f && xv < (float)card && (float)i == xv) ? i : -1;
                            } else {
                                i = bsearch_eq(img + r.dom_off[p], card, xv);
                            }
                            ok &= i >= 0;
                            row = row * card + (i < 0 ? 0 : i);
                        }
                    }
                    o = ok ? o + row * RS : -1;
                }
                my[f] = o;
            }
            if (refill) load_one(qn, cn, j);  // x[j] is consumed
        }
        }  // chunks
        // the offsets of this query were written by lanes of this same wave:
        // wait for the LDS writes, keep the compiler from reordering around it
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        if (first) CBN_STAMP(4);
        // (the next round's first chunk of evidence is already in flight)
#pragma unroll
        for (int i = 0; i < NV; ++i) acc[i] = 1.f;  // out_pdf = ones (bayesian_network.py:269)
        if constexpr (!USE_LDS) {
            // tables in L2 / MALL (image beyond LDS): KB factors' row loads in
            // flight before their products (memory-level parallelism for the
            // gather), multiplied in factor order
            constexpr int KB = VPL == 2 ? 6 : 8;  // 48 / 32 VGPRs of rows in flight (8 at VPL 2 spills)
            // Zero-product skip (round 5): table entries are finite and >= 0
            // (BruteForce conditionals and their free-parent means), so once
            // every accumulator of a lane is +0 no later factor can change that
            // lane's outputs -- its remaining row gathers are masked off (the
            // products then multiply +0 by +0: the same bits).  On the
            // configs[4] peaked grid the median lane is all-zero after 4 of
            // 100 factors and 84 % of the gathers are skippable per lane, none
            // per wave (62 % of queries keep a nonzero column):
            // profiles/r05_zero_histogram.json.
            bool alive = true;
            for (int f0 = 0; f0 < nf; f0 += KB) {
                if (__builtin_amdgcn_ballot_w64(alive) == 0) break;  // every lane of the wave is all-zero
                int oo[KB];
#pragma unroll
                for (int k = 0; k < KB; ++k) oo[k] = (f0 + k < nf && alive) ? my[f0 + k] : -1;
                float4 t[KB][VPL];
#pragma unroll
                for (int k = 0; k < KB; ++k) {
                    const int o = oo[k];
                    const int fk = f0 + k;  // wave-uniform: is this factor's table in LDS?
                    const bool in_lds = fk < nf && (((fk < 64 ? lmask0 >> fk : lmask1 >> (fk - 64)) & 1ull) != 0);
                    if (in_lds) {
#pragma unroll
                        for (int v = 0; v < VPL; ++v)
                            t[k][v] = o >= 0 ? reinterpret_cast<const float4*>(simg + (o < 0 ? 0 : o))[l * VPL + v]
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
                    } else {
                        const float4* row = reinterpret_cast<const float4*>(img + (o < 0 ? 0 : o)) + l * VPL;
#pragma unroll
                        for (int v = 0; v < VPL; ++v)
                            t[k][v] = (fk < nf && o >= 0) ? row[v] : make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
#pragma unroll
                for (int k = 0; k < KB; ++k) {
                    if (f0 + k < nf) {
#pragma unroll
                        for (int v = 0; v < VPL; ++v) {
                            acc[4 * v + 0] = acc[4 * v + 0] * t[k][v].x;
                            acc[4 * v + 1] = acc[4 * v + 1] * t[k][v].y;
                            acc[4 * v + 2] = acc[4 * v + 2] * t[k][v].z;
                            acc[4 * v + 3] = acc[4 * v + 3] * t[k][v].w;
                        }
                    }
                }
                bool nz = false;
#pragma unroll
                for (int i = 0; i < NV; ++i) nz |= acc[i] != 0.f;  // (NaN counts as alive)
                alive = nz;
            }
        } else if (pr) {
            // factor pairs (f, f + 1) in bank halves 0 / 1: four reads per pair,
            // the multiplies in the reference's factor order whatever the read order
            constexpr int H = 4 % NV;  // acc[H..H+3]: the lane's second column block (VPL 2)
            for (int f0 = 0; f0 < nf; f0 += 4) {
                const int4 o4 = *reinterpret_cast<const int4*>(my + f0);
                const int oo[4] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
                for (int k = 0; k < 4; k += 2) {
                    if (f0 + k + 1 < nf) {
                        const int o1 = swp ? oo[k + 1] : oo[k], o2 = swp ? oo[k] : oo[k + 1];
                        const float* b1 = img + (o1 < 0 ? 0 : o1);
                        const float* b2 = img + (o2 < 0 ? 0 : o2);
                        float4 r0 = *reinterpret_cast<const float4*>(b1 + col[0]);
                        float4 r1 = *reinterpret_cast<const float4*>(b1 + col[VPL - 1]);
                        float4 r2 = *reinterpret_cast<const float4*>(b2 + col[0]);
                        float4 r3 = *reinterpret_cast<const float4*>(b2 + col[VPL - 1]);
                        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
                        if (o1 < 0) r0 = r1 = z;
                        if (o2 < 0) r2 = r3 = z;
                        const float4 a0 = swp ? r2 : r0, a1 = swp ? r3 : r1;
                        const float4 c0 = swp ? r0 : r2, c1 = swp ? r1 : r3;
                        acc[0] *= a0.x; acc[1] *= a0.y; acc[2] *= a0.z; acc[3] *= a0.w;
                        acc[H + 0] *= a1.x; acc[H + 1] *= a1.y; acc[H + 2] *= a1.z; acc[H + 3] *= a1.w;
                        acc[0] *= c0.x; acc[1] *= c0.y; acc[2] *= c0.z; acc[3] *= c0.w;
                        acc[H + 0] *= c1.x; acc[H + 1] *= c1.y; acc[H + 2] *= c1.z; acc[H + 3] *= c1.w;
                    } else if (f0 + k < nf) {  // odd factor count: the last one alone
                        const int o = oo[k];
                        const float* b = img + (o < 0 ? 0 : o);
                        float4 r0 = *reinterpret_cast<const float4*>(b + col[0]);
                        float4 r1 = *reinterpret_cast<const float4*>(b + col[VPL - 1]);
                        if (o < 0) r0 = r1 = make_float4(0.f, 0.f, 0.f, 0.f);
                        acc[0] *= r0.x; acc[1] *= r0.y; acc[2] *= r0.z; acc[3] *= r0.w;
                        acc[H + 0] *= r1.x; acc[H + 1] *= r1.y; acc[H + 2] *= r1.z; acc[H + 3] *= r1.w;
                    }
                }
            }
        } else
        for (int f0 = 0; f0 < nf; f0 += 4) {
            const int4 o4 = *reinterpret_cast<const int4*>(my + f0);
            const int oo[4] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (f0 + k < nf) {
                    int o = oo[k];
#ifdef CBN_CHECKED
                    if (!CBN_OK_OR(o < 0 || o + (l + 1) * VPL * 4 <= image_floats, 4)) o = -1;
#endif
                    const float4* row = reinterpret_cast<const float4*>(img + (o < 0 ? 0 : o)) + l * VPL;
#pragma unroll
                    for (int v = 0; v < VPL; ++v) {
                        const float4 t = o >= 0 ? row[v] : make_float4(0.f, 0.f, 0.f, 0.f);
                        acc[4 * v + 0] = acc[4 * v + 0] * t.x;
                        acc[4 * v + 1] = acc[4 * v + 1] * t.y;
                        acc[4 * v + 2] = acc[4 * v + 2] * t.z;
                        acc[4 * v + 3] = acc[4 * v + 3] * t.w;
                    }
                }
            }
        }
        if (first) CBN_STAMP(5);
        if (valid && CBN_OK_OR(q < Q && (long long)(l + 1) * VPL * 4 <= N, 3)) {
            if (MODE == kModeFused) fq = q;
            if (MODE == kModeWrite) {
                float* o = out + q * N;
#pragma unroll
                for (int v = 0; v < VPL; ++v)
                    *reinterpret_cast<float4*>(o + col[v]) = make_float4(
                        acc[4 * v] / maxv, acc[4 * v + 1] / maxv, acc[4 * v + 2] / maxv, acc[4 * v + 3] / maxv);
            } else if (MODE == kModeRaw) {
                float* o = out + q * N;
#pragma unroll
                for (int v = 0; v < VPL; ++v)
                    *reinterpret_cast<float4*>(o + col[v]) =
                        make_float4(acc[4 * v], acc[4 * v + 1], acc[4 * v + 2], acc[4 * v + 3]);
#pragma unroll
                for (int i = 0; i < NV; ++i) lmax = fmaxf(lmax, acc[i]);
            } else {
#pragma unroll
                for (int i = 0; i < NV; ++i) lmax = fmaxf(lmax, acc[i]);
            }
        }
        __builtin_amdgcn_wave_barrier();  // next round rewrites this wave's offsets
        if (first) CBN_STAMP(6);
        first = false;
    }
    CBN_STAMP(7);
    if (MODE == kModeMax || MODE == kModeRaw) {
        lmax = wave_max(lmax);
        if (lane == 0) wmax[wid] = lmax;
        __syncthreads();
        if (tid == 0) {
            float m = 0.f;
            for (int i = 0; i < nthr / kWave; ++i) m = fmaxf(m, wmax[i]);
            max_out[blockIdx.x] = __float_as_uint(m);  // one word per block, plain store
        }
        if (blockIdx.x == 0)  // words of blocks this launch does not have
            for (int i = (int)gridDim.x + tid; i < n_max; i += nthr) max_out[i] = 0u;
    }
    if (MODE == kModeFused) {
        lmax = wave_max(lmax);
        if (lane == 0) wmax[wid] = lmax;
        __syncthreads();
        if (wid == 0) {
            const int nw = nthr / kWave;
            const unsigned gm = slot_barrier_max(sync, epoch, wave_max(lane < nw ? wmax[lane] : 0.f));
            if (lane == 0) {
                wmax[0] = __uint_as_float(gm);
                if (blockIdx.x == 0 && max_out) *max_out = gm;
            }
        }
        CBN_STAMP(8);
        __syncthreads();
        CBN_STAMP(9);
        maxv = wmax[0];
        if (fq >= 0) {
            float* o = out + fq * N;
#pragma unroll
            for (int v = 0; v < VPL; ++v)
                *reinterpret_cast<float4*>(o + col[v]) = make_float4(
                    acc[4 * v] / maxv, acc[4 * v + 1] / maxv, acc[4 * v + 2] / maxv, acc[4 * v + 3] / maxv);
        }
        CBN_STAMP(10);
    }
}

// ---------------------------------------------------------------------------
// Column-staged fast kernel (round 4; non-paired table plans: configs[2],
// configs[4]).  k_query_fast indexes evidence per (factor, observed parent):
// every lane issues kFastObs loads per factor (absent parents included, so the
// waits stay counted) and maps each to a domain index, in chunks of kLoc
// factors -- for ALARM-like X35 (26 factors, 36 evidence columns, one lane
// per query) that is 104 loads and 104 index computations per query in four
// dependent rounds, ~15.7 us of a 31 us launch.  But a domain index depends
// only on the EVIDENCE SLOT, not on the factor: here the L lanes of a query
// split its ns slots, load each column once (all loads of a chunk in flight),
// map the value to its domain index (dense: the value; else a binary search
// in the slot's sorted domain) and store it as an int16 in LDS
// ([slot][query of the block], -1 off-domain).  The product loop then forms
// each factor's row offset from its parents' indices (LDS reads, the record
// broadcast from LDS) right before gathering the row: no offset buffer, no
// per-factor evidence reloads.  Same factor order, same products, same
// outputs as k_query_fast (bit-identical); modes as there.
// CH: slot loads in flight per lane (all of a lane's slots in one round trip
// when ceil(ns / L) <= CH): 16 or 40, picked per plan, so a lane does not
// issue many clamped duplicate loads (configs[4]: 99 slots over 8 lanes = 13)
#ifndef CBN_COL_KB
#define CBN_COL_KB 2
#endif
// factors per gather batch.  Measured on one box (profiles/r04_colrec_ab.json),
// X35 / X36 / N = 16 chain at 262 144 queries, us: KB 6: 26.8 / 19.9 / 36.4;
// 4: 25.4 / 20.2 / 31.8; 2: 23.9 / 19.2 / 30.4; 1: 23.4 / 18.9 / 31.4; 8: 28.7.
// Smaller batches win: more waves are past their waits at any time (4 waves
// per SIMD), and fewer rows sit in VGPRs.
constexpr int kColKB = CBN_COL_KB;

// Per-factor record of the product loop (round 4, second form).  Lane f of
// every wave loads factor f's record once (nf <= 64); the loop takes each
// field with v_readlane into an SGPR -- no memory wait -- so it branches on
// SGPRs only, issues a whole batch's index reads, then its row reads, each
// with one wait, and gathers rows with ds_read_b128 (LDS tables) or
// global_load_dwordx4 (the image), never flat loads.  The first form read
// FastRec fields from LDS: the compiler serialised field read ->
// readfirstlane -> branch (3-5 dependent LDS round trips per factor) and
// gathered through flat loads.  (s_load of this record per factor measured
// the same.)  configs[2]: X35 27.6 -> 26.7 us, X36 21.6 -> 19.9 us.
struct alignas(16) ColRec {
    int base;            // float offset of the table (LDS copy when `lds`, else the image)
    int n_obs;           // observed parents (<= kFastObs)
    int par[kFastObs];   // (evidence slot << 24) | row weight in floats (= stride x RS, < 2^24)
    int lds;             // 1: table is in LDS
    int pad;
};
constexpr int kColRecInts = sizeof(ColRec) / 4;

template <int VPL, bool USE_LDS, int MODE, int CH>
__global__ void __launch_bounds__(kQueryThreads)
k_query_cols(int rec_off, int nf, int ns, const float* __restrict__ gimage, int image_floats,
             FPtrsT<kFastPtrsSmall> sp, long long Q, long long per, int N, int RS, int L,
             unsigned* __restrict__ sync, unsigned epoch, const unsigned* __restrict__ max_in, int n_max,
             unsigned* __restrict__ max_out, float* __restrict__ out, int lds_tab, const int* __restrict__ crec) {
    CBN_STAMP_INIT;
    extern __shared__ __attribute__((aligned(16))) float4 smem4[];
    float* simg = reinterpret_cast<float*>(smem4);
    if (USE_LDS) lds_tab = 0;
    // LDS: [tables (USE_LDS: the whole image) | small tables][records][slot records][slot ptrs][idx][wave max]
    const int recs_floats = nf * kRecFloats + ns * 4;  // FastRec[nf] then QSlot[ns], contiguous in the image
    const int lrec = USE_LDS ? rec_off : lds_tab;      // float offset of the records in LDS
    const float** sptr = reinterpret_cast<const float**>(simg + (USE_LDS ? image_floats : lds_tab + recs_floats));
    const int tid = threadIdx.x;
    const int nthr = kQueryThreads;
    const int QB = nthr / L;  // queries per block round
    short* sidx = reinterpret_cast<short*>(sptr + ((ns + 1) & ~1));  // [ns][QB]
    float* wmax = reinterpret_cast<float*>(sidx + (((size_t)ns * QB + 1) & ~size_t(1)));
    // a zero row (N <= 16 floats, 16-B aligned) after the wave maxima: the row
    // of an off-domain evidence value (the reference's factor value 0)
    const int zoff = (int)(((reinterpret_cast<uintptr_t>(wmax + nthr / kWave) - reinterpret_cast<uintptr_t>(simg)) + 15) &
                           ~uintptr_t(15)) / 4;
    const int lane = tid & (kWave - 1);
    const int wid = tid / kWave;
    const long long q0 = (long long)blockIdx.x * per;
    const long long q1 = q0 + per < Q ? q0 + per : Q;
    if (USE_LDS) lds_dma_copy(gimage, smem4, image_floats / 4);
    else {
        if (lds_tab > 0) lds_dma_copy(gimage, smem4, lds_tab / 4);
        lds_dma_copy(gimage + rec_off, smem4 + lds_tab / 4, recs_floats / 4);
    }
    if (tid < ns) sptr[tid] = sp.p[tid];
    if (tid < N) simg[zoff + tid] = 0.f;
    CBN_STAMP(1);
    __syncthreads();
    CBN_STAMP(2);
    const float* img = USE_LDS ? simg : gimage;
    const QSlot* srec = reinterpret_cast<const QSlot*>(simg + lrec + nf * kRecFloats);

    float maxv = 1.f;
    if (MODE == kModeWrite) {
        unsigned m = 0;
        for (int i = lane; i < n_max; i += kWave) m = max(m, max_in[i]);
        m = wave_max_u(m);
        maxv = __uint_as_float(m);
        if (max_out && blockIdx.x == 0 && tid == 0) *max_out = m;
    }
    // the product loop's records, lane f <- factor f (nf <= 64, host-checked)
    int4 cra, crb;
    {
        const int4* cr = reinterpret_cast<const int4*>(crec) + (size_t)(lane < nf ? lane : (nf > 0 ? nf - 1 : 0)) * (kColRecInts / 4);
        cra = cr[0];
        crb = cr[1];
    }
    float lmax = 0.f;
    const int ql = tid / L;        // this lane's query within the block round
    const int l = tid - ql * L;    // lane within the query
    const int nsl = (ns - l + L - 1) / L;  // slots this lane indexes: l, l + L, ...
    int col[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) col[v] = (l * VPL + v) * 4;
    constexpr int NV = 4 * VPL;
    float acc[NV];
    long long fq = -1;
    // fused: up to two rounds per block (as k_query_slots): round 0's products
    // wait in acc0 (query fq0) for the grid barrier
    long long fq0 = -1;
    float acc0[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) acc0[i] = 0.f;
    bool first = true;
    for (long long qb = q0; qb < q1; qb += QB) {  // block-uniform rounds
        const long long qq = qb + ql;
        const bool valid = qq < q1;
        const long long q = valid ? qq : q0;
        if (first) CBN_STAMP(3);
        // index phase: this lane's slots, CH loads in flight per chunk
        for (int c0 = 0; c0 < nsl; c0 += CH) {  // (uniform across the wave unless ns % L)
            float x[CH];
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                int s = l + (c0 + k) * L;
                s = s < ns ? s : ns - 1;  // unconditional loads: the compiler's waits stay counted
                x[k] = gload(sptr[s], q);
            }
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                const int s = l + (c0 + k) * L;
                if (c0 + k < nsl) {
                    const QSlot sr = srec[s];
                    const float xv = x[k];
                    int i;
                    if (sr.dense) {
                        i = (int)xv;
                        i = (xv >= 0.f && xv < (float)sr.card && (float)i == xv) ? i : -1;
                    } else {
                        i = bsearch_eq(img + sr.dom_off, sr.card, xv);
                    }
                    sidx[s * QB + ql] = (short)i;
                }
            }
        }
        // the L lanes of a query are in one wave: a wave-local LDS fence
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        if (first) CBN_STAMP(4);
#pragma unroll
        for (int i = 0; i < NV; ++i) acc[i] = 1.f;  // out_pdf = ones (bayesian_network.py:269)
        for (int f0 = 0; f0 < nf; f0 += kColKB) {
            // the batch's records: lane f holds factor f's, v_readlane -> SGPRs
            // (a partial batch re-reads the last record; its product is skipped)
            int base[kColKB], nob[kColKB], inl[kColKB], iv[kColKB][kFastObs], wt[kColKB][kFastObs];
#pragma unroll
            for (int k = 0; k < kColKB; ++k) {
                const int f = f0 + k < nf ? f0 + k : nf - 1;
                base[k] = __builtin_amdgcn_readlane(cra.x, f);
                nob[k] = __builtin_amdgcn_readlane(cra.y, f);
                inl[k] = USE_LDS ? 1 : __builtin_amdgcn_readlane(crb.z, f);
                // every observed parent's domain index of the batch (one LDS round trip)
#pragma unroll
                for (int p = 0; p < kFastObs; ++p) {
                    iv[k][p] = 0;
                    wt[k][p] = 0;
                    if (p < nob[k]) {
                        const int par = __builtin_amdgcn_readlane(p == 0 ? cra.z : p == 1 ? cra.w : p == 2 ? crb.x : crb.y, f);
                        iv[k][p] = sidx[(par >> 24) * QB + ql];
                        wt[k][p] = par & 0xFFFFFF;
                    }
                }
            }
            // row offset = base + sum(index x weight) (the mixed-radix row of
            // k_query_fast times RS); any index < 0 (off-domain) -> the zero row
            // (absent parents add 0 x 0 branch-free: skipping them behind a
            // second round of uniform branches measured 27 -> 43 us on X35)
            int oo[kColKB];
#pragma unroll
            for (int k = 0; k < kColKB; ++k) {
                int o = base[k], neg = 0;
#pragma unroll
                for (int p = 0; p < kFastObs; ++p) {
                    neg |= iv[k][p];
                    o += (int)__umul24((unsigned)iv[k][p], (unsigned)wt[k][p]);
                }
                oo[k] = neg < 0 ? -1 : o;
            }
            float4 t[kColKB][VPL];
#pragma unroll
            for (int k = 0; k < kColKB; ++k) {
                if (inl[k]) {  // wave-uniform: LDS table (ds_read_b128)
                    const float4* row = reinterpret_cast<const float4*>(simg + (oo[k] < 0 ? zoff : oo[k])) + l * VPL;
#pragma unroll
                    for (int v = 0; v < VPL; ++v) t[k][v] = row[v];
                } else {  // global table (global_load_dwordx4)
                    typedef float f4v_t __attribute__((ext_vector_type(4)));
                    typedef const __attribute__((address_space(1))) f4v_t gf4v_t;
                    gf4v_t* row = (gf4v_t*)(gimage + (oo[k] < 0 ? 0 : oo[k])) + l * VPL;
#pragma unroll
                    for (int v = 0; v < VPL; ++v) {
                        const f4v_t x = row[v];
                        t[k][v] = oo[k] < 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : make_float4(x.x, x.y, x.z, x.w);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < kColKB; ++k) {
                if (f0 + k < nf) {
#pragma unroll
                    for (int v = 0; v < VPL; ++v) {
                        acc[4 * v + 0] = acc[4 * v + 0] * t[k][v].x;
                        acc[4 * v + 1] = acc[4 * v + 1] * t[k][v].y;
                        acc[4 * v + 2] = acc[4 * v + 2] * t[k][v].z;
                        acc[4 * v + 3] = acc[4 * v + 3] * t[k][v].w;
                    }
                }
            }
        }
        if (first) CBN_STAMP(5);
        if (MODE == kModeFused && first) {  // (block-uniform) round 0: held until the barrier
            fq0 = valid ? q : -1;
#pragma unroll
            for (int i = 0; i < NV; ++i) acc0[i] = acc[i];
        }
        if (valid) {
            if (MODE == kModeFused && !first) fq = q;
            if (MODE == kModeWrite) {
                float* o = out + q * N;
#pragma unroll
                for (int v = 0; v < VPL; ++v)
                    *reinterpret_cast<float4*>(o + col[v]) = make_float4(
                        acc[4 * v] / maxv, acc[4 * v + 1] / maxv, acc[4 * v + 2] / maxv, acc[4 * v + 3] / maxv);
            } else if (MODE == kModeRaw) {
                float* o = out + q * N;
#pragma unroll
                for (int v = 0; v < VPL; ++v)
                    *reinterpret_cast<float4*>(o + col[v]) =
                        make_float4(acc[4 * v], acc[4 * v + 1], acc[4 * v + 2], acc[4 * v + 3]);
#pragma unroll
                for (int i = 0; i < NV; ++i) lmax = fmaxf(lmax, acc[i]);
            } else {
#pragma unroll
                for (int i = 0; i < NV; ++i) lmax = fmaxf(lmax, acc[i]);
            }
        }
        // the next round rewrites this query slot's indices (lanes of one wave)
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        if (first) CBN_STAMP(6);
        first = false;
    }
    CBN_STAMP(7);
    if (MODE == kModeMax || MODE == kModeRaw) {
        lmax = wave_max(lmax);
        if (lane == 0) wmax[wid] = lmax;
        __syncthreads();
        if (tid == 0) {
            float m = 0.f;
            for (int i = 0; i < nthr / kWave; ++i) m = fmaxf(m, wmax[i]);
            max_out[blockIdx.x] = __float_as_uint(m);
        }
        if (blockIdx.x == 0)
            for (int i = (int)gridDim.x + tid; i < n_max; i += nthr) max_out[i] = 0u;
    }
    if (MODE == kModeFused) {
        lmax = wave_max(lmax);
        if (lane == 0) wmax[wid] = lmax;
        __syncthreads();
        if (wid == 0) {
            const int nw = nthr / kWave;
            const unsigned gm = slot_barrier_max(sync, epoch, wave_max(lane < nw ? wmax[lane] : 0.f));
            if (lane == 0) {
                wmax[0] = __uint_as_float(gm);
                if (blockIdx.x == 0 && max_out) *max_out = gm;
            }
        }
        CBN_STAMP(8);
        __syncthreads();
        CBN_STAMP(9);
        maxv = wmax[0];
        if (fq0 >= 0) {
            float* o = out + fq0 * N;
#pragma unroll
            for (int v = 0; v < VPL; ++v)
                *reinterpret_cast<float4*>(o + col[v]) = make_float4(
                    acc0[4 * v] / maxv, acc0[4 * v + 1] / maxv, acc0[4 * v + 2] / maxv, acc0[4 * v + 3] / maxv);
        }
        if (fq >= 0) {
            float* o = out + fq * N;
#pragma unroll
            for (int v = 0; v < VPL; ++v)
                *reinterpret_cast<float4*>(o + col[v]) = make_float4(
                    acc[4 * v] / maxv, acc[4 * v + 1] / maxv, acc[4 * v + 2] / maxv, acc[4 * v + 3] / maxv);
        }
        CBN_STAMP(10);
    }
}

// ---------------------------------------------------------------------------
// Slot-indexed kernel for global-table plans with >= 4 lanes per query (round
// 5: the configs[4] grid, L = 8, 100 factors over 99 evidence slots).
// k_query_fast loads each factor's parents' evidence itself: kFastObs = 4
// loads per factor (absent parents included, so the waits count), 400 loads
// per query for 99 distinct values, in two dependent chunks -- 15 us of a
// ~40 us wave (stamps, profiles/r05_grid_zero_skip_ab.json).  Here, as in
// k_query_cols, the L lanes of a query split its SLOTS: one load per slot,
// all in flight, mapped to an int16 domain index in LDS; then each lane forms
// the row offsets of factors l, l + L, ... from its parents' indices (ColRec:
// base + sum(index x row weight), any index < 0 -> -1 = the zero row) into
// the query's offset row in LDS -- once per factor, not once per lane as in
// k_query_cols' product loop -- and the product loop is k_query_fast's
// global-table loop (batches of row loads, LDS for the small tables in
// lmask, the zero-product lane skip).  Same factor order, same products:
// bit-identical to k_query_fast.  LDS: [small tables][QSlot ns][ColRec nf]
// [slot pointers][sidx ns x SQ][offsets QB x nf4][wave maxima]
// (slots_lds_bytes, host).
// sidx row stride (int16 units) of k_query_slots: QB plus a pad of 16 / L
// dwords (>= 1).  An unpadded [ns][QB] layout puts every lane of a query pair
// on one bank (QB / 2 dwords is a multiple of 32), so the index writes and the
// offset phase's parent reads were 8-way conflicts; with the pad a slot row
// shifts the bank by 16 / L, and the 32 / L query pairs of a 32-lane group x
// L consecutive slots land on distinct banks.
__host__ __device__ __forceinline__ int slots_sidx_stride(int L) {
    return kQueryThreads / L + 2 * (L >= 16 ? 1 : 16 / L);
}
#ifndef CBN_SLOTS_FUSED2
#define CBN_SLOTS_FUSED2 1  // fused single launch up to two block rounds (0: one round, beyond -> raw + scale)
#endif
#ifndef CBN_SLOTS_DPP
#define CBN_SLOTS_DPP 1  // phase B hands the running product on by DPP row shifts (0: ds_bpermute)
#endif
#ifndef CBN_SLOTS_FA
#define CBN_SLOTS_FA 2  // phase A: batches of KB factors for every lane
#endif
#ifndef CBN_SLOTS_R
#define CBN_SLOTS_R 4  // phase B: rows per lane per chunk
#endif
template <int VPL, int MODE>
__global__ void __launch_bounds__(kQueryThreads)
k_query_slots(int nf, int ns, const float* __restrict__ gimage, int qslot_off, const int* __restrict__ crec,
              FPtrsT<kFastPtrsSmall> sp, long long Q, long long per, int N, int L, unsigned* __restrict__ sync,
              unsigned epoch, const unsigned* __restrict__ max_in, int n_max, unsigned* __restrict__ max_out,
              float* __restrict__ out, int lds_tab, unsigned long long lmask0, unsigned long long lmask1, int coal) {
    CBN_STAMP_INIT;
    extern __shared__ __attribute__((aligned(16))) float4 smem4[];
    float* simg = reinterpret_cast<float*>(smem4);
    const int tid = threadIdx.x;
    constexpr int nthr = kQueryThreads;
    const int lane = tid & (kWave - 1);
    const int wid = tid / kWave;
    const int QB = nthr / L;  // queries per block round
    const int nf4 = (nf + 3) & ~3;
    const QSlot* srec = reinterpret_cast<const QSlot*>(simg + lds_tab);
    int* lcrec = reinterpret_cast<int*>(simg + lds_tab + ns * 4);
    const float** sptr = reinterpret_cast<const float**>(lcrec + nf * kColRecInts);
    short* sidx = reinterpret_cast<short*>(sptr + ((ns + 1) & ~1));
    const int SQ = slots_sidx_stride(L);
    int* woff = reinterpret_cast<int*>(sidx + (((size_t)ns * SQ + 7) & ~size_t(7)));
    float* wmax = reinterpret_cast<float*>(woff + (size_t)QB * nf4);
    const long long q0 = (long long)blockIdx.x * per;
    const long long q1 = q0 + per < Q ? q0 + per : Q;
    if (lds_tab > 0) lds_dma_copy(gimage, smem4, lds_tab / 4);            // the small tables
    lds_dma_copy(gimage + qslot_off, smem4 + lds_tab / 4, ns);            // QSlot[ns] (16 B each)
    for (int i = tid; i < nf * (kColRecInts / 4); i += nthr)
        reinterpret_cast<int4*>(lcrec)[i] = reinterpret_cast<const int4*>(crec)[i];
    if (tid < ns) sptr[tid] = sp.p[tid];
    CBN_STAMP(1);
    __syncthreads();
    CBN_STAMP(2);
    float maxv = 1.f;
    if (MODE == kModeWrite) {
        unsigned m = 0;
        for (int i = lane; i < n_max; i += kWave) m = max(m, max_in[i]);
        m = wave_max_u(m);
        maxv = __uint_as_float(m);
        if (max_out && blockIdx.x == 0 && tid == 0) *max_out = m;
    }
    float lmax = 0.f;
    const int ql = tid / L;  // this lane's query within the block round
    const int l = tid - ql * L;
    const int nsl = (ns - l + L - 1) / L;  // slots this lane indexes: l, l + L, ...
    int* my = woff + (size_t)ql * nf4;
    int col[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) col[v] = (l * VPL + v) * 4;
    constexpr int NV = 4 * VPL;
    constexpr int CH = 16;  // slot loads in flight per lane (configs[4]: 13)
    float acc[NV];
    long long fq = -1;
    // fused: up to two rounds per block (round 5) -- round 0's products wait in
    // acc0 (query fq0) for the grid barrier beside round 1's in acc (query fq)
    long long fq0 = -1;
    float acc0[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) acc0[i] = 0.f;
    bool first = true;
    for (long long qb = q0; qb < q1; qb += QB) {  // block-uniform rounds
        const long long qq = qb + ql;
        const bool valid = qq < q1;
        const long long q = valid ? qq : q0;
        if (first) CBN_STAMP(3);
        if (coal) {
            // Index phase, coalesced (round 6): the block round's ns x QB
            // evidence values as (slot, 4-query) units, one 16-B load each --
            // a wave reads 1 KB of one or two columns -- mapped to int16
            // indices in LDS; queries past the batch get -1 (the zero row).
            // Other waves' queries are written, so a block barrier before
            // (the previous round's offset reads) and after.
            if (!first) __syncthreads();
            const int QB4 = QB >> 2;
            const int nu = ns * QB4;
            const long long nv = q1 - qb;  // valid queries of this round
            constexpr int CU = 4;  // units in flight per lane
            for (int u0 = 0; u0 < nu; u0 += CU * nthr) {
                float4 x[CU];
#pragma unroll
                for (int k = 0; k < CU; ++k) {
                    const int u = u0 + k * nthr + tid;
                    const int uc = u < nu ? u : nu - 1;  // (unconditional loads: counted waits)
                    const int s = uc / QB4, c4 = (uc - s * QB4) * 4;
                    const float* src = sptr[s] + qb + c4;
                    if (c4 + 4 <= nv) {
                        x[k] = *reinterpret_cast<const float4*>(src);
                    } else {
                        x[k].x = c4 + 0 < nv ? src[0] : 0.f;
                        x[k].y = c4 + 1 < nv ? src[1] : 0.f;
                        x[k].z = c4 + 2 < nv ? src[2] : 0.f;
                        x[k].w = c4 + 3 < nv ? src[3] : 0.f;
                    }
                }
#pragma unroll
                for (int k = 0; k < CU; ++k) {
                    const int u = u0 + k * nthr + tid;
                    if (u < nu) {
                        const int s = u / QB4, c4 = (u - s * QB4) * 4;
                        const QSlot sr = srec[s];
                        const float xs[4] = {x[k].x, x[k].y, x[k].z, x[k].w};
                        int iv[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float xv = xs[e];
                            int i;
                            if (sr.dense) {
                                i = (int)xv;
                                i = (xv >= 0.f && xv < (float)sr.card && (float)i == xv) ? i : -1;
                            } else {
                                i = bsearch_eq(gimage + sr.dom_off, sr.card, xv);
                            }
                            iv[e] = c4 + e < nv ? i : -1;
                        }
                        int* w = reinterpret_cast<int*>(sidx + s * SQ + c4);  // (SQ even, c4 % 4 == 0: 4-B aligned)
                        w[0] = (iv[0] & 0xFFFF) | (iv[1] << 16);
                        w[1] = (iv[2] & 0xFFFF) | (iv[3] << 16);
                    }
                }
            }
            __syncthreads();
        } else
        for (int c0 = 0; c0 < nsl; c0 += CH) {
            float x[CH];
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                int s = l + (c0 + k) * L;
                s = s < ns ? s : ns - 1;  // unconditional loads: the compiler's waits stay counted
                x[k] = gload(sptr[s], q);
            }
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                const int s = l + (c0 + k) * L;
                if (c0 + k < nsl) {
                    const QSlot sr = srec[s];
                    const float xv = x[k];
                    int i;
                    if (sr.dense) {
                        i = (int)xv;
                        i = (xv >= 0.f && xv < (float)sr.card && (float)i == xv) ? i : -1;
                    } else {
                        i = bsearch_eq(gimage + sr.dom_off, sr.card, xv);
                    }
                    sidx[s * SQ + ql] = (short)i;
                }
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the query's lanes are in this wave
        __builtin_amdgcn_wave_barrier();
        // row offsets of factors l, l + L, ... of this query
        for (int f = l; f < nf; f += L) {
            const int4 ra = reinterpret_cast<const int4*>(lcrec)[f * 2];
            const int4 rb = reinterpret_cast<const int4*>(lcrec)[f * 2 + 1];
            const int par[kFastObs] = {ra.z, ra.w, rb.x, rb.y};
            int o = ra.x, neg = 0;
#pragma unroll
            for (int p = 0; p < kFastObs; ++p) {
                if (p < ra.y) {
                    const int iv = sidx[(par[p] >> 24) * SQ + ql];
                    neg |= iv;
                    o += (int)__umul24((unsigned)iv, (unsigned)(par[p] & 0xFFFFFF));
                }
            }
            my[f] = neg < 0 ? -1 : o;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        if (first) CBN_STAMP(4);
#pragma unroll
        for (int i = 0; i < NV; ++i) acc[i] = 1.f;  // out_pdf = ones (bayesian_network.py:269)
        // Phase A: the first FA factors for every lane -- k_query_fast's
        // global-table loop with the zero-product lane skip.  On a peaked
        // network most lanes are all-zero by then (configs[4]: 87 % of the
        // lanes by factor 12, profiles/r05_zero_histogram.json).
        constexpr int KB = VPL == 2 ? 6 : 8;
        const int FA = nf < CBN_SLOTS_FA * KB ? nf : CBN_SLOTS_FA * KB;
        bool alive = true;
        for (int f0 = 0; f0 < FA; f0 += KB) {
            if (__builtin_amdgcn_ballot_w64(alive) == 0) break;
            int oo[KB];
#pragma unroll
            for (int k = 0; k < KB; ++k) oo[k] = (f0 + k < FA && alive) ? my[f0 + k] : -1;
            float4 t[KB][VPL];
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                const int o = oo[k];
                const int fk = f0 + k;  // wave-uniform: is this factor's table in LDS?
                const bool in_lds = fk < FA && (((fk < 64 ? lmask0 >> fk : lmask1 >> (fk - 64)) & 1ull) != 0);
                if (in_lds) {
#pragma unroll
                    for (int v = 0; v < VPL; ++v)
                        t[k][v] = o >= 0 ? reinterpret_cast<const float4*>(simg + (o < 0 ? 0 : o))[l * VPL + v]
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
                } else {
                    const float4* row = reinterpret_cast<const float4*>(gimage + (o < 0 ? 0 : o)) + l * VPL;
#pragma unroll
                    for (int v = 0; v < VPL; ++v)
                        t[k][v] = (fk < FA && o >= 0) ? row[v] : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                if (f0 + k < FA) {
#pragma unroll
                    for (int v = 0; v < VPL; ++v) {
                        acc[4 * v + 0] = acc[4 * v + 0] * t[k][v].x;
                        acc[4 * v + 1] = acc[4 * v + 1] * t[k][v].y;
                        acc[4 * v + 2] = acc[4 * v + 2] * t[k][v].z;
                        acc[4 * v + 3] = acc[4 * v + 3] * t[k][v].w;
                    }
                }
            }
            bool nz = false;
#pragma unroll
            for (int i = 0; i < NV; ++i) nz |= acc[i] != 0.f;  // (NaN counts as alive)
            alive = nz;
        }
        // Phase B: the surviving lanes, up to 8 per pass, one per 8-lane group.
        // A lane's remaining factors are a dependent chain of row loads that
        // the survivors alone would walk 6 rows at a time (a wave waits one
        // load latency per batch however few lanes live); here the group's 8
        // lanes load the rows of 8 x R consecutive factors of ONE survivor at
        // once (its query's offsets, its column block), and the running
        // product then visits lane 0, 1, ..., 7 of the group -- each
        // multiplying its R rows in factor order -- so every survivor's
        // product is the same sequence of fp32 multiplies as in phase A's
        // loop: the same bits, one load latency per 8 x R factors.
        if (FA < nf) {
            constexpr int R = CBN_SLOTS_R;  // rows per lane per chunk: a chunk is 8 R factors
            unsigned long long am = __builtin_amdgcn_ballot_w64(alive);
            const int gq = lane >> 3, j = lane & 7;
            while (am) {  // wave-uniform
                unsigned long long pass = 0, m = am;
                int src = -1;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    if (m) {
                        const int b = __builtin_ctzll(m);
                        if (gq == k) src = b;
                        pass |= 1ull << b;
                        m &= m - 1;
                    }
                }
                am = m;
                const int sl = src < 0 ? lane : src;  // the group's survivor lane (idle group: its own, unused)
                float cur[NV];
#pragma unroll
                for (int i = 0; i < NV; ++i) cur[i] = __shfl(acc[i], sl, kWave);
                const int* qoff = woff + (size_t)((wid * kWave + sl) / L) * nf4;
                const int il = sl & (L - 1);  // the survivor's column block
                for (int c0 = FA; c0 < nf; c0 += 8 * R) {
                    float4 t[R][VPL];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int f = c0 + j * R + r;
                        const int o = (src >= 0 && f < nf) ? qoff[f] : -1;
                        const bool in_lds = f < nf && (((f < 64 ? lmask0 >> f : lmask1 >> (f - 64)) & 1ull) != 0);
#pragma unroll
                        for (int v = 0; v < VPL; ++v) t[r][v] = make_float4(0.f, 0.f, 0.f, 0.f);
                        if (o >= 0) {
                            if (in_lds) {
#pragma unroll
                                for (int v = 0; v < VPL; ++v)
                                    t[r][v] = reinterpret_cast<const float4*>(simg + o)[il * VPL + v];
                            } else {
#pragma unroll
                                for (int v = 0; v < VPL; ++v)
                                    t[r][v] = reinterpret_cast<const float4*>(gimage + o)[il * VPL + v];
                            }
                        }
                    }
#pragma unroll
                    for (int s2 = 0; s2 < 8; ++s2) {
                        if (j == s2) {
#pragma unroll
                            for (int r = 0; r < R; ++r) {
                                if (c0 + s2 * R + r < nf) {
#pragma unroll
                                    for (int v = 0; v < VPL; ++v) {
                                        cur[4 * v + 0] = cur[4 * v + 0] * t[r][v].x;
                                        cur[4 * v + 1] = cur[4 * v + 1] * t[r][v].y;
                                        cur[4 * v + 2] = cur[4 * v + 2] * t[r][v].z;
                                        cur[4 * v + 3] = cur[4 * v + 3] * t[r][v].w;
                                    }
                                }
                            }
                        }
                        if (CBN_SLOTS_DPP && s2 < 7) {
                            // to the next lane only: a DPP row shift (a VALU move, no
                            // LDS round trip); lanes other than s2 + 1 take values
                            // they overwrite before their own turn
#pragma unroll
                            for (int i = 0; i < NV; ++i)
                                cur[i] = __int_as_float(__builtin_amdgcn_update_dpp(
                                    __float_as_int(cur[i]), __float_as_int(cur[i]), 0x111 /* row_shr:1 */, 0xF, 0xF,
                                    false));
                        } else {
#pragma unroll
                            for (int i = 0; i < NV; ++i) cur[i] = __shfl(cur[i], (lane & ~7) | s2, kWave);
                        }
                    }
                }
                // back to the survivor's own lane (taken by group popcount(pass below it))
                const bool mine = ((pass >> lane) & 1ull) != 0;
                const int back = mine ? 8 * __builtin_popcountll(pass & ((1ull << lane) - 1ull)) : lane;
#pragma unroll
                for (int i = 0; i < NV; ++i) {
                    const float v = __shfl(cur[i], back, kWave);
                    if (mine) acc[i] = v;
                }
            }
        }
        if (first) CBN_STAMP(5);
        if (MODE == kModeFused && first) {  // (block-uniform) round 0: held until the barrier
            fq0 = valid ? q : -1;
#pragma unroll
            for (int i = 0; i < NV; ++i) acc0[i] = acc[i];
        }
        if (valid) {
            if (MODE == kModeFused && !first) fq = q;
            if (MODE == kModeWrite) {
                float* o = out + q * N;
#pragma unroll
                for (int v = 0; v < VPL; ++v)
                    *reinterpret_cast<float4*>(o + col[v]) = make_float4(
                        acc[4 * v] / maxv, acc[4 * v + 1] / maxv, acc[4 * v + 2] / maxv, acc[4 * v + 3] / maxv);
            } else if (MODE == kModeRaw) {
                float* o = out + q * N;
#pragma unroll
                for (int v = 0; v < VPL; ++v)
                    *reinterpret_cast<float4*>(o + col[v]) =
                        make_float4(acc[4 * v], acc[4 * v + 1], acc[4 * v + 2], acc[4 * v + 3]);
#pragma unroll
                for (int i = 0; i < NV; ++i) lmax = fmaxf(lmax, acc[i]);
            } else {
#pragma unroll
                for (int i = 0; i < NV; ++i) lmax = fmaxf(lmax, acc[i]);
            }
        }
        // the next round rewrites this query slot's indices and offsets (lanes of one wave)
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        if (first) CBN_STAMP(6);
        first = false;
    }
    CBN_STAMP(7);
    if (MODE == kModeMax || MODE == kModeRaw) {
        lmax = wave_max(lmax);
        if (lane == 0) wmax[wid] = lmax;
        __syncthreads();
        if (tid == 0) {
            float m = 0.f;
            for (int i = 0; i < nthr / kWave; ++i) m = fmaxf(m, wmax[i]);
            max_out[blockIdx.x] = __float_as_uint(m);
        }
        if (blockIdx.x == 0)
            for (int i = (int)gridDim.x + tid; i < n_max; i += nthr) max_out[i] = 0u;
    }
    if (MODE == kModeFused) {
        lmax = wave_max(lmax);
        if (lane == 0) wmax[wid] = lmax;
        __syncthreads();
        if (wid == 0) {
            const int nw = nthr / kWave;
            const unsigned gm = slot_barrier_max(sync, epoch, wave_max(lane < nw ? wmax[lane] : 0.f));
            if (lane == 0) {
                wmax[0] = __uint_as_float(gm);
                if (blockIdx.x == 0 && max_out) *max_out = gm;
            }
        }
        CBN_STAMP(8);
        __syncthreads();
        CBN_STAMP(9);
        maxv = wmax[0];
        if (fq0 >= 0) {
            float* o = out + fq0 * N;
#pragma unroll
            for (int v = 0; v < VPL; ++v)
                *reinterpret_cast<float4*>(o + col[v]) = make_float4(
                    acc0[4 * v] / maxv, acc0[4 * v + 1] / maxv, acc0[4 * v + 2] / maxv, acc0[4 * v + 3] / maxv);
        }
        if (fq >= 0) {
            float* o = out + fq * N;
#pragma unroll
            for (int v = 0; v < VPL; ++v)
                *reinterpret_cast<float4*>(o + col[v]) = make_float4(
                    acc[4 * v] / maxv, acc[4 * v + 1] / maxv, acc[4 * v + 2] / maxv, acc[4 * v + 3] / maxv);
        }
        CBN_STAMP(10);
    }
}

// ---------------------------------------------------------------------------
// Staged fast kernel: the paired N = 32 layout in LDS (four lanes per query,
// eight columns per lane, <= 32 factors), all four modes.  A block walks its
// query range in rounds of kSR = 256 queries (16 waves x 16 queries).
//
// Why a second kernel: k_query_fast's prologue is a serial chain per wave --
// kernel arguments -> LDS-DMA of the image + pointer table -> block barrier ->
// pointer reads -> evidence loads -> domain index (records read from LDS) ->
// products; phase stamps put 6 us of a 15 us launch before the first product.
// Here the evidence of a round is STAGED BY FACTOR: unit u = (factor f, 128
// queries) belongs to wave u % 16, whose factor is wave-uniform, so its column
// pointer and record come in on the scalar path, its loads are coalesced
// 256-B requests, and the domain index + table offset is computed right
// there; the offsets go to LDS ([query][slot], int2-readable).  The evidence
// loads are issued BEFORE the image's LDS-DMA, so both latencies overlap, and
// ONE block barrier covers both.
//
// Products (conflict-free, no selects): a factor f's rows live in bank half
// f & 1 (the paired layout).  The four queries of a ds_read_b128 lane group
// have distinct slot g = qi & 3; queries with g >= 2 ("lagged") run ONE FACTOR
// BEHIND: their offset slot j holds factor j - 1 (slot 0: a ones row), the
// others' slot j holds factor j.  Step t reads slots 2t and 2t + 1: at each
// read the lagged queries are in the other bank half, and the row half read
// first (g odd: the upper one) splits each half again -- four disjoint
// 16-bank quarters per group -- while every lane still multiplies in the
// reference's factor order.  A value outside a factor's domain points at a
// zero row, slots past the last factor at a ones row (x * 1 is exact), so the
// loop has no per-factor guards.
constexpr int kSR = 256;  // queries per block round
constexpr int kSQ = 128;  // queries per staging unit (two per lane)
constexpr int kSU = 4;    // staging units per wave per round (nf <= 32 -> nf * 2 / 16 <= 4)
#ifndef CBN_DMA_WAVES
#define CBN_DMA_WAVES 4  // A/B on the headline (tools/ab_libs.sh): 1: 15.7, 2: 11.4, 3: 10.35, 4: 10.1, 8: 10.5-11.3, 12: 12.1 us; not split: 10.3 us
#endif
constexpr int kDmaW = CBN_DMA_WAVES;                 // round 0: waves issuing the image's LDS-DMA
constexpr int kEvW = kQueryThreads / kWave - kDmaW;  // round 0: waves staging the evidence
constexpr int kSUp = (64 + kEvW - 1) / kEvW;         // round 0: units per evidence wave

// A raw launch of the pipelined sharded stepper also finishes an EARLIER step:
// it divides that step's unnormalised rows (n4 float4, this block's slice of
// `chunk` float4) by the max of its all-reduced words -- the in-place scale of
// bayesian_network.py:296 -- with the same correctly rounded quotient as
// k_scale, so a step's rows are bit for bit those of the separate scale.  The
// loads are issued after the prologue barrier and land during the products;
// the divided rows are stored before this launch's own rows.  rows == nullptr:
// nothing to fold.
struct FoldJob {
    float* rows;
    const unsigned* words;
    long long n4;
    long long chunk;
    int n_words;
};
constexpr int kFoldK = 2;   // float4 per thread held across the products (chunk <= 2048: one 65 536 x 32 step)
constexpr int kFoldW = 4;   // words per lane (<= 256 words)

template <int MODE>
__global__ void __launch_bounds__(kQueryThreads)
k_query_staged(const float* __restrict__ gimage, int image_floats, int rec_off, int nf, int zero_off, long long Q,
               long long per, unsigned* __restrict__ sync, unsigned epoch, const unsigned* __restrict__ max_in,
               int n_max, unsigned* __restrict__ max_out, float* __restrict__ out, FoldJob fold,
               FPtrsT<kFastPtrsSmall> fp) {
    CBN_STAMP_INIT;
    constexpr int N = 32;
    extern __shared__ __attribute__((aligned(16))) float4 smem4[];
    float* simg = reinterpret_cast<float*>(smem4);
    const int T = (nf + 2) >> 1;  // steps: slots 0 .. 2T-1 cover factors 0 .. nf-1 for both orders
    const int S = (T + 1) >> 1;   // step pairs (one int4 of offsets each)
    // offset slots per query (past the last factor: ones rows), plus one
    // padding pair: the product loop's prefetch reads it unconditionally
    const int nsl = 4 * (S + 1);
    int* offs = reinterpret_cast<int*>(simg + image_floats);  // [2][kSR][nsl]
    float* wmax = reinterpret_cast<float*>(offs + 2 * kSR * nsl);
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    // wave-uniform for the compiler too: the unit / factor indices derived from
    // it then stay on the scalar path (s_load of pointers and records)
    const int wid = __builtin_amdgcn_readfirstlane(tid / kWave);
    const long long q0 = (long long)blockIdx.x * per;
    const long long q1 = q0 + per < Q ? q0 + per : Q;
    const int nunits = nf * (kSR / kSQ);
    const FastRec* grec = reinterpret_cast<const FastRec*>(gimage + rec_off);
    const int one_off = zero_off + 64;  // ones super-row (zero super-row at zero_off)

    // evidence of round `qr` for this wave's units -> x (first observed parent
    // of each unit's factor), all loads in flight at once.  The column pointers
    // (argument block) are wave-uniform scalar loads, all issued before the
    // first is used.  Tags: kTagNone (no observed parent: a dummy column, row
    // 0), kTagMore (further parents, rare: loaded in stage_store).
    // Unit k of a wave = u = gw + k * GW (gw: the wave's index in a group of
    // GW waves that stages a round; KSU * GW >= 64 >= nunits).  Round 0 is
    // staged by the kEvW evidence waves alone (KSU = kSUp) while the other
    // waves issue the image's LDS-DMA; later rounds by all 16 waves (kSU).
    float x[kSUp][2] = {};
    auto stage_load = [&](long long qr, auto ksu, int gw, int GW) {
        constexpr int KSU = decltype(ksu)::value;
        // (unconditional: u / 2 < 32 stays inside the table whatever nf is, so
        // these scalar loads do not wait for the scalar arguments)
        uintptr_t pk[KSU];
#pragma unroll
        for (int k = 0; k < KSU; ++k) {
            const int u = gw + k * GW;
            pk[k] = reinterpret_cast<uintptr_t>(fp.p[((u / (kSR / kSQ)) & 31) * kFastObs]);
        }
#pragma unroll
        for (int k = 0; k < KSU; ++k) {
            const int u = gw + k * GW;
            if (u < nunits) {  // wave-uniform
                const float* col = reinterpret_cast<const float*>(pk[k] & ~(kTagMore | kTagNone));
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const long long q = qr + (u % (kSR / kSQ)) * kSQ + h * kWave + lane;
                    x[k][h] = gload(col, (pk[k] & kTagNone) ? 0 : (q < q1 ? q : q0));
                }
            }
        }
    };
    // x -> domain index -> table offset (a value outside the fitted domain: the
    // zero row of the factor's bank half) -> offs[buf][query][slot]; non-dense
    // domains binary-search the sorted domain in the image's L2 copy (the LDS
    // copy may not have landed yet)
    auto stage_store = [&](long long qr, int buf, auto ksu, int gw, int GW) {
        constexpr int KSU = decltype(ksu)::value;
        int* ob = offs + buf * kSR * nsl;
        int4 rk[KSU];  // {table_off, n_obs, card[0], card[1]} of each unit's factor: all loads issued first
#pragma unroll
        for (int k = 0; k < KSU; ++k) {
            const int u = gw + k * GW;
            rk[k] = sload_int4(grec + (u < nunits ? u / (kSR / kSQ) : 0));
        }
#pragma unroll
        for (int k = 0; k < KSU; ++k) {
            const int u = gw + k * GW;
            if (u < nunits) {
                const int f = u / (kSR / kSQ);
                const int n_obs = rk[k].y, c0 = rk[k].z;
                const int zoff = zero_off + (f & 1) * 32;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int ql = (u % (kSR / kSQ)) * kSQ + h * kWave + lane;
                    int o;
                    if (n_obs == 1 && (c0 & kDenseBit)) {  // common case: one parent, domain {0..card-1}
                        const int card = c0 & (kDenseBit - 1);
                        const float xv = x[k][h];
                        const int i = (int)xv;
                        o = (xv >= 0.f && xv < (float)card && (float)i == xv) ? rk[k].x + i * 64 : zoff;
                    } else if (n_obs == 0) {
                        o = rk[k].x;
                    } else {
                        const FastRec& r = grec[f];
                        float xs[kFastObs];
                        xs[0] = x[k][h];
                        if (n_obs > 1) {  // wave-uniform, rare
                            const long long q = qr + ql;
#pragma unroll
                            for (int p = 1; p < kFastObs; ++p)
                                if (p < n_obs) xs[p] = gload(fp.p[f * kFastObs + p], q < q1 ? q : q0);
                        }
                        int row = 0;
                        bool ok = true;
#pragma unroll
                        for (int p = 0; p < kFastObs; ++p) {
                            if (p < n_obs) {
                                const int card = r.card[p] & (kDenseBit - 1);
                                const float xv = xs[p];
                                int i;
                                if (r.card[p] & kDenseBit) {
                                    i = (int)xv;
                                    i = (xv >= 0.f && xv < (float)card && (float)i == xv) ? i : -1;
                                } else {
                                    i = bsearch_eq(gimage + r.dom_off[p], card, xv);
                                }
                                ok &= i >= 0;
                                row = row * card + (i < 0 ? 0 : i);
                            }
                        }
                        o = ok ? r.table_off + row * 64 : zoff;
                    }
                    // lagged queries ((ql & 2) != 0: slot g = qi & 3 >= 2) hold factor f in slot f + 1
                    ob[ql * nsl + f + ((ql >> 1) & 1)] = o;
                }
            }
        }
    };

    // padding slots (constant for the launch, both buffers): slot 0 of a lagged
    // query and every slot past its last factor point at the ones row of the
    // slot's bank half (slot j of a query with lag d holds factor j - d)
    if (tid < kSR) {
        const int d = (tid >> 1) & 1;
        for (int j = 0; j < nsl; ++j) {
            const int f = j - d;
            if (f < 0 || f >= nf) {
                const int o = one_off + (f & 1) * 32;
                offs[tid * nsl + j] = o;
                offs[kSR * nsl + tid * nsl + j] = o;
            }
        }
    }
    // evidence loads first, then the image's LDS-DMA: both latencies overlap
    // (a wave's vector-memory counter drains in issue order, so loads issued
    // after the DMA could not be consumed before it lands)
    // Round 0, warp-specialised: waves [0, kDmaW) issue the image's LDS-DMA at
    // once (its address is a preloaded argument), waves [kDmaW, 16) load and
    // stage the evidence (their column pointers are kernel arguments beyond the
    // preloaded ones: a memory round trip before the first load can issue).
    // Each wave's vector-memory counter then holds only its own kind of load,
    // so staging never waits for the DMA and the DMA never waits for the
    // argument fetch.
    long long qr = q0;
    const bool dma_wave = wid < kDmaW;  // wave-uniform
    if (!dma_wave) {
#ifndef CBN_ABL_NOSTAGE
        if (qr < q1) stage_load(qr, std::integral_constant<int, kSUp>{}, wid - kDmaW, kEvW);
#endif
    } else {
#ifndef CBN_ABL_NODMA
        lds_dma_copy(gimage, smem4, image_floats / 4, kDmaW);  // tables + zero/ones rows + domains + records
#endif
    }
    CBN_STAMP(1);
    if (!dma_wave && qr < q1)  // (CBN_ABL_NOSTAGE: x uninitialised, offsets still in range)
        stage_store(qr, 0, std::integral_constant<int, kSUp>{}, wid - kDmaW, kEvW);
    CBN_STAMP(2);
    __syncthreads();  // image landed (vmcnt(0) of the DMA) + round 0 offsets
    CBN_STAMP(3);
    // raw launch folding an earlier step's scale: its rows and words in flight
    // during the products (issued here, after the barrier's vmcnt(0))
    float4 fv[kFoldK];
    unsigned fw[kFoldW];
    const long long fb = (long long)blockIdx.x * fold.chunk;
    const long long fe = fb + fold.chunk < fold.n4 ? fb + fold.chunk : fold.n4;
    if (MODE == kModeRaw && fold.rows) {  // kernel-uniform
        const float4* r4 = reinterpret_cast<const float4*>(fold.rows);
#pragma unroll
        for (int k = 0; k < kFoldK; ++k) {
            const long long i = fb + tid + k * kQueryThreads;
            fv[k] = i < fe ? r4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < kFoldW; ++k) {
            const int w = lane + k * kWave;
            fw[k] = w < fold.n_words ? fold.words[w] : 0u;
        }
    }

    const int qi = lane >> 2;  // query slot in the wave (16 per wave)
    const int l = lane & 3;
    const int h0 = qi & 1;     // g odd: the row's upper half first
    const int clo = (l + 4 * h0) * 4, chi = (l + 4 * (h0 ^ 1)) * 4;  // this lane's columns
    float lmax = 0.f;
    float maxv = 1.f;
    if (MODE == kModeWrite) {
        unsigned m = 0;
        for (int i = lane; i < n_max; i += kWave) m = max(m, max_in[i]);
        m = wave_max_u(m);
        maxv = __uint_as_float(m);
        if (max_out && blockIdx.x == 0 && tid == 0) *max_out = m;
    }
    float acc[8];
    long long fq = -1;
    int buf = 0;
    // write-through stores (sc1: nothing left dirty in L2 for the end-of-kernel
    // release to write back): the fused launch's final rows, and a folding raw
    // launch's rows (read again only two groups later, never L2 hits)
    const bool wt_raw = MODE == kModeRaw && fold.rows != nullptr;  // kernel-uniform
    const __amdgpu_buffer_rsrc_t orsrc =
        rows_rsrc((MODE == kModeFused || wt_raw) ? out + q0 * N : nullptr,
                  (MODE == kModeFused || wt_raw) ? (q1 - q0) * (long long)(N * 4) : 0);
    for (; qr < q1; qr += kSR, buf ^= 1) {  // block-uniform
        const long long qn = qr + kSR;
        // next round's evidence flies during these products (the fused launch has one round)
        if (MODE != kModeFused && qn < q1) stage_load(qn, std::integral_constant<int, kSU>{}, wid, kQueryThreads / kWave);
        const int ql = wid * 16 + qi;
        const long long q = qr + ql;
        const int* my = offs + buf * kSR * nsl + ql * nsl;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 1.f;  // out_pdf = ones (bayesian_network.py:269)
        // step t: slots 2t, 2t + 1 -> four row reads (16 B each: this lane's two
        // column blocks of two rows); step t + 1's reads are in flight while
        // step t is multiplied
        // step pairs: one int4 of offsets = slots 4sp .. 4sp+3 = steps 2sp, 2sp+1,
        // each step four row reads (16 B each: this lane's two column blocks of
        // two rows).  The next pair's offsets are read one pair ahead and each
        // step's rows are issued while the other step of the pair is multiplied.
        auto mul_step = [&](const float4& r0, const float4& r1, const float4& r2, const float4& r3) {
            acc[0] *= r0.x; acc[1] *= r0.y; acc[2] *= r0.z; acc[3] *= r0.w;
            acc[4] *= r1.x; acc[5] *= r1.y; acc[6] *= r1.z; acc[7] *= r1.w;
            acc[0] *= r2.x; acc[1] *= r2.y; acc[2] *= r2.z; acc[3] *= r2.w;
            acc[4] *= r3.x; acc[5] *= r3.y; acc[6] *= r3.z; acc[7] *= r3.w;
        };
        auto load_step = [&](int oa, int ob, float4& r0, float4& r1, float4& r2, float4& r3) {
            r0 = *reinterpret_cast<const float4*>(simg + oa + clo);
            r1 = *reinterpret_cast<const float4*>(simg + oa + chi);
            r2 = *reinterpret_cast<const float4*>(simg + ob + clo);
            r3 = *reinterpret_cast<const float4*>(simg + ob + chi);
        };
        // the loop's first rows and offsets are read through volatile pointers:
        // otherwise the compiler folds them with the loop's own prefetch loads
        // (phi of loads -> load of phi) and the prefetch sinks to the top of the
        // next iteration, where nothing overlaps its latency
        typedef float vf4 __attribute__((ext_vector_type(4)));
        typedef const volatile __attribute__((address_space(3))) vf4 lds_vf4;
        auto vld = [&](int o) {
            const vf4 v = *(lds_vf4*)(simg + o);
            return make_float4(v.x, v.y, v.z, v.w);
        };
        auto vload_step = [&](int oa, int ob, float4& r0, float4& r1, float4& r2, float4& r3) {
            r0 = vld(oa + clo);
            r1 = vld(oa + chi);
            r2 = vld(ob + clo);
            r3 = vld(ob + chi);
        };
        float4 A0, A1, A2, A3, B0, B1, B2, B3;
        int4 on = *reinterpret_cast<const int4*>(my);
        vload_step(on.x, on.y, A0, A1, A2, A3);
        vload_step(on.z, on.w, B0, B1, B2, B3);
        {
            typedef int vi4 __attribute__((ext_vector_type(4)));
            typedef const volatile __attribute__((address_space(3))) vi4 lds_vi4;
            const vi4 v = *(lds_vi4*)(my + 4);  // pair 1 (padding when S == 1)
            on = make_int4(v.x, v.y, v.z, v.w);
        }
        CBN_STAMP(4);
#ifdef CBN_ABL_NOPROD
        mul_step(A0, A1, A2, A3);
#else
        // unconditional prefetch (the padding pair S holds ones rows): no
        // phi copies of the row registers in the loop
#pragma unroll 2
        for (int sp = 0; sp < S; ++sp) {  // wave-uniform
            mul_step(A0, A1, A2, A3);
            load_step(on.x, on.y, A0, A1, A2, A3);
            mul_step(B0, B1, B2, B3);
            load_step(on.z, on.w, B0, B1, B2, B3);
            on = *reinterpret_cast<const int4*>(my + 4 * min(sp + 2, S));
        }
#endif
        CBN_STAMP(5);
        if (q < q1) {
            if (MODE == kModeFused) fq = q;
            if (MODE == kModeRaw && wt_raw) {
                const int ob = (int)(q - q0) * (N * 4);
                store_wt(orsrc, ob + clo * 4, make_float4(acc[0], acc[1], acc[2], acc[3]));
                store_wt(orsrc, ob + chi * 4, make_float4(acc[4], acc[5], acc[6], acc[7]));
            } else if (MODE == kModeWrite || MODE == kModeRaw) {
                // plain stores: the raw rows are re-read by the scale pass (L2 hits)
                const float dv = MODE == kModeWrite ? maxv : 1.f;
                float* o = out + q * N;
                *reinterpret_cast<float4*>(o + clo) = MODE == kModeWrite
                    ? make_float4(acc[0] / dv, acc[1] / dv, acc[2] / dv, acc[3] / dv)
                    : make_float4(acc[0], acc[1], acc[2], acc[3]);
                *reinterpret_cast<float4*>(o + chi) = MODE == kModeWrite
                    ? make_float4(acc[4] / dv, acc[5] / dv, acc[6] / dv, acc[7] / dv)
                    : make_float4(acc[4], acc[5], acc[6], acc[7]);
            }
            if (MODE != kModeWrite)
#pragma unroll
                for (int i = 0; i < 8; ++i) lmax = fmaxf(lmax, acc[i]);
        }
        if (MODE != kModeFused && qn < q1) {
            stage_store(qn, buf ^ 1, std::integral_constant<int, kSU>{}, wid, kQueryThreads / kWave);
            __syncthreads();  // next round's offsets visible; this round's buffer free
        }
    }
    CBN_STAMP(6);
    if (MODE == kModeRaw && fold.rows) {  // kernel-uniform: the earlier step's slice, divided and stored
        unsigned m = 0;
#pragma unroll
        for (int k = 0; k < kFoldW; ++k) m = max(m, fw[k]);
        m = wave_max_u(m);
        const double y = 1.0 / (double)__uint_as_float(m);  // acc / max correctly rounded (see the fused epilogue)
        float4* r4 = reinterpret_cast<float4*>(fold.rows);
        const __amdgpu_buffer_rsrc_t frsrc = rows_rsrc(fold.rows + fb * 4, fe > fb ? (fe - fb) * 16 : 0);  // (write-through)
#pragma unroll
        for (int k = 0; k < kFoldK; ++k) {
            const long long i = fb + tid + k * kQueryThreads;
            if (i < fe)
                store_wt(frsrc, (int)(i - fb) * 16,
                         make_float4((float)((double)fv[k].x * y), (float)((double)fv[k].y * y),
                                     (float)((double)fv[k].z * y), (float)((double)fv[k].w * y)));
        }
        // a slice beyond kFoldK float4 per thread (batches larger than the launch's grid x 2048)
        for (long long i = fb + tid + kFoldK * kQueryThreads; i < fe; i += kQueryThreads) {
            const float4 v = r4[i];
            r4[i] = make_float4((float)((double)v.x * y), (float)((double)v.y * y), (float)((double)v.z * y),
                                (float)((double)v.w * y));
        }
    }
    if (MODE == kModeMax || MODE == kModeRaw) {
        lmax = wave_max(lmax);
        if (lane == 0) wmax[wid] = lmax;
        __syncthreads();
        if (tid == 0) {
            float m = 0.f;
            for (int i = 0; i < kQueryThreads / kWave; ++i) m = fmaxf(m, wmax[i]);
            max_out[blockIdx.x] = __float_as_uint(m);  // one word per block, plain store
        }
        if (blockIdx.x == 0)  // words of blocks this launch does not have
            for (int i = (int)gridDim.x + tid; i < n_max; i += kQueryThreads) max_out[i] = 0u;
    }
    if (MODE == kModeFused) {
        lmax = wave_max(lmax);
        if (lane == 0) wmax[wid] = lmax;
        __syncthreads();
        CBN_STAMP(7);
        if (wid == 0) {
#ifdef CBN_ABL_NOBAR
            const unsigned gm = __float_as_uint(wave_max(lane < kQueryThreads / kWave ? wmax[lane] : 0.f));
#else
            const unsigned gm = slot_barrier_max(sync, epoch, wave_max(lane < kQueryThreads / kWave ? wmax[lane] : 0.f));
#endif
            if (lane == 0) {
                wmax[0] = __uint_as_float(gm);
                if (blockIdx.x == 0 && max_out) *max_out = gm;
            }
        }
        CBN_STAMP(8);
        __syncthreads();
        CBN_STAMP(9);
        maxv = wmax[0];
        if (fq >= 0) {
            // acc / max correctly rounded, as the IEEE division (bayesian_network.py:296),
            // in ~4 VALU slots instead of ~10: (float)((double)acc * RN64(1 / max)).
            // The fp64 product is within 2^-52 of acc / max, while a quotient of
            // two 24-bit significands is either a float or at least 2^-49 (relative)
            // away from every midpoint between floats, so the final rounding is the
            // correct one; 0, inf, NaN and subnormal operands give the IEEE results.
            const double y = 1.0 / (double)maxv;
            float o[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = (float)((double)acc[i] * y);
            const int ob = (int)(fq - q0) * (N * 4);
            store_wt(orsrc, ob + clo * 4, make_float4(o[0], o[1], o[2], o[3]));
            store_wt(orsrc, ob + chi * 4, make_float4(o[4], o[5], o[6], o[7]));
        }
        CBN_STAMP(10);
        CBN_CLOCK_END;
    }
}

// max of the n per-block max words, in every lane of the wave.  Every wave of
// a scale launch needs it, and the words were written by other XCDs' blocks
// (an L2 miss each): 16 coalesced loads in flight per lane, so the common
// word counts (256 .. 1 024) cost one round trip instead of n / 64.
__device__ __forceinline__ unsigned max_words(const unsigned* __restrict__ w, int n) {
    const int lane = threadIdx.x & (kWave - 1);
    unsigned m = 0;
    int i = lane;
    for (; i + 15 * kWave < n; i += 16 * kWave) {
        unsigned t[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) t[k] = w[i + k * kWave];
#pragma unroll
        for (int k = 0; k < 16; ++k) m = max(m, t[k]);
    }
    for (; i + 3 * kWave < n; i += 4 * kWave) {
        unsigned t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = w[i + k * kWave];
#pragma unroll
        for (int k = 0; k < 4; ++k) m = max(m, t[k]);
    }
    for (; i < n; i += kWave) m = max(m, w[i]);
    return wave_max_u(m);
}

__device__ __forceinline__ float4 div4(float4 v, float m) {
    v.x = v.x / m;
    v.y = v.y / m;
    v.z = v.z / m;
    v.w = v.w / m;
    return v;
}

// out[0, n) /= max(max_in[0, n_max)) over a grid-stride float4 stream, U
// float4 per thread in flight; the thread's first U are loaded before the max
// words, so the two round trips overlap.
template <int U>
__device__ __forceinline__ void scale_stream(float* __restrict__ out, long long n, const unsigned* __restrict__ max_in,
                                             int n_max, unsigned* __restrict__ pub) {
    const long long n4 = n / 4;
    float4* o4 = reinterpret_cast<float4*>(out);
    const long long stride = (long long)gridDim.x * blockDim.x;
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * stride < n4) v[u] = o4[i + u * stride];
    const unsigned mb = max_words(max_in, n_max);
    if (pub && blockIdx.x == 0 && threadIdx.x == 0) *pub = mb;
    const float m = __uint_as_float(mb);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * stride < n4) o4[i + u * stride] = div4(v[u], m);
    i += U * stride;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = o4[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) o4[i + u * stride] = div4(v[u], m);
    }
    for (; i < n4; i += stride) o4[i] = div4(o4[i], m);
    for (long long j = n4 * 4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; j < n; j += stride)
        out[j] = out[j] / m;
}

// out[i] /= max (bayesian_network.py:296) after a raw launch and the
// cross-rank all-reduce of the max word; one float4 per thread in flight
// streams faster here than 8 (23 vs 32 us over 134 MB, session r06t) on the
// full grid launch_scale gives it.
__global__ void __launch_bounds__(256) k_scale(float* __restrict__ out, long long n, const unsigned* __restrict__ max_in,
                                               int n_max, unsigned* __restrict__ pub) {
    scale_stream<1>(out, n, max_in, n_max, pub);
}

// k_scale over up to kScaleBatch (out, n) pairs in one launch (blockIdx.y =
// pair b, dividing by the max of max_in[b * n_max, (b + 1) * n_max)): the
// pipelined sharded stepper exchanges and scales several steps at once; a
// small grid (it runs beside the next steps' raw launches on the comm stream,
// in the wave slots those leave free) still streams at HBM rate with
// kScaleU float4 per thread in flight.
constexpr int kScaleBatch = 8;
constexpr int kScaleU = 8;
struct ScaleBatch {
    float* out[kScaleBatch];
    long long n[kScaleBatch];
};

__global__ void __launch_bounds__(256) k_scale_batch(ScaleBatch sb, const unsigned* __restrict__ max_in, int n_max) {
    const int b = blockIdx.y;
    scale_stream<kScaleU>(sb.out[b], sb.n[b], max_in + (long long)b * n_max, n_max, nullptr);
}

// *out = max of n words (public query_max: per-block maxima -> one word)
__global__ void __launch_bounds__(64) k_reduce_max(const unsigned* __restrict__ in, int n, unsigned* __restrict__ out) {
    unsigned m = 0;
    for (int i = threadIdx.x; i < n; i += kWave) m = max(m, in[i]);
    m = wave_max_u(m);
    if (threadIdx.x == 0) *out = m;
}

int g_num_cu = 0;

}  // namespace

int cbn::num_cu() {
    if (g_num_cu == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
        g_num_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    }
    return g_num_cu;
}

int cbn::launch_scale(float* out, long long n, const unsigned* words, int n_words, unsigned* pub, hipStream_t s) {
    static const int per_cu = [] {  // blocks per CU at most (diagnostic: CBN_SCALE_CAP)
        const char* e = diag_env("CBN_SCALE_CAP");
        const int x = e ? atoi(e) : 0;
        return x >= 1 && x <= 32 ? x : 4;
    }();
    long long blocks = (n / 4 + 255) / 256;
    const long long cap = (long long)per_cu * num_cu();
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_scale, dim3((unsigned)blocks), dim3(256), 0, s, out, n, words, n_words, pub);
    HIP_TRY(hipGetLastError());
    return CBN_OK;
}

namespace {

// this call's column pointer of every (factor, observed parent)
template <int NP>
FPtrsT<NP> fast_ptrs(const cbn_plan* p, const EvPtrs& ev, int first_factor = 0) {
    FPtrsT<NP> fp;
    // dummy for factors with no observed parent: any column of >= 1 row
    const float* dummy = p->ns > 0 ? ev.p[0] : p->d_image;
    for (int i = 0; i < NP; ++i) {
        const int j = i + first_factor * kFastObs;  // factors from first_factor on
        fp.p[i] = j < kFastPtrs && p->fast_slot[j] >= 0 ? ev.p[p->fast_slot[j]] : nullptr;
    }
    for (int f = 0; f < NP / kFastObs; ++f) {
        uintptr_t v = reinterpret_cast<uintptr_t>(fp.p[f * kFastObs]);
        if (!v) v = reinterpret_cast<uintptr_t>(dummy) | kTagNone;
        if (fp.p[f * kFastObs + 1]) v |= kTagMore;
        fp.p[f * kFastObs] = reinterpret_cast<const float*>(v);
    }
    return fp;
}

// this call's column pointer of every evidence slot (k_query_cols)
FPtrsT<kFastPtrsSmall> slot_ptrs(const cbn_plan* p, const EvPtrs& ev) {
    FPtrsT<kFastPtrsSmall> sp;
    for (int i = 0; i < kFastPtrsSmall; ++i) sp.p[i] = i < p->ns ? ev.p[i] : nullptr;
    return sp;
}

// dynamic LDS of k_query_slots (its layout, in order): the small tables,
// QSlot[ns], ColRec[nf], slot pointers, sidx[ns][SQ] (int16, SQ = QB + pad),
// offsets [QB][nf4], wave maxima
size_t slots_lds_bytes(long long lds_tab_floats, int ns, int nf, int QB) {
    const size_t nf4 = (size_t)((nf + 3) & ~3);
    const size_t SQ = (size_t)slots_sidx_stride(kQueryThreads / QB);
    size_t b = (size_t)lds_tab_floats * 4 + (size_t)ns * sizeof(QSlot) + (size_t)nf * sizeof(ColRec) +
               (size_t)((ns + 1) & ~1) * sizeof(void*) + ((((size_t)ns * SQ + 7) & ~size_t(7)) * 2) +
               (size_t)QB * nf4 * 4 + (kQueryThreads / kWave) * 4 + 64;
    return (b + 15) & ~size_t(15);
}

// one fast-kernel launch with the pointer table sized to the plan
template <int VPL, bool LDS, int MODE, int NP>
void launch_fast_np(const cbn_plan* p, unsigned blocks, hipStream_t s, const EvPtrs& ev, long long Q, int L,
                    unsigned epoch, const unsigned* max_in, int n_max, unsigned* max_out, float* out) {
    hipLaunchKernelGGL((k_query_fast<VPL, LDS, MODE, NP>), dim3(blocks), dim3(kQueryThreads), p->fast_lds_bytes, s,
                       p->rec_off, p->nf, p->ns, p->d_image, p->image_floats, fast_ptrs<NP>(p, ev), Q,
                       (Q + blocks - 1) / blocks, p->N, p->RS, L, p->paired ? 1 : 0, p->d_sync, epoch, max_in, n_max,
                       max_out, out, p->lds_tab_floats, p->lds_tab_mask[0], p->lds_tab_mask[1]);
}

template <int VPL, bool LDS, int MODE>
void launch_fast_k(const cbn_plan* p, unsigned blocks, hipStream_t s, const EvPtrs& ev, long long Q, int L,
                   unsigned epoch, const unsigned* max_in, int n_max, unsigned* max_out, float* out,
                   const FoldJob* fold = nullptr) {
    if (p->staged) {  // paired N = 32 layout in LDS: the staged kernel (same grid, same words)
        FoldJob fj;
        memset(&fj, 0, sizeof(fj));
        if (fold && fold->rows && fold->n4 > 0) {
            fj = *fold;
            fj.chunk = (fj.n4 + blocks - 1) / blocks;
        }
        // factors [prefix, nf): the prefix is folded into factor `prefix`'s table
        hipLaunchKernelGGL((k_query_staged<MODE>), dim3(blocks), dim3(kQueryThreads), p->staged_lds_bytes, s,
                           p->d_image, p->image_floats, p->rec_off + p->prefix * kRecFloats, p->nf - p->prefix,
                           p->zero_off, Q, (Q + blocks - 1) / blocks, p->d_sync, epoch, max_in, n_max, max_out, out,
                           fj, fast_ptrs<kFastPtrsSmall>(p, ev, p->prefix));
        return;
    }
    if (p->slots) {
        // Coalesced index phase (round 6: 16-B evidence loads per (slot, 4
        // queries), the block's waves index every query of the round, block
        // barriers around it) for launches of >= 3 block rounds: the
        // configs[4] grid at 262 144 queries 316.5-319.1 -> 279.0-280.1 us,
        // but at 65 536 (the fused launch's two rounds) 66.2-66.4 -> 73.7-74.1
        // us -- the barriers put the waves in lockstep across the rounds
        // (MEASUREMENTS.md, round 6).  Needs 16-B aligned columns and every
        // block's first query a multiple of 4.
        const int QBs = kQueryThreads / L;
        long long per = (Q + blocks - 1) / blocks;
        int coal = per > 2LL * QBs && !diag_env("CBN_SLOTS_NO_COAL") ? 1 : 0;
        if (diag_env("CBN_SLOTS_COAL")) coal = 1;
        for (int i = 0; i < p->ns; ++i) coal &= (reinterpret_cast<uintptr_t>(ev.p[i]) & 15) == 0 ? 1 : 0;
        if (coal) per = (per + 3) & ~3LL;
        hipLaunchKernelGGL((k_query_slots<VPL, MODE>), dim3(blocks), dim3(kQueryThreads), p->fast_lds_bytes, s, p->nf,
                           p->ns, p->d_image, p->rec_off + p->nf * kRecFloats, p->d_crec, slot_ptrs(p, ev), Q, per,
                           p->N, L, p->d_sync, epoch, max_in, n_max, max_out, out, p->lds_tab_floats,
                           p->lds_tab_mask[0], p->lds_tab_mask[1], coal);
        return;
    }
    if (p->cols) {
        auto k = (p->ns + L - 1) / L <= 16 ? k_query_cols<VPL, LDS, MODE, 16> : k_query_cols<VPL, LDS, MODE, 40>;
        hipLaunchKernelGGL(k, dim3(blocks), dim3(kQueryThreads), p->fast_lds_bytes, s,
                           p->rec_off, p->nf, p->ns, p->d_image, p->image_floats, slot_ptrs(p, ev), Q,
                           (Q + blocks - 1) / blocks, p->N, p->RS, L, p->d_sync, epoch, max_in, n_max, max_out, out,
                           p->lds_tab_floats, p->d_crec);
        return;
    }
    if (p->nf * kFastObs <= kFastPtrsSmall)
        launch_fast_np<VPL, LDS, MODE, kFastPtrsSmall>(p, blocks, s, ev, Q, L, epoch, max_in, n_max, max_out, out);
    else
        launch_fast_np<VPL, LDS, MODE, kFastPtrs>(p, blocks, s, ev, Q, L, epoch, max_in, n_max, max_out, out);
}

template <int VPL, bool LDS, int MODE>
const void* fast_kernel_fn(int nf, bool cols = false, int slots_per_lane = 0) {
    if (cols)
        return slots_per_lane <= 16 ? reinterpret_cast<const void*>(&k_query_cols<VPL, LDS, MODE, 16>)
                                    : reinterpret_cast<const void*>(&k_query_cols<VPL, LDS, MODE, 40>);
    return nf * kFastObs <= kFastPtrsSmall ? reinterpret_cast<const void*>(&k_query_fast<VPL, LDS, MODE, kFastPtrsSmall>)
                                           : reinterpret_cast<const void*>(&k_query_fast<VPL, LDS, MODE, kFastPtrs>);
}

template <int VPL, bool LDS, int MODE>
void allow_fast_lds(int bytes) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_query_slots<VPL, MODE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_query_fast<VPL, LDS, MODE, kFastPtrsSmall>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_query_fast<VPL, LDS, MODE, kFastPtrs>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_query_cols<VPL, LDS, MODE, 16>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_query_cols<VPL, LDS, MODE, 40>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// WRITE=false: per-block maxima -> max_out[0, max_slots); WRITE=true: divide by
// the max of max_in[0, n_max) (and publish it in *max_out when non-null)
template <int VPL, bool LDS, bool WRITE>
int launch_fast_v(cbn_plan* p, long long Q, const EvPtrs& ev, const unsigned* max_in, int n_max, unsigned* max_out,
                  float* out, hipStream_t s) {
    const int L = p->N / (4 * VPL);
    const long long cap = p->max_slots;  // #CUs x blocks per CU, one max word each
    long long blocks = (Q * L + kQueryThreads - 1) / kQueryThreads;
    if (blocks > cap) blocks = cap;
    if (!WRITE) n_max = p->max_slots;
    launch_fast_k<VPL, LDS, WRITE ? kModeWrite : kModeMax>(p, (unsigned)blocks, s, ev, Q, L, 0u, max_in, n_max,
                                                          max_out, out);
    HIP_TRY(hipGetLastError());
    return CBN_OK;
}

// Single-launch path: one round per wave, so Q <= blocks * 16 waves * (64 / L);
// blocks <= #CUs with one block per CU, so every block is resident at once.
template <int VPL, bool LDS>
int launch_fused_v(cbn_plan* p, long long Q, const EvPtrs& ev, unsigned* max_bits, float* out, hipStream_t s) {
    const int L = p->N / (4 * VPL);
    const long long per_block = (long long)(kQueryThreads / kWave) * (kWave / L);
    long long blocks = (Q + per_block - 1) / per_block;
    // k_query_slots / k_query_cols: beyond one round per block, every CU's block takes two
    // (fused_capacity allows Q <= 2 rounds of the co-resident grid)
    if ((p->slots || p->cols) && CBN_SLOTS_FUSED2) blocks = std::min<long long>(blocks, std::min<long long>(num_cu(), kMaxSlots));
    const unsigned epoch = ++p->fused_epoch;  // 1, 2, ... (0 = never published)
    if (p->fused_epoch == 0xFFFFFFFFu) p->fused_epoch = 0;
    launch_fast_k<VPL, LDS, kModeFused>(p, (unsigned)blocks, s, ev, Q, L, epoch, nullptr, 0, max_bits, out);
    HIP_TRY(hipGetLastError());
    return CBN_OK;
}

// CUs a raw launch leaves free (CBN_RAW_RESERVE_CU, diagnostic A/B knob): room
// for a concurrently running collective's workgroups, so no block of the raw
// launch waits for one to finish
int raw_reserve_cu() {
    static int v = [] {
        const char* e = diag_env("CBN_RAW_RESERVE_CU");
        const int x = e ? atoi(e) : 0;
        return x >= 0 && x <= 64 ? x : 0;
    }();
    return v;
}

template <int VPL, bool LDS>
int launch_raw_v(cbn_plan* p, long long Q, const EvPtrs& ev, unsigned* max_bits, float* out, hipStream_t s,
                 const FoldJob* fold = nullptr) {
    const int L = p->N / (4 * VPL);
    const long long cap = std::max(1, p->max_slots - raw_reserve_cu());
    long long blocks = (Q * L + kQueryThreads - 1) / kQueryThreads;
    if (blocks > cap) blocks = cap;
    launch_fast_k<VPL, LDS, kModeRaw>(p, (unsigned)blocks, s, ev, Q, L, 0u, nullptr, p->max_slots, max_bits, out,
                                      fold);
    HIP_TRY(hipGetLastError());
    return CBN_OK;
}

// public pass API on the fast kernel: max pass -> per-block words -> one word
template <int VEC, bool LDS, bool WRITE>
int launch_fast(cbn_plan* p, long long Q, const EvPtrs& ev, unsigned* max_bits, float* out, hipStream_t s) {
    unsigned* slots = p->d_sync + kMaxWordOff;
    int rc;
    if (WRITE)
        rc = p->vpl == 2 ? launch_fast_v<2, LDS, true>(p, Q, ev, max_bits, 1, nullptr, out, s)
                         : launch_fast_v<1, LDS, true>(p, Q, ev, max_bits, 1, nullptr, out, s);
    else
        rc = p->vpl == 2 ? launch_fast_v<2, LDS, false>(p, Q, ev, nullptr, 0, slots, nullptr, s)
                         : launch_fast_v<1, LDS, false>(p, Q, ev, nullptr, 0, slots, nullptr, s);
    if (rc || WRITE) return rc;
    hipLaunchKernelGGL(k_reduce_max, dim3(1), dim3(kWave), 0, s, slots, p->max_slots, max_bits);
    HIP_TRY(hipGetLastError());
    return CBN_OK;
}

template <int VEC, bool LDS, bool WRITE>
int launch_query(cbn_plan* p, long long Q, const EvPtrs& ev, unsigned* max_bits, float* out, hipStream_t s) {
    if (Q == 0) return CBN_OK;
    if (p->fast) return launch_fast<VEC, LDS, WRITE>(p, Q, ev, max_bits, out, s);
    // every CU busy once there are >= 64 queries per block; a block walks its
    // contiguous range in LDS-sized chunks of CH queries
    const long long cap = (long long)num_cu() * p->blocks_per_cu;
    long long blocks = (Q + 63) / 64;
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL((k_query<VEC, LDS, WRITE>), dim3((unsigned)blocks), dim3(kQueryThreads), p->lds_bytes, s,
                       p->d_fac, p->nf, p->d_slots, p->ns, p->d_image, p->image_floats, ev, Q, p->N, p->RS, p->L, p->CH,
                       p->d_sync, max_bits, out);
    HIP_TRY(hipGetLastError());
    return CBN_OK;
}

template <bool WRITE>
int dispatch_query(cbn_plan* p, long long Q, const float* const* evidence, int n_ev, unsigned* max_bits,
                   float* out, hipStream_t s) {
    if (!p->d_fac || !p->d_slots || !p->d_image || !p->d_sync)
        return set_err(CBN_E_ARG, "plan has no device buffers");
    if (n_ev != p->ns) return set_err(CBN_E_ARG, "plan expects %d evidence columns, got %d", p->ns, n_ev);
    EvPtrs ev;
    memset(&ev, 0, sizeof(ev));
    for (int i = 0; i < n_ev; ++i) {
        if (!evidence[i] && Q > 0) return set_err(CBN_E_ARG, "null evidence column %d", i);
        ev.p[i] = evidence[i];
    }
    if (p->vec == 4)
        return p->use_lds ? launch_query<4, true, WRITE>(p, Q, ev, max_bits, out, s)
                          : launch_query<4, false, WRITE>(p, Q, ev, max_bits, out, s);
    return p->use_lds ? launch_query<1, true, WRITE>(p, Q, ev, max_bits, out, s)
                      : launch_query<1, false, WRITE>(p, Q, ev, max_bits, out, s);
}

template <int VEC, bool LDS, bool WRITE>
void allow_lds(size_t bytes) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_query<VEC, LDS, WRITE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if constexpr (VEC == 4) {
        constexpr int M = WRITE ? kModeWrite : kModeMax;
        allow_fast_lds<1, LDS, M>((int)bytes);
        allow_fast_lds<2, LDS, M>((int)bytes);
        allow_fast_lds<1, LDS, kModeFused>((int)bytes);
        allow_fast_lds<2, LDS, kModeFused>((int)bytes);
        allow_fast_lds<1, LDS, kModeRaw>((int)bytes);
        allow_fast_lds<2, LDS, kModeRaw>((int)bytes);
    }
}

long long fused_capacity(const cbn_plan* p) {
    if (!p->fast || !p->fused_ok) return 0;
    const int L = p->N / (4 * p->vpl);
    const long long blocks = std::min(num_cu(), kMaxSlots);  // one block per CU, one barrier slot each
    // k_query_slots and k_query_cols hold two rounds of products per lane across the barrier
    return blocks * (kQueryThreads / kWave) * (kWave / L) * ((p->slots || p->cols) && CBN_SLOTS_FUSED2 ? 2 : 1);
}

}  // namespace

// ================================================================ C ABI ====
extern "C" {

int cbn_abi_version(void) { return CBN_AMD_ABI_VERSION; }

#ifdef CBN_CHECKED
int cbn_debug_set_check_buffer(void* dev_ptr) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), &dev_ptr, sizeof(void*)));
    return CBN_OK;
}
#endif

// 1 when CBN_DIAG=1 was set at load: the diagnostic CBN_* switches count.
int32_t cbn_diag_enabled(void) { return g_diag ? 1 : 0; }

// Test hook: mark the plan's host-mapped status as if a fused launch had timed
// out (the reporting path of CBN_E_TIMEOUT without starving the GPU).
int cbn_debug_flag_timeout(cbn_plan* plan) {
    if (!plan || !plan->h_status) return set_err(CBN_E_ARG, "cbn_debug_flag_timeout: plan has no status word");
    __atomic_store_n(plan->h_status, 1u, __ATOMIC_RELEASE);
    return CBN_OK;
}

#ifdef CBN_STAMPS

int cbn_debug_set_stamp_buffer(void* dev_ptr) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dev_ptr, sizeof(void*)));
    return CBN_OK;
}

// the clock ring of k_query_staged (CBN_CLOCK_END): dev_ptr = [kClockRing][4]
// unsigned long long (nullptr: off); resets the launch counter
int cbn_debug_set_clock_buffer(void* dev_ptr) {
    const unsigned zero = 0;
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_clock), &dev_ptr, sizeof(void*)));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_clock_n), &zero, sizeof(zero)));
    return CBN_OK;
}
#endif

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
    const int vec = (N % 4 == 0) ? 4 : 1;
    const int L = N / vec;
    if (L > kQueryThreads) return set_err(CBN_E_LIMIT, "N_max %d too large for one block row", N);
    // Table rows: in LDS, +16 B per row so consecutive rows start 4 banks apart;
    // an image that cannot fit LDS is read from L2/HBM, where the pad would make
    // every row straddle one more cache line: unpadded rows, 128-B aligned tables.
    long long total_rows = 0;
    for (int f = 0; f < n_factors; ++f) {
        long long rows = 1;
        for (int p = 0; p < factors[f].n_parents && p < kMaxP; ++p)
            if (factors[f].parent_ev_slot[p] >= 0 && factors[f].parent_card[p] > 0)
                rows = std::min(rows * factors[f].parent_card[p], 1LL << 40);
        total_rows += rows;
    }
    const bool global_tables = vec == 4 && total_rows * (N + 4) * 4 > (long long)kLdsBudget;
    // Paired layout (N = 32, tables in LDS, 8 columns per lane): factor f's rows
    // sit in bank half (f & 1) of 256-B super-rows -- even factors in banks 0-31,
    // odd factors in banks 32-63, each class packed from super-row 0.  The fast
    // kernel then reads the two factors of a pair (and the two halves of a row)
    // in an order that gives the four queries of every ds_read_b128 lane group
    // four disjoint 16-bank quarters: conflict-free row gathers (the padded
    // layout's random rows collide ~2x, profiles/r02_lds_pmc.txt).
    long long class_rows[2] = {0, 0};
    int want_vpl = 2;
    if (const char* e = diag_env("CBN_FAST_VPL")) want_vpl = atoi(e);
    for (int f = 0; f < n_factors; ++f) {
        long long rows = 1;
        for (int p = 0; p < factors[f].n_parents && p < kMaxP; ++p)
            if (factors[f].parent_ev_slot[p] >= 0 && factors[f].parent_card[p] > 0)
                rows = std::min(rows * factors[f].parent_card[p], 1LL << 40);
        class_rows[f & 1] += rows;
    }
    bool paired = vec == 4 && N == 32 && !global_tables && want_vpl >= 2 && !diag_env("CBN_NO_PAIRED") &&
                  std::max(class_rows[0], class_rows[1]) * 64 * 4 <= (long long)kLdsBudget * 3 / 4;
    // leading 1-row factors (roots / unobserved-parent factors) fold into the
    // first multi-row factor (k_merge_prefix); the staged kernel skips them
    int prefix = 0;
    if (paired && !diag_env("CBN_NO_PREFIX")) {
        while (prefix < n_factors - 1 && prefix < 8) {
            long long rows = 1;
            for (int p = 0; p < factors[prefix].n_parents && p < kMaxP; ++p)
                if (factors[prefix].parent_ev_slot[p] >= 0 && factors[prefix].parent_card[p] > 0)
                    rows *= factors[prefix].parent_card[p];
            if (rows != 1) break;
            ++prefix;
        }
    }
    const int RS = paired ? 64 : vec == 4 && !global_tables ? N + 4 : N;
    const long long talign = global_tables ? 32 : 4;
    // Global-table plans: the smallest tables go first in the image, as many as
    // fit the LDS the fast kernel leaves free (without costing it its second
    // block per CU), and k_query_fast copies that prefix into LDS -- an
    // ALARM-like plan is 24 tables of <= 2 KB beside two of 128 KB, and
    // gathering the small ones from L2 cost as much as the large ones.
    std::vector<long long> pre_off(n_factors, -1);
    long long lds_tab_end = 0;
    unsigned long long lds_mask[2] = {0, 0};
    if (global_tables && vec == 4 && n_factors <= 128 && !diag_env("CBN_NO_LDS_SPLIT")) {
        int vp = 0, Lp = 0;
        for (int c : {2, 1}) {  // the fast path's choice (below)
            if (c > want_vpl || (N / 4) % c) continue;
            const int Lc = N / (4 * c);
            if (Lc <= kWave && (kWave % Lc) == 0) { vp = c; Lp = Lc; break; }
        }
        if (vp > 0) {
            const long long nf4 = (n_factors + 3) & ~3;
            long long side = (long long)kFastPtrs * sizeof(void*) +
                             (long long)(kQueryThreads / kWave) * (kWave / Lp) * nf4 * 4 + (kQueryThreads / kWave) * 4 + 64;
            long long recb = (long long)n_factors * kRecFloats * 4;  // the records go to LDS too
            if (Lp > 2 && !diag_env("CBN_NO_SLOTS")) {
                // k_query_slots (>= 4 lanes per query) takes the plan if it can:
                // budget the small tables beside ITS side buffers -- or beside
                // k_query_fast's side + records where those are larger, since
                // the fast gate (below) runs first and k_query_slots may still
                // decline the plan (a card > 32767, a row weight >= 2^24)
                int ns_est = 0;
                for (int f = 0; f < n_factors; ++f)
                    for (int q = 0; q < factors[f].n_parents && q < kMaxP; ++q)
                        ns_est = std::max(ns_est, factors[f].parent_ev_slot[q] + 1);
                side = std::max((long long)slots_lds_bytes(0, ns_est, n_factors, kQueryThreads / Lp), side + recb);
                recb = 0;
            }
            long long budget = (long long)kLdsBudget - side - recb - 1024;  // bytes
            if (2 * (side + recb) <= (long long)kLdsBudget)
                budget = std::min(budget, (long long)kLdsBudget / 2 - side - recb - 1024);
            std::vector<std::pair<long long, int>> by_size;
            for (int f = 0; f < n_factors; ++f) {
                long long rows = 1;
                for (int q = 0; q < factors[f].n_parents && q < kMaxP; ++q)
                    if (factors[f].parent_ev_slot[q] >= 0 && factors[f].parent_card[q] > 0)
                        rows = std::min(rows * factors[f].parent_card[q], 1LL << 40);
                by_size.push_back({(rows * RS + talign - 1) & ~(talign - 1), f});
            }
            std::stable_sort(by_size.begin(), by_size.end());
            for (const auto& [tf, f] : by_size) {
                if ((lds_tab_end + tf) * 4 > budget) break;  // floats vs bytes
                pre_off[f] = lds_tab_end;
                lds_tab_end += tf;
                lds_mask[f >> 6] |= 1ull << (f & 63);
            }
            if (lds_tab_end == 0 || lds_tab_end * 4 > (1LL << 20)) {
                std::fill(pre_off.begin(), pre_off.end(), -1);
                lds_tab_end = 0;
                lds_mask[0] = lds_mask[1] = 0;
            }
        }
    }
    long long class_start[2] = {0, 0};
    std::vector<DevFactor> fac(n_factors);
    std::vector<const float*> slot_dom(CBN_MAX_EVIDENCE, nullptr);
    std::vector<int> slot_card(CBN_MAX_EVIDENCE, 0);
    int ns = 0;
    long long off = lds_tab_end;  // after the LDS-copied small tables (global-table plans)
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
        long long stride = h.node_card, rows = 1, F = 1;
        for (int p = h.n_parents - 1; p >= 0; --p) {
            if (h.parent_card[p] <= 0) return set_err(CBN_E_ARG, "factor %d: parent %d card", f, p);
            d.parent_card[p] = h.parent_card[p];
            d.ev_slot[p] = h.parent_ev_slot[p];
            d.cpd_stride[p] = (int)stride;
            stride *= h.parent_card[p];
            if (stride >= (1LL << 31)) return set_err(CBN_E_LIMIT, "factor %d: CPD too large", f);
            const int sl = h.parent_ev_slot[p];
            if (sl >= 0) {
                if (sl >= CBN_MAX_EVIDENCE || !h.parent_domain[p])
                    return set_err(CBN_E_ARG, "factor %d: bad evidence slot/domain", f);
                if (!slot_dom[sl]) {
                    slot_dom[sl] = h.parent_domain[p];
                    slot_card[sl] = h.parent_card[p];
                } else if (slot_card[sl] != h.parent_card[p]) {
                    return set_err(CBN_E_ARG, "evidence slot %d used with different domains", sl);
                }
                ns = std::max(ns, sl + 1);
                rows *= h.parent_card[p];
            } else {
                if (!h.parent_sample_idx) return set_err(CBN_E_ARG, "factor %d: free parent without samples", f);
                F *= N;
                if (F >= (1LL << 31)) return set_err(CBN_E_LIMIT, "factor %d: too many free combos", f);
                d.n_free++;
            }
        }
        if ((h.kind == CBN_FACTOR_QUERY) != (rows > 1 || d.n_parents - d.n_free > 0))
            return set_err(CBN_E_ARG, "factor %d: QUERY iff some parent observed", f);
        if (rows * (long long)RS >= (1LL << 30)) return set_err(CBN_E_LIMIT, "factor %d: table too large", f);
        d.rows = (int)rows;
        d.free_combos = (int)F;
        d.n_entries = (int)(rows * N);
        const long long F_eff = h.kind == CBN_FACTOR_SCALAR ? N : F;
        d.wave_mode = F_eff >= kWave ? 1 : 0;
        if (paired) {
            // bank half by the index the staged kernel sees (prefix factors: half 0, never read there)
            const int c = f < prefix ? 0 : (f - prefix) & 1;
            d.table_off = (int)(class_start[c] * 64 + c * 32);
            class_start[c] += rows;
            off = std::max(class_start[0], class_start[1]) * 64;
        } else if (pre_off[f] >= 0) {
            if (pre_off[f] + rows * RS > lds_tab_end) return set_err(CBN_E_ARG, "factor %d: table size changed", f);
            d.table_off = (int)pre_off[f];
        } else {
            d.table_off = (int)off;
            off += (rows * RS + talign - 1) & ~(talign - 1);
        }
    }
    for (int sl = 0; sl < ns; ++sl)
        if (!slot_dom[sl]) return set_err(CBN_E_ARG, "evidence slot %d is not used by any factor", sl);
    // paired layout: a zero super-row (values outside a domain) and a ones
    // super-row (padding slots) after the tables, both bank halves each
    const long long zero_off = paired ? off : -1;
    if (paired) off += 128;
    const long long table_floats = off;
    std::vector<QSlot> qs(ns);
    std::vector<float> hdom;
    for (int sl = 0; sl < ns; ++sl) {
        qs[sl].dom_off = (int)off;
        qs[sl].card = slot_card[sl];
        hdom.resize(slot_card[sl]);
        if (hipMemcpy(hdom.data(), slot_dom[sl], sizeof(float) * slot_card[sl], hipMemcpyDeviceToHost) != hipSuccess)
            return set_err(CBN_E_HIP, "cbn_plan_create: domain read failed");
        int dense = 1;
        for (int i = 0; i < slot_card[sl] && dense; ++i) dense = hdom[i] == (float)i;
        qs[sl].dense = dense;
        off += (slot_card[sl] + 3) & ~3LL;
    }
    const long long rec_off = off;  // FastRec array (fast path), copied to LDS with the tables
    off += (long long)n_factors * kRecFloats;
    off += (long long)ns * 4;  // QSlot array right after it (k_query_cols: one LDS-DMA for both)
    if (off >= (1LL << 30)) return set_err(CBN_E_LIMIT, "plan image too large");

    cbn_plan* P = new cbn_plan();
    P->nf = n_factors;
    P->ns = ns;
    P->N = N;
    P->vec = vec;
    P->L = L;
    P->image_floats = (int)off;
    P->table_floats = (int)table_floats;
    P->zero_off = (int)zero_off;
    P->prefix = prefix;
    for (int i = 0; i <= prefix && i < 9; ++i) P->prefix_offs[i] = fac[i].table_off;
    P->prefix_rows = prefix > 0 ? fac[prefix].rows : 0;
    P->rec_off = (int)rec_off;
    P->RS = RS;
    P->lds_tab_floats = (int)lds_tab_end;
    P->lds_tab_mask[0] = lds_mask[0];
    P->lds_tab_mask[1] = lds_mask[1];
    // LDS: [image (if staged)] [factor records] [slots] [CH x (ns + nf) ints] [wave maxima]
    const size_t fixed = (size_t)n_factors * kFqInts * 4 + (size_t)ns * sizeof(QSlot) + (kQueryThreads / kWave) * 4 +
                         (size_t)CBN_MAX_EVIDENCE * sizeof(void*) + 64;
    const size_t per_q = (size_t)(ns + n_factors) * 4;
    const size_t img_bytes = (size_t)off * 4;
    auto chunk_for = [&](size_t avail) -> int {
        if (avail <= fixed) return 0;
        size_t ch = (avail - fixed) / per_q;
        return (int)std::min<size_t>(ch, 1024);
    };
    int ch = global_tables ? 0 : chunk_for(kLdsBudget > img_bytes ? kLdsBudget - img_bytes : 0);
    P->use_lds = ch >= 64;  // (a global-table layout stays in L2/HBM even if the unpadded image would fit)
    if (!P->use_lds) ch = chunk_for(kLdsBudget);
    if (ch < 1) {
        delete P;
        return set_err(CBN_E_LIMIT, "plan needs more LDS than a CU has (nf=%d, ns=%d)", n_factors, ns);
    }
    P->CH = ch;
    P->lds_bytes = ((P->use_lds ? img_bytes : 0) + fixed + (size_t)ch * per_q + 15) & ~size_t(15);
    P->blocks_per_cu = 2 * P->lds_bytes <= (size_t)kLdsBudget ? 2 : 1;

    std::vector<BuildItem> build;
    int units = 0;
    for (int f = 0; f < n_factors; ++f) {
        const DevFactor& d = fac[f];
        const int nu = d.wave_mode ? d.n_entries : (d.n_entries + kWave - 1) / kWave;
        build.push_back({f, units});
        units += nu;
    }
    P->n_build = (int)build.size();
    P->build_units = units;

    bool ok = hipMalloc(&P->d_fac, sizeof(DevFactor) * n_factors) == hipSuccess &&
              hipMalloc(&P->d_slots, sizeof(QSlot) * std::max(ns, 1)) == hipSuccess &&
              hipMalloc(&P->d_build, sizeof(BuildItem) * std::max<size_t>(build.size(), 1)) == hipSuccess &&
              hipMalloc(&P->d_image, sizeof(float) * std::max<long long>(off, 4)) == hipSuccess &&
              hipMalloc(&P->d_sync, sizeof(unsigned) * kSyncWords) == hipSuccess;
    ok = ok && hipMemcpy(P->d_fac, fac.data(), sizeof(DevFactor) * n_factors, hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && (ns == 0 || hipMemcpy(P->d_slots, qs.data(), sizeof(QSlot) * ns, hipMemcpyHostToDevice) == hipSuccess);
    ok = ok && (build.empty() ||
                hipMemcpy(P->d_build, build.data(), sizeof(BuildItem) * build.size(), hipMemcpyHostToDevice) == hipSuccess);
    ok = ok && hipMemset(P->d_image, 0, sizeof(float) * std::max<long long>(off, 4)) == hipSuccess;
    if (ok && paired) {
        const std::vector<float> ones(64, 1.f);
        ok = hipMemcpy(P->d_image + zero_off + 64, ones.data(), sizeof(float) * 64, hipMemcpyHostToDevice) == hipSuccess;
    }
    ok = ok && hipMemset(P->d_sync, 0, sizeof(unsigned) * kSyncWords) == hipSuccess;
    // host-mapped status word of the fused launches' timeout (polled for free by cbn_plan_run);
    // its device address lives in the sync buffer for the (rare) timeout path
    ok = ok && hipHostMalloc(reinterpret_cast<void**>(&P->h_status), sizeof(unsigned),
                             hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess;
    if (ok) {
        *P->h_status = 0;
        unsigned* dh = nullptr;
        ok = hipHostGetDevicePointer(reinterpret_cast<void**>(&dh), P->h_status, 0) == hipSuccess &&
             hipMemcpy(P->d_sync + kHostStatusWordOff, &dh, sizeof(dh), hipMemcpyHostToDevice) == hipSuccess;
    }
    for (int sl = 0; ok && sl < ns; ++sl)
        ok = hipMemcpy(P->d_image + qs[sl].dom_off, slot_dom[sl], sizeof(float) * slot_card[sl],
                       hipMemcpyDeviceToDevice) == hipSuccess;
    ok = ok && hipDeviceSynchronize() == hipSuccess;  // uploads complete before any launch uses them
    if (!ok) {
        cbn_plan_destroy(P);
        return set_err(CBN_E_HIP, "cbn_plan_create: device allocation/upload failed");
    }

    // fast path eligibility: N % 4 == 0, lanes per query L = N / (4 VPL) a power
    // of two <= 64, <= kLoc factors per lane, <= kFastObs observed parents each
    bool fast = vec == 4 && n_factors * kFastObs <= kFastPtrs;
    std::vector<FastRec> recs(n_factors);
    for (int& sl : P->fast_slot) sl = -1;
    for (int f = 0; f < n_factors && fast; ++f) {
        FastRec& r = recs[f];
        memset(&r, 0, sizeof(r));
        r.table_off = fac[f].table_off;
        for (int p = 0; p < fac[f].n_parents; ++p) {
            const int sl = fac[f].ev_slot[p];
            if (sl >= 0) {
                if (r.n_obs == kFastObs) { fast = false; break; }
                r.card[r.n_obs] = fac[f].parent_card[p] | (qs[sl].dense ? kDenseBit : 0);
                r.dom_off[r.n_obs] = qs[sl].dom_off;
                r.slot[r.n_obs] = sl;
                P->fast_slot[f * kFastObs + r.n_obs] = sl;
                ++r.n_obs;
            }
        }
    }
    int vpl = 0, Lf = 0;
    if (fast) {
        int want = 2;  // 8 output values per lane (tuned on MI355X: chain20 d32)
        if (const char* e = diag_env("CBN_FAST_VPL")) want = atoi(e);
        for (int c : {2, 1}) {  // VPL 4 exceeds 128 VGPRs at 1024 threads (spills)
            if (c > want || (N / 4) % c) continue;
            const int Lc = N / (4 * c);
            if (Lc <= kWave && (kWave % Lc) == 0) { vpl = c; Lf = Lc; break; }
        }
        fast = vpl > 0;
    }
    if (fast) {
        const int nf4 = (n_factors + 3) & ~3;
        const size_t side = (size_t)kFastPtrs * sizeof(void*) +
                            (size_t)(kQueryThreads / kWave) * (kWave / Lf) * nf4 * 4 + (kQueryThreads / kWave) * 4 + 64;
        const bool lds_ok = img_bytes + side <= (size_t)kLdsBudget;
        if (!lds_ok && P->use_lds) fast = false;  // keep one LDS mode per plan
        // global tables: the LDS-copied small tables + the records + the side buffers must fit
        if (!P->use_lds && (size_t)P->lds_tab_floats * 4 + (size_t)n_factors * kRecFloats * 4 + side > (size_t)kLdsBudget)
            fast = false;
        if (fast) {
            P->fast = true;
            P->vpl = vpl;
            P->paired = paired && vpl == 2 && P->use_lds;
            const int st_T = (n_factors - P->prefix + 2) >> 1, st_S = (st_T + 1) >> 1;  // k_query_staged's nsl
            const size_t st_bytes =
                img_bytes + (size_t)2 * kSR * (4 * (st_S + 1)) * 4 + (kQueryThreads / kWave) * 4 + 64;
            if (P->paired && (n_factors - P->prefix) * kFastObs <= kFastPtrsSmall && st_bytes <= (size_t)kLdsBudget &&
                !diag_env("CBN_NO_STAGED")) {
                P->staged = true;
                P->staged_lds_bytes = (st_bytes + 15) & ~size_t(15);
                for (const void* fn : {reinterpret_cast<const void*>(&k_query_staged<kModeMax>),
                                       reinterpret_cast<const void*>(&k_query_staged<kModeWrite>),
                                       reinterpret_cast<const void*>(&k_query_staged<kModeFused>),
                                       reinterpret_cast<const void*>(&k_query_staged<kModeRaw>)})
                    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBudget);
            }
            P->fast_lds_bytes =
                ((P->use_lds ? img_bytes : (size_t)P->lds_tab_floats * 4 + (size_t)n_factors * kRecFloats * 4) + side +
                 15) & ~size_t(15);
            // column-staged kernel (k_query_cols): non-paired plans of <= 2
            // lanes per query (N <= 16) whose slot indices fit int16 and whose
            // per-slot index buffer fits LDS.  With more lanes per query every
            // lane re-forms every factor's offset: the configs[4] grid (L = 8)
            // ran 459 -> 534 us at 262 144 queries (profiles/r04_cols_ab.json)
            if (!P->staged && !P->paired && Lf <= 2 && ns <= kFastPtrsSmall && n_factors <= kWave &&
                !diag_env("CBN_NO_COLS")) {
                bool ok_c = true;
                for (int sl = 0; sl < ns; ++sl) ok_c = ok_c && slot_card[sl] <= 32767;
                for (int f = 0; f < n_factors && ok_c; ++f)
                    for (int q = 0; q < recs[f].n_obs; ++q)
                        ok_c = ok_c && (recs[f].card[q] & (kDenseBit - 1)) == slot_card[recs[f].slot[q]];
                const size_t QBc = (size_t)kQueryThreads / Lf;
                const size_t cols_bytes =
                    ((P->use_lds ? img_bytes
                                 : (size_t)P->lds_tab_floats * 4 + ((size_t)n_factors * kRecFloats + (size_t)ns * 4) * 4) +
                     (size_t)((ns + 1) & ~1) * sizeof(void*) + (((size_t)ns * QBc + 1) & ~size_t(1)) * 2 +
                     (kQueryThreads / kWave) * 4 + 64 + 16 + (size_t)N * 4 + 15) & ~size_t(15);  // (+ zero row)
                // the product loop's scalar records: (slot << 24) | row weight, weights < 2^24
                std::vector<ColRec> cr(n_factors);
                for (int f = 0; f < n_factors && ok_c; ++f) {
                    ColRec& c = cr[f];
                    memset(&c, 0, sizeof(c));
                    c.base = recs[f].table_off;
                    c.n_obs = recs[f].n_obs;
                    c.lds = P->use_lds || ((lds_mask[f >> 6] >> (f & 63)) & 1ull) ? 1 : 0;
                    long long w = RS;
                    for (int q = recs[f].n_obs - 1; q >= 0; --q) {
                        ok_c = ok_c && w < (1LL << 24) && recs[f].slot[q] < 256;
                        c.par[q] = (recs[f].slot[q] << 24) | (int)(w & 0xFFFFFF);
                        w *= recs[f].card[q] & (kDenseBit - 1);
                    }
                }
                if (ok_c && cols_bytes <= (size_t)kLdsBudget) {
                    ok_c = hipMalloc(&P->d_crec, sizeof(ColRec) * n_factors) == hipSuccess &&
                           hipMemcpy(P->d_crec, cr.data(), sizeof(ColRec) * n_factors, hipMemcpyHostToDevice) ==
                               hipSuccess;
                    if (!ok_c) {
                        cbn_plan_destroy(P);
                        return set_err(CBN_E_HIP, "cbn_plan_create: column records upload failed");
                    }
                    P->cols = true;
                    P->fast_lds_bytes = cols_bytes;
                }
            }
            // slot-indexed kernel (k_query_slots, round 5): global-table plans of
            // >= 4 lanes per query (the configs[4] grid) -- the slots' evidence
            // loaded once per query instead of kFastObs loads per factor
            if (!P->staged && !P->paired && !P->cols && !P->use_lds && Lf > 2 && ns <= kFastPtrsSmall &&
                n_factors <= 128 && !diag_env("CBN_NO_SLOTS")) {
                bool ok_s = true;
                for (int sl = 0; sl < ns; ++sl) ok_s = ok_s && slot_card[sl] <= 32767;
                for (int f = 0; f < n_factors && ok_s; ++f)
                    for (int q = 0; q < recs[f].n_obs; ++q)
                        ok_s = ok_s && (recs[f].card[q] & (kDenseBit - 1)) == slot_card[recs[f].slot[q]];
                std::vector<ColRec> cr(n_factors);
                for (int f = 0; f < n_factors && ok_s; ++f) {
                    ColRec& c = cr[f];
                    memset(&c, 0, sizeof(c));
                    c.base = recs[f].table_off;
                    c.n_obs = recs[f].n_obs;
                    c.lds = ((lds_mask[f >> 6] >> (f & 63)) & 1ull) ? 1 : 0;
                    long long w = RS;
                    for (int q = recs[f].n_obs - 1; q >= 0; --q) {
                        ok_s = ok_s && w < (1LL << 24) && recs[f].slot[q] < 256;
                        c.par[q] = (recs[f].slot[q] << 24) | (int)(w & 0xFFFFFF);
                        w *= recs[f].card[q] & (kDenseBit - 1);
                    }
                    // the offset (table base + row x RS) must fit an int
                    ok_s = ok_s && (long long)recs[f].table_off + w < (1LL << 31);
                }
                const size_t sb = slots_lds_bytes(P->lds_tab_floats, ns, n_factors, kQueryThreads / Lf);
                if (ok_s && sb <= (size_t)kLdsBudget) {
                    if (hipMalloc(&P->d_crec, sizeof(ColRec) * n_factors) != hipSuccess ||
                        hipMemcpy(P->d_crec, cr.data(), sizeof(ColRec) * n_factors, hipMemcpyHostToDevice) !=
                            hipSuccess) {
                        cbn_plan_destroy(P);
                        return set_err(CBN_E_HIP, "cbn_plan_create: slot records upload failed");
                    }
                    P->slots = true;
                    P->fast_lds_bytes = sb;
                }
            }
            P->fast_blocks_per_cu = 2 * P->fast_lds_bytes <= (size_t)kLdsBudget ? 2 : 1;
            if (P->slots)
                if (const char* e = diag_env("CBN_SLOTS_BPC")) P->fast_blocks_per_cu = atoi(e) == 2 ? 2 : 1;
            P->max_slots = std::min(num_cu() * P->fast_blocks_per_cu, kMaxSlots);
            if (hipMemcpy(P->d_image + rec_off, recs.data(), sizeof(FastRec) * n_factors, hipMemcpyHostToDevice) !=
                    hipSuccess ||
                (ns > 0 && hipMemcpy(P->d_image + rec_off + (long long)n_factors * kRecFloats, qs.data(),
                                     sizeof(QSlot) * ns, hipMemcpyHostToDevice) != hipSuccess)) {
                cbn_plan_destroy(P);
                return set_err(CBN_E_HIP, "cbn_plan_create: fast records upload failed");
            }
            if (!diag_env("CBN_NO_FUSED")) {
                // the grid barrier needs every block resident: check one block per CU fits
                // (tables in LDS, or -- image beyond LDS -- read from L2/HBM)
                allow_fast_lds<1, true, kModeFused>(kLdsBudget);
                allow_fast_lds<2, true, kModeFused>(kLdsBudget);
                allow_fast_lds<1, false, kModeFused>(kLdsBudget);
                allow_fast_lds<2, false, kModeFused>(kLdsBudget);
                int nb = 0;
                const int spl = (ns + Lf - 1) / Lf;  // k_query_cols: slots per lane
                const void* fn = P->staged ? reinterpret_cast<const void*>(&k_query_staged<kModeFused>)
                                 : P->slots ? (vpl == 2 ? reinterpret_cast<const void*>(&k_query_slots<2, kModeFused>)
                                                        : reinterpret_cast<const void*>(&k_query_slots<1, kModeFused>))
                                 : P->use_lds ? (vpl == 2 ? fast_kernel_fn<2, true, kModeFused>(n_factors, P->cols, spl)
                                                          : fast_kernel_fn<1, true, kModeFused>(n_factors, P->cols, spl))
                                              : (vpl == 2 ? fast_kernel_fn<2, false, kModeFused>(n_factors, P->cols, spl)
                                                          : fast_kernel_fn<1, false, kModeFused>(n_factors, P->cols, spl));
                const size_t lb = P->staged ? P->staged_lds_bytes : P->fast_lds_bytes;
                if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kQueryThreads, lb) == hipSuccess && nb >= 1)
                    P->fused_ok = true;
            }
        }
    }
    if (!P->staged && P->prefix) {
        // the merge is only valid for the staged kernel (the others multiply every
        // factor): a non-staged plan with a paired layout keeps its tables as built
        P->prefix = 0;
        P->prefix_rows = 0;
    }
    allow_lds<4, true, false>(kLdsBudget); allow_lds<4, true, true>(kLdsBudget);
    allow_lds<1, true, false>(kLdsBudget); allow_lds<1, true, true>(kLdsBudget);
    allow_lds<4, false, false>(kLdsBudget); allow_lds<4, false, true>(kLdsBudget);
    allow_lds<1, false, false>(kLdsBudget); allow_lds<1, false, true>(kLdsBudget);
    // invariant: every buffer a launch dereferences exists (a plan missing one
    // must never reach a kernel)
    if (!P->d_fac || !P->d_slots || !P->d_build || !P->d_image || !P->d_sync) {
        cbn_plan_destroy(P);
        return set_err(CBN_E_HIP, "cbn_plan_create: internal error, plan buffer missing");
    }
    *plan = P;
    return CBN_OK;
}

int cbn_plan_destroy(cbn_plan* plan) {
    if (!plan) return CBN_OK;
    for (int i = 0; i < cbn_plan::kRing; ++i)
        for (int k = 0; k < 3; ++k)
            if (plan->ev[i][k]) (void)hipEventDestroy(plan->ev[i][k]);
    if (plan->d_fac) (void)hipFree(plan->d_fac);
    if (plan->d_crec) (void)hipFree(plan->d_crec);
    if (plan->d_slots) (void)hipFree(plan->d_slots);
    if (plan->d_build) (void)hipFree(plan->d_build);
    if (plan->d_image) (void)hipFree(plan->d_image);
    if (plan->d_sync) (void)hipFree(plan->d_sync);
    if (plan->h_status) (void)hipHostFree(plan->h_status);
    if (plan->param) param_destroy(plan->param);
    if (plan->direct) direct_destroy(plan->direct);
    delete plan;
    return CBN_OK;
}

int64_t cbn_plan_table_bytes(const cbn_plan* plan) {
    return plan ? (int64_t)plan->image_floats * (int64_t)sizeof(float) : -1;
}

int cbn_plan_uses_lds(const cbn_plan* plan) { return plan && plan->use_lds ? 1 : 0; }

int cbn_plan_build_tables(cbn_plan* plan, void* stream) {
    if (!plan) return set_err(CBN_E_ARG, "null plan");
    if (plan->direct) return direct_build_consts(plan->direct, reinterpret_cast<hipStream_t>(stream));
    if (plan->build_units == 0) return CBN_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    long long blocks = ((long long)plan->build_units * kWave + kBuildThreads - 1) / kBuildThreads;
    blocks = std::max(1LL, std::min(blocks, (long long)num_cu() * 8));
    hipLaunchKernelGGL(k_build_tables, dim3((unsigned)blocks), dim3(kBuildThreads), 0, s, plan->d_fac,
                       plan->d_build, plan->n_build, plan->build_units, plan->N, plan->RS, plan->d_image);
    HIP_TRY(hipGetLastError());
    if (plan->prefix > 0) {
        PrefixOffs po;
        for (int i = 0; i < 9; ++i) po.off[i] = plan->prefix_offs[i];
        const int n = plan->prefix_rows * plan->N;
        hipLaunchKernelGGL(k_merge_prefix, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, plan->d_image, po,
                           plan->prefix, plan->prefix_rows, plan->N, plan->RS);
        HIP_TRY(hipGetLastError());
    }
    return CBN_OK;
}

int cbn_plan_query_max(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                       uint32_t* max_bits, void* stream) {
    if (!plan || !max_bits || n_queries < 0) return set_err(CBN_E_ARG, "cbn_plan_query_max: bad arguments");
    if (plan->param || plan->direct)
        return set_err(CBN_E_UNSUPPORTED, "parametric / direct plans run through cbn_plan_run (raw + scale)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (n_queries == 0) {
        HIP_TRY(hipMemsetAsync(max_bits, 0, sizeof(uint32_t), s));
        return CBN_OK;
    }
    return dispatch_query<false>(plan, n_queries, evidence, n_evidence, max_bits, nullptr, s);
}

int cbn_plan_query_write(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                         const uint32_t* max_bits, float* out, void* stream) {
    if (!plan || !max_bits || n_queries < 0 || (n_queries > 0 && !out))
        return set_err(CBN_E_ARG, "cbn_plan_query_write: bad arguments");
    if (plan->param || plan->direct)
        return set_err(CBN_E_UNSUPPORTED, "parametric / direct plans run through cbn_plan_run (raw + scale)");
    return dispatch_query<true>(plan, n_queries, evidence, n_evidence, const_cast<uint32_t*>(max_bits), out,
                                reinterpret_cast<hipStream_t>(stream));
}

int cbn_plan_run(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                 uint32_t* max_bits, float* out, int32_t flags, void* stream) {
    if (!plan) return set_err(CBN_E_ARG, "null plan");
    if (plan->h_status && __atomic_load_n(plan->h_status, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(plan->h_status, 0u, __ATOMIC_RELEASE);
        return set_err(CBN_E_TIMEOUT, "an earlier single-launch call of this plan timed out in its grid barrier "
                                      "(not every block was resident); its rows are NaN");
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if (plan->direct) return direct_run(plan, n_queries, evidence, n_evidence, max_bits, out, flags, s);
    if (plan->param) {
        hipEvent_t* e = nullptr;
        if ((flags & CBN_RUN_TIMED) && plan->ev_n < cbn_plan::kRing) {
            e = plan->ev[plan->ev_n];
            for (int k = 0; k < 3; ++k)
                if (!e[k]) HIP_TRY(hipEventCreate(&e[k]));
            ++plan->ev_n;
            HIP_TRY(hipEventRecord(e[0], s));
            HIP_TRY(hipEventRecord(e[1], s));
        }
        rc = param_run(plan, n_queries, evidence, n_evidence, max_bits, out, flags, s);
        if (rc) return rc;
        if (e) HIP_TRY(hipEventRecord(e[2], s));
        return CBN_OK;
    }
    if (flags & CBN_RUN_BUILD_TABLES) {
        rc = cbn_plan_build_tables(plan, stream);
        if (rc) return rc;
    }
    hipEvent_t* e = nullptr;
    if ((flags & CBN_RUN_TIMED) && plan->ev_n < cbn_plan::kRing) {
        e = plan->ev[plan->ev_n];
        for (int k = 0; k < 3; ++k)
            if (!e[k]) HIP_TRY(hipEventCreate(&e[k]));
        ++plan->ev_n;
        HIP_TRY(hipEventRecord(e[0], s));
    }
    if (flags & CBN_RUN_RAW) {
        if (!plan->fast) return set_err(CBN_E_UNSUPPORTED, "cbn_plan_run: raw launch needs a fast-path plan");
        if (n_evidence != plan->ns) return set_err(CBN_E_ARG, "plan expects %d evidence columns, got %d", plan->ns, n_evidence);
        if (!out || !max_bits) return set_err(CBN_E_ARG, "cbn_plan_run: null output");
        if (!plan->d_image || !plan->d_sync) return set_err(CBN_E_ARG, "plan has no device buffers");
        if (n_queries <= 0) return set_err(CBN_E_ARG, "cbn_plan_run: raw launch needs >= 1 query");
        EvPtrs ev;
        memset(&ev, 0, sizeof(ev));
        for (int i = 0; i < n_evidence; ++i) {
            if (!evidence[i]) return set_err(CBN_E_ARG, "null evidence column %d", i);
            ev.p[i] = evidence[i];
        }
        if (e) HIP_TRY(hipEventRecord(e[1], s));
        if (plan->use_lds)
            rc = plan->vpl == 2 ? launch_raw_v<2, true>(plan, n_queries, ev, max_bits, out, s)
                                : launch_raw_v<1, true>(plan, n_queries, ev, max_bits, out, s);
        else
            rc = plan->vpl == 2 ? launch_raw_v<2, false>(plan, n_queries, ev, max_bits, out, s)
                                : launch_raw_v<1, false>(plan, n_queries, ev, max_bits, out, s);
        if (rc) return rc;
        if (e) HIP_TRY(hipEventRecord(e[2], s));
        return CBN_OK;
    }
    if (n_queries > 0 && !(flags & CBN_RUN_TWO_PASS) && fused_capacity(plan) >= n_queries) {
        // one launch: both passes with the products held in registers across a grid barrier
        if (n_evidence != plan->ns) return set_err(CBN_E_ARG, "plan expects %d evidence columns, got %d", plan->ns, n_evidence);
        if (!out || !max_bits) return set_err(CBN_E_ARG, "cbn_plan_run: null output");
        EvPtrs ev;
        memset(&ev, 0, sizeof(ev));
        for (int i = 0; i < n_evidence; ++i) ev.p[i] = evidence[i];
        if (e) HIP_TRY(hipEventRecord(e[1], s));
        if (plan->use_lds)
            rc = plan->vpl == 2 ? launch_fused_v<2, true>(plan, n_queries, ev, max_bits, out, s)
                                : launch_fused_v<1, true>(plan, n_queries, ev, max_bits, out, s);
        else
            rc = plan->vpl == 2 ? launch_fused_v<2, false>(plan, n_queries, ev, max_bits, out, s)
                                : launch_fused_v<1, false>(plan, n_queries, ev, max_bits, out, s);
        if (rc) return rc;
        if (e) HIP_TRY(hipEventRecord(e[2], s));
        return CBN_OK;
    }
    if (plan->fast && n_queries > 0 && !(flags & CBN_RUN_TWO_PASS) && reinterpret_cast<uintptr_t>(out) % 16 == 0) {
        // beyond the single launch: ONE compute pass (raw: unnormalised rows +
        // per-block maxima) and an HBM-bound in-place scale that reduces the
        // words, divides and publishes the max in *max_bits -- instead of
        // computing every product twice (max pass + write pass)
        if (n_evidence != plan->ns) return set_err(CBN_E_ARG, "plan expects %d evidence columns, got %d", plan->ns, n_evidence);
        if (!max_bits) return set_err(CBN_E_ARG, "cbn_plan_run: null output");
        EvPtrs ev;
        memset(&ev, 0, sizeof(ev));
        for (int i = 0; i < n_evidence; ++i) {
            if (!evidence[i]) return set_err(CBN_E_ARG, "null evidence column %d", i);
            ev.p[i] = evidence[i];
        }
        unsigned* words = plan->d_sync + kMaxWordOff;
        if (plan->use_lds)
            rc = plan->vpl == 2 ? launch_raw_v<2, true>(plan, n_queries, ev, words, out, s)
                                : launch_raw_v<1, true>(plan, n_queries, ev, words, out, s);
        else
            rc = plan->vpl == 2 ? launch_raw_v<2, false>(plan, n_queries, ev, words, out, s)
                                : launch_raw_v<1, false>(plan, n_queries, ev, words, out, s);
        if (rc) return rc;
        if (e) HIP_TRY(hipEventRecord(e[1], s));
        rc = launch_scale(out, n_queries * (long long)plan->N, words, plan->max_slots, max_bits, s);
        if (rc) return rc;
        if (e) HIP_TRY(hipEventRecord(e[2], s));
        return CBN_OK;
    }
    if (plan->fast && n_queries > 0) {
        // two launches: per-block maxima into the plan's words, then the write
        // pass reduces them itself and publishes the max in *max_bits
        if (n_evidence != plan->ns) return set_err(CBN_E_ARG, "plan expects %d evidence columns, got %d", plan->ns, n_evidence);
        if (!out || !max_bits) return set_err(CBN_E_ARG, "cbn_plan_run: null output");
        EvPtrs ev;
        memset(&ev, 0, sizeof(ev));
        for (int i = 0; i < n_evidence; ++i) {
            if (!evidence[i]) return set_err(CBN_E_ARG, "null evidence column %d", i);
            ev.p[i] = evidence[i];
        }
        unsigned* words = plan->d_sync + kMaxWordOff;
        const bool lds = plan->use_lds;
        if (plan->vpl == 2)
            rc = lds ? launch_fast_v<2, true, false>(plan, n_queries, ev, nullptr, 0, words, nullptr, s)
                     : launch_fast_v<2, false, false>(plan, n_queries, ev, nullptr, 0, words, nullptr, s);
        else
            rc = lds ? launch_fast_v<1, true, false>(plan, n_queries, ev, nullptr, 0, words, nullptr, s)
                     : launch_fast_v<1, false, false>(plan, n_queries, ev, nullptr, 0, words, nullptr, s);
        if (rc) return rc;
        if (e) HIP_TRY(hipEventRecord(e[1], s));
        if (plan->vpl == 2)
            rc = lds ? launch_fast_v<2, true, true>(plan, n_queries, ev, words, plan->max_slots, max_bits, out, s)
                     : launch_fast_v<2, false, true>(plan, n_queries, ev, words, plan->max_slots, max_bits, out, s);
        else
            rc = lds ? launch_fast_v<1, true, true>(plan, n_queries, ev, words, plan->max_slots, max_bits, out, s)
                     : launch_fast_v<1, false, true>(plan, n_queries, ev, words, plan->max_slots, max_bits, out, s);
        if (rc) return rc;
        if (e) HIP_TRY(hipEventRecord(e[2], s));
        return CBN_OK;
    }
    rc = cbn_plan_query_max(plan, n_queries, evidence, n_evidence, max_bits, stream);
    if (rc) return rc;
    if (e) HIP_TRY(hipEventRecord(e[1], s));
    rc = cbn_plan_query_write(plan, n_queries, evidence, n_evidence, max_bits, out, stream);
    if (rc) return rc;
    if (e) HIP_TRY(hipEventRecord(e[2], s));
    return CBN_OK;
}

int cbn_plan_run_fold(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                      uint32_t* max_bits, float* out, float* fold_rows, int64_t fold_n_elems,
                      const uint32_t* fold_words, int32_t fold_n_words, int32_t flags, void* stream) {
    if (!plan) return set_err(CBN_E_ARG, "null plan");
    if (!fold_rows || fold_n_elems <= 0) return cbn_plan_run(plan, n_queries, evidence, n_evidence, max_bits, out,
                                                             flags | CBN_RUN_RAW, stream);
    if (!plan->fast || !plan->staged || plan->direct || plan->param)
        return set_err(CBN_E_UNSUPPORTED, "cbn_plan_run_fold: needs a staged (paired N = 32) table plan");
    if (fold_n_elems % 4 || reinterpret_cast<uintptr_t>(fold_rows) % 16 || !fold_words || fold_n_words < 1 ||
        fold_n_words > kFoldW * kWave)
        return set_err(CBN_E_ARG, "cbn_plan_run_fold: fold rows must be 16-B aligned float4s, 1..%d words",
                       kFoldW * kWave);
    if (plan->h_status && __atomic_load_n(plan->h_status, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(plan->h_status, 0u, __ATOMIC_RELEASE);
        return set_err(CBN_E_TIMEOUT, "an earlier single-launch call of this plan timed out in its grid barrier "
                                      "(not every block was resident); its rows are NaN");
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc;
    if (flags & CBN_RUN_BUILD_TABLES) {
        rc = cbn_plan_build_tables(plan, stream);
        if (rc) return rc;
    }
    if (n_evidence != plan->ns) return set_err(CBN_E_ARG, "plan expects %d evidence columns, got %d", plan->ns, n_evidence);
    if (!out || !max_bits) return set_err(CBN_E_ARG, "cbn_plan_run_fold: null output");
    if (n_queries <= 0) return set_err(CBN_E_ARG, "cbn_plan_run_fold: raw launch needs >= 1 query");
    EvPtrs ev;
    memset(&ev, 0, sizeof(ev));
    for (int i = 0; i < n_evidence; ++i) {
        if (!evidence[i]) return set_err(CBN_E_ARG, "null evidence column %d", i);
        ev.p[i] = evidence[i];
    }
    hipEvent_t* e = nullptr;
    if ((flags & CBN_RUN_TIMED) && plan->ev_n < cbn_plan::kRing) {
        e = plan->ev[plan->ev_n];
        for (int k = 0; k < 3; ++k)
            if (!e[k]) HIP_TRY(hipEventCreate(&e[k]));
        ++plan->ev_n;
        HIP_TRY(hipEventRecord(e[0], s));
        HIP_TRY(hipEventRecord(e[1], s));
    }
    FoldJob fj;
    memset(&fj, 0, sizeof(fj));
    fj.rows = fold_rows;
    fj.words = fold_words;
    fj.n4 = fold_n_elems / 4;
    fj.n_words = fold_n_words;
    rc = plan->vpl == 2 ? launch_raw_v<2, true>(plan, n_queries, ev, max_bits, out, s, &fj)
                        : launch_raw_v<1, true>(plan, n_queries, ev, max_bits, out, s, &fj);
    if (rc) return rc;
    if (e) HIP_TRY(hipEventRecord(e[2], s));
    return CBN_OK;
}

int cbn_plan_status(cbn_plan* plan, int32_t* status) {
    if (!plan || !status) return set_err(CBN_E_ARG, "cbn_plan_status: bad arguments");
    unsigned v = 0;
    HIP_TRY(hipMemcpy(&v, plan->d_sync + 2, sizeof(unsigned), hipMemcpyDeviceToHost));
    *status = (int32_t)v;
    if (plan->h_status) __atomic_store_n(plan->h_status, 0u, __ATOMIC_RELEASE);  // reported here
    return CBN_OK;
}

int cbn_plan_check(cbn_plan* plan) {
    if (!plan) return set_err(CBN_E_ARG, "cbn_plan_check: null plan");
    if (plan->h_status && __atomic_load_n(plan->h_status, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(plan->h_status, 0u, __ATOMIC_RELEASE);
        return set_err(CBN_E_TIMEOUT, "a single-launch call of this plan timed out in its grid barrier (another "
                                      "stream held CUs its blocks needed): its rows are NaN");
    }
    return CBN_OK;
}

int64_t cbn_plan_fused_capacity(const cbn_plan* plan) { return plan ? fused_capacity(plan) : 0; }

int32_t cbn_plan_flags(const cbn_plan* plan) {
    if (!plan) return 0;
    return (plan->fast ? CBN_PLAN_FAST : 0) | (plan->use_lds ? CBN_PLAN_LDS : 0) |
           (plan->paired ? CBN_PLAN_PAIRED : 0) | (plan->staged ? CBN_PLAN_STAGED : 0) |
           (plan->fused_ok ? CBN_PLAN_FUSED : 0) | (plan->param ? CBN_PLAN_PARAMETRIC : 0) |
           (plan->vpl == 2 ? CBN_PLAN_VPL2 : 0) | (plan->direct ? CBN_PLAN_DIRECT : 0) |
           (plan->cols ? CBN_PLAN_COLS : 0) | (plan->slots ? CBN_PLAN_SLOTS : 0);
}

int32_t cbn_plan_max_words(const cbn_plan* plan) {
    if (plan && plan->param) return param_max_words(plan->param);
    if (plan && plan->direct) return direct_max_words(plan->direct);
    return plan && plan->fast ? plan->max_slots : 0;
}

int cbn_scale(float* out, int64_t n, const uint32_t* max_bits, int32_t n_max, void* stream) {
    if (n < 0 || n_max < 1 || (n > 0 && (!out || !max_bits))) return set_err(CBN_E_ARG, "cbn_scale: bad arguments");
    if (n == 0) return CBN_OK;
    if (reinterpret_cast<uintptr_t>(out) % 16) return set_err(CBN_E_ARG, "cbn_scale: out must be 16-B aligned");
    return launch_scale(out, (long long)n, max_bits, (int)n_max, nullptr, reinterpret_cast<hipStream_t>(stream));
}

namespace {
// blocks per CU of the batched scale (CBN_SCALE_BLOCKS_PER_CU, A/B knob)
int scale_blocks_per_cu() {
    static int v = [] {
        const char* e = diag_env("CBN_SCALE_BLOCKS_PER_CU");
        const int x = e ? atoi(e) : 0;
        return x >= 1 && x <= 16 ? x : 1;
    }();
    return v;
}
}  // namespace

int cbn_scale_batch(float* const* outs, const int64_t* n_elems, int32_t n_batches, const uint32_t* max_bits,
                    int32_t n_max, void* stream) {
    if (n_batches < 0 || n_batches > kScaleBatch || n_max < 1 || (n_batches > 0 && (!outs || !n_elems || !max_bits)))
        return set_err(CBN_E_ARG, "cbn_scale_batch: bad arguments (at most %d batches)", kScaleBatch);
    if (n_batches == 0) return CBN_OK;
    ScaleBatch sb;
    memset(&sb, 0, sizeof(sb));
    long long most = 0;
    for (int b = 0; b < n_batches; ++b) {
        if (n_elems[b] < 0 || (n_elems[b] > 0 && !outs[b])) return set_err(CBN_E_ARG, "cbn_scale_batch: bad batch %d", b);
        if (reinterpret_cast<uintptr_t>(outs[b]) % 16) return set_err(CBN_E_ARG, "cbn_scale_batch: out must be 16-B aligned");
        sb.out[b] = outs[b];
        sb.n[b] = n_elems[b];
        most = std::max(most, (long long)n_elems[b]);
    }
    // grid: scale_blocks_per_cu() 256-thread blocks per CU over all batches (each
    // thread kScaleU float4 in flight)
    long long blocks = (most / 4 + 256LL * kScaleU - 1) / (256LL * kScaleU);
    const long long cap = std::max(1LL, (long long)scale_blocks_per_cu() * num_cu() / n_batches);
    blocks = std::max(1LL, std::min(blocks, cap));
    hipLaunchKernelGGL(k_scale_batch, dim3((unsigned)blocks, (unsigned)n_batches), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), sb, max_bits, (int)n_max);
    HIP_TRY(hipGetLastError());
    return CBN_OK;
}

int cbn_plan_timing(cbn_plan* plan, int32_t* n_timed, float* avg_max_ms, float* avg_write_ms) {
    if (!plan || !n_timed || !avg_max_ms || !avg_write_ms) return set_err(CBN_E_ARG, "cbn_plan_timing: bad arguments");
    double a = 0, b = 0;
    for (int i = 0; i < plan->ev_n; ++i) {
        float t0 = 0, t1 = 0;
        HIP_TRY(hipEventSynchronize(plan->ev[i][2]));
        HIP_TRY(hipEventElapsedTime(&t0, plan->ev[i][0], plan->ev[i][1]));
        HIP_TRY(hipEventElapsedTime(&t1, plan->ev[i][1], plan->ev[i][2]));
        a += t0;
        b += t1;
    }
    *n_timed = plan->ev_n;
    *avg_max_ms = plan->ev_n ? (float)(a / plan->ev_n) : 0.f;
    *avg_write_ms = plan->ev_n ? (float)(b / plan->ev_n) : 0.f;
    plan->ev_n = 0;
    return CBN_OK;
}

int cbn_plan_infer(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                   uint32_t* max_bits, float* out, void* stream) {
    int rc = cbn_plan_build_tables(plan, stream);
    if (rc) return rc;
    rc = cbn_plan_query_max(plan, n_queries, evidence, n_evidence, max_bits, stream);
    if (rc) return rc;
    return cbn_plan_query_write(plan, n_queries, evidence, n_evidence, max_bits, out, stream);
}

}  // extern "C"
