// cbn_param.hip -- MI355X (gfx950) kernels for the parametric (continuous)
// CPDs on the inference path of BayesianNetwork.infer:
//   LinearRegression   (cbn/parameter_learning/linear_regression.py:104-124)
//   LogisticRegression (cbn/parameter_learning/logistIc_regression.py:70-100)
//   NeuralNetwork      (cbn/parameter_learning/neural_network.py:99-131)
// fed through Node.get_prob (cbn/base/node.py:115-204) and the factor loop of
// bayesian_network.py:269-296.
//
// Unlike the BruteForce tables, a parametric factor depends on the evidence
// VALUES (mu = model(parents)), so nothing per query can be tabulated: the
// query kernel evaluates, per query and factor, the model and the density at
// the node's N sample points, averages over the free parents' sample combos
// (torch.mean over the parent axes) and multiplies into the running product
// in the reference's factor order.  The work is transcendental-bound (one
// exp per (query, factor, column)), not HBM-bound.
//
// Layout: the plan image (global, read-only) holds per-factor records,
// weights, sample points and the query-independent factors' rows; a wave's
// lanes are 64 consecutive queries sharing one column chunk, so every image
// read is wave-uniform (scalar loads into SGPRs, no LDS, no VGPRs for
// weights) and the evidence loads are coalesced along the query axis.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "cbn_internal.h"

using namespace cbn;

namespace {

constexpr int kMaxP = CBN_MAX_PARENTS;
constexpr int kMaxL = CBN_MAX_LAYERS;
constexpr int kThreads = 256;   // const / eval kernels
constexpr int kQThreads = 512;  // query kernel: 8 waves per block, so the <= 1024-block grid holds 8 waves per SIMD
constexpr int kColPad = 32;
constexpr int kInputNone = -3;  // unused model input slot (reads the {0, 1} cell)  // sample / constant rows padded to the widest column chunk

#define PHIP_TRY(expr)                                                                    \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return set_err(CBN_E_HIP, "%s failed: %s", #expr, hipGetErrorString(_e));     \
    } while (0)

// Model shape (wave-uniform): nn.Linear stack, activation between layers.
struct MDesc {
    int n_layers;
    int act;
    int width[kMaxL + 1];
};

// Per-factor record in the plan image (128 B).
struct alignas(16) PRec {
    int kind;      // CBN_FACTOR_*
    int family;    // CBN_FAMILY_*
    int unit;      // scale == 1 exactly: (x - mu) / 1 == x - mu, skip the division
    int M;         // free-parent sample combos N^n_free (1: none)
    MDesc m;       // 7 ints
    int w_off;     // float offsets in the image: weights, node samples [N],
    int s_off;     //   free-input samples [width0][N], query-independent row [N]
    int fs_off;
    int c_off;
    float scale;
    float norm;
    int in_slot[kMaxP];
    float inv_scale;  // fp32 1 / scale (Newton-refined division by the scale)
    int free_mask;    // bit i: model input i is a free parent (sampled per combo)
    int pw_off;       // one-hidden-layer models: image offset of the pair-packed weights (0: none)
    int pad[4];
};
static_assert(sizeof(PRec) == 128, "PRec layout");
constexpr int kRecFloats = sizeof(PRec) / 4;

// Per-factor hot header (64 B, one scalar load) of the column-table kernels
// whose factors all have every parent observed (M1): everything the factor
// loop reads per factor, at an address known without a dependent load (the
// header array follows the {0, 1} cell), so the next factor's header is in
// flight while the current one is evaluated.
struct alignas(16) PHead {
    int kind;      // CBN_FACTOR_*
    int row;       // image offset: node samples (QUERY) or the query-independent row
    int wp;        // image offset: pair-packed MLP weights (n_layers 2) or [w0..w3, bias] (linear)
    int n_in;
    int hid;       // hidden width (n_layers 2)
    int n_layers;
    int act;
    float scale;
    float inv_scale;
    float norm;
    int pad[6];
};
static_assert(sizeof(PHead) == 64, "PHead layout");
constexpr int kHeadFloats = sizeof(PHead) / 4;

// Kernel-argument pointer table (3 KiB of the 4 KiB kernarg space).  Table
// mode: p[f * kTabIn + i] = column of input i of factor f (evidence, or null
// for inputs that are not evidence: not loaded), read with scalar loads into SGPRs.
// Slot mode (plans beyond the table): p[slot] = evidence column of the slot.
constexpr int kTabIn = 4;
constexpr int kTabCols = 384;  // 96 factors x 4 inputs
struct PEv {
    const float* p[kTabCols];
};

typedef const __attribute__((address_space(1))) float gfloat_t;
__device__ __forceinline__ float gload(const float* p, long long i) { return ((gfloat_t*)p)[i]; }
// element at a 32-bit byte offset: a uniform base plus one VGPR offset shared
// by every column (global_load ... saddr), not a 64-bit address per column
__device__ __forceinline__ float gload_b(const float* p, unsigned byte_off) {
    typedef const __attribute__((address_space(1))) char gchar_t;
    return *(gfloat_t*)((gchar_t*)p + byte_off);
}

__device__ __forceinline__ unsigned wave_max_u(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (unsigned)__shfl_xor((int)v, o, kWave));
    return v;
}

// n / d to within one ulp of the correctly rounded quotient: v_rcp_f32 + one
// Newton step (4 VALU slots instead of the ~12 of the IEEE division
// sequence).  v_rcp_f32 flushes reciprocals below 2^-126, so denominators
// above 2^126 (a logistic (1 + e)^2 near FLT_MAX), inf and NaN take the IEEE
// division -- a branch no lane takes in range, skipped by the whole wave.
__device__ __forceinline__ float div_nr(float n, float d, float r) {
    const float q = n * r;
    float res = fmaf(fmaf(-d, q, n), r, q);
    if (!(d <= 0x1p126f)) res = n / d;
    return res;
}
__device__ __forceinline__ float div_nr(float n, float d) { return div_nr(n, d, __builtin_amdgcn_rcpf(d)); }

// exp(x) within ~2 ulp for results >= 2^-126 in 7 VALU slots (libm expf: 13):
// x log2(e) = hi + lo exactly (product residual by fma, plus x times the
// low part of log2(e)), 2^hi by v_exp_f32, 2^lo ~ 1 + lo ln2 (|lo| <= 2^-24
// |hi|).  x below -104 (exp underflows) is clamped so the residual stays
// finite; NaN passes through (comparisons false).  v_exp_f32 returns 0 where
// 2^hi is subnormal (hi < -126), so there 2^(hi + 64) is scaled by 2^-64: the
// subnormal results the reference keeps (a branch the wave skips unless a
// lane needs it) -- bounded in tests/test_gpu_param.py::test_density_accuracy_full_range.
__device__ __forceinline__ float exp_split(float x) {
#pragma clang fp contract(off)
    constexpr float kL = 1.44269502162933349609375f;  // fp32(log2 e)
    constexpr float kLlo = 1.925963033500e-8f;       // log2 e - kL
    constexpr float kLn2 = 0.693147180559945309f;
    x = x < -104.f ? -104.f : x;
    const float ph = x * kL;
    const float pl = fmaf(x, kLlo, fmaf(x, kL, -ph));
    float r = __builtin_amdgcn_exp2f(ph);
    // ph + 64 is exact -- and must not be contracted into fma(x, kL, 64), whose
    // different rounding pl would not correct.  A wave-uniform branch: the
    // second transcendental runs only when some lane needs it
    if (__builtin_expect(__any(ph < -126.f), 0)) {
        const float rs = __builtin_amdgcn_exp2f(ph + 64.f) * 0x1p-64f;
        r = ph < -126.f ? rs : r;
    }
    return fmaf(r, pl * kLn2, r);
}

// Two fp32 lanes per VALU op: gfx950's packed fp32 FMA / MUL / ADD
// (v_pk_*_f32) run two independent columns / hidden units per instruction at
// the rate of one -- the parametric kernel is VALU-issue bound.  The packed
// ops are the same IEEE operations, so a pair gives the bits of two scalar
// evaluations.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 f2s(float a) { return f2{a, a}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// exp_split on a pair (the two v_exp_f32 are scalar: transcendentals do not pack)
__device__ __forceinline__ f2 exp_split2_full(f2 x) {
#pragma clang fp contract(off)
    constexpr float kL = 1.44269502162933349609375f;
    constexpr float kLlo = 1.925963033500e-8f;
    constexpr float kLn2 = 0.693147180559945309f;
    x.x = x.x < -104.f ? -104.f : x.x;
    x.y = x.y < -104.f ? -104.f : x.y;
    const f2 ph = x * f2s(kL);
    const f2 pl = fma2(x, f2s(kLlo), fma2(x, f2s(kL), -ph));
    f2 r = f2{__builtin_amdgcn_exp2f(ph.x), __builtin_amdgcn_exp2f(ph.y)};
    if (__builtin_expect(__any(fminf(ph.x, ph.y) < -126.f), 0)) {  // subnormal results (see exp_split)
        const float sx = __builtin_amdgcn_exp2f(ph.x + 64.f) * 0x1p-64f;
        const float sy = __builtin_amdgcn_exp2f(ph.y + 64.f) * 0x1p-64f;
        r.x = ph.x < -126.f ? sx : r.x;
        r.y = ph.y < -126.f ? sy : r.y;
    }
    return fma2(r, pl * f2s(kLn2), r);
}

// exp_split2 with the clamp and the subnormal fix-up taken only when some
// lane of the wave needs them: where no lane has x log2(e) < -126 (so x >
// -104 and the result is normal) the clamp is a no-op and the fix-up is
// skipped by exp_split2_full too, so the bits are the same; otherwise the
// whole wave runs exp_split2_full.  4 VALU slots fewer per pair.
__device__ __forceinline__ f2 exp_split2(f2 x) {
#pragma clang fp contract(off)
    constexpr float kL = 1.44269502162933349609375f;
    constexpr float kLlo = 1.925963033500e-8f;
    constexpr float kLn2 = 0.693147180559945309f;
    const f2 ph = x * f2s(kL);
    if (__builtin_expect(__any(fminf(ph.x, ph.y) < -126.f), 0)) return exp_split2_full(x);
    const f2 pl = fma2(x, f2s(kLlo), fma2(x, f2s(kL), -ph));
    const f2 r = f2{__builtin_amdgcn_exp2f(ph.x), __builtin_amdgcn_exp2f(ph.y)};
    return fma2(r, pl * f2s(kLn2), r);
}

// exp(-0.5 t2) (the Gaussian's exp(-0.5 ((x - mu) / s)^2)) == exp_split2(-0.5f * t2)
// bit for bit without the multiply: -0.5 t2 is exact (a power-of-two scale;
// t2 >= 0, and where it would round, t2 < 2^-125, the result is 1 either
// way), so x log2(e) = t2 (-0.5 log2(e)) and the residual fmas take the
// halved constants exactly.
__device__ __forceinline__ f2 exp_neg_half2(f2 t2) {
#pragma clang fp contract(off)
    constexpr float kHL = -0.5f * 1.44269502162933349609375f;
    constexpr float kHLlo = -0.5f * 1.925963033500e-8f;
    constexpr float kLn2 = 0.693147180559945309f;
    const f2 ph = t2 * f2s(kHL);
    if (__builtin_expect(__any(fminf(ph.x, ph.y) < -126.f), 0)) return exp_split2_full(f2s(-0.5f) * t2);
    const f2 pl = fma2(t2, f2s(kHLlo), fma2(t2, f2s(kHL), -ph));
    const f2 r = f2{__builtin_amdgcn_exp2f(ph.x), __builtin_amdgcn_exp2f(ph.y)};
    return fma2(r, pl * f2s(kLn2), r);
}

// div_nr on a pair (same operations; the IEEE fallback per component)
__device__ __forceinline__ f2 div_nr2(f2 n, f2 d, f2 r) {
    const f2 q = n * r;
    f2 res = fma2(fma2(-d, q, n), r, q);
    if (!(d.x <= 0x1p126f)) res.x = n.x / d.x;
    if (!(d.y <= 0x1p126f)) res.y = n.y / d.y;
    return res;
}
__device__ __forceinline__ f2 div_nr2(f2 n, f2 d) {
    return div_nr2(n, d, f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)});
}

// tanh (nn.Tanh) within ~2 ulp in ~16 VALU slots (libm tanhf: ~30): |x| <
// 0.625: x + x^3 P(x^2), the odd minimax polynomial of the Cephes tanhf;
// else 1 - 2 / (1 + e^(2|x|)) (e^(2|x|) = inf -> 1); sign restored.  Both
// branches are evaluated (lanes of a wave diverge) and selected; NaN
// propagates through the second.
template <typename T>
__device__ __forceinline__ T tanh_poly(T ax) {
    const T z = ax * ax;
    T p = fma(z, T(-5.70498872745e-3f), T(2.06390887954e-2f));
    p = fma(p, z, T(-5.37397155531e-2f));
    p = fma(p, z, T(1.33314422036e-1f));
    p = fma(p, z, T(-3.33332819422e-1f));
    return fma(p * z, ax, ax);
}
__device__ __forceinline__ float tanh_fast(float x) {
    const float ax = fabsf(x);
    const float small = tanh_poly(ax);
    const float e = __builtin_amdgcn_exp2f(ax * 2.88539008177792681472f);  // 2 log2(e)
    const float big = fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + e), 1.f);
    return copysignf(ax < 0.625f ? small : big, x);
}
// (the pair form works on the signed x: the odd polynomial's IEEE operations
// are sign-symmetric, so it returns copysign(poly(|x|), x) bit for bit, and
// |x| reaches the exponential as a source modifier -- no separate |x|)
__device__ __forceinline__ f2 tanh_fast2(f2 x) {
    const f2 z = x * x;
    f2 p = fma2(z, f2s(-5.70498872745e-3f), f2s(2.06390887954e-2f));
    p = fma2(p, z, f2s(-5.37397155531e-2f));
    p = fma2(p, z, f2s(1.33314422036e-1f));
    p = fma2(p, z, f2s(-3.33332819422e-1f));
    const f2 small = fma2(p * z, x, x);
    const f2 t = x * f2s(2.88539008177792681472f);
    const f2 u = f2{__builtin_amdgcn_exp2f(fabsf(t.x)), __builtin_amdgcn_exp2f(fabsf(t.y))} + f2s(1.f);
    const f2 big = fma2(f2s(-2.f), f2{__builtin_amdgcn_rcpf(u.x), __builtin_amdgcn_rcpf(u.y)}, f2s(1.f));
    return f2{fabsf(x.x) < 0.625f ? small.x : copysignf(big.x, x.x),
              fabsf(x.y) < 0.625f ? small.y : copysignf(big.y, x.y)};
}

// activation_map of neural_network.py:10-18 (torch CPU formulas)
__device__ __forceinline__ float act1(int act, float x) {
    switch (act) {
        case CBN_ACT_TANH: return tanh_fast(x);
        case CBN_ACT_RELU: return x > 0.f ? x : 0.f;
        case CBN_ACT_SIGMOID:  // exp(-x) clamped below FLT_MAX: 1 / (1 + 3.3e38) for x < -88.7 (torch: 0)
            return div_nr(1.f, 1.f + exp_split(-x > 88.7f ? 88.7f : -x));  // NaN stays NaN
        case CBN_ACT_LEAKYRELU: return x > 0.f ? x : x * 0.01f;
        case CBN_ACT_GELU: return x * 0.5f * (1.f + erff(x * 0.70710678118654752440f));
        case CBN_ACT_ELU: return x > 0.f ? x : expm1f(x);
        default: return x;
    }
}

template <int H>
__device__ __forceinline__ void activate(int act, int w, float (&h)[H]) {
    switch (act) {  // wave-uniform: one unrolled loop per activation
        case CBN_ACT_TANH:
#pragma unroll
            for (int o = 0; o < H; ++o)
                if (o < w) h[o] = tanh_fast(h[o]);
            break;
        case CBN_ACT_RELU:
#pragma unroll
            for (int o = 0; o < H; ++o) h[o] = h[o] > 0.f ? h[o] : 0.f;
            break;
        case CBN_ACT_LEAKYRELU:
#pragma unroll
            for (int o = 0; o < H; ++o) h[o] = h[o] > 0.f ? h[o] : h[o] * 0.01f;
            break;
        default:
#pragma unroll
            for (int o = 0; o < H; ++o)
                if (o < w) h[o] = act1(act, h[o]);
            break;
    }
}

template <int ACT>
__device__ __forceinline__ f2 act2(int act, f2 x) {
    if (ACT == CBN_ACT_TANH) return tanh_fast2(x);
    if (ACT == CBN_ACT_RELU) return f2{x.x > 0.f ? x.x : 0.f, x.y > 0.f ? x.y : 0.f};
    return f2{act1(act, x.x), act1(act, x.y)};
}

// One hidden layer (the reference's default, neural_network.py:37): stream
// over the hidden units -- mu = b2 + sum_o W2[o] act(W1[o] . z + b1[o]) in o
// order (the output layer's fma chain) -- four units per step, so the
// wave-uniform weight reads of a step are issued together (scalar loads) and
// their latency is paid once per four units.  ACT 0: runtime activation.
template <int ACT>
__device__ __forceinline__ float mlp1(const float* __restrict__ W, int n_in, int H, const float (&z)[kMaxP],
                                      int act = ACT) {
    const float* B1 = W + H * n_in;
    const float* W2 = B1 + H;
    float mu = 0.f;
    int o = 0;
    for (; o + 4 <= H; o += 4) {  // units (o, o+1) and (o+2, o+3) as packed pairs
        f2 h[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            f2 a = f2s(0.f);
#pragma unroll
            for (int i = 0; i < kMaxP; ++i)
                if (i < n_in) a = fma2(f2{W[(o + 2 * u) * n_in + i], W[(o + 2 * u + 1) * n_in + i]}, f2s(z[i]), a);
            h[u] = act2<ACT>(act, a + f2{B1[o + 2 * u], B1[o + 2 * u + 1]});
        }
        mu = fmaf(W2[o], h[0].x, mu);
        mu = fmaf(W2[o + 1], h[0].y, mu);
        mu = fmaf(W2[o + 2], h[1].x, mu);
        mu = fmaf(W2[o + 3], h[1].y, mu);
    }
    for (; o < H; ++o) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < kMaxP; ++i)
            if (i < n_in) a = fmaf(W[o * n_in + i], z[i], a);
        mu = fmaf(W2[o], act1(act, a + B1[o]), mu);
    }
    return mu + W2[H];
}

// One hidden layer from the pair-packed weights (the query kernel's form of
// mlp1; same operations in the same order): per unit pair P the record
//   [W(2P, i), W(2P+1, i)] for i < NIN, [B1(2P), B1(2P+1)], [W2(2P), W2(2P+1)]
// (2 NIN + 4 floats; a padding unit of odd H has zeros and is never summed),
// then the output bias.  With NIN a compile-time constant every weight read
// is an immediate-offset scalar load from one pointer, and each (unit pair,
// input) weight pair sits in an SGPR pair the packed FMA takes as is.
template <int ACT, int NIN>
__device__ __forceinline__ float mlp1p(const float* __restrict__ PW, int H, const float (&z)[kMaxP], int act) {
    constexpr int kRec = 2 * NIN + 4;
    const int npairs = (H + 1) >> 1;
    float mu = 0.f;
    int P = 0;
    for (; P + 2 <= npairs; P += 2, PW += 2 * kRec) {
        f2 h[2], w2[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const f2* R = reinterpret_cast<const f2*>(PW + u * kRec);
            f2 a = f2s(0.f);
#pragma unroll
            for (int i = 0; i < NIN; ++i) a = fma2(R[i], f2s(z[i]), a);
            h[u] = act2<ACT>(act, a + R[NIN]);
            w2[u] = R[NIN + 1];
        }
        mu = fmaf(w2[0].x, h[0].x, mu);
        mu = fmaf(w2[0].y, h[0].y, mu);
        mu = fmaf(w2[1].x, h[1].x, mu);
        mu = fmaf(w2[1].y, h[1].y, mu);
    }
    if (P < npairs) {
        const f2* R = reinterpret_cast<const f2*>(PW);
        f2 a = f2s(0.f);
#pragma unroll
        for (int i = 0; i < NIN; ++i) a = fma2(R[i], f2s(z[i]), a);
        const f2 h = act2<ACT>(act, a + R[NIN]);
        const f2 w2 = R[NIN + 1];
        mu = fmaf(w2.x, h.x, mu);
        if (2 * P + 1 < H) mu = fmaf(w2.y, h.y, mu);
        PW += kRec;
    }
    return mu + PW[0];
}

// NMAX: the most inputs a factor of the launch can have (the column-table
// kernels take <= kTabIn): input counts beyond it are not instantiated, so
// their weight registers do not weigh on the kernel's SGPR allocation
template <int ACT, int NMAX>
__device__ __forceinline__ float mlp1p_nin(const float* __restrict__ PW, int n_in, int H, const float (&z)[kMaxP],
                                           int act) {
    switch (n_in) {  // wave-uniform
        case 1: return mlp1p<ACT, 1>(PW, H, z, act);
        case 2: return mlp1p<ACT, 2>(PW, H, z, act);
        case 3: return mlp1p<ACT, 3>(PW, H, z, act);
        case 4: return mlp1p<ACT, 4>(PW, H, z, act);
        case 5: if (NMAX >= 5) return mlp1p<ACT, 5 <= NMAX ? 5 : 1>(PW, H, z, act); [[fallthrough]];
        case 6: if (NMAX >= 6) return mlp1p<ACT, 6 <= NMAX ? 6 : 1>(PW, H, z, act); [[fallthrough]];
        case 7: if (NMAX >= 7) return mlp1p<ACT, 7 <= NMAX ? 7 : 1>(PW, H, z, act); [[fallthrough]];
        default: return mlp1p<ACT, NMAX>(PW, H, z, act);
    }
}

// the other activations: one instantiation, input count at run time
__device__ __forceinline__ float mlp1p_rt(const float* __restrict__ PW, int n_in, int H, const float (&z)[kMaxP],
                                       int act) {
    const int rec = 2 * n_in + 4;
    const int npairs = (H + 1) >> 1;
    float mu = 0.f;
    for (int P = 0; P < npairs; ++P, PW += rec) {
        const f2* R = reinterpret_cast<const f2*>(PW);
        f2 a = f2s(0.f);
#pragma unroll
        for (int i = 0; i < kMaxP; ++i)
            if (i < n_in) a = fma2(R[i], f2s(z[i]), a);
        const f2 h = act2<0>(act, a + R[n_in]);
        const f2 w2 = R[n_in + 1];
        mu = fmaf(w2.x, h.x, mu);
        if (2 * P + 1 < H) mu = fmaf(w2.y, h.y, mu);
    }
    return mu + PW[0];
}

template <int NMAX>
__device__ __forceinline__ float mlp1_packed(const PRec& r, const float* __restrict__ img, const float (&z)[kMaxP]) {
    const float* PW = img + r.pw_off;
    switch (r.m.act) {
        case CBN_ACT_TANH: return mlp1p_nin<CBN_ACT_TANH, NMAX>(PW, r.m.width[0], r.m.width[1], z, CBN_ACT_TANH);
        case CBN_ACT_RELU: return mlp1p_nin<CBN_ACT_RELU, NMAX>(PW, r.m.width[0], r.m.width[1], z, CBN_ACT_RELU);
        default: return mlp1p_rt(PW, r.m.width[0], r.m.width[1], z, r.m.act);
    }
}

// mu of a query factor: HMAX 1 plans hold linear and one-hidden-layer models
// (the latter always pair-packed)
template <int HMAX, int NMAX = kMaxP>
__device__ __forceinline__ float query_mu(const PRec& r, const float* __restrict__ img, const float* __restrict__ W,
                                          const float (&z)[kMaxP], float* deep);

// mu = model(z): y = W x + b per nn.Linear (dot product first, then the bias:
// addmm's order), activation after every layer but the last.  HMAX = 0: the
// linear-model instantiation (n_layers == 1 only).  The first hidden layer
// lives in registers; further hidden layers (the reference's default is one,
// neural_network.py:37) go through this thread's LDS scratch `deep`
// (2 x HMAX floats, stride kThreads), a compact runtime loop.
template <int HMAX, int STRIDE = kThreads>
__device__ __forceinline__ float model_mu(const MDesc& m, const float* __restrict__ W, const float (&z)[kMaxP],
                                          float* deep) {
    const int n_in = m.width[0];
    if (HMAX == 0 || m.n_layers == 1) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < kMaxP; ++i)
            if (i < n_in) s = fmaf(W[i], z[i], s);
        return s + W[n_in];
    } else if (HMAX == 1 || m.n_layers == 2) {
        switch (m.act) {  // wave-uniform: one branch per model evaluation, not per unit
            case CBN_ACT_TANH: return mlp1<CBN_ACT_TANH>(W, n_in, m.width[1], z);
            case CBN_ACT_RELU: return mlp1<CBN_ACT_RELU>(W, n_in, m.width[1], z);
            case CBN_ACT_SIGMOID: return mlp1<CBN_ACT_SIGMOID>(W, n_in, m.width[1], z);
            case CBN_ACT_LEAKYRELU: return mlp1<CBN_ACT_LEAKYRELU>(W, n_in, m.width[1], z);
            default: return mlp1<0>(W, n_in, m.width[1], z, m.act);
        }
    } else {
        constexpr int H = HMAX > 1 ? HMAX : 1;
        float h[H];
        int win = m.width[1];
        const float* B = W + win * n_in;
#pragma unroll
        for (int o = 0; o < H; ++o) {
            float s = 0.f;
            if (o < win) {
#pragma unroll
                for (int i = 0; i < kMaxP; ++i)
                    if (i < n_in) s = fmaf(W[o * n_in + i], z[i], s);
                s = s + B[o];
            }
            h[o] = s;
        }
        activate<H>(m.act, win, h);
        W = B + win;
        if (m.n_layers > 2) {
            float* src = deep;
            float* dst = deep + H * STRIDE;
#pragma unroll
            for (int i = 0; i < H; ++i) src[i * STRIDE] = h[i];
            for (int layer = 1; layer < m.n_layers - 1; ++layer) {
                const int wo = m.width[layer + 1];
                const float* Bl = W + wo * win;
                for (int o = 0; o < wo; ++o) {
                    float s = 0.f;
                    for (int i = 0; i < win; ++i) s = fmaf(W[o * win + i], src[i * STRIDE], s);
                    dst[o * STRIDE] = act1(m.act, s + Bl[o]);
                }
                float* t = src;
                src = dst;
                dst = t;
                W = Bl + wo;
                win = wo;
            }
#pragma unroll
            for (int i = 0; i < H; ++i) h[i] = i < win ? src[i * STRIDE] : 0.f;
        }
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < H; ++i)
            if (i < win) s = fmaf(W[i], h[i], s);
        return s + W[win];
    }
}

template <int HMAX, int NMAX>
__device__ __forceinline__ float query_mu(const PRec& r, const float* __restrict__ img, const float* __restrict__ W,
                                          const float (&z)[kMaxP], float* deep) {
    if (HMAX == 0) return model_mu<0>(r.m, W, z, deep);
    if (HMAX == 1) return r.m.n_layers == 2 ? mlp1_packed<NMAX>(r, img, z) : model_mu<0>(r.m, W, z, deep);
    return model_mu<HMAX, 512>(r.m, W, z, deep);
}

// Densities, in the reference's fp32 operation order (divisions within one
// ulp, see div_nr; exp within ~2 ulp, see exp_split).  MODE: 0 Gauss with scale 1, 1 Gauss, 2 logistic with
// scale 1, 3 logistic.  With scale == 1 exactly, (x - mu) / scale == x - mu.
template <int MODE>
__device__ __forceinline__ float pdf_t(float scale, float inv_scale, float norm, float x, float mu) {
    if (MODE <= 1) {
        // linear_regression.py:91-95
        const float t = MODE == 0 ? (x - mu) : div_nr(x - mu, scale, inv_scale);
        return norm * exp_split(-0.5f * (t * t));
    }
    // logistIc_regression.py:90-98 / neural_network.py:120-124
    const float d = MODE == 2 ? (x - mu) : div_nr(x - mu, scale, inv_scale);
    const float e = exp_split(-d);
    const float u = 1.f + e;
    return div_nr(e, MODE == 2 ? u * u : scale * (u * u));
}

__device__ __forceinline__ int mode_of(int family, bool unit) {
    return (family == CBN_FAMILY_GAUSS ? 0 : 2) + (unit ? 0 : 1);
}

__device__ __forceinline__ float pdf_eval(int mode, float scale, float inv_scale, float norm, float x, float mu) {
    switch (mode) {
        case 0: return pdf_t<0>(scale, inv_scale, norm, x, mu);
        case 1: return pdf_t<1>(scale, inv_scale, norm, x, mu);
        case 2: return pdf_t<2>(scale, inv_scale, norm, x, mu);
        default: return pdf_t<3>(scale, inv_scale, norm, x, mu);
    }
}

// pdf_t on two columns (packed; the same operations, so the same bits)
template <int MODE>
__device__ __forceinline__ f2 pdf2_t(float scale, float inv_scale, float norm, f2 x, float mu) {
    if (MODE <= 1) {
        const f2 t = MODE == 0 ? (x - f2s(mu)) : div_nr2(x - f2s(mu), f2s(scale), f2s(inv_scale));
        return f2s(norm) * exp_neg_half2(t * t);
    }
    const f2 d = MODE == 2 ? (x - f2s(mu)) : div_nr2(x - f2s(mu), f2s(scale), f2s(inv_scale));
    const f2 e = exp_split2(-d);
    const f2 u = f2s(1.f) + e;
    return div_nr2(e, MODE == 2 ? u * u : f2s(scale) * (u * u));
}

// s + x with the rounding error of the addition carried in c (TwoSum): the
// sum over the M free-parent combos of a mean stays within ~1 ulp whatever M
// (torch.mean's reduction is blocked/pairwise; a plain running fp32 sum over
// N^k terms drifts by ~M/2 ulp)
__device__ __forceinline__ void two_sum(float& s, float& c, float x) {
    const float t = s + x;
    const float z = t - s;
    c += (s - (t - z)) + (x - z);
    s = t;
}

// fx[j] (+ cx[j]) += pdf(S[j]; mu) over the chunk (S, scale, norm
// wave-uniform; S rows are padded to a multiple of kColPad, so no column
// predicates); column pairs packed
template <int NC, int MODE>
__device__ __forceinline__ void add_row_t(float (&fx)[NC], float (&cx)[NC], const float* __restrict__ S, float sc,
                                          float isc, float nm, float mu) {
    static_assert(NC % 2 == 0, "column pairs");
#pragma unroll
    for (int j = 0; j < NC; j += 2) {
        const f2 p = pdf2_t<MODE>(sc, isc, nm, f2{S[j], S[j + 1]}, mu);
        const f2 a = f2{fx[j], fx[j + 1]};
        const f2 t = a + p;
        const f2 z = t - a;
        const f2 c = f2{cx[j], cx[j + 1]} + ((a - (t - z)) + (p - z));
        fx[j] = t.x;
        fx[j + 1] = t.y;
        cx[j] = c.x;
        cx[j + 1] = c.y;
    }
}

#ifndef CBN_MULROW_GROUP
#define CBN_MULROW_GROUP 8
#endif
// pdf2_t's fast form on NP column pairs at once -- every wave-uniform
// fall-back of exp_split2 / exp_neg_half2 / div_nr2 assumed not taken -- plus
// what decides it: lo = the smallest x log2(e) of the exponentials (their
// fall-back: < -126), bad = a division whose fall-back (denominator > 2^126,
// inf or NaN) some lane needs.  Where neither is set the fast form IS
// pdf2_t, operation for operation.  Written step by step across the pairs
// (every pair's t, then every pair's t^2, ...): independent packed ops back
// to back, so the packed-math hazard nops of one pair's dependent chain are
// filled by the other pairs' work.
template <int NP, int MODE>
__device__ __forceinline__ void pdf2_fast(float scale, float inv_scale, float norm, const float* sv, float mu,
                                          f2 (&out)[NP], float& lo, bool& bad) {
#pragma clang fp contract(off)
    constexpr float kL = 1.44269502162933349609375f;
    constexpr float kLlo = 1.925963033500e-8f;
    constexpr float kLn2 = 0.693147180559945309f;
    f2 t[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) t[k] = f2{sv[2 * k], sv[2 * k + 1]} - f2s(mu);
    if (MODE == 1 || MODE == 3) {  // div_nr2 by the scale (uniform)
        f2 q[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) q[k] = t[k] * f2s(inv_scale);
#pragma unroll
        for (int k = 0; k < NP; ++k) t[k] = fma2(fma2(-f2s(scale), q[k], t[k]), f2s(inv_scale), q[k]);
        bad |= !(scale <= 0x1p126f);
    }
    f2 a[NP], ph[NP], pl[NP], r[NP];
    if (MODE <= 1) {  // exp_neg_half2(t * t)
        constexpr float kHL = -0.5f * kL, kHLlo = -0.5f * kLlo;
#pragma unroll
        for (int k = 0; k < NP; ++k) a[k] = t[k] * t[k];
#pragma unroll
        for (int k = 0; k < NP; ++k) ph[k] = a[k] * f2s(kHL);
#pragma unroll
        for (int k = 0; k < NP; ++k) r[k] = f2{__builtin_amdgcn_exp2f(ph[k].x), __builtin_amdgcn_exp2f(ph[k].y)};
#pragma unroll
        for (int k = 0; k < NP; ++k) pl[k] = fma2(a[k], f2s(kHL), -ph[k]);
#pragma unroll
        for (int k = 0; k < NP; ++k) pl[k] = fma2(a[k], f2s(kHLlo), pl[k]);
#pragma unroll
        for (int k = 0; k < NP; ++k) lo = fminf(lo, fminf(ph[k].x, ph[k].y));
#pragma unroll
        for (int k = 0; k < NP; ++k) pl[k] = pl[k] * f2s(kLn2);
#pragma unroll
        for (int k = 0; k < NP; ++k) r[k] = fma2(r[k], pl[k], r[k]);
#pragma unroll
        for (int k = 0; k < NP; ++k) out[k] = f2s(norm) * r[k];
        return;
    }
    // exp_split2(-t), then div_nr2(e, u^2 [* scale])
#pragma unroll
    for (int k = 0; k < NP; ++k) a[k] = -t[k];
#pragma unroll
    for (int k = 0; k < NP; ++k) ph[k] = a[k] * f2s(kL);
#pragma unroll
    for (int k = 0; k < NP; ++k) r[k] = f2{__builtin_amdgcn_exp2f(ph[k].x), __builtin_amdgcn_exp2f(ph[k].y)};
#pragma unroll
    for (int k = 0; k < NP; ++k) pl[k] = fma2(a[k], f2s(kL), -ph[k]);
#pragma unroll
    for (int k = 0; k < NP; ++k) pl[k] = fma2(a[k], f2s(kLlo), pl[k]);
#pragma unroll
    for (int k = 0; k < NP; ++k) lo = fminf(lo, fminf(ph[k].x, ph[k].y));
#pragma unroll
    for (int k = 0; k < NP; ++k) pl[k] = pl[k] * f2s(kLn2);
#pragma unroll
    for (int k = 0; k < NP; ++k) r[k] = fma2(r[k], pl[k], r[k]);  // e
#pragma unroll
    for (int k = 0; k < NP; ++k) a[k] = f2s(1.f) + r[k];  // u
#pragma unroll
    for (int k = 0; k < NP; ++k) a[k] = MODE == 2 ? a[k] * a[k] : f2s(scale) * (a[k] * a[k]);  // d
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        ph[k] = f2{__builtin_amdgcn_rcpf(a[k].x), __builtin_amdgcn_rcpf(a[k].y)};
        bad |= !(a[k].x <= 0x1p126f) || !(a[k].y <= 0x1p126f);
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) pl[k] = r[k] * ph[k];  // q
#pragma unroll
    for (int k = 0; k < NP; ++k) out[k] = fma2(fma2(-a[k], pl[k], r[k]), ph[k], pl[k]);
}

// acc[j] *= pdf(S[j]; mu): the M == 1 factor (a mean over size-1 axes is the
// pdf itself).  Round 5: the NC sample values are read first (one scalar-load
// burst, one wait) and every column pair runs the fast form straight through
// (no per-pair branch, so the compiler interleaves the pairs and the
// packed-math hazard nops disappear); one wave-uniform test per 8 columns
// decides whether some lane needed a fall-back of pdf2_t in one of their pairs
// -- then those pairs are redone by pdf2_t itself.  Either way every product is
// pdf2_t's, so the bits are those of the per-pair form.
template <int NC, int MODE>
__device__ __forceinline__ void mul_row_t(float (&acc)[NC], const float* __restrict__ S, float sc, float isc,
                                          float nm, float mu) {
    static_assert(NC % 2 == 0, "column pairs");
#if CBN_MULROW_GROUP == 0  // diagnostic A/B: the per-pair form
#pragma unroll
    for (int j = 0; j < NC; j += 2) {
        const f2 r = f2{acc[j], acc[j + 1]} * pdf2_t<MODE>(sc, isc, nm, f2{S[j], S[j + 1]}, mu);
        acc[j] = r.x;
        acc[j + 1] = r.y;
    }
#else
    // columns per wave-uniform test: 8 (Gaussian); 4 for the logistic
    // densities, whose division keeps more values live (register budget)
    constexpr int GM = MODE >= 2 && CBN_MULROW_GROUP > 4 ? 4 : CBN_MULROW_GROUP;
    constexpr int G = NC < GM ? NC : GM;
#pragma unroll
    for (int g = 0; g < NC; g += G) {
        float sv[G];  // this group's sample values: one scalar-load burst, one wait
#pragma unroll
        for (int j = 0; j < G; ++j) sv[j] = S[g + j];
        f2 p[G / 2];
        float lo = __builtin_inff();
        bool bad = false;
        pdf2_fast<G / 2, MODE>(sc, isc, nm, sv, mu, p, lo, bad);
        if (__builtin_expect(__any(lo < -126.f || bad), 0)) {
#pragma unroll
            for (int j = 0; j < G; j += 2) p[j / 2] = pdf2_t<MODE>(sc, isc, nm, f2{sv[j], sv[j + 1]}, mu);
        }
#pragma unroll
        for (int j = 0; j < G; j += 2) {
            const f2 r = f2{acc[g + j], acc[g + j + 1]} * p[j / 2];
            acc[g + j] = r.x;
            acc[g + j + 1] = r.y;
        }
    }
#endif
}

template <int NC, int MODE>
__device__ __forceinline__ void add_row(int mode, float (&fx)[NC], float (&cx)[NC], const float* __restrict__ S,
                                        float sc, float isc, float nm, float mu) {
    if (MODE < 4) {
        add_row_t<NC, MODE < 4 ? MODE : 0>(fx, cx, S, sc, isc, nm, mu);
    } else {
        switch (mode) {
            case 0: add_row_t<NC, 0>(fx, cx, S, sc, isc, nm, mu); break;
            case 1: add_row_t<NC, 1>(fx, cx, S, sc, isc, nm, mu); break;
            case 2: add_row_t<NC, 2>(fx, cx, S, sc, isc, nm, mu); break;
            default: add_row_t<NC, 3>(fx, cx, S, sc, isc, nm, mu); break;
        }
    }
}

template <int NC, int MODE>
__device__ __forceinline__ void mul_row(int mode, float (&acc)[NC], const float* __restrict__ S, float sc, float isc,
                                        float nm, float mu) {
    if (MODE < 4) {
        mul_row_t<NC, MODE < 4 ? MODE : 0>(acc, S, sc, isc, nm, mu);
    } else {
        switch (mode) {
            case 0: mul_row_t<NC, 0>(acc, S, sc, isc, nm, mu); break;
            case 1: mul_row_t<NC, 1>(acc, S, sc, isc, nm, mu); break;
            case 2: mul_row_t<NC, 2>(acc, S, sc, isc, nm, mu); break;
            default: mul_row_t<NC, 3>(acc, S, sc, isc, nm, mu); break;
        }
    }
}

// mu of a linear model with <= kTabIn inputs from its zero-padded weights
// [w0..w3, bias]: the same fma chain as model_mu<0> (a padding term adds
// fma(0, 0, s) == s), every weight an unconditional scalar load
__device__ __forceinline__ float lin4(const float* __restrict__ LW, const float (&z)[kMaxP]) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kTabIn; ++i) s = fmaf(LW[i], z[i], s);  // z[i] = 0 beyond n_in (load_inputs_tab)
    return s + LW[kTabIn];
}

// Column of one model input, resolved once per block into LDS: element
// q of the input is p[q * stride] (stride 0: a constant / unused input reading
// the image's {0, 1} cell).
struct alignas(16) InCol {
    const float* p;
    long long stride;
};

// Evidence inputs of a factor (its kMaxP InCol entries): independent LDS reads
// and vector loads, issued back to back; nothing waits on them until the
// factor is evaluated.  Free inputs are overwritten per combo.
__device__ __forceinline__ void load_inputs(const InCol* __restrict__ cols, long long qs, float (&z)[kMaxP]) {
#pragma unroll
    for (int i = 0; i < kMaxP; ++i) {
        const InCol c = cols[i];
        z[i] = gload(c.p, qs * c.stride);
    }
}

// (table mode: a null column -- an input that is not evidence -- is not
// loaded, a wave-uniform branch; its z is 0 until a free-parent combo sets it)
struct PEv4 {  // (8-B aligned like the kernel-argument pointer table it views)
    const float* p[kTabIn];
};
__device__ __forceinline__ void load_inputs_tab(const PEv& ev, int f, unsigned qb, float (&z)[kMaxP]) {
    const PEv4 c = reinterpret_cast<const PEv4*>(ev.p)[f];  // the factor's column pointers: one scalar load
#pragma unroll
    for (int i = 0; i < kTabIn; ++i) z[i] = c.p[i] ? gload_b(c.p[i], qb) : 0.f;
#pragma unroll
    for (int i = kTabIn; i < kMaxP; ++i) z[i] = 0.f;
}

// Query kernel.  Wave task t -> column chunk l = t / QW and the 64
// consecutive queries (t % QW) * 64 + lane (t, l, the chunk and every image
// read wave-uniform: scalar loads into SGPRs); every lane keeps its NC
// outputs' running product in registers and prefetches the next factor's
// evidence while it evaluates the current one.  MODE: the density family of
// every query factor (0..3, see pdf_t) or 4 = per-factor switch.  Writes the
// UNnormalised rows and one max word per block (the global-max division of
// bayesian_network.py:296 runs after, in k_scale, possibly after a cross-rank
// all-reduce of the words).
// Factor split: a block's 8 waves = (8 / parts) query groups x `parts`
// contiguous factor ranges [f[p], f[p + 1]) (balanced by estimated cost on
// the host).  Wave (group g, part p) multiplies its range's factors for the
// group's 64 queries; parts 1.. leave their products in LDS (comb_off floats
// into the dynamic LDS), part 0 multiplies them in (part order) and writes.
// Batches too small to give every SIMD several waves (131 072 queries of an
// MLP: 2 048 waves for 1 024 SIMDs) run 2-4 parts.
// Threads of a query-kernel block: 8 waves, or 6 when the factor split has
// 3 or 6 parts (a block holds whole query groups of `parts` waves).
inline int query_block_threads(int parts) { return parts % 3 == 0 ? 6 * kWave : kQThreads; }

struct FSplit {
    int parts;
    int comb_off;
    int f[7];
    // Order guard (round 6): each part p >= 1 multiplies its range from 1,
    // the reference from the running product (bayesian_network.py:293).  The
    // two agree to rounding whenever neither ever leaves the normal range;
    // lo[p] = 2^-125 G_p and hi[p] = 2^126 / G_p, G_p = the product over part
    // p's factors of max(1, the density's peak) -- an upper bound on any
    // partial product of the range (cbn_param.hip param_split_guard).
    // A column whose checks fail may have rounded in the subnormal range in
    // either order: each such rounding errs by <= 2^-150 absolute, later
    // multiplied by at most prod_q G_q, so the orders differ there by <= ucap
    // = n_factors 2^-148 prod_q G_q beyond their ordinary relative rounding.
    // mono: every peak <= 1, so every running product only falls and the
    // final product alone decides (>= 2^-125).
    float lo[7];
    float hi[7];
    float ucap;
    float screen;  // 2^-125 G^2 (G = prod_q G_q <= 2^60), else +inf: the exact test runs
    int mono;
};

// Occupancy target per instantiation (waves per SIMD the register
// allocation must allow).  The grid holds up to 8 waves per SIMD
// (1 024 blocks x 8 waves); a linear-model wave's latency chain (scalar
// weight / sample loads, the next factor's evidence) is only hidden with all
// of them resident.
#ifndef CBN_WPE_LIN
#define CBN_WPE_LIN 6  // round 5: 8 -> 6 (80 VGPRs: the column-pair groups of mul_row_t without spills)
#endif
#ifndef CBN_WPE_MLP
// one-hidden-layer M1 kernels of <= 16 columns per lane (configs[3]'s NN
// [16]): 6 waves per SIMD, 80 VGPRs -- the spills this costs sit in the cold
// order-guard tail; same box, two rounds, bit-identical rows: 116.5-117.1 ->
// 114.1-114.2 us at 131 072 queries, 851-852 -> 830-837 us at 1 M (round 6,
// MEASUREMENTS.md).  32-column kernels: 4 waves (<= 128 VGPRs, round 5's
// occupancy; at 80 they would spill 130+ registers, unconstrained the cold
// tail takes them to 152).
#define CBN_WPE_MLP 6
#endif
// M1: every query factor of the plan has all its parents observed (M == 1,
// e.g. full evidence): the free-combo mean and its TwoSum state (2 x NC
// registers) are not compiled, which keeps the wave within the register
// budget of the occupancy above.
template <int NC, int HMAX, int MODE, bool TAB, bool M1>
__global__ void __launch_bounds__(kQThreads)
__attribute__((amdgpu_waves_per_eu(!M1 ? 1 : HMAX == 0 ? CBN_WPE_LIN : HMAX == 1 ? (NC <= 16 ? CBN_WPE_MLP : 4) : 1, 8)))
k_param_query(const float* __restrict__ img, int cst_off, int nf, PEv ev, long long Q, int N, int L, int QW,
              int n_words, unsigned* __restrict__ max_out, float* __restrict__ out, FSplit sp) {
    const PRec* __restrict__ rec = reinterpret_cast<const PRec*>(img);
    constexpr int kNMax = TAB ? kTabIn : kMaxP;  // inputs per factor (column-table plans: <= kTabIn)
    // dynamic LDS: [nf x kMaxP InCol] [deep-model scratch, models with >= 2 hidden layers]
    extern __shared__ __attribute__((aligned(16))) float4 smem_q[];
    InCol* incol = reinterpret_cast<InCol*>(smem_q);
    float* deep = reinterpret_cast<float*>(incol + (TAB ? 0 : nf * kMaxP)) + threadIdx.x;
    if (!TAB) {
        const float* cst = img + cst_off;
        for (int e = threadIdx.x; e < nf * kMaxP; e += blockDim.x) {
            const int sl = rec[e / kMaxP].in_slot[e % kMaxP];
            InCol c;
            c.p = sl >= 0 ? ev.p[sl] : (sl == CBN_INPUT_ONE ? cst + 1 : cst);
            c.stride = sl >= 0 ? 1 : 0;
            incol[e] = c;
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int wpb = blockDim.x / kWave;  // 8 waves; 6 for a 3- or 6-part split (query_block_threads)
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int tasks = QW * L;
    const int parts = sp.parts;
    const int gpb = wpb / parts;  // query groups per block
    const int part = wid % parts, grp = wid / parts;
    const int f0 = sp.f[part], f1 = sp.f[part + 1];
    float* comb = reinterpret_cast<float*>(smem_q) + sp.comb_off;  // [wpb][NC][64]
    float lmax = 0.f;
    // block-uniform trip count (the combine step has block barriers)
    for (int tb = blockIdx.x * gpb; tb < tasks; tb += gridDim.x * gpb) {
        const int t = tb + grp;
        const bool active = t < tasks;
        const int l = (active ? t : tasks - 1) / QW;
        const long long q = (long long)(t - l * QW) * kWave + lane;
        const bool valid = q < Q;
        const long long qs = valid ? q : Q - 1;
        const unsigned qb = (unsigned)qs * 4u;  // table mode: Q <= 2^30 (param_run)
        const int col0 = l * NC;
        const int ncol = min(NC, N - col0);
        float acc[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) acc[j] = 1.f;  // out_pdf = ones (bayesian_network.py:269)
        float z[kMaxP];
        const int fa = active ? f0 : f1;  // an idle wave (batch tail) skips its factors
        if constexpr (!(M1 && TAB)) {  // (the M1 table loop loads its own, two factors ahead)
            if (TAB) load_inputs_tab(ev, fa < nf ? fa : nf - 1, qb, z);
            else load_inputs(incol + (fa < nf ? fa : nf - 1) * kMaxP, qs, z);
        }
        if constexpr (M1 && TAB) {  // hot headers, one factor ahead
            const PHead* __restrict__ hd = reinterpret_cast<const PHead*>(img + cst_off + 4);
            PHead h = hd[fa < nf ? fa : nf - 1];
            // Evidence two factors ahead in two buffers used in turn (round
            // 5): no register copy at the end of a factor, and every input
            // is loaded (an input that is not evidence reads the image's 0
            // cell), so the compiler's waits count the loads -- the
            // next factor's loads stay in flight while this one's are
            // consumed.  (One buffer + a copy waited for vmcnt(0) every
            // factor: the prefetch covered one factor's VALU, not a miss.)
            const float* zcell = img + cst_off;  // {0, 1}: element 0 is 0
            auto load_z = [&](int f, float (&zz)[kMaxP]) {
                const int fi = f < f1 ? f : f1 - 1;  // (past the range: reload the last one, unused)
                const PEv4 c = reinterpret_cast<const PEv4*>(ev.p)[fi > 0 ? fi : 0];
#pragma unroll
                for (int i = 0; i < kTabIn; ++i) zz[i] = gload_b(c.p[i] ? c.p[i] : zcell, c.p[i] ? qb : 0u);
#pragma unroll
                for (int i = kTabIn; i < kMaxP; ++i) zz[i] = 0.f;
            };
            auto eval = [&](int f, const float (&zz)[kMaxP]) {
                const int fn = f + 1 < f1 ? f + 1 : f;
                const PHead hn = hd[fn];
                const float* R = img + h.row + col0;
                if (h.kind != CBN_FACTOR_QUERY) {
#pragma unroll
                    for (int j = 0; j < NC; ++j) acc[j] = acc[j] * R[j];
                } else {
                    float mu;
                    if (HMAX == 0 || h.n_layers == 1) {
                        mu = lin4(img + h.wp, zz);
                    } else {
                        const float* PW = img + h.wp;
                        switch (h.act) {
                            case CBN_ACT_TANH: mu = mlp1p_nin<CBN_ACT_TANH, kTabIn>(PW, h.n_in, h.hid, zz, CBN_ACT_TANH); break;
                            case CBN_ACT_RELU: mu = mlp1p_nin<CBN_ACT_RELU, kTabIn>(PW, h.n_in, h.hid, zz, CBN_ACT_RELU); break;
                            default: mu = mlp1p_rt(PW, h.n_in, h.hid, zz, h.act); break;
                        }
                    }
                    mul_row_t<NC, MODE < 4 ? MODE : 0>(acc, R, h.scale, h.inv_scale, h.norm, mu);
                }
                h = hn;
            };
            float zb[kMaxP];
            load_z(fa, z);
            load_z(fa + 1, zb);
            for (int f = fa; f < f1; f += 2) {
                eval(f, z);
                load_z(f + 2, z);
                if (f + 1 < f1) {
                    eval(f + 1, zb);
                    load_z(f + 3, zb);
                }
            }
        } else
        for (int f = fa; f < f1; ++f) {
            const PRec& r = rec[f];
            float zn[kMaxP];
            const int fn = f + 1 < f1 ? f + 1 : f;  // next factor's evidence in flight during this one
            if (TAB) load_inputs_tab(ev, fn, qb, zn);
            else load_inputs(incol + fn * kMaxP, qs, zn);
            if (r.kind != CBN_FACTOR_QUERY) {  // query-independent row, built with the plan
                const float* c = img + r.c_off + col0;
#pragma unroll
                for (int j = 0; j < NC; ++j) acc[j] = acc[j] * c[j];
            } else {
                const float* W = img + r.w_off;
                const float* S = img + r.s_off + col0;
                const int mode = mode_of(r.family, r.unit != 0);
                const float sc = r.scale, isc = r.inv_scale, nm = r.norm;
                if (M1 || r.M == 1) {  // every parent observed: x = pdf (a mean over size-1 axes)
                    mul_row<NC, MODE>(mode, acc, S, sc, isc, nm, query_mu<HMAX, kNMax>(r, img, W, z, deep));
                } else if constexpr (!M1) {
                    float fx[NC], cx[NC];
#pragma unroll
                    for (int j = 0; j < NC; ++j) fx[j] = cx[j] = 0.f;
                    const float* FS = img + r.fs_off;
                    const int fm = r.free_mask;
                    for (int c = 0; c < r.M; ++c) {
                        int cc = c;  // meshgrid 'ij' order: last free input fastest (node.py:335-375)
#pragma unroll
                        for (int i = kMaxP - 1; i >= 0; --i) {
                            if (fm & (1 << i)) {
                                const int qd = cc / N;
                                z[i] = FS[i * N + (cc - qd * N)];
                                cc = qd;
                            }
                        }
                        add_row<NC, MODE>(mode, fx, cx, S, sc, isc, nm, query_mu<HMAX, kNMax>(r, img, W, z, deep));
                    }
                    const float Mf = (float)r.M;
#pragma unroll
                    for (int j = 0; j < NC; ++j) acc[j] = acc[j] * ((fx[j] + cx[j]) / Mf);  // torch.mean = sum / count
                }
            }
#pragma unroll
            for (int i = 0; i < kMaxP; ++i) z[i] = zn[i];
        }
        if (parts > 1) {
            float* mine = comb + (wid * NC) * kWave + lane;
            if (active) {  // parts 1..: their products; part 0: its own (kept for the order guard)
#pragma unroll
                for (int j = 0; j < NC; ++j) mine[j * kWave] = acc[j];
            }
            __syncthreads();
            if (part == 0 && active) {
                for (int p = 1; p < parts; ++p) {
#pragma unroll
                    for (int j = 0; j < NC; ++j) acc[j] = acc[j] * mine[(p * NC + j) * kWave];
                }
                // Order guard (FSplit, round 6).  Screen: every column's
                // product >= sp.screen = 2^-125 G^2 (G = prod_q G_q <= 2^60)
                // implies every partial product of either order stayed
                // normal and finite, so the split equals the reference's
                // running product to rounding.  A wave with a lane below it
                // (NaN included) takes the exact test below.
                bool scr = false;
#pragma unroll
                for (int j = 0; j < NC; ++j) scr |= j < ncol && !(acc[j] >= sp.screen);
                if (__builtin_expect(__any(scr), 0)) {
                    // per lane: `must` = the reference's running product may
                    // overflow where the split's does not; `haz` = some
                    // column's product may have rounded in the subnormal
                    // range in one order, where the orders differ by <= ucap
                    // beyond rounding (FSplit).  A lane whose ucap is below
                    // 2^-30 of its own largest product differs by less than
                    // 2^-30 of the global max after the division (that max is
                    // at least this row's) and keeps the split's product; any
                    // other failing lane takes the reference's order.  The
                    // decision is the row's own: its bits never depend on its
                    // wave-mates (sharding).
                    bool must = false, haz = false;
                    float tmax = 0.f;
#pragma unroll
                    for (int j = 0; j < NC; ++j) {
                        if (j < ncol) {
                            float pr = mine[j * kWave];  // part 0's product: the reference's prefix
                            if (!sp.mono) {
                                for (int p = 1; p < parts; ++p) {
                                    const float P = mine[(p * NC + j) * kWave];
                                    must |= !(pr <= sp.hi[p]);
                                    const float pn = pr * P;
                                    haz |= !(P >= sp.lo[p]) || !(pn >= sp.lo[p]);
                                    pr = pn;
                                }
                            }
                            haz |= !(acc[j] >= 0x1p-125f);
                            tmax = fmaxf(tmax, acc[j]);
                        }
                    }
                    const bool seq = must || (haz && sp.ucap > tmax * 0x1p-30f);
                    if (__any(seq)) {
                        // the reference's order for the `seq` lanes: continue
                        // the running product from part 0's through factors
                        // f[1] .. f[parts] (the other lanes park their split
                        // products in their own slot and take them back)
#pragma unroll
                        for (int j = 0; j < NC; ++j) {
                            const float p0 = mine[j * kWave];
                            if (!seq) mine[j * kWave] = acc[j];
                            acc[j] = seq ? p0 : acc[j];
                        }
                        const int ft = sp.f[1], fend = sp.f[parts];
                        for (int f = ft; f < fend; ++f) {
                            float zt[kMaxP];
                            if (TAB) load_inputs_tab(ev, f, qb, zt);
                            else load_inputs(incol + f * kMaxP, qs, zt);
                            if constexpr (M1 && TAB) {
                                const PHead h = reinterpret_cast<const PHead*>(img + cst_off + 4)[f];
                                const float* R = img + h.row + col0;
                                if (h.kind != CBN_FACTOR_QUERY) {
#pragma unroll
                                    for (int j = 0; j < NC; ++j) acc[j] = acc[j] * R[j];
                                } else {
                                    float mu;
                                    if (HMAX == 0 || h.n_layers == 1) {
                                        mu = lin4(img + h.wp, zt);
                                    } else {
                                        const float* PW = img + h.wp;
                                        switch (h.act) {
                                            case CBN_ACT_TANH: mu = mlp1p_nin<CBN_ACT_TANH, kTabIn>(PW, h.n_in, h.hid, zt, CBN_ACT_TANH); break;
                                            case CBN_ACT_RELU: mu = mlp1p_nin<CBN_ACT_RELU, kTabIn>(PW, h.n_in, h.hid, zt, CBN_ACT_RELU); break;
                                            default: mu = mlp1p_rt(PW, h.n_in, h.hid, zt, h.act); break;
                                        }
                                    }
                                    mul_row_t<NC, MODE < 4 ? MODE : 0>(acc, R, h.scale, h.inv_scale, h.norm, mu);
                                }
                            } else {
                                const PRec& r = rec[f];
                                if (r.kind != CBN_FACTOR_QUERY) {
                                    const float* c = img + r.c_off + col0;
#pragma unroll
                                    for (int j = 0; j < NC; ++j) acc[j] = acc[j] * c[j];
                                } else {
                                    const float* W = img + r.w_off;
                                    const float* S = img + r.s_off + col0;
                                    const int mode = mode_of(r.family, r.unit != 0);
                                    const float sc = r.scale, isc = r.inv_scale, nm = r.norm;
                                    if (M1 || r.M == 1) {
                                        mul_row<NC, MODE>(mode, acc, S, sc, isc, nm, query_mu<HMAX, kNMax>(r, img, W, zt, deep));
                                    } else if constexpr (!M1) {
                                        float fx[NC], cx[NC];
#pragma unroll
                                        for (int j = 0; j < NC; ++j) fx[j] = cx[j] = 0.f;
                                        const float* FS = img + r.fs_off;
                                        const int fm = r.free_mask;
                                        for (int c = 0; c < r.M; ++c) {
                                            int cc = c;
#pragma unroll
                                            for (int i = kMaxP - 1; i >= 0; --i) {
                                                if (fm & (1 << i)) {
                                                    const int qd = cc / N;
                                                    zt[i] = FS[i * N + (cc - qd * N)];
                                                    cc = qd;
                                                }
                                            }
                                            add_row<NC, MODE>(mode, fx, cx, S, sc, isc, nm, query_mu<HMAX, kNMax>(r, img, W, zt, deep));
                                        }
                                        const float Mf = (float)r.M;
#pragma unroll
                                        for (int j = 0; j < NC; ++j) acc[j] = acc[j] * ((fx[j] + cx[j]) / Mf);
                                    }
                                }
                            }
                        }
                        if (!seq) {
#pragma unroll
                            for (int j = 0; j < NC; ++j) acc[j] = mine[j * kWave];
                        }
                    }
                }
            }
            __syncthreads();
        }
        if (part == 0 && active && valid) {
            float* o = out + q * N + col0;
            if ((N & 3) == 0 && (NC & 3) == 0 && ncol == NC) {
#pragma unroll
                for (int v = 0; v < NC / 4; ++v)
                    reinterpret_cast<float4*>(o)[v] = make_float4(acc[4 * v], acc[4 * v + 1], acc[4 * v + 2], acc[4 * v + 3]);
            } else {
#pragma unroll
                for (int j = 0; j < NC; ++j)
                    if (j < ncol) o[j] = acc[j];
            }
            // torch.max propagates NaN (an overflowed logistic density): so does this
            // max, and as an unsigned word NaN outranks every non-negative float
#pragma unroll
            for (int j = 0; j < NC; ++j)
                if (j < ncol) lmax = (acc[j] > lmax || acc[j] != acc[j]) ? acc[j] : lmax;
        }
    }
    // block max -> one word per block (non-negative floats: uint order == float order)
    __shared__ unsigned wm[kQThreads / kWave];
    const unsigned wmx = wave_max_u(__float_as_uint(lmax));
    if (lane == 0) wm[threadIdx.x / kWave] = wmx;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned m = 0;
        for (int i = 0; i < wpb; ++i) m = max(m, wm[i]);
        max_out[blockIdx.x] = m;
    }
    if (blockIdx.x == 0)  // words of blocks this launch does not have
        for (int i = (int)gridDim.x + threadIdx.x; i < n_words; i += blockDim.x) max_out[i] = 0u;
}

// Query-independent factors, once per plan: SHARED x[j] = mean_c pdf(s_j;
// mu(c)); SCALAR x = mean_j pdf(s_j; mu(1)) replicated over the row.  One
// block per factor, thread per column.
template <int HMAX>
__global__ void __launch_bounds__(kThreads)
k_param_const(float* __restrict__ img, const int* __restrict__ which, int N) {
    extern __shared__ float deep_smem[];
    float* deep = deep_smem + threadIdx.x;
    const PRec& r = reinterpret_cast<const PRec*>(img)[which[blockIdx.x]];
    const float* W = img + r.w_off;
    const float* S = img + r.s_off;
    const float* FS = img + r.fs_off;
    float* C = img + r.c_off;
    const int n_in = r.m.width[0];
    const bool unit = r.unit != 0;
    for (int j0 = 0; j0 < N; j0 += blockDim.x) {  // uniform trip count (model uses LDS scratch)
        const int j = j0 + threadIdx.x;
        const int js = j < N ? j : N - 1;
        float s = 0.f, sc = 0.f;
        float z[kMaxP];
#pragma unroll
        for (int i = 0; i < kMaxP; ++i) z[i] = (i < n_in && r.in_slot[i] == CBN_INPUT_ONE) ? 1.f : 0.f;
        for (int c = 0; c < r.M; ++c) {
            int cc = c;
#pragma unroll
            for (int i = kMaxP - 1; i >= 0; --i) {
                if (i < n_in && r.in_slot[i] == CBN_INPUT_FREE) {
                    const int qd = cc / N;
                    z[i] = FS[i * N + (cc - qd * N)];
                    cc = qd;
                }
            }
            two_sum(s, sc, pdf_eval(mode_of(r.family, unit), r.scale, r.inv_scale, r.norm, S[js],
                                    model_mu<HMAX>(r.m, W, z, deep)));
        }
        s = s + sc;
        if (j < N) C[j] = r.kind == CBN_FACTOR_SCALAR ? s : s / (float)r.M;
    }
    if (r.kind == CBN_FACTOR_SCALAR) {  // mean over the N sample points (dim 1 of [1, N])
        __syncthreads();
        __shared__ float xs;
        if (threadIdx.x == 0) {
            float t = 0.f;
            for (int j = 0; j < N; ++j) t += C[j];
            xs = t / (float)N;
        }
        __syncthreads();
        for (int j = threadIdx.x; j < N; j += blockDim.x) C[j] = xs;
    }
}

// Estimator get_prob: thread per row, mu once, then the row's points.
template <int HMAX>
__global__ void __launch_bounds__(kThreads)
k_param_eval(MDesc m, int family, int unit, float scale, float norm, const float* __restrict__ W,
             const float* __restrict__ pts, long long n_rows, int n_pts, const float* __restrict__ query, int bias_only,
             float* __restrict__ out) {
    extern __shared__ float deep_smem[];
    float* deep = deep_smem + threadIdx.x;
    for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < n_rows;
         r += (long long)gridDim.x * blockDim.x) {
        const int n_in = m.width[0];
        float mu;
        if (bias_only) {
            mu = 0.f + W[m.width[0] * m.width[1]];  // zeros + bias (linear_regression.py:112-117)
        } else {
            float z[kMaxP];
#pragma unroll
            for (int i = 0; i < kMaxP; ++i) z[i] = i < n_in ? (query ? query[r * n_in + i] : 1.f) : 0.f;
            mu = model_mu<HMAX>(m, W, z, deep);
        }
        const int mode = mode_of(family, unit != 0);
        const float inv_scale = 1.f / scale;
        for (int v = 0; v < n_pts; ++v)
            out[r * n_pts + v] = pdf_eval(mode, scale, inv_scale, norm, pts[r * n_pts + v], mu);
    }
}

// ------------------------------------------------------------------------
// Generic kernels: models of any shape within CBN_MAX_MODEL_* (more than
// kMaxP inputs, hidden layers wider than CBN_MAX_WIDTH or more than kMaxL
// layers).  Thread per (query, 16-column chunk); the layer activations of a
// thread live in two LDS buffers of `wbuf` floats (element k of a thread at
// k * T + tid: consecutive lanes, consecutive banks), the weights stream
// through wave-uniform scalar loads.  Same operations in the same order as
// model_mu: per layer and unit the dot product over the inputs, then the
// bias, then the activation (all but the last layer).
struct alignas(16) GRec {
    int kind, family, unit, M;
    int n_layers, n_in, act, w_off;
    int s_off, fs_off, c_off, widths_off;
    int slots_off;
    float scale, inv_scale, norm;
};
static_assert(sizeof(GRec) == 64, "GRec layout");
constexpr int kGenNC = 16;

__device__ float mlp_gen(const float* __restrict__ W, const int* __restrict__ widths, int n_layers, int act, float* A,
                         float* B, int T) {
    int win = widths[0];
    float* src = A;
    float* dst = B;
    for (int l = 0; l < n_layers; ++l) {
        const int wout = widths[l + 1];
        const float* Bl = W + (long long)wout * win;
        if (l == n_layers - 1) {  // output layer: one unit
            float s = 0.f;
            for (int i = 0; i < win; ++i) s = fmaf(W[i], src[i * T], s);
            return s + Bl[0];
        }
        for (int o = 0; o < wout; ++o) {
            const float* Wo = W + (long long)o * win;
            float s = 0.f;
            for (int i = 0; i < win; ++i) s = fmaf(Wo[i], src[i * T], s);
            dst[o * T] = act1(act, s + Bl[o]);
        }
        W = Bl + wout;
        float* t = src;
        src = dst;
        dst = t;
        win = wout;
    }
    return 0.f;
}

// model inputs of combo c into A: evidence of query q, free-parent sample
// points (meshgrid 'ij' order: the last free input fastest), constant 1
__device__ __forceinline__ void gen_inputs(const float* __restrict__ img, const GRec& r, const PEv* ev, long long q,
                                           int c, int N, float* A, int T) {
    const int* slots = reinterpret_cast<const int*>(img + r.slots_off);
    const float* FS = img + r.fs_off;
    int cc = c;
    for (int i = r.n_in - 1; i >= 0; --i) {
        const int sl = slots[i];
        float v = 1.f;  // CBN_INPUT_ONE
        if (sl >= 0) {
            v = gload(ev->p[sl], q);
        } else if (sl == CBN_INPUT_FREE) {
            const int qd = cc / N;
            v = FS[i * N + (cc - qd * N)];
            cc = qd;
        }
        A[i * T] = v;
    }
}

__global__ void __launch_bounds__(256) k_param_query_gen(const float* __restrict__ img, int nf, PEv ev, long long Q,
                                                         int N, int L, int wbuf, int n_words,
                                                         unsigned* __restrict__ max_out, float* __restrict__ out) {
    extern __shared__ float smem_g[];
    const int T = blockDim.x;
    float* A = smem_g + threadIdx.x;
    float* B = A + wbuf * T;
    const GRec* rec = reinterpret_cast<const GRec*>(img);
    unsigned lmaxb = 0;
    const long long tasks = Q * L;
    for (long long t = blockIdx.x * (long long)T + threadIdx.x; t < tasks; t += (long long)gridDim.x * T) {
        const int l = (int)(t / Q);
        const long long q = t - (long long)l * Q;
        const int col0 = l * kGenNC;
        const int ncol = min(kGenNC, N - col0);
        float acc[kGenNC];
#pragma unroll
        for (int j = 0; j < kGenNC; ++j) acc[j] = 1.f;  // out_pdf = ones (bayesian_network.py:269)
        for (int f = 0; f < nf; ++f) {
            const GRec& r = rec[f];
            if (r.kind != CBN_FACTOR_QUERY) {
                const float* c = img + r.c_off + col0;
#pragma unroll
                for (int j = 0; j < kGenNC; ++j) acc[j] = acc[j] * c[j];
                continue;
            }
            const float* S = img + r.s_off + col0;
            const float* W = img + r.w_off;
            const int* widths = reinterpret_cast<const int*>(img + r.widths_off);
            const int mode = mode_of(r.family, r.unit != 0);
            if (r.M == 1) {
                gen_inputs(img, r, &ev, q, 0, N, A, T);
                const float mu = mlp_gen(W, widths, r.n_layers, r.act, A, B, T);
#pragma unroll
                for (int j = 0; j < kGenNC; ++j) acc[j] = acc[j] * pdf_eval(mode, r.scale, r.inv_scale, r.norm, S[j], mu);
                continue;
            }
            float fx[kGenNC], cx[kGenNC];
#pragma unroll
            for (int j = 0; j < kGenNC; ++j) fx[j] = cx[j] = 0.f;
            for (int c = 0; c < r.M; ++c) {
                gen_inputs(img, r, &ev, q, c, N, A, T);
                const float mu = mlp_gen(W, widths, r.n_layers, r.act, A, B, T);
#pragma unroll
                for (int j = 0; j < kGenNC; ++j) two_sum(fx[j], cx[j], pdf_eval(mode, r.scale, r.inv_scale, r.norm, S[j], mu));
            }
            const float Mf = (float)r.M;
#pragma unroll
            for (int j = 0; j < kGenNC; ++j) acc[j] = acc[j] * ((fx[j] + cx[j]) / Mf);  // torch.mean = sum / count
        }
        float* o = out + q * N + col0;
#pragma unroll
        for (int j = 0; j < kGenNC; ++j)
            if (j < ncol) {
                o[j] = acc[j];
                lmaxb = max(lmaxb, __float_as_uint(acc[j]));  // NaN bits outrank every non-negative float
            }
    }
    __shared__ unsigned wm[256 / kWave];
    const unsigned wmx = wave_max_u(lmaxb);
    if ((threadIdx.x & (kWave - 1)) == 0) wm[threadIdx.x / kWave] = wmx;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned m = 0;
        for (int i = 0; i < T / kWave; ++i) m = max(m, wm[i]);
        max_out[blockIdx.x] = m;
    }
    if (blockIdx.x == 0)
        for (int i = (int)gridDim.x + threadIdx.x; i < n_words; i += T) max_out[i] = 0u;
}

// query-independent factors of a generic plan (k_param_const's semantics)
__global__ void __launch_bounds__(256) k_param_const_gen(float* __restrict__ img, const int* __restrict__ which, int N,
                                                         int wbuf) {
    extern __shared__ float smem_g[];
    const int T = blockDim.x;
    float* A = smem_g + threadIdx.x;
    float* B = A + wbuf * T;
    const GRec& r = reinterpret_cast<const GRec*>(img)[which[blockIdx.x]];
    const float* S = img + r.s_off;
    float* C = img + r.c_off;
    const int* widths = reinterpret_cast<const int*>(img + r.widths_off);
    const int mode = mode_of(r.family, r.unit != 0);
    for (int j0 = 0; j0 < N; j0 += T) {
        const int j = j0 + threadIdx.x;
        const int js = j < N ? j : N - 1;
        float s = 0.f, sc = 0.f;
        for (int c = 0; c < r.M; ++c) {
            gen_inputs(img, r, nullptr, 0, c, N, A, T);
            two_sum(s, sc, pdf_eval(mode, r.scale, r.inv_scale, r.norm, S[js],
                                    mlp_gen(img + r.w_off, widths, r.n_layers, r.act, A, B, T)));
        }
        s = s + sc;
        if (j < N) C[j] = r.kind == CBN_FACTOR_SCALAR ? s : s / (float)r.M;
    }
    if (r.kind == CBN_FACTOR_SCALAR) {  // mean over the N sample points (dim 1 of [1, N])
        __syncthreads();
        __shared__ float xs;
        if (threadIdx.x == 0) {
            float t = 0.f;
            for (int j = 0; j < N; ++j) t += C[j];
            xs = t / (float)N;
        }
        __syncthreads();
        for (int j = threadIdx.x; j < N; j += blockDim.x) C[j] = xs;
    }
}

struct GWidths {
    int w[CBN_MAX_MODEL_LAYERS + 1];
};

// Estimator get_prob for a generic model: thread per row
__global__ void __launch_bounds__(256) k_param_eval_gen(GWidths gw, int n_layers, int act, int family, int unit,
                                                        float scale, float norm, const float* __restrict__ W,
                                                        const float* __restrict__ pts, long long n_rows, int n_pts,
                                                        const float* __restrict__ query, int wbuf,
                                                        float* __restrict__ out) {
    extern __shared__ float smem_g[];
    __shared__ int widths[CBN_MAX_MODEL_LAYERS + 1];
    for (int l = threadIdx.x; l <= n_layers; l += blockDim.x) widths[l] = gw.w[l];
    __syncthreads();
    const int T = blockDim.x;
    float* A = smem_g + threadIdx.x;
    float* B = A + wbuf * T;
    const int n_in = widths[0];
    const int mode = mode_of(family, unit != 0);
    const float inv_scale = 1.f / scale;
    for (long long r = blockIdx.x * (long long)T + threadIdx.x; r < n_rows; r += (long long)gridDim.x * T) {
        for (int i = 0; i < n_in; ++i) A[i * T] = query ? query[r * n_in + i] : 1.f;
        const float mu = mlp_gen(W, widths, n_layers, act, A, B, T);
        for (int v = 0; v < n_pts; ++v)
            out[r * n_pts + v] = pdf_eval(mode, scale, inv_scale, norm, pts[r * n_pts + v], mu);
    }
}

// threads per block of the generic kernels: the two per-thread LDS buffers
// of wbuf floats must fit the dynamic LDS
int gen_threads(int wbuf) {
    for (int T = 256; T >= 64; T >>= 1)
        if ((size_t)2 * wbuf * T * sizeof(float) <= (size_t)(kLdsBudget - 512)) return T;
    return 0;
}

// model kernel class: 0 linear, 1 one hidden layer (streamed), 32 deeper
// (first hidden layer in registers, further ones in LDS)
int hmax_for(const MDesc& m) {
    if (m.n_layers == 1) return 0;
    if (m.n_layers == 2) return 1;
    int w = 0;
    for (int l = 1; l < m.n_layers; ++l) w = std::max(w, m.width[l]);
    return 32;
}

// Model shape of a cbn_param_model (widths[] when given, else width[]),
// validated against the generic kernel's limits.  `fast`: the shape the
// register-resident kernels take (<= kMaxP inputs and either one hidden layer
// of any width -- streamed -- or <= kMaxL layers of <= CBN_MAX_WIDTH units).
struct HostModel {
    int n_layers = 0;
    int act = 0;
    std::vector<int> w;
    bool fast = false;
    long long n_weights = 0;
    int wmax = 0;  // widest input / hidden layer
};

int resolve_model(const cbn_param_model& h, HostModel& m, const char* what, int idx) {
    if (h.family != CBN_FAMILY_GAUSS && h.family != CBN_FAMILY_LOGISTIC)
        return set_err(CBN_E_ARG, "%s %d: bad family %d", what, idx, h.family);
    if (h.n_layers < 1 || h.n_layers > CBN_MAX_MODEL_LAYERS)
        return set_err(CBN_E_LIMIT, "%s %d: %d layers (1..%d)", what, idx, h.n_layers, CBN_MAX_MODEL_LAYERS);
    if (h.n_layers > kMaxL && !h.widths)
        return set_err(CBN_E_ARG, "%s %d: %d layers need the widths array", what, idx, h.n_layers);
    m.n_layers = h.n_layers;
    m.act = h.act;
    m.w.assign(h.n_layers + 1, 0);
    for (int l = 0; l <= h.n_layers; ++l) m.w[l] = h.widths ? h.widths[l] : h.width[l];
    if (m.w[0] < 1 || m.w[0] > CBN_MAX_MODEL_WIDTH)
        return set_err(CBN_E_LIMIT, "%s %d: %d model inputs (1..%d)", what, idx, m.w[0], CBN_MAX_MODEL_WIDTH);
    if (m.w[h.n_layers] != 1) return set_err(CBN_E_ARG, "%s %d: the last layer must have 1 output", what, idx);
    int hid = 0;
    for (int l = 1; l < h.n_layers; ++l) {
        if (m.w[l] < 1 || m.w[l] > CBN_MAX_MODEL_WIDTH)
            return set_err(CBN_E_LIMIT, "%s %d: hidden width %d (1..%d)", what, idx, m.w[l], CBN_MAX_MODEL_WIDTH);
        hid = std::max(hid, m.w[l]);
    }
    if (h.n_layers > 1 && (h.act < CBN_ACT_TANH || h.act > CBN_ACT_ELU))
        return set_err(CBN_E_ARG, "%s %d: bad activation %d", what, idx, h.act);
    if (!h.weights) return set_err(CBN_E_ARG, "%s %d: null weights", what, idx);
    if (!(h.scale > 0.f)) return set_err(CBN_E_ARG, "%s %d: scale must be > 0", what, idx);
    m.n_weights = 0;
    for (int l = 0; l < h.n_layers; ++l) m.n_weights += (long long)m.w[l + 1] * (m.w[l] + 1);
    m.wmax = std::max(m.w[0], hid);
    m.fast = h.n_layers <= kMaxL && m.w[0] <= kMaxP && (h.n_layers <= 2 || hid <= CBN_MAX_WIDTH);
    return CBN_OK;
}

// the register-resident kernels' descriptor of a fast model
int check_model(const cbn_param_model& h, MDesc& m, long long& n_weights, const char* what, int idx) {
    HostModel hm;
    const int rc = resolve_model(h, hm, what, idx);
    if (rc) return rc;
    if (!hm.fast) return set_err(CBN_E_LIMIT, "%s %d: model shape needs the generic kernel", what, idx);
    memset(&m, 0, sizeof(m));
    m.n_layers = hm.n_layers;
    m.act = hm.act;
    for (int l = 0; l <= hm.n_layers; ++l) m.width[l] = hm.w[l];
    n_weights = hm.n_weights;
    return CBN_OK;
}

// [W1 (H x n_in), B1 (H), W2 (H), b2] (nn.Linear order, parametric.py
// packed()) -> the pair records of mlp1p
void pack_pairs(const std::vector<float>& w, int n_in, int H, std::vector<float>& pw) {
    const int npairs = (H + 1) / 2;
    const float* W1 = w.data();
    const float* B1 = W1 + (size_t)H * n_in;
    const float* W2 = B1 + H;
    pw.assign((size_t)npairs * (2 * n_in + 4) + 1, 0.f);
    float* o = pw.data();
    for (int P = 0; P < npairs; ++P) {
        for (int u = 0; u < 2; ++u) {
            const int k = 2 * P + u;
            if (k >= H) continue;
            for (int i = 0; i < n_in; ++i) o[2 * i + u] = W1[(size_t)k * n_in + i];
            o[2 * n_in + u] = B1[k];
            o[2 * n_in + 2 + u] = W2[k];
        }
        o += 2 * n_in + 4;
    }
    *o = W2[H];
}

// LDS scratch of the deep-model path (>= 2 hidden layers): 2 x HMAX floats per thread
size_t deep_bytes(const MDesc& m, int hmax, int threads = kThreads) {
    return m.n_layers > 2 ? (size_t)2 * hmax * threads * sizeof(float) : 0;
}

// dynamic LDS beyond the 64 KiB default (the kernels' static LDS is < 256 B);
// a refusal must not linger as the thread's sticky last error
constexpr int kDynLdsMax = kLdsBudget - 256;
template <typename K>
void allow_deep(K* k) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, kDynLdsMax) !=
        hipSuccess)
        (void)hipGetLastError();
}

template <int HMAX>
void launch_const_t(float* img, const int* which, int n, int N, size_t lds, hipStream_t s) {
    allow_deep(&k_param_const<HMAX>);
    hipLaunchKernelGGL(k_param_const<HMAX>, dim3(n), dim3(kThreads), lds, s, img, which, N);
}


}  // namespace

namespace cbn {
struct ParamPlan {
    int nf = 0;
    int N = 0;
    int ns = 0;
    int nc = 16;     // output columns per lane
    int L = 1;       // column chunks per query
    int hmax = 0;    // 0 / 16 / 32
    int mode = 4;    // density family of every query factor (0..3) or 4: mixed
    int cst_off = 0; // image offset of the {0, 1} cell read by constant inputs
    bool tab_ok = false;  // <= kTabIn inputs per factor and nf * kTabIn <= kTabCols: kernarg column table
    bool all_m1 = false;  // every query factor has all its parents observed (M == 1): the M1 kernels
    int parts = 1;        // factor ranges per query group (a plan constant: the product order)
    bool lin16 = false;   // linear M1 plan with N >= 16: 16-column chunks (mu once per 16 columns)
    std::vector<int> in_slot;  // [nf][kTabIn] host copy (table mode)
    size_t deep = 0; // dynamic LDS of the deep-model path (query kernel)
    size_t deep_const = 0;  // ... and of the const kernel
    int max_slots = 0;
    int split[7][8] = {};  // factor ranges for 1, 2, 3, 4 and 6 parts (index: parts)
    float guard_lo[7][8] = {}, guard_hi[7][8] = {}, guard_ucap[7] = {}, guard_screen[7] = {};  // order guard (FSplit)
    bool guard_ok[7] = {};  // every part's bound G_p <= 2^100 (else the plan runs 1 part)
    bool mono = false;      // every density's peak <= 1
    float* d_image = nullptr;
    int* d_which = nullptr;
    int image_floats = 0;
    bool generic = false;  // GRec image, k_param_query_gen (models beyond the fast kernels)
    int wbuf = 0;          // generic: floats per LDS activation buffer
    int gT = 0;            // generic: threads per block
};
}  // namespace cbn

namespace {
template <int NC, int HMAX, int MODE, bool M1 = false, bool TAB = (MODE < 4)>
void launch_query_t(const cbn::ParamPlan* pp, unsigned grid, const PEv& ev, long long Q, int QW, int L,
                    unsigned* words, float* out, hipStream_t s, int parts) {
    allow_deep(&k_param_query<NC, HMAX, MODE, TAB, M1>);
    FSplit sp;
    memset(&sp, 0, sizeof(sp));
    sp.parts = parts;
    for (int p = 0; p <= parts; ++p) sp.f[p] = pp->split[parts][p];
    const bool guard = !diag_env("CBN_PARAM_NO_GUARD");  // (A/B: the split's products kept everywhere)
    for (int p = 0; p < parts; ++p) {
        sp.lo[p] = guard ? pp->guard_lo[parts][p] : 0.f;
        sp.hi[p] = guard ? pp->guard_hi[parts][p] : HUGE_VALF;
    }
    sp.ucap = pp->guard_ucap[parts];
    sp.screen = guard ? pp->guard_screen[parts] : 0.f;
    sp.mono = pp->mono && guard ? 1 : 0;
    size_t lds = (TAB ? 0 : (size_t)pp->nf * kMaxP * sizeof(InCol)) + pp->deep;
    lds = (lds + 15) & ~(size_t)15;
    sp.comb_off = (int)(lds / sizeof(float));
    if (parts > 1) lds += (size_t)(kQThreads / kWave) * NC * kWave * sizeof(float);
    hipLaunchKernelGGL((k_param_query<NC, HMAX, MODE, TAB, M1>), dim3(grid), dim3(query_block_threads(parts)), lds, s,
                       pp->d_image,
                       pp->cst_off, pp->nf, ev, Q, pp->N, L, QW, pp->max_slots, words, out, sp);
}

// Instantiated (HMAX, MODE) pairs: linear models (HMAX 0) of either family,
// MLPs with the logistic density (NeuralNetwork); anything else runs the
// per-factor switch at NC = 16, HMAX = 32 (plan_create picks nc/L for it).
bool specialised(int hmax, int mode) { return mode < 4 && (hmax == 0 || mode >= 2); }

// MLP (NeuralNetwork, logistic density) kernels for one column chunk
// (one-hidden-layer plans with every parent observed: the M1 forms)
template <int NC>
void launch_query_mlp(const cbn::ParamPlan* pp, unsigned grid, const PEv& ev, long long Q, int QW, int L,
                      unsigned* words, float* out, hipStream_t s, int parts) {
#define CBN_Q(H, M, M1) launch_query_t<NC, H, M, M1>(pp, grid, ev, Q, QW, L, words, out, s, parts)
    switch (pp->hmax * 8 + pp->mode) {
        case 1 * 8 + 2: if (pp->all_m1) CBN_Q(1, 2, true); else CBN_Q(1, 2, false); break;
        case 1 * 8 + 3: if (pp->all_m1) CBN_Q(1, 3, true); else CBN_Q(1, 3, false); break;
        case 32 * 8 + 2: CBN_Q(32, 2, false); break;
        default: CBN_Q(32, 3, false); break;
    }
#undef CBN_Q
}

// linear models (LinearRegression / LogisticRegression): NCL-column chunks
template <int NCL, bool M1>
void launch_query_lin(const cbn::ParamPlan* pp, unsigned grid, const PEv& ev, long long Q, int QW, int L,
                      unsigned* words, float* out, hipStream_t s, int parts) {
    switch (pp->mode) {
        case 0: launch_query_t<NCL, 0, 0, M1>(pp, grid, ev, Q, QW, L, words, out, s, parts); break;
        case 1: launch_query_t<NCL, 0, 1, M1>(pp, grid, ev, Q, QW, L, words, out, s, parts); break;
        case 2: launch_query_t<NCL, 0, 2, M1>(pp, grid, ev, Q, QW, L, words, out, s, parts); break;
        default: launch_query_t<NCL, 0, 3, M1>(pp, grid, ev, Q, QW, L, words, out, s, parts); break;
    }
}
}  // namespace

void cbn::param_destroy(ParamPlan* pp) {
    if (!pp) return;
    if (pp->d_image) (void)hipFree(pp->d_image);
    if (pp->d_which) (void)hipFree(pp->d_which);
    delete pp;
}

int cbn::param_max_words(const ParamPlan* pp) { return pp ? pp->max_slots : 0; }

int cbn::param_run(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
                   uint32_t* max_bits, float* out, int32_t flags, hipStream_t s) {
    const ParamPlan* pp = plan->param;
    if (n_evidence != pp->ns) return set_err(CBN_E_ARG, "plan expects %d evidence columns, got %d", pp->ns, n_evidence);
    if (n_queries <= 0) return set_err(CBN_E_ARG, "cbn_plan_run: parametric plans need >= 1 query");
    if (!out || !max_bits) return set_err(CBN_E_ARG, "cbn_plan_run: null output");
    if (!pp->d_image || !plan->d_sync) return set_err(CBN_E_ARG, "plan has no device buffers");
    PEv ev;
    memset(&ev, 0, sizeof(ev));
    for (int i = 0; i < n_evidence; ++i)
        if (!evidence[i]) return set_err(CBN_E_ARG, "null evidence column %d", i);
    if (specialised(pp->hmax, pp->mode)) {  // table mode: one pointer per (factor, input)
        for (size_t e = 0; e < pp->in_slot.size(); ++e) {
            const int sl = pp->in_slot[e];
            ev.p[e] = sl >= 0 ? evidence[sl] : nullptr;  // not evidence: not loaded (z = 0 / a free combo's sample)
        }
    } else {
        for (int i = 0; i < n_evidence; ++i) ev.p[i] = evidence[i];
    }
    if (pp->generic) {
        for (int i = 0; i < n_evidence; ++i) ev.p[i] = evidence[i];
        const int L = (pp->N + kGenNC - 1) / kGenNC;
        const long long tasks = n_queries * L;
        long long grid = std::max(1LL, std::min((tasks + pp->gT - 1) / pp->gT, (long long)pp->max_slots));
        const size_t lds = (size_t)2 * pp->wbuf * pp->gT * sizeof(float);
        allow_deep(&k_param_query_gen);
        const bool raw = (flags & CBN_RUN_RAW) != 0;
        unsigned* words = raw ? max_bits : plan->d_sync + kMaxWordOff;
        hipLaunchKernelGGL(k_param_query_gen, dim3((unsigned)grid), dim3(pp->gT), lds, s, pp->d_image, pp->nf, ev,
                           (long long)n_queries, pp->N, L, pp->wbuf, pp->max_slots, words, out);
        PHIP_TRY(hipGetLastError());
        if (raw) return CBN_OK;
        if (reinterpret_cast<uintptr_t>(out) % 16) return set_err(CBN_E_ARG, "cbn_plan_run: out must be 16-B aligned");
        return launch_scale(out, n_queries * (long long)pp->N, words, pp->max_slots, max_bits, s);
    }
    const long long QW = (n_queries + kWave - 1) / kWave;
    // column chunk: linear models (mu costs a few FMAs) take 8 columns per lane
    // (<= 64 VGPRs: 8 waves per SIMD); MLPs keep whole rows up to 32 columns
    // (every extra chunk re-evaluates the network)
    int nc = pp->nc;
    const bool lin16 = pp->lin16 && !diag_env("CBN_PARAM_LIN8");
    if (pp->hmax == 0 && specialised(pp->hmax, pp->mode)) nc = lin16 ? 16 : 8;
    const int L = (pp->N + nc - 1) / nc;
    const long long waves = QW * L;
    if (waves >= (1LL << 31) || n_queries > (1LL << 30))
        return set_err(CBN_E_LIMIT, "cbn_plan_run: batch too large for one launch");
    // factor split (ParamPlan::parts; CBN_PARAM_PARTS overrides it for A/B)
    int parts = pp->parts;
    if (const char* e = diag_env("CBN_PARAM_PARTS")) {
        const int v = atoi(e);
        if (v == 1 || v == 2 || v == 3 || v == 4 || v == 6) parts = v;
    }
    if (!pp->guard_ok[parts]) parts = 1;  // a range whose products could overflow: the reference's order only
    const int wpb = query_block_threads(parts) / kWave;
    long long grid = (waves * parts + wpb - 1) / wpb;
    grid = std::max(1LL, std::min(grid, (long long)pp->max_slots));
    const bool raw = (flags & CBN_RUN_RAW) != 0;
    unsigned* words = raw ? max_bits : plan->d_sync + kMaxWordOff;
    if (!specialised(pp->hmax, pp->mode)) {
        launch_query_t<16, 32, 4>(pp, (unsigned)grid, ev, n_queries, (int)QW, L, words, out, s, parts);
    } else if (pp->hmax == 0) {  // linear models: 8-column chunks
        if (lin16) launch_query_lin<16, true>(pp, (unsigned)grid, ev, n_queries, (int)QW, L, words, out, s, parts);
        else if (pp->all_m1) launch_query_lin<8, true>(pp, (unsigned)grid, ev, n_queries, (int)QW, L, words, out, s, parts);
        else launch_query_lin<8, false>(pp, (unsigned)grid, ev, n_queries, (int)QW, L, words, out, s, parts);
    } else {
        switch (nc) {
            case 8: launch_query_mlp<8>(pp, (unsigned)grid, ev, n_queries, (int)QW, L, words, out, s, parts); break;
            case 16: launch_query_mlp<16>(pp, (unsigned)grid, ev, n_queries, (int)QW, L, words, out, s, parts); break;
            default: launch_query_mlp<32>(pp, (unsigned)grid, ev, n_queries, (int)QW, L, words, out, s, parts); break;
        }
    }
    PHIP_TRY(hipGetLastError());
    if (raw) return CBN_OK;
    if (reinterpret_cast<uintptr_t>(out) % 16) return set_err(CBN_E_ARG, "cbn_plan_run: out must be 16-B aligned");
    return launch_scale(out, n_queries * (long long)pp->N, words, pp->max_slots, max_bits, s);
}

namespace {
// Plan of a network with a model beyond the fast kernels: GRec image
// (records, then per factor widths / input slots as ints, weights, node
// samples, free-input samples, query-independent row)
int create_param_generic(const cbn_param_factor* factors, int n_factors, int N, cbn_plan** plan) {
    std::vector<GRec> recs(n_factors);
    std::vector<HostModel> hm(n_factors);
    std::vector<int> consts;
    long long off = (long long)n_factors * (sizeof(GRec) / 4);
    const long long row = (N + kColPad - 1) / kColPad * kColPad;
    int ns = 0, wbuf = 1;
    for (int f = 0; f < n_factors; ++f) {
        const cbn_param_factor& h = factors[f];
        GRec& r = recs[f];
        memset(&r, 0, sizeof(r));
        int rc = resolve_model(h.model, hm[f], "factor", f);
        if (rc) return rc;
        const HostModel& m = hm[f];
        if (h.kind < CBN_FACTOR_SCALAR || h.kind > CBN_FACTOR_QUERY)
            return set_err(CBN_E_ARG, "factor %d: bad kind %d", f, h.kind);
        if (!h.node_samples) return set_err(CBN_E_ARG, "factor %d: null node samples", f);
        if (m.w[0] > kMaxP && !h.input_slots)
            return set_err(CBN_E_ARG, "factor %d: %d inputs need the input_slots array", f, m.w[0]);
        int n_obs = 0, n_free = 0;
        long long M = 1;
        for (int i = 0; i < m.w[0]; ++i) {
            const int sl = h.input_slots ? h.input_slots[i] : h.input_slot[i];
            if (sl >= 0) {
                if (sl >= CBN_MAX_EVIDENCE) return set_err(CBN_E_LIMIT, "factor %d: evidence slot %d", f, sl);
                ns = std::max(ns, sl + 1);
                ++n_obs;
            } else if (sl == CBN_INPUT_FREE) {
                ++n_free;
                M *= N;
                if (M >= (1LL << 31)) return set_err(CBN_E_LIMIT, "factor %d: too many free-parent combos", f);
            } else if (sl != CBN_INPUT_ONE) {
                return set_err(CBN_E_ARG, "factor %d: bad input slot %d", f, sl);
            }
        }
        if (n_free > 0 && !h.input_samples) return set_err(CBN_E_ARG, "factor %d: free inputs without samples", f);
        if ((h.kind == CBN_FACTOR_QUERY) != (n_obs > 0))
            return set_err(CBN_E_ARG, "factor %d: QUERY iff some parent observed", f);
        if (h.kind == CBN_FACTOR_SCALAR && n_free > 0) return set_err(CBN_E_ARG, "factor %d: SCALAR with free inputs", f);
        r.kind = h.kind;
        r.family = h.model.family;
        r.unit = h.model.scale == 1.f ? 1 : 0;
        r.M = (int)M;
        r.n_layers = m.n_layers;
        r.n_in = m.w[0];
        r.act = m.act;
        r.scale = h.model.scale;
        r.inv_scale = 1.f / h.model.scale;
        r.norm = h.model.norm;
        r.widths_off = (int)off;
        off += (m.n_layers + 1 + 3) & ~3LL;
        r.slots_off = (int)off;
        off += (m.w[0] + 3) & ~3LL;
        r.w_off = (int)off;
        off += (m.n_weights + 3) & ~3LL;
        r.s_off = (int)off;
        off += row;
        if (n_free > 0) {
            r.fs_off = (int)off;
            off += ((long long)m.w[0] * N + 3) & ~3LL;
        }
        if (h.kind != CBN_FACTOR_QUERY) {
            r.c_off = (int)off;
            off += row;
            consts.push_back(f);
        }
        if (off >= (1LL << 30)) return set_err(CBN_E_LIMIT, "parametric plan image too large");
        wbuf = std::max(wbuf, m.wmax);
    }
    const int T = gen_threads(wbuf);
    if (T == 0) return set_err(CBN_E_LIMIT, "parametric plan: layers of %d units exceed the LDS", wbuf);
    // host copy of the record / int region (weights and samples are copied device to device)
    std::vector<float> host((size_t)off, 0.f);
    memcpy(host.data(), recs.data(), sizeof(GRec) * n_factors);
    for (int f = 0; f < n_factors; ++f) {
        const cbn_param_factor& h = factors[f];
        int* wi = reinterpret_cast<int*>(host.data() + recs[f].widths_off);
        for (int l = 0; l <= hm[f].n_layers; ++l) wi[l] = hm[f].w[l];
        int* si = reinterpret_cast<int*>(host.data() + recs[f].slots_off);
        for (int i = 0; i < hm[f].w[0]; ++i) si[i] = h.input_slots ? h.input_slots[i] : h.input_slot[i];
    }
    ParamPlan* pp = new ParamPlan();
    pp->generic = true;
    pp->nf = n_factors;
    pp->N = N;
    pp->ns = ns;
    pp->wbuf = wbuf;
    pp->gT = T;
    pp->image_floats = (int)off;
    pp->max_slots = std::min(4 * num_cu(), kMaxSlots);
    cbn_plan* P = new cbn_plan();
    P->param = pp;
    P->nf = n_factors;
    P->ns = ns;
    P->N = N;
    bool ok = hipMalloc(&pp->d_image, sizeof(float) * (size_t)off) == hipSuccess &&
              hipMalloc(&pp->d_which, sizeof(int) * std::max<size_t>(consts.size(), 1)) == hipSuccess &&
              hipMalloc(&P->d_sync, sizeof(unsigned) * kSyncWords) == hipSuccess;
    ok = ok && hipMemcpy(pp->d_image, host.data(), sizeof(float) * (size_t)off, hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMemset(P->d_sync, 0, sizeof(unsigned) * kSyncWords) == hipSuccess;
    ok = ok && (consts.empty() ||
                hipMemcpy(pp->d_which, consts.data(), sizeof(int) * consts.size(), hipMemcpyHostToDevice) == hipSuccess);
    for (int f = 0; ok && f < n_factors; ++f) {
        const cbn_param_factor& h = factors[f];
        const GRec& r = recs[f];
        ok = hipMemcpy(pp->d_image + r.w_off, h.model.weights, sizeof(float) * hm[f].n_weights,
                       hipMemcpyDeviceToDevice) == hipSuccess;
        ok = ok && hipMemcpy(pp->d_image + r.s_off, h.node_samples, sizeof(float) * N, hipMemcpyDeviceToDevice) ==
                       hipSuccess;
        if (ok && r.fs_off)
            ok = hipMemcpy(pp->d_image + r.fs_off, h.input_samples, sizeof(float) * (size_t)r.n_in * N,
                           hipMemcpyDeviceToDevice) == hipSuccess;
    }
    ok = ok && hipDeviceSynchronize() == hipSuccess;
    if (ok && !consts.empty()) {
        allow_deep(&k_param_const_gen);
        hipLaunchKernelGGL(k_param_const_gen, dim3((unsigned)consts.size()), dim3(T),
                           (size_t)2 * wbuf * T * sizeof(float), nullptr, pp->d_image, pp->d_which, N, wbuf);
        ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess;
    }
    if (!ok) {
        cbn_plan_destroy(P);
        return set_err(CBN_E_HIP, "cbn_plan_create_param: device allocation/upload/build failed");
    }
    *plan = P;
    return CBN_OK;
}
// The split query kernel's order guard (FSplit).  peak_f bounds factor f's
// values: a Gaussian density's norm (linear_regression.py:91-95), a logistic
// density's 1 / (4 scale) (logistIc_regression.py:90-98), with 2^-10 slack
// for the rounding of the fp32 forms; a mean over free combos or a
// query-independent row is a mean of such values.  G_p = prod over part p of
// max(1, peak_f) bounds every partial product of the range; with G_p <=
// 2^100 the split is kept and the kernel checks, per lane and column, that
// the range's product and the reference's running product through part p
// stayed within [2^-125, 2^126]; where one may not have, the two orders
// differ by at most ucap = n_factors 2^-148 prod_q G_q (each subnormal
// rounding errs by <= 2^-150, then grows by at most the remaining factors'
// bound) beyond their ordinary relative rounding -- a lane for which that is
// not below 2^-30 of its own largest value takes the reference's order (the
// kernel's combine step).
void param_split_guard(cbn::ParamPlan* pp, const PRec* recs, int n_factors) {
    std::vector<double> peak(n_factors);
    bool mono = true;
    for (int f = 0; f < n_factors; ++f) {
        const PRec& r = recs[f];
        const double pk = (r.family == CBN_FAMILY_GAUSS ? (double)r.norm : 0.25 / (double)r.scale) * (1.0 + 0x1p-10);
        peak[f] = pk == pk ? pk : HUGE_VAL;  // a NaN parameter: no bound
        mono = mono && peak[f] <= 1.0;
    }
    pp->mono = mono;
    for (int parts : {1, 2, 3, 4, 6}) {
        const int* b = pp->split[parts];
        bool ok = true;
        double Gall = 1.0;  // prod_q G_q
        for (int p = 0; p < parts; ++p) {
            double G = 1.0;
            for (int f = b[p]; f < b[p + 1]; ++f) G *= std::max(1.0, peak[f]);
            ok = ok && G <= 0x1p100;
            Gall *= G;
            pp->guard_lo[parts][p] = ok ? (float)(0x1p-125 * G) : 0.f;
            pp->guard_hi[parts][p] = ok ? (float)(0x1p126 / G) : 0.f;
        }
        // (beyond the float range: +inf, no hazard lane keeps the split there)
        const double uc = (double)n_factors * 0x1p-148 * Gall;
        pp->guard_ucap[parts] = uc <= 0x1p127 ? (float)uc : HUGE_VALF;
        pp->guard_screen[parts] = Gall <= 0x1p60 ? (float)(0x1p-125 * Gall * Gall) : HUGE_VALF;
        pp->guard_ok[parts] = parts == 1 || ok;
    }
}

}  // namespace

extern "C" {

int cbn_plan_create_param(const cbn_param_factor* factors, int32_t n_factors, int32_t n_samples, cbn_plan** plan) {
    if (!plan || !factors || n_factors <= 0 || n_samples <= 0)
        return set_err(CBN_E_ARG, "cbn_plan_create_param: bad arguments");
    *plan = nullptr;
    const int N = n_samples;
    for (int f = 0; f < n_factors; ++f) {  // any model beyond the fast kernels: the whole plan runs generic
        HostModel hm;
        const int rc = resolve_model(factors[f].model, hm, "factor", f);
        if (rc) return rc;
        if (!hm.fast || diag_env("CBN_PARAM_GENERIC")) return create_param_generic(factors, n_factors, N, plan);
    }
    std::vector<PRec> recs(n_factors);
    std::vector<int> consts;
    const long long cst_off = (long long)n_factors * kRecFloats;  // {0, 1}: constant model inputs
    long long off = cst_off + 4 + (long long)n_factors * kHeadFloats;  // then the PHead array
    std::vector<int> lw_off(n_factors, 0);  // linear models with <= kTabIn inputs: [w0..w3, bias] copy
    int ns = 0, hmax = 0;
    for (int f = 0; f < n_factors; ++f) {
        const cbn_param_factor& h = factors[f];
        PRec& r = recs[f];
        memset(&r, 0, sizeof(r));
        long long nw = 0;
        int rc = check_model(h.model, r.m, nw, "factor", f);
        if (rc) return rc;
        hmax = std::max(hmax, hmax_for(r.m));
        if (h.kind < CBN_FACTOR_SCALAR || h.kind > CBN_FACTOR_QUERY)
            return set_err(CBN_E_ARG, "factor %d: bad kind %d", f, h.kind);
        if (!h.node_samples) return set_err(CBN_E_ARG, "factor %d: null node samples", f);
        int n_obs = 0, n_free = 0;
        long long M = 1;
        for (int i = 0; i < kMaxP; ++i) r.in_slot[i] = kInputNone;
        for (int i = 0; i < r.m.width[0]; ++i) {
            const int sl = h.input_slots ? h.input_slots[i] : h.input_slot[i];
            if (sl >= 0) {
                if (sl >= CBN_MAX_EVIDENCE) return set_err(CBN_E_LIMIT, "factor %d: evidence slot %d", f, sl);
                ns = std::max(ns, sl + 1);
                ++n_obs;
            } else if (sl == CBN_INPUT_FREE) {
                ++n_free;
                r.free_mask |= 1 << i;
                M *= N;
                if (M >= (1LL << 31)) return set_err(CBN_E_LIMIT, "factor %d: too many free-parent combos", f);
            } else if (sl != CBN_INPUT_ONE) {
                return set_err(CBN_E_ARG, "factor %d: bad input slot %d", f, sl);
            }
            r.in_slot[i] = sl;
        }
        if (n_free > 0 && !h.input_samples) return set_err(CBN_E_ARG, "factor %d: free inputs without samples", f);
        if ((h.kind == CBN_FACTOR_QUERY) != (n_obs > 0))
            return set_err(CBN_E_ARG, "factor %d: QUERY iff some parent observed", f);
        if (h.kind == CBN_FACTOR_SCALAR && n_free > 0) return set_err(CBN_E_ARG, "factor %d: SCALAR with free inputs", f);
        r.kind = h.kind;
        r.family = h.model.family;
        r.scale = h.model.scale;
        r.inv_scale = 1.f / h.model.scale;
        r.norm = h.model.norm;
        r.unit = h.model.scale == 1.f ? 1 : 0;
        r.M = (int)M;
        r.w_off = (int)off;
        off += (nw + 3) & ~3LL;
        if (r.m.n_layers == 2) {  // pair-packed copy for the query kernel (mlp1p)
            const long long npairs = (r.m.width[1] + 1) / 2;
            r.pw_off = (int)off;
            off += (npairs * (2LL * r.m.width[0] + 4) + 1 + 3) & ~3LL;
        } else if (r.m.n_layers == 1 && r.m.width[0] <= kTabIn) {
            lw_off[f] = (int)off;
            off += 8;
        }
        const long long row = (N + kColPad - 1) / kColPad * kColPad;  // padded: chunk reads never leave the row
        r.s_off = (int)off;
        off += row;
        if (n_free > 0) {
            r.fs_off = (int)off;
            off += ((long long)r.m.width[0] * N + 3) & ~3LL;
        }
        if (h.kind != CBN_FACTOR_QUERY) {
            r.c_off = (int)off;
            off += row;
            consts.push_back(f);
        }
        if (off >= (1LL << 30)) return set_err(CBN_E_LIMIT, "parametric plan image too large");
    }
    ParamPlan* pp = new ParamPlan();
    pp->nf = n_factors;
    pp->N = N;
    pp->ns = ns;
    pp->hmax = hmax;
    for (const PRec& r : recs) {
        pp->deep = std::max(pp->deep, deep_bytes(r.m, hmax, kQThreads));
        pp->deep_const = std::max(pp->deep_const, deep_bytes(r.m, hmax));
    }
    pp->mode = -1;
    for (const PRec& r : recs) {
        if (r.kind != CBN_FACTOR_QUERY) continue;
        const int m = (r.family == CBN_FAMILY_GAUSS ? 0 : 2) + (r.unit ? 0 : 1);
        pp->mode = pp->mode < 0 || pp->mode == m ? m : 4;
    }
    if (pp->mode < 0) pp->mode = 0;  // no query factor
    pp->all_m1 = !diag_env("CBN_PARAM_NO_M1");
    for (const PRec& r : recs) pp->all_m1 = pp->all_m1 && (r.kind != CBN_FACTOR_QUERY || r.M == 1);
    // factor split: a plan constant (never a function of the batch size), so
    // the product order -- and every row bit -- is the same however the batch
    // is sharded.  Two parts by default (configs[3] NN [16] at 131 072
    // queries 304 -> 218 us in round 1, profiles/r01_bench_cont.json); four
    // for one-hidden-layer M1 plans, whose kernel holds 6 waves per SIMD
    // (NN [16] at 131 072 queries 136 -> 125 us, 1 M queries +3 %).
    // Linear M1 plans with N >= 16 take 16-column chunks and four parts
    // (half the evidence loads and model evaluations of 8-column chunks at the
    // same 8 waves per SIMD): LR at 131 072 queries 54 -> 48 us, 1 M 377 -> 331 us.
    // (Round 5: at 6 waves per SIMD, 4 parts make 1.33 rounds of waves; 3
    // parts in 6-wave blocks -- one whole round at 131 072 queries --
    // measured slower, 47.8-48.1 vs 43.3-43.6 us, 6 parts 52.2-52.5:
    // profiles/r05_param_ab.json.  CBN_PARAM_PARTS=3|6 under CBN_DIAG.)
    pp->parts = n_factors >= 2 ? 2 : 1;
    pp->lin16 = pp->all_m1 && hmax == 0 && N >= 16;
    if (pp->all_m1 && (hmax == 1 || pp->lin16) && n_factors >= 8) pp->parts = 4;
    pp->image_floats = (int)off;
    pp->cst_off = (int)cst_off;
    pp->tab_ok = (long long)n_factors * kTabIn <= kTabCols;
    for (const PRec& r : recs)
        for (int i = kTabIn; i < kMaxP; ++i) pp->tab_ok = pp->tab_ok && r.in_slot[i] == kInputNone;
    if (pp->tab_ok) {
        pp->in_slot.resize((size_t)n_factors * kTabIn);
        for (int f = 0; f < n_factors; ++f)
            for (int i = 0; i < kTabIn; ++i) pp->in_slot[f * kTabIn + i] = recs[f].in_slot[i];
    } else {
        pp->mode = 4;  // the slot-mode (LDS column table) kernel is the generic one
    }
    if ((size_t)n_factors * kMaxP * sizeof(InCol) + pp->deep > (size_t)kDynLdsMax) {
        delete pp;
        return set_err(CBN_E_LIMIT, "parametric plan: %d factors need more LDS than a CU has", n_factors);
    }
    // column chunk per lane: whole rows when they fit (the model runs once
    // per query and factor), else 32-column chunks
    int nc = 32;
    if (N <= 8) nc = 8;
    else if (N <= 16) nc = 16;
    if (const char* e = diag_env("CBN_PARAM_NC")) {
        const int v = atoi(e);
        if (v == 8 || v == 16 || v == 32) nc = v;
    }
    if (!specialised(hmax, pp->mode)) {
        nc = 16;  // the one generic instantiation
        if (hmax > 0) pp->hmax = 32;
    }
    pp->nc = nc;
    pp->L = (N + nc - 1) / nc;
    pp->max_slots = std::min(4 * num_cu(), kMaxSlots);
    {   // factor ranges of the split query kernel, balanced by estimated VALU cost
        std::vector<double> cost(n_factors, 1.0);
        double total = 0;
        for (int f = 0; f < n_factors; ++f) {
            const PRec& r = recs[f];
            if (r.kind == CBN_FACTOR_QUERY) {
                double mc = 0;
                for (int l = 0; l < r.m.n_layers; ++l) mc += (double)r.m.width[l + 1] * (r.m.width[l] + 1);
                for (int l = 1; l < r.m.n_layers; ++l) mc += 20.0 * r.m.width[l];  // activations
                cost[f] = (double)r.M * (mc + 15.0 * N);
            }
            total += cost[f];
        }
        for (int parts : {1, 2, 3, 4, 6}) {
            int* b = pp->split[parts];
            b[0] = 0;
            int p = 1;
            double acc = 0;
            for (int f = 0; f < n_factors && p < parts; ++f) {
                acc += cost[f];
                while (p < parts && acc >= total * p / parts) b[p++] = f + 1;
            }
            while (p <= parts) b[p++] = n_factors;
        }
        param_split_guard(pp, recs.data(), n_factors);
    }
    cbn_plan* P = new cbn_plan();
    P->param = pp;
    P->nf = n_factors;
    P->ns = ns;
    P->N = N;
    bool ok = hipMalloc(&pp->d_image, sizeof(float) * (size_t)off) == hipSuccess &&
              hipMalloc(&pp->d_which, sizeof(int) * std::max<size_t>(consts.size(), 1)) == hipSuccess &&
              hipMalloc(&P->d_sync, sizeof(unsigned) * kSyncWords) == hipSuccess;
    ok = ok && hipMemset(pp->d_image, 0, sizeof(float) * (size_t)off) == hipSuccess;
    ok = ok && hipMemset(P->d_sync, 0, sizeof(unsigned) * kSyncWords) == hipSuccess;
    ok = ok && hipMemcpy(pp->d_image, recs.data(), sizeof(PRec) * n_factors, hipMemcpyHostToDevice) == hipSuccess;
    const float cst[4] = {0.f, 1.f, 0.f, 0.f};
    ok = ok && hipMemcpy(pp->d_image + cst_off, cst, sizeof(cst), hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && (consts.empty() ||
                hipMemcpy(pp->d_which, consts.data(), sizeof(int) * consts.size(), hipMemcpyHostToDevice) == hipSuccess);
    for (int f = 0; ok && f < n_factors; ++f) {
        const cbn_param_factor& h = factors[f];
        const PRec& r = recs[f];
        long long nw = 0;
        for (int l = 0; l < r.m.n_layers; ++l) nw += (long long)r.m.width[l + 1] * (r.m.width[l] + 1);
        ok = hipMemcpy(pp->d_image + r.w_off, h.model.weights, sizeof(float) * nw, hipMemcpyDeviceToDevice) == hipSuccess;
        ok = ok && hipMemcpy(pp->d_image + r.s_off, h.node_samples, sizeof(float) * N, hipMemcpyDeviceToDevice) == hipSuccess;
        if (ok && r.fs_off)
            ok = hipMemcpy(pp->d_image + r.fs_off, h.input_samples, sizeof(float) * (size_t)r.m.width[0] * N,
                           hipMemcpyDeviceToDevice) == hipSuccess;
        if (ok && r.pw_off) {
            std::vector<float> w(nw), pw;
            ok = hipMemcpy(w.data(), h.model.weights, sizeof(float) * nw, hipMemcpyDeviceToHost) == hipSuccess;
            pack_pairs(w, r.m.width[0], r.m.width[1], pw);
            ok = ok && hipMemcpy(pp->d_image + r.pw_off, pw.data(), sizeof(float) * pw.size(), hipMemcpyHostToDevice) ==
                           hipSuccess;
        }
        if (ok && lw_off[f]) {  // zero-padded linear weights: [w0..w_{n-1}, 0.., bias at kTabIn]
            const int n = r.m.width[0];
            std::vector<float> w(n + 1), lw(8, 0.f);
            ok = hipMemcpy(w.data(), h.model.weights, sizeof(float) * (n + 1), hipMemcpyDeviceToHost) == hipSuccess;
            for (int i = 0; i < n; ++i) lw[i] = w[i];
            lw[kTabIn] = w[n];
            ok = ok && hipMemcpy(pp->d_image + lw_off[f], lw.data(), sizeof(float) * 8, hipMemcpyHostToDevice) == hipSuccess;
        }
    }
    if (ok) {  // hot headers (PHead) of the M1 column-table kernels
        std::vector<PHead> heads(n_factors);
        for (int f = 0; f < n_factors; ++f) {
            const PRec& r = recs[f];
            PHead& hh = heads[f];
            memset(&hh, 0, sizeof(hh));
            hh.kind = r.kind;
            hh.row = r.kind == CBN_FACTOR_QUERY ? r.s_off : r.c_off;
            hh.wp = r.m.n_layers == 2 ? r.pw_off : lw_off[f];
            hh.n_in = r.m.width[0];
            hh.hid = r.m.n_layers == 2 ? r.m.width[1] : 0;
            hh.n_layers = r.m.n_layers;
            hh.act = r.m.act;
            hh.scale = r.scale;
            hh.inv_scale = r.inv_scale;
            hh.norm = r.norm;
        }
        ok = hipMemcpy(pp->d_image + cst_off + 4, heads.data(), sizeof(PHead) * n_factors, hipMemcpyHostToDevice) ==
             hipSuccess;
    }
    ok = ok && hipDeviceSynchronize() == hipSuccess;
    if (ok && !consts.empty()) {
        switch (hmax) {
            case 0: launch_const_t<0>(pp->d_image, pp->d_which, (int)consts.size(), N, pp->deep_const, nullptr); break;
            case 1: launch_const_t<1>(pp->d_image, pp->d_which, (int)consts.size(), N, pp->deep_const, nullptr); break;
            default: launch_const_t<32>(pp->d_image, pp->d_which, (int)consts.size(), N, pp->deep_const, nullptr); break;
        }
        ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess;
    }
    if (!ok) {
        cbn_plan_destroy(P);
        return set_err(CBN_E_HIP, "cbn_plan_create_param: device allocation/upload/build failed");
    }
    *plan = P;
    return CBN_OK;
}

int cbn_param_eval(const cbn_param_model* model, const float* points, int64_t n_rows, int32_t n_points,
                   const float* query, int32_t root_bias_only, float* out, void* stream) {
    if (!model || n_rows < 0 || n_points < 0 || (n_rows > 0 && n_points > 0 && (!points || !out)))
        return set_err(CBN_E_ARG, "cbn_param_eval: bad arguments");
    HostModel hm;
    int rc = resolve_model(*model, hm, "model", 0);
    if (rc) return rc;
    if (root_bias_only && hm.n_layers != 1) return set_err(CBN_E_ARG, "cbn_param_eval: bias-only needs a linear model");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (!hm.fast || diag_env("CBN_PARAM_GENERIC")) {
        const int T = gen_threads(hm.wmax);
        if (T == 0) return set_err(CBN_E_LIMIT, "cbn_param_eval: layers of %d units exceed the LDS", hm.wmax);
        if (n_rows == 0 || n_points == 0) return CBN_OK;
        GWidths gw;
        memset(&gw, 0, sizeof(gw));
        for (int l = 0; l <= hm.n_layers; ++l) gw.w[l] = hm.w[l];
        const long long blocks = std::max(1LL, std::min<long long>((n_rows + T - 1) / T, 8192));
        allow_deep(&k_param_eval_gen);
        hipLaunchKernelGGL(k_param_eval_gen, dim3((unsigned)blocks), dim3(T), (size_t)2 * hm.wmax * T * sizeof(float),
                           s, gw, hm.n_layers, hm.act, model->family, model->scale == 1.f ? 1 : 0, model->scale,
                           model->norm, model->weights, points, (long long)n_rows, (int)n_points, query, hm.wmax, out);
        PHIP_TRY(hipGetLastError());
        return CBN_OK;
    }
    MDesc m;
    long long nw = 0;
    rc = check_model(*model, m, nw, "model", 0);
    if (rc) return rc;
    if (n_rows == 0 || n_points == 0) return CBN_OK;
    const long long blocks = std::max(1LL, std::min<long long>((n_rows + kThreads - 1) / kThreads, 8192));
    const int unit = model->scale == 1.f ? 1 : 0;
#define CBN_EVAL(H)                                                                                                 \
    allow_deep(&k_param_eval<H>);                                                                                   \
    hipLaunchKernelGGL(k_param_eval<H>, dim3((unsigned)blocks), dim3(kThreads), deep_bytes(m, H), s, m, model->family, unit, \
                       model->scale, model->norm, model->weights, points, (long long)n_rows, (int)n_points, query, \
                       (int)root_bias_only, out)
    switch (hmax_for(m)) {
        case 0: CBN_EVAL(0); break;
        case 1: CBN_EVAL(1); break;
        default: CBN_EVAL(32); break;
    }
#undef CBN_EVAL
    PHIP_TRY(hipGetLastError());
    return CBN_OK;
}

}  // extern "C"
