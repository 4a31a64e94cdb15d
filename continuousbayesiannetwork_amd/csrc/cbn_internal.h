// cbn_internal.h -- internal layout shared by the translation units of
// libcbn_amd.so (cbn_infer.hip: discrete/table path + C ABI plumbing;
// cbn_param.hip: parametric CPD path).  Not part of the public C ABI
// (include/cbn_amd.h).
#ifndef CBN_INTERNAL_H
#define CBN_INTERNAL_H

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/cbn_amd.h"

namespace cbn {

constexpr int kWave = 64;
constexpr int kLdsBudget = 160 * 1024;
constexpr int kFastPtrs = 416;  // fast table path: 104 factors x 4 observed parents (3.3 KiB of kernel arguments)

// plan sync buffer (unsigned words): line 0 = timeout flag (word 2) and the
// max/raw passes' max staging + arrival counter (words 4-5); from word
// kSlotWordOff, the fused barrier's slots: block b publishes {epoch, max} in
// its own 8-byte slot and every block polls all of them.
constexpr int kSyncLine = 32;
constexpr int kHostStatusWordOff = 8;  // words 8-9 of line 0: device address of the plan's host-mapped status
constexpr int kMaxSlots = 1024;
constexpr int kSlotWordOff = kSyncLine;
// then the max/raw passes' per-block maxima (one word per block; the
// consumer -- write pass, k_scale, k_reduce_max, or RCCL -- reduces them: no
// same-address fan-in, ~12 ns per arrival serialised at the memory side)
constexpr int kMaxWordOff = kSlotWordOff + 2 * kMaxSlots;
constexpr int kSyncWords = kMaxWordOff + kMaxSlots;

struct DevFactor;
struct QSlot;
struct BuildItem;
struct ParamPlan;  // cbn_param.hip
struct DirectPlan;  // cbn_direct.hip

int set_err(int code, const char* fmt, ...);
// getenv(name) when the library was loaded with CBN_DIAG=1, else nullptr
// (diagnostic kernel-selection switches; cbn_infer.hip)
const char* diag_env(const char* name);
int num_cu();

// out[i] /= max(words[0, n_words)) in place on `s`; block 0 also stores that
// max word in *pub when pub is non-null.
int launch_scale(float* out, long long n, const unsigned* words, int n_words, unsigned* pub, hipStream_t s);

// parametric plans (cbn_param.hip)
int param_run(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
              uint32_t* max_bits, float* out, int32_t flags, hipStream_t s);
void param_destroy(ParamPlan* pp);
int param_max_words(const ParamPlan* pp);

// direct plans (cbn_direct.hip)
int direct_run(cbn_plan* plan, int64_t n_queries, const float* const* evidence, int32_t n_evidence,
               uint32_t* max_bits, float* out, int32_t flags, hipStream_t s);
int direct_build_consts(DirectPlan* dp, hipStream_t s);
void direct_destroy(DirectPlan* dp);
int direct_max_words(const DirectPlan* dp);

}  // namespace cbn

struct cbn_plan {
    int nf = 0;
    int ns = 0;
    int N = 0;
    int vec = 1;
    int L = 1;
    int CH = 1;  // queries per block chunk (LDS-sized)
    cbn::DevFactor* d_fac = nullptr;
    int* d_crec = nullptr;       // k_query_cols: per-factor scalar records (ColRec)
    cbn::QSlot* d_slots = nullptr;
    cbn::BuildItem* d_build = nullptr;
    int n_build = 0;
    int build_units = 0;
    float* d_image = nullptr;    // [tables | observed-column domains | records], 16-B padded pieces
    unsigned* d_sync = nullptr;  // max pass: staging max word + arrival counter
    bool fast = false;           // k_query_fast eligible (records live in the image)
    int fast_slot[cbn::kFastPtrs];  // evidence slot of observed parent p of factor f at [f*4+p] (-1: none)
    static constexpr int kRing = 512;
    hipEvent_t ev[kRing][3] = {};  // timing ring (created on first timed call)
    int ev_n = 0;
    int rec_off = 0;             // float offset of the FastRec array in the image
    int RS = 1;                  // table row stride in floats (>= N; padded to spread LDS banks)
    int vpl = 1;                 // fast path: float4 chunks of one query row per lane
    bool paired = false;         // N = 32 bank-half layout (RS = 64, factor f in half f & 1), VPL 2 in LDS
    bool staged = false;         // paired plans of <= 32 factors: k_query_staged (evidence staged by factor)
    size_t staged_lds_bytes = 0;
    bool cols = false;           // non-paired fast plans: k_query_cols (evidence indexed per slot, round 4)
    bool slots = false;          // global-table plans of >= 4 lanes per query: k_query_slots (round 5)
    int zero_off = -1;
    int prefix = 0;              // staged plans: leading 1-row factors folded into factor `prefix` (k_merge_prefix)
    int prefix_offs[9] = {};     // table offsets of factors 0..prefix
    int prefix_rows = 0;         // rows of factor `prefix`'s table
    unsigned* h_status = nullptr;  // host-mapped: 1 after a fused launch timed out (reported by the next run)           // paired layout: float offset of the zero super-row (ones super-row at +64)
    unsigned fused_epoch = 0;    // tag of the published {epoch, max} granule
    bool fused_ok = false;       // one block per CU fits (LDS/VGPR) -> grid barrier is safe
    size_t fast_lds_bytes = 0;
    int lds_tab_floats = 0;      // global-table plans: the small tables packed first, copied to LDS by k_query_fast
    unsigned long long lds_tab_mask[2] = {0, 0};  // ... and which factors' tables those are (bit f)
    int fast_blocks_per_cu = 1;
    int max_slots = 0;           // fast max/raw passes: blocks per launch at most = words of per-block maxima
    int image_floats = 0;
    int table_floats = 0;
    bool use_lds = false;
    size_t lds_bytes = 0;
    int blocks_per_cu = 1;
    cbn::ParamPlan* param = nullptr;  // parametric-CPD plan (cbn_plan_create_param); table fields unused
    cbn::DirectPlan* direct = nullptr;  // direct plan (cbn_plan_create_direct); table fields unused
};

#endif  // CBN_INTERNAL_H
