// Native host fast path of InferenceEngine.infer for a cached plan.
//
// The per-call work the reference does in Python (bayesian_network.py:208-305:
// gather the evidence columns, allocate out_pdf, run the factor loop) shrinks
// here to: look up each evidence column of the plan in the caller's dict,
// check dtype / device / shape / contiguity (any mismatch -> None, and the
// Python slow path converts or raises exactly as the reference does),
// allocate the [Q, N] output and hand plain pointers to the C ABI
// (cbn_plan_run, include/cbn_amd.h).  Python attribute access on 19 tensors
// cost ~20 us per call -- more than the GPU work of a 65k-query batch.
//
// This is a torch extension (it reads torch tensors); the C ABI it calls stays
// torch-free.  cbn_plan_run is passed in as a function address, so this module
// does not link against libcbn_amd.so.
#include <torch/extension.h>

#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>

#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

using run_fn = int (*)(void*, int64_t, const float* const*, int32_t, unsigned*, float*, int32_t, hipStream_t);

// Diagnostic A/B switches (CBN_COMM_HIGH_PRIO, CBN_FOLD_EAGER) count only when
// CBN_DIAG=1 is set, as in libcbn_amd.so (cbn_diag_enabled, include/cbn_amd.h).
bool diag_switch(const char* name) {
    static const bool diag = [] {
        const char* e = getenv("CBN_DIAG");
        return e && e[0] == '1' && e[1] == 0;
    }();
    const char* e = diag ? getenv(name) : nullptr;
    return e && e[0] == '1';
}

// Returns the output tensor; None when a fast check failed (the caller takes
// the slow path); an int = the C ABI's (negative) error code (the caller
// raises with cbn_last_error()).
// Evidence columns of the plan's slots -> plain pointers (cols, n); false
// when any fast check fails.
struct Cols {
    const float* small[64];
    std::vector<const float*> big;
    const float** p = small;
    int64_t n = 1;
};

bool gather(py::dict& evidence, py::tuple& slots, py::object& first, int64_t device_index, bool target_observed,
            Cols& c) {
    const Py_ssize_t ns = PyTuple_GET_SIZE(slots.ptr());
    int64_t n = 1;
    if (!first.is_none()) {
        PyObject* f = PyDict_GetItem(evidence.ptr(), first.ptr());
        if (!f || !THPVariable_Check(f)) return false;
        const at::Tensor& t = THPVariable_Unpack(f);
        if (t.dim() < 1) return false;
        n = t.size(0);
    }
    if (n == 0 || (!target_observed && n != 1)) return false;
    if (ns > 64) {
        c.big.resize(ns);
        c.p = c.big.data();
    }
    for (Py_ssize_t i = 0; i < ns; ++i) {
        PyObject* v = PyDict_GetItem(evidence.ptr(), PyTuple_GET_ITEM(slots.ptr(), i));
        if (!v || !THPVariable_Check(v)) return false;
        const at::Tensor& t = THPVariable_Unpack(v);
        // [n, 1] only: the kernels read element q of the column as query q's
        // value, and any other width raises in the reference (node.py:233-248;
        // the Python path raises it)
        if (t.scalar_type() != at::kFloat || !t.is_cuda() || t.get_device() != device_index || t.dim() != 2 ||
            t.size(0) != n || t.size(1) != 1 || !t.is_contiguous())
            return false;
        c.p[i] = static_cast<const float*>(t.data_ptr());
    }
    if (c10::hip::current_device() != device_index) return false;
    c.n = n;
    return true;
}

at::Tensor check_out(py::object& out_obj, int64_t n, int64_t n_samples, int64_t dev);

// An empty shard (the first evidence column has no rows) is a valid sharded
// step when every slot column is a [0, 1] tensor; a malformed one returns
// false, so the caller's slow path raises the reference's shape error before
// any collective of the step is issued.
bool empty_shard(py::dict& evidence, py::tuple& slots, py::object& first) {
    if (first.is_none()) return false;
    PyObject* f = PyDict_GetItem(evidence.ptr(), first.ptr());
    if (!f || !THPVariable_Check(f)) return false;
    const at::Tensor& t0 = THPVariable_Unpack(f);
    if (t0.dim() < 1 || t0.size(0) != 0) return false;
    for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(slots.ptr()); ++i) {
        PyObject* v = PyDict_GetItem(evidence.ptr(), PyTuple_GET_ITEM(slots.ptr(), i));
        if (!v || !THPVariable_Check(v)) return false;
        const at::Tensor& t = THPVariable_Unpack(v);
        if (t.dim() != 2 || t.size(0) != 0 || t.size(1) != 1) return false;
    }
    return true;
}

py::object run(uintptr_t fn, uintptr_t plan, py::dict evidence, py::tuple slots, py::object first,
               int64_t device_index, int64_t n_samples, bool target_observed, uintptr_t max_ptr, int32_t flags,
               py::object out_obj) {
    Cols c;
    if (!gather(evidence, slots, first, device_index, target_observed, c)) return py::none();
    at::Tensor out = check_out(out_obj, c.n, n_samples, device_index);
    const hipStream_t s = c10::hip::getCurrentHIPStream(device_index).stream();
    const int rc = reinterpret_cast<run_fn>(fn)(reinterpret_cast<void*>(plan), c.n, c.p,
                                                (int32_t)PyTuple_GET_SIZE(slots.ptr()),
                                                reinterpret_cast<unsigned*>(max_ptr),
                                                static_cast<float*>(out.data_ptr()), flags, s);
    if (rc) return py::int_(rc);
    return py::cast(out);
}

using scale_fn = int (*)(float*, int64_t, const unsigned*, int32_t, hipStream_t);
using scale_batch_fn = int (*)(float* const*, const int64_t*, int32_t, const unsigned*, int32_t, hipStream_t);

#define CBN_HIP_OK(x)                                                                   \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

// The steppers' cross-stream events order the two streams of ONE device (the
// comm stream's all-reduce reads words the compute stream's launches wrote;
// RCCL fences its own peer traffic), so a device-scope release is enough.  The
// default system-scope fence writes back and invalidates L2 at every record:
// measured, the compute stream lost ~20 us per group of 8 steps to the group's
// two records (no-comm folded stepper 13.0-13.4 -> 10.6-10.9 us per step
// without them, tools/slow_probe.py).
constexpr unsigned kEvFlags = hipEventDisableTiming | hipEventReleaseToDevice;

// The stepper's comm stream: a pooled stream of NORMAL priority.  Measured
// (tools/slow_probe.py, profiles/r03_stepper_probe.txt): with the first pooled
// high-priority stream as the comm stream, the raw launches on the compute
// stream ran at ~52 us per step instead of ~12.5 for as long as the stepper
// lived.  CBN_COMM_HIGH_PRIO=1 restores the high-priority stream (A/B).
c10::hip::HIPStream comm_stream(c10::DeviceIndex dev) {
    static const bool high = diag_switch("CBN_COMM_HIGH_PRIO");
    return c10::hip::getStreamFromPool(high, dev);
}

// ---------------------------------------------------------------- RCCL comm --
// A communicator of our own (not c10d's): the sharded step's all-reduce is
// enqueued on the stepper's comm stream straight from C++.  The entry points
// are resolved from the librccl.so instance torch itself loaded (the caller
// passes its path): one RCCL in the process, no second copy from /opt/rocm.
struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
} g_rccl;

void rccl_load(const std::string& path) {
    if (g_rccl.all_reduce) return;
    void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) throw std::runtime_error("cannot load " + path + ": " + dlerror());
    auto sym = [&](const char* name) {
        void* f = dlsym(h, name);
        if (!f) throw std::runtime_error(std::string("librccl: missing ") + name);
        return f;
    };
    g_rccl.get_unique_id = reinterpret_cast<decltype(g_rccl.get_unique_id)>(sym("ncclGetUniqueId"));
    g_rccl.comm_init_rank = reinterpret_cast<decltype(g_rccl.comm_init_rank)>(sym("ncclCommInitRank"));
    g_rccl.comm_destroy = reinterpret_cast<decltype(g_rccl.comm_destroy)>(sym("ncclCommDestroy"));
    g_rccl.error_string = reinterpret_cast<decltype(g_rccl.error_string)>(sym("ncclGetErrorString"));
    g_rccl.all_reduce = reinterpret_cast<decltype(g_rccl.all_reduce)>(sym("ncclAllReduce"));
    g_rccl.all_gather = reinterpret_cast<decltype(g_rccl.all_gather)>(sym("ncclAllGather"));
    g_rccl.broadcast = reinterpret_cast<decltype(g_rccl.broadcast)>(sym("ncclBroadcast"));
    g_rccl.group_start = reinterpret_cast<decltype(g_rccl.group_start)>(sym("ncclGroupStart"));
    g_rccl.group_end = reinterpret_cast<decltype(g_rccl.group_end)>(sym("ncclGroupEnd"));
    g_rccl.comm_count = reinterpret_cast<decltype(g_rccl.comm_count)>(sym("ncclCommCount"));
}

#define CBN_NCCL_OK(x)                                                                                   \
    do {                                                                                                 \
        ncclResult_t r_ = (x);                                                                           \
        if (r_ != ncclSuccess) throw std::runtime_error(std::string(#x ": ") + g_rccl.error_string(r_)); \
    } while (0)

py::bytes nccl_unique_id(std::string rccl_path) {
    rccl_load(rccl_path);
    ncclUniqueId id;
    CBN_NCCL_OK(g_rccl.get_unique_id(&id));
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

uintptr_t nccl_comm_init(std::string rccl_path, py::bytes id_bytes, int world, int rank, int device_index) {
    rccl_load(rccl_path);
    std::string b = id_bytes;
    if (b.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, b.data(), sizeof(id));
    CBN_HIP_OK(hipSetDevice(device_index));
    ncclComm_t comm = nullptr;
    {
        py::gil_scoped_release nogil;  // blocks until every rank joined
        CBN_NCCL_OK(g_rccl.comm_init_rank(&comm, world, id, rank));
    }
    return reinterpret_cast<uintptr_t>(comm);
}

// ranks of one of our communicators as RCCL itself reports them (bench.py's
// rccl_ranks: the N > 1 line checks it against --gpus)
int nccl_comm_count(uintptr_t comm) {
    if (!comm || !g_rccl.comm_count) throw std::invalid_argument("nccl_comm_count: no communicator");
    int n = 0;
    CBN_NCCL_OK(g_rccl.comm_count(reinterpret_cast<ncclComm_t>(comm), &n));
    return n;
}

void nccl_comm_destroy(uintptr_t comm) {
    if (comm && g_rccl.comm_destroy) CBN_NCCL_OK(g_rccl.comm_destroy(reinterpret_cast<ncclComm_t>(comm)));
}

// ------------------------------------------------------- pipelined stepper --
// distributed.ShardedStepper's per-step work in one host call (the Python
// version -- events, stream switch, c10d all_reduce, record_stream -- cost
// ~50 us of host time per step, 4x the GPU time of a 65k-query raw launch).
// Steps are exchanged in groups of G:
//   compute stream A: raw launch of each step -> its words slot
//   comm stream C:    after the group's last raw launch (hand-off), ONE
//                     all-reduce(MAX) over the group's G x W words, ONE scale
//                     launch dividing each step's rows by its own max, and --
//                     with gather -- every step's all-gather of the rank shards
//                     into the full [Q, N] marginal tensor
// so the per-exchange host costs are paid once per G steps.  Word slots form a
// ring of two groups (halves); A waits for C only when it starts a group in a
// half whose previous exchange may still be reading it.  flush() (wait(),
// synchronize()) exchanges a partial group.
//
// StepRing holds exactly that bookkeeping and nothing device-specific: the
// device actions are an Ops object -- HipOps (HIP streams/events, RCCL,
// cbn_scale_batch) for the GPU, PyOps (Python callbacks, CPU tensors) for the
// world-size-2 gloo test that drives the same ring with partial groups,
// wait() mid-group, empty and uneven shards.
struct Slot {
    int half;   // ring half of the group
    int index;  // position in the group
};

template <class Ops>
class StepRing {
  public:
    StepRing(Ops ops, int group) : ops_(std::move(ops)), G_(group < 1 ? 1 : (group > 8 ? 8 : group)) {}

    // enqueue one step: `launch(slot)` writes the step's rows and its words slot
    // (an empty shard zeroes the slot); `item` is what the exchange scales (and
    // gathers) for it.  Returns 0 or a C ABI error code.
    template <class Launch>
    int step(Launch&& launch, typename Ops::Item item) {
        const int half = (int)(g_ & 1);
        if (pend_.empty() && used_[half]) ops_.wait_done(half);  // the exchange two groups back read this half
        const Slot slot{half, (int)pend_.size()};
        int rc = launch(slot);
        if (rc) return rc;
        pend_.push_back(std::move(item));
        ++k_;
        if ((int)pend_.size() == G_) return flush();
        return 0;
    }
    int flush() {
        if (pend_.empty()) return 0;
        const int half = (int)(g_ & 1);
        ops_.handoff();  // C waits for every raw launch of the group (enqueued on A)
        int rc = ops_.exchange(half, (int)pend_.size());  // all-reduce(MAX) of the group's words
        if (!rc) rc = ops_.scale(half, pend_);            // each step / its own global max
        if (!rc) rc = ops_.gather(pend_);                 // optional: reassemble the full tensors
        if (rc) return rc;
        ops_.done(half, pend_);
        used_[half] = true;
        pend_.clear();
        ++g_;
        return 0;
    }
    // every enqueued exchange is ordered before the caller's later work
    int wait() {
        const int rc = flush();
        if (!rc && k_) ops_.join();
        return rc;
    }
    Ops& ops() { return ops_; }
    int64_t steps() const { return k_; }
    int group() const { return G_; }
    int pending() const { return (int)pend_.size(); }

  private:
    Ops ops_;
    int G_;
    std::vector<typename Ops::Item> pend_;
    bool used_[2] = {false, false};
    int64_t k_ = 0, g_ = 0;
};

// What one step contributes to its group's exchange.
struct StepItem {
    at::Tensor rows;  // this rank's [q_r, N] rows (a view into `full` when gathering)
    at::Tensor full;  // gather: the [Q, N] marginal tensor (undefined otherwise)
    std::vector<int64_t> counts;  // gather: rows of every rank, rank order
};

// ---- GPU: HIP streams / events, RCCL, cbn_scale_batch
struct HipOps {
    using Item = StepItem;
    scale_batch_fn scale_batch = nullptr;
    ncclComm_t comm = nullptr;
    int world = 1, rank = 0;
    int64_t dev = 0, W = 0;
    int G = 1;
    c10::hip::HIPStream cs;
    at::Tensor words;  // [2G, W] int32 on the device
    hipEvent_t ready = nullptr, tail = nullptr;
    hipEvent_t done_ev[2] = {nullptr, nullptr};

    HipOps(scale_batch_fn sb, ncclComm_t c, int world_, int rank_, int64_t dev_, int64_t W_, int G_)
        : scale_batch(sb), comm(c), world(world_), rank(rank_), dev(dev_), W(W_), G(G_),
          cs(comm_stream((c10::DeviceIndex)dev_)) {
        words = at::zeros({2 * G, W}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev));
        CBN_HIP_OK(hipEventCreateWithFlags(&ready, kEvFlags));
        CBN_HIP_OK(hipEventCreateWithFlags(&tail, kEvFlags));
        for (auto& e : done_ev) CBN_HIP_OK(hipEventCreateWithFlags(&e, kEvFlags));
    }
    HipOps(HipOps&& o) noexcept
        : scale_batch(o.scale_batch), comm(o.comm), world(o.world), rank(o.rank), dev(o.dev), W(o.W), G(o.G),
          cs(o.cs), words(std::move(o.words)), ready(o.ready), tail(o.tail) {
        done_ev[0] = o.done_ev[0];
        done_ev[1] = o.done_ev[1];
        o.ready = o.tail = o.done_ev[0] = o.done_ev[1] = nullptr;
    }
    ~HipOps() {
        if (ready) (void)hipEventDestroy(ready);
        if (tail) (void)hipEventDestroy(tail);
        for (auto e : done_ev)
            if (e) (void)hipEventDestroy(e);
    }
    hipStream_t A() const { return c10::hip::getCurrentHIPStream(dev).stream(); }
    int* slot_words(Slot s) { return words.data_ptr<int>() + ((int64_t)s.half * G + s.index) * W; }

    // (an event that already completed needs no wait packet: a stream wait
    // costs the queue a barrier packet per group even when satisfied)
    void wait_done(int half) {
        if (hipEventQuery(done_ev[half]) != hipSuccess) CBN_HIP_OK(hipStreamWaitEvent(A(), done_ev[half], 0));
    }
    void handoff() {
        CBN_HIP_OK(hipEventRecord(ready, A()));
        CBN_HIP_OK(hipStreamWaitEvent(cs.stream(), ready, 0));
    }
    int exchange(int half, int nb) {
        if (comm) {
            int* w = words.data_ptr<int>() + (int64_t)half * G * W;
            CBN_NCCL_OK(g_rccl.all_reduce(w, w, (size_t)nb * W, ncclInt32, ncclMax, comm, cs.stream()));
        }
        return 0;
    }
    int scale(int half, const std::vector<Item>& items) {
        float* outs[8];
        int64_t ns[8];
        const int nb = (int)items.size();
        for (int b = 0; b < nb; ++b) {
            outs[b] = static_cast<float*>(items[b].rows.data_ptr());
            ns[b] = items[b].rows.numel();
        }
        return scale_batch(outs, ns, nb, reinterpret_cast<const unsigned*>(words.data_ptr<int>() + (int64_t)half * G * W),
                           (int32_t)W, cs.stream());
    }
    // all-gather of every step's shards into its full tensor: equal shards ->
    // ncclAllGather in place; uneven -> one ncclBroadcast per rank (root r sends
    // its rows to their offset in every rank's full tensor), all in one group
    int gather(const std::vector<Item>& items) {
        bool any = false;
        for (const auto& it : items) any |= it.full.defined();
        if (!any) return 0;
        if (!comm || world == 1) return 0;  // one rank: rows already in place
        CBN_NCCL_OK(g_rccl.group_start());
        for (const auto& it : items) {
            if (!it.full.defined()) continue;
            float* full = static_cast<float*>(it.full.data_ptr());
            const int64_t N = it.full.size(1);
            bool equal = true;
            for (int r = 1; r < world; ++r) equal &= it.counts[r] == it.counts[0];
            if (equal) {
                const size_t cnt = (size_t)(it.counts[0] * N);
                CBN_NCCL_OK(g_rccl.all_gather(full + (int64_t)rank * cnt, full, cnt, ncclFloat32, comm, cs.stream()));
            } else {
                int64_t off = 0;
                for (int r = 0; r < world; ++r) {
                    const size_t cnt = (size_t)(it.counts[r] * N);
                    CBN_NCCL_OK(g_rccl.broadcast(full + off * N, full + off * N, cnt, ncclFloat32, r, comm,
                                                 cs.stream()));
                    off += it.counts[r];
                }
            }
        }
        CBN_NCCL_OK(g_rccl.group_end());
        return 0;
    }
    void done(int half, const std::vector<Item>& items) {
        CBN_HIP_OK(hipEventRecord(done_ev[half], cs.stream()));
        // rows / full tensors are used on C: the caching allocator must not recycle them early
        for (const auto& it : items) {
            c10::hip::HIPCachingAllocator::recordStream(it.rows.storage().data_ptr(), cs);
            if (it.full.defined()) c10::hip::HIPCachingAllocator::recordStream(it.full.storage().data_ptr(), cs);
        }
    }
    void join() {
        CBN_HIP_OK(hipEventRecord(tail, cs.stream()));
        CBN_HIP_OK(hipStreamWaitEvent(A(), tail, 0));
    }
};

at::Tensor check_out(py::object& out_obj, int64_t n, int64_t n_samples, int64_t dev) {
    if (out_obj.is_none())
        return at::empty({n, n_samples}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev));
    if (!THPVariable_Check(out_obj.ptr())) throw std::invalid_argument("out must be a torch tensor");
    at::Tensor out = THPVariable_Unpack(out_obj.ptr());
    if (out.scalar_type() != at::kFloat || !out.is_cuda() || out.get_device() != dev || !out.is_contiguous() ||
        out.dim() != 2 || out.size(0) != n || out.size(1) != n_samples ||
        reinterpret_cast<uintptr_t>(out.data_ptr()) % 16)
        throw std::invalid_argument("out must be a contiguous, 16-B aligned float32 [" + std::to_string(n) + ", " +
                                    std::to_string(n_samples) + "] tensor on cuda:" + std::to_string(dev));
    return out;
}

// One cached (target, evidence keys, N) of InferenceEngine.infer, callable
// straight from BayesianNetwork.infer (round 4): the caller's dict is matched
// against the key tuple it was built for by walking the dict once in
// insertion order (key identity, else string equality) -- no key tuple built
// and hashed, no engine dict lookup, no per-call Python frames -- the slot
// columns are picked by position during that walk, the output is allocated
// and the plan launched; returns (out, target domain view), or None when the
// dict does not match / a fast check fails (the engine's general path then
// runs: conversions, the reference's errors), or the C ABI's error code.
// Only deterministic plans with their tables built (flags fixed at
// construction) get a runner.
class Runner {
  public:
    Runner(uintptr_t fn, uintptr_t plan, py::tuple keys, py::tuple slots, int64_t device_index, int64_t n_samples,
           bool target_observed, uintptr_t max_ptr, int32_t flags, py::object target_domain)
        : run_(reinterpret_cast<run_fn>(fn)), plan_(reinterpret_cast<void*>(plan)), keys_(keys), dev_(device_index),
          n_samples_(n_samples), target_observed_(target_observed), max_ptr_(reinterpret_cast<unsigned*>(max_ptr)),
          flags_(flags), tdom_(THPVariable_Unpack(target_domain.ptr())) {
        const Py_ssize_t nk = PyTuple_GET_SIZE(keys.ptr());
        for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(slots.ptr()); ++i) {
            Py_ssize_t pos = -1;
            for (Py_ssize_t j = 0; j < nk && pos < 0; ++j) {
                const int eq =
                    PyObject_RichCompareBool(PyTuple_GET_ITEM(keys.ptr(), j), PyTuple_GET_ITEM(slots.ptr(), i), Py_EQ);
                if (eq < 0) throw py::error_already_set();
                if (eq == 1) pos = j;
            }
            if (pos < 0) throw std::invalid_argument("Runner: slot key not among the evidence keys");
            slot_pos_.push_back(pos);
        }
        vals_.resize(nk);
        ptrs_.resize(std::max<size_t>(1, slot_pos_.size()));
    }

    py::object call(py::handle evidence, py::object out_obj) {
        PyObject* d = evidence.ptr();
        if (!PyDict_CheckExact(d)) return py::none();
        const Py_ssize_t nk = PyTuple_GET_SIZE(keys_.ptr());
        if (PyDict_GET_SIZE(d) != nk) return py::none();
        Py_ssize_t it = 0, j = 0;
        PyObject *k, *v;
        while (PyDict_Next(d, &it, &k, &v)) {
            PyObject* want = PyTuple_GET_ITEM(keys_.ptr(), j);
            if (k != want) {
                const int eq = PyObject_RichCompareBool(k, want, Py_EQ);
                if (eq != 1) {
                    if (eq < 0) PyErr_Clear();  // a key whose __eq__ raised: no match, the general path decides
                    return py::none();
                }
            }
            vals_[j++] = v;
        }
        int64_t n = 1;
        if (nk > 0) {
            PyObject* f = vals_[0];
            if (!THPVariable_Check(f)) return py::none();
            const at::Tensor& t = THPVariable_Unpack(f);
            if (t.dim() < 1) return py::none();
            n = t.size(0);
        }
        if (n == 0 || (!target_observed_ && n != 1)) return py::none();
        for (size_t i = 0; i < slot_pos_.size(); ++i) {
            PyObject* x = vals_[slot_pos_[i]];
            if (!THPVariable_Check(x)) return py::none();
            const at::Tensor& t = THPVariable_Unpack(x);
            if (t.scalar_type() != at::kFloat || !t.is_cuda() || t.get_device() != dev_ || t.dim() != 2 ||
                t.size(0) != n || t.size(1) != 1 || !t.is_contiguous())
                return py::none();
            ptrs_[i] = static_cast<const float*>(t.data_ptr());
        }
        if (c10::hip::current_device() != dev_) return py::none();
        at::Tensor out = check_out(out_obj, n, n_samples_, dev_);
        const hipStream_t s = c10::hip::getCurrentHIPStream(dev_).stream();
        const int rc = run_(plan_, n, ptrs_.data(), (int32_t)slot_pos_.size(), max_ptr_,
                            static_cast<float*>(out.data_ptr()), flags_, s);
        if (rc) return py::int_(rc);
        const int64_t tn = target_observed_ ? n : 1;
        if (tn != tdom_n_) {
            tdom_view_ = tdom_.unsqueeze(0).expand({tn, -1});
            tdom_n_ = tn;
        }
        return py::make_tuple(out, tdom_view_);
    }

  private:
    run_fn run_;
    void* plan_;
    py::tuple keys_;
    int64_t dev_, n_samples_;
    bool target_observed_;
    unsigned* max_ptr_;
    int32_t flags_;
    at::Tensor tdom_, tdom_view_;
    int64_t tdom_n_ = -1;
    std::vector<Py_ssize_t> slot_pos_;
    std::vector<PyObject*> vals_;
    std::vector<const float*> ptrs_;
};

class Stepper {
  public:
    Stepper(uintptr_t run_addr, uintptr_t scale_batch_addr, uintptr_t plan, py::tuple slots, py::object first,
            int64_t device_index, int64_t n_samples, bool target_observed, int64_t n_words, int group,
            uintptr_t comm, int world, int rank)
        : run_(reinterpret_cast<run_fn>(run_addr)), plan_(reinterpret_cast<void*>(plan)), slots_(slots),
          first_(first), dev_(device_index), n_samples_(n_samples), target_observed_(target_observed),
          ring_(HipOps(reinterpret_cast<scale_batch_fn>(scale_batch_addr), reinterpret_cast<ncclComm_t>(comm), world,
                       rank, device_index, n_words, group < 1 ? 1 : (group > 8 ? 8 : group)),
                group) {}

    // rows (final once this step's group has been exchanged and scaled on the
    // comm stream -- after wait()); with counts (every rank's rows of this
    // step, rank order): the full [sum(counts), N] tensor, this rank's rows
    // written at its offset and the others' all-gathered into it.  None when a
    // fast check failed (the caller converts the evidence and retries), or an
    // int error code from the C ABI.
    py::object step(py::dict evidence, py::object out_obj, int32_t flags, py::object counts_obj) {
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        Cols c;
        int64_t n = 0;
        if (!gather_cols(evidence, c, n)) return py::none();
        HipOps& ops = ring_.ops();
        StepItem item;
        if (!counts_obj.is_none()) {
            item.counts = counts_obj.cast<std::vector<int64_t>>();
            if ((int)item.counts.size() != ops.world || item.counts[ops.rank] != n)
                throw std::invalid_argument("counts must hold every rank's rows of this step (this rank: " +
                                            std::to_string(n) + ")");
            int64_t total = 0, lo = 0;
            for (int r = 0; r < ops.world; ++r) {
                if (r == ops.rank) lo = total;
                total += item.counts[r];
            }
            item.full = out_obj.is_none()
                            ? at::empty({total, n_samples_}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev_))
                            : check_out(out_obj, total, n_samples_, dev_);
            item.rows = item.full.narrow(0, lo, n);
        } else {
            item.rows = check_out(out_obj, n, n_samples_, dev_);
        }
        const auto t1 = clk::now();
        at::Tensor ret = item.full.defined() ? item.full : item.rows;
        float* rows = static_cast<float*>(item.rows.data_ptr());
        int launch_rc = 0;
        int rc = ring_.step(
            [&](Slot s) -> int {
                int* w = ops.slot_words(s);
                if (n > 0) {
                    launch_rc = run_(plan_, n, c.p, (int32_t)PyTuple_GET_SIZE(slots_.ptr()),
                                     reinterpret_cast<unsigned*>(w), rows, flags, ops.A());
                    if (!launch_rc) return 0;
                }
                // empty shard, or a launch the library refused (e.g. the plan's
                // earlier fused call timed out): zero words, and the step still
                // joins its group's collectives so every rank's exchanges stay
                // paired; a refusal is reported after the step is enqueued
                CBN_HIP_OK(hipMemsetAsync(w, 0, sizeof(int) * ops.W, ops.A()));
                return 0;
            },
            std::move(item));
        if (rc) return py::int_(rc);
        if (launch_rc) return py::int_(launch_rc);
        const auto t2 = clk::now();
        tacc_[0] += std::chrono::duration<double, std::micro>(t1 - t0).count();
        tacc_[1] += std::chrono::duration<double, std::micro>(t2 - t1).count();
        ++tn_;
        return py::cast(ret);
    }

    void wait() { check_(ring_.wait()); }
    void synchronize() {
        check_(ring_.flush());
        py::gil_scoped_release nogil;  // a watchdog thread may need to report a stuck peer
        CBN_HIP_OK(hipStreamSynchronize(ring_.ops().cs.stream()));
    }
    uintptr_t comm_stream() { return reinterpret_cast<uintptr_t>(ring_.ops().cs.stream()); }
    int64_t steps() const { return ring_.steps(); }
    int group() const { return ring_.group(); }

    // mean host microseconds per step: gather + alloc, launch + the step's
    // share of the group exchange (hand-off, all-reduce, scale, all-gathers)
    std::vector<double> host_timing() {
        std::vector<double> r(2, 0.0);
        for (int i = 0; i < 2; ++i) r[i] = tn_ ? tacc_[i] / tn_ : 0.0;
        tacc_.fill(0.0);
        tn_ = 0;
        return r;
    }

  private:
    // like gather(), but an empty shard is a valid step (n = 0)
    bool gather_cols(py::dict& evidence, Cols& c, int64_t& n) {
        if (empty_shard(evidence, slots_, first_)) {
            n = 0;
            return true;
        }
        if (!gather(evidence, slots_, first_, dev_, target_observed_, c)) return false;
        n = c.n;
        return true;
    }
    static void check_(int rc) {
        if (rc) throw std::runtime_error("cbn_scale_batch failed (rc=" + std::to_string(rc) + ")");
    }

    run_fn run_;
    void* plan_;
    py::tuple slots_;
    py::object first_;
    int64_t dev_, n_samples_;
    bool target_observed_;
    StepRing<HipOps> ring_;
    std::array<double, 2> tacc_{};
    int64_t tn_ = 0;
};

// ---- CPU test double: the same ring driven by Python callbacks
//   launch(slot_half, slot_index, payload) -> None   (rows + words of the step)
//   exchange(half, n_steps)                          (all-reduce of the group's words)
//   scale(half, [payload, ...])                      (divide each step's rows)
//   gather([payload, ...])                           (reassemble full tensors)
//   and the ordering hooks wait_done(half), handoff(), done(half), join() --
// the test logs every call and checks the ring's protocol from the log.
struct PyOps {
    using Item = py::object;
    py::object cb;  // an object with the methods above
    void wait_done(int half) { cb.attr("wait_done")(half); }
    void handoff() { cb.attr("handoff")(); }
    int exchange(int half, int nb) { return cb.attr("exchange")(half, nb).cast<int>(); }
    int scale(int half, const std::vector<Item>& items) { return cb.attr("scale")(half, py::cast(items)).cast<int>(); }
    int gather(const std::vector<Item>& items) { return cb.attr("gather")(py::cast(items)).cast<int>(); }
    void done(int half, const std::vector<Item>&) { cb.attr("done")(half); }
    void join() { cb.attr("join")(); }
};

class CpuStepRing {
  public:
    CpuStepRing(py::object cb, int group) : ring_(PyOps{cb}, group) {}
    int step(py::object payload) {
        py::object cb = ring_.ops().cb;
        return ring_.step([&](Slot s) -> int { return cb.attr("launch")(s.half, s.index, payload).cast<int>(); },
                          payload);
    }
    int wait() { return ring_.wait(); }
    int flush() { return ring_.flush(); }
    int pending() const { return ring_.pending(); }
    int group() const { return ring_.group(); }

  private:
    StepRing<PyOps> ring_;
};

// cbn_scale on the current stream of out's device (sharded path, after the
// cross-rank all-reduce of the per-block max words).
int scale(uintptr_t fn, const at::Tensor& out, uintptr_t max_ptr, int32_t n_max) {
    const hipStream_t s = c10::hip::getCurrentHIPStream(out.get_device()).stream();
    return reinterpret_cast<scale_fn>(fn)(static_cast<float*>(out.data_ptr()), out.numel(),
                                          reinterpret_cast<const unsigned*>(max_ptr), n_max, s);
}

// ------------------------------------------------- folded-scale stepper ring --
// The rank-local sharded step without a scale launch: every raw launch also
// divides ONE earlier step's rows by that step's all-reduced max
// (cbn_plan_run_fold), so the scale's HBM traffic overlaps the launch's LDS-
// bound products instead of competing with the next launches for the CUs.
//   compute stream A: raw launch of step s (words -> set g % kSets, slot i),
//                     folding the oldest unfinished step of a group exchanged
//                     two groups back (its all-reduce had a whole group of
//                     launches to complete)
//   comm stream C:    per group, ONE all-reduce(MAX) of the group's words in
//                     place, enqueued once A has passed the group's last
//                     launch (host-side event query / wait, no stream wait)
// Word sets form a ring of kSets groups.  Before a group writes set s, any
// step whose words are still in s and not yet folded (a group with empty
// shards or a partial group flushed by wait()) is scaled on A first, and A
// waits for C's last use of s.  wait() exchanges the partial group and scales
// every unfinished step on C, then joins.  FoldRing is that bookkeeping only;
// FoldHipOps binds it to HIP / RCCL / cbn_plan_run_fold, PyFoldOps to Python
// callbacks (the world-size-2 gloo test drives the same ring on CPU).
#ifndef CBN_FOLD_SETS
#define CBN_FOLD_SETS 3
#endif
constexpr int kSets = CBN_FOLD_SETS;
// a group's steps are folded kFoldLag groups later.  Measured (NB=64,
// profiles/r03_stepper_probe.txt): 4 sets (lag 3, rows 24-31 steps old) 11.9
// vs 11.2 us per step for 3 -- the folded rows fall out of the MALL.
constexpr int kFoldLag = kSets - 1;
constexpr int kFoldGroupMax = 32;

template <class Item>
struct FoldPending {
    Item item;
    int set;
    int index;
};

template <class Ops>
class FoldRing {
  public:
    using Item = typename Ops::Item;
    using Pending = FoldPending<Item>;
    // (groups up to kFoldGroupMax steps: a group's leftovers are scaled in runs of <= 8)
    FoldRing(Ops ops, int group) : ops_(std::move(ops)), G_(group < 1 ? 1 : (group > kFoldGroupMax ? kFoldGroupMax : group)) {}

    // launch(slot, fold, consumed) writes the step's rows and words slot and,
    // when `fold` is non-null and the step launches a kernel, finishes that
    // earlier step (consumed = true).  Returns 0 or a C ABI error code.
    template <class Launch>
    int step(Launch&& launch, Item item) {
        if (cur_.empty()) {
            const int brc = begin_group();
            if (brc) return brc;
        }
        const int set = (int)(g_ % kSets);
        const Slot slot{set, (int)cur_.size()};
        const Pending* f = foldq_.empty() ? nullptr : &foldq_.front();
        bool consumed = false;
        const int rc = launch(slot, f, consumed);
        if (rc) return rc;
        if (consumed) {
            ops_.folded(foldq_.front());
            foldq_.pop_front();
        }
        cur_.push_back(Pending{std::move(item), set, slot.index});
        ++k_;
        if ((int)cur_.size() == G_) return exchange_group();
        return 0;
    }
    // every enqueued step final before the caller's later work on A
    int wait() {
        int rc = exchange_group();
        if (rc) return rc;
        for (auto& grp : exch_)
            if (!grp.handed && (rc = hand(grp, /*eager=*/true))) return rc;
        for (auto& grp : exch_)
            for (auto& p : grp.items) foldq_.push_back(std::move(p));
        exch_.clear();
        rc = scale_runs(foldq_, /*on_comm=*/true);
        foldq_.clear();
        if (!rc && k_) ops_.join();
        return rc;
    }
    Ops& ops() { return ops_; }
    int64_t steps() const { return k_; }
    int group() const { return G_; }
    int pending() const { return (int)cur_.size(); }
    int unfinished() const {
        size_t n = foldq_.size() + cur_.size();
        for (auto& g : exch_) n += g.items.size();
        return (int)n;
    }

  private:
    struct Group {
        int64_t g;
        std::vector<Pending> items;
        bool handed = false;
    };
    // Hand exchanged groups to C, oldest first: a group needed for folding by
    // this group (exchanged two groups back) now, waiting on the host for A to
    // pass its last launch; a later one only when A has already passed it.
    // Either way C's all-reduce needs no stream wait on A: measured, a comm
    // stream waiting on the compute stream's event slowed the raw launches by
    // ~2.5 us per step (tools/slow_probe.py, CBN_FOLD_DIAG_SKIP).  eager_
    // (CBN_FOLD_EAGER=1, A/B) hands each group at its exchange with the wait.
    int hand_ready() {
        for (auto& grp : exch_) {
            if (grp.handed) continue;
            const int gset = (int)(grp.g % kSets);
            const bool need = grp.g <= g_ - kFoldLag;
            if (!ops_.passed(gset, /*block=*/need)) break;
            const int rc = hand(grp, /*eager=*/false);
            if (rc) return rc;
        }
        return 0;
    }
    int hand(Group& grp, bool eager) {
        const int gset = (int)(grp.g % kSets);
        if (eager) ops_.handoff(gset);  // C after A's record of the group's last launch
        const int rc = ops_.exchange(gset, (int)grp.items.size());
        if (rc) return rc;
        ops_.mark_set(gset, /*on_comm=*/true);
        grp.handed = true;
        return 0;
    }
    int begin_group() {
        const int hrc = hand_ready();
        if (hrc) return hrc;
        const int set = (int)(g_ % kSets);
        // steps whose words still sit in `set`: finish them before this group overwrites it
        std::deque<Pending> here, keep;
        for (auto& p : foldq_) (p.set == set ? here : keep).push_back(std::move(p));
        foldq_.swap(keep);
        for (auto it = exch_.begin(); it != exch_.end();) {
            if (!it->items.empty() && it->items.front().set == set) {
                for (auto& p : it->items) here.push_back(std::move(p));
                it = exch_.erase(it);
            } else {
                ++it;
            }
        }
        ops_.wait_set(set);  // A after C's last use of the set (its exchange / a wait() scale)
        if (!here.empty()) {
            const int rc = scale_runs(here, /*on_comm=*/false);
            if (rc) return rc;
        }
        // groups exchanged two or more groups back (handed above) become foldable
        while (!exch_.empty() && exch_.front().g <= g_ - kFoldLag) {
            Group& grp = exch_.front();
            if (!grp.items.empty()) ops_.wait_set(grp.items.front().set);  // their all-reduce done
            for (auto& p : grp.items) foldq_.push_back(std::move(p));
            exch_.pop_front();
        }
        return 0;
    }
    int exchange_group() {
        if (cur_.empty()) return 0;
        const int set = (int)(g_ % kSets);
        ops_.record(set);  // A's position after the group's raw launches (and their folds)
        exch_.push_back(Group{g_, std::move(cur_)});
        cur_.clear();
        ++g_;
        if (eager_) return hand(exch_.back(), /*eager=*/true);
        return 0;
    }
    // scale the given steps (runs of consecutive slots of one set per call)
    int scale_runs(std::deque<Pending>& q, bool on_comm) {
        size_t i = 0;
        while (i < q.size()) {
            size_t j = i + 1;
            while (j < q.size() && j - i < 8 && q[j].set == q[i].set && q[j].index == q[j - 1].index + 1) ++j;
            std::vector<const Pending*> run;
            for (size_t k = i; k < j; ++k) run.push_back(&q[k]);
            const int rc = ops_.scale(run, on_comm);
            if (rc) return rc;
            ops_.mark_set(q[i].set, on_comm);
            i = j;
        }
        return 0;
    }

    Ops ops_;
    int G_;
    bool eager_ = diag_switch("CBN_FOLD_EAGER");
    std::vector<Pending> cur_;
    std::deque<Group> exch_;
    std::deque<Pending> foldq_;
    int64_t k_ = 0, g_ = 0;
};

struct FoldItem {
    at::Tensor rows;  // this rank's [q_r, N] rows (unnormalised until folded / scaled)
};

// ---- GPU: HIP streams / events, RCCL, cbn_plan_run_fold / cbn_scale_batch
struct FoldHipOps {
    using Item = FoldItem;
    using P = FoldPending<FoldItem>;
    scale_batch_fn scale_batch = nullptr;
    ncclComm_t comm = nullptr;
    int64_t dev = 0, W = 0;
    int G = 1;
    c10::hip::HIPStream cs;
    at::Tensor words;  // [kSets * G, W] int32 on the device
    hipEvent_t tail = nullptr;
    hipEvent_t set_ev[kSets] = {}, ready_ev[kSets] = {};
    bool set_used[kSets] = {};

    FoldHipOps(scale_batch_fn sb, ncclComm_t c, int64_t dev_, int64_t W_, int G_)
        : scale_batch(sb), comm(c), dev(dev_), W(W_), G(G_),
          cs(comm_stream((c10::DeviceIndex)dev_)) {
        words = at::zeros({kSets * G, W}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev));
        CBN_HIP_OK(hipEventCreateWithFlags(&tail, kEvFlags));
        for (auto& e : set_ev) CBN_HIP_OK(hipEventCreateWithFlags(&e, kEvFlags));
        for (auto& e : ready_ev) CBN_HIP_OK(hipEventCreateWithFlags(&e, kEvFlags));
    }
    FoldHipOps(FoldHipOps&& o) noexcept
        : scale_batch(o.scale_batch), comm(o.comm), dev(o.dev), W(o.W), G(o.G), cs(o.cs), words(std::move(o.words)),
          tail(o.tail) {
        for (int s = 0; s < kSets; ++s) {
            set_ev[s] = o.set_ev[s];
            ready_ev[s] = o.ready_ev[s];
            set_used[s] = o.set_used[s];
            o.set_ev[s] = o.ready_ev[s] = nullptr;
        }
        o.tail = nullptr;
    }
    ~FoldHipOps() {
        if (tail) (void)hipEventDestroy(tail);
        for (auto e : set_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto e : ready_ev)
            if (e) (void)hipEventDestroy(e);
    }
    hipStream_t A() const { return c10::hip::getCurrentHIPStream(dev).stream(); }
    int* slot_words(int set, int index) { return words.data_ptr<int>() + ((int64_t)set * G + index) * W; }

    void wait_set(int set) {  // (skipped when the event already completed, as HipOps::wait_done)
        if (set_used[set] && hipEventQuery(set_ev[set]) != hipSuccess)
            CBN_HIP_OK(hipStreamWaitEvent(A(), set_ev[set], 0));
    }
    void mark_set(int set, bool on_comm) {
        CBN_HIP_OK(hipEventRecord(set_ev[set], on_comm ? cs.stream() : A()));
        set_used[set] = true;
    }
    void record(int set) { CBN_HIP_OK(hipEventRecord(ready_ev[set], A())); }
    bool passed(int set, bool block) {
        if (block) {
            py::gil_scoped_release nogil;  // (watchdog: see Stepper::synchronize)
            CBN_HIP_OK(hipEventSynchronize(ready_ev[set]));
            return true;
        }
        const hipError_t e = hipEventQuery(ready_ev[set]);
        if (e == hipErrorNotReady) return false;
        CBN_HIP_OK(e);
        return true;
    }
    void handoff(int set) { CBN_HIP_OK(hipStreamWaitEvent(cs.stream(), ready_ev[set], 0)); }
    int exchange(int set, int nb) {
        if (comm) {
            int* w = slot_words(set, 0);
            CBN_NCCL_OK(g_rccl.all_reduce(w, w, (size_t)nb * W, ncclInt32, ncclMax, comm, cs.stream()));
        }
        return 0;
    }
    int scale(const std::vector<const P*>& run, bool on_comm) {
        float* outs[8];
        int64_t ns[8];
        const int nb = (int)run.size();
        for (int b = 0; b < nb; ++b) {
            outs[b] = static_cast<float*>(run[b]->item.rows.data_ptr());
            ns[b] = run[b]->item.rows.numel();
            if (on_comm)  // rows used on C: the caching allocator must not recycle them early
                c10::hip::HIPCachingAllocator::recordStream(run[b]->item.rows.storage().data_ptr(), cs);
        }
        return scale_batch(outs, ns, nb, reinterpret_cast<const unsigned*>(slot_words(run[0]->set, run[0]->index)),
                           (int32_t)W, on_comm ? cs.stream() : A());
    }
    void folded(const P&) {}
    void join() {
        CBN_HIP_OK(hipEventRecord(tail, cs.stream()));
        CBN_HIP_OK(hipStreamWaitEvent(A(), tail, 0));
    }
};

using fold_fn = int (*)(void*, int64_t, const float* const*, int32_t, unsigned*, float*, float*, int64_t,
                        const unsigned*, int32_t, int32_t, hipStream_t);

// distributed.ShardedStepper's rank-local step with folded scales (no gather)
class FoldStepper {
  public:
    FoldStepper(uintptr_t fold_addr, uintptr_t scale_batch_addr, uintptr_t plan, py::tuple slots, py::object first,
                int64_t device_index, int64_t n_samples, bool target_observed, int64_t n_words, int group,
                uintptr_t comm)
        : fold_(reinterpret_cast<fold_fn>(fold_addr)), plan_(reinterpret_cast<void*>(plan)), slots_(slots),
          first_(first), dev_(device_index), n_samples_(n_samples), target_observed_(target_observed),
          ring_(FoldHipOps(reinterpret_cast<scale_batch_fn>(scale_batch_addr), reinterpret_cast<ncclComm_t>(comm),
                           device_index, n_words, group < 1 ? 1 : (group > kFoldGroupMax ? kFoldGroupMax : group)),
                group) {}

    // this step's rows (final after wait()); None when a fast check failed (the
    // caller converts the evidence and retries); an int: the C ABI's error code
    py::object step(py::dict evidence, py::object out_obj, int32_t flags) {
        Cols c;
        int64_t n = 0;
        if (!gather_cols(evidence, c, n)) return py::none();
        FoldHipOps& ops = ring_.ops();
        FoldItem item{check_out(out_obj, n, n_samples_, dev_)};
        at::Tensor ret = item.rows;
        float* rows = static_cast<float*>(item.rows.data_ptr());
        int launch_rc = 0;
        const int rc = ring_.step(
            [&](Slot s, const FoldPending<FoldItem>* f, bool& consumed) -> int {
                int* w = ops.slot_words(s.half, s.index);
                if (n > 0) {
                    float* fr = f ? static_cast<float*>(f->item.rows.data_ptr()) : nullptr;
                    const int64_t fn = f ? f->item.rows.numel() : 0;
                    launch_rc = fold_(plan_, n, c.p, (int32_t)PyTuple_GET_SIZE(slots_.ptr()),
                                      reinterpret_cast<unsigned*>(w), rows, fn > 0 ? fr : nullptr, fn,
                                      f ? reinterpret_cast<const unsigned*>(ops.slot_words(f->set, f->index))
                                        : nullptr,
                                      (int32_t)ops.W, flags, ops.A());
                    if (!launch_rc) {
                        consumed = f != nullptr;
                        return 0;
                    }
                }
                // empty shard, or a launch the library refused: zero words; the
                // step still joins its group's all-reduce (paired collectives)
                CBN_HIP_OK(hipMemsetAsync(w, 0, sizeof(int) * ops.W, ops.A()));
                return 0;
            },
            std::move(item));
        if (rc) return py::int_(rc);
        if (launch_rc) return py::int_(launch_rc);
        return py::cast(ret);
    }
    void wait() { check_(ring_.wait()); }
    void synchronize() {
        check_(ring_.wait());
        py::gil_scoped_release nogil;
        CBN_HIP_OK(hipStreamSynchronize(ring_.ops().A()));
    }
    int64_t steps() const { return ring_.steps(); }
    int group() const { return ring_.group(); }
    int unfinished() const { return ring_.unfinished(); }

  private:
    bool gather_cols(py::dict& evidence, Cols& c, int64_t& n) {
        if (empty_shard(evidence, slots_, first_)) {
            n = 0;
            return true;
        }
        if (!gather(evidence, slots_, first_, dev_, target_observed_, c)) return false;
        n = c.n;
        return true;
    }
    static void check_(int rc) {
        if (rc) throw std::runtime_error("cbn_scale_batch failed (rc=" + std::to_string(rc) + ")");
    }
    fold_fn fold_;
    void* plan_;
    py::tuple slots_;
    py::object first_;
    int64_t dev_, n_samples_;
    bool target_observed_;
    FoldRing<FoldHipOps> ring_;
};

// ---- CPU test double of the folded ring: Python callbacks
//   launch(set, index, payload, fold_payload or None, fold_set, fold_index) -> consumed (bool)
//   exchange(set, n), scale([(payload, set, index), ...], on_comm), wait_set(set),
//   mark_set(set, on_comm), record(set), passed(set, block) -> bool, handoff(set), join()
struct PyFoldOps {
    using Item = py::object;
    using P = FoldPending<py::object>;
    py::object cb;
    void wait_set(int set) { cb.attr("wait_set")(set); }
    void mark_set(int set, bool on_comm) { cb.attr("mark_set")(set, on_comm); }
    void record(int set) { cb.attr("record")(set); }
    bool passed(int set, bool block) { return cb.attr("passed")(set, block).cast<bool>(); }
    void handoff(int set) { cb.attr("handoff")(set); }
    int exchange(int set, int nb) { return cb.attr("exchange")(set, nb).cast<int>(); }
    int scale(const std::vector<const P*>& run, bool on_comm) {
        py::list l;
        for (auto* p : run) l.append(py::make_tuple(p->item, p->set, p->index));
        return cb.attr("scale")(l, on_comm).cast<int>();
    }
    void folded(const P&) {}
    void join() { cb.attr("join")(); }
};

class CpuFoldRing {
  public:
    CpuFoldRing(py::object cb, int group) : ring_(PyFoldOps{cb}, group) {}
    int step(py::object payload) {
        py::object cb = ring_.ops().cb;
        return ring_.step(
            [&](Slot s, const FoldPending<py::object>* f, bool& consumed) -> int {
                consumed = cb.attr("launch")(s.half, s.index, payload, f ? f->item : py::none(), f ? f->set : -1,
                                             f ? f->index : -1)
                               .cast<bool>() &&
                           f != nullptr;
                return 0;
            },
            payload);
    }
    int wait() { return ring_.wait(); }
    int unfinished() const { return ring_.unfinished(); }
    int group() const { return ring_.group(); }

  private:
    FoldRing<PyFoldOps> ring_;
};

// ------------------------------------------------------ redrawn sample domains --
// A plan whose sample domains are redrawn on every call (N > |domain|: the
// reference pads the domain with random.uniform draws and sorts, node.py:
// 302-333) keeps its device plan; per call only its sample-index arrays
// change.  This computes all of them from the call's uniforms in one host
// call.  Job j (one sample_domain call, in the reference's order) takes the
// next need_j values of r, forms lo_j + span_j * float(r) in float32 (what
// random.uniform does on the 0-dim float32 tensors of Node.info), sorts them
// together with the variable's domain (torch.sort of the concatenation) and
// writes the index of every point in the estimator's domain (-1: absent;
// the BruteForce lookup is by value) to idx[dest_j .. dest_j + N); the
// target's points also go to pts.
//   meta  int64 [J, 7]: need, sdom_off, sdom_len, ldom_off, ldom_len, dest (-1: none), want_pts
//   lospan float32 [J, 2]; doms float32 (flat sample / lookup domains, sorted)
void redraw(py::list r, const at::Tensor& meta, const at::Tensor& lospan, const at::Tensor& doms, at::Tensor idx,
            at::Tensor pts, int64_t N) {
    if (meta.scalar_type() != at::kLong || lospan.scalar_type() != at::kFloat || doms.scalar_type() != at::kFloat ||
        idx.scalar_type() != at::kInt || !meta.is_contiguous() || !lospan.is_contiguous() || !idx.is_contiguous() ||
        meta.dim() != 2 || meta.size(1) != 7 || lospan.size(0) != meta.size(0) || meta.is_cuda() || idx.is_cuda())
        throw std::invalid_argument("redraw: bad job tables");
    const int64_t J = meta.size(0), R = (int64_t)py::len(r);
    const int64_t* m = meta.data_ptr<int64_t>();
    const float* ls = lospan.data_ptr<float>();
    const float* dm = doms.data_ptr<float>();
    int32_t* out = idx.data_ptr<int32_t>();
    const int64_t nidx = idx.numel(), ndoms = doms.numel();
    std::vector<float> p;
    int64_t k = 0;
    for (int64_t j = 0; j < J; ++j, m += 7) {
        const int64_t need = m[0], soff = m[1], slen = m[2], loff = m[3], llen = m[4], dest = m[5];
        if (need < 0 || k + need > R || soff < 0 || soff + slen > ndoms || loff < 0 || loff + llen > ndoms ||
            slen + need != N || (dest >= 0 && dest + N > nidx))
            throw std::invalid_argument("redraw: job " + std::to_string(j) + " out of range");
        p.assign(dm + soff, dm + soff + slen);
        const float lo = ls[2 * j], span = ls[2 * j + 1];
        for (int64_t i = 0; i < need; ++i) {
            const float u = (float)PyFloat_AsDouble(PyList_GET_ITEM(r.ptr(), k + i));  // .to(float32): nearest
            const float t = span * u;  // two rounded float32 operations, as torch does them
            p.push_back(lo + t);
        }
        k += need;
        if (PyErr_Occurred()) throw py::error_already_set();
        if (dest < 0 && !m[6]) continue;  // bayesian_network.py:265-267: drawn for its shape only
        // torch.sort: ascending, NaN last
        std::sort(p.begin(), p.end(), [](float a, float b) { return std::isnan(b) ? !std::isnan(a) : a < b; });
        if (m[6]) {
            if (pts.numel() != N || pts.scalar_type() != at::kFloat || pts.is_cuda())
                throw std::invalid_argument("redraw: pts must be a host float32 [N] tensor");
            std::memcpy(pts.data_ptr<float>(), p.data(), sizeof(float) * N);
        }
        if (dest < 0) continue;
        const float* ld = dm + loff;
        for (int64_t i = 0; i < N; ++i) {
            const float v = p[i];
            const float* it = std::lower_bound(ld, ld + llen, v);
            out[dest + i] = (it != ld + llen && *it == v) ? (int32_t)(it - ld) : -1;
        }
    }
    if (k != R) throw std::invalid_argument("redraw: " + std::to_string(R - k) + " uniforms left over");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.def("redraw", &redraw);
    m.doc() = "cbn MI355X host fast path (cached-plan infer)";
    m.def("run", &run);
    m.def("scale", &scale);
    m.def("nccl_unique_id", &nccl_unique_id);
    m.def("nccl_comm_init", &nccl_comm_init);
    m.def("nccl_comm_destroy", &nccl_comm_destroy);
    m.def("nccl_comm_count", &nccl_comm_count);
    py::class_<Runner>(m, "Runner")
        .def(py::init<uintptr_t, uintptr_t, py::tuple, py::tuple, int64_t, int64_t, bool, uintptr_t, int32_t,
                      py::object>())
        .def("__call__", &Runner::call, py::arg("evidence"), py::arg("out") = py::none());
    py::class_<Stepper>(m, "Stepper")
        .def(py::init<uintptr_t, uintptr_t, uintptr_t, py::tuple, py::object, int64_t, int64_t, bool, int64_t, int,
                      uintptr_t, int, int>())
        .def("step", &Stepper::step)
        .def("wait", &Stepper::wait)
        .def("synchronize", &Stepper::synchronize)
        .def("comm_stream", &Stepper::comm_stream)
        .def("steps", &Stepper::steps)
        .def("group", &Stepper::group)
        .def("host_timing", &Stepper::host_timing);
    py::class_<FoldStepper>(m, "FoldStepper")
        .def(py::init<uintptr_t, uintptr_t, uintptr_t, py::tuple, py::object, int64_t, int64_t, bool, int64_t, int,
                      uintptr_t>())
        .def("step", &FoldStepper::step)
        .def("wait", &FoldStepper::wait)
        .def("synchronize", &FoldStepper::synchronize)
        .def("steps", &FoldStepper::steps)
        .def("group", &FoldStepper::group)
        .def("unfinished", &FoldStepper::unfinished);
    py::class_<CpuFoldRing>(m, "CpuFoldRing")
        .def(py::init<py::object, int>())
        .def("step", &CpuFoldRing::step)
        .def("wait", &CpuFoldRing::wait)
        .def("unfinished", &CpuFoldRing::unfinished)
        .def("group", &CpuFoldRing::group);
    py::class_<CpuStepRing>(m, "CpuStepRing")
        .def(py::init<py::object, int>())
        .def("step", &CpuStepRing::step)
        .def("wait", &CpuStepRing::wait)
        .def("flush", &CpuStepRing::flush)
        .def("pending", &CpuStepRing::pending)
        .def("group", &CpuStepRing::group);
}
