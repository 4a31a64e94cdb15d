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

#include <array>
#include <chrono>

#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

using run_fn = int (*)(void*, int64_t, const float* const*, int32_t, unsigned*, float*, int32_t, hipStream_t);

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
        if (t.scalar_type() != at::kFloat || !t.is_cuda() || t.get_device() != device_index || t.dim() != 2 ||
            t.size(0) != n || !t.is_contiguous())
            return false;
        c.p[i] = static_cast<const float*>(t.data_ptr());
    }
    if (c10::hip::current_device() != device_index) return false;
    c.n = n;
    return true;
}

py::object run(uintptr_t fn, uintptr_t plan, py::dict evidence, py::tuple slots, py::object first,
               int64_t device_index, int64_t n_samples, bool target_observed, uintptr_t max_ptr, int32_t flags,
               py::object out_obj) {
    Cols c;
    if (!gather(evidence, slots, first, device_index, target_observed, c)) return py::none();
    at::Tensor out = out_obj.is_none() ? at::empty({c.n, n_samples},
                                                   at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_index))
                                       : THPVariable_Unpack(out_obj.ptr());
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

void nccl_comm_destroy(uintptr_t comm) {
    if (comm && g_rccl.comm_destroy) CBN_NCCL_OK(g_rccl.comm_destroy(reinterpret_cast<ncclComm_t>(comm)));
}

// ------------------------------------------------------- pipelined stepper --
// distributed.ShardedStepper's per-step work in one host call (the Python
// version -- events, stream switch, c10d all_reduce, record_stream -- cost
// ~50 us of host time per step, 4x the GPU time of a 65k-query raw launch).
// Steps are exchanged in groups of G:
//   compute stream A: raw launch of each step -> its words slot
//   comm stream C:    after the group's G-th raw launch (ready event), ONE
//                     ncclAllReduce(MAX) over the group's G x W words and ONE
//                     cbn_scale_batch launch dividing each step's rows by its max
// so the per-exchange host costs (event record + cross-stream wait ~5.5 us,
// scale launch ~4.3 us, measured on MI355X by host_timing()) are paid once
// per G steps.  Word slots form a ring of two groups; A waits for C only when
// it starts a group whose slots the exchange two groups back still reads.
// Rows are recorded on C for the caching allocator.  flush() (wait(),
// synchronize()) exchanges a partial group.
class Stepper {
  public:
    Stepper(uintptr_t run_addr, uintptr_t scale_batch_addr, uintptr_t plan, py::tuple slots, py::object first,
            int64_t device_index, int64_t n_samples, bool target_observed, int64_t n_words, int group,
            uintptr_t comm)
        : run_(reinterpret_cast<run_fn>(run_addr)), scale_batch_(reinterpret_cast<scale_batch_fn>(scale_batch_addr)),
          plan_(reinterpret_cast<void*>(plan)), slots_(slots), first_(first), dev_(device_index),
          n_samples_(n_samples), target_observed_(target_observed), W_(n_words),
          G_(group < 1 ? 1 : (group > 8 ? 8 : group)), comm_(reinterpret_cast<ncclComm_t>(comm)),
          cs_(c10::hip::getStreamFromPool(/*isHighPriority=*/true, (c10::DeviceIndex)device_index)) {
        words_ = at::zeros({2 * G_, W_}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev_));
        CBN_HIP_OK(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
        for (auto& e : done_) CBN_HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        CBN_HIP_OK(hipEventCreateWithFlags(&tail_, hipEventDisableTiming));
    }
    ~Stepper() {
        (void)hipEventDestroy(ready_);
        for (auto e : done_) (void)hipEventDestroy(e);
        (void)hipEventDestroy(tail_);
    }

    // rows (final once this step's group has been exchanged and scaled on the
    // comm stream -- after wait()), None when a fast check failed, or an int
    // error code from the C ABI.
    py::object step(py::dict evidence, py::object out_obj, int32_t flags) {
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        Cols c;
        if (!gather(evidence, slots_, first_, dev_, target_observed_, c)) return py::none();
        const hipStream_t A = c10::hip::getCurrentHIPStream(dev_).stream();
        const int half = (int)(g_ & 1);
        if (pend_.empty() && used_[half]) CBN_HIP_OK(hipStreamWaitEvent(A, done_[half], 0));
        at::Tensor out = out_obj.is_none()
                             ? at::empty({c.n, n_samples_}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev_))
                             : THPVariable_Unpack(out_obj.ptr());
        int* w = words_.data_ptr<int>() + ((int64_t)half * G_ + (int64_t)pend_.size()) * W_;
        const auto t1 = clk::now();
        int rc = run_(plan_, c.n, c.p, (int32_t)PyTuple_GET_SIZE(slots_.ptr()), reinterpret_cast<unsigned*>(w),
                      static_cast<float*>(out.data_ptr()), flags, A);
        if (rc) return py::int_(rc);
        const auto t2 = clk::now();
        pend_.push_back(out);
        ++k_;
        if ((int)pend_.size() == G_) {
            rc = flush_();
            if (rc) return py::int_(rc);
        }
        py::object r = py::cast(out);
        const auto t3 = clk::now();
        tacc_[0] += std::chrono::duration<double, std::micro>(t1 - t0).count();
        tacc_[1] += std::chrono::duration<double, std::micro>(t2 - t1).count();
        tacc_[2] += std::chrono::duration<double, std::micro>(t3 - t2).count();
        ++tn_;
        return r;
    }

    // exchange + scale the pending partial group, then the current stream
    // waits for every enqueued exchange
    void wait() {
        check_(flush_());
        if (!k_) return;
        CBN_HIP_OK(hipEventRecord(tail_, cs_.stream()));
        CBN_HIP_OK(hipStreamWaitEvent(c10::hip::getCurrentHIPStream(dev_).stream(), tail_, 0));
    }
    void synchronize() {
        check_(flush_());
        CBN_HIP_OK(hipStreamSynchronize(cs_.stream()));
    }
    uintptr_t comm_stream() const { return reinterpret_cast<uintptr_t>(cs_.stream()); }
    int64_t steps() const { return k_; }
    int group() const { return G_; }

    // mean host microseconds per step: gather + alloc, raw launch, the
    // step's share of the group exchange (event, ncclAllReduce, scale) + return
    std::vector<double> host_timing() {
        std::vector<double> r(3, 0.0);
        for (int i = 0; i < 3; ++i) r[i] = tn_ ? tacc_[i] / tn_ : 0.0;
        tacc_.fill(0.0);
        tn_ = 0;
        return r;
    }

  private:
    int flush_() {
        if (pend_.empty()) return 0;
        const hipStream_t A = c10::hip::getCurrentHIPStream(dev_).stream();
        const hipStream_t C = cs_.stream();
        const int half = (int)(g_ & 1);
        const int nb = (int)pend_.size();
        int* w = words_.data_ptr<int>() + (int64_t)half * G_ * W_;
        CBN_HIP_OK(hipEventRecord(ready_, A));
        CBN_HIP_OK(hipStreamWaitEvent(C, ready_, 0));
        if (comm_) CBN_NCCL_OK(g_rccl.all_reduce(w, w, (size_t)nb * W_, ncclInt32, ncclMax, comm_, C));
        float* outs[8];
        int64_t ns[8];
        for (int b = 0; b < nb; ++b) {
            outs[b] = static_cast<float*>(pend_[b].data_ptr());
            ns[b] = pend_[b].numel();
        }
        const int rc = scale_batch_(outs, ns, nb, reinterpret_cast<const unsigned*>(w), (int32_t)W_, C);
        if (rc) return rc;
        CBN_HIP_OK(hipEventRecord(done_[half], C));
        used_[half] = true;
        for (auto& t : pend_) c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), cs_);
        pend_.clear();
        ++g_;
        return 0;
    }
    static void check_(int rc) {
        if (rc) throw std::runtime_error("cbn_scale_batch failed (rc=" + std::to_string(rc) + ")");
    }

    run_fn run_;
    scale_batch_fn scale_batch_;
    void* plan_;
    py::tuple slots_;
    py::object first_;
    int64_t dev_, n_samples_;
    bool target_observed_;
    int64_t W_;
    int G_;
    ncclComm_t comm_;
    c10::hip::HIPStream cs_;
    at::Tensor words_;
    std::vector<at::Tensor> pend_;
    hipEvent_t ready_ = nullptr, tail_ = nullptr;
    hipEvent_t done_[2] = {nullptr, nullptr};
    bool used_[2] = {false, false};
    int64_t k_ = 0, g_ = 0;
    std::array<double, 3> tacc_{};
    int64_t tn_ = 0;
};

// cbn_scale on the current stream of out's device (sharded path, after the
// cross-rank all-reduce of the per-block max words).
int scale(uintptr_t fn, const at::Tensor& out, uintptr_t max_ptr, int32_t n_max) {
    const hipStream_t s = c10::hip::getCurrentHIPStream(out.get_device()).stream();
    return reinterpret_cast<scale_fn>(fn)(static_cast<float*>(out.data_ptr()), out.numel(),
                                          reinterpret_cast<const unsigned*>(max_ptr), n_max, s);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.doc() = "cbn MI355X host fast path (cached-plan infer)";
    m.def("run", &run);
    m.def("scale", &scale);
    m.def("nccl_unique_id", &nccl_unique_id);
    m.def("nccl_comm_init", &nccl_comm_init);
    m.def("nccl_comm_destroy", &nccl_comm_destroy);
    py::class_<Stepper>(m, "Stepper")
        .def(py::init<uintptr_t, uintptr_t, uintptr_t, py::tuple, py::object, int64_t, int64_t, bool, int64_t, int,
                      uintptr_t>())
        .def("step", &Stepper::step)
        .def("wait", &Stepper::wait)
        .def("synchronize", &Stepper::synchronize)
        .def("comm_stream", &Stepper::comm_stream)
        .def("steps", &Stepper::steps)
        .def("group", &Stepper::group)
        .def("host_timing", &Stepper::host_timing);
}
