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

#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <vector>

namespace {

using run_fn = int (*)(void*, int64_t, const float* const*, int32_t, unsigned*, float*, int32_t, hipStream_t);

// Returns the output tensor; None when a fast check failed (the caller takes
// the slow path); an int = the C ABI's (negative) error code (the caller
// raises with cbn_last_error()).
py::object run(uintptr_t fn, uintptr_t plan, py::dict evidence, py::tuple slots, py::object first,
               int64_t device_index, int64_t n_samples, bool target_observed, uintptr_t max_ptr, int32_t flags,
               py::object out_obj) {
    const Py_ssize_t ns = PyTuple_GET_SIZE(slots.ptr());
    int64_t n = 1;
    if (!first.is_none()) {
        PyObject* f = PyDict_GetItem(evidence.ptr(), first.ptr());
        if (!f || !THPVariable_Check(f)) return py::none();
        const at::Tensor& t = THPVariable_Unpack(f);
        if (t.dim() < 1) return py::none();
        n = t.size(0);
    }
    if (n == 0 || (!target_observed && n != 1)) return py::none();
    const float* cols_small[64];
    std::vector<const float*> cols_big;
    const float** cols = cols_small;
    if (ns > 64) {
        cols_big.resize(ns);
        cols = cols_big.data();
    }
    for (Py_ssize_t i = 0; i < ns; ++i) {
        PyObject* v = PyDict_GetItem(evidence.ptr(), PyTuple_GET_ITEM(slots.ptr(), i));
        if (!v || !THPVariable_Check(v)) return py::none();
        const at::Tensor& t = THPVariable_Unpack(v);
        if (t.scalar_type() != at::kFloat || !t.is_cuda() || t.get_device() != device_index || t.dim() != 2 ||
            t.size(0) != n || !t.is_contiguous())
            return py::none();
        cols[i] = static_cast<const float*>(t.data_ptr());
    }
    if (c10::hip::current_device() != device_index) return py::none();
    at::Tensor out;
    if (out_obj.is_none()) {
        out = at::empty({n, n_samples}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_index));
    } else {
        out = THPVariable_Unpack(out_obj.ptr());
    }
    const hipStream_t s = c10::hip::getCurrentHIPStream(device_index).stream();
    const int rc = reinterpret_cast<run_fn>(fn)(reinterpret_cast<void*>(plan), n, cols, (int32_t)ns,
                                                reinterpret_cast<unsigned*>(max_ptr),
                                                static_cast<float*>(out.data_ptr()), flags, s);
    if (rc) return py::int_(rc);
    return py::cast(out);
}

using scale_fn = int (*)(float*, int64_t, const unsigned*, int32_t, hipStream_t);

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
}
