// nf4_torch_ext.cpp -- tensor-level fast entry of the drop-in API (host code only).
//
// triton_dequantize_nf4(module) (reference kernel_optimized.py:113-139) costs one
// Python call per weight; the reference harness issues three per step on three
// streams (benchmark.py:68-84).  Through ctypes the host side of that call was
// 7-10 us, above the 7 us the 4096^2 kernel itself takes.  This module takes the
// three tensors the attribute reads produce and does the rest in C++: type /
// contiguity / device checks, the output allocation on the caching allocator,
// the current HIP stream of the weight's device, and the C-ABI call
// (nf4_dequant_ref, include/nf4_dequant.h).  It returns None whenever the inputs
// need the general path (casts, strided views, another device, empty absmax),
// which kernel.py then takes -- same kernels, same results; there is no CPU
// compute here.
#include <torch/extension.h>

#include <ATen/hip/EmptyTensor.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPFunctions.h>

#include "../../include/nf4_dequant.h"

namespace py = pybind11;

namespace {

c10::ScalarType out_type(int code) {
    switch (code) {
        case NF4DQ_F16: return at::kHalf;
        case NF4DQ_BF16: return at::kBFloat16;
        default: return at::kFloat;
    }
}

// The fast path of kernel._dequantize: uint8 packed / uint8 absmax / fp32 nested
// absmax, all contiguous and on one ROCm device.
py::object dequant_ref(const at::Tensor& q, const at::Tensor& a1, const at::Tensor& a2, int64_t m, int64_t n,
                       int code) {
    if (!q.is_cuda() || q.scalar_type() != at::kByte || a1.scalar_type() != at::kByte ||
        a2.scalar_type() != at::kFloat || !q.is_contiguous() || !a1.is_contiguous() || !a2.is_contiguous() ||
        a1.device() != q.device() || a2.device() != q.device() || a1.numel() == 0 || a2.numel() == 0 || m <= 0 ||
        n <= 0 || code < NF4DQ_F16 || code > NF4DQ_F32)
        return py::none();
    const c10::Device dev = q.device();
    // a guard only when the weight is not on the current device (the common case
    // skips the get/set-device pair)
    std::optional<c10::DeviceGuard> guard;
    if (dev.index() != c10::hip::current_device()) guard.emplace(dev);
    // the caching allocator directly (at::detail::empty_cuda), not through the
    // dispatcher: the output allocation is the largest host cost of the call
    const int64_t size[2] = {m, n};
    at::Tensor out(at::detail::empty_cuda(at::IntArrayRef(size, 2), out_type(code), dev, std::nullopt));
    hipStream_t st = c10::hip::getCurrentHIPStream(dev.index()).stream();
    const int rc = nf4_dequant_ref(q.data_ptr<uint8_t>(), q.numel(), a1.data_ptr<uint8_t>(), a1.numel(),
                                   a2.data_ptr<float>(), a2.numel(), out.data_ptr(), code, m, n, st);
    if (rc != NF4DQ_OK)
        throw std::runtime_error(std::string("nf4 dequantize failed: ") + nf4_strerror(rc) + " (code " +
                                 std::to_string(rc) + ")");
    return py::cast(out);
}

}  // namespace

PYBIND11_MODULE(nf4ext, mod) {
    mod.doc() = "tensor-level fast entry of triton_dequantize_nf4 (calls libnf4dq.so's C ABI)";
    mod.def("dequant_ref", &dequant_ref, "uint8/uint8/fp32 contiguous device tensors -> new [m, n] tensor, or None",
            py::arg("packed"), py::arg("absmax"), py::arg("absmax2"), py::arg("m"), py::arg("n"), py::arg("code"));
}
