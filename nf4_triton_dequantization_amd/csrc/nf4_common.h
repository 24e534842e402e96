// nf4_common.h -- device helpers shared by the dequant (nf4_dequant.hip) and
// fused dequant-GEMM (nf4_gemm.hip) kernels of libnf4dq.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nf4_dequant.h"

namespace nf4dq {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Division by a run-time constant for n < 2^31: q = (umulhi(n, mul) + n) >> shift.
struct FastDiv {
    uint32_t d, mul, shift;
};

inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f{d, 0u, 0u};
    uint32_t s = 0;
    while (s < 32 && (uint64_t(1) << s) < d) ++s;
    f.shift = s;
    f.mul = uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << s) - d)) / d + 1);
    return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    return (__umulhi(n, f.mul) + n) >> f.shift;
}
__device__ __forceinline__ uint32_t fmodu(uint32_t n, const FastDiv& f) {
    return n - fdiv(n, f) * f.d;
}

// Keep an fp32 product opaque to the backend: without this, hipcc folds
// fptrunc(fmul) into v_fma_mix*_f16(a, b, +0), which rounds once instead of
// twice (fp32 product, then fp16 -- the reference's order) and turns -0 into +0.
__device__ __forceinline__ float opaque(float x) {
    asm volatile("" : "+v"(x));
    return x;
}

// The pair as one opaque 64-bit value (non-volatile: the scheduler may still
// move it; the products stay one v_pk_mul_f32).
__device__ __forceinline__ f32x2 opaque2(f32x2 v) {
    asm("" : "+v"(v));
    return v;
}

template <int DT>
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
    f32x2 v = {lo, hi};
    if constexpr (DT == NF4DQ_F16) v = opaque2(v);
    if constexpr (DT == NF4DQ_BF16) {
        return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
    } else {
        return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2));
    }
}

// The 16 NF4 code points: fp32 bit patterns of kernel_optimized.py:234-239.
constexpr uint32_t kNf4Bits[16] = {0xbf800000u, 0xbf3239b1u, 0xbf066b30u, 0xbeca32a0u, 0xbe91a24du, 0xbe3d353fu,
                                   0xbdba7871u, 0x00000000u, 0x3da2faffu, 0x3e24cae3u, 0x3e7c04ddu, 0x3ead033au,
                                   0x3ee1a4b8u, 0x3f1007abu, 0x3f3913b3u, 0x3f800000u};

// The code table into LDS from immediates (no global load on the kernel's
// critical path): thread 0 writes four 16-byte rows.
__device__ __forceinline__ void write_lut(float* lut) {
    if (threadIdx.x == 0) {
        u32x4* l4 = reinterpret_cast<u32x4*>(lut);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            l4[r] = u32x4{kNf4Bits[4 * r], kNf4Bits[4 * r + 1], kNf4Bits[4 * r + 2], kNf4Bits[4 * r + 3]};
    }
}

// Code point i: a constant for constant i, a select chain otherwise.
__device__ __forceinline__ float nf4_code(uint32_t i) {
    uint32_t v = kNf4Bits[0];
#pragma unroll
    for (uint32_t j = 1; j < 16; ++j) v = i == j ? kNf4Bits[j] : v;
    return __uint_as_float(v);
}

// Buffer-resource flags word (raw buffer, dword format) for gfx950.
constexpr int kRsrcFlags = 0x00020000;

}  // namespace nf4dq
