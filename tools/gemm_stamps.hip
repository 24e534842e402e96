// Diagnostic build of the fused-GEMM kernels with per-wave phase stamps (tools only).
//
// Defines the NF4_GSTAMP* hooks of nf4_gemm.hip and includes it: lane 0 of every
// wave writes s_memrealtime (100 MHz) at each hook into a buffer of its own,
// [workgroup][wave][16] u64, set by nf4_dbg_set_gemm_stamps() -- never into an
// output or the workspace.  Slots (see the hooks in nf4_gemm.hip): 0 entry,
// 1 prologue barrier passed, 2 first strip / chunk consumed, 3 strip loop done,
// 4 final barrier passed, 5 results stored (slab: drained), 6 tickets drawn (the
// reducing wave only), 7 summed time in the partial-tile stores + barrier,
// 8 summed time in the reducer's sums, 9 exit, 10-12 prologue steps (register-resident
// kernel: 11 x issued, 10 ring issued, 12 tables written), 14 HW_ID, 15 XCC_ID.
// Built into tools/_build/libnf4dq_gstamps.so with the product's dequant and
// host objects (tools/Makefile `gstamps`); read by tools/gemm_stamps.py.
#include <hip/hip_runtime.h>

__device__ unsigned long long* g_nf4_gstamps;

__device__ __forceinline__ unsigned long long nf4_gs_now() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

#define NF4_GSTAMP_INIT(waves_)                                                                   \
    const uint32_t nf4_gs_base = (blockIdx.x * (uint32_t)(waves_) + (threadIdx.x >> 6)) * 16u;  \
    unsigned long long nf4_gs_t0 = 0;                                                             \
    do {                                                                                          \
        if ((threadIdx.x & 63u) == 0) {                                                           \
            uint32_t hw_, xcc_;                                                                   \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                     \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                   \
            g_nf4_gstamps[nf4_gs_base + 14u] = hw_;                                               \
            g_nf4_gstamps[nf4_gs_base + 15u] = xcc_;                                              \
            g_nf4_gstamps[nf4_gs_base + 7u] = 0ull;                                               \
            g_nf4_gstamps[nf4_gs_base + 8u] = 0ull;                                               \
        }                                                                                         \
    } while (0)

#define NF4_GSTAMP(slot_)                                                                 \
    do {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                \
        const unsigned long long t_ = nf4_gs_now();                                       \
        if ((threadIdx.x & 63u) == 0) g_nf4_gstamps[nf4_gs_base + (slot_)] = t_;          \
        __builtin_amdgcn_sched_barrier(0);                                                \
    } while (0)

#define NF4_GSPAN_BEGIN()                  \
    do {                                   \
        __builtin_amdgcn_sched_barrier(0); \
        nf4_gs_t0 = nf4_gs_now();          \
        __builtin_amdgcn_sched_barrier(0); \
    } while (0)

#define NF4_GSPAN_END(slot_)                                                                              \
    do {                                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                                \
        const unsigned long long t_ = nf4_gs_now();                                                       \
        if ((threadIdx.x & 63u) == 0) g_nf4_gstamps[nf4_gs_base + (slot_)] += t_ - nf4_gs_t0;             \
        __builtin_amdgcn_sched_barrier(0);                                                                \
    } while (0)

// ablation hooks (none unless -DABL_<part>: the gstamps_<part> builds)
#include "gemm_ablate_hooks.h"
// the product's fused-GEMM sources, all in this one translation unit
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_k128.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_persist.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_stream.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_xr.hip"
#include "../nf4_triton_dequantization_amd/csrc/nf4_gemm_launch_xs.hip"

extern "C" int nf4_dbg_set_gemm_stamps(void* buf) {
    unsigned long long* p = reinterpret_cast<unsigned long long*>(buf);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_nf4_gstamps), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
