// nf4_gemm_launch_xr.hip -- launcher of the register-resident kernels (nf4_gemm_xr_kernel / nf4_gemm_xrg_kernel) (instantiates its kernels;
// compiled on its own so that the kernel families build in parallel).
#include "nf4_gemm_plan.h"

namespace nf4gemm {

int launch_xr(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
                     const nf4_gemm_cfg& cfg, void* workspace, hipStream_t st) {
    const uint32_t ks = (uint32_t)cfg.ksplit;
    GemmArgs A{};
    A.nmat = (uint32_t)count;
    A.x = x;
    A.counters = reinterpret_cast<uint32_t*>(workspace);
    A.slab = ks > 1 ? reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(workspace) + kHeaderBytes) : nullptr;
    A.M = (uint32_t)M;
    A.K = (uint32_t)K;
    A.ksplit = ks;
    A.chunks = (uint32_t)(K / kChunkK);
    A.chunks_per_split = (uint32_t)(cfg.waves * cfg.strips);
    A.bpr = (uint32_t)(K / 64);
    A.groups = (A.bpr + 3) / 4;
    uint32_t strips = 0;
    for (int i = 0; i < count; ++i) {
        const HostMat& h = mats[i];
        K128Mat& m = A.mat[i];
        m.packed = h.packed;
        m.a1 = h.a1;
        m.a2 = h.a2;
        m.y = h.y;
        m.N = (uint32_t)h.N;
        m.cg_begin = strips;        // first 16-column strip of the weight in the launch
        m.col_begin = strips * 16u;
        m.nb = make_fastdiv((uint32_t)(h.nb > (int64_t(1) << 31) ? (int64_t(1) << 31) : h.nb));
        m.n2 = make_fastdiv((uint32_t)(h.n2 > (int64_t(1) << 29) ? (int64_t(1) << 29) : h.n2));
        strips += (uint32_t)(h.N / 16);
    }
    A.col_groups = strips;
    A.ncols = strips * 16u;
    A.per_wg = xr_per_wg(M, strips, cfg);
    const uint32_t groups = (strips + A.per_wg - 1) / A.per_wg;
    const dim3 grid(groups * ks), block(64 * cfg.waves);
    const uint32_t lds = xr_lds_dynamic(M, cfg.waves, A.per_wg);
#define NF4_R2(DT_, MT_, W_, KPW_, D_, GU_)                                                                          \
    do {                                                                                                             \
        static bool attr_ = false; /* dynamic LDS above 64 KiB needs the opt-in */                                   \
        if (!attr_) {                                                                                                \
            (void)hipFuncSetAttribute(                                                                               \
                GU_ ? reinterpret_cast<const void*>(&nf4_gemm_xrg_kernel<DT_, MT_, W_, KPW_, D_, GU_>)               \
                    : reinterpret_cast<const void*>(&nf4_gemm_xr_kernel<DT_, MT_, W_, KPW_, D_, GU_>),               \
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsPerCu - xr_lds_static(KPW_)));                 \
            attr_ = true;                                                                                            \
        }                                                                                                            \
        if (GU_) hipLaunchKernelGGL((nf4_gemm_xrg_kernel<DT_, MT_, W_, KPW_, D_, GU_>), grid, block, lds, st, A);    \
        else hipLaunchKernelGGL((nf4_gemm_xr_kernel<DT_, MT_, W_, KPW_, D_, GU_>), grid, block, lds, st, A);         \
    } while (0)
    // two K slices of 8 waves x 256-deep chunks with at most 4 or 8 reduction groups
    // (8 or 16 strips) per workgroup: the groups unrolled, exchanges issued inside the loop
#define NF4_R1(DT_, MT_, W_, KPW_, D_)                                                   \
    do {                                                                                 \
        if constexpr (W_ == 8 && KPW_ == 2 && D_ == 2) {                                 \
            if (ks == 2 && A.per_wg <= 8) NF4_R2(DT_, MT_, W_, KPW_, D_, 4);             \
            else if (ks == 2 && A.per_wg <= 16) NF4_R2(DT_, MT_, W_, KPW_, D_, 8);       \
            else NF4_R2(DT_, MT_, W_, KPW_, D_, 0);                                      \
        } else {                                                                         \
            NF4_R2(DT_, MT_, W_, KPW_, D_, 0);                                           \
        }                                                                                \
    } while (0)
#define NF4_RD(DT_, MT_, W_, KPW_)                         \
    do {                                                   \
        if (cfg.depth == 4) NF4_R1(DT_, MT_, W_, KPW_, 4); \
        else NF4_R1(DT_, MT_, W_, KPW_, 2);                \
    } while (0)
#define NF4_RK(DT_, MT_, W_)                          \
    do {                                              \
        if (cfg.strips == 2) NF4_RD(DT_, MT_, W_, 2); \
        else NF4_RD(DT_, MT_, W_, 1);                 \
    } while (0)
#define NF4_RW(DT_, MT_)                                \
    do {                                                \
        if (cfg.strips == 4) NF4_RD(DT_, MT_, 8, 4);    \
        else if (cfg.waves == 16) NF4_RK(DT_, MT_, 16); \
        else NF4_RK(DT_, MT_, 8);                       \
    } while (0)
#define NF4_RM(DT_)                 \
    do {                            \
        if (M > 16) NF4_RW(DT_, 2); \
        else NF4_RW(DT_, 1);        \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_RM(NF4DQ_BF16);
    else NF4_RM(NF4DQ_F16);
#undef NF4_RM
#undef NF4_RW
#undef NF4_RK
#undef NF4_RD
#undef NF4_R1
#undef NF4_R2
    return hip_rc2(hipGetLastError());
}

}  // namespace nf4gemm
