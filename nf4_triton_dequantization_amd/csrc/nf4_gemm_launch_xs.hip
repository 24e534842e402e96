// nf4_gemm_launch_xs.hip -- launcher of the shared-activation kernel (nf4_gemm_xs_kernel) (instantiates its kernels;
// compiled on its own so that the kernel families build in parallel).
#include "nf4_gemm_plan.h"

namespace nf4gemm {

// One launch of the shared-activation kernel over `count` weights sharing x (shapes
// and cfg validated: cfg.depth = KC chunks per slice, cfg.ksplit = ceil(chunks / KC)).
int launch_xs(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
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
    A.chunks_per_split = (uint32_t)cfg.depth;
    A.bpr = (uint32_t)(K / 64);
    A.groups = (A.bpr + 3) / 4;
    const uint32_t cols_per_group = 16u * (uint32_t)cfg.waves;
    uint32_t cgs = 0, cols = 0;
    for (int i = 0; i < count; ++i) {
        const HostMat& h = mats[i];
        K128Mat& m = A.mat[i];
        m.packed = h.packed;
        m.a1 = h.a1;
        m.a2 = h.a2;
        m.y = h.y;
        m.N = (uint32_t)h.N;
        m.cg_begin = cgs;
        m.col_begin = cols;
        m.nb = make_fastdiv((uint32_t)(h.nb > (int64_t(1) << 31) ? (int64_t(1) << 31) : h.nb));
        m.n2 = make_fastdiv((uint32_t)(h.n2 > (int64_t(1) << 31) ? (int64_t(1) << 31) : h.n2));
        cgs += ((uint32_t)h.N + cols_per_group - 1u) / cols_per_group;
        cols += (uint32_t)h.N;
    }
    A.col_groups = cgs;
    A.ncols = cols;
    const dim3 grid(cgs * ks), block(64 * cfg.waves);
    const uint32_t lds = xs_lds_bytes(M, cfg.depth, cfg.waves);
#define NF4_X1(DT_, MT_, KC_, W_)                                                                                   \
    do {                                                                                                            \
        static bool attr_ = false; /* dynamic LDS above 64 KiB needs the opt-in */                                  \
        if (!attr_) {                                                                                               \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&nf4_gemm_xs_kernel<DT_, MT_, KC_, W_>),        \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCu);                  \
            attr_ = true;                                                                                           \
        }                                                                                                           \
        hipLaunchKernelGGL((nf4_gemm_xs_kernel<DT_, MT_, KC_, W_>), grid, block, lds, st, A);                       \
    } while (0)
#define NF4_XW(DT_, MT_, KC_)                          \
    do {                                               \
        if (cfg.waves == 8) NF4_X1(DT_, MT_, KC_, 8);  \
        else NF4_X1(DT_, MT_, KC_, 4);                 \
    } while (0)
#define NF4_XK(DT_, MT_)                              \
    do {                                              \
        if (cfg.depth == 8) NF4_XW(DT_, MT_, 8);      \
        else if (cfg.depth == 4) NF4_XW(DT_, MT_, 4); \
        else NF4_XW(DT_, MT_, 2);                     \
    } while (0)
#define NF4_XM(DT_)                        \
    do {                                   \
        if (M > 16) NF4_XK(DT_, 2);        \
        else NF4_XK(DT_, 1);               \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_XM(NF4DQ_BF16);
    else NF4_XM(NF4DQ_F16);
#undef NF4_XM
#undef NF4_XK
#undef NF4_XW
#undef NF4_X1
    return hip_rc2(hipGetLastError());
}

}  // namespace nf4gemm
