// nf4_gemm_launch_sk.hip -- launcher of the balanced kernel (nf4_gemm_sk_kernel) (instantiates its kernels;
// compiled on its own so that the kernel families build in parallel).
#include "nf4_gemm_plan.h"

namespace nf4gemm {

int launch_sk(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
                     const nf4_gemm_cfg& cfg, void* workspace, size_t workspace_bytes, hipStream_t st) {
    int64_t ncols = 0;
    for (int i = 0; i < count; ++i) ncols += mats[i].N;
    SkPlan p{};
    if (!sk_plan(M, K, ncols, cfg.waves, p)) return NF4DQ_ERR_ARG;
    if (p.slots > 1 && (!workspace || workspace_bytes < sk_workspace(M, K, ncols, cfg.waves) || !aligned16(workspace)))
        return NF4DQ_ERR_ARG;
    SkArgs A{};
    A.nmat = (uint32_t)count;
    A.x = x;
    A.counters = reinterpret_cast<uint32_t*>(workspace);
    A.slab = p.slots > 1 ? reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(workspace) + kHeaderBytes) : nullptr;
    A.xslab = A.slab ? A.slab + (size_t)p.slots * (size_t)M * (size_t)ncols / 2u : nullptr;
    A.M = (uint32_t)M;
    A.K = (uint32_t)K;
    A.C = make_fastdiv(p.C);
    A.ppr = make_fastdiv((uint32_t)(K / 8));
    A.U = (uint32_t)p.U;
    A.GW = p.GW;
    A.fGW = make_fastdiv(p.GW);
    A.fU = make_fastdiv((uint32_t)p.U);
    A.ncols = (uint32_t)ncols;
    A.bpr = (uint32_t)(K / 64);
    A.groups = (A.bpr + 3) / 4;
    A.xstride = p.xstride;
    A.zero_off = p.zero_off;
    uint32_t strips = 0;
    for (int i = 0; i < count; ++i) {
        const HostMat& h = mats[i];
        StreamMat& m = A.mat[i];
        m.packed = h.packed;
        m.a1 = h.a1;
        m.a2 = h.a2;
        m.y = h.y;
        m.N = (uint32_t)h.N;
        m.sg_begin = 0;
        m.strip_begin = strips;
        const int64_t nbc = h.nb > (int64_t(1) << 31) ? (int64_t(1) << 31) : h.nb;
        const int64_t n2c = h.n2 > (int64_t(1) << 29) ? (int64_t(1) << 29) : h.n2;
        m.nb = make_fastdiv((uint32_t)nbc);
        m.n2 = make_fastdiv((uint32_t)n2c);
        m.nb_bytes = (uint32_t)nbc;
        m.n2_bytes = (uint32_t)(n2c * 4);
        strips += (uint32_t)(h.N / 16);
    }
    const dim3 grid(p.G), block(64 * p.W);
#define NF4_SK2(DT_, LM_, D_)                                                                              \
    do {                                                                                                   \
        static bool attr_ = false; /* static + dynamic LDS above 64 KiB needs the opt-in */                \
        if (!attr_) {                                                                                      \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&nf4_gemm_sk_kernel<DT_, 8, LM_, D_>),    \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSkLdsCap);         \
            attr_ = true;                                                                                  \
        }                                                                                                  \
        hipLaunchKernelGGL((nf4_gemm_sk_kernel<DT_, 8, LM_, D_>), grid, block, p.lds, st, A);                 \
    } while (0)
#define NF4_SK1(DT_, LM_)                            \
    do {                                             \
        if (cfg.depth == 8) NF4_SK2(DT_, LM_, 8);    \
        else if (cfg.depth == 2) NF4_SK2(DT_, LM_, 2); \
        else NF4_SK2(DT_, LM_, 4);                   \
    } while (0)
#define NF4_SKL(DT_)                          \
    do {                                      \
        if (p.LM == 1) NF4_SK1(DT_, 1);       \
        else if (p.LM == 2) NF4_SK1(DT_, 2);  \
        else if (p.LM == 4) NF4_SK1(DT_, 4);  \
        else if (p.LM == 8) NF4_SK1(DT_, 8);  \
        else NF4_SK1(DT_, 16);                \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_SKL(NF4DQ_BF16);
    else NF4_SKL(NF4DQ_F16);
#undef NF4_SKL
#undef NF4_SK1
#undef NF4_SK2
    return hip_rc2(hipGetLastError());
}

}  // namespace nf4gemm
