// nf4_gemm_launch_persist.hip -- launcher of the persistent kernel (nf4_gemm_persist_kernel) (instantiates its kernels;
// compiled on its own so that the kernel families build in parallel).
#include "nf4_gemm_plan.h"

namespace nf4gemm {

// One launch of the persistent kernel over `count` weights sharing x (cfg
// validated per weight).  Grid: as many workgroups as fit the CUs at once.
int launch_persist(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
                          const nf4_gemm_cfg& cfg, void* workspace, hipStream_t st) {
    StreamArgs S{};
    const uint32_t ks = (uint32_t)cfg.ksplit;
    S.nmat = (uint32_t)count;
    S.x = x;
    S.counters = reinterpret_cast<uint32_t*>(workspace);
    S.slab = ks > 1 ? reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(workspace) + kHeaderBytes) : nullptr;
    S.M = (uint32_t)M;
    S.K = (uint32_t)K;
    S.T = (uint32_t)cfg.strips;
    S.parts = (uint32_t)(cfg.waves / cfg.strips);
    S.ksplit = ks;
    S.chunks = (uint32_t)(K / kSChunkK);
    S.cps = S.chunks / ks;
    S.cpp = S.cps / S.parts;
    S.bpr = (uint32_t)(K / 64);
    S.groups = (S.bpr + 3) / 4;
    S.ppr = make_fastdiv(S.cps * 32u);
    S.xstride = S.cps * 512u + 16u;
    uint32_t sg = 0, strips = 0;
    for (int i = 0; i < count; ++i) {
        const HostMat& h = mats[i];
        if (!(h.nb % (K / 64) == 0 || h.nb >= h.N * (K / 64)) ||
            !(h.n2 % (int64_t)S.groups == 0 || h.n2 >= h.N * (int64_t)S.groups))
            return NF4DQ_ERR_ARG;  // absmax wrapping inside a row: the streaming kernel's case
        StreamMat& m = S.mat[i];
        m.packed = h.packed;
        m.a1 = h.a1;
        m.a2 = h.a2;
        m.y = h.y;
        m.N = (uint32_t)h.N;
        m.sg_begin = sg;
        m.strip_begin = strips;
        const int64_t nbc = h.nb > (int64_t(1) << 31) ? (int64_t(1) << 31) : h.nb;
        const int64_t n2c = h.n2 > (int64_t(1) << 29) ? (int64_t(1) << 29) : h.n2;
        m.nb = make_fastdiv((uint32_t)nbc);
        m.n2 = make_fastdiv((uint32_t)n2c);
        m.nb_bytes = (uint32_t)nbc;
        m.n2_bytes = (uint32_t)(n2c * 4);
        sg += (uint32_t)(h.N / (16 * cfg.strips));
        strips += (uint32_t)(h.N / 16);
    }
    S.sg_total = sg;
    S.ncols = strips * 16u;
    if (ks > 1 && sg * 4u > kCounterBytes) return NF4DQ_ERR_TOO_LARGE;  // one ticket per strip group
    const uint32_t base = persist_dyn_bytes(M, K, cfg, 1) + kStreamStatic;
    const uint32_t per_cu = kLdsPerCu / base > 0 ? kLdsPerCu / base : 1u;
    uint32_t G = (uint32_t)device_cus() * per_cu;  // workgroups; G / ks per K slice
    if (G > sg * ks) G = sg * ks;
    G = G / ks * ks;
    if (G < ks) G = ks;
    const uint32_t per_wg = (sg + G / ks - 1) / (G / ks);
    const uint32_t dyn = persist_dyn_bytes(M, K, cfg, per_wg);
    if (dyn + kStreamStatic > kLdsPerCu) return NF4DQ_ERR_TOO_LARGE;
    S.zero_off = kLdsX + (uint32_t)M * S.xstride;
    S.red_off = S.zero_off + 128u;
    S.out_off = S.red_off + 2u * (uint32_t)cfg.waves * 1024u;
    const dim3 grid(G), block(64 * cfg.waves);
#define NF4_PK1(DT_, W_, P_, SP_)                                                                               \
    do {                                                                                                        \
        static bool attr_ = false;                                                                              \
        if (!attr_) {                                                                                           \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&nf4_gemm_persist_kernel<DT_, W_, P_, SP_>), \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStreamLdsCap);          \
            attr_ = true;                                                                                       \
        }                                                                                                       \
        hipLaunchKernelGGL((nf4_gemm_persist_kernel<DT_, W_, P_, SP_>), grid, block, dyn, st, S);              \
    } while (0)
#define NF4_PK(DT_, W_, P_)                        \
    do {                                           \
        if (ks > 1) NF4_PK1(DT_, W_, P_, true);    \
        else NF4_PK1(DT_, W_, P_, false);          \
    } while (0)
#define NF4_PW(DT_)                                            \
    do {                                                       \
        if (cfg.waves == 4) {                                  \
            if (cfg.depth == 2) NF4_PK(DT_, 4, 2);             \
            else NF4_PK(DT_, 4, 4);                            \
        } else if (cfg.waves == 8) {                           \
            if (cfg.depth == 2) NF4_PK(DT_, 8, 2);             \
            else NF4_PK(DT_, 8, 4);                            \
        } else {                                               \
            if (cfg.depth == 2) NF4_PK(DT_, 16, 2);            \
            else NF4_PK(DT_, 16, 4);                           \
        }                                                      \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_PW(NF4DQ_BF16);
    else NF4_PW(NF4DQ_F16);
#undef NF4_PW
#undef NF4_PK
#undef NF4_PK1
    return hip_rc2(hipGetLastError());
}

}  // namespace nf4gemm
