// nf4_gemm_launch_stream.hip -- launcher of the streaming kernel (nf4_gemm_stream_kernel) (instantiates its kernels;
// compiled on its own so that the kernel families build in parallel).
#include "nf4_gemm_plan.h"

namespace nf4gemm {

// One launch of the streaming kernel over `count` weights sharing x (shapes and
// cfg already validated; workspace = counters + ksplit * M * sum(N) / 2 64-bit slab entries).
int launch_stream(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
                         const nf4_gemm_cfg& cfg, void* workspace, hipStream_t st) {
    const StreamPlan pl = stream_plan(M, K, cfg);
    const uint32_t ks = (uint32_t)cfg.ksplit;
    StreamArgs S{};
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
    S.cps = pl.cps;
    S.cpp = (pl.cps + S.parts - 1) / S.parts;
    S.bpr = (uint32_t)(K / 64);
    S.groups = (S.bpr + 3) / 4;
    S.ppr = make_fastdiv(pl.cps * 32u);
    S.xstride = pl.xstride;
    S.zero_off = pl.zero_off;
    S.red_off = pl.red_off;
    // vector scales: no absmax wrap inside any row of any weight, and each wave's chunks <= kVsMax
    bool vs = S.cpp <= (uint32_t)kVsMax;
    uint32_t sg = 0, strips = 0;
    for (int i = 0; i < count; ++i) {
        const HostMat& h = mats[i];
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
        vs = vs && (h.nb % (K / 64) == 0 || h.nb >= h.N * (K / 64)) &&
             (h.n2 % (int64_t)S.groups == 0 || h.n2 >= h.N * (int64_t)S.groups);
    }
    S.sg_total = sg;
    S.ncols = strips * 16u;
    const dim3 grid(sg * ks), block(64 * cfg.waves);
    const int mt = (int)((M + 15) / 16);
#define NF4_K1(DT_, MT_, W_, P_, VS_)                                                                       \
    do {                                                                                                    \
        static bool attr_ = false; /* static + dynamic LDS above 64 KiB needs the opt-in */                  \
        if (!attr_) {                                                                                       \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&nf4_gemm_stream_kernel<DT_, MT_, W_, P_, VS_>), \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStreamLdsCap);      \
            attr_ = true;                                                                                   \
        }                                                                                                   \
        hipLaunchKernelGGL((nf4_gemm_stream_kernel<DT_, MT_, W_, P_, VS_>), grid, block, pl.lds, st, S);    \
    } while (0)
#define NF4_K(DT_, MT_, W_, P_)                 \
    do {                                        \
        if (vs) NF4_K1(DT_, MT_, W_, P_, true); \
        else NF4_K1(DT_, MT_, W_, P_, false);   \
    } while (0)
#define NF4_P(DT_, MT_, W_)                                \
    do {                                                   \
        if (cfg.depth == 2) NF4_K(DT_, MT_, W_, 2);        \
        else if (cfg.depth == 4) NF4_K(DT_, MT_, W_, 4);   \
        else NF4_K(DT_, MT_, W_, (W_ == 16 ? 4 : 8));      \
    } while (0)
#define NF4_WW(DT_)                                        \
    do {                                                   \
        if (mt == 1) {                                     \
            if (cfg.waves == 4) NF4_P(DT_, 1, 4);          \
            else if (cfg.waves == 8) NF4_P(DT_, 1, 8);     \
            else NF4_P(DT_, 1, 16);                        \
        } else { /* 16 waves only for M <= 16 */           \
            if (cfg.waves == 4) NF4_P(DT_, 2, 4);          \
            else NF4_P(DT_, 2, 8);                         \
        }                                                  \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_WW(NF4DQ_BF16);
    else NF4_WW(NF4DQ_F16);
#undef NF4_WW
#undef NF4_P
#undef NF4_K
#undef NF4_K1
    return hip_rc2(hipGetLastError());
}

}  // namespace nf4gemm
