// nf4_gemm_launch_k128.hip -- launcher of the 128-deep kernel (nf4_gemm_smallm_kernel) (instantiates its kernels;
// compiled on its own so that the kernel families build in parallel).
#include "nf4_gemm_plan.h"

namespace nf4gemm {

int launch_k128(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
                       const nf4_gemm_cfg& cfg, void* workspace, hipStream_t st) {
    const uint32_t ks = (uint32_t)cfg.ksplit;
    const int nt = cfg.strips > 1 ? cfg.strips : 1;  // 16-column strips per wave
    GemmArgs A{};
    A.nmat = (uint32_t)count;
    A.x = x;
    A.counters = reinterpret_cast<uint32_t*>(workspace);
    A.slab = ks > 1 ? reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(workspace) + kHeaderBytes) : nullptr;
    A.M = (uint32_t)M;
    A.K = (uint32_t)K;
    A.ksplit = ks;
    A.chunks = (uint32_t)(K / kChunkK);
    A.chunks_per_split = (A.chunks + ks - 1) / ks;
    A.bpr = (uint32_t)(K / 64);
    A.groups = (A.bpr + 3) / 4;
    // scale table in LDS when absmax does not wrap inside a row (any weight) and the slice's table is small
    const uint32_t scl_bytes = 16u * (uint32_t)nt * 2u * A.chunks_per_split * 4u;
    bool vs = scl_bytes <= 48u * 1024u;
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
        cgs += (uint32_t)(h.N / (16 * nt));
        cols += (uint32_t)h.N;
        vs = vs && (h.nb % (K / 64) == 0 || h.nb >= h.N * (K / 64)) &&
             (h.n2 % (int64_t)A.groups == 0 || h.n2 >= h.N * (int64_t)A.groups);
    }
    A.col_groups = cgs;
    A.ncols = cols;
    const dim3 grid(A.col_groups * ks), block(64 * cfg.waves);
    const int mt = (int)((M + 15) / 16);
    const uint32_t dyn = vs ? scl_bytes : 0u;
#define NF4_G(DT_, MT_, D_, W_, NT_)                                                                          \
    do {                                                                                                      \
        if (vs) hipLaunchKernelGGL((nf4_gemm_smallm_kernel<DT_, MT_, D_, W_, NT_, true>), grid, block, dyn, st, A); \
        else hipLaunchKernelGGL((nf4_gemm_smallm_kernel<DT_, MT_, D_, W_, NT_, false>), grid, block, 0, st, A);    \
    } while (0)
#define NF4_N(DT_, MT_, D_, W_)                   \
    do {                                          \
        if (nt == 4) NF4_G(DT_, MT_, D_, W_, 4);  \
        else if (nt == 2) NF4_G(DT_, MT_, D_, W_, 2); \
        else NF4_G(DT_, MT_, D_, W_, 1);          \
    } while (0)
#define NF4_W(DT_, MT_, D_)                        \
    do {                                           \
        if (cfg.waves == 8) NF4_N(DT_, MT_, D_, 8); \
        else NF4_N(DT_, MT_, D_, 4);               \
    } while (0)
#define NF4_S(DT_)                                  \
    do {                                            \
        if (mt == 1) {                              \
            if (cfg.depth == 4) NF4_W(DT_, 1, 4);   \
            else if (cfg.depth == 2) NF4_W(DT_, 1, 2); \
            else NF4_W(DT_, 1, 1);                  \
        } else {                                    \
            if (cfg.depth == 2) NF4_W(DT_, 2, 2);   \
            else NF4_W(DT_, 2, 1);                  \
        }                                           \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_S(NF4DQ_BF16);
    else NF4_S(NF4DQ_F16);
#undef NF4_S
#undef NF4_W
#undef NF4_N
#undef NF4_G
    return hip_rc2(hipGetLastError());
}

}  // namespace nf4gemm
