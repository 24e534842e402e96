// nf4_gemm_plan.h -- host-side plans of the fused-GEMM kernels (LDS budgets,
// grid shapes, workspace layout) and the launcher interface between the host
// dispatch (nf4_gemm.hip) and the per-family launchers (nf4_gemm_launch_*.hip).
#pragma once

#include "nf4_gemm_dev.h"

namespace nf4gemm {

// One weight of a launch (host view).
struct HostMat {
    const uint8_t* packed;
    int64_t packed_len;
    const uint8_t* a1;
    int64_t nb;
    const float* a2;
    int64_t n2;
    void* y;
    int64_t N;
};


// Launchers (shapes and cfg validated by the dispatch; workspace sized by it).
int launch_stream(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
                  const nf4_gemm_cfg& cfg, void* workspace, hipStream_t st);
int launch_persist(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
                   const nf4_gemm_cfg& cfg, void* workspace, hipStream_t st);
int launch_xs(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
              const nf4_gemm_cfg& cfg, void* workspace, hipStream_t st);
int launch_xr(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
              const nf4_gemm_cfg& cfg, void* workspace, hipStream_t st);
int launch_k128(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
                const nf4_gemm_cfg& cfg, void* workspace, hipStream_t st);
int launch_gemv(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
                const nf4_gemm_cfg& cfg, hipStream_t st);

}  // namespace nf4gemm

namespace {

using nf4gemm::HostMat;

// ---- decomposition choice --------------------------------------------------
constexpr uint32_t kLdsPerCu = 160 * 1024;
constexpr uint32_t kStreamStatic = 256 * 32 * 8 + 1024;  // pair table, q/127 table
constexpr uint32_t kStreamLdsCap = kLdsPerCu - kStreamStatic;  // dynamic part

struct StreamPlan {
    uint32_t cps, xstride, zero_off, red_off, lds;
};

inline StreamPlan stream_plan(int64_t M, int64_t K, const nf4_gemm_cfg& c) {
    const uint32_t chunks = (uint32_t)(K / kSChunkK);
    const uint32_t mt = (uint32_t)((M + 15) / 16);
    StreamPlan p{};
    p.cps = (chunks + (uint32_t)c.ksplit - 1) / (uint32_t)c.ksplit;
    p.xstride = p.cps * 512u + 16u;  // +16 B: consecutive rows start 4 banks apart
    p.zero_off = kLdsX + (uint32_t)M * p.xstride;
    p.red_off = kLdsX;
    const uint32_t xend = p.zero_off + 128u, rend = p.red_off + (uint32_t)c.waves * mt * 1024u;
    p.lds = xend > rend ? xend : rend;
    return p;
}

inline bool stream_fits(int64_t M, int64_t K, const nf4_gemm_cfg& c) {
    const StreamPlan p = stream_plan(M, K, c);
    const int64_t xr = kXR * ((M + 15) / 16);
    return p.lds <= kStreamLdsCap && M * (int64_t)p.cps * 32 <= xr * 64 * c.waves;
}


inline uint32_t persist_dyn_bytes(int64_t M, int64_t K, const nf4_gemm_cfg& c, uint32_t groups_per_wg) {
    const uint32_t ks = c.ksplit > 1 ? (uint32_t)c.ksplit : 1u;
    const uint32_t xstride = (uint32_t)(K / ks) * 2u + 16u;
    const uint32_t ob = ks > 1 ? 64u : 32u;  // bytes per held row of a strip
    const uint32_t out = (groups_per_wg * (uint32_t)c.strips * (uint32_t)M * ob + 15u) & ~15u;
    return kLdsX + (uint32_t)M * xstride + 128u + 2u * (uint32_t)c.waves * 1024u + out;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int hip_rc2(hipError_t e) { return e == hipSuccess ? NF4DQ_OK : NF4DQ_ERR_HIP_BASE + (int)e; }

// Workspace: [64 KiB of uint32 ticket counters][256 B: the error word + spare]
// [ksplit * M * N / 2 64-bit slab entries].  The header has a fixed size so that no
// call's partials ever overlay another call's counters (those must stay 0 between
// calls): N <= 2^18.  The error word (kErrWord, sticky) is set by a reducer whose
// poll gave up (nf4_gemm_check_workspace reads it).
constexpr size_t kCounterBytes = 64 * 1024;
constexpr size_t kHeaderBytes = kCounterBytes + 256;
static_assert(kErrWord * 4u == kCounterBytes, "the error word follows the counters");
inline size_t counters_bytes(int64_t) { return kHeaderBytes; }


inline int device_cus() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cached[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cached[dev] = n;
    }
    return cached[dev];
}

// One launch of the 128-deep kernel over `count` weights sharing x (shapes and
// cfg validated; workspace = counters + ksplit * M * sum(N) / 2 64-bit slab entries when ksplit > 1).
// LDS bytes of the shared-activation kernel: x slice (16 MT rows) + scale table + LUT.
inline uint32_t xs_lds_bytes(int64_t M, int kc, int waves) {
    const uint32_t mt = M > 16 ? 2u : 1u;
    return 16u * mt * ((uint32_t)kc * 256u + 16u) + 16u * (uint32_t)waves * 2u * (uint32_t)kc * 4u + 64u;
}

// Register-resident kernel: grid = ksplit x (strip groups of T strips); T from
// the CUs the launch can hold at once (one 16-wave workgroup per CU), at most 64
// (ticket flags) and within LDS.
inline uint32_t xr_lds_static(int kpw) {  // pair table + q/127 (256-deep chunks), static in the kernel
    return kpw >= 2 ? 256u * 32u * 8u + 1024u : 64u;
}
inline uint32_t xr_lds_dynamic(int64_t M, int waves, uint32_t T) {
    const uint32_t mt = M > 16 ? 2u : 1u;
    const uint32_t r = waves == 8 ? 2u : 1u;  // strips per reduction group (kernel's R; depth is even)
    return 2u * r * (uint32_t)waves * mt * 1024u + 64u + 256u + T * mt * 1024u;  // partials, codes, flags, held
}
inline uint32_t xr_lds_bytes(int64_t M, int waves, int kpw, uint32_t T) {
    return xr_lds_static(kpw) + xr_lds_dynamic(M, waves, T);
}

inline uint32_t xr_per_wg(int64_t M, int64_t strips, const nf4_gemm_cfg& c) {
    const uint32_t wg_per_cu = c.waves == 16 || c.strips >= 2 ? 1u : 2u;  // the pair table leaves room for one
    uint32_t P = (uint32_t)device_cus() * wg_per_cu / (uint32_t)c.ksplit;  // workgroups per K slice
    if (P < 1) P = 1;
    uint32_t T = (uint32_t)((strips + P - 1) / P);
    while (T > 1 && (T > 64 || xr_lds_bytes(M, c.waves, c.strips, T) > kLdsPerCu)) T = (T + 1) / 2;
    return T < 1 ? 1u : T;
}

}  // namespace
