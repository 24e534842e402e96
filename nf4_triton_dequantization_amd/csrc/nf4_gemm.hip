// nf4_gemm.hip -- fused NF4 dequant + GEMM for small M: the host dispatch (library
// choice of kernel and decomposition, validation, workspace sizing) and the C ABI of
// include/nf4_dequant.h.  The kernels are in nf4_gemm_dev.h (see its comment for the
// design), their launchers in nf4_gemm_launch_*.hip.
#include "nf4_gemm_plan.h"

namespace {

using namespace nf4gemm;

// Defaults, from tools/sweep_gemm.py on MI355X (Llama-3-8B shapes and the grouped
// q/k/v and gate/up column totals, M = 1..32; re-checked in round 4,
// profiles/r04/gemm/sweep_gemm_m1_12.jsonl, sweep_gemm_m16_32.jsonl: the default is
// the fastest or within 2 % of it except where noted below).  N = all columns of the
// launch (a grouped launch passes the sum).
//  * M = 1, N <= 4096, K % 2048 == 0: the decode GEMV (round 6, gemv_choice below).
//  * M <= 8: the persistent kernel whenever x[M][K] fits its LDS (the streaming
//    kernel if absmax wraps inside a row), strips by width.
//  * 8 < M <= 16: the persistent kernel with K slices; the register-resident
//    kernel for N <= 1024.
//  * 16 < M <= 32: the register-resident kernel (two K slices at K = 4096; 16 waves
//    and no slices for the widest launches at M <= 24); the 128-deep and
//    shared-activation kernels where K % 256 != 0 or N < 1024.
bool valid_gemm_cfg(const nf4_gemm_cfg& c, int64_t M, int64_t N, int64_t K);

static nf4_gemm_cfg k128_cfg(int64_t M, int64_t N, int64_t K, int waves, int depth, int ksplit, int strips) {
    nf4_gemm_cfg c{NF4DQ_GEMM_K128, waves, depth, ksplit, strips};
    if (M > 16 && c.depth > 2) c.depth = 2;
    while (c.strips > 1 && N % (16 * c.strips)) c.strips /= 2;
    if (c.ksplit > K / kChunkK) c.ksplit = (int)(K / kChunkK);
    if (c.ksplit < 1) c.ksplit = 1;
    return c;
}

// The library's choice when the persistent kernel is not used (or cannot run:
// absmax wrapping inside a row, held outputs beyond its LDS).
static nf4_gemm_cfg nonpersist_cfg(int64_t M, int64_t N, int64_t K) {
    const bool k256 = K % kSChunkK == 0;
    if (k256 && M <= 8) {
        nf4_gemm_cfg c{NF4DQ_GEMM_STREAM, 8, 2, 1, 1};
        if (M > 4) c = nf4_gemm_cfg{NF4DQ_GEMM_STREAM, 8, 2, 4, 4};
        else if (M > 1) c = nf4_gemm_cfg{NF4DQ_GEMM_STREAM, 8, 2, 2, 2};
        while (c.strips > 1 && N % (16 * c.strips)) c.strips /= 2;
        if (c.ksplit > K / kSChunkK) c.ksplit = (int)(K / kSChunkK);
        while (c.ksplit < K / kSChunkK && !stream_fits(M, K, c)) ++c.ksplit;
        if (valid_gemm_cfg(c, M, N, K)) return c;
        return k128_cfg(M, N, K, 8, 2, 1, 1);
    }
    if (M <= 16) {
        if (k256 && K < 8192 && N > 4096) {
            nf4_gemm_cfg c{NF4DQ_GEMM_STREAM, 8, 2, 2, 4};
            while (c.strips > 1 && N % (16 * c.strips)) c.strips /= 2;
            while (c.ksplit < K / kSChunkK && !stream_fits(M, K, c)) ++c.ksplit;
            if (valid_gemm_cfg(c, M, N, K)) return c;
        }
        if (K >= 8192) return k128_cfg(M, N, K, 8, 1, 2, 2);
        if (N < 4096) return k128_cfg(M, N, K, 4, 2, 4, 1);
        return k128_cfg(M, N, K, 8, 2, 1, 1);
    }
    if (K % kSChunkK == 0 && N >= 1024) {
        // the register-resident kernel with pair-table lookups, 8 waves x 256-deep
        // chunks: per launch at M = 32 (profiles/r02/sweep_gemm_xr.jsonl) 20.4 vs 21.7 us
        // on 14336x4096, 11.9 vs 12.3 on 4096^2, 23.5 vs 24.6 on 4096x14336, 13.8 vs 14.2
        // on grouped q/k/v (6144), 31.4 vs 37.2 on grouped gate/up (28672); from N = 1024
        // since round 4 (7.7 vs 8.6-9.0 us at M = 24 / 32, profiles/r04/gemm/sweep_gemm_m16_32.jsonl)
        if (M <= 24 && N >= 24576) {
            // the widest launches (grouped gate/up) at M <= 24: 16 waves span K = 4096,
            // no split-K hand-off: 26.0 vs 27.6 us (profiles/r04/gemm/xr_no_handoff_m24_m32.jsonl)
            const nf4_gemm_cfg w{NF4DQ_GEMM_XR, 16, 2, (int)((K / kChunkK + 31) / 32), 2};
            if (valid_gemm_cfg(w, M, N, K)) return w;
        }
        const nf4_gemm_cfg c{NF4DQ_GEMM_XR, 8, 2, (int)((K / kChunkK + 15) / 16), 2};
        if (valid_gemm_cfg(c, M, N, K)) return c;
    }
    if (K >= 8192) return k128_cfg(M, N, K, 8, 1, 4, 4);
    if (N >= 6144) {
        // wide launches (gate/up, grouped q/k/v): the shared-activation kernel,
        // 10-13 % faster than the 128-deep one at M = 24 / 32 (profiles/r02/sweep_gemm_xs.jsonl)
        const int waves = N >= 12288 ? 8 : 4, kc = N >= 12288 ? 8 : 4;
        const nf4_gemm_cfg c{NF4DQ_GEMM_XS, waves, kc, (int)((K / kChunkK + kc - 1) / kc), 1};
        if (valid_gemm_cfg(c, M, N, K)) return c;
    }
    if (N < 4096) return k128_cfg(M, N, K, 4, 2, 4, 1);
    if (N <= 4096) return k128_cfg(M, N, K, 8, 1, 2, 2);
    if (N < 8192) return k128_cfg(M, N, K, 4, 1, 4, 2);
    return k128_cfg(M, N, K, N >= 16384 ? 4 : 8, 1, 1, 4);
}

nf4_gemm_cfg default_gemm_cfg(int64_t M, int64_t N, int64_t K) {
    if (K % kSChunkK == 0 && M <= 8) {
        const int strips = N >= 16384 ? 1 : N >= 8192 ? 4 : N > 4096 ? 2 : 1;
        const nf4_gemm_cfg c{NF4DQ_GEMM_PERSIST, 8, 2, 1, strips};
        if (valid_gemm_cfg(c, M, N, K)) return c;
    } else if (K % kSChunkK == 0 && M <= 16) {
        if (N <= 1024) {
            // too few strips to cover the CUs with slices of the persistent kernel: the
            // register-resident kernel, 6.6 vs 7.7 us on 1024x4096 at M = 12
            // (profiles/r04/gemm/sweep_gemm_m1_12.jsonl)
            const nf4_gemm_cfg c{NF4DQ_GEMM_XR, 8, 2, (int)((K / kChunkK + 15) / 16), 2};
            if (valid_gemm_cfg(c, M, N, K)) return c;
        }
        // persistent with K slices: the fewest slices whose x fits, while the
        // (strip group, slice) pairs still cover every CU
        for (int strips = 2; strips <= 4; strips *= 2)
            for (int ks = 2; ks <= 16; ++ks) {
                const nf4_gemm_cfg c{NF4DQ_GEMM_PERSIST, 8, 2, ks, strips};
                if (N / (16 * strips) * ks >= 256 && valid_gemm_cfg(c, M, N, K)) return c;
            }
    }
    return nonpersist_cfg(M, N, K);
}

// M = 1: the decode GEMV (nf4_gemm_launch_gemv.hip) where it beats the persistent kernel:
// up to 4096 columns (profiles/r06/gemm/s29_gemv_ab.jsonl, s30_gemv_ab.jsonl, one box each:
// 4096^2 5.77-5.99 vs 6.33 us, 4096 x 14336 10.25-10.61 vs 11.16-11.62); wider launches
// stay persistent (14336 x 4096: 11.6 vs 10.5; grouped q/k/v 7.6 vs 7.3).  N = all columns
// of the launch.  The caller falls back to default_gemm_cfg when it cannot run (absmax
// wrapping inside a row).
static bool gemv_choice(int64_t M, int64_t N, int64_t K, nf4_gemm_cfg* c) {
    if (M != 1 || K % 2048 || K > 16384 || N > 4096) return false;
    *c = nf4_gemm_cfg{NF4DQ_GEMM_GEMV, 16, 1, 1, 0};
    return true;
}

// Dynamic LDS of the persistent kernel: x slice, zero block, two partial-sum
// sets, the held outputs (16-bit finished values; fp32 partials when K is split).
bool valid_gemm_cfg(const nf4_gemm_cfg& c, int64_t M, int64_t N, int64_t K) {
    if (c.kernel == NF4DQ_GEMM_PERSIST) {
        if (K % kSChunkK || M > 16) return false;
        if (c.waves != 4 && c.waves != 8 && c.waves != 16) return false;
        if (c.depth != 2 && c.depth != 4) return false;
        if (c.strips != 1 && c.strips != 2 && c.strips != 4) return false;
        if (c.waves % c.strips || N % (16 * c.strips) || c.ksplit < 1 || c.ksplit > 16) return false;
        const int64_t chunks = K / kSChunkK, parts = c.waves / c.strips;
        if (chunks % c.ksplit) return false;
        const int64_t cps = chunks / c.ksplit;  // chunks per K slice
        if (cps % parts || (cps / parts) % c.depth) return false;
        if (M * cps * 32 > (int64_t)kXR * 64 * c.waves) return false;
        return persist_dyn_bytes(M, K, c, 1) + kStreamStatic <= kLdsPerCu;
    }
    if (c.kernel == NF4DQ_GEMM_STREAM) {
        if (K % kSChunkK) return false;
        if (c.waves != 4 && c.waves != 8 && c.waves != 16) return false;
        if (c.depth != 2 && c.depth != 4 && c.depth != 8) return false;
        if (c.waves == 16 && (M > 16 || c.depth == 8)) return false;
        if (c.strips != 1 && c.strips != 2 && c.strips != 4) return false;
        if (c.waves % c.strips || N % (16 * c.strips)) return false;
        if (c.ksplit < 1 || c.ksplit > K / kSChunkK) return false;
        return stream_fits(M, K, c);
    }
    if (c.kernel == NF4DQ_GEMM_XR) {
        if (c.waves != 8 && c.waves != 16) return false;
        if (c.depth != 2 && c.depth != 4) return false;
        if (c.strips != 1 && c.strips != 2 && c.strips != 4) return false;  // 128-deep chunks per wave
        if (c.strips == 4 && (c.waves != 8 || K % 512)) return false;          // two 256-deep chunks per wave
        if (c.strips == 4 && c.depth == 4 && M > 16) return false;             // 64 x VGPRs + a 4-deep ring spill
        // x + a 4-deep ring spill within 16 waves' 128 registers (8 waves: 256)
        if (M > 16 && c.strips == 2 && c.depth == 4 && c.waves == 16) return false;
        if (c.strips >= 2 && K % 256) return false;                 // 256-deep chunks
        const int64_t chunks = K / kChunkK, per = (int64_t)c.waves * c.strips;
        return c.ksplit == (chunks + per - 1) / per && c.ksplit <= 1024;
    }
    // NF4DQ_GEMM_SK (the balanced stream-K kernel, rounds 4-5) was never the library's
    // choice -- 13.1-15.1 vs 10.6 us on 14336x4096 at M = 1,
    // profiles/r04/gemm/sk_depth_vs_persist.jsonl -- and was removed in round 6: its
    // number is rejected like any unknown kernel (git history holds the source)
    if (c.kernel == NF4DQ_GEMM_GEMV) {
        if (M != 1 || K % 2048 || K > 16384 || c.ksplit != 1) return false;
        if (c.waves != 8 && c.waves != 16) return false;
        if (c.depth != 1 && c.depth != 2 && c.depth != 4) return false;
        return c.strips >= 0 && c.strips <= 2 && N % c.depth == 0;
    }
    if (c.kernel == NF4DQ_GEMM_XS) {
        if (c.waves != 4 && c.waves != 8) return false;
        if (c.depth != 2 && c.depth != 4 && c.depth != 8) return false;
        if (c.strips != 0 && c.strips != 1) return false;
        const int64_t chunks = K / kChunkK;
        return c.ksplit == (chunks + c.depth - 1) / c.depth && c.ksplit <= 256;
    }
    if (c.kernel != NF4DQ_GEMM_K128) return false;
    if (c.waves != 4 && c.waves != 8) return false;
    if (c.strips != 0 && c.strips != 1 && c.strips != 2 && c.strips != 4) return false;  // strips per wave
    if (M > 16 ? (c.depth != 1 && c.depth != 2) : (c.depth != 1 && c.depth != 2 && c.depth != 4)) return false;
    return c.ksplit >= 1 && c.ksplit <= K / kChunkK && c.ksplit <= 64;
}

static size_t workspace_for(int64_t M, int64_t N, int64_t K, const nf4_gemm_cfg& c) {
    if (M <= 0 || N <= 0 || K <= 0 || N % 64 || K % kChunkK) return 0;
    return c.ksplit > 1 ? counters_bytes(N) + (size_t)c.ksplit * (size_t)M * (size_t)N * 4u : 0;  // 8-B entry per 2 columns
}

static int gemm_impl(const void* x, int64_t M, const uint8_t* packed, int64_t packed_len, const uint8_t* absmax_q,
                     int64_t nb, const float* absmax2, int64_t n2, void* y, int32_t dtype, int64_t N, int64_t K,
                     void* workspace, size_t workspace_bytes, const nf4_gemm_cfg* cfgp, hipStream_t st) {
    if (dtype != NF4DQ_F16 && dtype != NF4DQ_BF16) return NF4DQ_ERR_ARG;
    if (M < 0 || N < 0 || K < 0 || nb <= 0 || n2 <= 0) return NF4DQ_ERR_ARG;
    if (M == 0 || N == 0) return NF4DQ_OK;
    if (!x || !packed || !absmax_q || !absmax2 || !y) return NF4DQ_ERR_ARG;
    if (M > NF4DQ_GEMM_MAX_M || N % 64 || K % kChunkK || packed_len != N * (K / 2)) return NF4DQ_ERR_SHAPE;
    if ((size_t)(N / 16) * 4 > kCounterBytes) return NF4DQ_ERR_TOO_LARGE;
    if (packed_len >= (int64_t(1) << 31) || M * K * 2 >= (int64_t(1) << 31)) return NF4DQ_ERR_TOO_LARGE;
    nf4_gemm_cfg gv{};
    if (!cfgp && gemv_choice(M, N, K, &gv)) {
        const HostMat h{packed, packed_len, absmax_q, nb, absmax2, n2, y, N};
        const int rc = launch_gemv(&h, 1, x, M, K, dtype, gv, st);
        if (rc != NF4DQ_ERR_ARG) return rc;  // else absmax wraps inside a row: the next choice
    }
    nf4_gemm_cfg cfg = cfgp ? *cfgp : default_gemm_cfg(M, N, K);
    if (cfg.kernel == 0) {
        const nf4_gemm_cfg d = default_gemm_cfg(M, N, K);
        cfg.kernel = d.kernel;
    }
    if (!valid_gemm_cfg(cfg, M, N, K)) return NF4DQ_ERR_ARG;
    const size_t need = workspace_for(M, N, K, cfg);
    // the kernels address the split-K slab through one buffer descriptor (32-bit range)
    if (need >= (size_t(1) << 32)) return NF4DQ_ERR_TOO_LARGE;
    if (need && (!workspace || workspace_bytes < need || !aligned16(workspace))) return NF4DQ_ERR_ARG;
    if (cfg.kernel == NF4DQ_GEMM_STREAM || cfg.kernel == NF4DQ_GEMM_PERSIST) {
        const HostMat h{packed, packed_len, absmax_q, nb, absmax2, n2, y, N};
        if (cfg.kernel == NF4DQ_GEMM_PERSIST) {
            const int rc = launch_persist(&h, 1, x, M, K, dtype, cfg, workspace, st);
            if ((rc != NF4DQ_ERR_ARG && rc != NF4DQ_ERR_TOO_LARGE) || cfgp) return rc;
            // library choice that cannot run here (absmax wrapping in a row, held
            // outputs beyond LDS): the next choice; its workspace need is covered
            // (callers size the workspace with nf4_gemm_workspace_bytes = the max)
            cfg = nonpersist_cfg(M, N, K);
            const size_t w2 = workspace_for(M, N, K, cfg);
            if (!valid_gemm_cfg(cfg, M, N, K) || (w2 && (!workspace || workspace_bytes < w2 || !aligned16(workspace))))
                return NF4DQ_ERR_ARG;
            if (cfg.kernel == NF4DQ_GEMM_K128)
                return gemm_impl(x, M, packed, packed_len, absmax_q, nb, absmax2, n2, y, dtype, N, K, workspace,
                                 workspace_bytes, &cfg, st);
        }
        return launch_stream(&h, 1, x, M, K, dtype, cfg, workspace, st);
    }
    const HostMat h{packed, packed_len, absmax_q, nb, absmax2, n2, y, N};
    if (cfg.kernel == NF4DQ_GEMM_GEMV) return launch_gemv(&h, 1, x, M, K, dtype, cfg, st);
    if (cfg.kernel == NF4DQ_GEMM_XS) return launch_xs(&h, 1, x, M, K, dtype, cfg, workspace, st);
    if (cfg.kernel == NF4DQ_GEMM_XR) return launch_xr(&h, 1, x, M, K, dtype, cfg, workspace, st);
    return launch_k128(&h, 1, x, M, K, dtype, cfg, workspace, st);
}

// Weights that share x, one launch of whichever kernel cfg names (workgroups
// numbered over all the weights' strips / column groups); the library's
// persistent choice, when it cannot run, falls back to per-weight launches.
static int gemm_grouped_impl(const void* x, int64_t M, int64_t K, const nf4_gemm_mat* mats, int32_t count,
                             int32_t dtype, void* workspace, size_t workspace_bytes, const nf4_gemm_cfg* cfgp,
                             hipStream_t st) {
    if (count < 0 || count > NF4DQ_GEMM_GROUP_MAX || (count > 0 && !mats)) return NF4DQ_ERR_ARG;
    if (dtype != NF4DQ_F16 && dtype != NF4DQ_BF16) return NF4DQ_ERR_ARG;
    if (M < 0 || K < 0) return NF4DQ_ERR_ARG;
    int64_t ntot = 0;
    for (int i = 0; i < count; ++i) {
        const nf4_gemm_mat& m = mats[i];
        if (m.N < 0 || m.nb <= 0 || m.n2 <= 0) return NF4DQ_ERR_ARG;
        if (!m.packed || !m.absmax_q || !m.absmax2 || !m.y) return NF4DQ_ERR_ARG;
        if (m.N % 64 || m.packed_len != m.N * (K / 2)) return NF4DQ_ERR_SHAPE;
        ntot += m.N;
    }
    if (M == 0 || ntot == 0 || count == 0) return NF4DQ_OK;
    if (!x) return NF4DQ_ERR_ARG;
    if (M > NF4DQ_GEMM_MAX_M || K % kChunkK) return NF4DQ_ERR_SHAPE;
    if ((size_t)(ntot / 16) * 4 > kCounterBytes) return NF4DQ_ERR_TOO_LARGE;
    nf4_gemm_cfg cfg = cfgp ? *cfgp : default_gemm_cfg(M, ntot, K);
    if (cfg.kernel == 0) cfg.kernel = default_gemm_cfg(M, ntot, K).kernel;
    static_assert(kK128GroupMax == NF4DQ_GEMM_GROUP_MAX && kGroupMax == NF4DQ_GEMM_GROUP_MAX, "group sizes");
    for (int i = 0; i < count; ++i) {
        // an empty weight cannot own strip groups (the 128-deep kernel numbers
        // column groups per weight: an empty one simply owns none)
        if (mats[i].N == 0 && cfg.kernel != NF4DQ_GEMM_K128 && cfg.kernel != NF4DQ_GEMM_XS &&
            cfg.kernel != NF4DQ_GEMM_XR)
            return NF4DQ_ERR_SHAPE;
        if (mats[i].N == 0) continue;
        if (!valid_gemm_cfg(cfg, M, mats[i].N, K)) return NF4DQ_ERR_ARG;
        if (mats[i].packed_len >= (int64_t(1) << 31)) return NF4DQ_ERR_TOO_LARGE;
    }
    if (M * K * 2 >= (int64_t(1) << 31)) return NF4DQ_ERR_TOO_LARGE;
    const size_t need = cfg.ksplit > 1 ? kHeaderBytes + (size_t)cfg.ksplit * (size_t)M * (size_t)ntot * 4u : 0;
    if (need >= (size_t(1) << 32)) return NF4DQ_ERR_TOO_LARGE;  // one buffer descriptor over the slab
    if (need && (!workspace || workspace_bytes < need || !aligned16(workspace))) return NF4DQ_ERR_ARG;
    HostMat h[NF4DQ_GEMM_GROUP_MAX];
    for (int i = 0; i < count; ++i)
        h[i] = HostMat{mats[i].packed, mats[i].packed_len, mats[i].absmax_q, mats[i].nb, mats[i].absmax2,
                       mats[i].n2, mats[i].y, mats[i].N};
    nf4_gemm_cfg gv{};
    if (!cfgp && gemv_choice(M, ntot, K, &gv)) {
        bool empty = false;
        for (int i = 0; i < count; ++i) empty = empty || mats[i].N == 0;
        if (!empty) {
            const int rc = launch_gemv(h, count, x, M, K, dtype, gv, st);
            if (rc != NF4DQ_ERR_ARG) return rc;  // else absmax wraps inside a row: the next choice
        }
    }
    if (cfg.kernel == NF4DQ_GEMM_K128) return launch_k128(h, count, x, M, K, dtype, cfg, workspace, st);
    if (cfg.kernel == NF4DQ_GEMM_GEMV) return launch_gemv(h, count, x, M, K, dtype, cfg, st);
    if (cfg.kernel == NF4DQ_GEMM_XS) return launch_xs(h, count, x, M, K, dtype, cfg, workspace, st);
    if (cfg.kernel == NF4DQ_GEMM_XR) return launch_xr(h, count, x, M, K, dtype, cfg, workspace, st);
    if (cfg.kernel == NF4DQ_GEMM_PERSIST) {
        const int rc = launch_persist(h, count, x, M, K, dtype, cfg, workspace, st);
        if ((rc != NF4DQ_ERR_ARG && rc != NF4DQ_ERR_TOO_LARGE) || cfgp) return rc;
        // library choice that cannot run here: per-weight launches with each weight's own choice
        for (int i = 0; i < count; ++i) {
            const nf4_gemm_mat& m = mats[i];
            nf4_gemm_cfg c = nonpersist_cfg(M, m.N, K);
            const int r2 = gemm_impl(x, M, m.packed, m.packed_len, m.absmax_q, m.nb, m.absmax2, m.n2, m.y, dtype, m.N,
                                     K, workspace, workspace_bytes, &c, st);
            if (r2) return r2;
        }
        return NF4DQ_OK;
    }
    return launch_stream(h, count, x, M, K, dtype, cfg, workspace, st);
}

static size_t grouped_workspace(int64_t M, int64_t K, const nf4_gemm_mat* mats, int32_t count,
                                const nf4_gemm_cfg* cfgp) {
    if (count <= 0 || !mats || M <= 0 || K <= 0 || K % kChunkK) return 0;
    int64_t ntot = 0, nmax = 0;
    for (int i = 0; i < count; ++i) {
        ntot += mats[i].N;
        nmax = mats[i].N > nmax ? mats[i].N : nmax;
    }
    if (ntot <= 0) return 0;
    nf4_gemm_cfg cfg = cfgp ? *cfgp : default_gemm_cfg(M, ntot, K);
    if (cfg.kernel == 0) cfg.kernel = default_gemm_cfg(M, ntot, K).kernel;
    size_t w = cfg.ksplit > 1 ? kHeaderBytes + (size_t)cfg.ksplit * (size_t)M * (size_t)ntot * 4u : 0;
    if (cfgp || cfg.kernel != NF4DQ_GEMM_PERSIST) return w;
    // the library's persistent choice may fall back to per-weight launches
    // (gemm_grouped_impl): the largest of their needs as well
    for (int i = 0; i < count; ++i) {
        const size_t wi = workspace_for(M, mats[i].N, K, nonpersist_cfg(M, mats[i].N, K));
        w = wi > w ? wi : w;
    }
    (void)nmax;
    return w;
}

}  // namespace

extern "C" {

size_t nf4_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
    if (M <= 0 || N <= 0 || K <= 0 || N % 64 || K % kChunkK) return 0;
    // the library's choice, or the next one if that cannot run (see gemm_impl)
    const size_t a = workspace_for(M, N, K, default_gemm_cfg(M, N, K));
    const size_t b = workspace_for(M, N, K, nonpersist_cfg(M, N, K));
    return a > b ? a : b;
}

size_t nf4_gemm_workspace_bytes_cfg(int64_t M, int64_t N, int64_t K, const nf4_gemm_cfg* cfg) {
    if (!cfg) return nf4_gemm_workspace_bytes(M, N, K);
    return workspace_for(M, N, K, *cfg);
}

int nf4_gemm_ref(const void* x, int64_t M, const uint8_t* packed, int64_t packed_len, const uint8_t* absmax_q,
                 int64_t nb, const float* absmax2, int64_t n2, void* y, int32_t dtype, int64_t N, int64_t K,
                 void* workspace, size_t workspace_bytes, void* hip_stream) {
    return gemm_impl(x, M, packed, packed_len, absmax_q, nb, absmax2, n2, y, dtype, N, K, workspace, workspace_bytes,
                     nullptr, reinterpret_cast<hipStream_t>(hip_stream));
}

size_t nf4_gemm_grouped_workspace_bytes(int64_t M, int64_t K, const nf4_gemm_mat* mats, int32_t count,
                                        const nf4_gemm_cfg* cfg) {
    return grouped_workspace(M, K, mats, count, cfg);
}

int nf4_gemm_ref_grouped(const void* x, int64_t M, int64_t K, const nf4_gemm_mat* mats, int32_t count,
                         int32_t out_dtype, void* workspace, size_t workspace_bytes, const nf4_gemm_cfg* cfg,
                         void* hip_stream) {
    return gemm_grouped_impl(x, M, K, mats, count, out_dtype, workspace, workspace_bytes, cfg,
                             reinterpret_cast<hipStream_t>(hip_stream));
}

int nf4_gemm_check_workspace(void* workspace, size_t workspace_bytes, void* hip_stream) {
    if (!workspace || workspace_bytes == 0) return NF4DQ_OK;  // no split-K ran on it
    if (workspace_bytes < kHeaderBytes) return NF4DQ_ERR_ARG;  // never a split-K workspace
    const hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    uint32_t err = 0;
    hipError_t e = hipMemcpyAsync(&err, reinterpret_cast<char*>(workspace) + kCounterBytes, sizeof(err),
                                  hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_rc2(e);
    if (!err) return NF4DQ_OK;
    // every kernel of the stream has finished: no late store can land after this
    e = hipMemsetAsync(workspace, 0, workspace_bytes, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e != hipSuccess ? hip_rc2(e) : NF4DQ_ERR_SPLITK_TIMEOUT;
}

int nf4_gemm_ref_cfg(const void* x, int64_t M, const uint8_t* packed, int64_t packed_len, const uint8_t* absmax_q,
                     int64_t nb, const float* absmax2, int64_t n2, void* y, int32_t dtype, int64_t N, int64_t K,
                     void* workspace, size_t workspace_bytes, const nf4_gemm_cfg* cfg, void* hip_stream) {
    return gemm_impl(x, M, packed, packed_len, absmax_q, nb, absmax2, n2, y, dtype, N, K, workspace, workspace_bytes,
                     cfg, reinterpret_cast<hipStream_t>(hip_stream));
}

}  // extern "C"
