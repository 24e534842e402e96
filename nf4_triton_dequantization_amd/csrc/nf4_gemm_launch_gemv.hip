// nf4_gemm_launch_gemv.hip -- the decode GEMV (M = 1): y[N] = W[N][K] . x[K] with the
// weights nf4_dequant_ref would write (reference double-dequant semantics, bit for bit),
// fp32 accumulation on the VALU (v_dot2c_f32_bf16 / _f16), no MFMA.
//
// Why a kernel of its own.  At M = 1 the MFMA kernels use one row of a 16-row tile and
// pay the MFMA fragment layout: a lane owns a 64-weight block column-wise, the 64 KiB pair
// table sits beside a strip ring, and the launch is bound by the dependency latency of
// that loop at two waves per SIMD.  Here a lane owns 32 consecutive
// weights of a row (16 packed bytes, half a 64-block: one scale), a wave reads 1 KiB of a
// row per load instruction (fully coalesced), and a workgroup of 16 waves keeps four
// waves per SIMD in flight.  Per packed byte: one v_perm (pair-table address), one
// ds_read_b64 (the two fp32 codes), one v_pk_mul_f32 by the block scale, one
// v_cvt_pk_bf16_f32 (RNE: the exact weights), one v_dot2c with the two x values -- the
// same exact-weight arithmetic as the MFMA kernels plus the dot.
//
// Layout.  Unit = (row group of R rows, piece j of 1 KiB packed per row = 2048 columns);
// lane l of piece j owns columns 2048 j + 32 l .. +31.  x is staged once per workgroup
// in LDS, swizzled [j][fragment s][lane][16 B] so that a lane's four 16-byte fragments
// are conflict-free reads.  Waves walk row groups g = wave, wave + waves, ...; every unit's
// loads go out one unit ahead (two register sets, no copies).  A row group's R partial
// sums are reduced across the wave with cross-lane adds and lane 0 stores the rows.
// Scales: block b = 32 j + l / 2 of the row: a1[(row bpr) mod nb + b], a2[(row groups)
// mod n2 + b / 4] (absmax not wrapping inside a row, as the persistent kernel assumes),
// s = (a1 / 127) * a2 (IEEE; the q/127 table), as kernel_optimized.py:40-45, :97-98.
#include "nf4_gemm_plan.h"

namespace {

constexpr uint32_t kGvPiece = 2048;  // columns per piece (64 lanes x 32)

struct GemvMat {
    const uint8_t* packed;  // [N][K/2]
    const uint8_t* a1;
    const float* a2;
    void* y;                // [N]
    uint32_t row_begin;     // first row of this weight in the launch
    uint32_t N;
    FastDiv nb, n2;
    uint32_t nb_bytes, n2_bytes;
};

struct GemvArgs {
    GemvMat mat[kGroupMax];
    uint32_t nmat;
    uint32_t groups_total;  // row groups over all weights
    const void* x;          // [K]
    uint32_t K, J;          // J = K / 2048 pieces per row
    uint32_t bpr, groups;   // K / 64, ceil(bpr / 4)
};

template <int R>
struct GvUnit {
    u32x4 w[R];
    uint32_t qa[R];
    float qb[R];
};

// One unit's loads: R rows x 16 packed bytes per lane, and each row's absmax byte and
// nested scale for the lane's block.  Invalid (past the wave's last unit): offsets beyond
// every buffer range, no traffic.
template <int R>
__device__ __forceinline__ void gv_issue(const GemvArgs& A, __amdgpu_buffer_rsrc_t rw, __amdgpu_buffer_rsrc_t ra1,
                                         __amdgpu_buffer_rsrc_t ra2, uint32_t lr, uint32_t j, const uint32_t (&rb1)[R],
                                         const uint32_t (&rb2)[R], bool valid, uint32_t lane, GvUnit<R>& u) {
    const uint32_t oob = valid ? 0u : kOob;
    const uint32_t b = 32u * j + (lane >> 1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        u.w[r] = __builtin_amdgcn_raw_buffer_load_b128(rw, ((lr + r) * (A.K >> 1) + 1024u * j + 16u * lane) | oob, 0, 0);
        u.qa[r] = __builtin_amdgcn_raw_buffer_load_b8(ra1, (rb1[r] + b) | oob, 0, 0);
        u.qb[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ra2, ((rb2[r] + (b >> 2)) * 4u) | oob, 0, 0));
    }
}

template <int DT>
__device__ __forceinline__ float gv_dot(uint32_t w2, uint32_t x2, float c) {
    if constexpr (DT == NF4DQ_BF16) {
        return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, w2), __builtin_bit_cast(bf16x2, x2), c, false);
    } else {
        return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w2), __builtin_bit_cast(f16x2, x2), c, false);
    }
}

// Dequantize one unit (exact weights: fp32 code x block scale, RNE) and dot it with the
// lane's x fragments into acc[r] (two chains per row).
template <int DT, int R>
__device__ __forceinline__ void gv_body(const GvUnit<R>& u, const char* pt, const float* qtab, const u32x4 (&xf)[4],
                                        uint32_t slot8, float (&acc)[R][2]) {
    f32x2 sc2[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float sc = qtab[u.qa[r]] * u.qb[r];  // (:45, :97-98)
        sc2[r] = f32x2{sc, opaque(sc)};
    }
    // steps st = (row, dword): pair lookups run LA steps ahead of their use
    constexpr int S = 4 * R, LA = 3;
    f32x2 v[S][4];
    auto issue = [&](int st) {
        const uint32_t wd = u.w[st >> 2][st & 3];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t addr = __builtin_amdgcn_perm(wd, slot8, 0x0C0C0000u | ((4u + b) << 8));
            v[st][b] = *reinterpret_cast<const f32x2*>(pt + addr);
        }
    };
#pragma unroll
    for (int st = 0; st < LA && st < S; ++st) issue(st);
#pragma unroll
    for (int st = 0; st < S; ++st) {
        if (st + LA < S) issue(st + LA);
        const int r = st >> 2, q = st & 3;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const f32x2 p = v[st][b] * sc2[r];        // fp32 products (:97-98)
            const uint32_t w2 = pack2<DT>(p.x, p.y);  // RNE (:109-110): the exact weights
            acc[r][b & 1] = gv_dot<DT>(w2, xf[q][b], acc[r][b & 1]);
        }
    }
}

template <int DT>
__device__ __forceinline__ void gv_store(void* y, uint32_t i, float v) {
    if constexpr (DT == NF4DQ_BF16) {
        reinterpret_cast<__bf16*>(y)[i] = (__bf16)v;
    } else {
        reinterpret_cast<_Float16*>(y)[i] = (_Float16)opaque(v);
    }
}

// (Measured and not kept, profiles/r06/gemm/s30_gemv_ab.jsonl: x held in registers at
// K = 4096 instead of LDS reads, 4 units in flight per wave instead of 2.)
template <int DT, int W, int R>
__global__ __launch_bounds__(64 * W) void nf4_gemv_kernel(const GemvArgs A) {
    extern __shared__ __attribute__((aligned(16))) char xs[];        // x, swizzled (see top)
    __shared__ __attribute__((aligned(16))) f32x2 ptab[256 * 32];   // pair table, 32 lane slots
    __shared__ float qtab[256];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t nw = gridDim.x * W;
    uint32_t g = blockIdx.x * W + wave;  // this wave's first row group

    // x's loads first, then the wave's first unit's loads, all before the tables are built
    // (x waits only for its own loads: they are the oldest)
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, 0, A.K * 2u, kRsrcFlags);
    constexpr uint32_t kXp = 2048u / (64u * W);  // 8-column pieces per thread (K <= 16384)
    u32x4 xv[kXp];
#pragma unroll
    for (uint32_t p = 0; p < kXp; ++p) {
        const uint32_t i = tid + p * 64u * W;
        xv[p] = __builtin_amdgcn_raw_buffer_load_b128(rx, i < A.K / 8u ? 16u * i : kOob, 0, 0);
    }
    uint32_t mi = 0;
    for (uint32_t i = 1; i < A.nmat; ++i) mi = g * R >= A.mat[i].row_begin ? i : mi;
    auto rsrcs = [&](uint32_t m, __amdgpu_buffer_rsrc_t& rw, __amdgpu_buffer_rsrc_t& r1, __amdgpu_buffer_rsrc_t& r2) {
        const GemvMat& Mt = A.mat[m];
        rw = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.packed, 0, Mt.N * (A.K >> 1), kRsrcFlags);
        r1 = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.a1, 0, Mt.nb_bytes, kRsrcFlags);
        r2 = __builtin_amdgcn_make_buffer_rsrc((void*)Mt.a2, 0, Mt.n2_bytes, kRsrcFlags);
    };
    auto row_bases = [&](uint32_t m, uint32_t lr, uint32_t (&rb1)[R], uint32_t (&rb2)[R]) {
        const GemvMat& Mt = A.mat[m];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            rb1[r] = fmodu((lr + r) * A.bpr, Mt.nb);
            rb2[r] = fmodu((lr + r) * A.groups, Mt.n2);
        }
    };
    __amdgpu_buffer_rsrc_t rw, r1, r2;
    rsrcs(mi, rw, r1, r2);
    uint32_t lr = g * R - A.mat[mi].row_begin;  // local row of the group's first row
    uint32_t rb1[R], rb2[R];
    row_bases(mi, lr, rb1, rb2);
    constexpr int D = 2;
    GvUnit<R> ring[D];
    gv_issue<R>(A, rw, r1, r2, lr, 0u, rb1, rb2, g < A.groups_total, lane, ring[0]);

    // tables: q / 127 (IEEE division, :45), the pair table (code[b >> 4], code[b & 15])
    // in 32 lane slots; then x into its swizzled layout
    if (tid < 256u) qtab[tid] = (float)tid / 127.0f;
    for (uint32_t i = tid; i < 256u * 16u; i += 64u * W) {  // two slots per 16-byte write
        const uint32_t b = i >> 4;
        const float hi = nf4_code(b >> 4), lo = nf4_code(b & 15u);
        *reinterpret_cast<f32x4*>(ptab + 2u * i) = f32x4{hi, lo, hi, lo};
    }
#pragma unroll
    for (uint32_t p = 0; p < kXp; ++p) {
        const uint32_t i = tid + p * 64u * W;
        if (i < A.K / 8u) {
            const uint32_t k = 8u * i;
            const uint32_t off = 4096u * (k >> 11) + 1024u * ((k >> 3) & 3u) + 16u * ((k >> 5) & 63u);
            *reinterpret_cast<u32x4*>(xs + off) = xv[p];
        }
    }
    __syncthreads();
    if (g >= A.groups_total) return;

    const char* pt = reinterpret_cast<const char*>(ptab);
    const uint32_t slot8 = (lane & 31u) * 8u;
    float acc[R][2];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = 0.0f;
    uint32_t j = 0;

    // advance (g, j) to the next unit; on a new row group recompute the weight, its
    // buffer descriptors and the row bases (wave-uniform)
    auto next_unit = [&](uint32_t& gg, uint32_t& jj, uint32_t& m, uint32_t& l, __amdgpu_buffer_rsrc_t& w,
                         __amdgpu_buffer_rsrc_t& a1r, __amdgpu_buffer_rsrc_t& a2r, uint32_t (&b1)[R],
                         uint32_t (&b2)[R]) {
        if (++jj < A.J) return;
        jj = 0;
        gg += nw;
        if (gg >= A.groups_total) return;
        uint32_t mm = m;
        while (mm + 1 < A.nmat && gg * R >= A.mat[mm + 1].row_begin) ++mm;
        if (mm != m) {
            m = mm;
            rsrcs(m, w, a1r, a2r);
        }
        l = gg * R - A.mat[m].row_begin;
        row_bases(m, l, b1, b2);
    };
    // finish a row group: wave-wide sums, lane 0 stores the R outputs
    auto finish = [&](uint32_t m, uint32_t l) {
        const GemvMat& Mt = A.mat[m];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            float s = acc[r][0] + acc[r][1];
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
            if (lane == 0) gv_store<DT>(Mt.y, l + r, s);
            acc[r][0] = acc[r][1] = 0.0f;
        }
    };

    auto xfrag = [&](uint32_t jj, uint32_t sf) {
        return *reinterpret_cast<const u32x4*>(xs + 4096u * jj + 1024u * sf + 16u * lane);
    };
    // the ring: D = 2 unit register sets, the next unit in flight while one is decoded.
    // Cursor n = the last unit issued, cursor p = the unit being decoded.
    uint32_t pg = g, pj = 0, pm = mi, pl = lr;
    uint32_t ng = g, nj = 0, nm = mi, nl = lr;
    __amdgpu_buffer_rsrc_t nw_ = rw, n1 = r1, n2 = r2;
    uint32_t nb1[R], nb2[R];
#pragma unroll
    for (int r = 0; r < R; ++r) nb1[r] = rb1[r], nb2[r] = rb2[r];
    auto issue_next = [&](GvUnit<R>& u) {
        next_unit(ng, nj, nm, nl, nw_, n1, n2, nb1, nb2);
        gv_issue<R>(A, nw_, n1, n2, nl, nj, nb1, nb2, ng < A.groups_total, lane, u);
    };
    auto advance_p = [&]() {
        if (++pj < A.J) return;
        pj = 0;
        pg += nw;
        if (pg >= A.groups_total) return;
        while (pm + 1 < A.nmat && pg * R >= A.mat[pm + 1].row_begin) ++pm;
        pl = pg * R - A.mat[pm].row_begin;
    };
    (void)j;
    bool live = true;
    while (live) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
            if (!live) break;  // wave-uniform: every unit of the wave decoded
            issue_next(ring[(i + D - 1) % D]);
            const u32x4 xf[4] = {xfrag(pj, 0), xfrag(pj, 1), xfrag(pj, 2), xfrag(pj, 3)};
            gv_body<DT, R>(ring[i], pt, qtab, xf, slot8, acc);
            if (pj + 1 == A.J) finish(pm, pl);
            advance_p();
            live = pg < A.groups_total;
        }
    }
}

}  // namespace

namespace nf4gemm {

// LDS: the x staging (2 K bytes) beside the 64 KiB pair table and the q/127 table.
uint32_t gemv_lds_bytes(int64_t K) { return (uint32_t)(K * 2); }

// One launch over `count` weights sharing x (M = 1; K % 2048 == 0; absmax not wrapping
// inside a row).  cfg.waves: waves per workgroup (8 / 16); cfg.depth: rows per row group R
// (1 / 2 / 4); cfg.strips: workgroups per CU in the grid (0 / 1 / 2, 0 = 1), at most one
// row group per wave.
int launch_gemv(const HostMat* mats, int count, const void* x, int64_t M, int64_t K, int32_t dtype,
                const nf4_gemm_cfg& cfg, hipStream_t st) {
    if (M != 1 || K % kGvPiece || K > 16384) return NF4DQ_ERR_ARG;
    if (cfg.waves != 8 && cfg.waves != 16) return NF4DQ_ERR_ARG;
    if (cfg.depth != 1 && cfg.depth != 2 && cfg.depth != 4) return NF4DQ_ERR_ARG;
    GemvArgs A{};
    A.nmat = (uint32_t)count;
    A.x = x;
    A.K = (uint32_t)K;
    A.J = (uint32_t)(K / kGvPiece);
    A.bpr = (uint32_t)(K / 64);
    A.groups = (A.bpr + 3) / 4;
    const uint32_t R = (uint32_t)cfg.depth;
    uint32_t rows = 0;
    for (int i = 0; i < count; ++i) {
        const HostMat& h = mats[i];
        if (!(h.nb % (K / 64) == 0 || h.nb >= h.N * (K / 64)) ||
            !(h.n2 % (int64_t)A.groups == 0 || h.n2 >= h.N * (int64_t)A.groups))
            return NF4DQ_ERR_ARG;  // absmax wrapping inside a row
        if (h.N % R) return NF4DQ_ERR_ARG;
        GemvMat& m = A.mat[i];
        m.packed = h.packed;
        m.a1 = h.a1;
        m.a2 = h.a2;
        m.y = h.y;
        m.N = (uint32_t)h.N;
        m.row_begin = rows;
        const int64_t nbc = h.nb > (int64_t(1) << 31) ? (int64_t(1) << 31) : h.nb;
        const int64_t n2c = h.n2 > (int64_t(1) << 29) ? (int64_t(1) << 29) : h.n2;
        m.nb = make_fastdiv((uint32_t)nbc);
        m.n2 = make_fastdiv((uint32_t)n2c);
        m.nb_bytes = (uint32_t)nbc;
        m.n2_bytes = (uint32_t)(n2c * 4);
        rows += (uint32_t)h.N;
    }
    A.groups_total = rows / R;
    const uint32_t W = (uint32_t)cfg.waves;
    uint32_t G = (uint32_t)device_cus() * (cfg.strips > 0 ? (uint32_t)cfg.strips : 1u);
    const uint32_t need = (A.groups_total + W - 1) / W;
    if (G > need) G = need;
    if (G < 1) G = 1;
    const uint32_t dyn = gemv_lds_bytes(K);
    const dim3 grid(G), block(64 * W);
#define NF4_GV(DT_, W_, R_)                                                                                     \
    do {                                                                                                        \
        static bool attr_ = false;                                                                              \
        if (!attr_) {                                                                                           \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&nf4_gemv_kernel<DT_, W_, R_>),              \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 65536);                       \
            attr_ = true;                                                                                       \
        }                                                                                                       \
        hipLaunchKernelGGL((nf4_gemv_kernel<DT_, W_, R_>), grid, block, dyn, st, A);                            \
    } while (0)
#define NF4_GVR(DT_, W_)                        \
    do {                                        \
        if (R == 1) NF4_GV(DT_, W_, 1);         \
        else if (R == 2) NF4_GV(DT_, W_, 2);    \
        else NF4_GV(DT_, W_, 4);                \
    } while (0)
#define NF4_GVW(DT_)                            \
    do {                                        \
        if (W == 8) NF4_GVR(DT_, 8);            \
        else NF4_GVR(DT_, 16);                  \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_GVW(NF4DQ_BF16);
    else NF4_GVW(NF4DQ_F16);
#undef NF4_GVW
#undef NF4_GVR
#undef NF4_GV
    return hip_rc2(hipGetLastError());
}

}  // namespace nf4gemm
