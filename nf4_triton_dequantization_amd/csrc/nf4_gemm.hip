// nf4_gemm.hip -- fused NF4 dequant + GEMM for small M (decode-shaped
// activations): Y[M, N] = X[M, K] . W[N, K]^T with W in the bitsandbytes NF4
// layout, reference double-dequant semantics (the same bf16/fp16 weights
// nf4_dequant_ref would materialise, bit for bit), fp32 accumulation on MFMA.
//
// What it replaces: the consumer pattern of the reference harness,
// `X @ triton_dequantize_nf4(W).t()` (benchmark.py:61-66), which writes the
// dequantized weight to HBM and reads it back.  Here the 4-bit weight is read
// once (0.5 B/element) and dequantized in registers -- the roofline is HBM on
// the packed weight, not on a 2 B/element bf16 copy.
//
// Decomposition: a wave owns 16 output columns (one MFMA 16x16x32 column tile)
// over a K slice; a 4-wave workgroup owns 64 adjacent columns of one K slice.
// Per 128-deep K chunk a lane loads 16 packed bytes of its weight row
// (row n0 + (lane & 15), k = 128c + 32(lane >> 4) .. +32: one 64-block, one
// scale) and the matching 64 bytes of each activation row; packed dword s of
// the lane is exactly the MFMA B fragment of step s (k = 8s + j inside the
// lane's 32) and activation bytes [16s, 16s+16) its A fragment -- the same k
// permutation on both operands, so no shuffle is needed.  Chunks are
// software-pipelined two deep (register sets P/Q).  K slices > 1 write fp32
// partials to a workspace slab; the last workgroup to finish a column group
// (ticket counter) sums the slices in slice order and writes y -- one launch,
// bitwise reproducible, no float atomics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nf4_dequant.h"
#include "nf4_common.h"

namespace {

using namespace nf4dq;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kGemmWaves = 8;
constexpr int kAuxSc1 = 16;  // write-through stores / L2-bypassing loads (cross-XCD hand-off)

template <int DT>
__device__ __forceinline__ void store_y(void* y, uint32_t i, float v) {
    if constexpr (DT == NF4DQ_BF16) {
        reinterpret_cast<__bf16*>(y)[i] = (__bf16)v;
    } else {
        reinterpret_cast<_Float16*>(y)[i] = (_Float16)opaque(v);
    }
}
constexpr uint32_t kChunkK = 128;

struct GemmArgs {
    const uint8_t* packed;  // [N][K/2]
    const uint8_t* a1;      // [nb]
    const float* a2;        // [n2]
    const void* x;          // [M][K] fp16/bf16
    void* y;                // [M][N] fp16/bf16
    float* slab;            // [ksplit][M][N] fp32 partials (ksplit > 1)
    uint32_t* counters;     // [N / 64] split-K tickets, 0 between calls
    uint32_t M, N, K;
    uint32_t col_groups;    // N / 16 column strips
    uint32_t ksplit;
    uint32_t chunks_per_split;
    uint32_t chunks;        // K / 128
    uint32_t bpr, groups;   // K / 64, ceil(bpr / 4)
    FastDiv nb, n2;
};

// One 128-deep K chunk of one lane: 16 packed weight bytes of its row (one
// 64-block, so one scale) and MT x 4 activation fragments.
template <int MT>
struct Chunk {
    u32x4 w;
    uint32_t qa;    // absmax byte
    float qb;       // nested absmax
    u32x4 x[MT][4];
};

template <int MT>
__device__ __forceinline__ void chunk_issue(const GemmArgs& A, __amdgpu_buffer_rsrc_t rw, __amdgpu_buffer_rsrc_t rx,
                                            uint32_t c, bool valid, uint32_t row, uint32_t nl, uint32_t kh,
                                            Chunk<MT>& in) {
    const uint32_t kbase = c * kChunkK + 32u * kh;
    // past the wave's last chunk: offsets beyond the buffer ranges (zeros, no traffic)
    in.w = __builtin_amdgcn_raw_buffer_load_b128(rw, valid ? row * (A.K >> 1) + (kbase >> 1) : 0xFFFFFFF0u, 0, 0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const uint32_t xoff = valid ? ((16u * mt + nl) * A.K + kbase) * 2u : 0xFFFFFF00u;  // rows >= M: zeros
#pragma unroll
        for (int s = 0; s < 4; ++s) in.x[mt][s] = __builtin_amdgcn_raw_buffer_load_b128(rx, xoff + 16u * s, 0, 0);
    }
    const uint32_t b = 2u * (valid ? c : 0u) + (kh >> 1);  // 64-block within the row
    in.qa = A.a1[fmodu(row * A.bpr + b, A.nb)];               // (:173-177 wrap)
    in.qb = A.a2[fmodu(row * A.groups + (b >> 2), A.n2)];    // (:40-41, :183-186 wrap)
}

template <int DT, int MT>
__device__ __forceinline__ void chunk_mma(const Chunk<MT>& in, const float* lut, f32x4 (&acc)[MT]) {
    const float sc = ((float)in.qa / 127.0f) * in.qb;  // IEEE division, then fp32 multiply (:45)
    const char* t = reinterpret_cast<const char*>(lut);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const uint32_t wd = in.w[s];
        const uint32_t hi4 = (wd >> 2) & 0x3C3C3C3Cu;
        const uint32_t lo4 = (wd << 2) & 0x3C3C3C3Cu;
        float v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[2 * k] = *reinterpret_cast<const float*>(t + ((hi4 >> (8 * k)) & 0xFFu)) * sc;
            v[2 * k + 1] = *reinterpret_cast<const float*>(t + ((lo4 >> (8 * k)) & 0xFFu)) * sc;
        }
        // the exact weights nf4_dequant_ref writes: fp32 product, RNE to 16 bits
        const u32x4 bw = {pack2<DT>(v[0], v[1]), pack2<DT>(v[2], v[3]), pack2<DT>(v[4], v[5]),
                          pack2<DT>(v[6], v[7])};
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            if constexpr (DT == NF4DQ_BF16) {
                acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, in.x[mt][s]),
                                                                  __builtin_bit_cast(bf16x8, bw), acc[mt], 0, 0, 0);
            } else {
                acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, in.x[mt][s]),
                                                                 __builtin_bit_cast(f16x8, bw), acc[mt], 0, 0, 0);
            }
        }
    }
}

// Workgroup = kGemmWaves waves owning 16 output columns of one K slice; wave
// w takes every kGemmWaves-th group of D chunks, D chunks in flight at a time;
// the waves' partial sums are combined through LDS (fixed order).
template <int DT, int MT, int D>
__global__ __launch_bounds__(64 * kGemmWaves) void nf4_gemm_smallm_kernel(const GemmArgs A) {
    __shared__ __attribute__((aligned(16))) float lut[20];  // 16 codes + the last-arriver flag
    __shared__ __attribute__((aligned(16))) f32x4 red[kGemmWaves][MT][64];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t nl = lane & 15u, kh = lane >> 4;
    const uint32_t cg = blockIdx.x % A.col_groups;   // 16-column strip
    const uint32_t ks = blockIdx.x / A.col_groups;   // K slice
    const uint32_t row = cg * 16u + nl;
    const uint32_t c0 = ks * A.chunks_per_split;
    const uint32_t c1 = c0 + A.chunks_per_split < A.chunks ? c0 + A.chunks_per_split : A.chunks;

    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)A.packed, 0, A.N * (A.K >> 1), kRsrcFlags);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)A.x, 0, A.M * A.K * 2u, kRsrcFlags);

    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    bool first = true;
    for (uint32_t g = c0 + wave * D; g < c1 || first; g += kGemmWaves * D) {
        Chunk<MT> ch[D];
#pragma unroll
        for (int d = 0; d < D; ++d) chunk_issue<MT>(A, rw, rx, g + d, g + d < c1, row, nl, kh, ch[d]);
        if (first) {  // LUT + barrier overlap the first loads
            write_lut(lut);
            __syncthreads();
            first = false;
        }
#pragma unroll
        for (int d = 0; d < D; ++d) chunk_mma<DT, MT>(ch[d], lut, acc);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wave][mt][lane] = acc[mt];
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        f32x4 s = red[0][mt][lane];
#pragma unroll
        for (int w = 1; w < kGemmWaves; ++w) s += red[w][mt][lane];
        acc[mt] = s;
    }

    // acc[mt][r] = Y[16 mt + 4 kh + r][n0 + nl]
    if (A.ksplit == 1) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t m = 16u * mt + 4u * kh + r;
                if (m < A.M) store_y<DT>(A.y, m * A.N + row, acc[mt][r]);
            }
        }
        return;
    }

    // Split-K, reduced inside the launch (MI355X_MICROARCH.md / cdna guide G16,
    // write-through form): every slice writes its fp32 partials with sc1
    // stores, drains them, and one lane per workgroup takes a ticket on the
    // column group's counter; the workgroup drawing ksplit-1 sums all slices
    // in slice order (sc1 loads: no stale line from any L2), writes y, and
    // resets the counter to 0 for the next call.  Bitwise reproducible.
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)A.slab, 0, A.ksplit * A.M * A.N * 4u, kRsrcFlags);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t m = 16u * mt + 4u * kh + r;
            const uint32_t off = m < A.M ? ((ks * A.M + m) * A.N + row) * 4u : 0xFFFFFFF0u;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[mt][r]), rs, off, 0, kAuxSc1);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // only wave 0 is left: its own drain is the hand-off
    uint32_t last = 0;
    if (lane == 0) {
        const uint32_t ticket = __hip_atomic_fetch_add(&A.counters[cg], 1u, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        last = ticket == A.ksplit - 1u;
        if (last) __hip_atomic_store(&A.counters[cg], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last = __builtin_amdgcn_readfirstlane(last);
    if (!last) return;
    for (uint32_t i = lane; i < A.M * 16u; i += 64u) {
        const uint32_t m = i >> 4;
        const uint32_t n = cg * 16u + (i & 15u);
        float sum = 0.0f;
        for (uint32_t k = 0; k < A.ksplit; ++k) {
            sum += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, ((k * A.M + m) * A.N + n) * 4u, 0,
                                                                        kAuxSc1));
        }
        store_y<DT>(A.y, m * A.N + n, sum);
    }
}

// K split across workgroups only when there are too few 16-column strips to
// give every CU two workgroups; each slice keeps >= kGemmWaves chunks.
uint32_t choose_ksplit(int64_t M, int64_t N, int64_t K) {
    (void)M;
    const int64_t strips = N / 16, chunks = K / kChunkK;
    int64_t ks = (512 + strips - 1) / strips;
    const int64_t max_ks = chunks / kGemmWaves > 0 ? chunks / kGemmWaves : 1;
    if (ks > max_ks) ks = max_ks;
    return (uint32_t)(ks < 1 ? 1 : ks);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int hip_rc2(hipError_t e) { return e == hipSuccess ? NF4DQ_OK : NF4DQ_ERR_HIP_BASE + (int)e; }

}  // namespace

extern "C" {

// Workspace: [64 KiB of uint32 ticket counters][ksplit * M * N fp32 partials].
// The counter region has a fixed size so that no call's partials ever overlay
// another call's counters (those must stay 0 between calls): N <= 2^18.
constexpr size_t kCounterBytes = 64 * 1024;
static size_t counters_bytes(int64_t) { return kCounterBytes; }

size_t nf4_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
    if (M <= 0 || N <= 0 || K <= 0 || N % 64 || K % kChunkK) return 0;
    const uint32_t ks = choose_ksplit(M, N, K);
    return ks > 1 ? counters_bytes(N) + (size_t)ks * (size_t)M * (size_t)N * sizeof(float) : 0;
}

int nf4_gemm_ref(const void* x, int64_t M, const uint8_t* packed, int64_t packed_len, const uint8_t* absmax_q,
                 int64_t nb, const float* absmax2, int64_t n2, void* y, int32_t dtype, int64_t N, int64_t K,
                 void* workspace, size_t workspace_bytes, void* hip_stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
    if (dtype != NF4DQ_F16 && dtype != NF4DQ_BF16) return NF4DQ_ERR_ARG;
    if (M < 0 || N < 0 || K < 0 || nb <= 0 || n2 <= 0) return NF4DQ_ERR_ARG;
    if (M == 0 || N == 0) return NF4DQ_OK;
    if (!x || !packed || !absmax_q || !absmax2 || !y) return NF4DQ_ERR_ARG;
    if (M > NF4DQ_GEMM_MAX_M || N % 64 || K % kChunkK || packed_len != N * (K / 2)) return NF4DQ_ERR_SHAPE;
    if ((size_t)(N / 16) * 4 > kCounterBytes) return NF4DQ_ERR_TOO_LARGE;
    if (packed_len >= (int64_t(1) << 31) || M * K * 2 >= (int64_t(1) << 31)) return NF4DQ_ERR_TOO_LARGE;
    const uint32_t ks = choose_ksplit(M, N, K);
    const size_t need = nf4_gemm_workspace_bytes(M, N, K);
    if (need && (!workspace || workspace_bytes < need || !aligned16(workspace))) return NF4DQ_ERR_ARG;
    GemmArgs A{};
    A.packed = packed;
    A.a1 = absmax_q;
    A.a2 = absmax2;
    A.x = x;
    A.y = y;
    A.counters = reinterpret_cast<uint32_t*>(workspace);
    A.slab = ks > 1 ? reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + counters_bytes(N)) : nullptr;
    A.M = (uint32_t)M;
    A.N = (uint32_t)N;
    A.K = (uint32_t)K;
    A.col_groups = (uint32_t)(N / 16);
    A.ksplit = ks;
    A.chunks = (uint32_t)(K / kChunkK);
    A.chunks_per_split = (A.chunks + ks - 1) / ks;
    A.bpr = (uint32_t)(K / 64);
    A.groups = (A.bpr + 3) / 4;
    A.nb = make_fastdiv((uint32_t)(nb > (int64_t(1) << 31) ? (int64_t(1) << 31) : nb));
    A.n2 = make_fastdiv((uint32_t)(n2 > (int64_t(1) << 31) ? (int64_t(1) << 31) : n2));
    const dim3 grid(A.col_groups * ks), block(64 * kGemmWaves);
    const int mt = (int)((M + 15) / 16);
#define NF4_G(DT_, MT_, D_) hipLaunchKernelGGL((nf4_gemm_smallm_kernel<DT_, MT_, D_>), grid, block, 0, st, A)
#define NF4_S(DT_)                          \
    do {                                    \
        if (mt == 1) NF4_G(DT_, 1, 4);      \
        else NF4_G(DT_, 2, 2);              \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_S(NF4DQ_BF16);
    else NF4_S(NF4DQ_F16);
#undef NF4_S
#undef NF4_G
    return hip_rc2(hipGetLastError());
}

}  // extern "C"
