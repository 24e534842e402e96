// nf4_dequant_cpu.cpp -- the host-CPU NF4 double dequantization of libnf4dq.so
// ("nf4_dequant_ref_cpu(...), thread count as a parameter").
//
// What it replaces: the reference's CPU path, _aggressive_pytorch_t4
// (nf4_triton_dequantization/kernel_optimized.py:208-314), which loops over the
// 64-column blocks in Python (:267) and writes the output column by column
// (:305-312).  Same semantics, bit for bit (the HIP kernels' semantics too):
//
//   s(r, b)   = ((float)absmax_q[(r*bpr + b) mod nb] / 127.0f) * absmax2[(r*G + b/4) mod n2]
//   out[r][c] = RNE(NF4[nib(r, c)] * s(r, c/64)),  high nibble -> even column
//
// (single-quant branch :273-274: s(r, b) = absmax[r*(absmax_len/m) + b]).
//
// Design: every output of a 64-column block is one of only 16 values, so a block
// costs 16 fp32 products + 16 roundings (IEEE, no fused ops) into a 16-entry
// table of output bit patterns, and the 64 outputs are table lookups on the
// nibbles: with AVX2 one vpshufb per output byte plane per 32 outputs
// (the 16-bit outputs split into low-byte and high-byte tables), so the block
// is ~20 vector instructions and the loop runs at memory speed.  Rows are split
// over `threads` std::thread workers (no OpenMP runtime: the library is loaded
// into processes that already carry torch's).  A CPU without AVX2 takes the
// portable scalar table loop (same tables, same results).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include <immintrin.h>

#include "../../include/nf4_dequant.h"

namespace {

// The 16 NF4 code points (fp32 bit patterns of kernel_optimized.py:234-239).
constexpr uint32_t kCode[16] = {0xbf800000u, 0xbf3239b1u, 0xbf066b30u, 0xbeca32a0u, 0xbe91a24du, 0xbe3d353fu,
                                0xbdba7871u, 0x00000000u, 0x3da2faffu, 0x3e24cae3u, 0x3e7c04ddu, 0x3ead033au,
                                0x3ee1a4b8u, 0x3f1007abu, 0x3f3913b3u, 0x3f800000u};

enum Mode { kRef, kSingle };

inline float code_f(int i) {
    float f;
    memcpy(&f, &kCode[i], 4);
    return f;
}

inline uint16_t bf16_rne(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    if ((u & 0x7FFFFFFFu) > 0x7F800000u) return (uint16_t)((u >> 16) | 0x40u);  // NaN stays NaN (quiet)
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

inline uint16_t f16_rne(float x) {
    const _Float16 h = (_Float16)x;  // IEEE RNE incl. subnormals and overflow to inf
    uint16_t b;
    memcpy(&b, &h, 2);
    return b;
}

struct Job {
    const uint8_t* packed;
    int64_t stride;  // packed bytes per row (packed_len / m)
    const uint8_t* a1;
    int64_t nb;
    const float* a2;  // ref: nested absmax; single: fp32 absmax rows
    int64_t n2;       // ref: modulus; single: absmax row stride
    void* out;
    int64_t m, n, bpr, groups;
};

// 16 outputs of one block: products in fp32 (same op order as the kernels and
// the reference: LUT value times block scale), then the output rounding.
template <int DT>
inline void block_table(float s, uint16_t* t16, float* t32) {
    for (int k = 0; k < 16; ++k) {
        const float p = code_f(k) * s;  // one IEEE product (-ffp-contract=off; x86 has no fused multiply-round)
        if constexpr (DT == NF4DQ_F32) t32[k] = p;
        else if constexpr (DT == NF4DQ_BF16) t16[k] = bf16_rne(p);
        else t16[k] = f16_rne(p);
    }
}

// Scalar: any block width (partial last block, odd n).
template <int DT>
inline void block_scalar(const uint8_t* src, void* out, int64_t c0, int64_t cnt, const uint16_t* t16,
                         const float* t32) {
    for (int64_t k = 0; k < cnt; ++k) {
        const int64_t c = c0 + k;
        const uint8_t byte = src[c >> 1];
        const int nib = (c & 1) ? (byte & 15) : (byte >> 4);
        if constexpr (DT == NF4DQ_F32) reinterpret_cast<float*>(out)[c] = t32[nib];
        else reinterpret_cast<uint16_t*>(out)[c] = t16[nib];
    }
}

// AVX2: 32 packed bytes -> 64 16-bit outputs with four vpshufb per 32 outputs.
__attribute__((target("avx2"))) inline void block64_avx2(const uint8_t* src, uint16_t* dst, const uint16_t* t16) {
    alignas(16) uint8_t lo[16], hi[16];
    for (int k = 0; k < 16; ++k) {
        lo[k] = (uint8_t)(t16[k] & 0xFF);
        hi[k] = (uint8_t)(t16[k] >> 8);
    }
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i*>(lo)));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i*>(hi)));
    const __m256i m4 = _mm256_set1_epi8(0x0F);
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src));
    const __m256i nh = _mm256_and_si256(_mm256_srli_epi16(v, 4), m4);
    const __m256i nl = _mm256_and_si256(v, m4);
    // per 128-bit lane: (hi0, lo0, hi1, lo1, ...) = column order of the outputs
    const __m256i i0 = _mm256_unpacklo_epi8(nh, nl);  // lane0: bytes 0-7 (cols 0-15), lane1: bytes 16-23 (32-47)
    const __m256i i1 = _mm256_unpackhi_epi8(nh, nl);  // lane0: bytes 8-15 (16-31), lane1: bytes 24-31 (48-63)
    __m256i* d = reinterpret_cast<__m256i*>(dst);
    {
        const __m256i L = _mm256_shuffle_epi8(tlo, i0), H = _mm256_shuffle_epi8(thi, i0);
        const __m256i w0 = _mm256_unpacklo_epi8(L, H), w1 = _mm256_unpackhi_epi8(L, H);
        _mm256_storeu_si256(d + 0, _mm256_permute2x128_si256(w0, w1, 0x20));
        _mm256_storeu_si256(d + 2, _mm256_permute2x128_si256(w0, w1, 0x31));
    }
    {
        const __m256i L = _mm256_shuffle_epi8(tlo, i1), H = _mm256_shuffle_epi8(thi, i1);
        const __m256i w0 = _mm256_unpacklo_epi8(L, H), w1 = _mm256_unpackhi_epi8(L, H);
        _mm256_storeu_si256(d + 1, _mm256_permute2x128_si256(w0, w1, 0x20));
        _mm256_storeu_si256(d + 3, _mm256_permute2x128_si256(w0, w1, 0x31));
    }
}

template <int DT, int MODE, bool AVX2>
void run_rows(const Job& J, int64_t r0, int64_t r1) {
    const int64_t osz = DT == NF4DQ_F32 ? 4 : 2;
    alignas(32) uint16_t t16[16];
    alignas(32) float t32[16];
    for (int64_t r = r0; r < r1; ++r) {
        const uint8_t* src = J.packed + r * J.stride;
        void* orow = reinterpret_cast<uint8_t*>(J.out) + r * J.n * osz;
        int64_t i1 = 0, i2 = 0;
        if constexpr (MODE == kRef) {
            i1 = (r * J.bpr) % J.nb;        // (r*bpr + b) mod nb, advanced per block
            i2 = (r * J.groups) % J.n2;     // (r*G + b/4) mod n2, advanced every 4 blocks
        }
        for (int64_t b = 0; b < J.bpr; ++b) {
            float s;
            if constexpr (MODE == kRef) {
                s = ((float)J.a1[i1] / 127.0f) * J.a2[i2];  // IEEE division (:45, :270), then fp32 multiply
                if (++i1 == J.nb) i1 = 0;
                if ((b & 3) == 3 && ++i2 == J.n2) i2 = 0;
            } else {
                s = J.a2[r * J.n2 + b];
            }
            block_table<DT>(s, t16, t32);
            const int64_t c0 = b * 64;
            const int64_t cnt = J.n - c0 < 64 ? J.n - c0 : 64;
            if constexpr (AVX2 && DT != NF4DQ_F32) {
                if (cnt == 64) {
                    block64_avx2(src + (c0 >> 1), reinterpret_cast<uint16_t*>(orow) + c0, t16);
                    continue;
                }
            }
            block_scalar<DT>(src, orow, c0, cnt, t16, t32);
        }
    }
}

template <int MODE>
void dispatch_rows(const Job& J, int32_t dtype, int64_t r0, int64_t r1, bool avx2) {
#define NF4_CPU_ROWS(DT_)                                              \
    do {                                                               \
        if (avx2) run_rows<DT_, MODE, true>(J, r0, r1);                \
        else run_rows<DT_, MODE, false>(J, r0, r1);                    \
    } while (0)
    if (dtype == NF4DQ_BF16) NF4_CPU_ROWS(NF4DQ_BF16);
    else if (dtype == NF4DQ_F16) NF4_CPU_ROWS(NF4DQ_F16);
    else NF4_CPU_ROWS(NF4DQ_F32);
#undef NF4_CPU_ROWS
}

template <int MODE>
int run(const Job& J, int32_t dtype, int32_t threads) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    int64_t t = threads > 0 ? threads : (int64_t)std::max(1u, std::thread::hardware_concurrency());
    // at least 16 rows of work per worker (thread start-up is ~tens of us)
    t = std::max<int64_t>(1, std::min<int64_t>(t, (J.m + 15) / 16));
    if (t == 1) {
        dispatch_rows<MODE>(J, dtype, 0, J.m, avx2);
        return NF4DQ_OK;
    }
    std::vector<std::thread> pool;
    pool.reserve((size_t)t - 1);
    const int64_t per = (J.m + t - 1) / t;
    for (int64_t i = 1; i < t; ++i) {
        const int64_t r0 = i * per, r1 = std::min(J.m, r0 + per);
        if (r0 >= r1) break;
        pool.emplace_back([&J, dtype, r0, r1] { dispatch_rows<MODE>(J, dtype, r0, r1, avx2); });
    }
    dispatch_rows<MODE>(J, dtype, 0, std::min(J.m, per), avx2);
    for (auto& th : pool) th.join();
    return NF4DQ_OK;
}

// Same acceptance rules as the device entry points (what .view(m, -1) and the
// slicing of kernel_optimized.py:229, :288-312 accept).
int check(const uint8_t* packed, int64_t packed_len, const void* out, int32_t dtype, int64_t m, int64_t n) {
    if (dtype != NF4DQ_F16 && dtype != NF4DQ_BF16 && dtype != NF4DQ_F32) return NF4DQ_ERR_ARG;
    if (m < 0 || n < 0 || packed_len < 0) return NF4DQ_ERR_ARG;
    if (m == 0 || n == 0) return NF4DQ_OK;
    if (!packed || !out) return NF4DQ_ERR_ARG;
    if (packed_len % m) return NF4DQ_ERR_SHAPE;
    if (packed_len / m < (n + 1) / 2) return NF4DQ_ERR_SHAPE;
    return NF4DQ_OK;
}

}  // namespace

extern "C" {

int nf4_dequant_ref_cpu(const uint8_t* packed, int64_t packed_len, const uint8_t* absmax_q, int64_t nb,
                        const float* absmax2, int64_t n2, void* out, int32_t out_dtype, int64_t m, int64_t n,
                        int32_t threads) {
    const int rc = check(packed, packed_len, out, out_dtype, m, n);
    if (rc || m == 0 || n == 0) return rc;
    if (!absmax_q || !absmax2 || nb <= 0 || n2 <= 0) return NF4DQ_ERR_ARG;
    Job J{};
    J.packed = packed;
    J.stride = packed_len / m;
    J.a1 = absmax_q;
    J.nb = nb;
    J.a2 = absmax2;
    J.n2 = n2;
    J.out = out;
    J.m = m;
    J.n = n;
    J.bpr = (n + 63) / 64;
    J.groups = (J.bpr + 3) / 4;
    return run<kRef>(J, out_dtype, threads);
}

int nf4_dequant_single_cpu(const uint8_t* packed, int64_t packed_len, const float* absmax, int64_t absmax_len,
                           void* out, int32_t out_dtype, int64_t m, int64_t n, int32_t threads) {
    const int rc = check(packed, packed_len, out, out_dtype, m, n);
    if (rc || m == 0 || n == 0) return rc;
    if (!absmax || absmax_len < 0) return NF4DQ_ERR_ARG;
    const int64_t bpr = (n + 63) / 64;
    if (absmax_len % m || absmax_len / m < bpr) return NF4DQ_ERR_SHAPE;
    Job J{};
    J.packed = packed;
    J.stride = packed_len / m;
    J.a2 = absmax;
    J.n2 = absmax_len / m;
    J.out = out;
    J.m = m;
    J.n = n;
    J.bpr = bpr;
    return run<kSingle>(J, out_dtype, threads);
}

}  // extern "C"
