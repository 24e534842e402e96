/*
 * nf4_oracle.c -- CPU restatement of the reference NF4 double-dequantization.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product library (nf4_triton_dequantization_amd/_lib/libnf4dq.so) never
 * links or calls it, and the product raises if its HIP library is missing.
 *
 * Parity pin: tests/test_oracle_golden.py checks every function here against the
 * golden vectors in tests/golden/, which oracle/gen_golden.py produced by running
 * the reference's own fallback `_aggressive_pytorch_t4`
 * (/root/reference/nf4_triton_dequantization/kernel_optimized.py:208-314).
 *
 * Semantics restated (reference file:line in kernel_optimized.py):
 *   bpr = ceil(n/64)                         (:158, :231)
 *   G   = ceil(bpr/4)                        (:180, :255)
 *   A1 index wraps modulo nb                 (repeat/truncate :173-177, :246-251)
 *   A2 index r*G + b/4 wraps modulo n2       (:40-41, :183-186, :255-263)
 *   scale = fp32(A1/127.0f) * A2             (:45, :270) -- IEEE division, not rcp
 *   packed row stride = numel/m              (.view(m,-1) :229)
 *   even column <- high nibble, odd <- low   (:108-110, :303-312)
 *   out = RNE(fp32(NF4[nib]) * scale)        (:97-98, :300-301, cast :310/:312)
 * Single-quant branch (absmax not uint8):     scale = absmax.view(m,-1)[:, b] (:273-274)
 *
 * bnb semantics (bitsandbytes is absent here, so this
 * mode is "parity unpinned"): absmax_f32[i] = code2[A1[i]] * A2[i/256] + offset,
 * out_flat[k] = RNE(NF4[nib(k)] * absmax_f32[k/64]).
 *
 * Build: oracle/Makefile (gcc -O2, never -ffast-math: division and rounding
 * must stay IEEE).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#define NF4O_F16 0
#define NF4O_BF16 1
#define NF4O_F32 2

/* The 16 NF4 code points, as the fp32 bit patterns torch produces from the
 * decimal constants at kernel_optimized.py:234-239. */
static const uint32_t kNf4Bits[16] = {
    0xbf800000u, 0xbf3239b1u, 0xbf066b30u, 0xbeca32a0u,
    0xbe91a24du, 0xbe3d353fu, 0xbdba7871u, 0x00000000u,
    0x3da2faffu, 0x3e24cae3u, 0x3e7c04ddu, 0x3ead033au,
    0x3ee1a4b8u, 0x3f1007abu, 0x3f3913b3u, 0x3f800000u,
};

static float bits_to_f32(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f32_to_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

float nf4o_code(int i) { return bits_to_f32(kNf4Bits[i & 15]); }

/* fp32 -> bf16, round to nearest even.  NaN -> 0x7FC0 (torch's scalar rule;
 * torch's vectorised CPU path emits 0xFFFF instead, so tests compare NaN
 * positions, not NaN payloads). */
uint16_t nf4o_f32_to_bf16(float f) {
    uint32_t x = f32_to_bits(f);
    if ((x & 0x7FFFFFFFu) > 0x7F800000u) return 0x7FC0u;
    x += 0x7FFFu + ((x >> 16) & 1u);
    return (uint16_t)(x >> 16);
}

/* fp32 -> IEEE binary16, round to nearest even, with subnormals and overflow. */
uint16_t nf4o_f32_to_f16(float f) {
    uint32_t x = f32_to_bits(f);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7FFFFFFFu;
    if (ax > 0x7F800000u) return (uint16_t)(sign | 0x7E00u);        /* NaN */
    if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);       /* >= 65520 -> inf */
    if (ax < 0x38800000u) {                                          /* below 2^-14 */
        uint32_t e = ax >> 23;
        if (e < 102u) return (uint16_t)sign;                         /* < 2^-25 */
        uint32_t mant = (ax & 0x7FFFFFu) | 0x800000u;
        uint32_t shift = 126u - e;                                   /* 14..24 */
        uint32_t q = mant >> shift;
        uint32_t rem = mant & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1u);
        if (rem > half || (rem == half && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t r = ax - 0x38000000u;                                   /* rebias 127 -> 15 */
    r += 0xFFFu + ((r >> 13) & 1u);
    return (uint16_t)(sign | (r >> 13));
}

/* Store element i of the output as the requested dtype (fp32: unrounded). */
static inline void put(void* out, int64_t i, float v, int dtype) {
    if (dtype == NF4O_F32) ((float*)out)[i] = v;
    else if (dtype == NF4O_BF16) ((uint16_t*)out)[i] = nf4o_f32_to_bf16(v);
    else ((uint16_t*)out)[i] = nf4o_f32_to_f16(v);
}

/* Scale of one (row, 64-column block) under the reference's double-quant rule. */
float nf4o_ref_scale(const uint8_t* a1, int64_t nb, const float* a2, int64_t n2,
                     int64_t r, int64_t b, int64_t bpr) {
    int64_t g = (bpr + 3) / 4;
    float q = (float)a1[(r * bpr + b) % nb];
    float s1 = q / 127.0f;                 /* IEEE fp32 division (:45, :270) */
    return s1 * a2[(r * g + b / 4) % n2];
}

/* One row-major [m, n] plane, scale per (row, block) supplied by `scale_of`. */
typedef float (*scale_fn)(const void* ctx, int64_t r, int64_t b);

/* Rows are independent, so the CPU-baseline form splits them over
 * OpenMP threads; the arithmetic per element is identical for any thread count. */
static int g_threads = 1;
void nf4o_set_threads(int t) { g_threads = t < 1 ? 1 : t; }

static int dequant_rows(const uint8_t* packed, int64_t packed_len, int64_t m, int64_t n,
                        void* out, int dtype, scale_fn sf, const void* ctx) {
    if (m <= 0 || n <= 0) return 0;
    if (packed_len % m) return -1;                    /* .view(m, -1) must succeed */
    int64_t stride = packed_len / m;
    if (stride < (n + 1) / 2) return -1;               /* row too short for n columns */
    int64_t bpr = (n + 63) / 64;
#pragma omp parallel for num_threads(g_threads) schedule(static) if (g_threads > 1)
    for (int64_t r = 0; r < m; ++r) {
        const uint8_t* row = packed + r * stride;
        for (int64_t b = 0; b < bpr; ++b) {
            float s = sf(ctx, r, b);
            int64_t c_end = (b + 1) * 64 < n ? (b + 1) * 64 : n;
            for (int64_t c = b * 64; c < c_end; ++c) {
                uint8_t byte = row[c >> 1];
                int nib = (c & 1) ? (byte & 0xF) : (byte >> 4);
                put(out, r * n + c, nf4o_code(nib) * s, dtype);
            }
        }
    }
    return 0;
}

struct ref_ctx { const uint8_t* a1; int64_t nb; const float* a2; int64_t n2; int64_t bpr; };
static float ref_scale_cb(const void* c, int64_t r, int64_t b) {
    const struct ref_ctx* x = (const struct ref_ctx*)c;
    return nf4o_ref_scale(x->a1, x->nb, x->a2, x->n2, r, b, x->bpr);
}

/* Reference double-dequant (the path the HIP kernel replaces). */
int nf4o_dequant_ref(const uint8_t* packed, int64_t packed_len,
                     const uint8_t* a1, int64_t nb, const float* a2, int64_t n2,
                     void* out, int dtype, int64_t m, int64_t n) {
    if (nb <= 0 || n2 <= 0) return -1;
    struct ref_ctx c = {a1, nb, a2, n2, (n + 63) / 64};
    return dequant_rows(packed, packed_len, m, n, out, dtype, ref_scale_cb, &c);
}

struct single_ctx { const float* absmax; int64_t row_stride; };
static float single_scale_cb(const void* c, int64_t r, int64_t b) {
    const struct single_ctx* x = (const struct single_ctx*)c;
    return x->absmax[r * x->row_stride + b];
}

/* Reference single-quant branch: absmax already fp32 [m, >= bpr] (:273-274). */
int nf4o_dequant_single(const uint8_t* packed, int64_t packed_len,
                        const float* absmax, int64_t absmax_len,
                        void* out, int dtype, int64_t m, int64_t n) {
    if (m <= 0 || n <= 0) return 0;
    if (absmax_len % m) return -1;
    int64_t rs = absmax_len / m;
    if (rs < (n + 63) / 64) return -1;
    struct single_ctx c = {absmax, rs};
    return dequant_rows(packed, packed_len, m, n, out, dtype, single_scale_cb, &c);
}

/* bitsandbytes semantics over the flat element stream (parity unpinned). */
int nf4o_dequant_bnb(const uint8_t* packed, const uint8_t* a1, int64_t nb,
                     const float* code2, const float* a2, int64_t n2, float offset,
                     void* out, int dtype, int64_t numel,
                     int64_t blocksize, int64_t blocksize2) {
    if (numel <= 0) return 0;
    if (blocksize <= 0 || blocksize2 <= 0) return -1;
    if ((numel + blocksize - 1) / blocksize > nb) return -1;
    if (((numel + blocksize - 1) / blocksize + blocksize2 - 1) / blocksize2 > n2) return -1;
#pragma omp parallel for num_threads(g_threads) schedule(static) if (g_threads > 1)
    for (int64_t k = 0; k < numel; ++k) {
        int64_t blk = k / blocksize;
        float am = code2[a1[blk]] * a2[blk / blocksize2];
        am = am + offset;
        uint8_t byte = packed[k >> 1];
        int nib = (k & 1) ? (byte & 0xF) : (byte >> 4);
        put(out, k, nf4o_code(nib) * am, dtype);
    }
    return 0;
}

/* bitsandbytes single-level (compress_statistics=False): absmax fp32 per block. */
int nf4o_dequant_bnb_single(const uint8_t* packed, const float* absmax, int64_t nabs,
                            void* out, int dtype, int64_t numel, int64_t blocksize) {
    if (numel <= 0) return 0;
    if (blocksize <= 0 || (numel + blocksize - 1) / blocksize > nabs) return -1;
#pragma omp parallel for num_threads(g_threads) schedule(static) if (g_threads > 1)
    for (int64_t k = 0; k < numel; ++k) {
        uint8_t byte = packed[k >> 1];
        int nib = (k & 1) ? (byte & 0xF) : (byte >> 4);
        put(out, k, nf4o_code(nib) * absmax[k / blocksize], dtype);
    }
    return 0;
}
