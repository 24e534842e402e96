// Sanitizer harness for the library's host path (test infrastructure only).
//
// tests/test_cpu_sanitizers.py compiles this file together with the product
// source csrc/nf4_dequant_cpu.cpp and the C oracle (oracle/nf4_oracle.c, the
// checker) under -fsanitize=address,undefined and runs it: every case below goes
// through nf4_dequant_ref_cpu / nf4_dequant_single_cpu with exactly-sized heap
// buffers (so any read or write past an input or output is an ASan report) and
// must match the oracle bit for bit.  Cases: partial 64-blocks, odd n and padded
// packed rows (row stride > n/2), absmax / nested absmax shorter than the matrix
// (the reference's repeat-wrap, kernel_optimized.py:173-186), the single-quant
// branch (:273-274), every output dtype, and 1 / 3 / 0 (= all) worker threads,
// plus the argument errors (no memory touched).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <memory>
#include <vector>

#include "../../include/nf4_dequant.h"

extern "C" {
int nf4o_dequant_ref(const uint8_t* packed, int64_t packed_len, const uint8_t* a1, int64_t nb, const float* a2,
                     int64_t n2, void* out, int dtype, int64_t m, int64_t n);
int nf4o_dequant_single(const uint8_t* packed, int64_t packed_len, const float* absmax, int64_t absmax_len,
                        void* out, int dtype, int64_t m, int64_t n);
}

namespace {

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// exactly-sized heap copies: one element past the end is outside the allocation
template <class T>
std::unique_ptr<T[]> heap(size_t n) {
    return std::unique_ptr<T[]>(new T[n > 0 ? n : 1]);
}

int g_fail = 0, g_cases = 0;

size_t elem_bytes(int dt) { return dt == NF4DQ_F32 ? 4 : 2; }

void check(const char* what, int64_t m, int64_t n, int dt, int threads, const void* got, const void* want,
           int rc_got, int rc_want) {
    ++g_cases;
    const size_t bytes = (size_t)(m * n) * elem_bytes(dt);
    if ((rc_got != 0) != (rc_want != 0) || (rc_got == 0 && memcmp(got, want, bytes) != 0)) {
        ++g_fail;
        fprintf(stderr, "MISMATCH %s m=%lld n=%lld dt=%d threads=%d rc=%d/%d\n", what, (long long)m, (long long)n, dt,
                threads, rc_got, rc_want);
    }
}

void ref_case(int64_t m, int64_t n, int64_t stride, int64_t nb, int64_t n2, uint64_t seed) {
    uint64_t s = seed;
    const int64_t plen = m * stride;
    auto q = heap<uint8_t>((size_t)plen);
    auto a1 = heap<uint8_t>((size_t)nb);
    auto a2 = heap<float>((size_t)n2);
    for (int64_t i = 0; i < plen; ++i) q[i] = (uint8_t)splitmix(s);
    for (int64_t i = 0; i < nb; ++i) a1[i] = (uint8_t)splitmix(s);
    for (int64_t i = 0; i < n2; ++i) a2[i] = (float)((int64_t)(splitmix(s) % 20001) - 10000) * 1e-4f;
    for (int dt : {NF4DQ_F16, NF4DQ_BF16, NF4DQ_F32}) {
        const size_t ob = (size_t)(m * n) * elem_bytes(dt);
        auto want = heap<uint8_t>(ob);
        const int rw = nf4o_dequant_ref(q.get(), plen, a1.get(), nb, a2.get(), n2, want.get(), dt, m, n);
        for (int threads : {1, 3, 0}) {
            auto got = heap<uint8_t>(ob);
            const int rg = nf4_dequant_ref_cpu(q.get(), plen, a1.get(), nb, a2.get(), n2, got.get(), dt, m, n, threads);
            check("ref", m, n, dt, threads, got.get(), want.get(), rg, rw);
        }
    }
}

void single_case(int64_t m, int64_t n, int64_t stride, int64_t row_scales, uint64_t seed) {
    uint64_t s = seed;
    const int64_t plen = m * stride, alen = m * row_scales;
    auto q = heap<uint8_t>((size_t)plen);
    auto ab = heap<float>((size_t)alen);
    for (int64_t i = 0; i < plen; ++i) q[i] = (uint8_t)splitmix(s);
    for (int64_t i = 0; i < alen; ++i) ab[i] = (float)((int64_t)(splitmix(s) % 2001) - 1000) * 1e-3f;
    for (int dt : {NF4DQ_F16, NF4DQ_BF16, NF4DQ_F32}) {
        const size_t ob = (size_t)(m * n) * elem_bytes(dt);
        auto want = heap<uint8_t>(ob);
        const int rw = nf4o_dequant_single(q.get(), plen, ab.get(), alen, want.get(), dt, m, n);
        for (int threads : {1, 3}) {
            auto got = heap<uint8_t>(ob);
            const int rg = nf4_dequant_single_cpu(q.get(), plen, ab.get(), alen, got.get(), dt, m, n, threads);
            check("single", m, n, dt, threads, got.get(), want.get(), rg, rw);
        }
    }
}

}  // namespace

int main() {
    // (m, n, packed row stride, nb, n2): real bitsandbytes counts, partial blocks,
    // odd n with a padded row, and wrapping absmax / nested absmax
    const struct {
        int64_t m, n, stride, nb, n2;
    } refs[] = {
        {16, 128, 64, 32, 1},      {64, 512, 256, 512, 2},   {8, 96, 48, 9, 1},      {3, 128, 64, 6, 1},
        {5, 11008, 5504, 860, 4},  {7, 65, 33, 14, 1},        {9, 200, 110, 27, 2},   {1, 64, 32, 1, 1},
        {33, 4096, 2048, 37, 5},   {128, 1024, 512, 2048, 8}, {2, 6, 3, 1, 1},        {40, 2112, 1056, 1320, 6},
    };
    uint64_t seed = 17;
    for (const auto& c : refs) ref_case(c.m, c.n, c.stride, c.nb, c.n2, seed++);
    single_case(12, 256, 128, 4, 91);
    single_case(6, 200, 100, 5, 92);
    single_case(9, 130, 66, 3, 93);
    // argument errors: the library returns an error code and touches nothing
    {
        uint8_t q[8] = {0}, a1[2] = {1, 2};
        float a2[1] = {1.0f};
        uint16_t out[16];
        int bad = 0;
        bad += nf4_dequant_ref_cpu(q, 7, a1, 2, a2, 1, out, NF4DQ_BF16, 2, 8, 1) == 0;   // 7 % 2 != 0
        bad += nf4_dequant_ref_cpu(q, 8, a1, 0, a2, 1, out, NF4DQ_BF16, 2, 8, 1) == 0;   // empty absmax
        bad += nf4_dequant_ref_cpu(q, 8, a1, 2, a2, 1, out, 7, 2, 8, 1) == 0;            // unknown dtype
        bad += nf4_dequant_ref_cpu(q, 8, a1, 2, a2, 1, out, NF4DQ_BF16, 2, 16, 1) == 0;  // row too short
        ++g_cases;
        if (bad) {
            ++g_fail;
            fprintf(stderr, "argument errors accepted: %d\n", bad);
        }
    }
    printf("{\"cases\": %d, \"failures\": %d}\n", g_cases, g_fail);
    return g_fail ? 1 : 0;
}
