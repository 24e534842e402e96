// Load-pattern microbenchmark for the fused GEMM's weight stream (tools only).
// Each wave reads `cnt` chunks of a 16-row strip (one 128-byte line per row
// per chunk) of a [rows][row_bytes] matrix and folds the bytes into one value
// so that nothing is optimised away.  Patterns:
//   0  MFMA fragment order: lane (n = l & 15, kq = l >> 4) loads 2 x 16 B at
//      row n, bytes 32 kq .. 32 kq + 32 (what nf4_gemm_stream/persist do)
//   1  coalesced: instruction i, lane l loads row 8 i + (l >> 3), 16 B piece l & 7
//      (each 16-lane group reads two whole lines)
//   2  prepacked: the chunk's 2 KiB are contiguous, instruction i lane l at i*1024 + 16 l
//   3  pattern 0 with contiguous chunk ranges per part (part p: chunks [p cnt, p cnt + cnt))
//   4  pattern 3 with the range walked from a per-strip rotation (strip mod cnt)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int PAT, int P>
__global__ __launch_bounds__(256) void lp_kernel(const uint8_t* w, uint32_t rows, uint32_t row_bytes,
                                                 uint32_t strips_per_wave_group, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t strip = wave % (rows / 16u);
    const uint32_t part = wave / (rows / 16u);
    const uint32_t chunks = row_bytes / 128u;
    const uint32_t parts = strips_per_wave_group;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, rows * row_bytes, 0x00020000);
    uint32_t acc = 0;
    const uint32_t cnt = (chunks + parts - 1) / parts;
    if constexpr (PAT >= 3) {
        const uint32_t rot = PAT == 4 ? strip % cnt : 0u;
        for (uint32_t j0 = 0; j0 < cnt; j0 += P) {
            u32x4 v[P][2];
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const uint32_t j = j0 + p;
                const uint32_t jr = j + rot < cnt ? j + rot : j + rot - cnt;
                const uint32_t c = part * cnt + jr;
                const bool ok = j < cnt && c < chunks;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const uint32_t off = (strip * 16u + (lane & 15u)) * row_bytes + c * 128u + (lane >> 4) * 32u + 16u * i;
                    v[p][i] = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? off : 0x80000000u, 0, 0);
                }
            }
#pragma unroll
            for (int p = 0; p < P; ++p) acc ^= v[p][0].x ^ v[p][0].w ^ v[p][1].y ^ v[p][1].z;
        }
        if (acc == 0x12345678u) out[0] = acc;
        return;
    }
    for (uint32_t c0 = part; c0 < chunks; c0 += parts * P) {
        u32x4 v[P][2];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const uint32_t c = c0 + p * parts;
            const bool ok = c < chunks;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                uint32_t off;
                if constexpr (PAT == 0) {
                    off = (strip * 16u + (lane & 15u)) * row_bytes + c * 128u + (lane >> 4) * 32u + 16u * i;
                } else if constexpr (PAT == 1) {
                    off = (strip * 16u + 8u * i + (lane >> 3)) * row_bytes + c * 128u + (lane & 7u) * 16u;
                } else {
                    off = (strip * chunks + c) * 2048u + i * 1024u + lane * 16u;
                }
                v[p][i] = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? off : 0x80000000u, 0, 0);
            }
        }
#pragma unroll
        for (int p = 0; p < P; ++p) acc ^= v[p][0].x ^ v[p][0].w ^ v[p][1].y ^ v[p][1].z;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

extern "C" int lp_launch(int pat, int depth, const void* w, uint32_t rows, uint32_t row_bytes, uint32_t parts,
                         void* out, void* stream) {
    const uint32_t waves = (rows / 16u) * parts;
    const dim3 grid((waves + 3) / 4), block(256);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define L_(PA, PP) hipLaunchKernelGGL((lp_kernel<PA, PP>), grid, block, 0, st, (const uint8_t*)w, rows, row_bytes, parts, (uint32_t*)out)
    if (depth == 2) {
        if (pat == 0) L_(0, 2); else if (pat == 1) L_(1, 2); else if (pat == 2) L_(2, 2); else if (pat == 3) L_(3, 2); else L_(4, 2);
    } else {
        if (pat == 0) L_(0, 4); else if (pat == 1) L_(1, 4); else if (pat == 2) L_(2, 4); else if (pat == 3) L_(3, 4); else L_(4, 4);
    }
#undef L_
    return (int)hipGetLastError();
}
