// PMC calibration kernels (tools only, not product): stream a known byte count
// with the dequant kernel's exact access shapes, so FETCH_SIZE / WRITE_SIZE can
// be scaled to bytes for those shapes (MI355X_MICROARCH.md: counters are exact
// only for 16 B/lane streams; other widths must be calibrated).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Reads `nbytes` with 4 B/lane buffer_load_dword, 256 contiguous bytes per wave
// instruction, nt policy (the packed-weight load shape and policy, round 4); writes one
// dword per wave.
__global__ __launch_bounds__(256) void calib_read_dword(const uint32_t* p, uint32_t nbytes, uint32_t* sink) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, nbytes, 0x00020000);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * 4;
    uint32_t acc = 0;
    for (uint32_t base = wave * 2048u; base < nbytes; base += nw * 2048u) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, base + 256u * j + 4u * lane, 0, 2);
    }
    if (acc == 0x9E3779B9u) sink[wave] = acc;  // practically never: keeps the loads alive
}

// Writes `nbytes` with 16 B/lane sc1+nt buffer stores (the product default, aux 18), 1 KiB contiguous per wave
// instruction (the output store shape).
__global__ __launch_bounds__(256) void calib_write_x4(uint32_t* p, uint32_t nbytes) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, nbytes, 0x00020000);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * 4;
    const u32x4 v = {lane, wave, 1u, 2u};
    for (uint32_t base = wave * 8192u; base < nbytes; base += nw * 8192u) {
#pragma unroll
        for (int j = 0; j < 8; ++j) __builtin_amdgcn_raw_buffer_store_b128(v, r, base + 1024u * j + 16u * lane, 0, 18);
    }
}

extern "C" int calib_read(const void* p, uint32_t nbytes, void* sink, void* stream) {
    hipLaunchKernelGGL(calib_read_dword, dim3(2048), dim3(256), 0, (hipStream_t)stream, (const uint32_t*)p, nbytes,
                       (uint32_t*)sink);
    return (int)hipGetLastError();
}

extern "C" int calib_write(void* p, uint32_t nbytes, void* stream) {
    hipLaunchKernelGGL(calib_write_x4, dim3(2048), dim3(256), 0, (hipStream_t)stream, (uint32_t*)p, nbytes);
    return (int)hipGetLastError();
}

// Speed-of-light twin of nf4_flat_kernel: the same loads (4 B/lane, 256 B per
// wave instruction) and the same stores (16 B/lane, 1 KiB per wave instruction,
// sc1+nt), no decode -- what the memory system gives this access mix.
__global__ __launch_bounds__(256) void calib_mix(const uint32_t* p, uint32_t nbytes, uint32_t* o) {
    __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, nbytes, 0x00020000);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)o, 0, nbytes * 4u, 0x00020000);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t base = wave * 1024u; base < nbytes; base += nw * 1024u) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = __builtin_amdgcn_raw_buffer_load_b32(rp, base + 256u * j + 4u * lane, 0, 2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32x4 v = {w[j], w[j] ^ 1u, w[j] ^ 2u, w[j] ^ 3u};
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, (base + 256u * j + 4u * lane) * 4u, 0, 18);
        }
    }
}

extern "C" int calib_mix_launch(const void* p, uint32_t nbytes, void* o, void* stream) {
    const uint32_t tiles = (nbytes + 1023u) / 1024u;
    hipLaunchKernelGGL(calib_mix, dim3((tiles + 3) / 4), dim3(256), 0, (hipStream_t)stream, (const uint32_t*)p, nbytes,
                       (uint32_t*)o);
    return (int)hipGetLastError();
}

// Twin of a 16 B/lane load shape: lane l reads packed bytes tile+16l..+15 (one
// 1 KiB-contiguous b128 load per wave) and writes its 64 output bytes as four b128
// sc1+nt stores at 4*tile + 64l + 16s (each store instruction strided by 64 B; the
// four together cover the wave's 4 KiB). Probes whether fewer, wider loads beat the
// 4 B/lane shape of nf4_flat_kernel at one tile per wave.
__global__ __launch_bounds__(256) void calib_mix16(const uint32_t* p, uint32_t nbytes, uint32_t* o) {
    __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, nbytes, 0x00020000);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)o, 0, nbytes * 4u, 0x00020000);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t base = wave * 1024u; base < nbytes; base += nw * 1024u) {
        const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(rp, base + 16u * lane, 0, 0);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const u32x4 v = {w[s], w[s] ^ 1u, w[s] ^ 2u, w[s] ^ 3u};
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, (base + 16u * lane) * 4u + 16u * s, 0, 18);
        }
    }
}

extern "C" int calib_mix16_launch(const void* p, uint32_t nbytes, void* o, void* stream) {
    const uint32_t tiles = (nbytes + 1023u) / 1024u;
    hipLaunchKernelGGL(calib_mix16, dim3((tiles + 3) / 4), dim3(256), 0, (hipStream_t)stream, (const uint32_t*)p,
                       nbytes, (uint32_t*)o);
    return (int)hipGetLastError();
}
