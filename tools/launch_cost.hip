// Host cost of one kernel launch on this ROCm build, by launch API (tools only):
//   hipLaunchKernelGGL (host-stub lookup per call), hipModuleLaunchKernel with the
//   hipFunction_t from hipGetFuncBySymbol cached once, and hipExtLaunchKernel.
// The kernel is the shape of nf4_flat_kernel's launch (2048 x 256 threads, a
// by-value argument block of the single-matrix Batch's size) but does nothing.
//   hipcc --offload-arch=gfx950 -O2 -o tools/_build/launch_cost tools/launch_cost.hip && tools/_build/launch_cost [grid]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

struct Args {
    unsigned char bytes[112];
};

__global__ void empty_kernel(const Args a) {
    if (a.bytes[0] == 0xFF && threadIdx.x == 1024) asm volatile("s_nop 0");
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const unsigned grid = argc > 1 ? (unsigned)std::atoi(argv[1]) : 2048u;
    hipStream_t st;
    if (hipStreamCreate(&st) != hipSuccess) return 1;
    Args a;
    std::memset(&a, 0, sizeof(a));
    const int n = 20000;
    hipFunction_t f = nullptr;
    if (hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(&empty_kernel)) != hipSuccess) {
        std::printf("{\"error\": \"hipGetFuncBySymbol\"}\n");
        return 1;
    }
    for (int rep = 0; rep < 3; ++rep) {
        // warm
        for (int i = 0; i < 1000; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, st, a);
        hipStreamSynchronize(st);
        double t0 = now_us();
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, st, a);
        double t1 = now_us();
        hipStreamSynchronize(st);
        double t2 = now_us();
        void* params[] = {&a};
        for (int i = 0; i < n; ++i) hipModuleLaunchKernel(f, grid, 1, 1, 256, 1, 1, 0, st, params, nullptr);
        double t3 = now_us();
        hipStreamSynchronize(st);
        double t4 = now_us();
        for (int i = 0; i < n; ++i)
            hipExtLaunchKernel(reinterpret_cast<const void*>(&empty_kernel), dim3(grid), dim3(256), params, 0, st,
                               nullptr, nullptr, 0);
        double t5 = now_us();
        hipStreamSynchronize(st);
        double t6 = now_us();
        std::printf("{\"grid\": %u, \"rep\": %d, \"hipLaunchKernelGGL_us\": %.3f, \"hipModuleLaunchKernel_cached_us\": %.3f, "
                    "\"hipExtLaunchKernel_us\": %.3f, \"launches\": %d, \"drain_us\": [%.1f, %.1f, %.1f]}\n",
                    grid, rep, (t1 - t0) / n, (t3 - t2) / n, (t5 - t4) / n, n, t2 - t1, t4 - t3, t6 - t5);
    }
    hipStreamDestroy(st);
    return 0;
}
