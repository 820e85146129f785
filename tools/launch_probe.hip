// Per-launch cost on gfx950 (developer tool): back-to-back dependent
// launches on one stream, timed with events over many iterations.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct Big { uint64_t v[320]; };  // 2.5 KB of kernel arguments

__global__ void k_empty(int x) { if (x == 12345) asm volatile("s_nop 0"); }
__global__ void k_empty_big(Big b) { if (b.v[0] == 12345) asm volatile("s_nop 0"); }
__global__ void k_copy(ulonglong2* d, const ulonglong2* s, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

template <class F> float timeit(F f, int iters) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    f(); hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < iters; ++i) f();
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / iters;
}

int main() {
    void *x, *y;
    (void)hipMalloc(&x, 256 << 20); (void)hipMalloc(&y, 256 << 20);
    Big big{};
    std::printf("empty (4 B args)     : %6.2f us\n", timeit([&] { hipLaunchKernelGGL(k_empty, 1, 64, 0, 0, 1); }, 2000));
    std::printf("empty (2.5 KB args)  : %6.2f us\n", timeit([&] { hipLaunchKernelGGL(k_empty_big, 1, 64, 0, 0, big); }, 2000));
    std::printf("empty 4096 blocks    : %6.2f us\n", timeit([&] { hipLaunchKernelGGL(k_empty, 4096, 256, 0, 0, 1); }, 2000));
    for (size_t kb : {64, 512, 4096, 32768, 131072}) {
        size_t n = kb * 1024 / 16;
        unsigned blocks = (unsigned)((n + 255) / 256); if (blocks > 8192) blocks = 8192;
        float us = timeit([&] { hipLaunchKernelGGL(k_copy, blocks, 256, 0, 0, (ulonglong2*)x, (const ulonglong2*)y, n); }, 500);
        std::printf("copy %7zu KB       : %6.2f us  (%.0f GB/s r+w)\n", kb, us, 2.0 * kb * 1024 / us / 1e3);
    }
    return 0;
}
