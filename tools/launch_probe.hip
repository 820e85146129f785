// Per-launch cost on gfx950 (developer tool): back-to-back dependent
// launches on one stream, timed with events over many iterations.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <chrono>

struct Big { uint64_t v[320]; };  // 2.5 KB of kernel arguments

__global__ void k_empty(int x) { if (x == 12345) asm volatile("s_nop 0"); }
__global__ void k_empty_big(Big b) { if (b.v[0] == 12345) asm volatile("s_nop 0"); }
__global__ void k_copy(ulonglong2* d, const ulonglong2* s, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

static hipStream_t gS = 0;
template <class F> float timeit(F f, int iters) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    f(); hipDeviceSynchronize();
    hipEventRecord(a, gS);
    for (int i = 0; i < iters; ++i) f();
    hipEventRecord(b, gS); hipEventSynchronize(b);
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
    // the engine's setting: a non-blocking stream, and a graph of 100 launches
    (void)hipStreamCreateWithFlags(&gS, hipStreamNonBlocking);
    std::printf("nb-stream empty      : %6.2f us\n", timeit([&] { hipLaunchKernelGGL(k_empty, 1, 64, 0, gS, 1); }, 2000));
    std::printf("nb-stream empty 4096 : %6.2f us\n", timeit([&] { hipLaunchKernelGGL(k_empty, 4096, 256, 0, gS, 1); }, 2000));
    const size_t n8 = (8u << 20) / 16;
    std::printf("nb-stream copy 8 MB  : %6.2f us\n", timeit([&] { hipLaunchKernelGGL(k_copy, 2048, 256, 0, gS, (ulonglong2*)x, (const ulonglong2*)y, n8); }, 500));
    for (int which = 0; which < 2; ++which) {
        hipGraph_t g; hipGraphExec_t ge;
        (void)hipStreamBeginCapture(gS, hipStreamCaptureModeGlobal);
        for (int i = 0; i < 100; ++i) {
            if (which == 0) hipLaunchKernelGGL(k_empty, 1, 64, 0, gS, 1);
            else hipLaunchKernelGGL(k_copy, 2048, 256, 0, gS, (ulonglong2*)x, (const ulonglong2*)y, n8);
        }
        (void)hipStreamEndCapture(gS, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        float us = timeit([&] { (void)hipGraphLaunch(ge, gS); }, 50) / 100.f;
        std::printf("graph x100 %-10s: %6.2f us per kernel\n", which ? "copy 8MB" : "empty", us);
    }
    // concurrency: 400 small copies (1 MB each) spread over S streams
    hipStream_t ss[8];
    for (int i = 0; i < 8; ++i) (void)hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking);
    const size_t n1 = (1u << 20) / 16;
    for (int S : {1, 2, 4, 8}) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipDeviceSynchronize();
            auto t0 = std::chrono::high_resolution_clock::now();
            for (int i = 0; i < 400; ++i) {
                const int s = i % S;
                hipLaunchKernelGGL(k_copy, 256, 256, 0, ss[s], (ulonglong2*)x + s * n1 * 2, (const ulonglong2*)y + s * n1 * 2, n1);
            }
            (void)hipDeviceSynchronize();
            auto t1 = std::chrono::high_resolution_clock::now();
            if (rep) std::printf("400 x copy 1MB over %d streams: %6.2f us per kernel\n", S,
                                 std::chrono::duration<double, std::micro>(t1 - t0).count() / 400);
        }
    }
    // GPU-side concurrency: a graph of S parallel chains x (400/S) small copies
    for (int S : {1, 2, 4, 8}) {
        hipGraph_t g; hipGraphExec_t ge;
        hipEvent_t fork, join[8];
        (void)hipEventCreateWithFlags(&fork, hipEventDisableTiming);
        for (int i = 0; i < 8; ++i) (void)hipEventCreateWithFlags(&join[i], hipEventDisableTiming);
        (void)hipStreamBeginCapture(ss[0], hipStreamCaptureModeGlobal);
        (void)hipEventRecord(fork, ss[0]);
        for (int b = 1; b < S; ++b) (void)hipStreamWaitEvent(ss[b], fork, 0);
        for (int i = 0; i < 400; ++i) {
            const int b = i % S;
            hipLaunchKernelGGL(k_copy, 256, 256, 0, ss[b], (ulonglong2*)x + b * n1 * 2, (const ulonglong2*)y + b * n1 * 2, n1);
        }
        for (int b = 1; b < S; ++b) { (void)hipEventRecord(join[b], ss[b]); (void)hipStreamWaitEvent(ss[0], join[b], 0); }
        (void)hipStreamEndCapture(ss[0], &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        gS = ss[0];
        float us = timeit([&] { (void)hipGraphLaunch(ge, ss[0]); }, 20) / 400.f;
        std::printf("graph 400 x copy 1MB in %d chains: %6.2f us per kernel\n", S, us);
    }
    return 0;
}
