// Multiply-accumulate rates for the integer base conversion (developer tool):
// a 60-bit x 60-bit -> 128-bit accumulation (the engine's macc), against the
// same product as three 20-bit limbs each side in exact FP64 (nine FMAs into
// five diagonal sums).
//   make -C tools macrate && tools/build/mac_rate
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

typedef unsigned long long u64;
constexpr int kIters = 2048;
constexpr int kChains = 4;

__global__ __launch_bounds__(256) void k_macc(u64* out, u64 seed) {
    u64 lo[kChains], hi[kChains], a[kChains];
    const u64 b = (seed * 0x9E3779B97F4A7C15ull) >> 4;
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
        lo[c] = hi[c] = 0;
        a[c] = ((seed + threadIdx.x * 977ull + c) * 0xD1B54A32D192ED03ull) >> 4;
    }
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            const u64 p = a[c] * b, ph = __umul64hi(a[c], b);
            lo[c] += p;
            hi[c] += ph + (lo[c] < p);
            a[c] += p >> 40;  // (next operand depends on the product: no hoisting)
        }
    }
    u64 s = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += lo[c] ^ hi[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fp3(double* out, double seed) {
    double d[kChains][5], y[kChains][3];
    const double m0 = 1048575.0, m1 = 777777.0, m2 = 123457.0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
#pragma unroll
        for (int j = 0; j < 5; ++j) d[c][j] = 0.0;
        y[c][0] = seed + threadIdx.x + c;
        y[c][1] = seed * 3 + c;
        y[c][2] = 17.0 + c;
    }
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            d[c][0] = fma(y[c][0], m0, d[c][0]);
            d[c][1] = fma(y[c][0], m1, fma(y[c][1], m0, d[c][1]));
            d[c][2] = fma(y[c][0], m2, fma(y[c][1], m1, fma(y[c][2], m0, d[c][2])));
            d[c][3] = fma(y[c][1], m2, fma(y[c][2], m1, d[c][3]));
            d[c][4] = fma(y[c][2], m2, d[c][4]);
            y[c][0] = d[c][4] * 1e-30;  // (dependent operands)
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c)
#pragma unroll
        for (int j = 0; j < 5; ++j) s += d[c][j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 16;
    void* out;
    hipMalloc(&out, (size_t)blocks * 256 * 8);
    auto run = [&](const char* name, auto launch) {
        launch();
        hipDeviceSynchronize();
        auto t0 = std::chrono::high_resolution_clock::now();
        for (int r = 0; r < 5; ++r) launch();
        hipDeviceSynchronize();
        auto t1 = std::chrono::high_resolution_clock::now();
        const double s = std::chrono::duration<double>(t1 - t0).count() / 5;
        const double macs = (double)blocks * 256 * kIters * kChains;
        std::printf("%-28s %8.3f ms  %8.1f G MAC/s\n", name, s * 1e3, macs / s / 1e9);
    };
    run("macc 64x64->128", [&] { hipLaunchKernelGGL(k_macc, dim3(blocks), dim3(256), 0, 0, (u64*)out, 12345ull); });
    run("fp64 3x3 limbs (9 fma)", [&] { hipLaunchKernelGGL(k_fp3, dim3(blocks), dim3(256), 0, 0, (double*)out, 3.0); });
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) std::printf("ERROR %s\n", hipGetErrorString(e));
    hipFree(out);
    return e == hipSuccess ? 0 : 1;
}
