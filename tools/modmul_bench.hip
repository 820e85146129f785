// Throughput of modular-multiply formulations on gfx950 (developer tool).
//   hipcc --offload-arch=gfx950 -O3 tools/modmul_bench.hip -o tools/build/modmul_bench
// Each thread runs 4 independent chains of `iters` multiplications by a fixed
// twiddle (the NTT butterfly's multiply).  Prints Gmodmul/s for:
//   shoup64  : 64-bit Shoup (q < 2^62), integer multiplies
//   fp64     : double-precision FMA form (q < 2^50), operands held as doubles
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>

typedef uint64_t u64;

__device__ __forceinline__ u64 shoup(u64 a, u64 w, u64 wp, u64 q) {
    u64 qh = __umul64hi(a, wp);
    u64 r = a * w - qh * q;
    return r >= q ? r - q : r;
}

__device__ __forceinline__ u64 a_lazy(u64 a, u64 w, u64 wp, u64 q) {
    return a * w - __umul64hi(a, wp) * q;
}

__global__ void k_shoup(u64* out, u64 w, u64 wp, u64 q, int iters) {
    u64 a0 = threadIdx.x + 1, a1 = a0 + 7, a2 = a0 + 11, a3 = a0 + 13;
    for (int i = 0; i < iters; ++i) {
        a0 = shoup(a0, w, wp, q);
        a1 = shoup(a1, w, wp, q);
        a2 = shoup(a2, w, wp, q);
        a3 = shoup(a3, w, wp, q);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3;
}

__device__ __forceinline__ double fmod_mul(double a, double w, double wq, double q) {
    const double hi = a * w;
    const double lo = fma(a, w, -hi);
    const double qq = rint(a * wq);
    double r = fma(-qq, q, hi) + lo;
    r = r < 0 ? r + q : r;
    r = r >= q ? r - q : r;
    return r;
}

// signed lazy form: |a| < 2^12 q, result in (-q, q), no corrections
__device__ __forceinline__ double fmod_mul_lazy(double a, double w, double wq, double q) {
    const double hi = a * w;
    const double lo = fma(a, w, -hi);
    const double qq = rint(a * wq);
    return fma(-qq, q, hi) + lo;
}

__global__ void k_fp64lazy(double* out, double w, double wq, double q, int iters) {
    double a0 = threadIdx.x + 1, a1 = a0 + 7, a2 = a0 + 11, a3 = a0 + 13;
    for (int i = 0; i < iters; ++i) {
        a0 = fmod_mul_lazy(a0, w, wq, q);
        a1 = fmod_mul_lazy(a1, w, wq, q);
        a2 = fmod_mul_lazy(a2, w, wq, q);
        a3 = fmod_mul_lazy(a3, w, wq, q);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3;
}

// a full lazy CT butterfly pair in FP64 (x +- y*w), 4 independent butterflies
__global__ void k_fp64bfly(double* out, double w, double wq, double q, int iters) {
    double x0 = threadIdx.x + 1, y0 = x0 + 7, x1 = x0 + 11, y1 = x0 + 13;
    for (int i = 0; i < iters; ++i) {
        double r0 = fmod_mul_lazy(y0, w, wq, q), r1 = fmod_mul_lazy(y1, w, wq, q);
        double nx0 = x0 + r0, ny0 = x0 - r0, nx1 = x1 + r1, ny1 = x1 - r1;
        x0 = nx0 - q * rint(nx0 * (1.0 / q)); y0 = ny0; x1 = nx1; y1 = ny1 - q * rint(ny1 * (1.0 / q));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + y0 + x1 + y1;
}

// the integer lazy CT butterfly as the NTT kernel runs it
__global__ void k_intbfly(u64* out, u64 w, u64 wp, u64 q, int iters) {
    u64 x0 = threadIdx.x + 1, y0 = x0 + 7, x1 = x0 + 11, y1 = x0 + 13;
    const u64 q2 = 2 * q;
    for (int i = 0; i < iters; ++i) {
        u64 X0 = x0 >= q2 ? x0 - q2 : x0, X1 = x1 >= q2 ? x1 - q2 : x1;
        u64 r0 = a_lazy(y0, w, wp, q), r1 = a_lazy(y1, w, wp, q);
        x0 = X0 + r0; y0 = X0 - r0 + q2; x1 = X1 + r1; y1 = X1 - r1 + q2;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ y0 ^ x1 ^ y1;
}

__global__ void k_fp64(double* out, double w, double wq, double q, int iters) {
    double a0 = threadIdx.x + 1, a1 = a0 + 7, a2 = a0 + 11, a3 = a0 + 13;
    for (int i = 0; i < iters; ++i) {
        a0 = fmod_mul(a0, w, wq, q);
        a1 = fmod_mul(a1, w, wq, q);
        a2 = fmod_mul(a2, w, wq, q);
        a3 = fmod_mul(a3, w, wq, q);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3;
}

int main() {
    const int blocks = 256 * 16, threads = 256, iters = 4096;
    void* buf;
    hipMalloc(&buf, (size_t)blocks * threads * 8);
    const u64 q60 = 1152921504606584833ull;  // 60-bit NTT prime
    const u64 w = 123456789012345ull % q60;
    const u64 wp = (u64)(((unsigned __int128)w << 64) / q60);
    const double q50 = 1125899906826241.0;   // < 2^50
    const double wd = 98765432109.0, wq = wd / q50;
    const double total = (double)blocks * threads * iters * 4;
    for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        float ms;
        hipEventRecord(a);
        hipLaunchKernelGGL(k_shoup, dim3(blocks), dim3(threads), 0, 0, (u64*)buf, w, wp, q60, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        std::printf("shoup64 : %8.1f Gmodmul/s (%.3f ms)\n", total / ms / 1e6, ms);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_fp64, dim3(blocks), dim3(threads), 0, 0, (double*)buf, wd, wq, q50, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        std::printf("fp64    : %8.1f Gmodmul/s (%.3f ms)\n", total / ms / 1e6, ms);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_fp64lazy, dim3(blocks), dim3(threads), 0, 0, (double*)buf, wd, wq, q50, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        std::printf("fp64lazy: %8.1f Gmodmul/s (%.3f ms)\n", total / ms / 1e6, ms);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_intbfly, dim3(blocks), dim3(threads), 0, 0, (u64*)buf, w, wp, q60, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        std::printf("int bfly: %8.1f Gbutterfly/s (%.3f ms)\n", total / 2 / ms / 1e6, ms);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_fp64bfly, dim3(blocks), dim3(threads), 0, 0, (double*)buf, wd, wq, q50, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        std::printf("fp bfly : %8.1f Gbutterfly/s (%.3f ms)\n", total / 2 / ms / 1e6, ms);
    }
    return 0;
}
