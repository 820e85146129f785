// FP64 instruction-rate probe (gfx950): throughput of v_rndne_f64 against
// v_add_f64 / v_fma_f64, and of the two quotient forms fpMulMod can use:
// rint(t) and (t + 1.5*2^52) - 1.5*2^52 (identical for |t| < 2^51).
//   hipcc --offload-arch=gfx950 -O3 tools/fp64_rate.hip -o tools/build/fp64_rate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 4096;
constexpr int kChains = 8;

template <int OP>
__global__ __launch_bounds__(256) void k_rate(double* out, double seed) {
    double v[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) v[c] = seed + threadIdx.x * 1e-3 + c;
    const double M = 6755399441055744.0;  // 1.5 * 2^52
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            if (OP == 0) v[c] = __builtin_rint(v[c] * 1.0000001);      // mul + rndne
            if (OP == 1) v[c] = ((v[c] * 1.0000001) + M) - M;          // mul + add + add
            if (OP == 2) v[c] = v[c] * 1.0000001 + 0.5;                // mul + add (or fma)
            if (OP == 3) v[c] = __builtin_rint(v[c]) + 0.5;            // rndne + add
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += v[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
static float run(double* out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.0);
    hipEventRecord(a, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.0);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const int blocks = 256 * 8;
    double* out = nullptr;
    if (hipMalloc(&out, (size_t)blocks * 256 * 8) != hipSuccess) return 1;
    const double ops = (double)blocks * 256 * kIters * kChains;  // chain steps
    const char* names[4] = {"mul+rndne", "mul+add+add (magic)", "mul+add", "rndne+add"};
    float t[4] = {run<0>(out, blocks), run<1>(out, blocks), run<2>(out, blocks), run<3>(out, blocks)};
    for (int k = 0; k < 4; ++k)
        std::printf("%-22s %8.3f ms  %7.2f G steps/s\n", names[k], t[k], ops / t[k] / 1e6);
    hipFree(out);
    return 0;
}
