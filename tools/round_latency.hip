// Latency of one NTT-style register round against the number of resident
// blocks (developer tool).  A round = four doubles per
// thread read from LDS (XOR-swizzled), two radix-2 FP64 butterfly stages
// (fpMulMod: the product, its exact low part, the rint quotient), four
// writes, a barrier -- k_ntt's ROW round without its HBM traffic.  Each block
// runs R rounds; thread 0 records the shader clocks (clock64) and the 100 MHz
// real-time counter (wall_clock64) around them.
//   make -C tools roundlat && tools/build/round_latency
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kThreads = 256, kWords = 1024, kRounds = 64;

// MAGIC: the quotient rounded by adding and subtracting 1.5 * 2^52 (two
// adds, the same result for |t| < 2^51) instead of v_rndne_f64
template <bool MAGIC>
__device__ __forceinline__ double fpMulMod(double y, double w, double wq, double q) {
    const double hi = y * w;
    const double lo = fma(y, w, -hi);
    double qq;
    if (MAGIC) {
        const double M = 6755399441055744.0;
        qq = __builtin_fma(y, wq, M) - M;  // (the product and the first add fused)
    } else {
        qq = rint(y * wq);
    }
    return fma(-qq, q, hi) + lo;
}

template <bool MAGIC>
__global__ __launch_bounds__(kThreads) void k_rounds(double* out, unsigned long long* clk, double q, double w0) {
    __shared__ double s[kWords];
    const uint32_t t = threadIdx.x;
    for (uint32_t e = t; e < kWords; e += kThreads) s[e] = (double)((e * 2654435761u) % 1000003u);
    __syncthreads();
    const double qi = 1.0 / q;
    double w[3] = {w0, w0 * 3.0 - q * floor(w0 * 3.0 / q), w0 * 5.0 - q * floor(w0 * 5.0 / q)};
    const unsigned long long c0 = clock64(), r0 = wall_clock64();
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t h = 1u << (r & 7);  // stride of this round's butterflies
        const uint32_t a = ((t & ~(h - 1)) << 2) | (t & (h - 1));
        double v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = s[(a + j * h) & (kWords - 1)];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const int half = st == 0 ? 2 : 1;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (j & half) continue;
                const double W = w[st + (j >> 1) * st], WQ = W * qi;
                const double X = v[j], Y = fpMulMod<MAGIC>(v[j + half], W, WQ, q);
                v[j] = X + Y;
                v[j + half] = X - Y;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) s[(a + j * h) & (kWords - 1)] = v[j] - q * floor(v[j] * qi);
        __syncthreads();
    }
    const unsigned long long c1 = clock64(), r1 = wall_clock64();
    if (t == 0) {
        clk[2 * blockIdx.x] = c1 - c0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
    out[blockIdx.x * kThreads + t] = s[t];
}

int main() {
    const double q = 4398046511093.0;  // a prime below 2^42
    const int maxBlocks = 8192;
    double* out;
    unsigned long long* clk;
    hipMalloc(&out, (size_t)maxBlocks * kThreads * 8);
    hipMalloc(&clk, (size_t)maxBlocks * 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::printf("%6s %7s %12s %14s %16s %14s\n", "quot", "blocks", "clk/round", "rt-us/round", "wall-us/launch", "wall-us/round");
    for (int magic = 0; magic < 2; ++magic)
    for (int g : {16, 64, 256, 1024, 2048, 4096, 8192}) {
        auto k = magic ? k_rounds<true> : k_rounds<false>;
        hipLaunchKernelGGL(k, dim3(g), dim3(kThreads), 0, 0, out, clk, q, 123456789.0);
        hipDeviceSynchronize();
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k, dim3(g), dim3(kThreads), 0, 0, out, clk, q, 123456789.0);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<unsigned long long> h(2 * g);
        hipMemcpy(h.data(), clk, 16 * (size_t)g, hipMemcpyDeviceToHost);
        double c = 0, rt = 0;
        for (int b = 0; b < g; ++b) {
            c += (double)h[2 * b];
            rt += (double)h[2 * b + 1];
        }
        c /= g;
        rt /= g;
        std::printf("%6s %7d %12.0f %14.3f %16.2f %14.3f\n", magic ? "magic" : "rint", g, c / kRounds, rt / kRounds / 100.0, ms * 1e3,
                    ms * 1e3 / kRounds);
    }
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) std::printf("ERROR %s\n", hipGetErrorString(err));
    hipFree(out);
    hipFree(clk);
    return err == hipSuccess ? 0 : 1;
}
