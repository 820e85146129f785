// FETCH_SIZE calibration for the access widths the NTT uses (developer tool).
// MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a 16-B-per-lane
// coalesced stream; other widths are uncalibrated.  Each kernel here reads a
// known number of distinct bytes once; run under
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d D -o run -- tools/build/fetch_calib
// and divide FETCH_SIZE (KiB) by the bytes printed per kernel.
//   k_stream16: 16 B per lane, contiguous (the NTT tiles)
//   k_stream8:  8 B per lane, contiguous
//   k_rowtw:    the ROW pass's stage 8-13 twiddle gathers (rowTwIssue's
//               rounds 0-2: per 256-word row, entries 2^(S+k) + row 2^k + v,
//               k < 6, read by the row's 64 lanes with repeats), over every
//               row of 48 primes' tables -- the distinct bytes are 63 entries
//               per row
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned long long u64;

__global__ void k_stream16(const ulonglong2* __restrict__ a, size_t n2, u64* __restrict__ out) {
    u64 s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
        const ulonglong2 v = a[i];
        s += v.x ^ v.y;
    }
    if (s == 0x123456789ull) out[0] = s;  // (keeps the loads)
}

__global__ void k_stream8(const u64* __restrict__ a, size_t n, u64* __restrict__ out) {
    u64 s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 0x123456789ull) out[0] = s;
}

// one block = 4 rows of one prime (TILE 1024, 256 threads, as the ROW pass);
// grid = primes * (R / 4)
__global__ void k_rowtw(const double* __restrict__ tab, uint32_t logn, u64* __restrict__ out) {
    const uint32_t n = 1u << logn, S0 = logn - 8, R = n >> 8;
    const uint32_t prime = blockIdx.x / (R / 4), tile = blockIdx.x % (R / 4);
    const double* gd = tab + (size_t)prime * n;
    const uint32_t gid = threadIdx.x;
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const uint32_t k0 = 2 * r, logh = 8 - k0 - 2;
        const uint32_t lo = gid & ((1u << logh) - 1);
        const uint32_t hi = (gid >> logh) & ((1u << k0) - 1);
        const uint32_t u = hi * (256u >> k0) + lo;
        const uint32_t x0 = (tile * 4 + (gid >> 6)) * 256u + u;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const uint32_t k = k0 + t;
            const uint32_t b = (1u << (S0 + k)) + (x0 >> (8 - k));
#pragma unroll
            for (int qd = 0; qd < (1 << t); ++qd) acc += gd[b + qd];
        }
    }
    if (acc == 1.2345) out[0] = 1;
}

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? (size_t)std::atoi(argv[1]) : 1024;  // stream size, MiB
    const uint32_t logn = 16, primes = 48, n = 1u << logn;
    const size_t bytes = mb << 20;
    void* buf = nullptr;
    u64* out = nullptr;
    double* tab = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess ||
        hipMalloc(&tab, (size_t)primes * n * 8) != hipSuccess) {
        std::printf("alloc failed\n");
        return 1;
    }
    hipMemset(buf, 1, bytes);
    hipMemset(tab, 0, (size_t)primes * n * 8);
    hipDeviceSynchronize();
    // each kernel once; the streams cover 4x the Infinity Cache
    hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(256), 0, 0, (const ulonglong2*)buf, bytes / 16, out);
    hipDeviceSynchronize();
    std::printf("CALIB k_stream16 bytes=%zu\n", bytes);
    hipLaunchKernelGGL(k_stream8, dim3(4096), dim3(256), 0, 0, (const u64*)buf, bytes / 8, out);
    hipDeviceSynchronize();
    std::printf("CALIB k_stream8 bytes=%zu\n", bytes);
    const uint32_t R = n >> 8;
    hipLaunchKernelGGL(k_rowtw, dim3(primes * (R / 4)), dim3(256), 0, 0, (const double*)tab, logn, out);
    hipDeviceSynchronize();
    // distinct entries: per prime, stages k < 6 of every row: sum_k 2^(S0+k) .. = 63 R
    std::printf("CALIB k_rowtw bytes=%zu\n", (size_t)primes * 63 * R * 8);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        std::printf("ERROR %s\n", hipGetErrorString(e));
        return 1;
    }
    hipFree(buf);
    hipFree(out);
    hipFree(tab);
    return 0;
}
