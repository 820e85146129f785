// Developer probe: checks the lane maps the MFMA base conversion assumes for
// v_mfma_i32_16x16x64_i8 on gfx950 with exact, asymmetric integer data:
//   A: lane l holds A[row l&15][k = 16*(l>>4) + j], j = 0..15 (16 bytes)
//   B: lane l holds B[k = 16*(l>>4) + j][col l&15]
//   C: lane l, reg r holds C[row 4*(l>>4) + r][col l&15]
// Prints "mfma_i8 map ok" and exits 0, or the first mismatches and exits 1.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_probe(const int8_t* A, const int8_t* B, int32_t* C) {
    const int l = threadIdx.x;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; ++j) {
        a[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
        b[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
    }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
    int8_t hA[16 * 64], hB[64 * 16];
    for (int i = 0; i < 16; ++i)
        for (int k = 0; k < 64; ++k) hA[i * 64 + k] = (int8_t)((i * 7 + k * 3 + (i * k) % 5) % 255 - 127);
    for (int k = 0; k < 64; ++k)
        for (int j = 0; j < 16; ++j) hB[k * 16 + j] = (int8_t)((k * 11 + j * 5 + 3 * j * j) % 253 - 126);
    int8_t *dA, *dB;
    int32_t* dC;
    if (hipMalloc(&dA, sizeof hA) || hipMalloc(&dB, sizeof hB) || hipMalloc(&dC, 16 * 16 * 4)) return 2;
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    int32_t hC[256];
    if (hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            int32_t r = 0;
            for (int k = 0; k < 64; ++k) r += (int32_t)hA[i * 64 + k] * (int32_t)hB[k * 16 + j];
            if (r != hC[i * 16 + j] && bad++ < 8) std::printf("C[%d][%d] = %d, want %d\n", i, j, hC[i * 16 + j], r);
        }
    std::printf(bad ? "mfma_i8 map WRONG (%d mismatches)\n" : "mfma_i8 map ok\n", bad);
    return bad ? 1 : 0;
}
