// Micro check (GPU box): the census mismatch count as an fp4 block-scaled MFMA dot product.
// Each 32-bit census word w of a record becomes one lane's 16-B fp4 fragment (bit 4n + s of
// the word -> nibble n of dword s, value 2.0 = 0x4), lane l of MFMA kk carrying word
// 4 kk + (l >> 4) of row / column l & 15, so A and B place every bit at the same k and
// 16x16x128 x 3 = the 384 bits of 12 words.  Checks D[j][x] = 4 * sum_w popcount(A_j[w] &
// B_x[w]) for random records against the CPU, and the C/D map (col = lane & 15,
// row = 4 (lane >> 4) + reg).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/fp4dot tools/micro/fp4_census_dot.hip && /tmp/fp4dot
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <random>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v8i expand_fp4(uint32_t w) {
    v8i r;
    r[0] = (int)((w << 2) & 0x44444444u);
    r[1] = (int)((w << 1) & 0x44444444u);
    r[2] = (int)(w & 0x44444444u);
    r[3] = (int)((w >> 1) & 0x44444444u);
    r[4] = r[5] = r[6] = r[7] = 0;
    return r;
}

__global__ void k_dot(const uint32_t* A, const uint32_t* B, float* D) {
    const int l = threadIdx.x;
    v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
        const int w = 4 * kk + (l >> 4);
        const v8i a = expand_fp4(A[(l & 15) * 12 + w]);
        const v8i b = expand_fp4(B[(l & 15) * 12 + w]);
        acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 4, 4, 0, 127, 0, 127);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

int main() {
    std::mt19937 g(7);
    uint32_t A[16 * 12], B[16 * 12];
    for (auto& x : A) x = g();
    for (auto& x : B) x = g();
    A[3 * 12 + 5] = 0xffffffffu;  // extremes
    B[7 * 12 + 5] = 0xffffffffu;
    for (int w = 0; w < 12; ++w) A[0 * 12 + w] = B[0 * 12 + w] = 0xffffffffu;  // 384 matches
    uint32_t *dA, *dB;
    float* dD;
    hipMalloc(&dA, sizeof A);
    hipMalloc(&dB, sizeof B);
    hipMalloc(&dD, 256 * 4);
    hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_dot, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    float D[256];
    if (hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 2; }
    int bad = 0;
    for (int j = 0; j < 16; ++j)
        for (int x = 0; x < 16; ++x) {
            int c = 0;
            for (int w = 0; w < 12; ++w) c += __builtin_popcount(A[j * 12 + w] & B[x * 12 + w]);
            if (D[j * 16 + x] != 4.0f * c) {
                if (bad < 8) printf("j %d x %d: got %g want %d\n", j, x, D[j * 16 + x], 4 * c);
                ++bad;
            }
        }
    printf("fp4 census dot: %s (%d of 256 wrong; D[0][0] = %g)\n", bad ? "FAIL" : "ok", bad, D[0]);
    return bad ? 1 : 0;
}
