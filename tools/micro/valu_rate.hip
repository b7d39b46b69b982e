// Microbenchmark: VALU issue rate of the integer ops the cost walk uses (gfx950).
// Each thread runs N iterations of 8 independent chains; grid fills every SIMD with
// `waves` waves.  Reports wave-instructions per SIMD per cycle-equivalent (ns).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP>
__global__ void k_rate(uint32_t* out, int n, uint32_t seed) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + i + 1);
    const uint32_t b = seed ^ threadIdx.x, c = seed + 77u;
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (OP == 0) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                if (OP == 1) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(a[i]) : "v"(b));
                if (OP == 2) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                if (OP == 3) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                if (OP == 4) asm volatile("v_sad_u8 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                if (OP == 5) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if (OP == 6) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));
                if (OP == 7) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if (OP == 8) asm volatile("v_and_or_b32 %0, %0, %1, %2\n s_add_u32 s90, s90, 1" : "+v"(a[i]) : "v"(b), "v"(c) : "s90", "scc");
                if (OP == 9) asm volatile("v_and_b32 %0, %0, %1\n s_add_u32 s90, s90, 1" : "+v"(a[i]) : "v"(b) : "s90", "scc");
                if (OP == 10) asm volatile("v_and_or_b32 %0, %0, %1, %2\n s_nop 0" : "+v"(a[i]) : "v"(b), "v"(c));
                if (OP == 11) asm volatile("v_and_b32 %0, %0, %1\n v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            }
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s += a[i];
    if (s == 0x12345678u) out[threadIdx.x] = s;
}

int main() {
    uint32_t* out;
    hipMalloc(&out, 4096);
    const char* names[] = {"v_and_or_b32", "v_bcnt_u32_b32", "v_and_b32", "v_add_f32", "v_sad_u8",
                           "v_mov_dpp wave_shr", "v_cndmask", "v_mov_dpp row_shr", "and_or+s_add", "and+s_add", "and_or+s_nop", "2x v_and"};
    int dev;
    hipGetDevice(&dev);
    hipDeviceProp_t pr;
    hipGetDeviceProperties(&pr, dev);
    const int cus = pr.multiProcessorCount;
    const int n = 2000;
    for (int waves = 4; waves <= 8; waves *= 2) {
        for (int op = 0; op < 12; ++op) {
            dim3 grid(cus * waves), block(256);  // 4 waves per WG -> 1 per SIMD per WG
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            auto launch = [&] {
                switch (op) {
                    case 0: hipLaunchKernelGGL(k_rate<0>, grid, block, 0, 0, out, n, 3u); break;
                    case 1: hipLaunchKernelGGL(k_rate<1>, grid, block, 0, 0, out, n, 3u); break;
                    case 2: hipLaunchKernelGGL(k_rate<2>, grid, block, 0, 0, out, n, 3u); break;
                    case 3: hipLaunchKernelGGL(k_rate<3>, grid, block, 0, 0, out, n, 3u); break;
                    case 4: hipLaunchKernelGGL(k_rate<4>, grid, block, 0, 0, out, n, 3u); break;
                    case 5: hipLaunchKernelGGL(k_rate<5>, grid, block, 0, 0, out, n, 3u); break;
                    case 6: hipLaunchKernelGGL(k_rate<6>, grid, block, 0, 0, out, n, 3u); break;
                    case 7: hipLaunchKernelGGL(k_rate<7>, grid, block, 0, 0, out, n, 3u); break;
                    case 8: hipLaunchKernelGGL(k_rate<8>, grid, block, 0, 0, out, n, 3u); break;
                    case 9: hipLaunchKernelGGL(k_rate<9>, grid, block, 0, 0, out, n, 3u); break;
                    case 10: hipLaunchKernelGGL(k_rate<10>, grid, block, 0, 0, out, n, 3u); break;
                    case 11: hipLaunchKernelGGL(k_rate<11>, grid, block, 0, 0, out, n, 3u); break;
                }
            };
            launch();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_simd = (double)n * 128 * waves;  // wave-instructions per SIMD
            printf("waves/SIMD %d %-20s %.3f ns per wave-instr per SIMD\n", waves, names[op],
                   ms * 1e6 / instr_per_simd);
        }
    }
    return 0;
}
