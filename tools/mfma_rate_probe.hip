// Cycle costs on gfx950 (one wave, s_memtime): dependent / independent chains of
// v_mfma_f32_4x4x1_16b_f32, v_mfma_f32_16x16x4_f32 and v_fma_f32.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
#define N 256
__global__ void probe(float* out, unsigned long long* cyc, float a, float b) {
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    float x = a + threadIdx.x, y = b, z0 = 0, z1 = 0, z2 = 0, z3 = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N; ++i) c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(x, y, c0, 0, 0, 0);
    asm volatile("" :: "v"(c0));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(x, y, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(x, y, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(x, y, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(x, y, c3, 0, 0, 0);
    }
    asm volatile("" :: "v"(c0), "v"(c1), "v"(c2), "v"(c3));
    unsigned long long t2 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N; ++i) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, c1, 0, 0, 0);
    asm volatile("" :: "v"(c1));
    unsigned long long t3 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N; ++i) z0 = fmaf(x, z0, y);
    asm volatile("" :: "v"(z0));
    unsigned long long t4 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 4; ++i) { z0 = fmaf(x, z0, y); z1 = fmaf(x, z1, y); z2 = fmaf(x, z2, y); z3 = fmaf(x, z3, y); }
    asm volatile("" :: "v"(z0), "v"(z1), "v"(z2), "v"(z3));
    unsigned long long t5 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t5 - t4;
    }
    out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3] + z0 + z1 + z2 + z3;
}
int main() {
    float* d; unsigned long long *c, h[5];
    (void)hipMalloc(&d, 4096); (void)hipMalloc(&c, 64);
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, c, 1.0f, 0.5f);
    (void)hipMemcpy(h, c, 40, hipMemcpyDeviceToHost);
    printf("cycles/instr: mfma4x4x1 dep %.1f | 4 indep %.1f | mfma16x16x4 dep %.1f | fma dep %.1f | fma 4 indep %.1f\n",
           h[0] / (double)N, h[1] / (double)N, h[2] / (double)N, h[3] / (double)N, h[4] / (double)N);
    return 0;
}
