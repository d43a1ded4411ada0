// Probe of v_mfma_f32_4x4x1_16b_f32 operand/result lane layout on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out, float* out2) {
    int l = threadIdx.x;
    float a = (float)l;              // A
    float b = 1000.0f * (l + 1);     // B
    f4 c = {0, 0, 0, 0};
    f4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = d[r];
    // exactness: chain of two k-steps equals fma(a2,b2,fma(a1,b1,0))
    float a1 = 1.0f + l * 1e-3f, b1 = 3.0f - l * 7e-4f, a2 = -2.5f + l * 1.3e-3f, b2 = 0.7f + l * 1e-4f;
    f4 e = __builtin_amdgcn_mfma_f32_4x4x1f32(a1, b1, c, 0, 0, 0);
    e = __builtin_amdgcn_mfma_f32_4x4x1f32(a2, b2, e, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out2[l * 4 + r] = e[r];
}
int main() {
    float *d, *d2, h[256], h2[256];
    hipMalloc(&d, 1024); hipMalloc(&d2, 1024);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, d2);
    hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    hipMemcpy(h2, d2, 1024, hipMemcpyDeviceToHost);
    int ok = 1;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
            float want = (float)(4 * (l / 4) + r) * 1000.0f * (l + 1);
            if (h[l * 4 + r] != want) ok = 0;
        }
    printf("layout A lane=4b+i, B lane=4b+j, D lane=4b+j reg=i : %s\n", ok ? "YES" : "NO");
    if (!ok) for (int l = 0; l < 8; ++l) printf("lane %d: %g %g %g %g\n", l, h[l*4], h[l*4+1], h[l*4+2], h[l*4+3]);
    int ex = 1;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
            int ia = 4 * (l / 4) + r, ib = l;
            float a1 = 1.0f + ia * 1e-3f, b1 = 3.0f - ib * 7e-4f, a2 = -2.5f + ia * 1.3e-3f, b2 = 0.7f + ib * 1e-4f;
            float want = fmaf(a2, b2, fmaf(a1, b1, 0.0f));
            if (h2[l * 4 + r] != want) ex = 0;
        }
    printf("k-ordered fma chain exact: %s\n", ex ? "YES" : "NO");
    return 0;
}
