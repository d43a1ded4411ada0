// mz_mlp_device.h — the f32-MFMA Dense-layer block and the plan executor.
//
// One task = one wavefront computes  out[ob*16 + i][j] = act(W x_j + b)  for
// 16 output rows i and the 16 tile columns j, with K split into four
// contiguous quarters of kq = 4*nq values.  Each quarter is one accumulator
// chain of nq v_mfma_f32_16x16x4_f32 (a k-ordered fmaf chain from +0, bit for
// bit), and the block result is ((a0 + a1) + (a2 + a3)) + b — exactly the
// canonical order mz_dot of the oracle restates.  Four independent chains
// also hide the 40-cycle dependent-MFMA latency (MI355X_MICROARCH.md).
//
// Operand maps (16x16x4 f32): lane l holds A[i=l&15][k=l>>4] (a weight,
// pre-packed host-side so one coalesced 256-B load feeds one MFMA) and
// B[k=l>>4][j=l&15] = act[ks*4 + (l>>4)][l&15] = act + ks*64 + l (one
// conflict-free ds_read_b32 per MFMA); D: lane l holds rows (l>>4)*4 + r of
// column l&15.
#pragma once
#include "mz_internal.h"

typedef float mz_f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float mz_act(int act, float v) {
    if (act == MZ_ACT_RELU) return mz_relu(v);
    if (act == MZ_ACT_TANH) return det_tanhf(v);
    return v;
}

template <int NQ>
__device__ __forceinline__ void mlp_block_t(const LayerDesc& L, int ob, const float* __restrict__ Wp,
                                            const float* __restrict__ Bp, float* lds, int lane) {
    const float* wb = Wp + L.w_off + ob * (4 * NQ * 64) + lane;
    const float* xin = lds + L.in_off + lane;
    float w[4 * NQ], x[4 * NQ];
#pragma unroll
    for (int i = 0; i < 4 * NQ; ++i) w[i] = wb[i * 64];
#pragma unroll
    for (int i = 0; i < 4 * NQ; ++i) x[i] = xin[i * 64];
    mz_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w[0 * NQ + j], x[0 * NQ + j], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w[1 * NQ + j], x[1 * NQ + j], acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(w[2 * NQ + j], x[2 * NQ + j], acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(w[3 * NQ + j], x[3 * NQ + j], acc3, 0, 0, 0);
    }
    const float* bb = Bp + L.b_off + ob * 16 + (lane >> 4) * 4;
    float* out = lds + L.out_off + (ob * 16 + (lane >> 4) * 4) * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float d = (acc0[r] + acc1[r]) + (acc2[r] + acc3[r]);
        d = d + bb[r];
        out[r * 16] = mz_act(L.act, d);
    }
}

// any nq (K > 64): same order, runtime loop
__device__ __forceinline__ void mlp_block_any(const LayerDesc& L, int ob, const float* __restrict__ Wp,
                                              const float* __restrict__ Bp, float* lds, int lane) {
    const int NQ = L.nq;
    const float* wb = Wp + L.w_off + ob * (4 * NQ * 64) + lane;
    const float* xin = lds + L.in_off + lane;
    mz_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    for (int j = 0; j < NQ; ++j) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[(0 * NQ + j) * 64], xin[(0 * NQ + j) * 64], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[(1 * NQ + j) * 64], xin[(1 * NQ + j) * 64], acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[(2 * NQ + j) * 64], xin[(2 * NQ + j) * 64], acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[(3 * NQ + j) * 64], xin[(3 * NQ + j) * 64], acc3, 0, 0, 0);
    }
    const float* bb = Bp + L.b_off + ob * 16 + (lane >> 4) * 4;
    float* out = lds + L.out_off + (ob * 16 + (lane >> 4) * 4) * 16 + (lane & 15);
    for (int r = 0; r < 4; ++r) {
        float d = (acc0[r] + acc1[r]) + (acc2[r] + acc3[r]);
        d = d + bb[r];
        out[r * 16] = mz_act(L.act, d);
    }
}

// Execute a plan with all waves of the workgroup; every stage ends in a
// workgroup barrier.  Must be called by every thread of the workgroup.
__device__ __forceinline__ void run_plan(const int* plan, const float* __restrict__ Wp,
                                         const float* __restrict__ Bp, float* lds) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwaves = blockDim.x >> 6;
    PlanView pv = plan_view(plan);
    for (int s = 0; s < pv.n_stages; ++s) {
        const int t0 = pv.stage_begin[s], t1 = pv.stage_begin[s + 1];
        for (int t = t0 + wave; t < t1; t += nwaves) {
            const int li = pv.tasks[2 * t], ob = pv.tasks[2 * t + 1];
            const LayerDesc L = pv.layers[li];
            switch (L.nq) {
                case 1: mlp_block_t<1>(L, ob, Wp, Bp, lds, lane); break;
                case 2: mlp_block_t<2>(L, ob, Wp, Bp, lds, lane); break;
                case 3: mlp_block_t<3>(L, ob, Wp, Bp, lds, lane); break;
                case 4: mlp_block_t<4>(L, ob, Wp, Bp, lds, lane); break;
                default: mlp_block_any(L, ob, Wp, Bp, lds, lane); break;
            }
        }
        __syncthreads();
    }
}
