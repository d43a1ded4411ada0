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

// In-block activations are relu / identity only: the value and reward output
// layers (tanh, Learning.jl:110,140) are planned as identity and their
// activation is applied once where the value / reward is read (mz_post_act),
// which keeps the f64 tanh out of every block epilogue (instruction cache).
__device__ __forceinline__ float mz_act(int act, float v) {
    return act == MZ_ACT_RELU ? mz_relu(v) : v;
}
__device__ __forceinline__ float mz_post_act(int act, float v) {
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
        if (L.bn) d = mz_bn_apply(d, bb[L.n_ob * 16 + r], bb[2 * L.n_ob * 16 + r]);
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
        if (L.bn) d = mz_bn_apply(d, bb[L.n_ob * 16 + r], bb[2 * L.n_ob * 16 + r]);
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

// ---------------------------------------------------------------------------
// Register-resident plan (the simulation loop's prediction ‖ dynamics plan).
// Every wave owns a fixed list of <= MZ_RES_TASKS tasks; their weight
// fragments are loaded ONCE per kernel into wr[16*k .. 16*k + 4*nq) and the
// loop over k is fully unrolled so every register index is static.  With one
// 256-thread workgroup per CU a wave may use up to 512 VGPRs
// (__launch_bounds__(256, 1)).  Image (int array):
//   [0] n_stages, [1] NT (task slots per wave), then per wave w:
//   [ntasks, NT x ResTask].
#define MZ_RES_TASKS 16
struct ResTask { int stage, w_off, b_off, nq, ob, act, in_off, out_off, bn_ob; };   // bn_ob: n_ob if BatchNorm, else 0

__device__ __forceinline__ const ResTask* res_tasks(const int* img, int wave, int& nt) {
    const int NT = img[1];
    const int* wl = img + 2 + wave * (1 + NT * (int)(sizeof(ResTask) / sizeof(int)));
    nt = wl[0];
    return reinterpret_cast<const ResTask*>(wl + 1);
}

template <int K>
__device__ __forceinline__ void res_load_k(const ResTask* T, int nt, float (&wr)[16 * MZ_RES_TASKS],
                                           const float* __restrict__ Wp, int lane) {
    if constexpr (K < MZ_RES_TASKS) {
        if (K < nt) {
            const int nq = T[K].nq;
            const float* wb = Wp + T[K].w_off + T[K].ob * (4 * nq * 64) + lane;
#pragma unroll
            for (int i = 0; i < 16; ++i) wr[16 * K + i] = i < 4 * nq ? wb[i * 64] : 0.0f;
        }
        res_load_k<K + 1>(T, nt, wr, Wp, lane);
    }
}

__device__ __forceinline__ void res_load(const int* img, float (&wr)[16 * MZ_RES_TASKS], const float* __restrict__ Wp) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int nt;
    const ResTask* T = res_tasks(img, wave, nt);
    res_load_k<0>(T, nt, wr, Wp, lane);
}

template <int NQ, int OFF>
__device__ __forceinline__ void res_block(const ResTask& t, const float (&wr)[16 * MZ_RES_TASKS],
                                          const float* __restrict__ Bp, float* lds, int lane) {
    const float* xin = lds + t.in_off + lane;
    const float* bb = Bp + t.b_off + t.ob * 16 + (lane >> 4) * 4;
    const float b0 = bb[0], b1 = bb[1], b2 = bb[2], b3 = bb[3];
    float x[4 * NQ];
#pragma unroll
    for (int i = 0; i < 4 * NQ; ++i) x[i] = xin[i * 64];
    mz_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[OFF + 0 * NQ + j], x[0 * NQ + j], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[OFF + 1 * NQ + j], x[1 * NQ + j], acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[OFF + 2 * NQ + j], x[2 * NQ + j], acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[OFF + 3 * NQ + j], x[3 * NQ + j], acc3, 0, 0, 0);
    }
    float* out = lds + t.out_off + (t.ob * 16 + (lane >> 4) * 4) * 16 + (lane & 15);
    float d[4];
    d[0] = (acc0[0] + acc1[0]) + (acc2[0] + acc3[0]); d[0] = d[0] + b0;
    d[1] = (acc0[1] + acc1[1]) + (acc2[1] + acc3[1]); d[1] = d[1] + b1;
    d[2] = (acc0[2] + acc1[2]) + (acc2[2] + acc3[2]); d[2] = d[2] + b2;
    d[3] = (acc0[3] + acc1[3]) + (acc2[3] + acc3[3]); d[3] = d[3] + b3;
    if (t.bn_ob) {                                           // BatchNorm (test mode) after the affine
#pragma unroll
        for (int r = 0; r < 4; ++r) d[r] = mz_bn_apply(d[r], bb[t.bn_ob * 16 + r], bb[2 * t.bn_ob * 16 + r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) out[16 * r] = mz_act(t.act, d[r]);
}

template <int K>
__device__ __forceinline__ void res_run_k(const ResTask* T, int nt, int& cur, const float (&wr)[16 * MZ_RES_TASKS],
                                          const float* __restrict__ Bp, float* lds, int lane) {
    if constexpr (K < MZ_RES_TASKS) {
        if (K < nt) {
            const ResTask t = T[K];
            while (cur < t.stage) { __syncthreads(); ++cur; }
            switch (t.nq) {
                case 1: res_block<1, 16 * K>(t, wr, Bp, lds, lane); break;
                case 2: res_block<2, 16 * K>(t, wr, Bp, lds, lane); break;
                case 3: res_block<3, 16 * K>(t, wr, Bp, lds, lane); break;
                default: res_block<4, 16 * K>(t, wr, Bp, lds, lane); break;
            }
            res_run_k<K + 1>(T, nt, cur, wr, Bp, lds, lane);
        }
    }
}

// Run the resident plan: the same stage barriers as run_plan (every wave
// executes exactly n_stages barriers, advancing to each task's stage).
__device__ __forceinline__ void res_run(const int* img, const float (&wr)[16 * MZ_RES_TASKS],
                                        const float* __restrict__ Bp, float* lds) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ns = img[0];
    int nt;
    const ResTask* T = res_tasks(img, wave, nt);
    int cur = 0;
    res_run_k<0>(T, nt, cur, wr, Bp, lds, lane);
    while (cur < ns) { __syncthreads(); ++cur; }
}
