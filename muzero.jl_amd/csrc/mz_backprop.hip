// mz_backprop.hip — the corrected-gradient learner (mz_learner_set_mode
// MZ_LEARN_CORRECTED, FC nets): backpropagation through the K-step unroll of
// Learning.jl:347-370 on f32 MFMA.  See mz_backprop_params.h for the loss.
//
//   mz_bp_tile  one workgroup (4 waves) per tile of 16 samples: the forward
//               list of layer applications (each a 16-sample MFMA GEMM,
//               y = act(W x + b), wave w owning output row blocks w, w+4, ..),
//               the heads' loss gradients, then the list in reverse: dX +=
//               Wᵀ dZ (MFMA, K = out) with dZ = dY ⊙ act'(y) formed as the
//               operand is loaded (the dW kernel forms it the same way).
//   mz_bp_dw    one wave per 16x16 block of a layer's dW: Σ over tiles, the
//               layer's applications and the 16 samples of dZ ⊗ x (MFMA with
//               K = samples): the data term of the gradient; one wave per
//               bias block.
//   mz_bp_fold  Σθ² per net and the reported losses (deterministic f64 trees).
// The ADAM step that follows is mz_adam_kernel: ∇ = (Σ_ranks data term) ·
// 1/world + 2θ, the rank-invariant ∂Σθ²/∂θ added after the exchange.
#include "mz_internal.h"
#include "mz_backprop_params.h"

typedef float bp_f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bp_act(int act, float v) {
    return act == MZ_ACT_RELU ? mz_relu(v) : act == MZ_ACT_TANH ? det_tanhf(v) : v;
}

// dZ = dY ⊙ act'(y) (act' from the output y: relu y > 0, tanh 1 − y²)
__device__ __forceinline__ float bp_dz(int act, float g, float y) {
    return act == MZ_ACT_RELU ? (y > 0.0f ? g : 0.0f) : act == MZ_ACT_TANH ? g * (1.0f - y * y) : g;
}

// The epilogue of a dense unit's output row oo, sample m: t = W x + b; after a
// make_dense BatchNorm (use_batch_norm, Learning.jl:70-78) t is kept in the
// arena for mz_bp_dw and y = act(γ·(t/√(1+ε)) + β), else y = act(t)
// BN: the app has a BatchNorm (P.bn_off >= 0), a compile-time choice so the
// default nets' code carries no BatchNorm test or load (the level kernel
// dispatches per application)
template <bool BN>
__device__ __forceinline__ float bp_epi(const BpApp& P, const float* __restrict__ flat, float* T, int oo, int m,
                                        float t) {
    if (BN) {
        T[P.z + oo * 16 + m] = t;
        t = mz_bn_apply(t, flat[P.bn_off + P.out + oo], flat[P.bn_off + oo]);
    }
    return bp_act(P.act, t);
}
__device__ __forceinline__ float bp_epi(const BpApp& P, const float* __restrict__ flat, float* T, int oo, int m,
                                        float t) {
    return P.bn_off >= 0 ? bp_epi<true>(P, flat, T, oo, m, t) : bp_epi<false>(P, flat, T, oo, m, t);
}
// ∂L/∂t of output row o: dY ⊙ act'(y), times γ/√(1+ε) after a BatchNorm
template <bool BN>
__device__ __forceinline__ float bp_dt(const BpApp& P, const float* __restrict__ flat, int o, float g, float y) {
    const float du = bp_dz(P.act, g, y);
    return BN ? du * (flat[P.bn_off + P.out + o] / MZ_BN_S) : du;
}
__device__ __forceinline__ float bp_dt(const BpApp& P, const float* __restrict__ flat, int o, float g, float y) {
    return P.bn_off >= 0 ? bp_dt<true>(P, flat, o, g, y) : bp_dt<false>(P, flat, o, g, y);
}

// One 16-row block of a 16-sample MFMA GEMM, C[r][s] = Σ_k A(r, k) B(k, s),
// its operands gathered BP_KC k-steps at a time (all loads of a chunk in
// flight before its MFMAs: one memory latency per chunk, not per k-step).
// BP_SKIP: a chunk's groups of 4 k-steps past nk (wave-uniform; their operands
// are zeros, adding nothing) skip their MFMAs — the nets' 27- / 36-row inputs
// and 27 / 9 / 1-row outputs fill 7, 9, 7, 3 or 1 of the chunk's 16 k-steps
#define BP_KC 16
#ifndef BP_SKIP
#define BP_SKIP 1
#endif
template <class FA, class FB>
__device__ __forceinline__ bp_f32x4 bp_gemm_block(int nk, int kq, FA fa, FB fb) {
    bp_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < nk; k0 += BP_KC) {
        float a[BP_KC], b[BP_KC];
#pragma unroll
        for (int j = 0; j < BP_KC; ++j) {
            const int k = (k0 + j) * 4 + kq;
            a[j] = k0 + j < nk ? fa(k) : 0.0f;
            b[j] = k0 + j < nk ? fb(k) : 0.0f;
        }
#if BP_SKIP
#pragma unroll
        for (int q = 0; q < BP_KC; q += 4) {
            if (k0 + q < nk) {
#pragma unroll
                for (int j = q; j < q + 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
            }
        }
#else
#pragma unroll
        for (int j = 0; j < BP_KC; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
#endif
    }
    return acc;
}

// y = act(W x + b), output rows ob·16 .. ob·16 + 15 of the tile (one wave)
__device__ __forceinline__ void bp_dense_fwd_blk(const BpApp& P, const float* __restrict__ flat, float* T, int ob) {
    const int lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4;
    const float* W = flat + P.w_off;
    const float* X = T + P.x;
    float* Y = T + P.y;
    const int nk = (P.in + 3) >> 2;
    const int o = ob * 16 + m;
    const bool oin = o < P.out;
    const bp_f32x4 acc = bp_gemm_block(nk, kq,
        [&](int i) { return oin && i < P.in ? W[o + (size_t)P.out * i] : 0.0f; },
        [&](int i) { return i < P.in ? X[i * 16 + m] : 0.0f; });
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int oo = ob * 16 + kq * 4 + r;
        if (oo < P.out) Y[oo * 16 + m] = bp_epi(P, flat, T, oo, m, acc[r] + flat[P.b_off + oo]);
    }
}
// y = act(W x + b) for the tile (all 256 threads; rows in blocks of 16 per wave)
__device__ __forceinline__ void bp_dense_fwd(const BpApp& P, const float* __restrict__ flat, float* T) {
    const int wave = threadIdx.x >> 6, nob = (P.out + 15) >> 4;
    for (int ob = wave; ob < nob; ob += 4) bp_dense_fwd_blk(P, flat, T, ob);
}

// G[x] += Wᵀ dZ with dZ = G[y] ⊙ act'(y) formed as the operand is loaded;
// input rows ib·16 .. ib·16 + 15 (one wave)
__device__ __forceinline__ void bp_dense_dx_blk(const BpApp& P, const float* __restrict__ flat, const float* T,
                                                float* G, int ib) {
    const int lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4;
    const float* W = flat + P.w_off;
    const float* DY = G + P.y;
    const float* Y = T + P.y;
    float* DX = G + P.x;
    const int nk = (P.out + 3) >> 2;
    const int i = ib * 16 + m;
    const bool iin = i < P.in;
    const bp_f32x4 acc = bp_gemm_block(nk, kq,
        [&](int o) { return iin && o < P.out ? W[o + (size_t)P.out * i] : 0.0f; },
        [&](int o) { return o < P.out ? bp_dt(P, flat, o, DY[o * 16 + m], Y[o * 16 + m]) : 0.0f; });
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int ii = ib * 16 + kq * 4 + r;
        if (ii < P.in) DX[ii * 16 + m] += acc[r];
    }
}
__device__ __forceinline__ void bp_dense_dx(const BpApp& P, const float* __restrict__ flat, const float* T,
                                            float* G) {
    const int wave = threadIdx.x >> 6, nib = (P.in + 15) >> 4;
    for (int ib = wave; ib < nib; ib += 4) bp_dense_dx_blk(P, flat, T, G, ib);
}

// Tile arenas, loss terms and reward read-outs zeroed, the observation staged
__device__ __forceinline__ void bp_prologue(const BpParams& Q, float* T, float* G, float* C = nullptr) {
    const int tid = threadIdx.x, nt = blockDim.x, t0 = blockIdx.x * 16, K1 = Q.K + 1;
    for (int e = tid; e < Q.tile_floats; e += nt) G[e] = 0.0f;
    for (int e = tid; e < 16 * K1 * 3; e += nt) {
        const int b = t0 + e / (K1 * 3);
        if (b < Q.B) Q.terms[(size_t)t0 * K1 * 3 + e] = 0.0f;
    }
    for (int e = tid; e < 16 * K1; e += nt) {                 // rewards: 0 at step 0 (and without heads)
        const int b = t0 + e / K1;
        if (b < Q.B) Q.pr[(size_t)t0 * K1 + e] = 0.0f;
    }
    for (int e = tid; e < Q.obs_feat * 16; e += nt) {        // observation_batch (:347)
        const int f = e >> 4, s = e & 15, b = t0 + s;
        const float v = b < Q.B ? Q.obs[(size_t)b * Q.obs_feat + f] : 0.0f;
        T[Q.obs_t + e] = v;
        if (C && Q.obs_s >= 0) C[Q.obs_s + e] = v;
    }
}

// make_dynamics_input (:293-304) over the threads [t, t + nt) of the block
__device__ __forceinline__ void bp_concat_fwd(const BpParams& Q, const BpApp& P, float* T, int t, int nt) {
    const int t0 = blockIdx.x * 16, K1 = Q.K + 1;
    for (int e = t; e < P.out * 16; e += nt) {
        const int i = e >> 4, s = e & 15, b = t0 + s;
        float v;
        if (i < P.in) v = T[P.x + e] * 2.0f;
        else v = b < Q.B ? Q.actions[(size_t)b * K1 + P.step] / (float)Q.A : 0.0f;
        T[P.y + e] = v;
    }
}

__device__ void bp_heads(const BpParams& Q, float* T, float* G);

extern "C" __global__ __launch_bounds__(256) void mz_bp_tile(BpParams Q) {
    const int tid = threadIdx.x;
    float* T = Q.act + (size_t)blockIdx.x * Q.tile_floats;
    float* G = Q.grad + (size_t)blockIdx.x * Q.tile_floats;
    bp_prologue(Q, T, G);
    __syncthreads();
    // ---- forward: representation, K dynamics steps, K+1 predictions (Q10)
    for (int a = 0; a < Q.n_app; ++a) {
        const BpApp P = Q.apps[a];
        if (P.op == BP_DENSE) bp_dense_fwd(P, Q.flat, T);
        else bp_concat_fwd(Q, P, T, tid, 256);
        __syncthreads();
    }
    bp_heads(Q, T, G);
    __syncthreads();
    // ---- backward, reverse order
    for (int a = Q.n_app - 1; a >= 0; --a) {
        const BpApp P = Q.apps[a];
        if (P.op == BP_DENSE) {
            bp_dense_dx(P, Q.flat, T, G);
        } else {                                              // ∂(2h)/∂h
            for (int e = tid; e < P.in * 16; e += 256) G[P.x + e] += 2.0f * G[P.y + e];
        }
        __syncthreads();
    }
}

// The same computation on the host-built level schedule (BpParams.funits /
// bunits): every unit of a level runs on its own wave, one barrier per level
// instead of one per application.  A dense application's output (forward) or
// input (backward) row blocks are independent; applications of one level read
// only earlier levels and write distinct tensors; backward applications that
// accumulate into the same input gradient G[x] sit in distinct levels in the
// sequential kernel's (reverse) order — so every value, accumulation order
// included, equals mz_bp_tile's bit for bit.  The schedule and the
// application descriptors are staged in LDS, and a wave's operands of the next
// level that do not depend on this level — its unit, the weight fragment of
// the first k-chunk, the bias — are loaded before the barrier: after it, one
// memory round trip (the input rows) precedes the MFMAs.
struct BpPre {
    int app, blk;         // app < 0: no unit
    float a[BP_KC];       // A operands of the first k-chunk (dense)
    float bias[4];        // forward: the bias of the lane's four output rows
};

// dense forward / backward block with the first chunk's A operands preloaded
template <class FA, class FB>
__device__ __forceinline__ bp_f32x4 bp_gemm_block_pre(int nk, int kq, const float (&a0)[BP_KC], FA fa, FB fb) {
    bp_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < nk; k0 += BP_KC) {
        float a[BP_KC], b[BP_KC];
#pragma unroll
        for (int j = 0; j < BP_KC; ++j) {
            const int k = (k0 + j) * 4 + kq;
            a[j] = k0 == 0 ? a0[j] : k0 + j < nk ? fa(k) : 0.0f;
            b[j] = k0 + j < nk ? fb(k) : 0.0f;
        }
#if BP_SKIP
#pragma unroll
        for (int q = 0; q < BP_KC; q += 4) {
            if (k0 + q < nk) {
#pragma unroll
                for (int j = q; j < q + 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
            }
        }
#else
#pragma unroll
        for (int j = 0; j < BP_KC; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
#endif
    }
    return acc;
}

template <bool FWD>
__device__ __forceinline__ void bp_lv_fetch(const BpApp* apps, const int2* units, int u, int u_end,
                                            const float* __restrict__ flat, BpPre& pr) {
    const int lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4;
    pr.app = -1; pr.blk = 0;
    if (u >= u_end) return;
    const int2 un = units[u];
    pr.app = un.x; pr.blk = un.y;
    const BpApp P = apps[un.x];
    if (P.op != BP_DENSE) return;
    const float* W = flat + P.w_off;
    if (FWD) {
        const int o = un.y * 16 + m;
        const bool oin = o < P.out;
        const int nk = (P.in + 3) >> 2;
#pragma unroll
        for (int j = 0; j < BP_KC; ++j) {
            const int i = j * 4 + kq;
            pr.a[j] = oin && j < nk && i < P.in ? W[o + (size_t)P.out * i] : 0.0f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int oo = un.y * 16 + kq * 4 + r;
            pr.bias[r] = oo < P.out ? flat[P.b_off + oo] : 0.0f;
        }
    } else {
        const int i = un.y * 16 + m;
        const bool iin = i < P.in;
        const int nk = (P.out + 3) >> 2;
#pragma unroll
        for (int j = 0; j < BP_KC; ++j) {
            const int o = j * 4 + kq;
            pr.a[j] = iin && j < nk && o < P.out ? W[o + (size_t)P.out * i] : 0.0f;
        }
    }
}

template <bool FWD>
__device__ __forceinline__ void bp_lv_run(const BpParams& Q, const BpApp& P, const BpPre& pr, float* T, float* G) {
    const int lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4;
    const float* W = Q.flat + P.w_off;
    if (P.op != BP_DENSE) {
        if (FWD) bp_concat_fwd(Q, P, T, lane, 64);
        else for (int e = lane; e < P.in * 16; e += 64) G[P.x + e] += 2.0f * G[P.y + e];   // ∂(2h)/∂h
        return;
    }
    if (FWD) {                                               // as bp_dense_fwd_blk
        const int ob = pr.blk, o = ob * 16 + m;
        const bool oin = o < P.out;
        const float* X = T + P.x;
        float* Y = T + P.y;
        const bp_f32x4 acc = bp_gemm_block_pre((P.in + 3) >> 2, kq, pr.a,
            [&](int i) { return oin && i < P.in ? W[o + (size_t)P.out * i] : 0.0f; },
            [&](int i) { return i < P.in ? X[i * 16 + m] : 0.0f; });
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int oo = ob * 16 + kq * 4 + r;
            if (oo < P.out) Y[oo * 16 + m] = bp_epi(P, Q.flat, T, oo, m, acc[r] + pr.bias[r]);
        }
    } else {                                                 // as bp_dense_dx_blk
        const int ib = pr.blk, i = ib * 16 + m;
        const bool iin = i < P.in;
        const float* DY = G + P.y;
        const float* Y = T + P.y;
        float* DX = G + P.x;
        const bp_f32x4 acc = bp_gemm_block_pre((P.out + 3) >> 2, kq, pr.a,
            [&](int o) { return iin && o < P.out ? W[o + (size_t)P.out * i] : 0.0f; },
            [&](int o) { return o < P.out ? bp_dt(P, Q.flat, o, DY[o * 16 + m], Y[o * 16 + m]) : 0.0f; });
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int ii = ib * 16 + kq * 4 + r;
            if (ii < P.in) DX[ii * 16 + m] += acc[r];
        }
    }
}

// The level kernel's units with the LDS tensor cache C (BpApp xs / ys / gys /
// gxs): the same arithmetic as bp_dense_fwd_blk / bp_dense_dx_blk, operands
// read from the cache copies where the host placed them, outputs written to the
// arena and to their copy, ∂L/∂x accumulated in its copy (the first
// contribution adds to 0, as into the zeroed arena)
// MAYBN: the nets may hold BatchNorm layers (checked per application); false
// compiles the check and its loads out (the kernel for nets without any)
template <bool MAYBN>
__device__ __forceinline__ void bp_c_fwd_blk(const BpApp& P, const float* __restrict__ flat, float* T, float* C,
                                             int ob) {
    const int lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4;
    const float* W = flat + P.w_off;
    const int nk = (P.in + 3) >> 2;
    const int o = ob * 16 + m;
    const bool oin = o < P.out;
    auto fa = [&](int i) { return oin && i < P.in ? W[o + P.out * i] : 0.0f; };
    // the input from its LDS copy or the arena: one branch, so each side's
    // loads are LDS or global ones (not generic loads waiting on both counters)
    const bp_f32x4 acc =
        P.xs >= 0 ? bp_gemm_block(nk, kq, fa, [&](int i) { return i < P.in ? C[P.xs + i * 16 + m] : 0.0f; })
                  : bp_gemm_block(nk, kq, fa, [&](int i) { return i < P.in ? T[P.x + i * 16 + m] : 0.0f; });
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int oo = ob * 16 + kq * 4 + r;
        if (oo < P.out) {
            const float v = MAYBN ? bp_epi(P, flat, T, oo, m, acc[r] + flat[P.b_off + oo])
                                  : bp_epi<false>(P, flat, T, oo, m, acc[r] + flat[P.b_off + oo]);
            T[P.y + oo * 16 + m] = v;
            if (P.ys >= 0) C[P.ys + oo * 16 + m] = v;
        }
    }
}
template <bool MAYBN>
__device__ __forceinline__ void bp_c_dx_blk(const BpApp& P, const float* __restrict__ flat, const float* T, float* G,
                                            float* C, int ib) {
    const int lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4;
    const float* W = flat + P.w_off;
    const bool wout = P.gys >= 0 && ib == 0;                  // the copy's final value to the arena (mz_bp_dw)
    const int nk = (P.out + 3) >> 2;
    const int i = ib * 16 + m;
    const bool iin = i < P.in;
    // per k-chunk: every operand load issued first (W, y from the arena, ∂L/∂y
    // from its LDS copy or the arena, on one branch), the copy's write-out to
    // the arena after them, then the MFMAs (a store among the loads made each
    // k-step wait for the previous one's loads: one memory latency per k-step)
    bp_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < nk; k0 += BP_KC) {
        float a[BP_KC], g[BP_KC], y[BP_KC], b[BP_KC];
#pragma unroll
        for (int j = 0; j < BP_KC; ++j) {
            const int o = (k0 + j) * 4 + kq;
            const bool ok = k0 + j < nk && o < P.out;
            a[j] = ok && iin ? W[o + P.out * i] : 0.0f;          // (32-bit offsets from uniform bases)
            y[j] = ok ? T[P.y + o * 16 + m] : 0.0f;
        }
        if (P.gys >= 0) {
#pragma unroll
            for (int j = 0; j < BP_KC; ++j) {
                const int o = (k0 + j) * 4 + kq;
                g[j] = k0 + j < nk && o < P.out ? C[P.gys + o * 16 + m] : 0.0f;
            }
        } else {
#pragma unroll
            for (int j = 0; j < BP_KC; ++j) {
                const int o = (k0 + j) * 4 + kq;
                g[j] = k0 + j < nk && o < P.out ? G[P.y + o * 16 + m] : 0.0f;
            }
        }
#pragma unroll
        for (int j = 0; j < BP_KC; ++j) {
            const int o = (k0 + j) * 4 + kq;
            b[j] = k0 + j < nk && o < P.out
                       ? (MAYBN ? bp_dt(P, flat, o, g[j], y[j]) : bp_dt<false>(P, flat, o, g[j], y[j])) : 0.0f;
        }
        if (wout) {
#pragma unroll
            for (int j = 0; j < BP_KC; ++j) {
                const int o = (k0 + j) * 4 + kq;
                if (k0 + j < nk && o < P.out) G[P.y + o * 16 + m] = g[j];
            }
        }
#if BP_SKIP
#pragma unroll
        for (int q = 0; q < BP_KC; q += 4) {
            if (k0 + q < nk) {
#pragma unroll
                for (int j = q; j < q + 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
            }
        }
#else
#pragma unroll
        for (int j = 0; j < BP_KC; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
#endif
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int ii = ib * 16 + kq * 4 + r;
        if (ii >= P.in) continue;
        if (P.gxs >= 0) {
            float* d = C + P.gxs + ii * 16 + m;
            *d = (P.gxf ? 0.0f : *d) + acc[r];
        } else {
            G[P.x + ii * 16 + m] += acc[r];
        }
    }
}
__device__ __forceinline__ void bp_c_concat(const BpParams& Q, const BpApp& P, float* T, float* G, float* C, bool fwd) {
    const int lane = threadIdx.x & 63, t0 = blockIdx.x * 16, K1 = Q.K + 1;
    if (fwd) {                                                // make_dynamics_input (:293-304)
        for (int e = lane; e < P.out * 16; e += 64) {
            const int i = e >> 4, s = e & 15, b = t0 + s;
            float v;
            if (i < P.in) v = (P.xs >= 0 ? C[P.xs + e] : T[P.x + e]) * 2.0f;
            else v = b < Q.B ? Q.actions[(size_t)b * K1 + P.step] / (float)Q.A : 0.0f;
            T[P.y + e] = v;
            if (P.ys >= 0) C[P.ys + e] = v;
        }
    } else {                                                  // ∂(2h)/∂h
        for (int e = lane; e < P.in * 16; e += 64) {
            const float g = 2.0f * (P.gys >= 0 ? C[P.gys + e] : G[P.y + e]);
            if (P.gxs >= 0) C[P.gxs + e] = (P.gxf ? 0.0f : C[P.gxs + e]) + g;
            else G[P.x + e] += g;
        }
    }
}

template <bool FWD, bool MAYBN = true>
__device__ __forceinline__ void bp_lv_levels(const BpParams& Q, const BpApp* apps, const int2* units, const int* lev,
                                             int nlev, float* T, float* G, const int* sync = nullptr,
                                             float* C = nullptr) {
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#if BP_LV_SIMPLE
    const int lane = threadIdx.x & 63;
    if (C) {                                                  // with the LDS tensor cache
#ifdef MZ_STAMPS
        auto stampc = [&](int i) { if (blockIdx.x == 0 && threadIdx.x == 0) Q.stamps[i] = __builtin_amdgcn_s_memtime(); };
        if (FWD) stampc(0);
#endif
        for (int l = 0; l < nlev; ++l) {
            for (int u = lev[l] + wave; u < lev[l + 1]; u += nw) {
                const int2 un = units[u];
                const BpApp P = apps[un.x];
                if (P.op == BP_DENSE) {
                    if (FWD) bp_c_fwd_blk<MAYBN>(P, Q.flat, T, C, un.y);
                    else bp_c_dx_blk<MAYBN>(P, Q.flat, T, G, C, un.y);
                } else {
                    bp_c_concat(Q, P, T, G, C, FWD);
                }
            }
            if (sync[l]) {
                __syncthreads();
            } else {                                          // the level's hand-offs are in LDS only
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
            }
#ifdef MZ_STAMPS
            stampc((FWD ? 2 : 256) + l);
#endif
        }
        return;
    }
#ifdef MZ_STAMPS   // tile 0's level ends: [0] start, forward levels from 2, backward from 256
    auto stamp = [&](int i) { if (blockIdx.x == 0 && threadIdx.x == 0) Q.stamps[i] = __builtin_amdgcn_s_memtime(); };
    if (FWD) stamp(0);
#endif
    for (int l = 0; l < nlev; ++l) {
        for (int u = lev[l] + wave; u < lev[l + 1]; u += nw) {
            const int2 un = units[u];
            const BpApp P = apps[un.x];
            if (P.op == BP_DENSE) {
                if (FWD) bp_dense_fwd_blk(P, Q.flat, T, un.y);
                else bp_dense_dx_blk(P, Q.flat, T, G, un.y);
            } else if (FWD) {
                bp_concat_fwd(Q, P, T, lane, 64);
            } else {
                for (int e = lane; e < P.in * 16; e += 64) G[P.x + e] += 2.0f * G[P.y + e];
            }
        }
        __syncthreads();
#ifdef MZ_STAMPS
        stamp((FWD ? 2 : 256) + l);
#endif
    }
#elif BP_LV_PREFETCH
    BpPre cur;
    bp_lv_fetch<FWD>(apps, units, lev[0] + wave, lev[1], Q.flat, cur);
    for (int l = 0; l < nlev; ++l) {
        if (cur.app >= 0) bp_lv_run<FWD>(Q, apps[cur.app], cur, T, G);
        for (int u = lev[l] + wave + nw; u < lev[l + 1]; u += nw) {       // more units than waves (rare)
            BpPre x;
            bp_lv_fetch<FWD>(apps, units, u, lev[l + 1], Q.flat, x);
            bp_lv_run<FWD>(Q, apps[x.app], x, T, G);
        }
        BpPre nxt;
        nxt.app = -1;
        if (l + 1 < nlev) bp_lv_fetch<FWD>(apps, units, lev[l + 1] + wave, lev[l + 2], Q.flat, nxt);
        __syncthreads();
        cur = nxt;
    }
#else
    for (int l = 0; l < nlev; ++l) {
        for (int u = lev[l] + wave; u < lev[l + 1]; u += nw) {
            BpPre x;
            bp_lv_fetch<FWD>(apps, units, u, lev[l + 1], Q.flat, x);
            bp_lv_run<FWD>(Q, apps[x.app], x, T, G);
        }
        __syncthreads();
    }
#endif
}

template <bool MAYBN>
__device__ __forceinline__ void bp_tile_lv_body(const BpParams& Q) {
    extern __shared__ __attribute__((aligned(16))) int bp_lds[];
    float* T = Q.act + (size_t)blockIdx.x * Q.tile_floats;
    float* G = Q.grad + (size_t)blockIdx.x * Q.tile_floats;
    // the schedule and the descriptors in LDS: [apps][funits][bunits][flev][blev]
    const int nfu = 0, nbu = 0;
    (void)nfu; (void)nbu;
    BpApp* apps = reinterpret_cast<BpApp*>(bp_lds);
    int2* fun = reinterpret_cast<int2*>(apps + Q.n_app);
    int2* bun = fun + Q.n_funit;
    int* flev = reinterpret_cast<int*>(bun + Q.n_bunit);
    int* blev = flev + Q.n_flev + 2;
    int* fsy = blev + Q.n_blev + 2;
    int* bsy = fsy + Q.n_flev + 2;
    // (an offset from bp_lds, not an integer round trip: the cache accesses stay LDS instructions)
    const int c_off = ((int)(bsy + Q.n_blev + 2 - bp_lds) + 3) & ~3;
    float* C = Q.cache_floats > 0 ? reinterpret_cast<float*>(bp_lds + c_off) : nullptr;
    for (int i = threadIdx.x; i < Q.n_flev; i += blockDim.x) fsy[i] = Q.fsync[i];
    for (int i = threadIdx.x; i < Q.n_blev; i += blockDim.x) bsy[i] = Q.bsync[i];
    for (int i = threadIdx.x; i < Q.n_app; i += blockDim.x) apps[i] = Q.apps[i];
    for (int i = threadIdx.x; i < Q.n_funit; i += blockDim.x) fun[i] = Q.funits[i];
    for (int i = threadIdx.x; i < Q.n_bunit; i += blockDim.x) bun[i] = Q.bunits[i];
    for (int i = threadIdx.x; i < Q.n_flev + 2; i += blockDim.x) flev[i] = i <= Q.n_flev ? Q.flev[i] : Q.n_funit;
    for (int i = threadIdx.x; i < Q.n_blev + 2; i += blockDim.x) blev[i] = i <= Q.n_blev ? Q.blev[i] : Q.n_bunit;
    // one load per 128-byte line of the parameters: every level's weight reads
    // then hit this XCD's L2 (ADAM rewrote them through another XCD's)
    float warm = 0.0f;
    for (int i = threadIdx.x * 32; i < Q.nflat; i += blockDim.x * 32) warm += Q.flat[i];
    bp_prologue(Q, T, G, C);
    __syncthreads();
#if BP_LV_LDS
    bp_lv_levels<true, MAYBN>(Q, apps, fun, flev, Q.n_flev, T, G, fsy, C);
    bp_heads(Q, T, G);
    __syncthreads();
#ifdef MZ_STAMPS
    if (blockIdx.x == 0 && threadIdx.x == 0) Q.stamps[1] = __builtin_amdgcn_s_memtime();
#endif
    bp_lv_levels<false, MAYBN>(Q, apps, bun, blev, Q.n_blev, T, G, bsy, C);
    if (Q.B < 0) Q.terms[threadIdx.x] = warm;                // never: keeps the warm-up loads
#else   // descriptors by scalar loads (wave-uniform values straight into SGPRs)
    bp_lv_levels<true>(Q, Q.apps, Q.funits, Q.flev, Q.n_flev, T, G);
    bp_heads(Q, T, G);
    __syncthreads();
    bp_lv_levels<false>(Q, Q.apps, Q.bunits, Q.blev, Q.n_blev, T, G);
#endif
}

extern "C" __global__ __launch_bounds__(BP_LV_THREADS) void mz_bp_tile_lv(BpParams Q) { bp_tile_lv_body<true>(Q); }
// the same for nets without BatchNorm layers (use_batch_norm = false, the default)
extern "C" __global__ __launch_bounds__(BP_LV_THREADS) void mz_bp_tile_lv_nobn(BpParams Q) {
    bp_tile_lv_body<false>(Q);
}

// ---- heads: dL/dy of the value / policy / reward outputs, loss terms
__device__ void bp_heads(const BpParams& Q, float* T, float* G) {
    const int tid = threadIdx.x, nt = blockDim.x, t0 = blockIdx.x * 16, K1 = Q.K + 1;
    for (int e = tid; e < Q.n_head * 16; e += nt) {
        const BpHead hd = Q.heads[e >> 4];
        const int s = e & 15, b = t0 + s, k = hd.step;
        if (b >= Q.B) continue;
        const float w = Q.weights ? Q.weights[b] : 1.0f;
        const float c = w / (Q.gscale[b] * (float)Q.B);
        const size_t bk = (size_t)b * K1 + k;
        if (hd.kind == BP_HEAD_V || hd.kind == BP_HEAD_R) {
            const bool v = hd.kind == BP_HEAD_V;
            const float y = T[hd.y + s];
            const float d = y - (v ? Q.tv[bk] : Q.tr[bk]);
            const bool on = v || Q.intermediate_rewards;
            (v ? Q.pv : Q.pr)[bk] = y;
            G[hd.y + s] = on ? c * 2.0f * d : 0.0f;
            Q.terms[bk * 3 + (v ? 0 : 2)] = on ? d * d : 0.0f;
        } else {                                              // logitcrossentropy on the logits
            const float* l = T + hd.y + s;
            const float* pi = Q.tp + bk * Q.A;
            float mx = l[0];
            for (int a = 1; a < Q.A; ++a) mx = fmaxf(mx, l[a * 16]);
            float S = 0.0f, sp = 0.0f;
            for (int a = 0; a < Q.A; ++a) { S += det_expf(l[a * 16] - mx); sp += pi[a]; }
            const float lS = det_logf(S);
            float ce = 0.0f;
            for (int a = 0; a < Q.A; ++a) {
                const float z = l[a * 16] - mx;
                ce -= pi[a] * (z - lS);
                const float pa = det_expf(z) / S;
                G[hd.y + s + a * 16] = c * (pa * sp - pi[a]);
                Q.pp[bk * Q.A + a] = pa;
            }
            Q.terms[bk * 3 + 1] = ce;
        }
    }
}

// Σ over tiles, applications and samples of dZ ⊗ x for one 16x16 dW block
// (BN: dZ ⊙ γ/√(1+ε); compile-time, so the default nets' loop has no factor).
// The (tile, application) pairs run in groups of BP_DW_U: a group's operand
// loads are all issued before its MFMAs (one memory latency per group, not
// per pair), the MFMAs in the same ascending order
#ifndef BP_DW_U
#define BP_DW_U 4
#endif
template <bool BN>
__device__ __forceinline__ bp_f32x4 bp_dw_acc(const BpDwParams& Q, const BpLayer& L, int o, int i, bool oin, bool iin,
                                              int kq) {
    const float gr = BN && oin ? Q.flat[L.bn_off + L.out + o] / MZ_BN_S : 1.0f;
    bp_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int nu = L.n_use, nn = Q.tiles * nu;
    for (int n0 = 0; n0 < nn; n0 += BP_DW_U) {
        float a[BP_DW_U][4], b[BP_DW_U][4];
#pragma unroll
        for (int q = 0; q < BP_DW_U; ++q) {
            const bool ok = n0 + q < nn;
            const int n = ok ? n0 + q : 0, t = n / nu;        // (past the end: pair 0, its values unused)
            const BpUse U = Q.uses[L.use0 + n - t * nu];
            const float* gt = Q.grad + (size_t)t * Q.tile_floats;
            const float* at = Q.act + (size_t)t * Q.tile_floats;
#pragma unroll
            for (int c = 0; c < 4; ++c) {                     // K = the 16 samples, 4 per MFMA
                const int e = U.y + o * 16 + 4 * c + kq;
                const float dz = ok && oin ? bp_dz(L.act, gt[e], at[e]) : 0.0f;
                a[q][c] = BN ? dz * gr : dz;
                b[q][c] = ok && iin ? at[U.x + i * 16 + 4 * c + kq] : 0.0f;
            }
        }
#pragma unroll
        for (int q = 0; q < BP_DW_U; ++q) {
            if (n0 + q < nn) {
#pragma unroll
                for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][c], b[q][c], acc, 0, 0, 0);
            }
        }
    }
    return acc;
}

// db of output row o (one lane): Σ over tiles, applications and the 16 samples
// of dT in that order (16 contiguous floats per application: their loads are
// issued together, then the ordered sum); BatchNorm: also dβ, dγ.  Writes the
// data terms, returns the rows' θ² (bias, β, γ).
template <bool BN>
__device__ __forceinline__ double bp_db(const BpDwParams& Q, const BpLayer& L, int o) {
    const float gr = BN ? Q.flat[L.bn_off + L.out + o] / MZ_BN_S : 1.0f;
    float s = 0.0f, sbe = 0.0f, sga = 0.0f;
    const int nu = L.n_use, nn = Q.tiles * nu;
    for (int n0 = 0; n0 < nn; n0 += 2) {                      // two (tile, application) pairs' loads at once
        float g[2][16], y[2][16], z[2][16];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const bool ok = n0 + q < nn;
            const int n = ok ? n0 + q : 0, t = n / nu;        // (past the end: pair 0, its values unused)
            const BpUse U = Q.uses[L.use0 + n - t * nu];
            const size_t e = (size_t)t * Q.tile_floats + U.y + o * 16;
            const size_t ez = (size_t)t * Q.tile_floats + U.z + o * 16;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                g[q][j] = ok ? Q.grad[e + j] : 0.0f;
                y[q][j] = ok ? Q.act[e + j] : 0.0f;
                z[q][j] = BN && ok ? Q.act[ez + j] : 0.0f;
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (n0 + q >= nn) break;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const float du = bp_dz(L.act, g[q][j], y[q][j]);
                s += BN ? du * gr : du;
                if (BN) {
                    sbe += du;
                    sga += du * (z[q][j] / MZ_BN_S);
                }
            }
        }
    }
    const float th = Q.flat[L.b_off + o];
    Q.out[L.b_off + o] = s;                                   // data term (2θ: mz_adam_kernel)
    double q = (double)th * (double)th;
    if (BN) {
        const float be = Q.flat[L.bn_off + o], ga = Q.flat[L.bn_off + L.out + o];
        Q.out[L.bn_off + o] = sbe;
        Q.out[L.bn_off + L.out + o] = sga;
        q += (double)be * (double)be + (double)ga * (double)ga;
    }
    return q;
}

extern "C" __global__ __launch_bounds__(64) void mz_bp_dw(BpDwParams Q) {
    const BpJob J = Q.jobs[blockIdx.x];
    const BpLayer L = Q.layers[J.layer];
    const int lane = threadIdx.x, m = lane & 15, kq = lane >> 4;
    const bool bn = L.bn_off >= 0;
    if (J.ib < 0) {                                           // db = Σ dT (data term); BatchNorm: dβ, dγ
        const int o = J.ob * 16 + lane;
        const bool in = lane < 16 && o < L.out;
        double q = 0.0;
        if (in) q = bn ? bp_db<true>(Q, L, o) : bp_db<false>(Q, L, o);
        for (int d = 32; d > 0; d >>= 1) q += __shfl_xor(q, d);    // fixed tree: Σθ² of the block
        if (lane == 0) Q.sq[blockIdx.x] = q;
        return;
    }
    const int o = J.ob * 16 + m, i = J.ib * 16 + m;
    const bool oin = o < L.out, iin = i < L.in;
    const bp_f32x4 acc = bn ? bp_dw_acc<true>(Q, L, o, i, oin, iin, kq) : bp_dw_acc<false>(Q, L, o, i, oin, iin, kq);
    double q = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int oo = J.ob * 16 + kq * 4 + r;
        if (oo < L.out && iin) {
            const size_t p = (size_t)L.w_off + oo + (size_t)L.out * i;
            const float th = Q.flat[p];
            Q.out[p] = acc[r];
            q += (double)th * (double)th;
        }
    }
    for (int d = 32; d > 0; d >>= 1) q += __shfl_xor(q, d);        // fixed tree: Σθ² of the block
    if (lane == 0) Q.sq[blockIdx.x] = q;
}

// blocks 0..2: Σθ² of each net; block 3: the losses (per sample in ascending
// k, then a 256-thread f64 tree over samples)
extern "C" __global__ __launch_bounds__(256) void mz_bp_fold(BpFoldParams Q) {
    __shared__ double red[3][256];
    const int tid = threadIdx.x;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    if (blockIdx.x < 3) {                       // the net's per-block Σθ² of mz_bp_dw, ascending job order
        for (int j = Q.job0[blockIdx.x] + tid; j < Q.job0[blockIdx.x + 1]; j += 256) s0 += Q.sq[j];
    } else {
        const int K1 = Q.K + 1;
        for (int b = tid; b < Q.B; b += 256) {
            float v = 0.0f, p = 0.0f, r = 0.0f;
            for (int k = 0; k < K1; ++k) {
                const float* t = Q.terms + ((size_t)b * K1 + k) * 3;
                v += t[0]; p += t[1]; r += t[2];
            }
            const double c = (double)(Q.weights ? Q.weights[b] : 1.0f) / (double)Q.gscale[b];
            s0 += c * v; s1 += c * r; s2 += c * p;
        }
    }
    red[0][tid] = s0; red[1][tid] = s1; red[2][tid] = s2;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) { red[0][tid] += red[0][tid + o]; red[1][tid] += red[1][tid + o]; red[2][tid] += red[2][tid + o]; }
        __syncthreads();
    }
    if (tid == 0) {
        if (blockIdx.x < 3) {
            Q.losses[3 + blockIdx.x] = (float)red[0][0];
        } else {
            Q.losses[0] = (float)(red[0][0] / Q.B);
            Q.losses[1] = (float)(red[1][0] / Q.B);
            Q.losses[2] = (float)(red[2][0] / Q.B);
        }
    }
}

// ============================================================================
// The corrected learner for the ResNet nets (mz_backprop_params.h RbpApp):
// mz_rbp_sample, one workgroup per sample, its arena T (activations) and G
// (their gradients) in HBM; the current application's input and ∂L/∂t staged
// in LDS.  The parameter gradients: mz_rbp_dw.
#ifndef RBP_THREADS
#define RBP_THREADS 768                      // up to 12 waves: a Connect4 conv has 4 x 3 blocks per pass
#endif

// im2col operand of a conv, input element (k, p) for k = i + kw·j + kw·kh·c:
// x[c] at (px, py) = (p mod W + (kw−1−i) − kw/2, p div W + (kh−1−j) − kh/2),
// zero off the board (Flux's flipped kernel, "same" padding)
// n / d for 0 <= n < 2^20 and a small wave-uniform d, by an f32 reciprocal
// (the quotient's fraction is at least 1/d away from the next integer)
__device__ __forceinline__ int rbp_div(int n, int d, float rd) { return (int)(((float)n + 0.5f) * rd); }

__device__ __forceinline__ float rbp_xhat_k(const float* X, int cin, int kw, int kh, int P, int Wb, int k, int p) {
    const int kk = kw * kh;
    if (k >= kk * cin || p >= P) return 0.0f;
    if (kk == 1) return X[k * P + p];                        // 1x1 conv
    const int c = rbp_div(k, kk, 1.0f / (float)kk), r = k - c * kk;
    const int j = rbp_div(r, kw, 1.0f / (float)kw), i = r - j * kw;
    const int pyy = rbp_div(p, Wb, 1.0f / (float)Wb);
    const int px = p - pyy * Wb + (kw - 1 - i) - kw / 2, py = pyy + (kh - 1 - j) - kh / 2;
    return px >= 0 && px < Wb && py >= 0 && py < P / Wb ? X[c * P + px + Wb * py] : 0.0f;
}
__device__ __forceinline__ float rbp_xhat(const float* X, const RbpApp& L, int P, int Wb, int k, int p) {
    return rbp_xhat_k(X, L.cin, L.kw, L.kh, P, Wb, k, p);
}

// bp_gemm_block with RBP_KC k-steps of operands in flight per full chunk (one
// workgroup per sample leaves the registers for it), then the rest in chunks
// of RBP_KC / 2 whose k-steps past the end are skipped by wave-uniform tests
// (no padded MFMAs): a 1x1 conv over 64 channels (16 k-steps) is one memory
// round trip instead of four of the earlier four-k-step tail
#ifndef RBP_KC
#define RBP_KC 32
#endif
template <class FA, class FB>
__device__ __forceinline__ bp_f32x4 rbp_gemm_block(int nk, int kq, FA fa, FB fb) {
    bp_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int k0 = 0;
    for (; k0 + RBP_KC <= nk; k0 += RBP_KC) {                // full chunks
        float a[RBP_KC], b[RBP_KC];
#pragma unroll
        for (int j = 0; j < RBP_KC; ++j) {
            const int k = (k0 + j) * 4 + kq;
            a[j] = fa(k);
            b[j] = fb(k);
        }
#pragma unroll
        for (int j = 0; j < RBP_KC; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
    }
    constexpr int KH = RBP_KC / 2;
    for (; k0 < nk; k0 += KH) {                               // the rest, KH k-steps at a time
        float a[KH], b[KH];
#pragma unroll
        for (int j = 0; j < KH; ++j) {
            const int k = (k0 + j) * 4 + kq;
            a[j] = fa(k);                                     // fa / fb are zero past the end
            b[j] = fb(k);
        }
#pragma unroll
        for (int j = 0; j < KH; ++j)
            if (k0 + j < nk) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
    }
    return acc;
}

// A k x k conv (odd k, channels a multiple of 4) on a zero-padded board
// ([channel][(Hb + kh − 1)(Wb + kw − 1)], the halo zero): K in tap-major order
// (k = tap·nc + c), so a k-step's tap is wave-uniform and each operand address
// is the lane's base plus a constant — no im2col index arithmetic.  A(row, c,
// tap) = Ab[c·astride + tap]; B(c, tap) = Bp[c·Pp + bofs + sgn·δ(tap)], δ the
// tap's board offset dy·Wp + dx (sgn = −1: the transposed conv).  The sum runs
// in another order than rbp_gemm_block's (within the f32 tolerance).
__device__ __forceinline__ bool rbp_taps(int kw, int kh, int nc) {
    return kw * kh > 1 && (kw & 1) && (kh & 1) && (nc & 3) == 0;
}
__device__ __forceinline__ bp_f32x4 rbp_taps_gemm(const float* Ab, int astride, bool rok, int kw, int kh, int nc,
                                                  const float* Bp, int Pp, int Wp, int bofs, int kq, int sgn) {
    bp_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int ncs = nc >> 2, kk = kw * kh;
    for (int tap = 0; tap < kk; ++tap) {
        const int j = tap / kw, i = tap - j * kw;
        const int delta = sgn * (((kh - 1 - j) - kh / 2) * Wp + ((kw - 1 - i) - kw / 2));
        const float* ab = Ab + kq * astride + tap;
        const float* bb = Bp + kq * Pp + bofs + delta;
        for (int c0 = 0; c0 < ncs; c0 += 16) {
            float a[16], b[16];
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                const bool in = c0 + jj < ncs;
                a[jj] = rok && in ? ab[(size_t)(c0 + jj) * 4 * astride] : 0.0f;
                b[jj] = in ? bb[(c0 + jj) * 4 * Pp] : 0.0f;
            }
#pragma unroll
            for (int jj = 0; jj < 16; ++jj)
                if (c0 + jj < ncs) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[jj], b[jj], acc, 0, 0, 0);
        }
    }
    return acc;
}
// the padded board of a k x k conv: width, cells, the lane's base cell
__device__ __forceinline__ int rbp_pad_w(const RbpApp& L, int Wb) { return Wb + L.kw - 1; }
__device__ __forceinline__ int rbp_pad_n(const RbpApp& L, int Wb, int P) { return (P / Wb + L.kh - 1) * (Wb + L.kw - 1); }
__device__ __forceinline__ int rbp_pad_at(const RbpApp& L, int Wb, int p) {
    const int py = rbp_div(p, Wb, 1.0f / (float)Wb), px = p - py * Wb;
    return (py + L.kh / 2) * (Wb + L.kw - 1) + px + L.kw / 2;
}
// dst[c][padded cell] = src[c][p] (zero off the board), nc channels, all threads
__device__ __forceinline__ void rbp_pad_stage(const RbpApp& L, int Wb, int P, int nc, const float* src, float* dst) {
    const int Wp = rbp_pad_w(L, Wb), Pp = rbp_pad_n(L, Wb, P), Hb = P / Wb;
    const float rPp = 1.0f / (float)Pp, rWp = 1.0f / (float)Wp;
    for (int e = threadIdx.x; e < nc * Pp; e += blockDim.x) {
        const int c = rbp_div(e, Pp, rPp), r = e - c * Pp, ry = rbp_div(r, Wp, rWp), rx = r - ry * Wp;
        const int x = rx - L.kw / 2, y = ry - L.kh / 2;
        dst[e] = x >= 0 && x < Wb && y >= 0 && y < Hb ? src[c * P + y * Wb + x] : 0.0f;
    }
}

// forward: output block (16 channels x 16 positions) u of a conv; the output
// to the arena and to its ring slot Y, the residual from its slot R (or the arena).
// A k x k conv with rbp_taps reads X padded (rbp_pad_stage).
__device__ __forceinline__ void rbp_conv_fwd(const RbpParams& Q, const RbpApp& L, const float* X, float* T, int u,
                                             float* Y, const float* R) {
    const int lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4, P = Q.P;
    const int npb = (P + 15) >> 4, ob = u / npb, pb = u - ob * npb;
    const int K = L.kw * L.kh * L.cin, co = ob * 16 + m, p = pb * 16 + m;
    const float* W = Q.flat + L.w_off;
    bp_f32x4 acc;
    if (rbp_taps(L.kw, L.kh, L.cin))
        acc = rbp_taps_gemm(W + (size_t)K * (co < L.cout ? co : 0), L.kw * L.kh, co < L.cout, L.kw, L.kh, L.cin, X,
                            rbp_pad_n(L, Q.Wb, P), rbp_pad_w(L, Q.Wb), rbp_pad_at(L, Q.Wb, p < P ? p : P - 1), kq, 1);
    else
        acc = rbp_gemm_block((K + 3) >> 2, kq,
            [&](int k) { return co < L.cout && k < K ? W[k + (size_t)K * co] : 0.0f; },
            [&](int k) { return rbp_xhat(X, L, P, Q.Wb, k, p); });
    const int pc = pb * 16 + m;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int o = ob * 16 + kq * 4 + r;
        if (o >= L.cout || pc >= P) continue;
        const int e = o * P + pc;
        const float t = acc[r] + Q.flat[L.b_off + o];
        float v = t;
        if (L.bn_off >= 0) {
            T[L.z + e] = t;
            v = mz_bn_apply(t, Q.flat[L.bn_off + L.cout + o], Q.flat[L.bn_off + o]);
        }
        if (L.res >= 0) v = v + (R ? R[e] : T[L.res + e]);
        v = bp_act(L.act, v);
        T[L.y + e] = v;
        if (Y) Y[e] = v;
    }
}

// A dense layer for one sample, RBP_DS lanes per output (neighbouring lanes,
// strided over the inputs, combined by a fixed xor tree): the input staged in
// XS, so the loads of one lane are independent and in flight together
#define RBP_DS 8
__device__ __forceinline__ void rbp_dense_fwd(const RbpParams& Q, const RbpApp& L, const float* XS, float* T,
                                              float* Y) {
    const float* W = Q.flat + L.w_off;
    const int s0 = threadIdx.x & (RBP_DS - 1);
    for (int o = threadIdx.x / RBP_DS; o < L.cout; o += blockDim.x / RBP_DS) {    // whole lane groups
        float s = 0.0f;
        for (int i = s0; i < L.cin; i += RBP_DS) s = fmaf(W[o + (size_t)L.cout * i], XS[i], s);
#pragma unroll
        for (int w = 1; w < RBP_DS; w <<= 1) s += __shfl_xor(s, w);
        if (s0 == 0) {
            const float v = bp_act(L.act, s + Q.flat[L.b_off + o]);
            T[L.y + o] = v;
            if (Y) Y[o] = v;
        }
    }
}

// G[x] += Wᵀ DT of a dense layer, RBP_DS lanes per input as rbp_dense_fwd
__device__ __forceinline__ void rbp_dense_dx(const RbpParams& Q, const RbpApp& L, const float* DT, float* G,
                                             float* GX) {
    const float* W = Q.flat + L.w_off;
    const int s0 = threadIdx.x & (RBP_DS - 1);
    for (int i = threadIdx.x / RBP_DS; i < L.cin; i += blockDim.x / RBP_DS) {
        float s = 0.0f;
        for (int o = s0; o < L.cout; o += RBP_DS) s = fmaf(W[o + (size_t)L.cout * i], DT[o], s);
#pragma unroll
        for (int w = 1; w < RBP_DS; w <<= 1) s += __shfl_xor(s, w);
        if (s0 == 0) {
            if (GX) GX[i] = (L.gxf ? 0.0f : GX[i]) + s;
            else G[L.x + i] += s;
        }
    }
}

// ∂L/∂t of a conv (t = Wx + b) into DT and the residual input's share of ∂L/∂y;
// ∂L/∂y from its ring slot GY (then written out to the arena for mz_rbp_dw) or
// the arena, the residual share into its slot GR or the arena
__device__ __forceinline__ void rbp_conv_dt(const RbpParams& Q, const RbpApp& L, const float* T, float* G, float* DT,
                                            const float* GY, float* GR) {
    const int P = Q.P;
    // the transposed k x k conv reads DT padded (rbp_taps)
    const bool pad = !L.step && rbp_taps(L.kw, L.kh, L.cout);
    const int Pp = pad ? rbp_pad_n(L, Q.Wb, P) : P;
    for (int e = threadIdx.x; e < L.cout * P; e += blockDim.x) {
        const int o = rbp_div(e, P, 1.0f / (float)P);
        const float g = GY ? GY[e] : G[L.y + e];
        if (GY) G[L.y + e] = g;
        const float du = bp_dz(L.act, g, T[L.y + e]);
        if (L.res >= 0) {
            if (GR) GR[e] = (L.grf ? 0.0f : GR[e]) + du;   // the zeroed arena's sum
            else G[L.res + e] += du;
        }
        const float dt = L.bn_off >= 0 ? du * (Q.flat[L.bn_off + L.cout + o] / MZ_BN_S) : du;
        if (pad) DT[o * Pp + rbp_pad_at(L, Q.Wb, e - o * P)] = dt;
        else DT[e] = dt;
    }
    if (pad) {                                                // the halo of the padded DT
        const int Wp = rbp_pad_w(L, Q.Wb), Hb = P / Q.Wb;
        const float rPp = 1.0f / (float)Pp, rWp = 1.0f / (float)Wp;
        for (int e = threadIdx.x; e < L.cout * Pp; e += blockDim.x) {
            const int c = rbp_div(e, Pp, rPp), r = e - c * Pp, ry = rbp_div(r, Wp, rWp), rx = r - ry * Wp;
            const int x = rx - L.kw / 2, y = ry - L.kh / 2;
            if (!(x >= 0 && x < Q.Wb && y >= 0 && y < Hb)) DT[e] = 0.0f;
        }
    }
}

// G[x] += the transposed conv of DT: input block (16 channels x 16 positions) u
__device__ __forceinline__ void rbp_conv_dx(const RbpParams& Q, const RbpApp& L, const float* DT, float* G, int u,
                                            float* GX) {
    const int lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4, P = Q.P, Wb = Q.Wb;
    const int npb = (P + 15) >> 4, ib = u / npb, pb = u - ib * npb;
    const int kk = L.kw * L.kh, K = kk * L.cin, Kt = kk * L.cout, ci = ib * 16 + m, p = pb * 16 + m;
    const float rkk = 1.0f / (float)kk, rkw = 1.0f / (float)L.kw;
    const int py0 = rbp_div(p, Wb, 1.0f / (float)Wb), px0 = p - py0 * Wb;
    const float* W = Q.flat + L.w_off;
    bp_f32x4 acc;
    if (rbp_taps(L.kw, L.kh, L.cout))                        // DT padded by rbp_conv_dt
        acc = rbp_taps_gemm(W + (size_t)kk * (ci < L.cin ? ci : 0), K, ci < L.cin, L.kw, L.kh, L.cout, DT,
                            rbp_pad_n(L, Wb, P), rbp_pad_w(L, Wb), rbp_pad_at(L, Wb, p < P ? p : P - 1), kq, -1);
    else
    acc = rbp_gemm_block((Kt + 3) >> 2, kq,
        [&](int k) {
            if (ci >= L.cin || k >= Kt) return 0.0f;
            if (kk == 1) return W[ci + (size_t)L.cin * k];
            const int co = rbp_div(k, kk, rkk), tap = k - co * kk;
            return W[tap + kk * ci + (size_t)K * co];
        },
        [&](int k) {
            if (k >= Kt || p >= P) return 0.0f;
            if (kk == 1) return DT[k * P + p];
            const int co = rbp_div(k, kk, rkk), tap = k - co * kk, j = rbp_div(tap, L.kw, rkw), i = tap - j * L.kw;
            const int qx = px0 - ((L.kw - 1 - i) - L.kw / 2), qy = py0 - ((L.kh - 1 - j) - L.kh / 2);
            return qx >= 0 && qx < Wb && qy >= 0 && qy < P / Wb ? DT[co * P + qx + Wb * qy] : 0.0f;
        });
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int c = ib * 16 + kq * 4 + r;
        if (c < L.cin && p < P) {
            if (GX) GX[c * P + p] = (L.gxf ? 0.0f : GX[c * P + p]) + acc[r];
            else G[L.x + c * P + p] += acc[r];
        }
    }
}

// dL/dy of the heads for sample b (bp_heads for one sample)
__device__ __forceinline__ void rbp_heads(const RbpParams& Q, const float* T, float* G, int b) {
    const int K1 = Q.K + 1;
    for (int e = threadIdx.x; e < Q.n_head; e += blockDim.x) {
        const BpHead hd = Q.heads[e];
        const int k = hd.step;
        const float w = Q.weights ? Q.weights[b] : 1.0f;
        const float c = w / (Q.gscale[b] * (float)Q.B);
        const size_t bk = (size_t)b * K1 + k;
        if (hd.kind == BP_HEAD_V || hd.kind == BP_HEAD_R) {
            const bool v = hd.kind == BP_HEAD_V;
            const float y = T[hd.y];
            const float d = y - (v ? Q.tv[bk] : Q.tr[bk]);
            const bool on = v || Q.intermediate_rewards;
            (v ? Q.pv : Q.pr)[bk] = y;
            G[hd.y] = on ? c * 2.0f * d : 0.0f;
            Q.terms[bk * 3 + (v ? 0 : 2)] = on ? d * d : 0.0f;
        } else {                                              // logitcrossentropy on the logits
            const float* l = T + hd.y;
            const float* pi = Q.tp + bk * Q.A;
            float mx = l[0];
            for (int a = 1; a < Q.A; ++a) mx = fmaxf(mx, l[a]);
            float S = 0.0f, sp = 0.0f;
            for (int a = 0; a < Q.A; ++a) { S += det_expf(l[a] - mx); sp += pi[a]; }
            const float lS = det_logf(S);
            float ce = 0.0f;
            for (int a = 0; a < Q.A; ++a) {
                const float z = l[a] - mx;
                ce -= pi[a] * (z - lS);
                const float pa = det_expf(z) / S;
                G[hd.y + a] = c * (pa * sp - pi[a]);
                Q.pp[bk * Q.A + a] = pa;
            }
            Q.terms[bk * 3 + 1] = ce;
        }
    }
}

extern "C" __global__ __launch_bounds__(RBP_THREADS) void mz_rbp_sample(RbpParams Q) {
    extern __shared__ __attribute__((aligned(16))) float rbp_lds[];
    const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x, wave = tid >> 6, nw = nt >> 6, K1 = Q.K + 1;
    float* T = Q.act + (size_t)b * Q.arena;
    float* G = Q.grad + (size_t)b * Q.arena;
    float* DT = rbp_lds;                                      // [dt_floats] ∂L/∂t of the current application
    float* XS = rbp_lds + Q.dt_floats;                        // [xs_floats] its input, staged
    float* ring = XS + Q.xs_floats;                           // recent outputs / gradients, [slot][dt_floats]
    for (int r = 0; r < Q.n_gzero; ++r) {                     // the arena-resident ∂L/∂· (the rest: the ring)
        const int2 z = Q.gzero[r];
        for (int e = tid; e < z.y; e += nt) G[z.x + e] = 0.0f;
    }
    for (int e = tid; e < K1 * 3; e += nt) Q.terms[(size_t)b * K1 * 3 + e] = 0.0f;
    for (int e = tid; e < K1; e += nt) Q.pr[(size_t)b * K1 + e] = 0.0f;        // rewards: 0 at step 0
    for (int e = tid; e < Q.obs_feat; e += nt) T[Q.obs_t + e] = Q.obs[(size_t)b * Q.obs_feat + e];
    __syncthreads();
    const int npb = (Q.P + 15) >> 4;
#ifdef MZ_STAMPS
    if (b == 0 && tid == 0) Q.stamps[0] = __builtin_amdgcn_s_memtime();
#endif
    // ---- forward: representation, K dynamics steps, K+1 predictions (Q10)
    // An application's input comes from its ring slot or is staged from the
    // arena; its output goes to both.  The barrier after it is LDS-only unless a
    // later application reads the arena (fsync: the stores drained first).
    auto lds_barrier = [] {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    for (int a = 0; a < Q.n_app; ++a) {
        const RbpApp L = Q.apps[a];
        float* Y = L.yb >= 0 ? ring + L.yb * Q.dt_floats : nullptr;
        const float* X = L.xb >= 0 ? ring + L.xb * Q.dt_floats : nullptr;
        if (L.op == RBP_CONV && rbp_taps(L.kw, L.kh, L.cin)) {   // the padded input (rbp_taps_gemm)
            rbp_pad_stage(L, Q.Wb, Q.P, L.cin, X ? X : T + L.x, XS);
            lds_barrier();
            X = XS;
        } else if (L.op != RBP_CONCAT && !X) {
            const int n = L.op == RBP_CONV ? L.cin * Q.P : L.cin;
            for (int e = tid; e < n; e += nt) XS[e] = T[L.x + e];
            lds_barrier();
            X = XS;
        }
        if (L.op == RBP_CONV) {
            const float* R = L.rb >= 0 ? ring + L.rb * Q.dt_floats : nullptr;
            const int units = ((L.cout + 15) >> 4) * npb;
            for (int u = wave; u < units; u += nw) rbp_conv_fwd(Q, L, X, T, u, Y, R);
        } else if (L.op == RBP_DENSE) {
            rbp_dense_fwd(Q, L, X, T, Y);
        } else {                                              // make_dynamics_input (:293-304)
            const float av = Q.actions[(size_t)b * K1 + L.step] / (float)Q.A;
            for (int f = tid; f < L.cout; f += nt) {
                const float v = f < L.cin ? (X ? X[f] : T[L.x + f]) * 2.0f : av;
                T[L.y + f] = v;
                if (Y) Y[f] = v;
            }
        }
        if (L.fsync) __syncthreads();
        else lds_barrier();
#ifdef MZ_STAMPS   // sample 0: [0] start, forward application a ends at 1 + a, backward at 2 + n_app + a
        if (b == 0 && tid == 0) Q.stamps[1 + a] = __builtin_amdgcn_s_memtime();
#endif
    }
    rbp_heads(Q, T, G, b);
    __syncthreads();
#ifdef MZ_STAMPS
    if (b == 0 && tid == 0) Q.stamps[1 + Q.n_app] = __builtin_amdgcn_s_memtime();
#endif
    // ---- backward, reverse order: the input gradients (the parameter
    // gradients are mz_rbp_dw's, from the arenas this leaves behind)
    for (int a = Q.n_app - 1; a >= 0; --a) {
        const RbpApp L = Q.apps[a];
        const float* GY = L.gyb >= 0 ? ring + L.gyb * Q.dt_floats : nullptr;
        float* GX = L.gxb >= 0 ? ring + L.gxb * Q.dt_floats : nullptr;
        if (L.op == RBP_CONV) {
            rbp_conv_dt(Q, L, T, G, DT, GY, L.grb >= 0 ? ring + L.grb * Q.dt_floats : nullptr);
            if (!L.step) {
                lds_barrier();
                const int ndx = ((L.cin + 15) >> 4) * npb;
                for (int u = wave; u < ndx; u += nw) rbp_conv_dx(Q, L, DT, G, u, GX);
            }
        } else if (L.op == RBP_DENSE) {
            for (int o = tid; o < L.cout; o += nt) {
                const float g = GY ? GY[o] : G[L.y + o];
                if (GY) G[L.y + o] = g;
                DT[o] = bp_dz(L.act, g, T[L.y + o]);
            }
            if (!L.step) {
                lds_barrier();
                rbp_dense_dx(Q, L, DT, G, GX);
            }
        } else {                                              // ∂(2h)/∂h
            for (int f = tid; f < L.cout; f += nt) {
                const float g = GY ? GY[f] : G[L.y + f];
                if (GY) G[L.y + f] = g;
                if (f < L.cin) {
                    if (GX) GX[f] = (L.gxf ? 0.0f : GX[f]) + 2.0f * g;
                    else G[L.x + f] += 2.0f * g;
                }
            }
        }
        if (L.bsync) __syncthreads();
        else lds_barrier();
#ifdef MZ_STAMPS
        if (b == 0 && tid == 0) Q.stamps[2 + Q.n_app + a] = __builtin_amdgcn_s_memtime();
#endif
    }
}

// The parameter gradients of the ResNet nets, one workgroup of RBP_DW_WAVES
// waves per job (a 16x16 block of a layer's W, or the db / dβ / dγ of 16 output
// channels): Σ over samples b, the layer's applications u and positions p (f32
// MFMA with K = that flattened index, four per step) of ∂L/∂t ⊗ the im2col
// input — ∂L/∂t re-formed from the arenas (dt = du·γ/√(1+ε) with BatchNorm,
// du = ∂L/∂y ⊙ act'(y)) as mz_rbp_sample formed it.  Wave w sums the (b, u)
// pairs w, w + RBP_DW_WAVES, ..; a pair's addresses are wave-uniform and its
// positions' loads are issued together; the waves' partial sums are added in
// wave order.  Writes the data term and the block's Σθ² (f64, fixed tree).
#define RBP_DW_ST 12                          // k-steps (4 positions each) loaded at once
extern "C" __global__ __launch_bounds__(64 * RBP_DW_WAVES) void mz_rbp_dw(RbpDwParams Q) {
    __shared__ float red[RBP_DW_WAVES][4][64];
    const RbpJob J = Q.jobs[blockIdx.x];
    const RbpLayer L = Q.layers[J.layer];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4;
    const int P = L.conv ? Q.P : 1, npair = Q.B * L.n_use;
    const bool bn = L.conv && L.bn_off >= 0;
    // the wave's pairs: pr = wave + RBP_DW_WAVES·i, (b, u) kept incrementally
    auto pair_walk = [&](auto&& body) {
        int b = 0, u = wave;
        while (u >= L.n_use && L.n_use > 0) { u -= L.n_use; ++b; }
        for (int pr = wave; pr < npair; pr += RBP_DW_WAVES) {
            body(b, Q.uses[L.use0 + u]);
            u += RBP_DW_WAVES;
            while (u >= L.n_use) { u -= L.n_use; ++b; }
        }
    };
    float part[4] = {0.f, 0.f, 0.f, 0.f};
    if (J.kb < 0) {                                           // db, dβ, dγ of channels ob·16 + m
        const int o = J.ob * 16 + m;
        const bool in = o < L.cout;
        const float gr = bn && in ? Q.flat[L.bn_off + L.cout + o] / MZ_BN_S : 1.0f;
        float sb = 0.0f, sbe = 0.0f, sga = 0.0f;
        if (in)
            pair_walk([&](int b, const RbpUse& U) {
                const float* T = Q.act + (size_t)b * Q.arena;
                const float* G = Q.grad + (size_t)b * Q.arena;
                for (int p = kq; p < P; p += 4) {             // quarter kq of the positions
                    const int e = o * P + p;
                    const float du = bp_dz(L.act, G[U.y + e], T[U.y + e]);
                    sb += bn ? du * gr : du;
                    if (bn) { sbe += du; sga += du * (T[U.z + e] / MZ_BN_S); }
                }
            });
        // the four quarters in a fixed order: (q0 + q1) + (q2 + q3)
        sb += __shfl_xor(sb, 16); sb += __shfl_xor(sb, 32);
        sbe += __shfl_xor(sbe, 16); sbe += __shfl_xor(sbe, 32);
        sga += __shfl_xor(sga, 16); sga += __shfl_xor(sga, 32);
        part[0] = sb; part[1] = sbe; part[2] = sga;
    } else {                                                  // W block (rows ob·16.., columns kb·16..)
        const int K = L.conv ? L.kw * L.kh * L.cin : L.cin;
        const int co = J.ob * 16 + m, kc = J.kb * 16 + m;
        const bool oin = co < L.cout, kin = kc < K;
        const float gr = bn && oin ? Q.flat[L.bn_off + L.cout + co] / MZ_BN_S : 1.0f;
        bp_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if (L.conv) {
            // the lane's im2col column kc: channel c, tap offsets (dx, dy) (Flux's
            // flipped kernel, "same" padding: rbp_xhat_k)
            const int kk = L.kw * L.kh, c = kin ? kc / kk : 0, tap = kin ? kc - c * kk : 0;
            const int tj = tap / L.kw, ti = tap - tj * L.kw;
            const int dx = (L.kw - 1 - ti) - L.kw / 2, dy = (L.kh - 1 - tj) - L.kh / 2, Wb = Q.Wb, Hb = P / Wb;
            const float rW = 1.0f / (float)Wb;
            const int nst = (P + 3) >> 2;
            pair_walk([&](int b, const RbpUse& U) {
                const float* T = Q.act + (size_t)b * Q.arena;
                const float* G = Q.grad + (size_t)b * Q.arena;
                const float* X = T + U.x + c * P;
                for (int s0 = 0; s0 < nst; s0 += RBP_DW_ST) {
                    float a[RBP_DW_ST], x[RBP_DW_ST];
#pragma unroll
                    for (int j = 0; j < RBP_DW_ST; ++j) {
                        const int p = (s0 + j) * 4 + kq;
                        const bool pin = p < P;
                        const int e = U.y + co * P + p;
                        const float du = oin && pin ? bp_dz(L.act, G[e], T[e]) : 0.0f;
                        a[j] = bn ? du * gr : du;
                        float v = 0.0f;
                        if (kin && pin) {
                            if (kk == 1) {
                                v = X[p];
                            } else {
                                const int py = rbp_div(p, Wb, rW), px = p - py * Wb + dx, qy = py + dy;
                                v = px >= 0 && px < Wb && qy >= 0 && qy < Hb ? X[px + Wb * qy] : 0.0f;
                            }
                        }
                        x[j] = v;
                    }
#pragma unroll
                    for (int j = 0; j < RBP_DW_ST; ++j)
                        if (s0 + j < nst) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], x[j], acc, 0, 0, 0);
                }
            });
        } else {                                              // dense: K = the pairs, four per k-step
            const int nk = (npair + 3) >> 2, kb0 = nk * wave / RBP_DW_WAVES, kb1 = nk * (wave + 1) / RBP_DW_WAVES;
            const float rn = 1.0f / (float)L.n_use;
            acc = rbp_gemm_block(kb1 - kb0, kq,
                [&](int k) {
                    const int t = k + 4 * kb0;
                    if (!oin || t >= npair) return 0.0f;
                    const int b = rbp_div(t, L.n_use, rn), u = t - b * L.n_use;
                    const size_t base = (size_t)b * Q.arena + Q.uses[L.use0 + u].y + co;
                    return bp_dz(L.act, Q.grad[base], Q.act[base]);
                },
                [&](int k) {
                    const int t = k + 4 * kb0;
                    if (!kin || t >= npair) return 0.0f;
                    const int b = rbp_div(t, L.n_use, rn), u = t - b * L.n_use;
                    return Q.act[(size_t)b * Q.arena + Q.uses[L.use0 + u].x + kc];
                });
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) part[r] = acc[r];
    }
    // the waves' partial sums, added in wave order
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][r][lane] = part[r];
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float v = red[0][r][lane];
        for (int w = 1; w < RBP_DW_WAVES; ++w) v += red[w][r][lane];
        part[r] = v;
    }
    double q = 0.0;
    if (J.kb < 0) {
        const int o = J.ob * 16 + m;
        if (kq == 0 && o < L.cout) {
            const float tb = Q.flat[L.b_off + o];
            Q.out[L.b_off + o] = part[0];
            q = (double)tb * (double)tb;
            if (bn) {
                const float tbe = Q.flat[L.bn_off + o], tga = Q.flat[L.bn_off + L.cout + o];
                Q.out[L.bn_off + o] = part[1];
                Q.out[L.bn_off + L.cout + o] = part[2];
                q += (double)tbe * (double)tbe + (double)tga * (double)tga;
            }
        }
    } else {
        const int K = L.conv ? L.kw * L.kh * L.cin : L.cin, kc = J.kb * 16 + m;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int o = J.ob * 16 + kq * 4 + r;
            if (o < L.cout && kc < K) {
                const size_t w = (size_t)L.w_off + (L.conv ? kc + (size_t)K * o : o + (size_t)L.cout * kc);
                const float th = Q.flat[w];
                Q.out[w] = part[r];
                q += (double)th * (double)th;
            }
        }
    }
    for (int d = 32; d > 0; d >>= 1) q += __shfl_xor(q, d);        // fixed tree: Σθ² of the block
    if (lane == 0) Q.sq[blockIdx.x] = q;
}
