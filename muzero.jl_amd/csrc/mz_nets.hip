// mz_nets.hip — batched network forward (the Flux Chain calls of
// Learning.jl:87-142) and the learner step of Learning.jl:327-413 in
// ref_semantics: K-step unroll (Q10), losses (:261-288), gradient 2θ (Q11:
// a zero data term, 2θ added by the ADAM kernel),
// ADAM (Flux 0.12 ADAMW()[1]) and re-packing of the MFMA weight image.
#include "mz_mlp_device.h"
#include "mz_tree_device.h"
#include "mz_learner_device.h"
#include "mz_small_params.h"

// One plan over tiles of 16 samples: x (in_feat, n) column-major in HBM ->
// LDS -> plan -> out0 (o0 rows) / out1 (o1 rows, softmaxed if sm1).
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_forward_kernel(
    const int* plan, const float* Wp, const float* Bp, int total_lds, int in_off, int in_feat,
    const float* x, int n, int out0_off, int o0, float* out0, int out1_off, int o1, float* out1, int sm1,
    int act0, int act1) {
    extern __shared__ __attribute__((aligned(16))) float act[];
    const int tid = threadIdx.x;
    const int t0 = blockIdx.x * MZ_TILE;
    for (int i = tid; i < total_lds; i += blockDim.x) act[i] = 0.0f;
    __syncthreads();
    for (int i = tid; i < MZ_TILE * in_feat; i += blockDim.x) {
        const int j = i / in_feat, k = i - j * in_feat;
        if (t0 + j < n) act[in_off + k * 16 + j] = x[(size_t)(t0 + j) * in_feat + k];
    }
    __syncthreads();
    run_plan(plan, Wp, Bp, act);
    for (int i = tid; i < MZ_TILE * o0; i += blockDim.x) {
        const int j = i / o0, k = i - j * o0;
        if (t0 + j < n) out0[(size_t)(t0 + j) * o0 + k] = mz_post_act(act0, act[out0_off + k * 16 + j]);
    }
    if (out1) {
        if (sm1) {
            const int j = tid;
            if (j < MZ_TILE && t0 + j < n) {       // NNlib softmax, one lane per sample
                float m = act[out1_off + j];
                for (int k = 1; k < o1; ++k) { const float v = act[out1_off + k * 16 + j]; m = m > v ? m : v; }
                float s = 0.0f;
                for (int k = 0; k < o1; ++k) s = s + det_expf(act[out1_off + k * 16 + j] - m);
                for (int k = 0; k < o1; ++k)
                    out1[(size_t)(t0 + j) * o1 + k] = det_expf(act[out1_off + k * 16 + j] - m) / s;
            }
        } else {
            for (int i = tid; i < MZ_TILE * o1; i += blockDim.x) {
                const int j = i / o1, k = i - j * o1;
                if (t0 + j < n) out1[(size_t)(t0 + j) * o1 + k] = mz_post_act(act1, act[out1_off + k * 16 + j]);
            }
        }
    }
}



// The unroll of Learning.jl:347-370: representation(obs) then K steps of
// prediction(h) ‖ dynamics(2h ⊕ a_i/|A|).  prediction(h0) is evaluated once
// and stored twice (:351 and :356 at i=1 compute the same thing, Q10).
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_unroll_kernel(UnrollParams P) {
    extern __shared__ __attribute__((aligned(16))) float act[];
    const int tid = threadIdx.x;
    const int t0 = blockIdx.x * MZ_TILE;
    const int K = P.K, A = P.A, H = P.H;
    for (int i = tid; i < P.lay.total; i += blockDim.x) act[i] = 0.0f;
    __syncthreads();
    for (int i = tid; i < MZ_TILE * P.obs_feat; i += blockDim.x) {
        const int j = i / P.obs_feat, k = i - j * P.obs_feat;
        if (t0 + j < P.B) act[P.lay.x_rep + k * 16 + j] = P.obs[(size_t)(t0 + j) * P.obs_feat + k];
    }
    __syncthreads();
    run_plan(P.plan_repr, P.Wp, P.Bp, act);
    for (int i = 1; i <= K; ++i) {
        for (int t = tid; t < MZ_TILE * H; t += blockDim.x) {
            const int j = t / H, k = t - j * H;
            const float h = act[P.lay.h_out + k * 16 + j];
            act[P.lay.x_pred + k * 16 + j] = h;
            act[P.lay.x_dyn + k * 16 + j] = h * 2.0f;          // make_dynamics_input (:299)
        }
        for (int t = tid; t < MZ_TILE * P.plane; t += blockDim.x) {
            const int j = t / P.plane, k = t - j * P.plane;
            float av = 0.0f;
            if (t0 + j < P.B) av = P.actions[(size_t)(t0 + j) * (K + 1) + (i - 1)] / (float)A;  // :294
            act[P.lay.x_dyn + (H + k) * 16 + j] = av;
        }
        __syncthreads();
        run_plan(P.plan_sim, P.Wp, P.Bp, act);
        if (tid < MZ_TILE && t0 + tid < P.B) {        // raw outputs; read-outs in mz_learner_grad_kernel
            const int j = tid;
            const size_t b = (size_t)(t0 + j);
            for (int k = 0; k < A; ++k) {
                const float x = act[P.lay.p_out + k * 16 + j];
                P.pp[(b * (K + 1) + i) * A + k] = x;
                if (i == 1) P.pp[(b * (K + 1)) * A + k] = x;
            }
            const float v = act[P.lay.v_out + j];
            P.pv[b * (K + 1) + i] = v;
            P.pr[b * (K + 1) + i] = act[P.lay.r_out + j];
            if (i == 1) { P.pv[b * (K + 1)] = v; P.pr[b * (K + 1)] = 0.0f; }
        }
        __syncthreads();
    }
}

// One launch after the unroll (Learning.jl:261-288, 380-393 in ref_semantics;
// pieces in mz_learner_device.h):
//  * blocks [0, nlb): one GW-lane group per (sample, step), lg_step_terms;
//  * blocks [nlb, nlb + 3·MZ_L2_BLOCKS): lg_l2_slice (Σθ², the data term
//    of ∇ (0) or the fused ADAM);
//  * the last block out folds (lg_fold).
template <int GW>
__device__ __forceinline__ void learner_grad_body(
    int B, int K, int A, int v_act, int r_act, float* pv, float* pp, float* pr, const float* tv, const float* tp,
    const float* gscale, float* terms, float* flat, const size_t* netoff, float* G, double* part,
    unsigned* counter, float* out, const float* wts, LgAdam ad) {
    __shared__ double red[MZ_THREADS];
    __shared__ float stg[MZ_THREADS];
    const int tid = threadIdx.x;
    const int n = B * (K + 1);
    const int nlb = (n + MZ_THREADS / GW - 1) / (MZ_THREADS / GW);
    float* vsq = terms;
    float* cet = terms + n;
    if ((int)blockIdx.x < nlb) {
        const int t = blockIdx.x * (MZ_THREADS / GW) + tid / GW, a = tid % GW;
        if (t < n)                              // whole GW-lane groups are in or out
            lg_step_terms<GW>(t, a, A, v_act, r_act, pv, pp, pr, tv, tp, vsq, cet, stg + (tid & ~(GW - 1)));
    } else {
        const int nb = blockIdx.x - nlb;
        const int net = nb / MZ_L2_BLOCKS, blk = nb % MZ_L2_BLOCKS;
        red[tid] = lg_l2_slice(net, blk, tid, netoff, flat, G, ad);
        lg_tree256(red, tid);
        if (tid == 0) __hip_atomic_store(part + net * MZ_L2_BLOCKS + blk, red[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    lg_fold(B, K, vsq, cet, gscale, wts, part, counter, out);
}
#define MZ_LG_ARGS int B, int K, int A, int v_act, int r_act, float* pv, float* pp, float* pr, const float* tv, \
    const float* tp, const float* gscale, float* terms, float* flat, const size_t* netoff, float* G, \
    double* part, unsigned* counter, float* out, const float* wts, LgAdam ad
#define MZ_LG_CALL B, K, A, v_act, r_act, pv, pp, pr, tv, tp, gscale, terms, flat, netoff, G, part, counter, out, wts, ad
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_learner_grad_kernel(MZ_LG_ARGS) {
    learner_grad_body<16>(MZ_LG_CALL);
}
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_learner_grad_kernel32(MZ_LG_ARGS) {
    learner_grad_body<32>(MZ_LG_CALL);
}

// mz_learner_loss_multi: the loss blocks of mz_learner_grad_kernel for step
// blockIdx.y of a multi-step sub-chunk (LossMultiParams), folded per step
template <int GW>
__device__ __forceinline__ void loss_multi_body(const LossMultiParams& M) {
    __shared__ float stg[MZ_THREADS];
    const int tid = threadIdx.x, z = blockIdx.y;
    const int n = M.B * (M.K + 1);
    float* vsq = M.terms + 2 * z * M.s_k1;
    float* cet = vsq + M.s_k1;
    float* pv = M.pv + z * M.s_k1;
    float* pp = M.pp + z * M.s_tp;
    float* pr = M.pr + z * M.s_k1;
    const int t = blockIdx.x * (MZ_THREADS / GW) + tid / GW, a = tid % GW;
    if (t < n)
        lg_step_terms<GW>(t, a, M.A, M.v_act, M.r_act, pv, pp, pr, M.tv + z * M.s_k1, M.tp + z * M.s_tp, vsq, cet,
                          stg + (tid & ~(GW - 1)));
    lg_fold(M.B, M.K, vsq, cet, M.gs + (size_t)z * M.B, nullptr, M.part + (size_t)z * 3 * MZ_L2_BLOCKS,
            M.counter + z * MZ_MULTI_CNT_STRIDE, M.out_last && z == M.L - 1 ? M.out_last : M.out + 8 * z,
            (unsigned)M.nlb);
}
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_learner_loss_multi(LossMultiParams M) { loss_multi_body<16>(M); }
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_learner_loss_multi32(LossMultiParams M) {
    loss_multi_body<32>(M);
}

// ADAM over all parameters (adam_update): ∇ = G[i]·gscale + 2θ_i, G the
// data term of the gradient (summed over the ranks by the caller's
// all-reduce; zero in ref_semantics), gscale = 1/world, and 2θ = ∂Σθ²/∂θ
// added here, after the exchange: it is the same on every rank, so an
// exchange that carried it (Σ_r 2θ · 1/world) would round differently from
// 2θ for most worlds (a sequential f32 sum of eight equal terms is not 8x for
// ~44 % of inputs).  At world 1, G·1 + 2θ is the single-GPU gradient bit for
// bit (the corrected kernels' old s + 2θ).
extern "C" __global__ void mz_adam_kernel(float* P, float* M, float* V, const float* G, float gscale,
                                          size_t n, double bp1, double bp2, double eta, float* Wp, float* Bp,
                                          const int* inv_tile, float* smw, float* smb, const int* inv_small) {
    const LgAdam ad{1, M, V, bp1, bp2, eta, Wp, Bp, inv_tile, smw, smb, inv_small};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float d = G[i] * gscale;
        adam_update(ad, P, i, d + P[i] * 2.0f);
    }
}

// Rebuild the MFMA weight image from the Flux-order flat parameters:
// packed[i] = src[i] >= 0 ? flat[src[i]] : 0.
extern "C" __global__ void mz_repack_kernel(const float* flat, const int* src, float* packed, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int s = src[i];
        packed[i] = s >= 0 ? flat[s] : 0.0f;
    }
}
