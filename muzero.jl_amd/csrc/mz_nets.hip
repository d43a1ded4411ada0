// mz_nets.hip — batched network forward (the Flux Chain calls of
// Learning.jl:87-142) and the learner step of Learning.jl:327-413 in
// ref_semantics: K-step unroll (Q10), losses (:261-288), gradient 2θ (Q11),
// ADAM (Flux 0.12 ADAMW()[1]) and re-packing of the MFMA weight image.
#include "mz_mlp_device.h"

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
        if (tid < MZ_TILE && t0 + tid < P.B) {
            const int j = tid;
            const size_t b = (size_t)(t0 + j);
            const float v = mz_post_act(P.lay.v_act, act[P.lay.v_out + j]);
            float m = act[P.lay.p_out + j];
            for (int k = 1; k < A; ++k) { const float x = act[P.lay.p_out + k * 16 + j]; m = m > x ? m : x; }
            float s = 0.0f;
            for (int k = 0; k < A; ++k) s = s + det_expf(act[P.lay.p_out + k * 16 + j] - m);
            for (int k = 0; k < A; ++k) {
                const float p = det_expf(act[P.lay.p_out + k * 16 + j] - m) / s;
                P.pp[(b * (K + 1) + i) * A + k] = p;
                if (i == 1) P.pp[(b * (K + 1)) * A + k] = p;
            }
            P.pv[b * (K + 1) + i] = v;
            P.pr[b * (K + 1) + i] = mz_post_act(P.lay.r_act, act[P.lay.r_out + j]);
            if (i == 1) { P.pv[b * (K + 1)] = v; P.pr[b * (K + 1)] = 0.0f; }
        }
        __syncthreads();
    }
}

// Losses of Learning.jl:261-288 (diagnostic in ref_semantics, Q11): one
// workgroup.  The per-(sample, step) terms — squared value error and the
// policy cross-entropy of that step — are computed by all threads into
// `terms` (2 x B(K+1) floats, global scratch); then each sample folds its
// steps in ascending k as the oracle does, and the cross-sample sums are
// f64 (tolerance-checked, not bitwise).  out[0] value, out[2] policy.
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_loss_kernel(
    int B, int K, int A, const float* pv, const float* pp, const float* tv, const float* tp,
    const float* gscale, float* terms, float* out) {
    __shared__ double red_v[MZ_THREADS], red_p[MZ_THREADS], red_c[MZ_THREADS];
    const int tid = threadIdx.x;
    const int n = B * (K + 1);
    float* vsq = terms;
    float* cet = terms + n;
    for (int t = tid; t < n; t += blockDim.x) {
        const float d = pv[t] - tv[t];
        vsq[t] = d * d;
        const float* yh = pp + (size_t)t * A;
        const float* y = tp + (size_t)t * A;
        float m = yh[0];
        for (int i = 1; i < A; ++i) m = m > yh[i] ? m : yh[i];
        float se = 0.0f;
        for (int i = 0; i < A; ++i) se = se + det_expf(yh[i] - m);
        const float ls = det_logf(se);
        float ce = 0.0f;
        for (int i = 0; i < A; ++i) ce = ce + y[i] * ((yh[i] - m) - ls);
        cet[t] = ce;
    }
    __syncthreads();                            // block-scope: the terms are visible
    double sv = 0.0, sg = 0.0, sc = 0.0;
    for (int j = tid; j < B; j += blockDim.x) {
        float s = 0.0f, c = 0.0f;
        for (int k = 0; k <= K; ++k) {
            s = s + vsq[(size_t)j * (K + 1) + k];
            c = c + (-cet[(size_t)j * (K + 1) + k]);
        }
        sv += (double)(s / gscale[j]);
        sc += (double)c;                        // Σ_k ce_k
        sg += 1.0 / (double)gscale[j];          // Σ_j 1/g_j
    }
    red_v[tid] = sv; red_p[tid] = sg; red_c[tid] = sc;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (tid < o) { red_v[tid] += red_v[tid + o]; red_p[tid] += red_p[tid + o]; red_c[tid] += red_c[tid + o]; }
        __syncthreads();
    }
    if (tid == 0) {
        out[0] = (float)(red_v[0] / (double)B);
        out[1] = 0.0f;                          // intermediate_rewards = false (:276-280)
        out[2] = (float)(red_c[0] * red_p[0] / ((double)B * (double)B));  // mean over (1,B,B), Q11
    }
}

// Σθ² per net (sum(sqnorm, params), :287) in f64, deterministic: block b of
// net `blockIdx.y` sums a fixed slice in a fixed order into part[net][b];
// mz_l2_finish_kernel adds the partials in ascending b.
#define MZ_L2_BLOCKS 32
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_sqnorm_kernel(const float* flat, const size_t* off,
                                                                          const size_t* cnt, double* part) {
    __shared__ double red[MZ_THREADS];
    const int net = blockIdx.y;
    const float* P = flat + off[net];
    const size_t n = cnt[net];
    double s = 0.0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += (double)P[i] * (double)P[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[net * MZ_L2_BLOCKS + blockIdx.x] = red[0];
}

extern "C" __global__ void mz_l2_finish_kernel(const double* part, float* out) {
    if (threadIdx.x < 3) {
        double s = 0.0;
        for (int b = 0; b < MZ_L2_BLOCKS; ++b) s += part[threadIdx.x * MZ_L2_BLOCKS + b];
        out[3 + threadIdx.x] = (float)s;
    }
}

// gradient of the ref_semantics loss: only sum(sqnorm, params) depends on
// the parameters (Q11), so ∇ = 2θ exactly.
extern "C" __global__ void mz_grad_2theta_kernel(const float* P, float* G, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        G[i] = P[i] * 2.0f;
}

// Flux 0.12 apply!(ADAM) + WeightDecay(0) + `x .-= Δ` (Learning.jl:395-397).
// grad = G[i] * gscale (gscale = 1/world after an all-reduce sum; exact for
// power-of-two world sizes).  bp = (β1^t, β2^t) of the current step.
extern "C" __global__ void mz_adam_kernel(float* P, float* M, float* V, const float* G, float gscale,
                                          size_t n, double bp1, double bp2, double eta) {
    const double b1 = 0.9, b2 = 0.999, eps = 1e-8;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float g = G[i] * gscale;
        const float m = (float)(b1 * (double)M[i] + (1.0 - b1) * (double)g);
        const float g2 = g * g;
        const float v = (float)(b2 * (double)V[i] + (1.0 - b2) * (double)g2);
        M[i] = m; V[i] = v;
        const float d = (float)((double)m / (1.0 - bp1) / (sqrt((double)v / (1.0 - bp2)) + eps) * eta);
        P[i] = P[i] - d;
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
