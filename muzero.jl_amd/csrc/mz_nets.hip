// mz_nets.hip — batched network forward (the Flux Chain calls of
// Learning.jl:87-142) and the learner step of Learning.jl:327-413 in
// ref_semantics: K-step unroll (Q10), losses (:261-288), gradient 2θ (Q11),
// ADAM (Flux 0.12 ADAMW()[1]) and re-packing of the MFMA weight image.
#include "mz_mlp_device.h"
#include "mz_tree_device.h"

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

// One launch after the unroll (Learning.jl:261-288, 380-393 in ref_semantics):
//  * blocks [0, nlb): one 16-lane group per (sample, step) t, lane a = action
//    a: read-outs on the raw unroll outputs — policy = softmax of the logits
//    (max, det_expf, ascending sum, divide), value / reward = their
//    activations — then the step's terms: squared value error and the
//    logitcrossentropy of the probabilities (Q11's double softmax), every
//    sum in ascending action order (g16_seqsum);
//  * blocks [nlb, nlb + 3·MZ_L2_BLOCKS): θ² of a fixed slice summed in f64,
//    and ∇ = 2θ written for it (Q11: only sum(sqnorm, params) depends on θ);
//  * the last block to finish folds each sample's steps in ascending k, the
//    cross-sample sums in f64 (tolerance-checked, not bitwise), and the Σθ²
//    partials in a fixed order (one wave per net), then resets the counter.
// out: [0] value, [1] reward (0, intermediate_rewards = false), [2] policy,
// [3..5] Σθ² of repr / pred / dyn.

// Flux 0.12 apply!(ADAM) + WeightDecay(0) + `x .-= Δ` (Learning.jl:395-397)
// for parameter i with gradient g.  bp = (β1^t, β2^t) of the current step.
// The new value is also scattered into the search / unroll images through
// the inverse maps (each parameter has one position in each image), so the
// images never need a repack after a learner step.
__device__ __forceinline__ void mz_scatter(float x, int code, float* w, float* b) {
    if (code >= 0) w[code] = x;
    else if (code <= -2) b[-code - 2] = x;
}
// adam_update of P[i0 + u·stride] (u < 4, u·stride < rem) with g = 2·x[u]
// (x[u] = the current value): all loads first, then the four updates
__device__ __forceinline__ void adam_update4(const LgAdam& ad, float* P, size_t i0, size_t stride, size_t rem,
                                             const float (&x)[4]) {
    const double b1 = 0.9, b2 = 0.999, eps = 1e-8;
    float mo[4], vo[4];
    int it[4], is[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const size_t i = i0 + u * stride;
        const bool in = u * stride < rem;
        mo[u] = in ? ad.M[i] : 0.0f; vo[u] = in ? ad.V[i] : 0.0f;
        it[u] = in ? ad.inv_tile[i] : -1; is[u] = in ? ad.inv_small[i] : -1;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        if (u * stride >= rem) continue;
        const size_t i = i0 + u * stride;
        const float g = x[u] * 2.0f;
        const float m = (float)(b1 * (double)mo[u] + (1.0 - b1) * (double)g);
        const float g2 = g * g;
        const float v = (float)(b2 * (double)vo[u] + (1.0 - b2) * (double)g2);
        ad.M[i] = m; ad.V[i] = v;
        const float d = (float)((double)m / (1.0 - ad.bp1) / (sqrt((double)v / (1.0 - ad.bp2)) + eps) * ad.eta);
        const float xn = x[u] - d;
        P[i] = xn;
        mz_scatter(xn, it[u], ad.Wp, ad.Bp);
        mz_scatter(xn, is[u], ad.smw, ad.smb);
    }
}
__device__ __forceinline__ void adam_update(const LgAdam& ad, float* P, size_t i, float g) {
    const double b1 = 0.9, b2 = 0.999, eps = 1e-8;
    const float m = (float)(b1 * (double)ad.M[i] + (1.0 - b1) * (double)g);
    const float g2 = g * g;
    const float v = (float)(b2 * (double)ad.V[i] + (1.0 - b2) * (double)g2);
    ad.M[i] = m; ad.V[i] = v;
    const float d = (float)((double)m / (1.0 - ad.bp1) / (sqrt((double)v / (1.0 - ad.bp2)) + eps) * ad.eta);
    const float x = P[i] - d;
    P[i] = x;
    mz_scatter(x, ad.inv_tile[i], ad.Wp, ad.Bp);
    mz_scatter(x, ad.inv_small[i], ad.smw, ad.smb);
}
#define MZ_FOLD_K1 8    // K + 1 up to this: the fold stages the step terms in LDS
template <int GW>
__device__ __forceinline__ void learner_grad_body(
    int B, int K, int A, int v_act, int r_act, float* pv, float* pp, float* pr, const float* tv, const float* tp,
    const float* gscale, float* terms, float* flat, const size_t* netoff, float* G, double* part,
    unsigned* counter, float* out, const float* wts, LgAdam ad) {
    __shared__ double red_v[MZ_THREADS], red_p[MZ_THREADS], red_c[MZ_THREADS];
    __shared__ float stg[MZ_THREADS];
    __shared__ bool last;
    const int tid = threadIdx.x;
    const int n = B * (K + 1);
    const int nlb = (n + MZ_THREADS / GW - 1) / (MZ_THREADS / GW);
    float* vsq = terms;
    float* cet = terms + n;
    if ((int)blockIdx.x < nlb) {
        const int t = blockIdx.x * (MZ_THREADS / GW) + tid / GW, a = tid % GW;
        float* st = stg + (tid & ~(GW - 1));
        if (t < n) {                            // whole GW-lane groups are in or out
            const bool in = a < A;
            float* yh = pp + (size_t)t * A;
            const float x = in ? yh[a] : -INFINITY;
            const float m = gmax<GW>(x);
            const float e = in ? det_expf(x - m) : 0.0f;
            const float s = gseqsum<GW>(e, A, st, a);
            const float p = in ? e / s : -INFINITY;
            if (in) yh[a] = p;
            const float m2 = gmax<GW>(p);
            const float e2 = in ? det_expf(p - m2) : 0.0f;
            const float se = gseqsum<GW>(e2, A, st, a);
            const float ls = det_logf(se);
            const float term = in ? tp[(size_t)t * A + a] * ((p - m2) - ls) : 0.0f;
            const float ce = gseqsum<GW>(term, A, st, a);
            if (a == 0) {
                const float v = mz_post_act(v_act, pv[t]);
                pv[t] = v;
                pr[t] = mz_post_act(r_act, pr[t]);
                const float d = v - tv[t];
                vsq[t] = d * d;
                cet[t] = ce;
            }
        }
    } else {
        const int nb = blockIdx.x - nlb;
        const int net = nb / MZ_L2_BLOCKS, blk = nb % MZ_L2_BLOCKS;
        const size_t off = netoff[net], cnt = netoff[3 + net];
        double s = 0.0;
        // elements i, i + stride, ... as one thread's ascending f64 sum; four per
        // pass with every load issued before any store (the fused ADAM's f64
        // chains then overlap)
        const size_t stride = (size_t)MZ_L2_BLOCKS * blockDim.x;
        for (size_t i = (size_t)blk * blockDim.x + tid; i < cnt; i += 4 * stride) {
            float x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = i + u * stride < cnt ? flat[off + i + u * stride] : 0.0f;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * stride < cnt) s += (double)x[u] * (double)x[u];
            if (ad.on) {                        // = mz_adam_kernel with G = 2θ, gscale 1
                adam_update4(ad, flat, off + i, stride, cnt - i, x);
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (i + u * stride < cnt) G[off + i + u * stride] = x[u] * 2.0f;
            }
        }
        red_v[tid] = s;
        __syncthreads();
        for (int o = blockDim.x / 2; o > 0; o >>= 1) {
            if (tid < o) red_v[tid] += red_v[tid + o];
            __syncthreads();
        }
        if (tid == 0) part[net * MZ_L2_BLOCKS + blk] = red_v[0];
    }
    // the last block out folds
    __syncthreads();
    if (tid == 0) {
        __threadfence();
        last = atomicAdd(counter, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    double sv = 0.0, sg = 0.0, sc = 0.0;
    // per sample j (thread j mod blockDim): its K+1 steps in ascending k.  The
    // terms of blockDim samples at a time are first staged in LDS by all
    // threads (one load each, all in flight), so no thread walks a chain of
    // dependent global loads
    __shared__ float fv[MZ_THREADS * MZ_FOLD_K1], fc[MZ_THREADS * MZ_FOLD_K1];
    const int K1 = K + 1;
    for (int j0 = 0; j0 < B; j0 += blockDim.x) {
        const int nj = B - j0 < (int)blockDim.x ? B - j0 : (int)blockDim.x;
        const bool staged = K1 <= MZ_FOLD_K1;
        if (staged) {
            for (int e = tid; e < nj * K1; e += blockDim.x) {
                fv[e] = __hip_atomic_load(vsq + (size_t)j0 * K1 + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                fc[e] = __hip_atomic_load(cet + (size_t)j0 * K1 + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
        }
        if (tid < nj) {
            const int j = j0 + tid;
            float s = 0.0f, c = 0.0f;
            for (int k = 0; k < K1; ++k) {
                const float vk = staged ? fv[tid * K1 + k]
                                        : __hip_atomic_load(vsq + (size_t)j * K1 + k, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
                const float ck = staged ? fc[tid * K1 + k]
                                        : __hip_atomic_load(cet + (size_t)j * K1 + k, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
                s = s + vk;
                c = c + (-ck);
            }
            const float w = wts ? wts[j] : 1.0f;   // PER importance weights (Learning.jl:271-285)
            sv += (double)((s / gscale[j]) * w);
            sc += (double)c;                    // Σ_k ce_k
            sg += (double)w / (double)gscale[j];   // Σ_j w_j/g_j
        }
        if (staged) __syncthreads();
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
        *counter = 0u;
    }
    if (tid < 192) {                            // wave w folds net w's partials: fixed pairs, then a fixed tree
        const int net = tid >> 6, j = tid & 63;
        double s = 0.0;
        for (int b = j; b < MZ_L2_BLOCKS; b += 64)
            s += __hip_atomic_load(part + net * MZ_L2_BLOCKS + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        if (j == 0) out[3 + net] = (float)s;
    }
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

// ADAM over all parameters (adam_update): grad = G[i] * gscale (gscale =
// 1/world after an all-reduce sum; exact for power-of-two world sizes).
extern "C" __global__ void mz_adam_kernel(float* P, float* M, float* V, const float* G, float gscale,
                                          size_t n, double bp1, double bp2, double eta, float* Wp, float* Bp,
                                          const int* inv_tile, float* smw, float* smb, const int* inv_small) {
    const LgAdam ad{1, M, V, bp1, bp2, eta, Wp, Bp, inv_tile, smw, smb, inv_small};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        adam_update(ad, P, i, G[i] * gscale);
}

// Rebuild the MFMA weight image from the Flux-order flat parameters:
// packed[i] = src[i] >= 0 ? flat[src[i]] : 0.
extern "C" __global__ void mz_repack_kernel(const float* flat, const int* src, float* packed, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int s = src[i];
        packed[i] = s >= 0 ? flat[s] : 0.0f;
    }
}
