// mz_learner_device.h — the learner's loss / Σθ² / ADAM pieces, shared by
// mz_learner_grad_kernel* (mz_nets.hip, after an unroll launch) and the
// one-launch learner step mz_learn_small* (mz_small.hip, unroll + losses +
// ADAM in one grid).  Every piece runs on a 256-thread group (MZ_THREADS) so
// both kernels produce the same partial sums, bit for bit.
#pragma once
#include "mz_internal.h"
#include "mz_mlp_device.h"
#include "mz_tree_device.h"

// One launch after the unroll (Learning.jl:261-288, 380-393 in ref_semantics):
//  * blocks [0, nlb): one 16-lane group per (sample, step) t, lane a = action
//    a: read-outs on the raw unroll outputs — policy = softmax of the logits
//    (max, det_expf, ascending sum, divide), value / reward = their
//    activations — then the step's terms: squared value error and the
//    logitcrossentropy of the probabilities (Q11's double softmax), every
//    sum in ascending action order (g16_seqsum);
//  * blocks [nlb, nlb + 3·MZ_L2_BLOCKS): θ² of a fixed slice summed in f64,
//    and the data term of ∇ written for it: zero (Q11: only sum(sqnorm,
//    params) depends on θ; mz_adam_kernel adds the rank-invariant 2θ after a
//    data-parallel exchange, so the update is exact at every world size);
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
// One ADAM step of one parameter with ∇ = 2x (Q11): lg_adam_store's arithmetic
// in the same order (the multi-step chain, mz_learn_chain)
__device__ __forceinline__ float adam_2theta(float x, float& m, float& v, double bp1, double bp2, double eta) {
    const double b1 = 0.9, b2 = 0.999, eps = 1e-8;
    const float g = x * 2.0f;
    m = (float)(b1 * (double)m + (1.0 - b1) * (double)g);
    const float g2 = g * g;
    v = (float)(b2 * (double)v + (1.0 - b2) * (double)g2);
    const float d = (float)((double)m / (1.0 - bp1) / (sqrt((double)v / (1.0 - bp2)) + eps) * eta);
    return x - d;
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

// The terms of (sample, step) t for its GW-lane group (lane a = action a):
// read-outs on the raw unroll outputs — policy = softmax of the logits (max,
// det_expf, ascending sum, divide), value / reward = their activations — then
// the squared value error and the logitcrossentropy of the probabilities
// (Q11's double softmax), every sum in ascending action order.  st: this
// group's GW-float LDS staging slot.
template <int GW>
__device__ __forceinline__ void lg_step_terms(int t, int a, int A, int v_act, int r_act, float* pv, float* pp,
                                              float* pr, const float* tv, const float* tp, float* vsq, float* cet,
                                              float* st) {
    const bool in = a < A;
    float* yh = pp + (size_t)t * A;
    // every input loaded up front, in one round trip (the stores below could
    // alias them, so the compiler would otherwise issue each load after them)
    const float x = in ? yh[a] : -INFINITY;
    const float tpa = in ? tp[(size_t)t * A + a] : 0.0f;
    const float raw = a == 0 ? pv[t] : a == 1 ? pr[t] : 0.0f;
    const float tvt = a == 0 ? tv[t] : 0.0f;
    const float m = gmax<GW>(x);
    const float e = in ? det_expf(x - m) : 0.0f;
    const float s = gseqsum<GW>(e, A, st, a);
    const float p = in ? e / s : -INFINITY;
    if (in) yh[a] = p;
    const float m2 = gmax<GW>(p);
    const float e2 = in ? det_expf(p - m2) : 0.0f;
    const float se = gseqsum<GW>(e2, A, st, a);
    const float ls = det_logf(se);
    const float term = in ? tpa * ((p - m2) - ls) : 0.0f;
    const float ce = gseqsum<GW>(term, A, st, a);
    if (a < 2) {                                // lane 0 the value, lane 1 the reward read-out, at once
        const float y = mz_post_act(a == 0 ? v_act : r_act, raw);
        if (a == 0) {
            pv[t] = y;
            const float d = y - tvt;
            // read by the last block's fold: agent-scope stores (lg_fold)
            __hip_atomic_store(vsq + t, d * d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(cet + t, ce, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            pr[t] = y;
        }
    }
}

// Σθ² of slice blk of net (thread tid of 256): elements off + blk·256 + tid +
// j·(MZ_L2_BLOCKS·256) as one thread's ascending f64 sum; four per pass with
// every load issued before any store (the fused ADAM's f64 chains overlap).
// ad.on: ADAM with ∇ = 2θ in place (= mz_adam_kernel, gscale 1), else G = 0
// (the data term).
// ADAM operands of one 4-group (adam_update4's loads, issued ahead)
struct LgAdamOps { float x[4], mo[4], vo[4]; int it[4], is[4]; };
__device__ __forceinline__ void lg_adam_load(const LgAdam& ad, const float* P, size_t i0, size_t stride, size_t rem,
                                             bool on, LgAdamOps& o) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const size_t i = i0 + u * stride;
        const bool in = u * stride < rem;
        o.x[u] = in ? P[i] : 0.0f;
        o.mo[u] = in && on ? ad.M[i] : 0.0f; o.vo[u] = in && on ? ad.V[i] : 0.0f;
        o.it[u] = in && on ? ad.inv_tile[i] : -1; o.is[u] = in && on ? ad.inv_small[i] : -1;
    }
}
// adam_update4's arithmetic and stores on preloaded operands
__device__ __forceinline__ void lg_adam_store(const LgAdam& ad, float* P, size_t i0, size_t stride, size_t rem,
                                              const LgAdamOps& o) {
    const double b1 = 0.9, b2 = 0.999, eps = 1e-8;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        if (u * stride >= rem) continue;
        const size_t i = i0 + u * stride;
        const float g = o.x[u] * 2.0f;
        const float m = (float)(b1 * (double)o.mo[u] + (1.0 - b1) * (double)g);
        const float g2 = g * g;
        const float v = (float)(b2 * (double)o.vo[u] + (1.0 - b2) * (double)g2);
        ad.M[i] = m; ad.V[i] = v;
        const float d = (float)((double)m / (1.0 - ad.bp1) / (sqrt((double)v / (1.0 - ad.bp2)) + eps) * ad.eta);
        const float xn = o.x[u] - d;
        P[i] = xn;
        mz_scatter(xn, o.it[u], ad.Wp, ad.Bp);
        mz_scatter(xn, o.is[u], ad.smw, ad.smb);
    }
}

// Σθ² of slice blk of net (f64, this thread's elements in ascending order) and
// the ADAM step (∇ = 2θ) or the data term of ∇ (0) into G.  Software-pipelined: the next 4-group's
// loads are issued before this group's stores (the stores could alias them
// as far as the compiler knows, so a plain loop waits one memory latency per
// group).
__device__ __forceinline__ double lg_l2_slice(int net, int blk, int tid, const size_t* netoff, float* flat,
                                              float* G, const LgAdam& ad) {
    const size_t off = netoff[net], cnt = netoff[3 + net];
    double s = 0.0;
    const size_t stride = (size_t)MZ_L2_BLOCKS * MZ_THREADS;
    size_t i = (size_t)blk * MZ_THREADS + tid;
    if (i >= cnt) return s;
    LgAdam a = ad;                                  // the net's slice of the per-parameter arrays
    if (ad.on) { a.M += off; a.V += off; a.inv_tile += off; a.inv_small += off; }
    LgAdamOps cur;
    lg_adam_load(a, flat + off, i, stride, cnt - i, ad.on, cur);
    for (; i < cnt; i += 4 * stride) {
        LgAdamOps nxt;
        const size_t in = i + 4 * stride;
        if (in < cnt) lg_adam_load(a, flat + off, in, stride, cnt - in, ad.on, nxt);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * stride < cnt) s += (double)cur.x[u] * (double)cur.x[u];
        if (ad.on) {
            lg_adam_store(a, flat + off, i, stride, cnt - i, cur);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)          // the data term of ∇ (Q11: none); 2θ in mz_adam_kernel
                if (i + u * stride < cnt) G[off + i + u * stride] = 0.0f;
        }
        cur = nxt;
    }
    return s;
}

// Tree sum of red[0..255] (the 256 threads of one group; every thread of the
// block calls it: the barriers are block-wide) -> red[0].
__device__ __forceinline__ void lg_tree256(double* red, int tid) {
    __syncthreads();
    for (int o = MZ_THREADS / 2; o > 0; o >>= 1) {
        if (tid < o) red[tid] += red[tid + o];
        __syncthreads();
    }
}

// The last block out of the grid folds (all threads of the block call it;
// wave 0 does the losses, wave 1 the Σθ² partials): each sample's K+1 step
// terms in ascending k (lane j takes samples j, j+64, ... and issues all its
// loads first), the cross-sample sums in f64 (per lane ascending, then a
// fixed xor-shuffle tree; tolerance-checked against the oracle, not bitwise),
// the Σθ² partials in a fixed order (one 64-lane tree per net); resets the
// counter.  Returns without work in every other block.  out: [0] value, [1]
// reward (0, intermediate_rewards = false), [2] policy, [3..5] Σθ² of repr /
// pred / dyn.
// nblk: the blocks that count on `counter` (0: the whole grid).
__device__ __forceinline__ void lg_fold(int B, int K, const float* vsq, const float* cet, const float* gscale,
                                        const float* wts, const double* part, unsigned* counter, float* out,
                                        unsigned nblk = 0) {
    __shared__ bool last;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // the block's fold inputs (loss terms, Σθ² partial) are agent-scope stores,
    // complete once every wave has drained its stores; no per-block L2
    // write-back / invalidate (a __threadfence in each of the 3·MZ_L2_BLOCKS +
    // loss blocks cost 4 µs at 128 slices and 40 µs at 512)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
        last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (nblk ? nblk : gridDim.x) - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();
    const int K1 = K + 1;
    if (wave == 0) {
        double sv = 0.0, sg = 0.0, sc = 0.0;
        for (int j = lane; j < B; j += 64) {
            float vk[MZ_FOLD_K1], ck[MZ_FOLD_K1];
            const float gsj = gscale[j], w = wts ? wts[j] : 1.0f;   // issued with the terms below
            float s = 0.0f, c = 0.0f;
            for (int k0 = 0; k0 < K1; k0 += MZ_FOLD_K1) {
#pragma unroll
                for (int u = 0; u < MZ_FOLD_K1; ++u) {          // all loads of the chunk in flight
                    const bool in = k0 + u < K1;
                    const size_t e = (size_t)j * K1 + k0 + u;
                    vk[u] = in ? __hip_atomic_load(vsq + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
                    ck[u] = in ? __hip_atomic_load(cet + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
                }
#pragma unroll
                for (int u = 0; u < MZ_FOLD_K1; ++u)
                    if (k0 + u < K1) { s = s + vk[u]; c = c + (-ck[u]); }
            }
            // w: the PER importance weights (Learning.jl:271-285)
            sv += (double)((s / gsj) * w);
            sc += (double)c;                    // Σ_k ce_k
            sg += (double)w / (double)gsj;      // Σ_j w_j/g_j
        }
        for (int o = 32; o >= 1; o >>= 1) {
            sv += __shfl_xor(sv, o, 64); sg += __shfl_xor(sg, o, 64); sc += __shfl_xor(sc, o, 64);
        }
        if (lane == 0) {
            out[0] = (float)(sv / (double)B);
            out[1] = 0.0f;                      // intermediate_rewards = false (:276-280)
            out[2] = (float)(sc * sg / ((double)B * (double)B));  // mean over (1,B,B), Q11
        }
    } else if (wave == 1) {                     // Σθ² of the three nets: fixed pairs, then a fixed tree
        constexpr int NP = (MZ_L2_BLOCKS + 63) / 64;
        double pq[3][NP];                       // every partial loaded first: one round trip, not three
#pragma unroll
        for (int net = 0; net < 3; ++net)
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                const int b = lane + 64 * i;
                pq[net][i] = b < MZ_L2_BLOCKS ? __hip_atomic_load(part + net * MZ_L2_BLOCKS + b, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT) : 0.0;
            }
#pragma unroll
        for (int net = 0; net < 3; ++net) {
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < NP; ++i)
                if (lane + 64 * i < MZ_L2_BLOCKS) s += pq[net][i];
            for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
            if (lane == 0) out[3 + net] = (float)s;
        }
    }
    if (tid == 0) *counter = 0u;
}
