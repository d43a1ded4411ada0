// mz_replay_device.h — device replay-shard helpers shared by mz_rp_sample
// (mz_selfplay.hip) and the fused sample + unroll learner kernel
// (mz_small.hip): get_stacked_observations, compute_target_value and one
// sample of get_batch + make_target (ReplayBuffer.jl:5-50, 73-107, 188-217).
#pragma once
#include "mz_internal.h"
#include "mz_selfplay_params.h"

// get_stacked_observations (SelfPlay.jl:128-149, Q15) of record `obs`/`act`
// at 1-based index (cur = observation `index`): [obs_t, (action plane = raw
// id, obs_{t-1}) ...], zeros before the first move
__device__ __forceinline__ void stacked_obs(float* out, const uint8_t* cur, const uint8_t* obs, const int32_t* act,
                                            int index, int osz, int P, int stacked, int lane) {
    for (int k = lane; k < osz; k += 64) out[k] = (float)cur[k];
    int o = osz;
    for (int past = index - 1; past >= index - stacked; --past) {
        if (past >= 1) {
            const float av = (float)act[past - 1];
            for (int k = lane; k < P; k += 64) out[o + k] = av;
            const uint8_t* po = obs + (size_t)(past - 1) * osz;
            for (int k = lane; k < osz; k += 64) out[o + P + k] = (float)po[k];
        } else {
            for (int k = lane; k < P + osz; k += 64) out[o + k] = 0.0f;
        }
        o += P + osz;
    }
}

// The synthetic Atari-like env's observation at 1-based move `index`
// (games/atari_synth.py): channel c = frame index-n+1+c (newest last), zeros
// before move 1, byte x as f32(x) * f32(1/255).  frames = the record's
// per-move frames (osz bytes each, osz % 4 == 0, 4-byte aligned).
__device__ __forceinline__ void frame_stack_obs(float* out, const uint8_t* frames, int index, int osz, int n,
                                                int lane) {
    const float scale = 1.0f / 255.0f;
    const int nw = osz >> 2;
    for (int c = 0; c < n; ++c) {
        const int s = index - n + 1 + c;
        float4* o = reinterpret_cast<float4*>(out + (size_t)c * osz);
        if (s < 1) {
            for (int q = lane; q < nw; q += 64) o[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            continue;
        }
        const uint32_t* f = reinterpret_cast<const uint32_t*>(frames + (size_t)(s - 1) * osz);
        for (int q = lane; q < nw; q += 64) {
            const uint32_t w = f[q];
            o[q] = make_float4((float)(w & 255u) * scale, (float)((w >> 8) & 255u) * scale,
                               (float)((w >> 16) & 255u) * scale, (float)(w >> 24) * scale);
        }
    }
}

// compute_target_value (ReplayBuffer.jl:5-20, Q9), f32, 1-based index
__device__ __forceinline__ float rp_target_value(int td, const float* disc_pow, const float* rv, const int32_t* tp,
                                                 const float* rew, int T, int index) {
    const int bi = index + td;
    if (bi >= T) return 0.0f;
    const float r0 = rv[bi - 1];
    const float last = tp[bi - 1] == tp[index - 1] ? r0 : -r0;
    float value = last * disc_pow[td];
    for (int i = 1; i <= td + 1; ++i) {
        const float r = rew[index + i - 2];
        const float sr = tp[index - 1] == tp[index + i - 1] ? r : -r;
        value = value + sr * disc_pow[i];
    }
    return value;
}

// PER priority |x|^alpha (Julia Float32^Int): f64 repeated multiplication,
// rounded once to f32 (the host mirror's per_priority is the same loop)
__device__ __forceinline__ float per_priority(float x, int alpha) {
    const double ax = (double)fabsf(x);
    double r = 1.0;
    for (int i = 0; i < alpha; ++i) r = r * ax;
    return (float)r;
}

// uniform double in [0, 1) from a Philox draw: 24 bits, exact
__device__ __forceinline__ double per_uniform(uint32_t r) { return (double)(r >> 8) * 5.9604644775390625e-08; }

// Categorical(p) with f32 probabilities p[i] = w[i] / S (S = ascending f32
// sum of w): i = first index whose ascending f32 running sum is > u (the
// last index if none) — Distributions 0.25 rand(::DiscreteNonParametric)
// advances while cp <= draw, so a zero-probability entry is never drawn;
// *prob = p[i].  Sequential, one lane.
__device__ __forceinline__ int per_categorical(const float* w, int n, double u, float* prob) {
    float S = 0.0f;
    for (int i = 0; i < n; ++i) S = S + w[i];
    int i = 0;
    float p = w[0] / S, c = p;
    while ((double)c <= u && i < n - 1) {
        ++i;
        p = w[i] / S;
        c = c + p;
    }
    *prob = p;
    return i;
}

// save_game's initial priorities for ring slot `slot` of length len (PER,
// ReplayBuffer.jl:136-143): |root_value_i − target_value_i|^alpha, game
// priority = max.  Lanes over positions, lane 0 folds the max.
__device__ __forceinline__ void per_init_slot(SpHist& ring, int slot, int len, int Tmax, int td,
                                              const float* disc_pow, int alpha, int lane, int nlanes) {
    const size_t base = (size_t)slot * Tmax;
    for (int k = lane; k < len; k += nlanes)
        ring.prio[base + k] = per_priority(ring.rv[base + k] -
                                           rp_target_value(td, disc_pow, ring.rv + base, ring.tp + base,
                                                           ring.rew + base, len, k + 1), alpha);
}
__device__ __forceinline__ void per_game_max(SpHist& ring, int slot, int len, int Tmax) {
    const float* pr = ring.prio + (size_t)slot * Tmax;
    float m = pr[0];
    for (int k = 1; k < len; ++k) m = pr[k] > m ? pr[k] : m;
    ring.gprio[slot] = m;
}

// get_batch's sample b (sample_n_games :102, sample_position :80,
// make_target :25-50, gradient_scale :212) on one wave (lane 0..63): writes
// row b of the batch arrays of Q.
__device__ __forceinline__ void rp_sample_one(const RpSampleParams& Q, int b, int lane) {
    const long long played = Q.counters[0];
    const int n = (int)(played < Q.cap ? played : Q.cap);
    const long long oldest = played - n + 1;                       // game number of ids[0]
    const uint32_t rg = mz_rng_u32(Q.seed, MZ_RNG_GAME, (uint32_t)b, Q.step, 0);
    const uint32_t rp = mz_rng_u32(Q.seed, MZ_RNG_POS, (uint32_t)b, Q.step, 0);
    uint32_t gi;
    float gprob = 0.0f;
    if (Q.per) {                                                   // Categorical(game_probs), :96-103
        const double u = per_uniform(rg);
        int lo = 0, hi = n - 1;                                    // first i with cum[i] > u, else n-1
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((double)Q.per_cum[mid] > u) hi = mid; else lo = mid + 1;
        }
        gi = (uint32_t)lo;
        gprob = Q.per_p[lo];
    } else {
        gi = mz_rng_below(rg, (uint32_t)n);                        // :102
    }
    const long long num = oldest + gi;
    const int slot = (int)((num - 1) % Q.cap);
    const size_t base = (size_t)slot * Q.T;
    const int T = Q.ring.len[slot];
    int pos;
    if (Q.per) {                                                   // Categorical(position_probs), :75-78
        float pprob = 0.0f;
        pos = per_categorical(Q.ring.prio + base, T, per_uniform(rp), &pprob) + 1;
        if (lane == 0)                                             // :213
            Q.weights[b] = 1.0f / ((float)*Q.per_total * gprob * pprob);
    } else {
        pos = (int)mz_rng_below(rp, (uint32_t)T) + 1;              // :80
    }
    const int K1 = Q.K + 1, A = Q.A;
    const float* rv = Q.ring.rv + base;
    const int32_t* tp = Q.ring.tp + base;
    const float* rew = Q.ring.rew + base;
    const int32_t* act = Q.ring.act + base;
    const float* cv = Q.ring.cv + base * A;
    const float uni = 1.0f / (float)A;
    for (int k = lane; k < K1; k += 64) {                          // make_target (:25-50)
        const int ci = pos + k;
        float v = 0.0f, r = 0.0f, a;
        if (ci < T) {
            v = rp_target_value(Q.td, Q.disc_pow, rv, tp, rew, T, ci);
            r = rew[ci - 1];
            a = (float)act[ci - 1];
        } else if (ci == T) {
            r = rew[ci - 1];
            a = (float)act[ci - 1];
        } else {                                                   // absorbing states
            a = (float)(mz_rng_below(mz_rng_u32(Q.seed, MZ_RNG_ABSORB, (uint32_t)b, Q.step, (uint32_t)k), (uint32_t)A) + 1);
        }
        Q.tv[(size_t)b * K1 + k] = v;
        Q.tr[(size_t)b * K1 + k] = r;
        Q.actions[(size_t)b * K1 + k] = a;
    }
    for (int e = lane; e < K1 * A; e += 64) {
        const int k = e / A, a = e - k * A, ci = pos + k;
        Q.tpol[(size_t)b * K1 * A + e] = ci < T ? cv[(size_t)(ci - 1) * A + a] : uni;
    }
    if (Q.frames)
        frame_stack_obs(Q.obs + (size_t)b * Q.F, Q.ring.obs + base * Q.osz, pos, Q.osz, Q.frames, lane);
    else
        stacked_obs(Q.obs + (size_t)b * Q.F, Q.ring.obs + (base + pos - 1) * Q.osz, Q.ring.obs + base * Q.osz, act,
                    pos, Q.osz, Q.P, Q.stacked, lane);
    if (lane == 0) {
        const int gs = T + 1 - pos;                                // :212 min(K, len(action_history)+1-pos)
        // write-through (agent scope): the fold of a learner launch that draws its
        // batch in place reads every sample's gradient_scale from another workgroup
        __hip_atomic_store(Q.gscale + b, (float)(Q.K < gs ? Q.K : gs), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        Q.index[2 * b] = (int)num;
        Q.index[2 * b + 1] = pos;
    }
}
