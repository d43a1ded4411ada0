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

// compute_target_value (ReplayBuffer.jl:5-20, Q9), f32, 1-based index
__device__ __forceinline__ float rp_target_value(const RpSampleParams& Q, const float* rv, const int32_t* tp, const float* rew, int T,
                                 int index) {
    const int bi = index + Q.td;
    if (bi >= T) return 0.0f;
    const float r0 = rv[bi - 1];
    const float last = tp[bi - 1] == tp[index - 1] ? r0 : -r0;
    float value = last * Q.disc_pow[Q.td];
    for (int i = 1; i <= Q.td + 1; ++i) {
        const float r = rew[index + i - 2];
        const float sr = tp[index - 1] == tp[index + i - 1] ? r : -r;
        value = value + sr * Q.disc_pow[i];
    }
    return value;
}

// get_batch's sample b (sample_n_games :102, sample_position :80,
// make_target :25-50, gradient_scale :212) on one wave (lane 0..63): writes
// row b of the batch arrays of Q.
__device__ __forceinline__ void rp_sample_one(const RpSampleParams& Q, int b, int lane) {
    const long long played = Q.counters[0];
    const int n = (int)(played < Q.cap ? played : Q.cap);
    const long long oldest = played - n + 1;                       // game number of ids[0]
    const uint32_t gi = mz_rng_below(mz_rng_u32(Q.seed, MZ_RNG_GAME, (uint32_t)b, Q.step, 0), (uint32_t)n);   // :102
    const long long num = oldest + gi;
    const int slot = (int)((num - 1) % Q.cap);
    const size_t base = (size_t)slot * Q.T;
    const int T = Q.ring.len[slot];
    const int pos = (int)mz_rng_below(mz_rng_u32(Q.seed, MZ_RNG_POS, (uint32_t)b, Q.step, 0), (uint32_t)T) + 1;  // :80
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
            v = rp_target_value(Q, rv, tp, rew, T, ci);
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
    stacked_obs(Q.obs + (size_t)b * Q.F, Q.ring.obs + (base + pos - 1) * Q.osz, Q.ring.obs + base * Q.osz, act, pos,
                Q.osz, Q.P, Q.stacked, lane);
    if (lane == 0) {
        const int gs = T + 1 - pos;                                // :212 min(K, len(action_history)+1-pos)
        Q.gscale[b] = (float)(Q.K < gs ? Q.K : gs);
        Q.index[2 * b] = (int)num;
        Q.index[2 * b + 1] = pos;
    }
}
