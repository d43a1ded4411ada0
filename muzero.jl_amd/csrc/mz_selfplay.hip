// mz_selfplay.hip — device self-play loop body and device replay shard
// (SURVEY §8f-1, §8f-2).  One move of G lockstep games (play_game's loop body,
// SelfPlay.jl:343-380) is: mz_sp_prepare (observation append, stacked
// observations, legal mask, to_play) -> the batched search -> mz_sp_commit
// (env step, history append, finish test) -> mz_sp_order (ring slots of the
// finished games in slot order, replay counters) -> mz_sp_store (finished
// game -> replay ring, slot reset).  Nothing crosses PCIe.  mz_rp_sample is
// get_batch + make_target on the ring, writing an mz_batch in HBM.
//
// Env rules: TicTacToe exactly as games/tictactoe/game.jl with quirk Q14 (the
// win test looks at the plane of the player TO MOVE; reward ±1 by the mover's
// id), Connect4 as games/connect4.py, the synthetic Atari-like env of
// configs[4] as games/atari_synth.py (Philox-keyed frames, one frame per move
// in the records, a four-frame stack as the observation).  Host mirrors:
// muzero.jl_amd/games/{tictactoe,connect4,atari_synth}.py, selfplay.py,
// replay_buffer.py.
#include "mz_internal.h"
#include "mz_selfplay_params.h"
#include "mz_replay_device.h"

// ------------------------------------------------------------------- envs
__constant__ int8_t c_ttt_lines[8][3] = {{0, 3, 6}, {1, 4, 7}, {2, 5, 8}, {0, 1, 2},
                                          {3, 4, 5}, {6, 7, 8}, {0, 4, 8}, {6, 4, 2}};

// TicTacToe (game.jl:102-115, Q14): a line on the plane of player p
__device__ __forceinline__ bool ttt_line(const uint8_t* b, int p) {
    const uint8_t* pl = b + 9 * (p - 1);
    bool any = false;
#pragma unroll
    for (int l = 0; l < 8; ++l) any |= pl[c_ttt_lines[l][0]] && pl[c_ttt_lines[l][1]] && pl[c_ttt_lines[l][2]];
    return any;
}

__device__ __forceinline__ bool c4_wins(const uint8_t* stones, int w, int h, int W, int H) {
    const int dw[4] = {1, 0, 1, 1}, dh[4] = {0, 1, 1, -1};
    for (int d = 0; d < 4; ++d) {
        int n = 1;
        for (int s = 1; s >= -1; s -= 2) {
            int ww = w + s * dw[d], hh = h + s * dh[d];
            while (ww >= 0 && ww < W && hh >= 0 && hh < H && stones[ww + W * hh]) {
                ++n;
                ww += s * dw[d];
                hh += s * dh[d];
            }
        }
        if (n >= 4) return true;
    }
    return false;
}

// ---- synthetic Atari-like env (games/atari_synth.py): the frame of key
// `key` (osz = 84·84 bytes = 441 Philox blocks of 16 bytes), written by the
// 64 lanes of one wave
__device__ void atari_frame(const SpParams& S, int g, uint32_t key, int lane) {
    uint4* f = reinterpret_cast<uint4*>(S.board + (size_t)g * S.osz);
    for (int j = lane; j < (S.osz >> 4); j += 64) {
        const mz_u32x4 r = mz_philox((uint32_t)j, key, 0u, MZ_RNG_FRAME, (uint32_t)S.seed, (uint32_t)(S.seed >> 32));
        f[j] = make_uint4(r.v[0], r.v[1], r.v[2], r.v[3]);
    }
}
// reset: key = u32(seed, ENV, global game id = game_offset + slot, step, ~0)
__device__ void atari_reset(const SpParams& S, int g, uint32_t step, int lane) {
    const uint32_t key = mz_rng_u32(S.seed, MZ_RNG_ENV, S.game_offset + (uint32_t)g, step, 0xFFFFFFFFu);
    atari_frame(S, g, key, lane);
    if (lane == 0) { S.ekey[g] = key; S.player[g] = 1; S.over[g] = 0; }
}

// legal actions (1..A) as a bit mask
__device__ uint32_t env_legal(const SpParams& S, int g) {
    const uint8_t* b = S.board + (size_t)g * S.osz;
    uint32_t m = 0;
    if (S.env == MZ_ENV_ATARI) return S.A >= 32 ? 0xFFFFFFFFu : (1u << S.A) - 1u;
    if (S.env == MZ_ENV_TICTACTOE) {                    // game.jl:37-43
        if (ttt_line(b, S.player[g])) return 0;
        for (int c = 0; c < 9; ++c) m |= (uint32_t)b[18 + c] << c;
    } else {
        if (S.over[g]) return 0;
        const int cells = S.W * S.H;
        for (int h = 0; h < S.H; ++h) m |= (uint32_t)b[2 * cells + (S.W - 1) + S.W * h] << h;
    }
    return m;
}

// env(action) (game.jl:45-52) + is_terminated / reward (:85-100): returns the
// reward recorded for the mover, sets *done
__device__ float env_step(const SpParams& S, int g, int a, bool* done) {
    uint8_t* b = S.board + (size_t)g * S.osz;
    const int p = S.player[g];
    if (S.env == MZ_ENV_TICTACTOE) {
        const int c = a - 1;
        b[18 + c] = 0;
        b[9 * (p - 1) + c] = 1;
        const int np = p % 2 + 1;
        S.player[g] = np;
        const bool win = ttt_line(b, np);
        bool full = true;
        for (int k = 0; k < 9; ++k) full &= b[18 + k] == 0;
        *done = full || win;
        return (*done && win) ? (p == 1 ? 1.0f : -1.0f) : 0.0f;
    }
    const int W = S.W, cells = S.W * S.H, h = a - 1;
    int w = 0;
    while (w < W && !b[2 * cells + w + W * h]) ++w;
    const int cell = w + W * h;
    b[2 * cells + cell] = 0;
    b[(p - 1) * cells + cell] = 1;
    const bool win = c4_wins(b + (p - 1) * cells, w, h, W, S.H);
    bool full = true;
    for (int k = 0; k < cells; ++k) full &= b[2 * cells + k] == 0;
    *done = win || full;
    S.over[g] = *done;
    S.player[g] = 3 - p;
    return win ? 1.0f : 0.0f;
}

// Winner of a finished game from its last move (0 = draw / unfinished).
// TicTacToe (Q14): the win test after a move looks at the plane of the player
// now to move, so a nonzero reward means THAT player (3 - mover) holds a line;
// Connect4: a nonzero reward is the mover's own four in a row.
__device__ __forceinline__ int game_winner(const SpParams& S, float last_reward, int last_mover) {
    if (last_reward == 0.0f) return 0;
    return S.env == MZ_ENV_TICTACTOE ? 3 - last_mover : last_mover;
}

__device__ void env_reset(const SpParams& S, int g, int lane) {
    if (S.env == MZ_ENV_ATARI) { atari_reset(S, g, S.step, lane); return; }
    uint8_t* b = S.board + (size_t)g * S.osz;
    const int cells = S.osz / 3;
    for (int k = lane; k < S.osz; k += 64) b[k] = k >= 2 * cells;
    if (lane == 0) { S.player[g] = 1; S.over[g] = 0; }
}

// ------------------------------------------------------------ self-play move
// one wave per game slot
extern "C" __global__ __launch_bounds__(256) void mz_sp_prepare(SpParams S) {
    const int g = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (g >= S.G) return;
    const int t = S.hist.len[g];                                   // moves so far
    uint8_t* ho = S.hist.obs + ((size_t)g * S.T + t) * S.osz;     // observation_history append (:352)
    const uint8_t* b = S.board + (size_t)g * S.osz;
    for (int k = lane; k < S.osz; k += 64) ho[k] = b[k];
    if (S.frames)                                                  // the env's frame stack (same lanes wrote ho)
        frame_stack_obs(S.obs + (size_t)g * S.F, S.hist.obs + (size_t)g * S.T * S.osz, t + 1, S.osz, S.frames, lane);
    else
        stacked_obs(S.obs + (size_t)g * S.F, b, S.hist.obs + (size_t)g * S.T * S.osz, S.hist.act + (size_t)g * S.T,
                    t + 1, S.osz, S.P, S.stacked, lane);            // :355
    if (lane == 0) {
        const uint32_t m = env_legal(S, g);
        for (int a = 0; a < S.A; ++a) S.legal[(size_t)g * S.A + a] = (m >> a) & 1u;
        S.tp[g] = S.player[g];                                     // :351
        float tg = S.temperature;
        if (S.tgame) {                                             // one temperature per game (:396-407)
            if (t == 0) S.tgame[g] = S.temperature;
            tg = S.tgame[g];
        }
        if (S.temp_g)                                              // :344-346
            S.temp_g[g] = S.temp_threshold >= 0 && t >= S.temp_threshold ? 0.0f : tg;
    }
}

extern "C" __global__ __launch_bounds__(256) void mz_sp_commit(SpParams S) {
    const int g = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (g >= S.G) return;
    const int t = S.hist.len[g];
    const size_t r = (size_t)g * S.T + t;
    for (int a = lane; a < S.A; a += 64) S.hist.cv[r * S.A + a] = S.cv[(size_t)g * S.A + a];   // :375-379
    if (S.env == MZ_ENV_ATARI) {                                   // every lane steps the env (the frame is wave work)
        const int a = S.act[g];
        const uint32_t key = S.ekey[g];
        const mz_u32x4 v = mz_philox(0u, key, (uint32_t)a, MZ_RNG_ENV, (uint32_t)S.seed, (uint32_t)(S.seed >> 32));
        atari_frame(S, g, v.v[2], lane);
        if (lane == 0) {
            S.ekey[g] = v.v[2];
            S.hist.act[r] = a;
            S.hist.rew[r] = (int)mz_rng_below(v.v[0], (uint32_t)S.A) == a - 1 ? 1.0f : 0.0f;
            S.hist.tp[r] = S.player[g];
            S.hist.rv[r] = S.rv[g];
            S.hist.len[g] = t + 1;
            S.done[g] = (v.v[1] & 127u) == 0 || t + 1 > S.max_moves;
        }
        return;
    }
    if (lane == 0) {
        int a = S.act[g];
        const int mover = S.player[g];
        if (S.eval && S.opponent == MZ_OPP_RANDOM && mover != S.muzero_player) {   // :319-321
            uint32_t legal = 0;
            for (int b = 0; b < S.A; ++b) legal |= (uint32_t)(S.legal[(size_t)g * S.A + b] != 0) << b;
            const int n = __builtin_popcount(legal);
            if (n > 0) {
                const uint32_t r = mz_rng_u32(S.seed, MZ_RNG_OPPONENT, S.game_offset + (uint32_t)g, S.step, 0);
                uint32_t m = legal;
                for (int k = (int)mz_rng_below(r, (uint32_t)n); k > 0; --k) m &= m - 1;
                a = __builtin_ctz(m) + 1;
            }
        }
        bool done = false;
        const float rew = env_step(S, g, a, &done);                // :366-368
        S.hist.act[r] = a;
        S.hist.rew[r] = rew;
        S.hist.tp[r] = mover;
        S.hist.rv[r] = S.rv[g];
        S.hist.len[g] = t + 1;
        S.done[g] = done || t + 1 > S.max_moves;                  // :343 (> max_moves)
    }
}

// initial games of the synthetic Atari-like env (mz_selfplay_init's slots, at
// the first mz_selfplay_move: S.game_offset is that move's), one wave per slot
extern "C" __global__ __launch_bounds__(256) void mz_sp_reset(SpParams S) {
    const int g = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (g < S.G) atari_reset(S, g, S.reset_step, lane);
}

// Ring slots of this move's finished games in slot order (the host driver
// saves them in ascending slot order) and the replay counters (save_game,
// ReplayBuffer.jl:133-161).  One workgroup.
extern "C" __global__ __launch_bounds__(1024) void mz_sp_order(SpParams S) {
    __shared__ int cnt[1024];
    __shared__ long long red[3][1024];
    const int tid = threadIdx.x, per = (S.G + 1023) / 1024;
    const int g0 = tid * per, g1 = min(S.G, g0 + per);
    int n = 0;
    for (int g = g0; g < g1; ++g) n += S.done[g] != 0;
    cnt[tid] = n;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {                           // inclusive scan
        const int v = tid >= o ? cnt[tid - o] : 0;
        __syncthreads();
        cnt[tid] += v;
        __syncthreads();
    }
    if (S.eval) {                                                   // tally; nothing is saved
        long long t[4] = {0, 0, 0, 0};
        for (int g = g0; g < g1; ++g) {
            S.ring_pos[g] = -1;
            if (!S.done[g]) continue;
            const size_t last = (size_t)g * S.T + S.hist.len[g] - 1;
            const int w = game_winner(S, S.hist.rew[last], S.hist.tp[last]);
            t[0] += 1;
            t[w == 0 ? 3 : w == S.muzero_player ? 1 : 2] += 1;
        }
        for (int k = 0; k < 4; ++k)                                 // integer sums: any order is exact
            if (t[k]) atomicAdd(reinterpret_cast<unsigned long long*>(S.eval_counts + k), (unsigned long long)t[k]);
        return;
    }
    const long long played = S.counters[0];
    long long rank = cnt[tid] - n, steps = 0, evicted = 0;
    for (int g = g0; g < g1; ++g) {
        if (!S.done[g]) { S.ring_pos[g] = -1; continue; }
        const long long num = played + rank + 1;                   // game number (1-based)
        const int slot = (int)((num - 1) % S.cap);
        const int len = S.hist.len[g];
        if (num > S.cap) evicted += S.ring.len[slot];              // the game it replaces
        S.ring_pos[g] = slot;
        steps += len;
        ++rank;
    }
    red[0][tid] = n; red[1][tid] = steps; red[2][tid] = evicted;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if (tid < o)
            for (int k = 0; k < 3; ++k) red[k][tid] += red[k][tid + o];
        __syncthreads();
    }
    if (tid == 0) {
        S.counters[0] = played + red[0][0];
        S.counters[1] += red[1][0];
        S.counters[2] += red[1][0] - red[2][0];
    }
}

// finished game -> its ring slot; the slot starts a new game (one workgroup per slot)
extern "C" __global__ __launch_bounds__(256) void mz_sp_store(SpParams S) {
    const int g = blockIdx.x;
    if (!S.done[g]) return;
    const int slot = S.ring_pos[g], len = S.hist.len[g], tid = threadIdx.x;
    const size_t src = (size_t)g * S.T, dst = (size_t)(slot < 0 ? 0 : slot) * S.T;
    if (slot < 0) {                                // evaluation: the slot just restarts
        __syncthreads();
        if (tid == 0) { S.hist.len[g] = 0; S.done[g] = 0; }
        if (tid < 64) env_reset(S, g, tid);
        return;
    }
    for (int k = tid; k < len * S.osz; k += blockDim.x) S.ring.obs[dst * S.osz + k] = S.hist.obs[src * S.osz + k];
    for (int k = tid; k < len * S.A; k += blockDim.x) S.ring.cv[dst * S.A + k] = S.hist.cv[src * S.A + k];
    for (int k = tid; k < len; k += blockDim.x) {
        S.ring.act[dst + k] = S.hist.act[src + k];
        S.ring.rew[dst + k] = S.hist.rew[src + k];
        S.ring.tp[dst + k] = S.hist.tp[src + k];
        S.ring.rv[dst + k] = S.hist.rv[src + k];
    }
    __syncthreads();                               // every thread has read len and done
    if (S.per) {                                   // save_game's initial priorities (:136-143)
        SpHist ring = S.ring;
        per_init_slot(ring, slot, len, S.T, S.td, S.disc_pow, S.per_alpha, tid, blockDim.x);
        __syncthreads();
        if (tid == 0) per_game_max(ring, slot, len, S.T);
    }
    if (tid == 0) { S.ring.len[slot] = len; S.hist.len[g] = 0; S.done[g] = 0; }
    if (tid < 64) env_reset(S, g, tid);
}

// ------------------------------------------------------------------- PER
// initial priorities of one ring slot written by mz_replay_save_game
extern "C" __global__ void mz_rp_per_init(SpHist ring, int slot, int len, int Tmax, int td, const float* disc_pow,
                                          int alpha) {
    per_init_slot(ring, slot, len, Tmax, td, disc_pow, alpha, threadIdx.x, blockDim.x);
    __syncthreads();
    if (threadIdx.x == 0) per_game_max(ring, slot, len, Tmax);
}

// sample_n_games' game probabilities (:91-99): the held games oldest first
// (the Dict's game-number order), p_i = gprio_i / S with S the ascending f32
// sum, cum_i the ascending f32 running sum of p; total_samples = Σ len.  One
// lane: the f32 sums are sequential by definition.
extern "C" __global__ void mz_rp_per_prep(SpHist ring, const long long* counters, int cap, float* cum, float* prob,
                                          long long* total) {
    if (threadIdx.x != 0) return;
    const long long played = counters[0];
    const int n = (int)(played < cap ? played : cap);
    const long long oldest = played - n + 1;
    float S = 0.0f;
    long long tot = 0;
    for (int i = 0; i < n; ++i) {
        const int slot = (int)((oldest + i - 1) % cap);
        S = S + ring.gprio[slot];
        tot += ring.len[slot];
    }
    float c = 0.0f;
    for (int i = 0; i < n; ++i) {
        const float p = ring.gprio[(int)((oldest + i - 1) % cap)] / S;
        c = c + p;
        prob[i] = p;
        cum[i] = c;
    }
    *total = tot;
}

// weight_batch ./= maximum(weight_batch) (:215)
extern "C" __global__ void mz_rp_per_norm(float* w, int B) {
    __shared__ float red[256];
    const int tid = threadIdx.x;
    float m = -INFINITY;
    for (int i = tid; i < B; i += blockDim.x) m = w[i] > m ? w[i] : m;
    red[tid] = m;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (tid < o) red[tid] = red[tid + o] > red[tid] ? red[tid + o] : red[tid];
        __syncthreads();
    }
    const float mx = red[0];
    for (int i = tid; i < B; i += blockDim.x) w[i] = w[i] / mx;
}

// update_priorities! (ReplayBuffer.jl:168-183, Learning.jl:400-404) in its
// intended reading (the reference's `minimum(a, b)` and its K+2-element slice
// cannot run): for sample i in batch order, if game index[i] is still held,
// positions pos..min(pos+K, len) get |pv − tv|^alpha of steps 0.., then the
// game priority is their max.  Samples run in order (later ones overwrite),
// lanes over the steps of one sample.
extern "C" __global__ void mz_rp_per_update(SpHist ring, const long long* counters, int cap, int Tmax, int B, int K,
                                            int alpha, const int32_t* index, const float* pv, const float* tv) {
    const int lane = threadIdx.x;
    const long long played = counters[0];
    const long long held_from = played - (played < cap ? played : cap) + 1;
    for (int i = 0; i < B; ++i) {
        const long long num = index[2 * i];
        const int pos = index[2 * i + 1];
        if (num < held_from) continue;                     // evicted since it was sampled
        const int slot = (int)((num - 1) % cap), len = ring.len[slot];
        const int end = pos + K < len ? pos + K : len;     // 1-based, inclusive
        float* pr = ring.prio + (size_t)slot * Tmax;
        for (int k = pos + lane; k <= end; k += blockDim.x)
            pr[k - 1] = per_priority(pv[(size_t)i * (K + 1) + (k - pos)] - tv[(size_t)i * (K + 1) + (k - pos)], alpha);
        __syncthreads();
        if (lane == 0) per_game_max(ring, slot, len, Tmax);
        __syncthreads();
    }
}

// ------------------------------------------------------------- replay sample
// one wave per sample (get_batch, :188-217); the body is shared with the
// fused sample + unroll kernel (mz_replay_device.h)
extern "C" __global__ __launch_bounds__(256) void mz_rp_sample(RpSampleParams Q) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (b < Q.B) rp_sample_one(Q, b, lane);
}
