"""Replay buffer and targets — host mirror of src/ReplayBuffer.jl.

FIFO buffer of GameHistory keyed by game id (save_game, :133-161; the
RemoteBufferChannel Dict semantics, src/RemoteBufferChannel.jl), uniform
or prioritized (PER, :73-107, 133-145, 168-183) sampling with the engine's Philox streams instead of
Julia's global RNG (quirk Q6), n-step value targets with the reference's
exact indexing (quirk Q9), and batch assembly in the reference's column-major
tuple layout (get_batch, :188-217).  One buffer per GPU shard.
"""
import math
from collections import OrderedDict

import numpy as np

from .selfplay import GameHistory, frame_stack_obs, get_stacked_observations

MZ_RNG_GAME, MZ_RNG_POS, MZ_RNG_ABSORB = 4, 5, 6
from .rng import _M, _philox, rng_below, rng_u32  # noqa: F401  (re-exported)


def disc_pow(g, n):
    """discount^n as Julia's Float32^Int (llvm.pow.f32) ≈ f32(pow(f64))."""
    return np.float32(math.pow(float(np.float32(g)), float(n)))


def compute_target_value(conf, h, index):
    """ReplayBuffer.jl:5-20 (Q9); index is 1-based.  Float32 arithmetic."""
    f32 = np.float32
    T = len(h.root_values)
    bi = index + conf.td_steps
    if bi < T:
        rv = f32(h.root_values[bi - 1])
        last = rv if h.to_play_history[bi - 1] == h.to_play_history[index - 1] else -rv
        value = f32(last * disc_pow(conf.discount, conf.td_steps))
        for i in range(1, conf.td_steps + 2):
            r = f32(h.reward_history[index + i - 2])
            sr = r if h.to_play_history[index - 1] == h.to_play_history[index + i - 1] else -r
            value = f32(value + f32(sr * disc_pow(conf.discount, i)))
    else:
        value = f32(0.0)
    return value


def make_target(conf, h, state_index, seed=0, sample=0, step=0):
    """ReplayBuffer.jl:25-50 -> (values (K+1,), rewards (K+1,), policies (K+1, A), actions (K+1,))."""
    K, A = conf.num_unroll_steps, len(conf.action_space)
    T = len(h.root_values)
    tv = np.zeros(K + 1, np.float32)
    tr = np.zeros(K + 1, np.float32)
    tp = np.zeros((K + 1, A), np.float32)
    ta = np.zeros(K + 1, np.float32)
    uni = np.float32(1.0) / np.float32(A)
    for k in range(K + 1):
        ci = state_index + k
        if ci < T:
            tv[k] = compute_target_value(conf, h, ci)
            tr[k] = h.reward_history[ci - 1]
            tp[k] = h.child_visits[ci - 1]
            ta[k] = h.action_history[ci - 1]
        elif ci == T:
            tr[k] = h.reward_history[ci - 1]
            tp[k] = uni
            ta[k] = h.action_history[ci - 1]
        else:                                              # absorbing states
            tp[k] = uni
            ta[k] = rng_below(rng_u32(seed, MZ_RNG_ABSORB, sample, step, k), A) + 1
    return tv, tr, tp, ta


def per_priority(x, alpha):
    """|x|^PER_alpha as Julia's Float32^Int, restated as f64 repeated
    multiplication rounded once to f32 (the kernels' per_priority)."""
    ax = abs(float(np.float32(x)))
    r = 1.0
    for _ in range(alpha):
        r = r * ax
    return np.float32(r)


def per_uniform(r):
    """uniform in [0, 1) from a Philox draw (24 bits, exact)."""
    return (r >> 8) * 5.9604644775390625e-08


def per_categorical(w, u):
    """Categorical over p_i = w_i / S (S = ascending f32 sum): the first index
    whose ascending f32 running sum of p is > u (else the last; Distributions
    0.25 advances while cp <= draw, so zero-probability entries are never
    drawn); returns
    (index, p_index).  The restatement of rand(rng, Categorical(p)) used by
    sample_n_games / sample_position with PER (ReplayBuffer.jl:75-78, 96-103)."""
    f32 = np.float32
    S = f32(0.0)
    for x in w:
        S = f32(S + f32(x))
    i = 0
    p = f32(f32(w[0]) / S)
    c = p
    while float(c) <= u and i < len(w) - 1:
        i += 1
        p = f32(f32(w[i]) / S)
        c = f32(c + p)
    return i, p


class ReplayBuffer:
    """Per-GPU buffer: Dict{game_id => GameHistory} with FIFO eviction."""

    def __init__(self, conf, seed=0, frame_stack=0):
        """frame_stack: the env's own frame stacking (games/atari_synth.py,
        observation_history holds one frame per move), 0 for board games."""
        self.conf = conf
        self.seed = seed
        self.frame_stack = frame_stack
        self.buffer = OrderedDict()
        self.num_played_games = 0
        self.num_played_steps = 0
        self.total_samples = 0

    def __len__(self):
        return len(self.buffer)

    def save_game(self, history: GameHistory):                  # :133-161
        n = len(history.root_values)
        if self.conf.PER:                                       # initial priorities :136-143
            history.priorities = np.array([per_priority(np.float32(history.root_values[i]) -
                                                        compute_target_value(self.conf, history, i + 1),
                                                        self.conf.PER_alpha) for i in range(n)], np.float32)
            history.game_priority = np.float32(history.priorities.max())
        self.num_played_games += 1
        self.num_played_steps += n
        self.total_samples += n
        self.buffer[self.num_played_games] = history
        if self.conf.replay_buffer_size < self.num_played_games:
            del_id = self.num_played_games - self.conf.replay_buffer_size
            removed = self.buffer.pop(del_id)
            self.total_samples -= len(removed.root_values)

    def get_batch(self, step):
        """:188-217 with uniform sampling keyed by the learner step.
        Returns (index_batch, batch dict in the engine's layout)."""
        c = self.conf
        B, K, A = c.batch_size, c.num_unroll_steps, len(c.action_space)
        ids = list(self.buffer.keys())
        n = len(ids)
        if n == 0:
            raise ValueError("replay buffer is empty")
        plane = c.observation_shape[0] * c.observation_shape[1]
        feat = plane * (c.observation_shape[2] * (c.stacked_observations + 1) + c.stacked_observations)
        obs = np.zeros((B, feat), np.float32)
        acts = np.zeros((B, K + 1), np.float32)
        tv = np.zeros((B, K + 1), np.float32)
        tr = np.zeros((B, K + 1), np.float32)
        tp = np.zeros((B, K + 1, A), np.float32)
        gs = np.zeros(B, np.float32)
        index_batch = []
        per = bool(c.PER)
        if per:                                                 # :190, :91-99
            total = sum(len(h.root_values) for h in self.buffer.values())
            gprio = [self.buffer[i].game_priority for i in ids]
            wts = np.zeros(B, np.float32)
        for b in range(B):
            rg = rng_u32(self.seed, MZ_RNG_GAME, b, step, 0)
            rp = rng_u32(self.seed, MZ_RNG_POS, b, step, 0)
            if per:
                gi, gprob = per_categorical(gprio, per_uniform(rg))                # sample_n_games :96-103
            else:
                gi = rng_below(rg, n)                                              # sample_n_games :102
            h = self.buffer[ids[gi]]
            T = len(h.root_values)
            if per:                                                                # sample_position :75-78
                pi, pprob = per_categorical(h.priorities, per_uniform(rp))
                pos = pi + 1
                wts[b] = np.float32(1.0) / np.float32(np.float32(np.float32(total) * gprob) * pprob)   # :213
            else:
                pos = rng_below(rp, T) + 1                                         # sample_position :80
            tv[b], tr[b], tp[b], acts[b] = make_target(c, h, pos, self.seed, b, step)
            if self.frame_stack:
                obs[b] = frame_stack_obs(h.observation_history, pos, self.frame_stack)
            else:
                obs[b] = get_stacked_observations(h.observation_history, h.action_history, pos,
                                                  c.stacked_observations, plane)
            gs[b] = min(K, len(h.action_history) + 1 - pos)                        # :212
            index_batch.append((ids[gi], pos))
        out = dict(observation=obs, actions=acts, target_values=tv, target_rewards=tr,
                   target_policies=tp, gradient_scale=gs)
        if per:
            out["weights"] = (wts / wts.max()).astype(np.float32)                 # :215
        return index_batch, out

    def update_priorities(self, index_batch, predicted_values, target_values):
        """update_priorities! (ReplayBuffer.jl:168-183, Learning.jl:400-404) in its
        intended reading: sample i (batch order) sets positions pos..min(pos+K, len)
        of its game, if still held, to |v̂ − v|^alpha of steps 0.., then the game
        priority to their max.  predicted / target values: (B, K+1)."""
        K, alpha = self.conf.num_unroll_steps, self.conf.PER_alpha
        for i, (gid, pos) in enumerate(index_batch):
            if gid not in self.buffer:
                continue
            h = self.buffer[gid]
            end = min(pos + K, len(h.priorities))
            for k in range(pos, end + 1):
                h.priorities[k - 1] = per_priority(np.float32(predicted_values[i][k - pos]) -
                                                   np.float32(target_values[i][k - pos]), alpha)
            h.game_priority = np.float32(h.priorities.max())
