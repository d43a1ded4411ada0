"""Replay buffer and targets — host mirror of src/ReplayBuffer.jl.

FIFO buffer of GameHistory keyed by game id (save_game, :133-161; the
RemoteBufferChannel Dict semantics, src/RemoteBufferChannel.jl), uniform
sampling (PER=false, params.jl:11) with the engine's Philox streams instead of
Julia's global RNG (quirk Q6), n-step value targets with the reference's
exact indexing (quirk Q9), and batch assembly in the reference's column-major
tuple layout (get_batch, :188-217).  One buffer per GPU shard.
"""
import math
from collections import OrderedDict

import numpy as np

from .selfplay import GameHistory, get_stacked_observations

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


class ReplayBuffer:
    """Per-GPU buffer: Dict{game_id => GameHistory} with FIFO eviction."""

    def __init__(self, conf, seed=0):
        self.conf = conf
        self.seed = seed
        self.buffer = OrderedDict()
        self.num_played_games = 0
        self.num_played_steps = 0
        self.total_samples = 0

    def __len__(self):
        return len(self.buffer)

    def save_game(self, history: GameHistory):                  # :133-161 (PER=false)
        n = len(history.root_values)
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
        for b in range(B):
            gi = rng_below(rng_u32(self.seed, MZ_RNG_GAME, b, step, 0), n)       # sample_n_games :102
            h = self.buffer[ids[gi]]
            T = len(h.root_values)
            pos = rng_below(rng_u32(self.seed, MZ_RNG_POS, b, step, 0), T) + 1   # sample_position :80
            tv[b], tr[b], tp[b], acts[b] = make_target(c, h, pos, self.seed, b, step)
            obs[b] = get_stacked_observations(h.observation_history, h.action_history, pos,
                                              c.stacked_observations, plane)
            gs[b] = min(K, len(h.action_history) + 1 - pos)                        # :212
            index_batch.append((ids[gi], pos))
        return index_batch, dict(observation=obs, actions=acts, target_values=tv, target_rewards=tr,
                                 target_policies=tp, gradient_scale=gs)
