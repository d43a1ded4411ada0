"""PER host mirror (replay_buffer.py; ReplayBuffer.jl:73-107, 133-145, 168-183,
188-217): initial priorities, the Categorical restatement, importance weights
and update_priorities! in its intended reading.  CPU only; the device shard
is checked against this mirror in tests/test_selfplay_gpu.py."""
import dataclasses

import numpy as np

from muzero_jl_amd.replay_buffer import (ReplayBuffer, compute_target_value, per_categorical, per_priority,
                                         per_uniform)
from muzero_jl_amd.rng import rng_u32
from muzero_jl_amd.selfplay import GameHistory


def _game(rng, T, A=9):
    h = GameHistory()
    for t in range(T):
        h.observation_history.append(np.zeros(27, np.float32))
        h.action_history.append(int(rng.integers(1, A + 1)))
        h.reward_history.append(float(rng.choice([0.0, 0.0, 1.0, -1.0])))
        h.to_play_history.append(1 + t % 2)
        cv = rng.random(A).astype(np.float32)
        h.child_visits.append(cv / cv.sum())
        h.root_values.append(float(np.float32(rng.uniform(-1, 1))))
    return h


def _conf(ttt, **kw):
    return dataclasses.replace(ttt.conf, PER=True, PER_alpha=1, **kw)


def test_per_priority_is_integer_power():
    assert per_priority(np.float32(-0.75), 1) == np.float32(0.75)
    assert per_priority(np.float32(0.5), 2) == np.float32(0.25)
    assert per_priority(np.float32(3.0), 0) == np.float32(1.0)


def test_categorical_frequencies_follow_the_probabilities():
    w = np.array([1.0, 3.0, 0.0, 4.0], np.float32)
    counts = np.zeros(4)
    for i in range(20000):
        k, p = per_categorical(w, per_uniform(rng_u32(9, 4, i, 0, 0)))
        counts[k] += 1
        assert p == np.float32(w[k] / np.float32(8.0))
    np.testing.assert_allclose(counts / counts.sum(), w / w.sum(), atol=0.015)
    assert counts[2] == 0                                   # zero priority: never drawn


def test_save_game_sets_initial_priorities(ttt):
    rng = np.random.default_rng(0)
    conf = _conf(ttt)
    rb = ReplayBuffer(conf, seed=3)
    h = _game(rng, 9)
    rb.save_game(h)
    want = [abs(np.float32(h.root_values[i]) - compute_target_value(conf, h, i + 1)) for i in range(9)]
    assert np.array_equal(h.priorities, np.array(want, np.float32))
    assert h.game_priority == h.priorities.max()


def test_prioritized_batch_weights_and_update(ttt):
    rng = np.random.default_rng(1)
    conf = _conf(ttt, batch_size=64)
    rb = ReplayBuffer(conf, seed=3)
    for T in (3, 9, 5, 7, 2, 8):
        rb.save_game(_game(rng, T))
    idx, b = rb.get_batch(4)
    w = b["weights"]
    assert w.shape == (64,) and w.max() == np.float32(1.0) and (w > 0).all()
    # prioritized: the highest-priority game is drawn at least as often as under uniform sampling
    gp = {g: h.game_priority for g, h in rb.buffer.items()}
    top = max(gp, key=gp.get)
    assert sum(g == top for g, _ in idx) >= 64 / len(gp) * 0.8
    # update_priorities!: positions pos..min(pos+K, len) of each sampled game, batch order
    K = conf.num_unroll_steps
    pv = rng.uniform(-1, 1, (64, K + 1)).astype(np.float32)
    rb.update_priorities(idx, pv, b["target_values"])
    for i, (g, pos) in enumerate(idx):
        h = rb.buffer[g]
        last = max(j for j, (g2, p2) in enumerate(idx) if g2 == g and p2 <= pos <= p2 + K)
        g2, p2 = idx[last]
        assert h.priorities[pos - 1] == per_priority(pv[last][pos - p2] - b["target_values"][last][pos - p2], 1)
        assert h.game_priority == h.priorities.max()


def test_per_categorical_tie_rule():
    """Distributions 0.25 rand(::DiscreteNonParametric) advances while
    cp <= draw: an exact tie moves on, and a zero-probability entry is never
    drawn, even at draw 0."""
    w = np.array([0.0, 0.0, 2.0, 2.0], np.float32)
    assert per_categorical(w, 0.0) == (2, np.float32(0.5))          # leading zeros skipped at u = 0
    assert per_categorical(w, 0.5)[0] == 3                          # cp = 0.5 <= 0.5: the tie advances
    assert per_categorical(w, 0.49)[0] == 2
    assert per_categorical(np.array([1.0, 0.0], np.float32), 0.9999)[0] == 0


def test_oracle_per_categorical_matches_mirror():
    """The oracle's restatement of Categorical sampling (ora_per_categorical)
    and of the priority power agree with the host mirror on random weights,
    ties and zero entries."""
    import ctypes
    from oracle import lib
    L = lib()
    rng = np.random.default_rng(3)
    for n in (1, 2, 5, 17):
        for _ in range(50):
            w = rng.random(n).astype(np.float32) * (rng.random(n) < 0.8)
            if w.sum() == 0:
                w[0] = 1.0
            u = float(rng.integers(0, 1 << 24)) * 5.9604644775390625e-08
            pr = np.zeros(1, np.float32)
            k = L.ora_per_categorical(w.ctypes.data_as(ctypes.c_void_p), n, u, pr.ctypes.data_as(ctypes.c_void_p))
            assert (k, pr[0]) == per_categorical(w, u)
    for x in (-1.5, 0.0, 0.3, 7.25):
        for a in (1, 2, 3):
            assert np.float32(L.ora_per_priority(x, a)) == per_priority(np.float32(x), a)
