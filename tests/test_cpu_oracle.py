"""CPU tests of the oracle (no GPU): numerics contract, the independent Python
mirror of the reference's search, TicTacToe rules (Q14), value targets (Q9),
the learner's ADAM/schedule, and the networks against torch fp32."""
import dataclasses
import math

import numpy as np
import pytest

from conftest import random_positions

f32 = np.float32


def _oracle(conf, hyper, nets, seed=5):
    from muzero_jl_amd.config import to_c_config, to_c_ffhp
    from oracle import Oracle
    o = Oracle(to_c_config(conf), to_c_ffhp(hyper), seed=seed)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
    return o


# ------------------------------------------------------------ numerics contract
def test_philox_known_answers():
    """Random123 Philox4x32-10 known-answer vectors."""
    import ctypes
    from oracle import lib
    L = lib()
    out = (ctypes.c_uint32 * 4)()
    kats = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
            ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
            ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
             (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, exp in kats:
        L.ora_philox(*ctr, *key, out)
        assert tuple(out) == exp


def test_python_philox_matches_oracle():
    from muzero_jl_amd.replay_buffer import rng_u32
    from oracle import lib
    L = lib()
    for args in [(0, 4, 3, 7, 1), (2 ** 40 + 5, 5, 123456, 99, 0), (7, 6, 1, 2, 3)]:
        assert rng_u32(*args) == L.ora_rng_u32(*args)


def _ulps(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


def test_det_elementary_functions_accuracy():
    from oracle import lib
    L = lib()
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(-30, 30, 4000), rng.uniform(-1, 1, 2000), [0.0, -0.0, 1e-30, 88.0, -87.0]])
    xs = xs.astype(np.float32)
    e = np.array([L.ora_det_expf(float(x)) for x in xs], np.float32)
    assert _ulps(e, np.exp(xs.astype(np.float64)).astype(np.float32)).max() <= 2
    t = np.array([L.ora_det_tanhf(float(x)) for x in xs], np.float32)
    assert _ulps(t, np.tanh(xs.astype(np.float64)).astype(np.float32)).max() <= 2
    pos = np.abs(xs) + np.float32(1e-3)
    lg = np.array([L.ora_det_logf(float(x)) for x in pos], np.float32)
    assert _ulps(lg, np.log(pos.astype(np.float64)).astype(np.float32)).max() <= 2
    d = rng.uniform(-700, 700, 2000)
    ed = np.array([L.ora_det_exp(x) for x in d])
    assert np.max(np.abs(ed / np.exp(d) - 1)) < 4e-16
    pd = rng.uniform(1e-300, 1e300, 2000)
    ld = np.array([L.ora_det_log(x) for x in pd])
    assert np.max(np.abs(ld - np.log(pd)) / np.maximum(1, np.abs(np.log(pd)))) < 4e-16


def test_dirichlet_statistics():
    """Dirichlet(α=0.25) noise: mean 1/n, marginal variance (1/n)(1-1/n)/(nα+1)."""
    import ctypes
    from oracle import lib
    L = lib()
    n, N = 6, 4000
    out = np.zeros(n, np.float32)
    xs = np.zeros((N, n))
    for i in range(N):
        L.ora_dirichlet(9, i, 3, n, 0.25, out.ctypes.data_as(ctypes.c_void_p))
        xs[i] = out
    assert np.allclose(xs.sum(1), 1.0, atol=1e-5)
    assert np.allclose(xs.mean(0), 1 / n, atol=0.02)
    var = (1 / n) * (1 - 1 / n) / (n * 0.25 + 1)
    assert np.allclose(xs.var(0), var, rtol=0.15)


def test_cos_schedule_matches_oracle():
    from muzero_jl_amd.config import cos_schedule
    from oracle import lib
    L = lib()
    for t in range(1, 30):
        assert cos_schedule(t) == L.ora_cos_schedule(1e-4, 1e-1, 10, t)
    assert abs(cos_schedule(1) - 0.1) < 1e-15 and abs(cos_schedule(6) - 1e-4) < 1e-12


# ------------------------------------------------------------------- networks
def test_oracle_nets_match_torch(ttt, nets):
    import torch
    from muzero_jl_amd.networks import unflatten
    o = _oracle(ttt.conf, ttt.hyper, nets)
    rng = np.random.default_rng(3)
    for net, feat in [(0, 63), (1, 27), (2, 36)]:
        x = rng.standard_normal((50, feat)).astype(np.float32)
        layers = unflatten(ttt.conf, ttt.hyper, net, nets[net])

        def chain(ch, v):
            for c, W, b, act in layers:
                if c == ch:
                    v = v @ torch.from_numpy(W.T.copy()) + torch.from_numpy(b.copy())
                    v = torch.relu(v) if act == 1 else torch.tanh(v) if act == 2 else v
            return v
        t = chain(0, torch.from_numpy(x))
        out = o.forward(net, x)
        if net == 0:
            np.testing.assert_allclose(out, t.numpy(), rtol=1e-5, atol=1e-5)
        else:
            o0, o1 = chain(1, t), chain(2, t)
            if net == 1:
                o1 = torch.softmax(o1, 1)
            np.testing.assert_allclose(out[0], o0.numpy(), rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(out[1], o1.numpy(), rtol=1e-5, atol=1e-5)


def test_param_counts(ttt):
    from muzero_jl_amd.networks import param_count
    assert [param_count(ttt.conf, ttt.hyper, n) for n in range(3)] == [18331, 23242, 33308]


# ----------------------------------------------------- search vs Python mirror
@pytest.mark.parametrize("S,players,explore", [(10, 2, True), (25, 2, True), (15, 1, True), (12, 2, False)])
def test_oracle_search_matches_independent_mirror(ttt, nets, S, players, explore):
    from mirror_ref import Mirror
    conf = dataclasses.replace(ttt.conf, num_iters=S, players=list(range(1, players + 1)))
    o = _oracle(conf, ttt.hyper, nets, seed=13)
    G = 6
    obs, legal, tp = random_positions(G, 31)
    if players == 1:
        tp[:] = 1
    cv, rv, act, tree, _ = o.mcts_search(obs, legal, tp, exploration=explore, rng_step=4, game_offset=2, dump=True)
    m = Mirror(o, conf)
    cv2, rv2, act2, roots = m.search(obs, legal, tp, explore, 2, 4)
    assert np.array_equal(cv, cv2)
    assert np.array_equal(rv, rv2)
    assert np.array_equal(act, act2)
    for g in range(G):        # root children statistics from the dump
        for a, ch in roots[g].children.items():
            assert tree["N"][g, 0, a - 1] == ch.visit_count
            assert tree["W"][g, 0, a - 1] == ch.value_sum
            assert tree["P"][g, 0, a - 1] == ch.prior


# ------------------------------------------------------------- TicTacToe (Q14)
def test_tictactoe_rules_q14():
    from muzero_jl_amd.games.tictactoe import TicTacToe
    env = TicTacToe()
    env.reset()
    # player 1 completes column 1 (cells 1,2,3) — not detected until player 2 moves
    for a in [1, 4, 2, 5, 3]:
        env(a)
    assert not env.is_terminated()
    assert env.legal_action_space() == [6, 7, 8, 9]
    env(9)                                    # player 2 moves; now player 1 (to move) has a line
    assert env.is_terminated()
    assert env.reward(2) == -1 and env.reward(1) == 1
    # player 2 completes a line: labelled winner=1 after player 1's next move
    env.reset()
    for a in [1, 4, 2, 5, 9, 6]:
        env(a)
    assert not env.is_terminated()            # player 2's line is unchecked while player 1 is to move
    env(7)
    assert env.is_terminated()
    assert env.reward(1) == 1                 # the mover (player 1) is credited the "win"


def test_tictactoe_python_matches_oracle():
    import ctypes
    from muzero_jl_amd.games.tictactoe import BatchedTicTacToe, TicTacToe
    from oracle import lib
    L = lib()
    rng = np.random.default_rng(1)
    for game in range(200):
        env, benv = TicTacToe(), BatchedTicTacToe(1)
        env.reset()
        board = np.zeros(27, np.uint8)
        board[18:] = 1
        player = ctypes.c_int32(1)
        done = False
        while not done:
            la = env.legal_action_space()
            assert la == [i + 1 for i in np.flatnonzero(benv.legal_mask()[0])]
            a = int(rng.choice(la))
            p = env.current_player()
            env(a)
            r_b, d_b = benv.step(np.array([a], np.int32))
            legal = np.zeros(9, np.uint8)
            rew = ctypes.c_float()
            dn = ctypes.c_int32()
            L.ora_ttt_step(board.ctypes.data_as(ctypes.c_void_p), ctypes.byref(player), a,
                           legal.ctypes.data_as(ctypes.c_void_p), ctypes.byref(rew), ctypes.byref(dn))
            assert np.array_equal(board.astype(bool), env.board)
            assert env.reward(p) == rew.value == r_b[0]
            done = env.is_terminated()
            assert done == bool(dn.value) == bool(d_b[0])


# -------------------------------------------------------- replay targets (Q9)
def _history_from(d):
    from muzero_jl_amd.selfplay import GameHistory
    h = GameHistory()
    h.observation_history = list(d["observation"])
    h.action_history = list(map(int, d["action"]))
    h.reward_history = list(map(float, d["reward"]))
    h.to_play_history = list(map(int, d["to_play"]))
    h.child_visits = list(d["child_visits"])
    h.root_values = list(map(float, d["root_values"]))
    return h


def test_value_targets_and_batch_match_oracle(ttt, nets):
    import ctypes
    from muzero_jl_amd.config import to_c_config
    from muzero_jl_amd.replay_buffer import ReplayBuffer, compute_target_value
    from oracle import histories_to_c, lib
    conf = dataclasses.replace(ttt.conf, num_iters=8, td_steps=3)
    o = _oracle(conf, ttt.hyper, nets, seed=3)
    games = [o.play_game(game_id=g, step0=0) for g in range(12)]
    hist = [_history_from(d) for d in games]
    arr, keep = histories_to_c(games)
    cc = to_c_config(conf)
    L = lib()
    for gi, h in enumerate(hist):
        for idx in range(1, len(h.root_values) + 1):
            a = compute_target_value(conf, h, idx)
            b = L.ora_compute_target_value(ctypes.byref(cc), ctypes.byref(arr[gi]), idx)
            assert a == f32(b)
    buf = ReplayBuffer(conf, seed=77)
    for h in hist:
        buf.save_game(h)
    _, batch = buf.get_batch(step=5)
    B, K, A = conf.batch_size, conf.num_unroll_steps, 9
    out = dict(observation=np.zeros((B, 63), np.float32), actions=np.zeros((B, K + 1), np.float32),
               target_values=np.zeros((B, K + 1), np.float32), target_rewards=np.zeros((B, K + 1), np.float32),
               target_policies=np.zeros((B, K + 1, A), np.float32), gradient_scale=np.zeros(B, np.float32))
    idx = np.zeros((B, 2), np.int32)
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    L.ora_get_batch(ctypes.byref(cc), arr, len(games), 1, 77, 5, p(out["observation"]), p(out["actions"]),
                    p(out["target_values"]), p(out["target_rewards"]), p(out["target_policies"]),
                    p(out["gradient_scale"]), p(idx))
    for k in out:
        assert np.array_equal(batch[k], out[k]), k


def test_replay_fifo_eviction(ttt):
    from muzero_jl_amd.replay_buffer import ReplayBuffer
    from muzero_jl_amd.selfplay import GameHistory
    conf = dataclasses.replace(ttt.conf, replay_buffer_size=3)
    buf = ReplayBuffer(conf)
    for i in range(5):
        h = GameHistory()
        h.root_values = [0.0] * (i + 1)
        buf.save_game(h)
    assert list(buf.buffer.keys()) == [3, 4, 5]
    assert buf.total_samples == 3 + 4 + 5 and buf.num_played_games == 5


# --------------------------------------------------------------- learner (Q11)
def test_adam_matches_flux_formula():
    """Flux 0.12 ADAM (Float64 β/η/ϵ over Float32 state) on ∇ = 2θ, restated in numpy."""
    import ctypes
    from oracle import lib
    L = lib()
    rng = np.random.default_rng(4)
    P = rng.standard_normal(1000).astype(np.float32)
    m = np.zeros_like(P)
    v = np.zeros_like(P)
    Pn, mn, vn = P.copy(), m.copy(), v.copy()
    bp = np.array([0.9, 0.999])
    for t in range(1, 6):
        eta = 0.05 * t
        L.ora_adam_2theta(P.ctypes.data_as(ctypes.c_void_p), m.ctypes.data_as(ctypes.c_void_p),
                          v.ctypes.data_as(ctypes.c_void_p), P.size, bp.ctypes.data_as(ctypes.c_void_p), eta)
        g = (Pn * f32(2)).astype(np.float32)
        mn = (0.9 * mn.astype(np.float64) + (1 - 0.9) * g.astype(np.float64)).astype(np.float32)
        vn = (0.999 * vn.astype(np.float64) + (1 - 0.999) * (g * g).astype(np.float64)).astype(np.float32)
        d = (mn.astype(np.float64) / (1 - bp[0]) / (np.sqrt(vn.astype(np.float64) / (1 - bp[1])) + 1e-8) * eta)
        Pn = (Pn - d.astype(np.float32)).astype(np.float32)
        bp = bp * np.array([0.9, 0.999])
        assert np.array_equal(P, Pn) and np.array_equal(m, mn) and np.array_equal(v, vn)


def test_unroll_prediction_alignment_q10(ttt, nets):
    """values = [v(h0), v(h0), v(h1), ...], rewards = [0, r1, ...] (Learning.jl:347-370)."""
    o = _oracle(ttt.conf, ttt.hyper, nets)
    rng = np.random.default_rng(5)
    B, K = 4, ttt.conf.num_unroll_steps
    obs = (rng.random((B, 63)) < 0.4).astype(np.float32)
    acts = rng.integers(1, 10, (B, K + 1)).astype(np.float32)
    pv, pp, pr = o.unroll(obs, acts)
    h = o.forward(0, obs)
    v0, p0 = o.forward(1, h)
    assert np.array_equal(pv[:, 0], v0[:, 0]) and np.array_equal(pv[:, 1], v0[:, 0])
    assert np.array_equal(pp[:, 0], p0) and np.array_equal(pp[:, 1], p0)
    assert np.all(pr[:, 0] == 0)
    sa = np.concatenate([h * f32(2), np.repeat((acts[:, :1] / f32(9)).astype(np.float32), 9, 1)], 1)
    h1, r1 = o.forward(2, sa)
    v1, _ = o.forward(1, h1)
    assert np.array_equal(pr[:, 1], r1[:, 0]) and np.array_equal(pv[:, 2], v1[:, 0])
