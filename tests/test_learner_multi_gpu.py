"""L ref_semantics learner steps per launch pair (mz_learner_train_multi_dev,
Learning.jl:327-404 with Q11: θ_{s+1} = ADAM(θ_s, 2θ_s) does not read the data,
and with PER off step s's batch is keyed by s) against the sequential learner,
bit for bit at every step of the chunk: the six losses, the unroll read-outs
and all three nets' θ after the step —
* against L mz_learner_train_dev calls on an engine holding the same replay
  shard (FC TicTacToe / Connect4, FC + BatchNorm, chunks of 1..50 steps —
  several sub-chunks with alternating bank halves — T = 1 and T = 2 samples
  per workgroup, single steps before and after the chunk; the ResNet nets of
  TicTacToe (configs[2], the fused unroll launch), Connect4 and the Atari-like
  env (downsampler, split unroll launches) with the steps on gridDim.z);
* against the oracle's ora_learner_step fed the same device get_batch samples.
"""
import dataclasses

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mods(kind):
    from muzero_jl_amd import abi
    from muzero_jl_amd.games import atari_synth, connect4, tictactoe
    if kind == "atari":
        return atari_synth, abi.ENV_ATARI
    return (tictactoe, abi.ENV_TICTACTOE) if kind.startswith("ttt") else (connect4, abi.ENV_CONNECT4)


def _pair(kind, G=16, cap=64, seed=5):
    """Two engines with the same weights whose device self-play fills identical replay shards
    (kinds: FC TicTacToe / Connect4, "ttt-bn" FC + BatchNorm, "ttt-rn" / "c4-rn" / "atari" ResNet)."""
    from muzero_jl_amd import abi
    from muzero_jl_amd.networks import init_nets
    mod, env_kind = _mods(kind)
    conf = dataclasses.replace(mod.conf, num_iters=6 if kind != "atari" else 2, replay_buffer_size=cap)
    hyper = mod.resnet_hyper if kind.endswith("-rn") or kind == "atari" else mod.hyper
    if kind == "ttt-bn":
        hyper = dataclasses.replace(hyper, use_batch_norm=True)
    if kind == "atari":
        G = 32
    nets = init_nets(conf, hyper, seed=seed + 100)
    moves = {"ttt": 14, "ttt-bn": 14, "ttt-rn": 14, "c4": 30, "c4-rn": 30, "atari": 48}[kind]
    out = []
    for _ in range(2):
        e = abi.Engine(conf, hyper, device=0, max_games=G, rng_seed=seed)
        for n, w in enumerate(nets):
            e.set_weights(n, w)
        e.selfplay_init(env_kind, G, cap)
        for m in range(moves):
            e.selfplay_move(100 + m, game_offset=7)
        out.append(e)
    assert out[0].replay_counts()[0][0] > 0
    return conf, hyper, nets, out


def _theta(e):
    return np.concatenate([e.get_weights(n) for n in range(3)])


@pytest.mark.parametrize("kind,B,L", [("ttt", 32, 8), ("ttt", 32, 16), ("ttt", 32, 1), ("ttt", 40, 5),
                                      ("c4", 24, 10), ("ttt-bn", 32, 6), ("ttt", 32, 37), ("ttt", 40, 50),
                                      ("ttt-rn", 32, 8), ("ttt-rn", 32, 21), ("ttt-rn", 7, 3), ("c4-rn", 16, 6),
                                      ("atari", 8, 5)])
def test_multi_matches_sequential_steps(kind, B, L):
    import torch
    from muzero_jl_amd.config import cos_schedule
    _, _, _, (e1, e2) = _pair(kind)
    nflat = sum(e1.param_count(n) for n in range(3))
    l1 = torch.zeros(8, dtype=torch.float32, device="cuda")
    lm = torch.zeros((L, 8), dtype=torch.float32, device="cuda")
    th = torch.zeros((L, nflat), dtype=torch.float32, device="cuda")
    for step in (1, 2):                               # the one-step path first (image sets swapped)
        for e in (e1, e2):                            # (own loss buffers: the engines' streams run concurrently)
            e.learner_train_dev(B, step, cos_schedule(step), None)
    for rnd, t0 in enumerate((3, 3 + L + 1)):
        etas = [cos_schedule(t0 + i) for i in range(L)]
        want = []
        for i in range(L):
            e1.learner_train_dev(B, t0 + i, etas[i], l1.data_ptr())
            e1.sync()
            want.append((l1.cpu().numpy()[:6].copy(), _theta(e1), [x.copy() for x in e1.debug_unroll(B)]))
        e2.learner_train_multi_dev(B, t0, etas, lm.data_ptr(), th.data_ptr())
        e2.sync()
        # FC: the two-launch form wherever the one-launch step runs (else the steps one after
        # another); ResNet: always the multi-step form
        rn = kind.endswith("-rn") or kind == "atari"
        assert ("multi" in e2.learner_variant()) == (rn or e1.learner_variant().startswith("mz_learn_small")), \
            (e1.learner_variant(), e2.learner_variant())
        multi = "multi" in e2.learner_variant()
        got_l, got_t = lm.cpu().numpy(), th.cpu().numpy()
        for i, (wl, wt, wu) in enumerate(want):
            assert np.array_equal(got_l[i, :6], wl), (rnd, i, got_l[i, :6], wl)
            assert np.array_equal(got_t[i], wt), (rnd, i, "theta")
            # (steps one after another: the last unroll's; the multi-step read-outs are a ring of >= 33
            # steps, mz_debug_unroll_step)
            if (multi and i >= L - 33) or i == L - 1:
                for g, w in zip(e2.debug_unroll_step(i, B) if multi else e2.debug_unroll(B), wu):
                    assert np.array_equal(g, w), (rnd, i, "read-outs")
        assert np.array_equal(_theta(e2), want[-1][1])
        # a single step after the chunk: the engine's images, moments and β powers are current
        s = t0 + L
        for e in (e1, e2):
            e.learner_train_dev(B, s, cos_schedule(s), l1.data_ptr() if e is e1 else lm.data_ptr())
        e1.sync(); e2.sync()
        assert np.array_equal(l1.cpu().numpy()[:6], lm.cpu().numpy()[0, :6])
        assert np.array_equal(_theta(e1), _theta(e2))
    e1.close(); e2.close()


def test_multi_matches_oracle_steps():
    """The chunk against ora_learner_step on the host copies of the device
    batches (get_batch keyed by the step), the oracle's unroll of θ_{t+i}
    against step i's read-outs."""
    import torch
    from muzero_jl_amd.config import cos_schedule, to_c_config, to_c_ffhp
    from oracle import Oracle
    B, L, t0 = 32, 8, 1
    conf, hyper, nets, (e1, e2) = _pair("ttt")
    o = Oracle(to_c_config(dataclasses.replace(conf, batch_size=B)), to_c_ffhp(hyper), seed=5)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
    st = o.learner_state()
    nflat = sum(o.param_count(n) for n in range(3))
    lm = torch.zeros((L, 8), dtype=torch.float32, device="cuda")
    th = torch.zeros((L, nflat), dtype=torch.float32, device="cuda")
    etas = [cos_schedule(t0 + i) for i in range(L)]
    e2.learner_train_multi_dev(B, t0, etas, lm.data_ptr(), th.data_ptr())
    e2.sync()
    got_l, got_t = lm.cpu().numpy(), th.cpu().numpy()
    for i in range(L):
        b, _ = e1.replay_sample(B, t0 + i)
        batch = e1.batch_to_host(b)
        want_u = o.unroll(batch["observation"], batch["actions"])
        for g, w in zip(e2.debug_unroll_step(i, B), want_u):
            assert np.array_equal(g, w), (i, "read-outs")
        lo = o.learner_step(st, batch, etas[i])
        assert np.array_equal(got_l[i, :6], lo), (i, got_l[i, :6], lo)
        assert np.array_equal(got_t[i], np.concatenate(o.params)), (i, "theta")
    e1.close(); e2.close()


def test_multi_rejects_bad_arguments():
    from muzero_jl_amd.abi import MzError
    _, _, _, (e1, e2) = _pair("ttt")
    with pytest.raises(MzError, match="L must be"):
        e1.learner_train_multi_dev(32, 1, [1e-3] * 257)
    with pytest.raises(MzError, match="L must be"):
        e1.learner_train_multi_dev(32, 1, [])
    e1.close(); e2.close()
