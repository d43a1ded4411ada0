"""The synthetic Atari-like env of configs[4] (games/atari_synth.py) and its
data path: self-play -> replay shard -> get_batch / make_target -> learner
(SelfPlay.jl:330-382, ReplayBuffer.jl:133-217, Learning.jl:327-404).

CPU: the vectorised Philox against the scalar one, the env's rules (reset and
step keys, rewards, terminal draws, frame bytes), the four-frame observation,
and the host ReplayBuffer's frame-stacked batches.  GPU: the device env
(mz_selfplay.hip, one frame per move in the records) against the host driver
(selfplay.BatchedSelfPlay over the same engine search) move for move —
finished games, games in progress, replay counters — then device get_batch
against the host ReplayBuffer and a learner step on the device batch against
mz_learner_step on the host batch, bit for bit.
"""
import dataclasses

import numpy as np
import pytest


def test_philox_np_matches_scalar():
    from muzero_jl_amd.rng import _philox, philox_np
    rng = np.random.default_rng(0)
    c = rng.integers(0, 2**32, (6, 50), dtype=np.uint64)
    vec = philox_np(*c)
    for i in range(50):
        assert tuple(int(v[i]) for v in vec) == _philox(*(int(x[i]) for x in c))


def test_env_rules():
    from muzero_jl_amd.games import atari_synth as at
    from muzero_jl_amd.rng import _philox, rng_below, rng_u32
    env = at.BatchedAtariSynth(3, seed=5)
    for g in range(3):
        key = rng_u32(5, at.MZ_RNG_ENV, g, 0xFFFFFFFF, 0xFFFFFFFF)
        assert env.key[g] == key
        w = _philox(7, key, 0, at.MZ_RNG_FRAME, 5, 0)                  # block 7 = bytes 112..127
        assert list(env.board[g, 112:128]) == [(w[q] >> (8 * b)) & 255 for q in range(4) for b in range(4)]
    assert env.legal_mask().all() and env.legal_mask().shape == (3, 18)
    keys = env.key.copy()
    r, d = env.step(np.array([1, 5, 18]))
    for g, a in enumerate((1, 5, 18)):
        v = _philox(0, int(keys[g]), a, at.MZ_RNG_ENV, 5, 0)
        assert r[g] == (1.0 if rng_below(v[0], 18) == a - 1 else 0.0)
        assert d[g] == ((v[1] & 127) == 0)
        assert env.key[g] == v[2] and np.array_equal(env.board[g], at.frame(5, v[2]))
    env.reset([1], step=42)
    assert env.key[1] == rng_u32(5, at.MZ_RNG_ENV, 1, 42, 0xFFFFFFFF)
    # keyed by the global game id: slot g of a shard at game_offset o is game o + g
    sh = at.BatchedAtariSynth(2, seed=5, game_offset=1)
    assert sh.key[0] == rng_u32(5, at.MZ_RNG_ENV, 1, 0xFFFFFFFF, 0xFFFFFFFF)
    assert np.array_equal(sh.board[1], at.BatchedAtariSynth(3, seed=5).board[2])
    # episode lengths: terminal with p = 1/128 per move
    env = at.BatchedAtariSynth(64, seed=1)
    ends = 0
    for _ in range(64):
        _, d = env.step(np.ones(64, np.int32))
        ends += d.sum()
    assert 8 <= ends <= 64


def test_frame_stack_observation():
    from muzero_jl_amd.games import atari_synth as at
    from muzero_jl_amd.selfplay import frame_stack_obs
    rng = np.random.default_rng(2)
    frames = [rng.integers(0, 256, at.FRAME, dtype=np.uint8) for _ in range(6)]
    o = frame_stack_obs(frames, 2, 4)
    assert o.shape == (4 * at.FRAME,) and not o[:2 * at.FRAME].any()
    assert np.array_equal(o[2 * at.FRAME:3 * at.FRAME], frames[0].astype(np.float32) * at.FRAME_SCALE)
    assert np.array_equal(o[3 * at.FRAME:], frames[1].astype(np.float32) * at.FRAME_SCALE)
    o = frame_stack_obs(frames, 6, 4)
    assert np.array_equal(o[:at.FRAME], frames[2].astype(np.float32) * at.FRAME_SCALE)
    assert o.max() <= 1.0 and at.FRAME_SCALE == np.float32(1 / 255)


def test_replay_buffer_frame_stacked_batch():
    from muzero_jl_amd.games import atari_synth as at
    from muzero_jl_amd.replay_buffer import ReplayBuffer
    from muzero_jl_amd.selfplay import GameHistory, frame_stack_obs
    conf = dataclasses.replace(at.conf, batch_size=6)
    rng = np.random.default_rng(3)
    rb = ReplayBuffer(conf, seed=1, frame_stack=4)
    for n in (5, 9):
        h = GameHistory()
        for t in range(n):
            h.observation_history.append(rng.integers(0, 256, at.FRAME, dtype=np.uint8))
            h.action_history.append(int(rng.integers(1, 19)))
            h.reward_history.append(float(rng.integers(0, 2)))
            h.to_play_history.append(1)
            h.child_visits.append(np.full(18, 1 / 18, np.float32))
            h.root_values.append(float(rng.standard_normal()))
        rb.save_game(h)
    idx, b = rb.get_batch(3)
    assert b["observation"].shape == (6, 4 * at.FRAME)
    for i, (gid, pos) in enumerate(idx):
        assert np.array_equal(b["observation"][i], frame_stack_obs(rb.buffer[gid].observation_history, pos, 4))


def _atari_pair(G, moves, cap, S=6, max_moves=12, step0=100):
    from muzero_jl_amd import abi
    from muzero_jl_amd.games import atari_synth as at
    from muzero_jl_amd.networks import init_nets
    from muzero_jl_amd.selfplay import BatchedSelfPlay
    conf = dataclasses.replace(at.conf, num_iters=S, max_moves=max_moves, replay_buffer_size=cap)
    nets = init_nets(conf, at.resnet_hyper, seed=105)
    eh, ed = (abi.Engine(conf, at.resnet_hyper, device=0, max_games=G, rng_seed=5) for _ in range(2))
    for e in (eh, ed):
        for n, w in enumerate(nets):
            e.set_weights(n, w)
    sp = BatchedSelfPlay(eh, at.BatchedAtariSynth, G, game_offset=7, step0=step0)
    ed.selfplay_init(abi.ENV_ATARI, G, cap)
    for m in range(moves):
        sp.play_move(1.0)
        ed.selfplay_move(step0 + m, game_offset=7, temperature=1.0)
    return conf, sp, eh, ed


def _same_game(dev, host):
    a, b = dev.as_arrays(), host.as_arrays()
    assert np.array_equal(a["observation"], b["observation"])
    for k in ("action", "reward", "to_play", "child_visits", "root_values"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.gpu
def test_atari_selfplay_matches_host():
    G = 6
    conf, sp, eh, ed = _atari_pair(G, 20, cap=64)
    counts, held = ed.replay_counts()
    assert counts[0] == len(sp.finished) == held >= G              # max_moves = 12: every slot finished once
    assert counts[1] == sum(len(h.root_values) for h in sp.finished) == counts[2]
    for i, h in enumerate(sp.finished):
        _same_game(ed.replay_get_game(i), h)
    ln, board, player = ed.selfplay_slots()
    assert np.array_equal(ln, [len(h.action_history) for h in sp.histories])
    assert np.array_equal(board, sp.env.board) and (player == 1).all()
    eh.close(); ed.close()


@pytest.mark.gpu
def test_atari_replay_sample_and_learner_match_host():
    """Device get_batch on the frame records equals the host ReplayBuffer
    (frame_stack = 4); one learner step on the device batch (sampling +
    ResNet unroll with the downsampler + ADAM) equals mz_learner_step on the
    host batch."""
    from muzero_jl_amd.config import cos_schedule
    from muzero_jl_amd.replay_buffer import ReplayBuffer
    G, B = 6, 8
    conf, sp, eh, ed = _atari_pair(G, 16, cap=64)
    rb = ReplayBuffer(dataclasses.replace(conf, batch_size=B), seed=5, frame_stack=4)
    for h in sp.finished:
        rb.save_game(h)
    assert len(rb) > 0
    for step in (1, 2):
        idx_h, bh = rb.get_batch(step)
        b, idx_d = ed.replay_sample(B, step, index=True)
        bd = ed.batch_to_host(b)
        assert [tuple(x) for x in idx_d] == [tuple(x) for x in idx_h]
        for k in bh:
            assert np.array_equal(bd[k], bh[k]), (step, k)
    import torch
    losses = torch.empty(8, dtype=torch.float32, device="cuda")
    for step in (1, 2):
        eta = cos_schedule(step)
        _, bh = rb.get_batch(step)
        lh = eh.learner_step(bh, eta)
        ed.learner_train_dev(B, step, eta, losses.data_ptr())
        ed.sync()
        ld = losses.cpu().numpy()[:6]
        assert np.array_equal(ld, lh), (step, ld, lh)
        for n in range(3):
            assert np.array_equal(ed.get_weights(n), eh.get_weights(n)), (step, n)
    eh.close(); ed.close()
