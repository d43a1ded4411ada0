"""The device actor–learner loop (mz_train_run: mz_selfplay_move with the
actors' nets, one mz_learner_train_dev per saved game, actor refresh one
checkpoint behind) against the oracle's restatement ora_train_loop, bit for
bit: learner step count, replay counters, every held game, the games in
progress, the learner's / actors' / queued nets and the last losses.
Reference: src/SelfPlay.jl:384-419, src/Learning.jl:306-438 (quirk Q16)."""
import dataclasses

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("resnet,training_steps,thr", [(False, 10000, None), (False, 9, 3), (True, 10000, None)])
def test_train_loop_matches_oracle(ttt, resnet, training_steps, thr):
    import torch
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import to_c_config, to_c_ffhp, to_c_resnet_hp
    from muzero_jl_amd.networks import init_nets
    from oracle import Oracle, train_loop
    G, cap, moves, B = 12, 20, 26, 8
    hyper = ttt.resnet_hyper if resnet else ttt.hyper
    conf = dataclasses.replace(ttt.conf, num_iters=5 if resnet else 8, batch_size=B, checkpoint_interval=3,
                               training_steps=training_steps, temperature_threshold=thr)
    nets = init_nets(conf, hyper, seed=17)
    o = Oracle(to_c_config(conf), to_c_resnet_hp(hyper) if resnet else to_c_ffhp(hyper), seed=5)
    eng = abi.Engine(conf, hyper, device=0, max_games=G, rng_seed=5)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    eng.selfplay_init(abi.ENV_TICTACTOE, G, cap)
    eng.train_init(B)
    losses = torch.zeros(8, dtype=torch.float32, device="cuda")
    st1 = eng.train_run(moves // 2, move0=10, game_offset=3, losses_ptr=losses.data_ptr())
    st2 = eng.train_run(moves - moves // 2, move0=10 + moves // 2, game_offset=3, losses_ptr=losses.data_ptr())
    r = train_loop(o, G, cap, moves, move0=10, game_offset=3)
    assert st2[0] == r["t"] and st2[1] == r["counters"][0] and st1[3] + st2[3] == r["t"]
    assert st2[2] == r["t"] // 3                          # refreshes at t = 3, 6, ... (t > 1)
    counts, held = eng.replay_counts()
    assert np.array_equal(counts, r["counters"]) and held == len(r["held"])
    for i, h in enumerate(r["held"]):
        d = eng.replay_get_game(i).as_arrays()
        assert np.array_equal(d["observation"].reshape(-1, 27), h["observation"]), i
        for k in ("action", "reward", "to_play", "child_visits", "root_values"):
            assert np.array_equal(d[k], h[k]), (i, k)
    ln, board, player = eng.selfplay_slots()
    assert np.array_equal(ln, r["slot_len"]) and np.array_equal(board, r["slot_board"])
    assert np.array_equal(player, r["slot_player"])
    for n in range(3):
        assert np.array_equal(eng.train_weights(abi.TRAIN_LEARNER, n), o.params[n]), f"learner net {n}"
        assert np.array_equal(eng.train_weights(abi.TRAIN_ACTOR, n), r["actor"][n]), f"actor net {n}"
        assert np.array_equal(eng.train_weights(abi.TRAIN_QUEUED, n), r["queued"][n]), f"queued net {n}"
    assert np.array_equal(losses.cpu().numpy()[:6], r["losses"])
    eng.close()


def _loop_setup(ttt, G, cap, B, ci, training_steps, S=6, seed=5):
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import to_c_config, to_c_ffhp
    from muzero_jl_amd.networks import init_nets
    from oracle import Oracle
    conf = dataclasses.replace(ttt.conf, num_iters=S, batch_size=B, checkpoint_interval=ci,
                               training_steps=training_steps)
    nets = init_nets(conf, ttt.hyper, seed=seed + 12)
    o = Oracle(to_c_config(conf), to_c_ffhp(ttt.hyper), seed=seed)
    eng = abi.Engine(conf, ttt.hyper, device=0, max_games=G, rng_seed=seed)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    eng.selfplay_init(abi.ENV_TICTACTOE, G, cap)
    return conf, o, eng


def test_train_loop_temperature_per_game_across_the_500k_boundary(ttt):
    """Resume at t0 = 499,990 (mz_train_init_at): visit_softmax_temperature_fn
    drops from 1.0 to 0.5 at t = 500,000 (SelfPlay.jl:48-56) in the middle of the
    run.  Each game keeps the temperature of the step at which it started
    (play_game takes T once per game, SelfPlay.jl:396-407), so games in
    progress finish at 1.0 while new ones play at 0.5 — against the oracle."""
    from muzero_jl_amd import abi
    from oracle import train_loop
    G, cap, moves, B, t0 = 12, 40, 24, 8, 499_990
    conf, o, eng = _loop_setup(ttt, G, cap, B, 3, 500_100)
    eng.train_init(B, t0=t0)
    st = eng.train_run(moves, move0=7, game_offset=5)
    r = train_loop(o, G, cap, moves, move0=7, game_offset=5, t0=t0)
    assert st[0] == r["t"] and r["t"] > 500_000 + 10, r["t"]    # new games started past the boundary
    counts, held = eng.replay_counts()
    assert np.array_equal(counts, r["counters"]) and held == len(r["held"])
    for i, h in enumerate(r["held"]):
        d = eng.replay_get_game(i).as_arrays()
        for k in ("action", "child_visits", "root_values"):
            assert np.array_equal(d[k], h[k]), (i, k)
    ln, board, player = eng.selfplay_slots()
    assert np.array_equal(ln, r["slot_len"]) and np.array_equal(board, r["slot_board"])
    for n in range(3):
        assert np.array_equal(eng.train_weights(abi.TRAIN_LEARNER, n), o.params[n]), f"learner net {n}"
        assert np.array_equal(eng.train_weights(abi.TRAIN_ACTOR, n), r["actor"][n]), f"actor net {n}"
    eng.close()


def test_train_loop_periodic_checkpoints(ttt, tmp_path):
    """conf.networks_path set: past round(0.9 training_steps) every
    checkpoint_interval-th step writes the learner's nets (Learning.jl:416-432).
    training_steps = 39 -> the loop runs to t = 40 (while t <= 39), and only
    t = 40 > round(35.1) = 35 is a checkpoint step; its file holds the final
    learner nets, equal to the oracle's."""
    import os
    from muzero_jl_amd import abi
    from muzero_jl_amd import checkpoint as ck
    from oracle import train_loop
    G, cap, moves, B = 24, 60, 40, 8
    conf, o, eng = _loop_setup(ttt, G, cap, B, 10, 39)
    eng.train_set_networks_path(str(tmp_path))
    eng.train_init(B)
    st = eng.train_run(moves, move0=3)
    r = train_loop(o, G, cap, moves, move0=3)
    assert st[0] == r["t"] == 40
    assert sorted(os.listdir(tmp_path)) == ["40.safetensors"]
    tensors, meta = ck.read(str(tmp_path / "40.safetensors"))
    assert meta["training_step"] == "40"
    for n, flat in enumerate(ck.nets_from(tensors, conf, ttt.hyper)):
        assert np.array_equal(flat, o.params[n]), f"checkpoint net {n} != oracle learner"
        assert np.array_equal(flat, eng.train_weights(abi.TRAIN_LEARNER, n))
    eng.close()
