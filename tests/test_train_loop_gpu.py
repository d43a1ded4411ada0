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
