"""Golden fixtures (tests/golden/oracle_golden.npz, made by make_golden.py):
the oracle must keep reproducing them bit-exactly (regression pin), and the
GPU engine must reproduce them too."""
import dataclasses
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden():
    return dict(np.load(os.path.join(HERE, "golden", "oracle_golden.npz")))


@pytest.fixture(scope="module")
def gnets(ttt, golden):
    from muzero_jl_amd.networks import init_nets
    nets = init_nets(ttt.conf, ttt.hyper, seed=2024)
    assert np.array_equal([float(np.sum(w.astype(np.float64))) for w in nets], golden["weights_sum"])
    return nets


def _oracle(conf, hyper, nets):
    from muzero_jl_amd.config import to_c_config, to_c_ffhp
    from oracle import Oracle
    o = Oracle(to_c_config(conf), to_c_ffhp(hyper), seed=42)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
    return o


def test_oracle_reproduces_golden(ttt, golden, gnets):
    o = _oracle(ttt.conf, ttt.hyper, gnets)
    for net in range(3):
        r = o.forward(net, golden[f"fwd{net}_x"])
        if net == 0:
            assert np.array_equal(r, golden["fwd0_y0"])
        else:
            assert np.array_equal(r[0], golden[f"fwd{net}_y0"]) and np.array_equal(r[1], golden[f"fwd{net}_y1"])
    for S in (10, 25):
        o = _oracle(dataclasses.replace(ttt.conf, num_iters=S), ttt.hyper, gnets)
        cv, rv, act = o.mcts_search(golden[f"s{S}_obs"], golden[f"s{S}_legal"], golden[f"s{S}_tp"],
                                    exploration=True, rng_step=S, game_offset=3)
        assert np.array_equal(cv, golden[f"s{S}_cv"]) and np.array_equal(rv, golden[f"s{S}_rv"])
        assert np.array_equal(act, golden[f"s{S}_act"])
    g = o = _oracle(ttt.conf, ttt.hyper, gnets).play_game(game_id=5, step0=11)
    for k, v in g.items():
        assert np.array_equal(v, golden[f"game_{k}"]), k


@pytest.mark.gpu
def test_gpu_reproduces_golden(ttt, golden, gnets):
    from muzero_jl_amd.abi import Engine
    for S in (10, 25):
        conf = dataclasses.replace(ttt.conf, num_iters=S)
        eng = Engine(conf, ttt.hyper, device=0, max_games=16, rng_seed=42)
        for n, w in enumerate(gnets):
            eng.set_weights(n, w)
        if S == 10:
            for net in range(3):
                r = eng.forward(net, golden[f"fwd{net}_x"])
                r0 = r if net == 0 else r[0]
                assert np.array_equal(r0, golden[f"fwd{net}_y0"])
        cv, rv, act = eng.mcts_search(golden[f"s{S}_obs"], golden[f"s{S}_legal"], golden[f"s{S}_tp"],
                                      exploration=True, rng_step=S, game_offset=3)
        assert np.array_equal(cv, golden[f"s{S}_cv"]) and np.array_equal(rv, golden[f"s{S}_rv"])
        assert np.array_equal(act, golden[f"s{S}_act"])
        eng.close()


@pytest.mark.gpu
def test_gpu_selfplay_game_matches_oracle_play_game(ttt, golden, gnets):
    """Whole self-play games through the Python host driver + GPU search equal
    the oracle's play_game (SelfPlay.jl:330-382) move for move."""
    from muzero_jl_amd.abi import Engine
    from muzero_jl_amd.games.tictactoe import BatchedTicTacToe
    from muzero_jl_amd.selfplay import BatchedSelfPlay
    G = 8
    eng = Engine(ttt.conf, ttt.hyper, device=0, max_games=G, rng_seed=42)
    for n, w in enumerate(gnets):
        eng.set_weights(n, w)
    sp = BatchedSelfPlay(eng, BatchedTicTacToe, G, game_offset=0, step0=11)
    games = sp.play_games()
    o = _oracle(ttt.conf, ttt.hyper, gnets)
    for g in range(G):
        ref = o.play_game(game_id=g, step0=11)
        got = games[g].as_arrays()
        for k in ("action", "reward", "to_play", "child_visits", "root_values", "observation"):
            assert np.array_equal(got[k], ref[k]), (g, k)
    eng.close()
