"""GPU parity at the exact bench launches of configs[2], configs[3] and
configs[4] (VERDICT r2 "Next round" item 1).

Each test builds the inputs bench.py builds for that line — the same nets
(`init_nets(conf, hyper, seed=1234)`), the same positions
(`selfplay.random_positions(env, G, seed=100, ...)` / `atari_synth.observations(G,
seed=0)`), the engine RNG seed 1 — and runs ONE search through
`mz_mcts_search_dev` on device buffers and a non-null stream, as the bench's
timed step does, at the bench's G and S.  Trees (N, W, P, R, child slots),
child visits, root values and the 1-based actions are compared with the C
oracle bit for bit; the oracle searches game chunks on 16 host threads (game
ids are global, so the chunks are independent).

* configs[2]: TicTacToe ResNet (2 blocks x 64 filters), G = 2048, S = 50.
* configs[3]: Connect4 ResNet-8 (4 blocks x 64 filters, 3x3), G = 512 (one
  GPU's shard of 4096), S = 50.
* configs[4]: Atari-like 84x84x4 with the Learning.jl:175-187 downsampler,
  G = 512, S = 200, one player, every action legal.

Reference: src/SelfPlay.jl:230-306 (run_mcts, select_action,
store_search_stats!), src/Learning.jl:148-255 (the ResNet nets).
"""
import dataclasses

import numpy as np
import pytest

from test_bench_sizes_gpu import _oracle_search_threads
from test_gpu_parity import _compare_trees

pytestmark = pytest.mark.gpu


def _bench_launch(game, resnet, G, S, rng_step, explore=True, temp=1.0):
    import torch
    from muzero_jl_amd.abi import Engine
    from muzero_jl_amd.config import to_c_config, to_c_ffhp, to_c_resnet_hp
    from muzero_jl_amd.games import atari_synth as atari
    from muzero_jl_amd.games import connect4 as c4
    from muzero_jl_amd.games import tictactoe as ttt
    from muzero_jl_amd.networks import init_nets
    from muzero_jl_amd.selfplay import random_positions
    from oracle import Oracle

    conf = dataclasses.replace(game.conf, num_iters=S)
    hyper = game.resnet_hyper if resnet else game.hyper
    A = len(conf.action_space)
    nets = init_nets(conf, hyper, seed=1234)               # bench.py: identical replicas on every rank
    eng = Engine(conf, hyper, device=0, max_games=G, rng_seed=1)
    ora = Oracle(to_c_config(conf), to_c_resnet_hp(hyper) if resnet else to_c_ffhp(hyper), seed=1)
    for n, w in enumerate(nets):
        eng.set_weights(n, w)
        ora.set_weights(n, w)
    if game is atari:
        obs = atari.observations(G, seed=0)
        legal = np.ones((G, A), bool)
        tp = np.ones(G, np.int32)
    else:
        env_cls = c4.BatchedConnect4 if game is c4 else ttt.BatchedTicTacToe
        obs, legal, tp = random_positions(env_cls, G, seed=100, max_plies=6 if game is ttt else 16)

    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    d_obs = torch.from_numpy(np.ascontiguousarray(obs, np.float32)).to(dev)
    d_legal = torch.from_numpy(np.ascontiguousarray(legal, np.uint8)).to(dev)
    d_tp = torch.from_numpy(np.ascontiguousarray(tp, np.int32)).to(dev)
    d_cv = torch.empty((G, A), dtype=torch.float32, device=dev)
    d_rv = torch.empty(G, dtype=torch.float32, device=dev)
    d_act = torch.empty(G, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    eng.debug_enable(1)
    eng.mcts_search_dev(G, d_obs.data_ptr(), d_legal.data_ptr(), d_tp.data_ptr(), d_cv.data_ptr(),
                        d_rv.data_ptr(), d_act.data_ptr(), exploration=explore, rng_step=rng_step,
                        game_offset=0, temperature=temp, stream=stream.cuda_stream)
    stream.synchronize()
    tree_g = eng.debug_tree(G)
    variant = eng.search_variant()
    cv, rv, act = d_cv.cpu().numpy(), d_rv.cpu().numpy(), d_act.cpu().numpy()
    eng.close()
    cv2, rv2, act2, tree_o, stats = _oracle_search_threads(ora, obs, legal, tp, exploration=explore,
                                                           rng_step=rng_step, game_offset=0, temperature=temp)
    assert np.all(legal[np.arange(G), act - 1]), "illegal action"
    _compare_trees(tree_g, tree_o, G)
    assert np.array_equal(cv, cv2), "child visits differ"
    assert np.array_equal(rv, rv2), "root values differ"
    assert np.array_equal(act, act2), "actions differ"
    return variant, stats


def test_configs2_ttt_resnet_2048x50():
    from muzero_jl_amd.games import tictactoe as ttt
    variant, _ = _bench_launch(ttt, True, 2048, 50, rng_step=3)
    assert variant == "mz_rsearch"


def test_configs3_connect4_resnet8_512x50():
    from muzero_jl_amd.games import connect4 as c4
    variant, _ = _bench_launch(c4, True, 512, 50, rng_step=3)
    assert variant == "mz_rsearch"


def test_configs4_atari_512x200():
    from muzero_jl_amd.games import atari_synth as atari
    variant, stats = _bench_launch(atari, True, 512, 200, rng_step=3)
    assert variant == "mz_rsearch"
    assert stats[1] >= 32, f"max select depth {stats[1]}: the path store past the register-held levels unused"


def test_configs1_fc_512x50_dev_path():
    """configs[1] through the device-buffer entry point and the bench's own
    inputs (test_bench_sizes_gpu covers it through the host-buffer call)."""
    from muzero_jl_amd.games import tictactoe as ttt
    variant, _ = _bench_launch(ttt, False, 512, 50, rng_step=3)
    assert variant == "mz_search_small2"


def test_narrow_sync_stream():
    """mz_set_sync_stream: with the wait narrowed to the caller's
    stream, a host-synchronous call after `_dev` work queued on that stream
    still sees it complete — the device-buffer search and the host-buffer
    search give the same bits, and weights written before both read back."""
    import torch
    from muzero_jl_amd.abi import Engine
    from muzero_jl_amd.games import tictactoe as ttt
    from muzero_jl_amd.networks import init_nets
    from muzero_jl_amd.selfplay import random_positions

    G = 40
    conf = dataclasses.replace(ttt.conf, num_iters=16)
    eng = Engine(conf, ttt.hyper, device=0, max_games=G, rng_seed=1)
    nets = init_nets(conf, ttt.hyper, seed=5)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    eng.set_sync_stream(stream.cuda_stream)
    for n, w in enumerate(nets):
        eng.set_weights(n, w)
    obs, legal, tp = random_positions(ttt.BatchedTicTacToe, G, seed=100)
    d_obs = torch.from_numpy(np.ascontiguousarray(obs, np.float32)).to(dev)
    d_legal = torch.from_numpy(np.ascontiguousarray(legal, np.uint8)).to(dev)
    d_tp = torch.from_numpy(np.ascontiguousarray(tp, np.int32)).to(dev)
    d_cv = torch.empty((G, 9), dtype=torch.float32, device=dev)
    d_rv = torch.empty(G, dtype=torch.float32, device=dev)
    d_act = torch.empty(G, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    eng.mcts_search_dev(G, d_obs.data_ptr(), d_legal.data_ptr(), d_tp.data_ptr(), d_cv.data_ptr(),
                        d_rv.data_ptr(), d_act.data_ptr(), rng_step=2, stream=stream.cuda_stream)
    cv, rv, act = eng.mcts_search(obs, legal, tp, rng_step=2)      # narrow wait: `stream` + the handle's
    stream.synchronize()
    assert np.array_equal(d_cv.cpu().numpy(), cv)
    assert np.array_equal(d_rv.cpu().numpy(), rv)
    assert np.array_equal(d_act.cpu().numpy(), act)
    for n, w in enumerate(nets):
        assert np.array_equal(eng.get_weights(n), w)
    eng.set_sync_stream(None, narrow=False)
    cv2, _, _ = eng.mcts_search(obs, legal, tp, rng_step=2)
    assert np.array_equal(cv2, cv)
    eng.close()
