"""GPU parity at the sizes the bench runs (VERDICT r1 "Next round" item 1).

* configs[1] exactly: TicTacToe FC, G = 512 games x S = 50 simulations through
  the auto-dispatched kernel the bench times (mz_search_small2), trees, visits,
  values and actions bit-exact against the oracle (run on host threads, one
  game chunk per thread: game ids are global, so chunks are independent).
* configs[4] at its 200 simulations per move: the deep one-player regime —
  select depth >= 32 (the path store beyond the register-held levels,
  mz_tree_device.h), the multi-pass 1-player backup, and the LDS-cached tree
  step (mz_rsearch_tree_lds32, a 58 KB tree per game).  A game with a single
  legal action (Q4: every node then has one child) walks a chain to depth
  199; another has all 18 actions legal.
* configs[3]'s Connect4 ResNet-8 learner (B = 32, K = 5) against
  ora_learner_step: read-outs, losses and every parameter bit-exact.
Reference: src/SelfPlay.jl:254-283, src/Learning.jl:327-397.
"""
import dataclasses
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from conftest import random_positions
from test_gpu_parity import _compare_trees, _engine, _oracle
from test_resnet_oracle import _perturb_bn, _resnet_oracle

pytestmark = pytest.mark.gpu


def _oracle_search_threads(ora, obs, legal, tp, chunks=16, **kw):
    """ora.mcts_search over game chunks on host threads (ctypes drops the GIL);
    chunk c searches games [lo, hi) with game_offset + lo, as one call would."""
    G = obs.shape[0]
    off = kw.pop("game_offset", 0)
    bounds = np.linspace(0, G, chunks + 1).astype(int)

    def run(c):
        lo, hi = bounds[c], bounds[c + 1]
        return ora.mcts_search(obs[lo:hi], legal[lo:hi], tp[lo:hi], game_offset=off + int(lo), dump=True, **kw)

    with ThreadPoolExecutor(chunks) as ex:
        parts = list(ex.map(run, range(chunks)))
    cv = np.concatenate([p[0] for p in parts])
    rv = np.concatenate([p[1] for p in parts])
    act = np.concatenate([p[2] for p in parts])
    tree = {k: np.concatenate([p[3][k] for p in parts]) for k in parts[0][3]}
    stats = np.array([sum(p[4][0] for p in parts), max(p[4][1] for p in parts)])
    return cv, rv, act, tree, stats


def test_configs1_exact_launch_512x50(ttt, nets, monkeypatch):
    monkeypatch.delenv("MZ_SEARCH_KERNEL", raising=False)
    monkeypatch.delenv("MZ_SMALL_T", raising=False)
    G, S = 512, 50
    conf = dataclasses.replace(ttt.conf, num_iters=S)
    eng, ora = _engine(conf, ttt.hyper, nets, G, 77), _oracle(conf, ttt.hyper, nets, 77)
    obs, legal, tp = random_positions(G, 512)
    eng.debug_enable(1)
    cv, rv, act = eng.mcts_search(obs, legal, tp, exploration=True, rng_step=12, game_offset=4096, temperature=1.0)
    assert eng.search_variant() == "mz_search_small2"
    tree_g = eng.debug_tree(G)
    cv2, rv2, act2, tree_o, _ = _oracle_search_threads(ora, obs, legal, tp, exploration=True, rng_step=12,
                                                       game_offset=4096, temperature=1.0)
    _compare_trees(tree_g, tree_o, G)
    assert np.array_equal(cv, cv2) and np.array_equal(rv, rv2) and np.array_equal(act, act2)
    eng.close()


@pytest.mark.parametrize("explore,temp", [(True, 1.0), (False, 0.0)])
def test_configs4_200_sims_deep_tree(explore, temp):
    from muzero_jl_amd import abi
    from muzero_jl_amd.games import atari_synth as at
    G, S = 3, 200
    conf = dataclasses.replace(at.conf, num_iters=S)
    o, nets = _resnet_oracle(conf, at.resnet_hyper, seed=61)
    nets = _perturb_bn(conf, at.resnet_hyper, nets, seed=62)
    eng = abi.Engine(conf, at.resnet_hyper, device=0, max_games=G, rng_seed=o.seed)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    obs = at.observations(G, seed=63)
    legal = np.ones((G, 18), bool)                 # game 1: all 18 actions legal
    legal[0] = False
    legal[0, 5] = True                             # game 0: one legal action -> a chain, depth up to S - 1
    legal[2] = np.random.default_rng(64).random(18) < 0.5
    legal[2, 0] = True
    tp = np.ones(G, np.int32)
    eng.debug_enable(1)
    cv, rv, act = eng.mcts_search(obs, legal, tp, exploration=explore, rng_step=9, game_offset=40, temperature=temp)
    tree_g = eng.debug_tree(G)
    cv2, rv2, act2, tree_o, stats = _oracle_search_threads(o, obs, legal, tp, chunks=G, exploration=explore,
                                                           rng_step=9, game_offset=40, temperature=temp)
    assert stats[1] >= 129, f"max select depth {stats[1]}: the deep path was not exercised"
    _compare_trees(tree_g, tree_o, G)
    assert np.array_equal(cv, cv2) and np.array_equal(rv, rv2) and np.array_equal(act, act2)
    assert act[0] == 6
    eng.close()


def test_configs3_connect4_resnet8_learner():
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import cos_schedule
    from muzero_jl_amd.games import connect4
    from muzero_jl_amd.selfplay import random_positions as c4_positions
    B, K, A = 32, 5, 7
    conf = dataclasses.replace(connect4.conf, batch_size=B, num_unroll_steps=K)
    o, nets = _resnet_oracle(conf, connect4.resnet_hyper, seed=71)
    nets = _perturb_bn(conf, connect4.resnet_hyper, nets, seed=72)
    eng = abi.Engine(conf, connect4.resnet_hyper, device=0, max_games=8, rng_seed=1)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    st = o.learner_state()
    rng = np.random.default_rng(73)
    for t in range(1, 4):
        obs, _, _ = c4_positions(connect4.BatchedConnect4, B, seed=t, max_plies=14)
        tpol = rng.random((B, K + 1, A)).astype(np.float32)
        batch = dict(observation=obs, actions=rng.integers(1, A + 1, (B, K + 1)).astype(np.float32),
                     target_values=rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
                     target_rewards=rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
                     target_policies=tpol / tpol.sum(-1, keepdims=True),
                     gradient_scale=rng.integers(1, K + 1, B).astype(np.float32))
        eta = cos_schedule(t)
        with ThreadPoolExecutor(8) as ex:             # the oracle's unroll, 4 samples per thread
            parts = list(ex.map(lambda c: o.unroll(obs[4 * c: 4 * c + 4], batch["actions"][4 * c: 4 * c + 4]),
                                range(B // 4)))
        want = [np.concatenate([p[i] for p in parts]) for i in range(3)]
        lg = eng.learner_step(batch, eta)
        lo = o.learner_step(st, batch, eta)
        for g, w in zip(eng.debug_unroll(B), want):
            assert np.array_equal(g, w), f"step {t} unroll differs"
        assert np.array_equal(lg, lo), f"step {t} losses {lg} != oracle {lo}"
        for n in range(3):
            assert np.array_equal(eng.get_weights(n), o.params[n]), f"step {t} net {n} params differ"
    eng.close()
