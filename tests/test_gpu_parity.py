"""GPU parity tests: libmz (HIP, gfx950) through the C ABI vs the CPU oracle.

Bars: network tensors bit-exact vs the oracle's canonical order
and within 1e-5 of torch-CPU fp32; tree statistics, visit counts, root values
and chosen actions bit-exact under the same Philox streams; learner parameters
bit-exact after N ref_semantics steps, losses bit-exact (the oracle restates
the engine's deterministic loss fold, oracle/mz_oracle.c ora_losses_w).
"""
import dataclasses

import numpy as np
import pytest

from conftest import random_positions

pytestmark = pytest.mark.gpu


def _engine(conf, hyper, nets, G, seed=5):
    from muzero_jl_amd.abi import Engine
    eng = Engine(conf, hyper, device=0, max_games=G, rng_seed=seed)
    for n, w in enumerate(nets):
        eng.set_weights(n, w)
    return eng


def _oracle(conf, hyper, nets, seed=5):
    from muzero_jl_amd.config import to_c_config, to_c_ffhp
    from oracle import Oracle
    o = Oracle(to_c_config(conf), to_c_ffhp(hyper), seed=seed)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
    return o


def _torch_forward(conf, hyper, net, flat, x):
    import torch
    from muzero_jl_amd.networks import unflatten
    layers = unflatten(conf, hyper, net, flat)

    def chain(ch, v):
        for c, W, b, act in layers:
            if c != ch:
                continue
            v = v @ torch.from_numpy(W.T.copy()) + torch.from_numpy(b.copy())
            v = torch.relu(v) if act == 1 else torch.tanh(v) if act == 2 else v
        return v

    t = chain(0, torch.from_numpy(x))
    if net == 0:
        return t.numpy()
    o0, o1 = chain(1, t), chain(2, t)
    if net == 1:
        o1 = torch.softmax(o1, dim=1)
    return o0.numpy(), o1.numpy()


@pytest.mark.parametrize("n", [1, 16, 37, 256])
def test_net_forward_bitexact(ttt, nets, n):
    conf, hyper = ttt.conf, ttt.hyper
    eng, ora = _engine(conf, hyper, nets, 16), _oracle(conf, hyper, nets)
    rng = np.random.default_rng(n)
    for net, feat in [(0, 63), (1, 27), (2, 36)]:
        x = rng.standard_normal((n, feat)).astype(np.float32)
        g, o = eng.forward(net, x), ora.forward(net, x)
        t = _torch_forward(conf, hyper, net, nets[net], x)
        if net == 0:
            g, o, t = (g,), (o,), (t,)
        for gi, oi, ti in zip(g, o, t):
            assert np.array_equal(gi, oi), f"net {net}: GPU != oracle (max {np.abs(gi - oi).max()})"
            np.testing.assert_allclose(gi, ti, rtol=1e-5, atol=1e-5)
    eng.close()


def _compare_trees(tg, to, G):
    for k in ("N", "W", "P", "R", "C"):
        a, b = tg[k][:G], to[k][:G]
        if k == "C":
            assert np.array_equal(a, b), "child slots differ"
        else:
            assert np.array_equal(a, b), f"tree {k} differs at {np.argwhere(a != b)[:5]}"


KERNELS = [("tile16", None), ("small", "1"), ("small", "2"), ("small", "4")]


def _force(monkeypatch, kernel):
    fam, t = kernel
    monkeypatch.setenv("MZ_SEARCH_KERNEL", fam)
    if t:
        monkeypatch.setenv("MZ_SMALL_T", t)
    else:
        monkeypatch.delenv("MZ_SMALL_T", raising=False)


@pytest.mark.parametrize("kernel", KERNELS, ids=["tile16", "small1", "small2", "small4"])
@pytest.mark.parametrize("S,G,explore,temp,seed", [
    (1, 16, True, 1.0, 1), (10, 16, True, 1.0, 2), (25, 33, True, 1.0, 3),
    (50, 64, True, 1.0, 4), (50, 20, False, 0.0, 5), (12, 48, True, float("inf"), 6),
    (12, 17, True, 0.5, 7), (100, 16, True, 1.0, 8)])
def test_search_bitexact(ttt, nets, S, G, explore, temp, seed, kernel, monkeypatch):
    _force(monkeypatch, kernel)
    conf = dataclasses.replace(ttt.conf, num_iters=S)
    eng, ora = _engine(conf, ttt.hyper, nets, G, seed), _oracle(conf, ttt.hyper, nets, seed)
    obs, legal, tp = random_positions(G, seed)
    eng.debug_enable(1)
    cv, rv, act = eng.mcts_search(obs, legal, tp, exploration=explore, rng_step=seed * 3, game_offset=100,
                                  temperature=temp)
    tree_g = eng.debug_tree(G)
    if kernel[0] == "small" and S <= 50:             # (the kernel the case is for, not a silent fallback)
        assert eng.search_variant().startswith("mz_search_small"), eng.search_variant()
    cv2, rv2, act2, tree_o, _ = ora.mcts_search(obs, legal, tp, exploration=explore, rng_step=seed * 3,
                                                game_offset=100, temperature=temp, dump=True)
    _compare_trees(tree_g, tree_o, G)
    assert np.array_equal(cv, cv2)
    assert np.array_equal(rv, rv2)
    assert np.array_equal(act, act2)
    assert np.all(legal[np.arange(G), act - 1])
    np.testing.assert_allclose(cv.sum(1), 1.0, rtol=1e-6)
    eng.close()


@pytest.mark.parametrize("kernel", KERNELS, ids=["tile16", "small1", "small2", "small4"])
def test_search_single_legal_and_one_player(ttt, nets, kernel, monkeypatch):
    _force(monkeypatch, kernel)
    conf = dataclasses.replace(ttt.conf, num_iters=20, players=[1])
    G = 24
    eng, ora = _engine(conf, ttt.hyper, nets, G, 9), _oracle(conf, ttt.hyper, nets, 9)
    obs, legal, tp = random_positions(G, 9)
    legal[:8] = False
    legal[np.arange(8), np.arange(8)] = True            # exactly one legal action
    tp[:] = 1
    out_g = eng.mcts_search(obs, legal, tp, exploration=True, rng_step=1)
    out_o = ora.mcts_search(obs, legal, tp, exploration=True, rng_step=1)
    for a, b in zip(out_g, out_o):
        assert np.array_equal(a, b)
    assert np.array_equal(out_g[2][:8], np.arange(1, 9))
    eng.close()


def test_search_rejects_empty_legal(ttt, nets):
    from muzero_jl_amd.abi import MzError
    eng = _engine(ttt.conf, ttt.hyper, nets, 4)
    obs, legal, tp = random_positions(4, 1)
    legal[2] = False
    with pytest.raises(MzError, match="Legal actions should not be an empty array"):
        eng.mcts_search(obs, legal, tp)
    with pytest.raises(MzError, match="max_games"):
        eng.mcts_search(*random_positions(5, 1))
    eng.close()


def _random_batch(B, K, A, rng):
    obs = (rng.random((B, 63)) < 0.4).astype(np.float32)
    acts = rng.integers(1, A + 1, (B, K + 1)).astype(np.float32)
    tv = rng.uniform(-1, 1, (B, K + 1)).astype(np.float32)
    tr = rng.uniform(-1, 1, (B, K + 1)).astype(np.float32)
    tpol = rng.random((B, K + 1, A)).astype(np.float32)
    tpol /= tpol.sum(-1, keepdims=True)
    gs = rng.integers(1, max(K, 1) + 1, B).astype(np.float32)
    return dict(observation=obs, actions=acts, target_values=tv, target_rewards=tr, target_policies=tpol,
                gradient_scale=gs)


@pytest.mark.parametrize("B", [32, 45])
def test_learner_steps_bitexact(ttt, nets, B):
    from muzero_jl_amd.config import cos_schedule
    conf = dataclasses.replace(ttt.conf, batch_size=B)
    eng, ora = _engine(conf, ttt.hyper, nets, 16), _oracle(conf, ttt.hyper, nets)
    st = ora.learner_state()
    rng = np.random.default_rng(B)
    for t in range(1, 13):
        batch = _random_batch(B, conf.num_unroll_steps, 9, rng)
        eta = cos_schedule(t)
        want = ora.unroll(batch["observation"], batch["actions"])
        lg = eng.learner_step(batch, eta)
        lo = ora.learner_step(st, batch, eta)
        for g, o in zip(eng.debug_unroll(B), want):          # the unroll's read-outs, bit for bit
            assert np.array_equal(g, o), f"step {t} unroll differs"
        assert np.array_equal(lg, lo), f"step {t} losses {lg} != oracle {lo}"   # same fold order: bit-exact
        for n in range(3):
            assert np.array_equal(eng.get_weights(n), ora.params[n]), f"step {t} net {n} params differ"
    eng.close()


@pytest.mark.parametrize("S,G", [(50, 40), (100, 20)])
def test_search_bitexact_nonresident_kernel(ttt, nets, S, G, monkeypatch):
    """The generic (weights streamed from L2) plan executor must agree with the
    register-resident one and the oracle."""
    monkeypatch.setenv("MZ_NO_RESIDENT", "1")
    monkeypatch.setenv("MZ_SEARCH_KERNEL", "tile16")
    conf = dataclasses.replace(ttt.conf, num_iters=S)
    eng, ora = _engine(conf, ttt.hyper, nets, G, 21), _oracle(conf, ttt.hyper, nets, 21)
    obs, legal, tp = random_positions(G, 21)
    out_g = eng.mcts_search(obs, legal, tp, rng_step=2)
    out_o = ora.mcts_search(obs, legal, tp, rng_step=2)
    for a, b in zip(out_g, out_o):
        assert np.array_equal(a, b)
    eng.close()


def test_search_auto_dispatch_large_batches(ttt, nets, monkeypatch):
    """G = 512 (the benchmark batch) picks the 2-games-per-CU small kernel and
    G = 1536 the 16-game tile kernel; both bit-exact vs the oracle."""
    monkeypatch.delenv("MZ_SEARCH_KERNEL", raising=False)
    monkeypatch.delenv("MZ_SMALL_T", raising=False)
    conf = dataclasses.replace(ttt.conf, num_iters=12)
    for G, fam in [(512, "mz_search_small2"), (1536, "mz_search_kernel")]:
        eng, ora = _engine(conf, ttt.hyper, nets, G, 33), _oracle(conf, ttt.hyper, nets, 33)
        obs, legal, tp = random_positions(G, 40 + G)
        out_g = eng.mcts_search(obs, legal, tp, rng_step=3)
        assert eng.search_variant().startswith(fam), eng.search_variant()
        out_o = ora.mcts_search(obs, legal, tp, rng_step=3)
        for a, b in zip(out_g, out_o):
            assert np.array_equal(a, b)
        eng.close()
