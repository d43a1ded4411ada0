"""GPU parity of the ResNet networks (row a14) through the C ABI: the MFMA
kernels against the CPU oracle, bit for bit (same canonical dot order,
BatchNorm and softmax sequences), plus the torch fp32 pin at 1e-5."""
import numpy as np
import pytest

from test_resnet_oracle import _perturb_bn, _resnet_oracle, _torch_forward

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rn(ttt):
    from muzero_jl_amd import abi
    conf, hyper = ttt.conf, ttt.resnet_hyper
    o, nets = _resnet_oracle(conf, hyper, seed=9)
    nets = _perturb_bn(conf, hyper, nets, seed=4)
    eng = abi.Engine(conf, hyper, device=0, max_games=64, rng_seed=3)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    yield conf, hyper, o, eng, nets
    eng.close()


def _inputs(o, net, n, seed):
    rng = np.random.default_rng(seed)
    if net == 0:
        return (rng.random((n, 63)) < 0.4).astype(np.float32)
    if net == 1:
        return rng.normal(0, 1, (n, o.H)).astype(np.float32)
    return np.concatenate([rng.normal(0, 1, (n, o.H)), np.full((n, 9), 2 / 9)], 1).astype(np.float32)


@pytest.mark.parametrize("net", [0, 1, 2])
@pytest.mark.parametrize("n", [1, 7, 33])
def test_resnet_forward_bitexact(rn, net, n):
    conf, hyper, o, eng, nets = rn
    x = _inputs(o, net, n, 100 * net + n)
    want = o.forward(net, x)
    got = eng.forward(net, x)
    if net == 0:
        assert np.array_equal(got, want)
        np.testing.assert_allclose(got, _torch_forward(conf, hyper, net, nets[net], x), rtol=1e-5, atol=1e-5)
    else:
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


@pytest.mark.parametrize("S,G,explore,temp,seed", [
    (1, 5, True, 1.0, 1), (8, 20, True, 1.0, 2), (16, 33, False, 0.0, 3), (12, 17, True, float("inf"), 4),
    (25, 40, True, 0.5, 5)])
def test_resnet_search_bitexact(ttt, S, G, explore, temp, seed):
    """Batched search with the ResNet nets (root launch, S x (tree step,
    networks), final step) against the oracle: trees, visits, values, actions."""
    import dataclasses
    from conftest import random_positions
    from muzero_jl_amd import abi
    from test_gpu_parity import _compare_trees
    conf = dataclasses.replace(ttt.conf, num_iters=S)
    o, nets = _resnet_oracle(conf, ttt.resnet_hyper, seed=seed)
    nets = _perturb_bn(conf, ttt.resnet_hyper, nets, seed=seed)
    eng = abi.Engine(conf, ttt.resnet_hyper, device=0, max_games=G, rng_seed=o.seed)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    obs, legal, tp = random_positions(G, 40 + seed)
    eng.debug_enable(1)
    cv, rv, act = eng.mcts_search(obs, legal, tp, exploration=explore, rng_step=seed * 7, game_offset=11,
                                  temperature=temp)
    assert eng.search_variant() == "mz_rsearch"
    tree_g = eng.debug_tree(G)
    cv2, rv2, act2, tree_o, _ = o.mcts_search(obs, legal, tp, exploration=explore, rng_step=seed * 7,
                                              game_offset=11, temperature=temp, dump=True)
    _compare_trees(tree_g, tree_o, G)
    assert np.array_equal(cv, cv2) and np.array_equal(rv, rv2) and np.array_equal(act, act2)
    eng.close()


def test_resnet_search_hbm_tree_bitexact(ttt, monkeypatch):
    """The tree step on the HBM tree (`mz_rsearch_tree`, used when a game's tree
    exceeds the LDS; MZ_RTREE_HBM=1 at create forces it), with the parent's h by
    reference (use counts, 2^k in the network launch)."""
    import dataclasses
    from conftest import random_positions
    from muzero_jl_amd import abi
    from test_gpu_parity import _compare_trees
    monkeypatch.setenv("MZ_RTREE_HBM", "1")
    S, G, seed = 20, 24, 6
    conf = dataclasses.replace(ttt.conf, num_iters=S)
    o, nets = _resnet_oracle(conf, ttt.resnet_hyper, seed=seed)
    eng = abi.Engine(conf, ttt.resnet_hyper, device=0, max_games=G, rng_seed=o.seed)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    obs, legal, tp = random_positions(G, 60)
    eng.debug_enable(1)
    cv, rv, act = eng.mcts_search(obs, legal, tp, exploration=True, rng_step=5, game_offset=3, temperature=1.0)
    tree_g = eng.debug_tree(G)
    cv2, rv2, act2, tree_o, _ = o.mcts_search(obs, legal, tp, exploration=True, rng_step=5, game_offset=3,
                                              temperature=1.0, dump=True)
    _compare_trees(tree_g, tree_o, G)
    assert np.array_equal(cv, cv2) and np.array_equal(rv, rv2) and np.array_equal(act, act2)
    eng.close()


@pytest.mark.parametrize("B,K", [(20, 5), (33, 3), (7, 0), (832, 5)])
def test_resnet_learner_steps(ttt, B, K):
    """ResNet learner (unroll on the network kernels + the shared loss/∇ = 2θ
    kernel + ADAM): the unroll's read-outs bit-exact against ora_unroll, the
    losses within the f64 cross-sample tolerance, parameters bit-exact.
    B = 832: B·K / 16 >= #CUs, so the predictions run on the wide 16-item tiles
    (mz_runroll_pred) instead of one-item tiles; one step (the oracle is slow)."""
    import dataclasses
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import cos_schedule
    from test_gpu_parity import _random_batch
    conf = dataclasses.replace(ttt.conf, batch_size=B, num_unroll_steps=K)
    o, nets = _resnet_oracle(conf, ttt.resnet_hyper, seed=B)
    nets = _perturb_bn(conf, ttt.resnet_hyper, nets, seed=K)
    eng = abi.Engine(conf, ttt.resnet_hyper, device=0, max_games=8, rng_seed=1)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    st = o.learner_state()
    rng = np.random.default_rng(B + K)
    for t in range(1, 5 if B < 100 else 2):
        batch = _random_batch(B, K, 9, rng)
        eta = cos_schedule(t)
        want = o.unroll(batch["observation"], batch["actions"])
        lg = eng.learner_step(batch, eta)
        lo = o.learner_step(st, batch, eta)
        if B >= 100:
            assert eng.learner_variant().endswith("+mz_runroll_pred"), eng.learner_variant()
        for g, w in zip(eng.debug_unroll(B), want):
            assert np.array_equal(g, w), f"step {t} unroll differs"
        assert np.array_equal(lg, lo), f"step {t} losses {lg} != oracle {lo}"   # same fold order: bit-exact
        for n in range(3):
            assert np.array_equal(eng.get_weights(n), o.params[n]), f"step {t} net {n} params differ"
    eng.close()


@pytest.fixture(scope="module")
def rn_c4():
    """Connect4 ResNet-8 (configs[3]): a 6x7 board, tiles of 4 games."""
    from muzero_jl_amd import abi
    from muzero_jl_amd.games import connect4
    conf, hyper = connect4.conf, connect4.resnet_hyper
    o, nets = _resnet_oracle(conf, hyper, seed=21)
    nets = _perturb_bn(conf, hyper, nets, seed=22)
    eng = abi.Engine(conf, hyper, device=0, max_games=32, rng_seed=3)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    yield conf, hyper, o, eng
    eng.close()


@pytest.mark.parametrize("net", [0, 1, 2])
def test_resnet_connect4_forward_bitexact(rn_c4, net):
    conf, hyper, o, eng = rn_c4
    rng = np.random.default_rng(net)
    n = 9
    if net == 0:
        x = (rng.random((n, 294)) < 0.4).astype(np.float32)
    elif net == 1:
        x = rng.normal(0, 1, (n, o.H)).astype(np.float32)
    else:
        x = np.concatenate([rng.normal(0, 1, (n, o.H)), np.full((n, 42), 3 / 7)], 1).astype(np.float32)
    want, got = o.forward(net, x), eng.forward(net, x)
    if net == 0:
        assert np.array_equal(got, want)
    else:
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


def test_resnet_connect4_search_bitexact():
    import dataclasses
    from muzero_jl_amd import abi
    from muzero_jl_amd.games import connect4
    from muzero_jl_amd.selfplay import random_positions
    from test_gpu_parity import _compare_trees
    conf = dataclasses.replace(connect4.conf, num_iters=6)
    hyper = connect4.resnet_hyper
    o, nets = _resnet_oracle(conf, hyper, seed=23)
    G = 9
    eng = abi.Engine(conf, hyper, device=0, max_games=G, rng_seed=o.seed)
    for n, w in enumerate(nets):
        eng.set_weights(n, w)
    obs, legal, tp = random_positions(connect4.BatchedConnect4, G, seed=5, max_plies=12)
    eng.debug_enable(1)
    cv, rv, act = eng.mcts_search(obs, legal, tp, exploration=True, rng_step=3, game_offset=0, temperature=1.0)
    tree_g = eng.debug_tree(G)
    cv2, rv2, act2, tree_o, _ = o.mcts_search(obs, legal, tp, exploration=True, rng_step=3, game_offset=0,
                                              temperature=1.0, dump=True)
    assert np.all(legal[np.arange(G), act - 1])
    _compare_trees(tree_g, tree_o, G)
    assert np.array_equal(cv, cv2) and np.array_equal(rv, rv2) and np.array_equal(act, act2)
    eng.close()
