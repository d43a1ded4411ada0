"""GPU parity of BASELINE configs[4] (synthetic 84x84x4 observations, the
ResNet representation's downsampler of Learning.jl:175-187, 6x6 hidden board,
18 actions, one player) through the C ABI against the CPU oracle, bit for
bit: the downsampler + representation tail, prediction / dynamics, whole
searches on 32-lane select groups (A = 18 > 16), and learner steps.  The
oracle's downsampler is pinned against torch fp32 at 1e-5 in
test_resnet_oracle.py."""
import dataclasses

import numpy as np
import pytest

from test_resnet_oracle import _perturb_bn, _resnet_oracle, _torch_forward

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def at_eng():
    from muzero_jl_amd import abi
    from muzero_jl_amd.games import atari_synth as at
    conf, hyper = dataclasses.replace(at.conf, num_iters=4), at.resnet_hyper
    o, nets = _resnet_oracle(conf, hyper, seed=31)
    nets = _perturb_bn(conf, hyper, nets, seed=32)
    eng = abi.Engine(conf, hyper, device=0, max_games=16, rng_seed=3)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    yield conf, hyper, o, eng, nets
    eng.close()


@pytest.mark.parametrize("net", [0, 1, 2])
def test_atari_forward_bitexact(at_eng, net):
    from muzero_jl_amd.games import atari_synth as at
    conf, hyper, o, eng, nets = at_eng
    rng = np.random.default_rng(net)
    n = 5
    if net == 0:
        x = at.observations(n, seed=net + 1)
    elif net == 1:
        x = rng.normal(0, 1, (n, o.H)).astype(np.float32)
    else:
        x = np.concatenate([rng.normal(0, 1, (n, o.H)), np.full((n, 36), 7 / 18)], 1).astype(np.float32)
    want, got = o.forward(net, x), eng.forward(net, x)
    if net == 0:
        assert np.array_equal(got, want)
        np.testing.assert_allclose(got, _torch_forward(conf, hyper, net, nets[net], x), rtol=1e-5, atol=1e-5)
    else:
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


def test_atari_param_table(at_eng):
    """The engine's Flux.params table (checkpoints) lists the downsampler's
    arrays first, MeanPool contributing none, matching checkpoint.param_table."""
    from muzero_jl_amd.checkpoint import param_table
    conf, hyper, o, eng, nets = at_eng
    for n in range(3):
        assert eng.param_count(n) == o.param_count(n) == nets[n].size
    t = param_table(conf, hyper, 0)
    assert t[0][1] == (3, 3, 4, 4) and t[1][1] == (4,) and t[2][1] == (3, 3, 4, 4)


@pytest.mark.parametrize("S,G,explore,temp,seed", [(3, 5, True, 1.0, 1), (12, 9, False, 0.0, 2),
                                                   (8, 16, True, float("inf"), 3)])
def test_atari_search_bitexact(S, G, explore, temp, seed):
    from muzero_jl_amd import abi
    from muzero_jl_amd.games import atari_synth as at
    from test_gpu_parity import _compare_trees
    conf = dataclasses.replace(at.conf, num_iters=S)
    o, nets = _resnet_oracle(conf, at.resnet_hyper, seed=seed)
    nets = _perturb_bn(conf, at.resnet_hyper, nets, seed=seed)
    eng = abi.Engine(conf, at.resnet_hyper, device=0, max_games=G, rng_seed=o.seed)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    obs = at.observations(G, seed=seed)
    rng = np.random.default_rng(seed)
    legal = rng.random((G, 18)) < 0.8
    legal[:, 17] = True
    legal[0] = False
    legal[0, 16] = True                          # a single legal action
    tp = np.ones(G, np.int32)
    eng.debug_enable(1)
    cv, rv, act = eng.mcts_search(obs, legal, tp, exploration=explore, rng_step=seed, game_offset=3,
                                  temperature=temp)
    tree_g = eng.debug_tree(G)
    cv2, rv2, act2, tree_o, _ = o.mcts_search(obs, legal, tp, exploration=explore, rng_step=seed, game_offset=3,
                                              temperature=temp, dump=True)
    assert np.all(legal[np.arange(G), act - 1])
    _compare_trees(tree_g, tree_o, G)
    assert np.array_equal(cv, cv2) and np.array_equal(rv, rv2) and np.array_equal(act, act2)
    eng.close()


def test_atari_learner_steps():
    """Unroll (downsampler + tail, then K x (prediction, dynamics)) bit-exact
    vs ora_unroll, the 32-lane loss groups, ∇ = 2θ and ADAM: parameters
    bit-exact, downsampler parameters included."""
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import cos_schedule
    from muzero_jl_amd.games import atari_synth as at
    B, K = 6, 2
    conf = dataclasses.replace(at.conf, batch_size=B, num_unroll_steps=K, num_iters=2)
    o, nets = _resnet_oracle(conf, at.resnet_hyper, seed=41)
    nets = _perturb_bn(conf, at.resnet_hyper, nets, seed=42)
    eng = abi.Engine(conf, at.resnet_hyper, device=0, max_games=4, rng_seed=1)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
        eng.set_weights(n, w)
    st = o.learner_state()
    rng = np.random.default_rng(5)
    for t in range(1, 4):
        tpol = rng.random((B, K + 1, 18)).astype(np.float32)
        batch = dict(observation=at.observations(B, seed=t), actions=rng.integers(1, 19, (B, K + 1)).astype(np.float32),
                     target_values=rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
                     target_rewards=rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
                     target_policies=tpol / tpol.sum(-1, keepdims=True),
                     gradient_scale=rng.integers(1, K + 1, B).astype(np.float32))
        eta = cos_schedule(t)
        want = o.unroll(batch["observation"], batch["actions"])
        lg = eng.learner_step(batch, eta)
        lo = o.learner_step(st, batch, eta)
        for g, w in zip(eng.debug_unroll(B), want):
            assert np.array_equal(g, w), f"step {t} unroll differs"
        assert np.array_equal(lg, lo), f"step {t} losses {lg} != oracle {lo}"   # same fold order: bit-exact
        for n in range(3):
            assert np.array_equal(eng.get_weights(n), o.params[n]), f"step {t} net {n} params differ"
    eng.close()


def test_atari_slots_before_first_move(at_eng):
    """The Atari-like env keys its initial games by the first move's
    game_offset, so the slots hold no games between mz_selfplay_init and the
    first mz_selfplay_move: mz_selfplay_slots fails there instead of
    returning zeroed slots, and works after the move."""
    from muzero_jl_amd import abi
    conf, hyper, o, eng, nets = at_eng
    eng.selfplay_init(abi.ENV_ATARI, 4, 8)
    with pytest.raises(abi.MzError, match="first mz_selfplay_move"):
        eng.selfplay_slots()
    eng.selfplay_move(0, game_offset=3)
    ln, board, player = eng.selfplay_slots()
    assert np.all(player == 1) and np.all(ln == 1)
