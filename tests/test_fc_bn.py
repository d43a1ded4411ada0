"""FeedForwardHP(use_batch_norm = true): make_dense (src/Learning.jl:70-78) is
Chain(Dense(in, out), BatchNorm(out, relu)).  The reference's forward runs
outside the pullback (Q11), so BatchNorm is in test mode with the running
statistics it never updates (μ = 0, σ² = 1, ϵ = 1f-5): a fixed per-row affine
γ·((t − 0)/√(1 + ϵ)) + β before the relu, with β, γ after the Dense's W, b in
Flux.params.

CPU: the oracle's forward against torch fp32 (Linear, F.batch_norm in eval
mode, relu) at 1e-5, and the parameter layout (Python specs, oracle, the
checkpoint table).  GPU: the engine bit for bit against the oracle — the three
forwards, searches on the small and tile-16 kernels, learner steps (every
parameter including β and γ after ADAM) — and the corrected learner's
gradient through the BatchNorm layers against torch float64 autograd.
"""
import dataclasses

import numpy as np
import pytest

from conftest import random_positions


@pytest.fixture(scope="module")
def bn_hyper(ttt):
    return dataclasses.replace(ttt.hyper, use_batch_norm=True)


def _bn_nets(conf, hyper, seed=11):
    """init_nets, then β ~ U(-0.2, 0.2) and γ ~ U(0.5, 1.5) so that the BatchNorm affine matters."""
    from muzero_jl_amd.networks import init_nets, layer_specs
    nets = init_nets(conf, hyper, seed=seed)
    rng = np.random.default_rng(seed + 100)
    for net in range(3):
        off = 0
        for _, i, o, _, bn in layer_specs(conf, hyper, net, True):
            off += i * o + o
            if bn:
                nets[net][off:off + o] = rng.uniform(-0.2, 0.2, o).astype(np.float32)           # β
                nets[net][off + o:off + 2 * o] = rng.uniform(0.5, 1.5, o).astype(np.float32)    # γ
                off += 2 * o
        assert off == len(nets[net])
    return nets


def _torch_forward(conf, hyper, net, flat, x):
    import torch
    import torch.nn.functional as F
    from muzero_jl_amd.networks import unflatten
    layers = unflatten(conf, hyper, net, flat, with_bn=True)

    def chain(ch, v):
        for c, W, b, act, bg in layers:
            if c != ch:
                continue
            v = v @ torch.from_numpy(W.T.copy()) + torch.from_numpy(b.copy())
            if bg is not None:
                beta, gamma = (torch.from_numpy(a.copy()) for a in bg)
                v = F.batch_norm(v, torch.zeros(v.shape[1]), torch.ones(v.shape[1]), gamma, beta,
                                 training=False, eps=1e-5)
            v = torch.relu(v) if act == 1 else torch.tanh(v) if act == 2 else v
        return v

    t = chain(0, torch.from_numpy(x))
    if net == 0:
        return (t.numpy(),)
    o0, o1 = chain(1, t), chain(2, t)
    if net == 1:
        o1 = torch.softmax(o1, dim=1)
    return o0.numpy(), o1.numpy()


def _oracle(conf, hyper, nets, seed=5):
    from muzero_jl_amd.config import to_c_config, to_c_ffhp
    from oracle import Oracle
    o = Oracle(to_c_config(conf), to_c_ffhp(hyper), seed=seed)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
    return o


def test_bn_parameter_layout(ttt, bn_hyper):
    from muzero_jl_amd import checkpoint
    from muzero_jl_amd.networks import param_count
    ora = _oracle(ttt.conf, bn_hyper, _bn_nets(ttt.conf, bn_hyper))
    for net in range(3):
        n = param_count(ttt.conf, bn_hyper, net)
        assert ora.param_count(net) == n
        assert n == param_count(ttt.conf, ttt.hyper, net) + sum(
            2 * o for _, _, o, _, bn in __import__("muzero_jl_amd.networks", fromlist=["x"]).layer_specs(
                ttt.conf, bn_hyper, net, True) if bn)
        table = checkpoint.param_table(ttt.conf, bn_hyper, net)
        # representation: (W, b, β, γ) x 4 make_dense layers, then the output Dense's (W, b)
        if net == 0:
            shapes = [s for _, s, _ in table]
            assert shapes[:4] == [(64, 63), (64,), (64,), (64,)]
            assert shapes[-2:] == [(27, 64), (27,)]


@pytest.mark.parametrize("n", [1, 37])
def test_bn_oracle_forward_matches_torch(ttt, bn_hyper, n):
    nets = _bn_nets(ttt.conf, bn_hyper)
    ora = _oracle(ttt.conf, bn_hyper, nets)
    rng = np.random.default_rng(n)
    for net, feat in [(0, 63), (1, 27), (2, 36)]:
        x = rng.standard_normal((n, feat)).astype(np.float32)
        o = ora.forward(net, x)
        o = o if isinstance(o, tuple) else (o,)
        for oi, ti in zip(o, _torch_forward(ttt.conf, bn_hyper, net, nets[net], x)):
            np.testing.assert_allclose(oi, ti, rtol=1e-5, atol=1e-5)


def _engine(conf, hyper, nets, G, seed=5):
    from muzero_jl_amd.abi import Engine
    eng = Engine(conf, hyper, device=0, max_games=G, rng_seed=seed)
    for n, w in enumerate(nets):
        eng.set_weights(n, w)
    return eng


@pytest.mark.gpu
def test_bn_forward_bitexact(ttt, bn_hyper):
    nets = _bn_nets(ttt.conf, bn_hyper)
    eng, ora = _engine(ttt.conf, bn_hyper, nets, 16), _oracle(ttt.conf, bn_hyper, nets)
    rng = np.random.default_rng(3)
    for net, feat in [(0, 63), (1, 27), (2, 36)]:
        x = rng.standard_normal((37, feat)).astype(np.float32)
        g, o = eng.forward(net, x), ora.forward(net, x)
        g, o = (g if isinstance(g, tuple) else (g,)), (o if isinstance(o, tuple) else (o,))
        for gi, oi in zip(g, o):
            assert np.array_equal(gi, oi), f"net {net}: GPU != oracle (max {np.abs(gi - oi).max()})"
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [("tile16", None), ("small", "1"), ("small", "2")],
                         ids=["tile16", "small1", "small2"])
def test_bn_search_bitexact(ttt, bn_hyper, kernel, monkeypatch):
    from test_gpu_parity import _compare_trees
    fam, t = kernel
    monkeypatch.setenv("MZ_SEARCH_KERNEL", fam)
    if t:
        monkeypatch.setenv("MZ_SMALL_T", t)
    else:
        monkeypatch.delenv("MZ_SMALL_T", raising=False)
    conf = dataclasses.replace(ttt.conf, num_iters=25)
    nets = _bn_nets(conf, bn_hyper)
    G = 33
    eng, ora = _engine(conf, bn_hyper, nets, G, 4), _oracle(conf, bn_hyper, nets, 4)
    obs, legal, tp = random_positions(G, 4)
    eng.debug_enable(1)
    cv, rv, act = eng.mcts_search(obs, legal, tp, exploration=True, rng_step=7, game_offset=3)
    tree_g = eng.debug_tree(G)
    cv2, rv2, act2, tree_o, _ = ora.mcts_search(obs, legal, tp, exploration=True, rng_step=7, game_offset=3,
                                                dump=True)
    _compare_trees(tree_g, tree_o, G)
    assert np.array_equal(cv, cv2) and np.array_equal(rv, rv2) and np.array_equal(act, act2)
    eng.close()


@pytest.mark.gpu
def test_bn_learner_steps_bitexact(ttt, bn_hyper):
    from muzero_jl_amd.config import cos_schedule
    from test_gpu_parity import _random_batch
    B = 32
    conf = dataclasses.replace(ttt.conf, batch_size=B)
    nets = _bn_nets(conf, bn_hyper)
    eng, ora = _engine(conf, bn_hyper, nets, 16), _oracle(conf, bn_hyper, nets)
    st = ora.learner_state()
    rng = np.random.default_rng(B)
    for t in range(1, 7):
        batch = _random_batch(B, conf.num_unroll_steps, 9, rng)
        eta = cos_schedule(t)
        want = ora.unroll(batch["observation"], batch["actions"])
        lg = eng.learner_step(batch, eta)
        lo = ora.learner_step(st, batch, eta)
        for g, o in zip(eng.debug_unroll(B), want):
            assert np.array_equal(g, o), f"step {t} unroll differs"
        assert np.array_equal(lg, lo), f"step {t} losses {lg} != oracle {lo}"
        for n in range(3):                                   # β and γ too: ADAM on 2θ (Q11)
            assert np.array_equal(eng.get_weights(n), ora.params[n]), f"step {t} net {n} params differ"
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("B,K,ir,per", [(32, 5, True, False), (20, 3, False, True)])
def test_bn_corrected_gradient_matches_torch(ttt, bn_hyper, B, K, ir, per):
    """The corrected learner through the BatchNorm FC nets: the data gradient of
    every parameter (W, b, β, γ) of every net, the losses (Σθ² over β and γ
    too) and the read-outs against torch float64 autograd at 1e-5."""
    import torch
    from muzero_jl_amd import abi
    from test_corrected_learner_gpu import _batch
    from torch_learner_ref import corrected_loss_and_grads
    conf = dataclasses.replace(ttt.conf, batch_size=B, num_unroll_steps=K, intermediate_rewards=ir)
    nets = [n * np.float32(2.0) for n in _bn_nets(conf, bn_hyper, seed=B + K)]   # livelier activations
    eng = _engine(conf, bn_hyper, nets, 8)
    eng.learner_set_mode(abi.LEARN_CORRECTED)
    rng = np.random.default_rng(B)
    batch = _batch(B, K, 9, 63, rng)
    wts = (rng.random(B).astype(np.float32) * 0.9 + 0.1) if per else None
    dev = [torch.from_numpy(np.ascontiguousarray(batch[k])).cuda() for k in
           ("observation", "actions", "target_values", "target_rewards", "target_policies", "gradient_scale")]
    dev.append(torch.from_numpy(wts).cuda() if per else None)
    grad = torch.zeros(eng.grad_count(), dtype=torch.float32, device="cuda")
    losses = torch.zeros(8, dtype=torch.float32, device="cuda")
    eng.learner_grad_dev([t.data_ptr() if t is not None else None for t in dev], B, grad.data_ptr(),
                         losses.data_ptr())
    eng.sync()
    ref = corrected_loss_and_grads(conf, bn_hyper, nets, batch, wts)
    g = grad.cpu().numpy()
    off = 0
    for n in range(3):
        gn = g[off: off + nets[n].size].astype(np.float64)   # the data term (2θ: apply)
        rn = ref["grads"][n] - 2.0 * nets[n].astype(np.float64)
        off += nets[n].size
        scale = np.abs(rn).max()
        assert scale > 1e-4, f"net {n}: no data gradient reached it"
        err = np.abs(gn - rn).max() / scale
        assert err < 1e-5, f"net {n}: data gradient rel. error {err:.3g}"
    lo = losses.cpu().numpy()
    np.testing.assert_allclose([lo[0], lo[1], lo[2]], [ref["value"], ref["reward"], ref["policy"]],
                               rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(lo[3:6], ref["l2"], rtol=1e-5)
    pv, pp, pr = eng.debug_unroll(B)
    np.testing.assert_allclose(pv, ref["values"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(pp, ref["policies"], rtol=1e-5, atol=1e-6)
    if ir:
        np.testing.assert_allclose(pr, ref["rewards"], rtol=1e-5, atol=1e-6)
    eng.close()


@pytest.mark.gpu
def test_bn_fused_learner_matches_separate_calls(ttt, bn_hyper):
    """Device self-play with the BatchNorm nets fills a replay shard; the
    one-launch learner (sampling fused, ADAM scattering β / γ into the second
    image set's bias sections) equals mz_replay_sample + grad + apply (the
    images re-gathered from the parameters), bit for bit."""
    import torch
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import cos_schedule
    conf = dataclasses.replace(ttt.conf, num_iters=6, replay_buffer_size=64)
    nets = _bn_nets(conf, bn_hyper, seed=21)
    e1, e2 = (_engine(conf, bn_hyper, nets, 16, 5) for _ in range(2))
    for e in (e1, e2):
        e.selfplay_init(abi.ENV_TICTACTOE, 16, 64)
        for m in range(14):
            e.selfplay_move(100 + m, game_offset=7)
    assert e1.replay_counts()[0][0] > 0
    B = 32
    grad = torch.empty(e1.grad_count(), dtype=torch.float32, device="cuda")
    l1 = torch.empty(8, dtype=torch.float32, device="cuda")
    l2 = torch.empty(8, dtype=torch.float32, device="cuda")
    for step in (1, 2, 3):
        eta = cos_schedule(step)
        b, _ = e1.replay_sample(B, step)
        e1.learner_grad_dev([b.observation, b.actions, b.target_values, b.target_rewards, b.target_policies,
                             b.gradient_scale], B, grad.data_ptr(), l1.data_ptr())
        e1.learner_apply_dev(grad.data_ptr(), 1.0, eta)
        e2.learner_train_dev(B, step, eta, l2.data_ptr())
        e1.sync(); e2.sync()
        assert np.array_equal(l1.cpu().numpy()[:6], l2.cpu().numpy()[:6]), step
        for n in range(3):
            assert np.array_equal(e1.get_weights(n), e2.get_weights(n)), (step, n)
    # the searches that follow read the updated images (the fused set and the repacked set agree)
    obs, legal, tp = random_positions(16, 2)
    assert all(np.array_equal(a, b) for a, b in zip(e1.mcts_search(obs, legal, tp, rng_step=3),
                                                    e2.mcts_search(obs, legal, tp, rng_step=3)))
    e1.close(); e2.close()
