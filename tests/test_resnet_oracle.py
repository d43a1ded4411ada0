"""CPU tests of the ResNet networks (row a14: Learning.jl:148-255, the intended
architecture of SURVEY §2.1 Q12 / DESIGN.md §9).  The reference's ResNet
path cannot run, so the specification is pinned here against an independent
torch fp32 implementation (convolution = cross-correlation with the kernel
flipped, BatchNorm in test mode with μ=0, σ²=1, ε=1e-5, residual blocks,
column-major (W,H,C) flatten) at the 1e-5 tolerance of north_star, and the
oracle's search on ResNet nets against the independent Python mirror."""
import dataclasses

import numpy as np
import pytest

from conftest import random_positions

TOL = dict(rtol=1e-5, atol=1e-5)


def _resnet_oracle(conf, hyper, seed=7):
    from muzero_jl_amd.config import to_c_config, to_c_resnet_hp
    from muzero_jl_amd.networks import init_nets
    from oracle import Oracle
    o = Oracle(to_c_config(conf), to_c_resnet_hp(hyper), seed=seed)
    nets = init_nets(conf, hyper, seed=seed)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
    return o, nets


def _perturb_bn(conf, hyper, nets, seed=1):
    """β, γ away from (0, 1) so the BatchNorm terms are exercised."""
    from muzero_jl_amd.networks import resnet_specs
    rng = np.random.default_rng(seed)
    out = []
    for n, flat in enumerate(nets):
        flat = flat.copy()
        off = 0
        for op in resnet_specs(conf, hyper, n):
            if op["kind"] == "pool":
                continue
            if op["kind"] == "dense":
                off += op["cin"] * op["cout"] + op["cout"]
                continue
            off += op["kw"] * op["kh"] * op["cin"] * op["cout"]
            flat[off: off + op["cout"]] = rng.normal(0, 0.1, op["cout"]).astype(np.float32)        # bias
            off += op["cout"]
            if not op["bn"]:
                continue
            flat[off: off + op["cout"]] = rng.normal(0, 0.1, op["cout"]).astype(np.float32)        # β
            flat[off + op["cout"]: off + 2 * op["cout"]] = rng.uniform(0.5, 1.5, op["cout"]).astype(np.float32)
            off += 2 * op["cout"]
        out.append(flat)
    return out


def _torch_forward(conf, hyper, net, flat, x):
    """Independent fp32 forward of one net for a batch x (n, features)."""
    import torch
    import torch.nn.functional as F
    from muzero_jl_amd.config import ACT_RELU, ACT_TANH
    from muzero_jl_amd.networks import unflatten_resnet
    ops = unflatten_resnet(conf, hyper, net, flat)

    def act(t, a):
        return torch.relu(t) if a == ACT_RELU else torch.tanh(t) if a == ACT_TANH else t

    def chain(t, ch):
        res = None
        for op in [o for o in ops if o["chain"] == ch]:
            if op["kind"] == "pool":                   # MeanPool((3,3), stride 2, pad 1), padding counted
                t = F.avg_pool2d(t, 3, stride=2, padding=1, count_include_pad=True)
            elif op["kind"] == "conv":
                if t.dim() == 2:                       # (n, W*H*C) column-major -> (n, C, H, W)
                    t = t.reshape(t.shape[0], op["cin"], op["Hi"], op["Wi"])
                if op["res_save"]:
                    res = t
                w = torch.flip(torch.from_numpy(np.ascontiguousarray(op["w"])), dims=[2, 3])
                y = F.conv2d(t, w, torch.from_numpy(op["b"].copy()), stride=op["stride"],
                             padding=(op["kh"] // 2, op["kw"] // 2))
                if op["bn"]:
                    y = F.batch_norm(y, torch.zeros(op["cout"]), torch.ones(op["cout"]),
                                     torch.from_numpy(op["gamma"].copy()), torch.from_numpy(op["beta"].copy()),
                                     training=False, eps=1e-5)
                if op["res_add"]:
                    y = y + res
                t = act(y, op["act"])
            else:
                t = t.reshape(t.shape[0], -1)          # Flux.flatten of (W,H,C): C-order (C,H,W)
                y = t @ torch.from_numpy(np.ascontiguousarray(op["w"])).T + torch.from_numpy(op["b"].copy())
                t = act(y, op["act"])
        return t

    xt = torch.from_numpy(np.ascontiguousarray(x, np.float32))
    trunk = chain(xt, 0)
    if net == 0:
        return trunk.reshape(trunk.shape[0], -1).numpy()
    h1, h2 = chain(trunk, 1), chain(trunk, 2)
    if net == 1:
        return h1.numpy(), torch.softmax(h2, dim=1).numpy()
    return h1.reshape(h1.shape[0], -1).numpy(), h2.numpy()


def test_resnet_param_counts(ttt):
    from muzero_jl_amd.networks import param_count
    o, _ = _resnet_oracle(ttt.conf, ttt.resnet_hyper)
    counts = [param_count(ttt.conf, ttt.resnet_hyper, n) for n in range(3)]
    assert counts == [o.param_count(n) for n in range(3)]
    assert counts == [152448, 32467, 47876]


@pytest.mark.parametrize("net", [0, 1, 2])
def test_resnet_oracle_matches_torch(ttt, net):
    conf, hyper = ttt.conf, ttt.resnet_hyper
    o, nets = _resnet_oracle(conf, hyper)
    nets = _perturb_bn(conf, hyper, nets)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
    rng = np.random.default_rng(net)
    n = 5
    if net == 0:
        x = (rng.random((n, 63)) < 0.4).astype(np.float32)
    elif net == 1:
        x = rng.normal(0, 1, (n, o.H)).astype(np.float32)
    else:
        x = np.concatenate([rng.normal(0, 1, (n, o.H)), np.full((n, 9), 4 / 9)], 1).astype(np.float32)
    ref = _torch_forward(conf, hyper, net, nets[net], x)
    got = o.forward(net, x)
    if net == 0:
        np.testing.assert_allclose(got, ref, **TOL)
    else:
        np.testing.assert_allclose(got[0], ref[0], **TOL)
        np.testing.assert_allclose(got[1], ref[1], **TOL)


def test_resnet_oracle_search_matches_mirror(ttt):
    from mirror_ref import Mirror
    conf = dataclasses.replace(ttt.conf, num_iters=8)
    o, _ = _resnet_oracle(conf, ttt.resnet_hyper, seed=3)
    obs, legal, tp = random_positions(3, 17)
    cv, rv, act, _, _ = o.mcts_search(obs, legal, tp, exploration=True, rng_step=2, game_offset=5, dump=True)
    cv2, rv2, act2, _ = Mirror(o, conf).search(obs, legal, tp, True, 5, 2)
    assert np.array_equal(cv, cv2) and np.array_equal(rv, rv2) and np.array_equal(act, act2)


def test_downsample_param_counts_and_board():
    """configs[4]: the downsampler of Learning.jl:175-187 takes 84x84x4 to 6x6x8."""
    from muzero_jl_amd.games import atari_synth as at
    from muzero_jl_amd.networks import param_count, resnet_board, resnet_specs
    assert resnet_board(at.conf, at.resnet_hyper) == (6, 6)
    ops = resnet_specs(at.conf, at.resnet_hyper, 0)
    assert [(o["Wi"], o["W"]) for o in ops if o["kind"] != "dense" and o["stride"] == 2] == \
        [(84, 42), (42, 21), (21, 11), (11, 6)]
    o, _ = _resnet_oracle(at.conf, at.resnet_hyper)
    assert [param_count(at.conf, at.resnet_hyper, n) for n in range(3)] == [o.param_count(n) for n in range(3)]
    assert o.H == 6 * 6 * 64


@pytest.mark.parametrize("net", [0, 1, 2])
def test_downsample_oracle_matches_torch(net):
    """The downsampling representation (stride-2 convs without BatchNorm,
    MeanPool with the padding counted) and the 6x6 prediction / dynamics with
    18 actions, oracle vs torch fp32 at 1e-5."""
    from muzero_jl_amd.games import atari_synth as at
    conf, hyper = at.conf, at.resnet_hyper
    o, nets = _resnet_oracle(conf, hyper)
    nets = _perturb_bn(conf, hyper, nets)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
    rng = np.random.default_rng(net)
    n = 2
    if net == 0:
        x = at.observations(n, seed=net)
    elif net == 1:
        x = rng.normal(0, 1, (n, o.H)).astype(np.float32)
    else:
        x = np.concatenate([rng.normal(0, 1, (n, o.H)), np.full((n, 36), 5 / 18)], 1).astype(np.float32)
    ref = _torch_forward(conf, hyper, net, nets[net], x)
    got = o.forward(net, x)
    if net == 0:
        np.testing.assert_allclose(got, ref, **TOL)
    else:
        np.testing.assert_allclose(got[0], ref[0], **TOL)
        np.testing.assert_allclose(got[1], ref[1], **TOL)


def test_downsample_oracle_search_matches_mirror():
    """configs[4] search semantics (one player, 18 actions, 6x6 hidden board)
    in the oracle vs the independent mirror."""
    from mirror_ref import Mirror
    from muzero_jl_amd.games import atari_synth as at
    conf = dataclasses.replace(at.conf, num_iters=6)
    o, _ = _resnet_oracle(conf, at.resnet_hyper, seed=3)
    G = 2
    obs = at.observations(G, seed=1)
    legal = np.ones((G, 18), bool)
    legal[1, 5:9] = False
    tp = np.ones(G, np.int32)
    cv, rv, act = o.mcts_search(obs, legal, tp, exploration=True, rng_step=2, game_offset=5)
    cv2, rv2, act2, _ = Mirror(o, conf).search(obs, legal, tp, True, 5, 2)
    assert np.array_equal(cv, cv2) and np.array_equal(rv, rv2) and np.array_equal(act, act2)
