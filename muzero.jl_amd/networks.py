"""The FC representation / prediction / dynamics networks (Learning.jl:70-142)
as flat Flux-order parameter vectors.

Flux order per net: for every Dense in Chain order (Split paths in order),
W (out, in) column-major then b.  `layer_specs` lists (chain, in, out, act)
with chain 0 = trunk, 1 = first Split path, 2 = second Split path.
"""
import numpy as np

from .config import ACT_IDENTITY, ACT_RELU, ACT_TANH, stacked_features

NET_REPR, NET_PRED, NET_DYN = 0, 1, 2


def layer_specs(conf, hyper, net):
    w, h, c = conf.observation_shape
    hs, hid, A = hyper.width_hidden, hyper.hidden_state_size, len(conf.action_space)
    act_r = {"tanh": ACT_TANH, "relu": ACT_RELU, "identity": ACT_IDENTITY}[
        hyper.reward_activation if isinstance(hyper.reward_activation, str) else hyper.reward_activation.__name__]
    L = []
    if net == NET_REPR:                                   # init_representation (:87-98)
        L.append((0, stacked_features(conf), hs, ACT_RELU))
        L += [(0, hs, hs, ACT_RELU)] * hyper.depth_representation
        L.append((0, hs, hid, ACT_IDENTITY))
    elif net == NET_PRED:                                 # init_prediction (:100-116)
        L.append((0, hid, hs, ACT_RELU))
        L += [(0, hs, hs, ACT_RELU)] * hyper.depth_prediction
        L += [(1, hs, hs, ACT_RELU)] * hyper.depth_value
        L.append((1, hs, 1, ACT_TANH))
        L += [(2, hs, hs, ACT_RELU)] * hyper.depth_policy
        L.append((2, hs, A, ACT_IDENTITY))               # then softmax
    else:                                                 # init_dynamics (:118-142)
        L.append((0, w * h * (c + 1), hs, ACT_RELU))
        L += [(0, hs, hs, ACT_RELU)] * hyper.depth_dynamics
        L += [(1, hs, hs, ACT_RELU)] * hyper.depth_state_head
        L.append((1, hs, hid, ACT_IDENTITY))
        L += [(2, hs, hs, ACT_RELU)] * hyper.depth_reward
        L.append((2, hs, 1, act_r))
    return L


def param_count(conf, hyper, net):
    return sum(i * o + o for _, i, o, _ in layer_specs(conf, hyper, net))


def glorot_uniform(rng, out, inp):
    """Flux 0.12 glorot_uniform: (rand(Float32, out, in) .- 0.5f0) .* sqrt(24f0 / (in + out))."""
    u = rng.random((inp, out), dtype=np.float32)          # column-major (out, in) == C (in, out)
    return ((u - np.float32(0.5)) * np.float32(np.sqrt(np.float32(24.0) / np.float32(inp + out)))).astype(np.float32)


def init_net(conf, hyper, net, seed=0):
    """init_representation / init_prediction / init_dynamics: glorot W, zero b (Q17)."""
    rng = np.random.default_rng(seed * 3 + net)
    parts = []
    for _, i, o, _ in layer_specs(conf, hyper, net):
        parts.append(glorot_uniform(rng, o, i).reshape(-1))
        parts.append(np.zeros(o, np.float32))
    return np.concatenate(parts)


def init_nets(conf, hyper, seed=0):
    return [init_net(conf, hyper, n, seed) for n in range(3)]


def unflatten(conf, hyper, net, flat):
    """-> list of (chain, W (out,in) as numpy, b, act)."""
    out, off = [], 0
    for ch, i, o, act in layer_specs(conf, hyper, net):
        W = flat[off: off + i * o].reshape(i, o).T
        off += i * o
        b = flat[off: off + o]
        off += o
        out.append((ch, W, b, act))
    return out
