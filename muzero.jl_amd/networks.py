"""The representation / prediction / dynamics networks as flat Flux-order
parameter vectors: FC (Learning.jl:70-142) and ResNet (Learning.jl:148-255,
the intended architecture of SURVEY §2.1 Q12 / DESIGN.md §9).

Flux order per net, in Chain order with Split paths in order:
  Dense     W (out, in) column-major, then b
  Conv      weight (kw, kh, cin, cout) column-major, then b
  BatchNorm β, then γ (running μ = 0, σ² = 1 are state, not params)
`layer_specs` (FC) lists (chain, in, out, act); `resnet_specs` lists dicts
with chain 0 = trunk, 1 = first Split path, 2 = second Split path.
"""
import numpy as np

from .config import ACT_IDENTITY, ACT_RELU, ACT_TANH, ResNetHP, stacked_features

NET_REPR, NET_PRED, NET_DYN = 0, 1, 2


def layer_specs(conf, hyper, net, with_bn=False):
    """(chain, in, out, act) per Dense; with_bn: (chain, in, out, act, bn), bn
    set on make_dense's layers (Learning.jl:70-78) when use_batch_norm — the
    Dense then has no activation and BatchNorm(out, relu) follows it, whose β,
    γ come after the Dense's W, b in Flux.params."""
    w, h, c = conf.observation_shape
    hs, hid, A = hyper.width_hidden, hyper.hidden_state_size, len(conf.action_space)
    act_r = {"tanh": ACT_TANH, "relu": ACT_RELU, "identity": ACT_IDENTITY}[
        hyper.reward_activation if isinstance(hyper.reward_activation, str) else hyper.reward_activation.__name__]
    bn = bool(getattr(hyper, "use_batch_norm", False))
    md = lambda ch, i, o: (ch, i, o, ACT_RELU, bn)       # make_dense
    L = []
    if net == NET_REPR:                                   # init_representation (:87-98)
        L.append(md(0, stacked_features(conf), hs))
        L += [md(0, hs, hs)] * hyper.depth_representation
        L.append((0, hs, hid, ACT_IDENTITY, False))
    elif net == NET_PRED:                                 # init_prediction (:100-116)
        L.append(md(0, hid, hs))
        L += [md(0, hs, hs)] * hyper.depth_prediction
        L += [md(1, hs, hs)] * hyper.depth_value
        L.append((1, hs, 1, ACT_TANH, False))
        L += [md(2, hs, hs)] * hyper.depth_policy
        L.append((2, hs, A, ACT_IDENTITY, False))        # then softmax
    else:                                                 # init_dynamics (:118-142)
        L.append(md(0, w * h * (c + 1), hs))
        L += [md(0, hs, hs)] * hyper.depth_dynamics
        L += [md(1, hs, hs)] * hyper.depth_state_head
        L.append((1, hs, hid, ACT_IDENTITY, False))
        L += [md(2, hs, hs)] * hyper.depth_reward
        L.append((2, hs, 1, act_r, False))
    return L if with_bn else [x[:4] for x in L]


def _act(a):
    if callable(a):
        a = a.__name__
    return {"tanh": ACT_TANH, "relu": ACT_RELU, "identity": ACT_IDENTITY}[a]


def _s2(n, k):
    return (n + 2 * (k // 2) - k) // 2 + 1


def resnet_board(conf, hyper):
    """(W, H) of the hidden state: the observation board, or after the
    downsampler (two stride-2 convs, two MeanPool(3, stride 2, pad 1);
    84 -> 42 -> 21 -> 11 -> 6) — representation_output_size, which
    prediction / dynamics read (Learning.jl:173, 194, 229)."""
    W, H = conf.observation_shape[0], conf.observation_shape[1]
    if getattr(hyper, "downsample", False):
        kw, kh = hyper.conv_kernel_size
        W, H = _s2(_s2(W, kw), kw), _s2(_s2(H, kh), kh)
        W, H = _s2(_s2(W, 3), 3), _s2(_s2(H, 3), 3)
    return W, H


def resnet_specs(conf, hyper, net):
    """Intended ResNet architecture (Learning.jl:148-255 with Q12 fixed), in
    the oracle's op order (oracle/mz_oracle.c onet_build_resnet).  Conv ops
    carry their output board (W, H), input board (Wi, Hi) and stride; "pool"
    ops are the downsampler's MeanPool((3,3), stride 2, pad 1) (no params)."""
    C = conf.observation_shape[2]
    W, H = resnet_board(conf, hyper)
    nf, nb, hs, A = hyper.num_filters, hyper.num_blocks, hyper.width_hidden, len(conf.action_space)
    P, nvf, npf = W * H, hyper.num_first_head_filters, hyper.num_second_head_filters
    ops = []

    def conv(ch, cin, cout, k, act=ACT_RELU, board=(W, H), stride=1, bn=True, inb=None):
        ops.append(dict(chain=ch, kind="conv", cin=cin, cout=cout, kw=k[0], kh=k[1], W=board[0], H=board[1],
                        Wi=(inb or board)[0], Hi=(inb or board)[1], stride=stride, bn=bn, act=act,
                        res_save=False, res_add=False))

    def block(ch, n, k, board=(W, H)):                     # resnet_block (:148-158)
        conv(ch, n, n, k, board=board)
        ops[-1]["res_save"] = True
        conv(ch, n, n, k, board=board)
        ops[-1]["res_add"] = True

    def dense(ch, i, o, act):
        ops.append(dict(chain=ch, kind="dense", cin=i, cout=o, act=act))

    k1 = (1, 1)
    if net == NET_REPR:                                    # :160-191
        k = tuple(hyper.conv_kernel_size)
        cin = C * (conf.stacked_observations + 1) + conf.stacked_observations
        if getattr(hyper, "downsample", False):            # :175-187 (`size` read as ksize)
            b0 = tuple(conf.observation_shape[:2])
            b1 = (_s2(b0[0], k[0]), _s2(b0[1], k[1]))
            conv(0, cin, cin, k, act=ACT_IDENTITY, board=b1, stride=2, bn=False, inb=b0)
            for _ in range(2):
                block(0, cin, k, b1)
            b2 = (_s2(b1[0], k[0]), _s2(b1[1], k[1]))
            conv(0, cin, 2 * cin, k, act=ACT_IDENTITY, board=b2, stride=2, bn=False, inb=b1)
            for _ in range(3):
                block(0, 2 * cin, k, b2)
            b3 = (_s2(b2[0], 3), _s2(b2[1], 3))
            ops.append(dict(chain=0, kind="pool", cin=2 * cin, cout=2 * cin, kw=3, kh=3, W=b3[0], H=b3[1],
                            Wi=b2[0], Hi=b2[1], stride=2, act=ACT_IDENTITY, res_save=False, res_add=False))
            for _ in range(3):
                block(0, 2 * cin, k, b3)
            ops.append(dict(chain=0, kind="pool", cin=2 * cin, cout=2 * cin, kw=3, kh=3, W=W, H=H,
                            Wi=b3[0], Hi=b3[1], stride=2, act=ACT_IDENTITY, res_save=False, res_add=False))
            cin = 2 * cin
        conv(0, cin, nf, k)
        for _ in range(nb):
            block(0, nf, k)
    elif net == NET_PRED:                                  # :193-226
        conv(0, nf, nf, k1)
        for _ in range(nb):
            block(0, nf, k1)
        conv(1, nf, nvf, k1)
        dense(1, P * nvf, hs, ACT_RELU)
        for _ in range(hyper.depth_value):
            dense(1, hs, hs, ACT_RELU)
        dense(1, hs, 1, ACT_TANH)
        conv(2, nf, npf, k1)
        dense(2, P * npf, hs, ACT_IDENTITY)
        for _ in range(hyper.depth_value):                 # :222 reuses depth_value
            dense(2, hs, hs, ACT_RELU)
        dense(2, hs, A, ACT_IDENTITY)                      # then softmax
    else:                                                  # :228-255
        conv(0, nf + 1, nf, k1)
        for _ in range(nb):
            block(0, nf, k1)
        conv(1, nf, nf, k1)
        for _ in range(nb):
            block(1, nf, k1)
        conv(2, nf, nvf, k1)
        dense(2, P * nvf, hs, ACT_RELU)
        for _ in range(hyper.depth_value):
            dense(2, hs, hs, ACT_RELU)
        dense(2, hs, 1, _act(hyper.reward_activation))
    return ops


def _op_params(op):
    if op["kind"] == "pool":
        return 0
    if op["kind"] == "dense":
        return op["cin"] * op["cout"] + op["cout"]
    return op["kw"] * op["kh"] * op["cin"] * op["cout"] + op["cout"] + (2 * op["cout"] if op["bn"] else 0)


def param_count(conf, hyper, net):
    if isinstance(hyper, ResNetHP):
        return sum(_op_params(op) for op in resnet_specs(conf, hyper, net))
    return sum(i * o + o + (2 * o if bn else 0) for _, i, o, _, bn in layer_specs(conf, hyper, net, True))


def net_macs(conf, hyper, net):
    """Multiply-accumulates of one forward of `net` for one item (the
    algorithmic FLOP count is 2x this): Dense in*out, conv W*H*kw*kh*cin*cout
    over its output board, MeanPool W*H*kw*kh*c additions (counted as MACs)."""
    if isinstance(hyper, ResNetHP):
        def macs(op):
            if op["kind"] == "dense":
                return op["cin"] * op["cout"]
            if op["kind"] == "pool":
                return op["W"] * op["H"] * op["kw"] * op["kh"] * op["cin"]
            return op["cin"] * op["cout"] * op["kw"] * op["kh"] * op["W"] * op["H"]
        return sum(macs(op) for op in resnet_specs(conf, hyper, net))
    return sum(i * o for _, i, o, _ in layer_specs(conf, hyper, net))


def glorot_uniform(rng, out, inp):
    """Flux 0.12 glorot_uniform: (rand(Float32, out, in) .- 0.5f0) .* sqrt(24f0 / (in + out))."""
    u = rng.random((inp, out), dtype=np.float32)          # column-major (out, in) == C (in, out)
    return ((u - np.float32(0.5)) * np.float32(np.sqrt(np.float32(24.0) / np.float32(inp + out)))).astype(np.float32)


def glorot_uniform_conv(rng, kw, kh, cin, cout):
    """Flux glorot_uniform(kw, kh, cin, cout): nfan = (kw*kh*cin, kw*kh*cout); column-major flat."""
    u = rng.random(kw * kh * cin * cout, dtype=np.float32)
    return ((u - np.float32(0.5)) * np.float32(np.sqrt(np.float32(24.0) /
                                                       np.float32(kw * kh * (cin + cout))))).astype(np.float32)


def init_net(conf, hyper, net, seed=0):
    """init_representation / init_prediction / init_dynamics: glorot W, zero b (Q17);
    BatchNorm β = 0, γ = 1."""
    rng = np.random.default_rng(seed * 3 + net)
    parts = []
    if isinstance(hyper, ResNetHP):
        for op in resnet_specs(conf, hyper, net):
            if op["kind"] == "pool":
                continue
            if op["kind"] == "dense":
                parts.append(glorot_uniform(rng, op["cout"], op["cin"]).reshape(-1))
                parts.append(np.zeros(op["cout"], np.float32))
            else:
                parts.append(glorot_uniform_conv(rng, op["kw"], op["kh"], op["cin"], op["cout"]))
                parts.append(np.zeros(op["cout"], np.float32))
                if op["bn"]:
                    parts.append(np.zeros(op["cout"], np.float32))   # β
                    parts.append(np.ones(op["cout"], np.float32))    # γ
        return np.concatenate(parts)
    for _, i, o, _, bn in layer_specs(conf, hyper, net, True):
        parts.append(glorot_uniform(rng, o, i).reshape(-1))
        parts.append(np.zeros(o, np.float32))
        if bn:
            parts.append(np.zeros(o, np.float32))         # BatchNorm β
            parts.append(np.ones(o, np.float32))          # BatchNorm γ
    return np.concatenate(parts)


def init_nets(conf, hyper, seed=0):
    return [init_net(conf, hyper, n, seed) for n in range(3)]


def unflatten_resnet(conf, hyper, net, flat):
    """-> the resnet_specs dicts with arrays: conv "w" (cout, cin, kh, kw) — Flux (kw,kh,cin,cout)
    column-major transposed — "b", "beta", "gamma"; dense "w" (out, in), "b"."""
    out, off = [], 0
    for op in resnet_specs(conf, hyper, net):
        op = dict(op)
        if op["kind"] == "pool":
            out.append(op)
            continue
        if op["kind"] == "dense":
            i, o = op["cin"], op["cout"]
            op["w"] = flat[off: off + i * o].reshape(i, o).T
            off += i * o
        else:
            kw, kh, ci, co = op["kw"], op["kh"], op["cin"], op["cout"]
            n = kw * kh * ci * co
            op["w"] = flat[off: off + n].reshape(co, ci, kh, kw)
            off += n
        op["b"] = flat[off: off + op["cout"]]
        off += op["cout"]
        if op["kind"] == "conv" and op["bn"]:
            op["beta"] = flat[off: off + op["cout"]]
            op["gamma"] = flat[off + op["cout"]: off + 2 * op["cout"]]
            off += 2 * op["cout"]
        out.append(op)
    return out


def unflatten(conf, hyper, net, flat, with_bn=False):
    """-> list of (chain, W (out,in) as numpy, b, act); with_bn: (chain, W, b,
    act, (β, γ) or None)."""
    out, off = [], 0
    for ch, i, o, act, bn in layer_specs(conf, hyper, net, True):
        W = flat[off: off + i * o].reshape(i, o).T
        off += i * o
        b = flat[off: off + o]
        off += o
        bg = None
        if bn:
            bg = (flat[off: off + o], flat[off + o: off + 2 * o])
            off += 2 * o
        out.append((ch, W, b, act, bg) if with_bn else (ch, W, b, act))
    return out
