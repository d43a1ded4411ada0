"""Independent torch autograd reference of the corrected-gradient learner
(MZ_LEARN_CORRECTED; include/mz.h): the FC nets of Learning.jl:87-142 built
(or the ResNet nets of Learning.jl:148-255, Q12's intended architecture)
from the Flux-order flat vectors, the unroll of Learning.jl:347-370 (Q10
alignment: predictions on h0, h0, h1 .. h_{K-1}; make_dynamics_input's 2h and
a/|A| plane, :293-304) and the per-sample-mean loss

  L = (1/B) Σ_b (w_b/g_b) [Σ_k (v−z)² + Σ_k CE(logits, π) + ir·Σ_{k>=1} (r−u)²] + Σθ²

differentiated by torch.autograd (float64 by default)."""
import numpy as np
import torch


def _fc_chain(conf, hyper, nets, params):
    """FC nets; with use_batch_norm every make_dense is Dense then BatchNorm in
    test mode (μ = 0, σ² = 1, ε = 1e-5) before the relu (Learning.jl:70-78),
    β and γ after the Dense's W and b."""
    import torch.nn.functional as F
    from muzero_jl_amd.networks import layer_specs

    def layers(net):
        # the same slicing as networks.unflatten(with_bn=True), on the autograd leaves
        out, off = [], 0
        for ch, i, o, act, bn in layer_specs(conf, hyper, net, True):
            Wt = params[net][off: off + i * o].reshape(i, o).T
            off += i * o
            bt = params[net][off: off + o]
            off += o
            bg = None
            if bn:
                bg = (params[net][off: off + o], params[net][off + o: off + 2 * o])
                off += 2 * o
            out.append((ch, Wt, bt, act, bg))
        assert off == len(nets[net])
        return out

    L = [layers(n) for n in range(3)]

    def chain(net, ch, x):
        for c, W, b, act, bg in L[net]:
            if c != ch:
                continue
            x = x @ W.T + b
            if bg is not None:
                x = F.batch_norm(x, torch.zeros(x.shape[1], dtype=x.dtype), torch.ones(x.shape[1], dtype=x.dtype),
                                 bg[1], bg[0], training=False, eps=1e-5)
            x = torch.relu(x) if act == 1 else torch.tanh(x) if act == 2 else x
        return x
    return chain


def _resnet_chain(conf, hyper, params):
    """The ResNet nets (networks.resnet_specs, Flux-order slices of the leaves):
    convolution = cross-correlation with the kernel flipped, "same" padding,
    BatchNorm in test mode (μ = 0, σ² = 1, ε = 1e-5), residual blocks, the
    column-major (W,H,C) flatten; with ResNetHP.downsample the representation
    starts with the downsampler of Learning.jl:175-187 (stride-2 convs, blocks,
    MeanPool((3,3), stride 2, pad 1) counting the padding)."""
    import torch.nn.functional as F
    from muzero_jl_amd.networks import resnet_board, resnet_specs
    Wb, Hb = resnet_board(conf, hyper)

    def ops(net):
        out, off = [], 0
        p = params[net]
        for op in resnet_specs(conf, hyper, net):
            op = dict(op)
            if op["kind"] == "pool":
                out.append(op)
                continue
            if op["kind"] == "dense":
                i, o = op["cin"], op["cout"]
                op["w"] = p[off: off + i * o].reshape(i, o).T
                off += i * o
            else:
                kw, kh, ci, co = op["kw"], op["kh"], op["cin"], op["cout"]
                op["w"] = torch.flip(p[off: off + kw * kh * ci * co].reshape(co, ci, kh, kw), dims=[2, 3])
                off += kw * kh * ci * co
            op["b"] = p[off: off + op["cout"]]
            off += op["cout"]
            if op["kind"] == "conv" and op["bn"]:
                op["beta"] = p[off: off + op["cout"]]
                op["gamma"] = p[off + op["cout"]: off + 2 * op["cout"]]
                off += 2 * op["cout"]
            out.append(op)
        return out

    O = [ops(n) for n in range(3)]

    def act(t, a):
        return torch.relu(t) if a == 1 else torch.tanh(t) if a == 2 else t

    def chain(net, ch, t):
        res = None
        for op in O[net]:
            if op["chain"] != ch:
                continue
            if op["kind"] == "pool":
                t = F.avg_pool2d(t, 3, stride=2, padding=1, count_include_pad=True)
            elif op["kind"] == "conv":
                if t.dim() == 2:                       # (n, W*H*C) column-major -> (n, C, H, W)
                    t = t.reshape(t.shape[0], op["cin"], op.get("Hi", Hb), op.get("Wi", Wb))
                if op["res_save"]:
                    res = t
                y = F.conv2d(t, op["w"], op["b"], stride=op.get("stride", 1), padding=(op["kh"] // 2, op["kw"] // 2))
                if op["bn"]:
                    y = F.batch_norm(y, torch.zeros(op["cout"], dtype=y.dtype), torch.ones(op["cout"], dtype=y.dtype),
                                     op["gamma"], op["beta"], training=False, eps=1e-5)
                if op["res_add"]:
                    y = y + res
                t = act(y, op["act"])
            else:
                t = act(t.reshape(t.shape[0], -1) @ op["w"].T + op["b"], op["act"])
        return t.reshape(t.shape[0], -1) if t.dim() == 4 else t
    return chain


def corrected_loss_and_grads(conf, hyper, nets, batch, weights=None, dtype=torch.float64):
    from muzero_jl_amd.config import ResNetHP
    K, A = conf.num_unroll_steps, len(conf.action_space)
    params = [torch.tensor(np.asarray(f), dtype=dtype, requires_grad=True) for f in nets]
    chain = (_resnet_chain(conf, hyper, params) if isinstance(hyper, ResNetHP)
             else _fc_chain(conf, hyper, nets, params))

    obs = torch.tensor(batch["observation"], dtype=dtype)
    acts = torch.tensor(batch["actions"], dtype=dtype)
    tv = torch.tensor(batch["target_values"], dtype=dtype)
    tr = torch.tensor(batch["target_rewards"], dtype=dtype)
    tp = torch.tensor(batch["target_policies"], dtype=dtype)
    gs = torch.tensor(batch["gradient_scale"], dtype=dtype)
    w = torch.ones_like(gs) if weights is None else torch.tensor(weights, dtype=dtype)
    B = obs.shape[0]
    if isinstance(hyper, ResNetHP):                  # the hidden board (after the downsampler)
        from muzero_jl_amd.networks import resnet_board
        Wb, Hb = resnet_board(conf, hyper)
        plane = Wb * Hb
    else:
        plane = conf.observation_shape[0] * conf.observation_shape[1]
    hs = [chain(0, 0, obs)]
    rewards = [torch.zeros(B, dtype=dtype)]
    for k in range(1, K + 1):
        sa = torch.cat([2 * hs[k - 1], (acts[:, k - 1:k] / A).repeat(1, plane)], 1)
        t = chain(2, 0, sa)
        hs.append(chain(2, 1, t))
        rewards.append(chain(2, 2, t)[:, 0])
    vals, logits = [], []
    for k in range(K + 1):
        t = chain(1, 0, hs[0 if k <= 1 else k - 1])
        vals.append(chain(1, 1, t)[:, 0])
        logits.append(chain(1, 2, t))
    v = torch.stack(vals, 1)
    lg = torch.stack(logits, 1)
    r = torch.stack(rewards, 1)
    c = w / gs / B
    vloss = (c * ((v - tv) ** 2).sum(1)).sum()
    ce = -(tp * torch.log_softmax(lg, -1)).sum(-1)
    ploss = (c * ce.sum(1)).sum()
    rloss = (c * ((r[:, 1:] - tr[:, 1:]) ** 2).sum(1)).sum() if conf.intermediate_rewards else 0 * vloss
    data = vloss + ploss + rloss
    l2 = [(p ** 2).sum() for p in params]
    total = data + sum(l2)
    grads = torch.autograd.grad(total, params)
    vloss, ploss, rloss = vloss.detach(), ploss.detach(), rloss.detach()
    return dict(grads=[g.detach().numpy() for g in grads], value=float(vloss), policy=float(ploss),
                reward=float(rloss), l2=[float(x.detach()) for x in l2], values=v.detach().numpy(),
                policies=torch.softmax(lg, -1).detach().numpy(), rewards=r.detach().numpy())
