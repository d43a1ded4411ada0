"""The corrected-gradient learner on the ResNet nets (MZ_LEARN_CORRECTED;
mz_backprop.hip mz_rbp_sample / mz_rbp_dw: backpropagation through
convolutions, test-mode BatchNorm, residual blocks and the Dense heads of the
K-step unroll on f32 MFMA) against the independent torch autograd reference
(tests/torch_learner_ref.py, float64) at the 1e-5 tolerance of north_star:
every net's data gradient relative to its largest entry, the losses and the
read-outs.  TicTacToe ResNet (configs[2]'s nets, 3x3 kernels in the
representation) and Connect4 ResNet-8 (configs[3]).  Reference:
src/Learning.jl:148-255 (the nets, Q12), :261-288 (the loss, differentiated
unlike the reference's pullbacks, Q11), :347-370 (the unroll)."""
import dataclasses

import numpy as np
import pytest

from torch_learner_ref import corrected_loss_and_grads

pytestmark = pytest.mark.gpu


def _lively(conf, hyper, seed):
    """init_nets with β ~ N(0, 0.1), γ ~ U(0.5, 1.5), biases ~ N(0, 0.1)."""
    from test_resnet_oracle import _perturb_bn
    from muzero_jl_amd.networks import init_nets
    return _perturb_bn(conf, hyper, init_nets(conf, hyper, seed=seed), seed=seed + 1)


def _ds_param_count(conf, hyper):
    """Parameters of the downsampler: net 0's ops up to its last MeanPool (Flux.params order)."""
    from muzero_jl_amd.networks import resnet_specs
    ops = resnet_specs(conf, hyper, 0)
    last = max(i for i, o in enumerate(ops) if o["kind"] == "pool")
    n = 0
    for o in ops[:last]:
        if o["kind"] == "conv":
            n += o["kw"] * o["kh"] * o["cin"] * o["cout"] + o["cout"] + (2 * o["cout"] if o["bn"] else 0)
    return n


def _batch(B, K, A, feat, rng):
    obs = (rng.random((B, feat)) < 0.4).astype(np.float32)
    tpol = rng.random((B, K + 1, A)).astype(np.float32)
    return dict(observation=obs, actions=rng.integers(1, A + 1, (B, K + 1)).astype(np.float32),
                target_values=rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
                target_rewards=rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
                target_policies=tpol / tpol.sum(-1, keepdims=True),
                gradient_scale=rng.integers(1, max(K, 1) + 1, B).astype(np.float32))


@pytest.mark.parametrize("game,B,K,ir,per", [("ttt", 12, 3, True, False), ("ttt", 7, 0, False, True),
                                             ("c4", 4, 2, True, True), ("atari", 3, 2, True, True)])
def test_corrected_resnet_gradient_matches_torch(ttt, game, B, K, ir, per):
    """atari: configs[4]'s nets, the downsampler (mz_dsbp_*) in front of the
    representation's tail, 84x84x4 observations."""
    import torch
    from muzero_jl_amd import abi
    from muzero_jl_amd.games import atari_synth, connect4 as c4
    mod = {"ttt": ttt, "c4": c4, "atari": atari_synth}[game]
    conf = dataclasses.replace(mod.conf, batch_size=B, num_unroll_steps=K, intermediate_rewards=ir)
    hyper = mod.resnet_hyper
    nets = _lively(conf, hyper, B + K)
    eng = abi.Engine(conf, hyper, device=0, max_games=8, rng_seed=1)
    for n, w in enumerate(nets):
        eng.set_weights(n, w)
    eng.learner_set_mode(abi.LEARN_CORRECTED)
    A = len(conf.action_space)
    feat = int(np.prod(conf.observation_shape)) * (conf.stacked_observations + 1) + \
        conf.observation_shape[0] * conf.observation_shape[1] * conf.stacked_observations
    rng = np.random.default_rng(B)
    batch = _batch(B, K, A, feat, rng)
    wts = (rng.random(B).astype(np.float32) * 0.9 + 0.1) if per else None
    dev = [torch.from_numpy(np.ascontiguousarray(batch[k])).cuda() for k in
           ("observation", "actions", "target_values", "target_rewards", "target_policies", "gradient_scale")]
    dev.append(torch.from_numpy(wts).cuda() if per else None)
    grad = torch.zeros(eng.grad_count(), dtype=torch.float32, device="cuda")
    losses = torch.zeros(8, dtype=torch.float32, device="cuda")
    eng.learner_grad_dev([t.data_ptr() if t is not None else None for t in dev], B, grad.data_ptr(),
                         losses.data_ptr())
    eng.sync()
    ref = corrected_loss_and_grads(conf, hyper, nets, batch, wts)
    g = grad.cpu().numpy()
    off = 0
    for n in range(3):
        gn = g[off: off + nets[n].size].astype(np.float64)   # grad_dev holds the data term (2θ: apply)
        rn = ref["grads"][n] - 2.0 * nets[n].astype(np.float64)
        off += nets[n].size
        scale = np.abs(rn).max()
        if n == 2 and K == 0:                        # no unroll step: the dynamics net is not used
            assert scale == 0.0 and np.abs(gn).max() == 0.0
            continue
        assert scale > 1e-4, f"net {n}: no data gradient reached it"
        err = np.abs(gn - rn).max() / scale
        assert err < 1e-5, f"net {n}: data gradient rel. error {err:.3g}"
        if n == 0 and game == "atari":               # the downsampler's own slice, on its own scale
            nd = _ds_param_count(conf, hyper)
            sd = np.abs(rn[:nd]).max()
            assert sd > 1e-6, "no data gradient reached the downsampler"
            ed = np.abs(gn[:nd] - rn[:nd]).max() / sd
            assert ed < 1e-5, f"downsampler data gradient rel. error {ed:.3g}"
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


def test_corrected_resnet_learner_steps(ttt):
    """mz_learner_step in corrected mode = grad_dev + apply (ADAM into the
    ResNet images), bit for bit; the device-sampled learner runs on a
    self-play shard."""
    import torch
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import cos_schedule
    from muzero_jl_amd.games import atari_synth
    from muzero_jl_amd.networks import init_nets
    B = 16
    conf = dataclasses.replace(ttt.conf, batch_size=B, num_iters=4)
    nets = init_nets(conf, ttt.resnet_hyper, seed=3)
    e1, e2 = (abi.Engine(conf, ttt.resnet_hyper, device=0, max_games=16, rng_seed=2) for _ in range(2))
    for e in (e1, e2):
        for n, w in enumerate(nets):
            e.set_weights(n, w)
        e.learner_set_mode(abi.LEARN_CORRECTED)
    rng = np.random.default_rng(0)
    grad = torch.zeros(e2.grad_count(), dtype=torch.float32, device="cuda")
    for t in range(1, 4):
        batch = _batch(B, conf.num_unroll_steps, 9, 63, rng)
        l1 = e1.learner_step(batch, cos_schedule(t))
        dev = [torch.from_numpy(np.ascontiguousarray(batch[k])).cuda() for k in
               ("observation", "actions", "target_values", "target_rewards", "target_policies", "gradient_scale")]
        losses = torch.zeros(8, dtype=torch.float32, device="cuda")
        e2.learner_grad_dev([d.data_ptr() for d in dev] + [None], B, grad.data_ptr(), losses.data_ptr())
        e2.learner_apply_dev(grad.data_ptr(), 1.0, cos_schedule(t))
        e2.sync()
        assert np.array_equal(l1, losses.cpu().numpy()[:6])
        for n in range(3):
            assert np.array_equal(e1.get_weights(n), e2.get_weights(n))
    assert not np.array_equal(e1.get_weights(0), nets[0])
    # the searches read the updated images: both engines still agree
    obs = (rng.random((8, 63)) < 0.3).astype(np.float32)
    legal = np.ones((8, 9), bool)
    tp = np.ones(8, np.int32)
    assert all(np.array_equal(a, b) for a, b in zip(e1.mcts_search(obs, legal, tp, rng_step=5),
                                                    e2.mcts_search(obs, legal, tp, rng_step=5)))
    e1.selfplay_init(abi.ENV_TICTACTOE, 16, 64)
    for m in range(12):
        e1.selfplay_move(m)
    out = torch.zeros(8, dtype=torch.float32, device="cuda")
    for t in range(4, 7):
        e1.learner_train_dev(B, t, cos_schedule(t), out.data_ptr())
    e1.sync()
    assert np.all(np.isfinite(out.cpu().numpy()[:6]))
    e1.close(); e2.close()


def test_corrected_atari_learner_trains():
    """configs[4] in corrected mode: grad_dev + apply equals mz_learner_step bit
    for bit through the downsampler, and the device-sampled learner runs on an
    Atari-like self-play shard with finite losses."""
    import torch
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import cos_schedule
    from muzero_jl_amd.games import atari_synth
    B = 4
    conf = dataclasses.replace(atari_synth.conf, batch_size=B, num_iters=4, num_unroll_steps=2, max_moves=4,
                               replay_buffer_size=32)
    hyper = atari_synth.resnet_hyper
    nets = _lively(conf, hyper, 5)
    e1, e2 = (abi.Engine(conf, hyper, device=0, max_games=8, rng_seed=2) for _ in range(2))
    for e in (e1, e2):
        for n, w in enumerate(nets):
            e.set_weights(n, w * np.float32(0.5))
        e.learner_set_mode(abi.LEARN_CORRECTED)
    rng = np.random.default_rng(1)
    grad = torch.zeros(e2.grad_count(), dtype=torch.float32, device="cuda")
    A = len(conf.action_space)
    for t in range(1, 3):
        batch = _batch(B, conf.num_unroll_steps, A, 84 * 84 * 4, rng)
        l1 = e1.learner_step(batch, 1e-4)
        dev = [torch.from_numpy(np.ascontiguousarray(batch[k])).cuda() for k in
               ("observation", "actions", "target_values", "target_rewards", "target_policies", "gradient_scale")]
        losses = torch.zeros(8, dtype=torch.float32, device="cuda")
        e2.learner_grad_dev([d.data_ptr() for d in dev] + [None], B, grad.data_ptr(), losses.data_ptr())
        e2.learner_apply_dev(grad.data_ptr(), 1.0, 1e-4)
        e2.sync()
        assert np.array_equal(l1, losses.cpu().numpy()[:6])
        for n in range(3):
            assert np.array_equal(e1.get_weights(n), e2.get_weights(n))
    e1.selfplay_init(abi.ENV_ATARI, 8, 32)
    for m in range(10):
        e1.selfplay_move(m)
    out = torch.zeros(8, dtype=torch.float32, device="cuda")
    for t in range(3, 5):
        e1.learner_train_dev(B, t, cos_schedule(t), out.data_ptr())
    e1.sync()
    assert np.all(np.isfinite(out.cpu().numpy()[:6]))
    e1.close(); e2.close()
