"""The corrected-gradient learner (MZ_LEARN_CORRECTED: backpropagation
through the unroll on MFMA, mz_backprop.hip) against an independent torch
autograd reference (tests/torch_learner_ref.py, float64), at the 1e-5
tolerance of north_star: the data gradient of every net relative to its
largest entry, the read-outs and the losses.  Reference loss:
src/Learning.jl:261-288 (differentiated, unlike the reference's pullbacks,
quirk Q11), unroll :347-370."""
import dataclasses

import numpy as np
import pytest

from torch_learner_ref import corrected_loss_and_grads

pytestmark = pytest.mark.gpu


def _batch(B, K, A, feat, rng):
    obs = (rng.random((B, feat)) < 0.4).astype(np.float32)
    tpol = rng.random((B, K + 1, A)).astype(np.float32)
    return dict(observation=obs, actions=rng.integers(1, A + 1, (B, K + 1)).astype(np.float32),
                target_values=rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
                target_rewards=rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
                target_policies=tpol / tpol.sum(-1, keepdims=True),
                gradient_scale=rng.integers(1, max(K, 1) + 1, B).astype(np.float32))


@pytest.mark.parametrize("B,K,ir,per", [(32, 5, False, False), (20, 3, True, True), (40, 5, True, False),
                                        (7, 0, False, False)])
def test_corrected_gradient_matches_torch(ttt, B, K, ir, per):
    import torch
    from muzero_jl_amd import abi
    from muzero_jl_amd.networks import init_nets
    conf = dataclasses.replace(ttt.conf, batch_size=B, num_unroll_steps=K, intermediate_rewards=ir)
    nets = [n * np.float32(3.0) for n in init_nets(conf, ttt.hyper, seed=B + K)]   # livelier activations
    eng = abi.Engine(conf, ttt.hyper, device=0, max_games=8, rng_seed=1)
    for n, w in enumerate(nets):
        eng.set_weights(n, w)
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
    ref = corrected_loss_and_grads(conf, ttt.hyper, nets, batch, wts)
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


def test_corrected_learner_trains_and_matches_apply(ttt):
    """mz_learner_step in corrected mode = grad_dev + apply (ADAM); the
    device-sampled fused call runs too; a few steps move the losses."""
    import torch
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import cos_schedule
    from muzero_jl_amd.networks import init_nets
    B = 32
    conf = dataclasses.replace(ttt.conf, batch_size=B, num_iters=4)
    nets = init_nets(conf, ttt.hyper, seed=3)
    e1 = abi.Engine(conf, ttt.hyper, device=0, max_games=16, rng_seed=2)
    e2 = abi.Engine(conf, ttt.hyper, device=0, max_games=16, rng_seed=2)
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
    # the device-sampled learner in corrected mode
    e1.selfplay_init(abi.ENV_TICTACTOE, 16, 64)
    for m in range(12):
        e1.selfplay_move(m)
    out = torch.zeros(8, dtype=torch.float32, device="cuda")
    for t in range(4, 8):
        e1.learner_train_dev(B, t, cos_schedule(t), out.data_ptr())
    e1.sync()
    assert np.all(np.isfinite(out.cpu().numpy()[:6]))
    e1.close(); e2.close()


@pytest.mark.parametrize("B,K,ir", [(32, 5, True), (40, 3, False)])
def test_level_schedule_equals_sequential_tile_kernel(ttt, B, K, ir, monkeypatch):
    """mz_bp_tile_lv (the unroll's applications grouped into dependency
    levels, one barrier per level) against mz_bp_tile (one application per
    barrier, MZ_BP_SEQ=1): gradient, losses and read-outs identical bit for bit
    — the level schedule keeps every accumulation into a shared input gradient
    in the sequential kernel's order."""
    import torch
    from muzero_jl_amd import abi
    from muzero_jl_amd.networks import init_nets
    conf = dataclasses.replace(ttt.conf, batch_size=B, num_unroll_steps=K, intermediate_rewards=ir)
    nets = [n * np.float32(3.0) for n in init_nets(conf, ttt.hyper, seed=5)]
    eng = abi.Engine(conf, ttt.hyper, device=0, max_games=8, rng_seed=1)
    for n, w in enumerate(nets):
        eng.set_weights(n, w)
    eng.learner_set_mode(abi.LEARN_CORRECTED)
    batch = _batch(B, K, 9, 63, np.random.default_rng(B + 1))
    dev = [torch.from_numpy(np.ascontiguousarray(batch[k])).cuda() for k in
           ("observation", "actions", "target_values", "target_rewards", "target_policies", "gradient_scale")]
    out = []
    for seq in (False, True):
        if seq:
            monkeypatch.setenv("MZ_BP_SEQ", "1")
        grad = torch.zeros(eng.grad_count(), dtype=torch.float32, device="cuda")
        losses = torch.zeros(8, dtype=torch.float32, device="cuda")
        eng.learner_grad_dev([d.data_ptr() for d in dev] + [None], B, grad.data_ptr(), losses.data_ptr())
        eng.sync()
        out.append((grad.cpu().numpy(), losses.cpu().numpy()[:6], [x.copy() for x in eng.debug_unroll(B)]))
    (g0, l0, u0), (g1, l1, u1) = out
    assert np.array_equal(g0, g1), "gradients differ between the level and sequential schedules"
    assert np.array_equal(l0, l1)
    for a, b in zip(u0, u1):
        assert np.array_equal(a, b)
    eng.close()
