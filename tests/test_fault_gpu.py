"""Cross-workgroup hand-offs report a producer that never publishes.

mz_rsearch_nets (the prediction workgroup of a tile waits for the dynamics
workgroup's trunk output) and mz_runroll_fused_r (prediction / reward items
wait for their sample's chain block) poll a progress word with a bounded wait
(mz_poll_ge).  On timeout the kernel sets a bit in the engine's device fault
word; the host reads it at its next synchronisation and fails that call with
a message — the stale-input results are never returned as a success.

MZ_DEBUG_SKIP_PUBLISH=1 at engine creation makes tile / sample 0 skip its
publish and shortens the bound to 10 ms, so the error path runs once here.
An engine created without the switch runs the same calls cleanly."""
import dataclasses

import numpy as np
import pytest

from muzero_jl_amd import abi

pytestmark = pytest.mark.gpu


def _engine(ttt, monkeypatch, skip, G=16):
    if skip:
        monkeypatch.setenv("MZ_DEBUG_SKIP_PUBLISH", "1")
    else:
        monkeypatch.delenv("MZ_DEBUG_SKIP_PUBLISH", raising=False)
    from muzero_jl_amd.networks import init_nets
    conf = dataclasses.replace(ttt.conf, num_iters=3, batch_size=32, replay_buffer_size=64)
    eng = abi.Engine(conf, ttt.resnet_hyper, device=0, max_games=G, rng_seed=5)
    for n, w in enumerate(init_nets(conf, ttt.resnet_hyper, seed=6)):
        eng.set_weights(n, w)
    monkeypatch.delenv("MZ_DEBUG_SKIP_PUBLISH", raising=False)
    return eng


def _positions(G, seed=0):
    rng = np.random.default_rng(seed)
    obs = (rng.random((G, 63)) < 0.4).astype(np.float32)
    legal = rng.random((G, 9)) < 0.6
    legal[:, 4] = True
    return obs, legal, rng.integers(1, 3, G).astype(np.int32)


@pytest.mark.parametrize("skip", [True, False])
def test_search_trunk_handoff_fault_reported(ttt, monkeypatch, skip):
    eng = _engine(ttt, monkeypatch, skip)
    obs, legal, tp = _positions(16)
    if skip:
        with pytest.raises(abi.MzError, match="mz_rsearch_nets trunk hand-off"):
            eng.mcts_search(obs, legal, tp, rng_step=1)
        eng.sync()                                  # reported once, then cleared
    else:
        eng.mcts_search(obs, legal, tp, rng_step=1)
    assert eng.search_variant() == "mz_rsearch"
    eng.close()


@pytest.mark.parametrize("skip", [True, False])
def test_fused_learner_progress_fault_reported(ttt, monkeypatch, skip):
    import torch
    eng = _engine(ttt, monkeypatch, skip)
    eng.selfplay_init(abi.ENV_TICTACTOE, 16, 64)
    if skip:                                        # the search faults too: clear it before the learner
        eng.selfplay_move(0)
        with pytest.raises(abi.MzError, match="device fault"):
            eng.sync()
        for m in range(1, 12):
            eng.selfplay_move(m)
        with pytest.raises(abi.MzError, match="device fault"):
            eng.sync()
    else:
        for m in range(12):
            eng.selfplay_move(m)
        eng.sync()
    out = torch.zeros(8, dtype=torch.float32, device="cuda")
    eng.learner_train_dev(32, 1, 1e-4, out.data_ptr())
    assert eng.learner_variant() == "mz_runroll_fused_r"
    if skip:
        with pytest.raises(abi.MzError, match="mz_runroll_fused_r chain progress"):
            eng.sync()
    else:
        eng.sync()
        assert np.all(np.isfinite(out.cpu().numpy()[:6]))
    # the faulted step's outputs are invalid, its weights are not: the ref_semantics
    # ADAM step (∇ = 2θ, Q11) does not read the unroll — equal to a clean engine's step
    ref = _engine(ttt, monkeypatch, False)
    ref.selfplay_init(abi.ENV_TICTACTOE, 16, 64)
    for m in range(12):
        ref.selfplay_move(m)
    ref.learner_train_dev(32, 1, 1e-4, out.data_ptr())
    ref.sync()
    for n in range(3):
        assert np.array_equal(eng.get_weights(n), ref.get_weights(n)), n
    ref.close()
    eng.close()
