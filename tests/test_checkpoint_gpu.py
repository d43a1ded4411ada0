"""Checkpoints through the C ABI (mz_checkpoint_save / _load):
the engine's file reads back in Python with the Flux layout, a Python-written
file loads into the engine, and training resumes exactly (weights + ADAM
state + βp), for the FC and ResNet engines."""
import dataclasses

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _engine(conf, hyper, nets, seed=1):
    from muzero_jl_amd import abi
    e = abi.Engine(conf, hyper, device=0, max_games=8, rng_seed=seed)
    for n, w in enumerate(nets):
        e.set_weights(n, w)
    return e


@pytest.mark.parametrize("kind", ["fc", "resnet"])
def test_save_read_load_resume(ttt, tmp_path, kind):
    from muzero_jl_amd import checkpoint as ck
    from muzero_jl_amd.config import cos_schedule
    from muzero_jl_amd.networks import init_nets
    from test_gpu_parity import _random_batch
    hyper = ttt.hyper if kind == "fc" else ttt.resnet_hyper
    conf = dataclasses.replace(ttt.conf, batch_size=16)
    nets = init_nets(conf, hyper, seed=5)
    rng = np.random.default_rng(1)
    batches = [_random_batch(16, conf.num_unroll_steps, 9, rng) for _ in range(6)]
    e = _engine(conf, hyper, nets)
    for t in range(3):
        e.learner_step(batches[t], cos_schedule(t + 1))
    p = str(tmp_path / "ck.safetensors")
    e.checkpoint_save(p, 3)
    # Python reads the engine's file: Flux arrays equal the engine's weights
    tensors, meta = ck.read(p)
    assert meta["network"] == kind and meta["training_step"] == "3"
    for n, flat in enumerate(ck.nets_from(tensors, conf, hyper)):
        assert np.array_equal(flat, e.get_weights(n))
    bp = [0.9, 0.999]                                # βp .= βp .* β once per step, from (β1, β2)
    for _ in range(3):
        bp = [bp[0] * 0.9, bp[1] * 0.999]
    assert np.array_equal(tensors["adam.beta_pow"], bp)
    # resume: a fresh engine loads the checkpoint and both continue identically
    r = _engine(conf, hyper, init_nets(conf, hyper, seed=99))
    assert r.checkpoint_load(p) == 3
    for t in range(3, 6):
        la = e.learner_step(batches[t], cos_schedule(t + 1))
        lb = r.learner_step(batches[t], cos_schedule(t + 1))
        assert np.array_equal(la, lb)
    for n in range(3):
        assert np.array_equal(e.get_weights(n), r.get_weights(n))
    # a Python-written checkpoint loads into the engine
    q = str(tmp_path / "py.safetensors")
    ck.write(q, conf, hyper, nets, training_step=7)
    assert r.checkpoint_load(q) == 7
    for n in range(3):
        assert np.array_equal(r.get_weights(n), nets[n])
    e.close(); r.close()


def test_load_rejects_other_network(ttt, tmp_path):
    from muzero_jl_amd import checkpoint as ck
    from muzero_jl_amd.abi import MzError
    from muzero_jl_amd.networks import init_nets
    p = str(tmp_path / "resnet.safetensors")
    ck.write(p, ttt.conf, ttt.resnet_hyper, init_nets(ttt.conf, ttt.resnet_hyper, seed=1))
    e = _engine(ttt.conf, ttt.hyper, init_nets(ttt.conf, ttt.hyper, seed=1))
    with pytest.raises(MzError):
        e.checkpoint_load(p)
    with pytest.raises(MzError, match="cannot open"):
        e.checkpoint_load(str(tmp_path / "missing.safetensors"))
    e.close()
