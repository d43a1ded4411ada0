"""Checkpoints on the host: the safetensors layout of
muzero.jl_amd/checkpoint.py (Flux.params order, Julia column-major bytes,
reversed shapes), round trips, and the Julia-layout view of each array."""
import numpy as np
import pytest


@pytest.mark.parametrize("kind", ["fc", "resnet"])
def test_roundtrip_and_layout(ttt, tmp_path, kind):
    from muzero_jl_amd import checkpoint as ck
    from muzero_jl_amd.networks import init_nets, param_count
    hyper = ttt.hyper if kind == "fc" else ttt.resnet_hyper
    nets = init_nets(ttt.conf, hyper, seed=3)
    n = sum(param_count(ttt.conf, hyper, k) for k in range(3))
    rng = np.random.default_rng(0)
    adam = (rng.random(n).astype(np.float32), rng.random(n).astype(np.float32), np.array([0.9 ** 7, 0.999 ** 7]))
    p = str(tmp_path / "ck.safetensors")
    ck.write(p, ttt.conf, hyper, nets, training_step=123, adam=adam)
    t, meta = ck.read(p)
    assert meta["training_step"] == "123" and meta["network"] == kind and meta["format"] == ck.FORMAT
    for a, b in zip(ck.nets_from(t, ttt.conf, hyper), nets):
        assert np.array_equal(a, b)
    assert np.array_equal(t["adam.m"], adam[0]) and np.array_equal(t["adam.beta_pow"], adam[2])
    # the numpy array transposed is the Julia array: Dense W (out, in) / Conv W (kw, kh, cin, cout)
    first = ck.param_table(ttt.conf, hyper, 0)[0]
    jw = ck.flux_arrays(ttt.conf, hyper, 0, nets[0])[0]
    assert jw.shape == first[1] and np.array_equal(t[first[0]].transpose(), jw)
    if kind == "fc":
        from muzero_jl_amd.networks import unflatten
        _, W, _, _ = unflatten(ttt.conf, hyper, 0, nets[0])[0]
        assert np.array_equal(jw, W)


def test_names_and_counts(ttt):
    from muzero_jl_amd import checkpoint as ck
    t = ck.param_table(ttt.conf, ttt.hyper, 1)
    assert [x[0] for x in t[:2]] == ["prediction.0", "prediction.1"]
    assert t[0][1] == (64, 27) and t[1][1] == (64,)
    r = ck.param_table(ttt.conf, ttt.resnet_hyper, 0)
    assert r[0][1] == (3, 3, 7, 64) and len(r) == 4 * 5     # conv + 2 blocks x 2 convs, 4 arrays each


def test_shape_mismatch_rejected(ttt, tmp_path):
    from muzero_jl_amd import checkpoint as ck
    from muzero_jl_amd.networks import init_nets
    p = str(tmp_path / "fc.safetensors")
    ck.write(p, ttt.conf, ttt.hyper, init_nets(ttt.conf, ttt.hyper, seed=1))
    t, _ = ck.read(p)
    with pytest.raises((KeyError, ValueError)):
        ck.nets_from(t, ttt.conf, ttt.resnet_hyper)
