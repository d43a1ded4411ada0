"""Actor–learner loop (self_play! ‖ learning!, quirk Q16).

CPU: the oracle's restatement (ora_train_loop) checked against properties the
reference's coupling implies, independently of the search:
* one learner step per saved game while t <= training_steps (SelfPlay.jl:396,
  Learning.jl:327, 411);
* in ref_semantics the update is data-independent (∇ = 2θ, Q11), so the
  learner's nets after t steps are ADAM^t(N0) whatever the games were;
* the actors run one checkpoint behind (remote_NNs starts with N0 and is a
  capacity-1 channel, SelfPlay.jl:392, 399-401, Learning.jl:416-418): after t
  steps they hold N_{c(t)-ci} with c(t) the last checkpoint step, and the
  queue holds N_{c(t)}.
GPU (test_train_loop_gpu.py): mz_train_run against ora_train_loop bit for bit.
"""
import dataclasses

import numpy as np
import pytest


def _setup(S=6, B=8, ci=3, training_steps=10000, thr=None, seed=5):
    from muzero_jl_amd.config import to_c_config, to_c_ffhp
    from muzero_jl_amd.games import tictactoe as ttt
    from muzero_jl_amd.networks import init_nets
    from oracle import Oracle
    conf = dataclasses.replace(ttt.conf, num_iters=S, batch_size=B, checkpoint_interval=ci,
                               training_steps=training_steps, temperature_threshold=thr)
    o = Oracle(to_c_config(conf), to_c_ffhp(ttt.hyper), seed=seed)
    for n, w in enumerate(init_nets(conf, ttt.hyper, seed=seed + 1)):
        o.set_weights(n, w)
    return conf, o


def _adam_trajectory(o, n):
    """N_0 .. N_n under the ref_semantics update (∇ = 2θ, Cos schedule)."""
    from oracle import _p
    L = o.L
    flat = np.concatenate(o.params).copy()
    m, v, bp = np.zeros_like(flat), np.zeros_like(flat), np.array([0.9, 0.999])
    out = [flat.copy()]
    for t in range(1, n + 1):
        L.ora_adam_2theta(_p(flat), _p(m), _p(v), flat.size, _p(bp), L.ora_cos_schedule(1e-4, 1e-1, 10, t))
        bp *= np.array([0.9, 0.999])
        out.append(flat.copy())
    return out


@pytest.mark.parametrize("training_steps,thr", [(10000, None), (7, 2)])
def test_oracle_train_loop_coupling(training_steps, thr):
    from oracle import train_loop
    conf, o = _setup(training_steps=training_steps, thr=thr)
    N = _adam_trajectory(o, 40)
    r = train_loop(o, G=10, cap=16, moves=24, move0=3, game_offset=2)
    games = int(r["counters"][0])
    t = r["t"]
    assert games > conf.checkpoint_interval
    assert t == min(games, training_steps + 1)                      # one step per game, :327 bound
    assert r["counters"][1] == sum(len(h["action"]) for h in r["held"]) or games > 16
    flat = lambda ps: np.concatenate(ps)                             # noqa: E731
    assert np.array_equal(flat(o.params), N[t])                      # data-independent learner
    ci = conf.checkpoint_interval
    last = (t // ci) * ci if t >= max(ci, 2) else 0                  # last checkpoint step (t > 1)
    assert np.array_equal(flat(r["queued"]), N[last])
    assert np.array_equal(flat(r["actor"]), N[max(last - ci, 0)])     # one checkpoint behind
    assert len(r["held"]) == min(games, 16)
    for h in r["held"]:
        T = len(h["action"])
        assert 1 <= T <= conf.max_moves + 1
        assert np.allclose(h["child_visits"].sum(1), 1.0, atol=1e-6)
        if thr is not None:
            assert T > thr


def test_oracle_train_loop_deterministic():
    from oracle import train_loop
    _, o1 = _setup()
    _, o2 = _setup()
    a = train_loop(o1, G=6, cap=8, moves=15, move0=1)
    b = train_loop(o2, G=6, cap=8, moves=15, move0=1)
    assert a["t"] == b["t"] and np.array_equal(a["counters"], b["counters"])
    for x, y in zip(a["held"], b["held"]):
        for k in x:
            assert np.array_equal(x[k], y[k])
