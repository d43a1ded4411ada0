"""Data-parallel actor–learner loop and multi-step learner at world 2 (two spawned ranks on cuda:0, gloo
carrying the exchanges; RCCL needs one GPU per rank).  SURVEY §8e; src/Learning.jl:327-413,
src/SelfPlay.jl:384-419, games/tictactoe/main.jl:30-41.

In ref_semantics the update θ ← ADAM(θ, 2θ) does not read the data (Q11), so each rank runs the fast
multi-step form on its own shard and only counts and losses cross the ranks:
* the loop: per move every rank plays its G games (game_offset = rank·G, mz_train_move), the finished-game
  counts are summed (all_reduce) and every rank takes that many learner steps on B/world samples of its own
  shard (mz_train_learn);
* the learner: mz_learner_train_multi_dev with B/world samples per rank, the per-step losses all-reduced once
  per call.
Checked: the replicas (learner, actors, queued nets) are bit-identical across ranks, the learner's θ equals a
world-1 engine's θ after the same number of steps, and the actors / queued sets equal that run's θ at the
last two refresh steps; the split calls (mz_train_move + mz_train_learn) equal mz_train_run."""
import dataclasses
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G, CAP, B, MOVES, CI, L = 24, 64, 16, 12, 4, 20


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _conf():
    from muzero_jl_amd.games import tictactoe as ttt
    return ttt, dataclasses.replace(ttt.conf, num_iters=6, batch_size=B, replay_buffer_size=CAP,
                                    checkpoint_interval=CI)


def _engine(max_games):
    from muzero_jl_amd import abi
    from muzero_jl_amd.networks import init_nets
    ttt, conf = _conf()
    eng = abi.Engine(conf, ttt.hyper, device=0, max_games=max_games, rng_seed=21)
    for n, w in enumerate(init_nets(conf, ttt.hyper, seed=22)):
        eng.set_weights(n, w)
    return eng


def _sets(eng):
    from muzero_jl_amd import abi
    return [np.concatenate([eng.train_weights(w, n) for n in range(3)])
            for w in (abi.TRAIN_LEARNER, abi.TRAIN_ACTOR, abi.TRAIN_QUEUED)]


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist
    import _mzpkg
    _mzpkg.load()
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import cos_schedule
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _engine(G)
    eng.selfplay_init(abi.ENV_TICTACTOE, G, CAP)
    eng.train_init(B // world)
    steps = []
    for m in range(MOVES):
        n = torch.tensor([eng.train_move(50 + m, game_offset=rank * G)], dtype=torch.int64)
        dist.all_reduce(n)
        st = eng.train_learn(int(n.item()))
        steps.append((int(n.item()), st))
    loop_sets = _sets(eng)
    # the multi-step learner, B/world samples per rank, losses all-reduced once per call
    t0 = steps[-1][1][0] + 1
    losses = torch.zeros((L, 8), dtype=torch.float32, device="cuda")
    eng.learner_train_multi_dev(B // world, t0, [cos_schedule(t0 + i) for i in range(L)], losses.data_ptr())
    eng.sync()
    lc = losses.cpu()
    dist.all_reduce(lc)
    flat = np.concatenate([eng.get_weights(n) for n in range(3)])
    q.put((rank, steps, loop_sets, flat, lc.numpy() / world))
    dist.barrier()
    dist.destroy_process_group()
    eng.close()


def test_dp_train_loop_world2_replicas_match_world1():
    import torch
    import torch.multiprocessing as mp
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import cos_schedule
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=240) for _ in range(world)))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    # (t, refreshes, steps of the call) agree; num_played_games is each rank's own shard's
    steps0, steps1 = ([(n, st[0], st[2], st[3]) for n, st in res[r][0]] for r in (0, 1))
    assert steps0 == steps1, "the ranks took different learner steps"
    T = steps0[-1][1]
    assert T == sum(x[0] for x in steps0) and T > 2 * CI, T
    for a, b, name in zip(res[0][1], res[1][1], ("learner", "actors", "queued")):
        assert np.array_equal(a, b), f"{name} replicas diverged"
    assert np.array_equal(res[0][2], res[1][2]), "multi-step learner replicas diverged"
    assert np.isfinite(res[0][3]).all() and np.array_equal(res[0][3], res[1][3])
    # world 1: the same T (+ L) steps in one engine; θ after each step
    ref = _engine(G)
    ref.selfplay_init(abi.ENV_TICTACTOE, G, CAP)
    for m in range(12):
        ref.selfplay_move(500 + m)
    theta = torch.zeros((T + L, ref.param_count(0) + ref.param_count(1) + ref.param_count(2)), dtype=torch.float32,
                        device="cuda")
    for c0 in range(0, T + L, 200):
        n = min(200, T + L - c0)
        ref.learner_train_multi_dev(B, c0 + 1, [cos_schedule(c0 + 1 + i) for i in range(n)], None,
                                    theta[c0:].data_ptr())
    ref.sync()
    th = theta.cpu().numpy()
    assert np.array_equal(res[0][1][0], th[T - 1]), "DP loop learner θ != world-1 θ after the same steps"
    refresh = [t for t in range(CI, T + 1, CI) if t > 1]
    assert np.array_equal(res[0][1][2], th[refresh[-1] - 1]), "queued set != θ at the last refresh"
    assert np.array_equal(res[0][1][1], th[refresh[-2] - 1]), "actors != θ at the refresh before"
    assert np.array_equal(res[0][2], th[T + L - 1]), "DP multi-step learner θ != world-1 θ"
    ref.close()


def test_train_move_learn_equals_train_run():
    """mz_train_move + mz_train_learn (the host-exchanged halves) reproduce mz_train_run bit for bit."""
    from muzero_jl_amd import abi
    out = []
    for split in (False, True):
        eng = _engine(G)
        eng.selfplay_init(abi.ENV_TICTACTOE, G, CAP)
        eng.train_init(B)
        if split:
            tot = 0
            for m in range(MOVES):
                st = eng.train_learn(eng.train_move(50 + m, game_offset=7))
                tot += st[3]
            st = st[:3] + (tot,)
        else:
            st = eng.train_run(MOVES, move0=50, game_offset=7)
        out.append((st, _sets(eng), eng.replay_counts()[0]))
        eng.close()
    assert out[0][0] == out[1][0] and np.array_equal(out[0][2], out[1][2])
    for a, b in zip(out[0][1], out[1][1]):
        assert np.array_equal(a, b)
