"""Data-parallel learner through libmz with two spawned ranks on cuda:0
(gloo carries the all-reduce; RCCL needs one GPU per rank, so the RCCL path
is exercised only at world 1 on a one-GPU box, test_selfplay_gpu.py).

Each rank plays its own self-play shard (game_offset = rank·G), draws its
batch from it, computes a DATA-DEPENDENT gradient (the corrected learner,
MZ_LEARN_CORRECTED — in ref_semantics every rank's gradient is 2θ, which
would make the exchange vacuous), sums the gradients over the ranks and
applies ADAM with scale 1/world (mz_learner_grad_sampled_dev →
all_reduce → mz_learner_apply_dev).  Checked:
* the two ranks' gradients differ, and the replicas stay bit-identical;
* the replicas equal a single-process run that computes both shards'
  gradients with two engines, sums them (a + b = b + a: two ranks sum
  exactly as gloo does) and applies the same scaled ADAM step — so the
  exchange's count, dtype and 1/world scaling are right;
* the sharded self-play (rank r, game_offset r·G) equals one engine playing
  all 2G games.
Two nets: the TicTacToe FC net and configs[3]'s Connect4 ResNet-8 (the
exchange of that config's all-reduce on a real, data-dependent gradient).
SURVEY §8e; src/Learning.jl:385-397 (the update the gradient feeds)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G, CAP, B, MOVES, STEPS = 16, 64, 24, 14, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine(rank_offset, kind="fc"):
    import dataclasses
    from muzero_jl_amd import abi
    from muzero_jl_amd.games import connect4 as c4
    from muzero_jl_amd.games import tictactoe as ttt
    from muzero_jl_amd.networks import init_nets
    mod = c4 if kind == "c4_resnet" else ttt
    hyper = mod.resnet_hyper if kind == "c4_resnet" else mod.hyper
    conf = dataclasses.replace(mod.conf, num_iters=6, batch_size=B, replay_buffer_size=CAP)
    eng = abi.Engine(conf, hyper, device=0, max_games=2 * G, rng_seed=11)
    for n, w in enumerate(init_nets(conf, hyper, seed=12)):
        eng.set_weights(n, w)
    eng.learner_set_mode(abi.LEARN_CORRECTED)
    eng.kind_ = kind
    return eng


def _play(eng, G_, offset):
    from muzero_jl_amd import abi
    eng.selfplay_init(abi.ENV_CONNECT4 if eng.kind_ == "c4_resnet" else abi.ENV_TICTACTOE, G_, CAP)
    for m in range(MOVES if eng.kind_ == "fc" else 3 * MOVES):    # Connect4 games run longer
        eng.selfplay_move(100 + m, game_offset=offset)


def _eta(kind, t):
    """Cos(λ0=1e-4, λ1=1e-1) for the FC net; the deep ResNet-8 at λ1 = 0.1
    overflows to non-finite outputs within three ADAM steps, so 1e-4 there."""
    from muzero_jl_amd.config import cos_schedule
    return cos_schedule(t) if kind == "fc" else 1e-4


def _worker(rank, world, port, q, kind):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist
    import _mzpkg
    _mzpkg.load()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _engine(rank * G, kind)
    _play(eng, G, rank * G)
    grad = torch.zeros(eng.grad_count(), dtype=torch.float32, device="cuda")
    losses = torch.zeros(8, dtype=torch.float32, device="cuda")
    local = []
    for t in range(1, STEPS + 1):
        eng.learner_grad_sampled_dev(B, t, grad.data_ptr(), losses.data_ptr())
        eng.sync()
        local.append(grad.cpu().numpy().copy())
        dist.all_reduce(grad)                                   # sum over ranks
        torch.cuda.synchronize()
        eng.learner_apply_dev(grad.data_ptr(), 1.0 / world, _eta(kind, t))
        eng.sync()
    flat = np.concatenate([eng.get_weights(n) for n in range(3)])
    ln, board, player = eng.selfplay_slots()
    counts, _ = eng.replay_counts()
    q.put((rank, flat, np.stack(local), ln, board, player, counts))
    dist.barrier()
    dist.destroy_process_group()
    eng.close()


@pytest.mark.parametrize("kind", ["fc", "c4_resnet"])
def test_two_rank_dp_through_libmz(kind):
    import torch
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, kind)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=240) for _ in range(world)))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    w0, g0 = res[0][0], res[0][1]
    w1, g1 = res[1][0], res[1][1]
    assert not np.array_equal(g0[0], g1[0]), "the ranks' gradients do not depend on their data"
    assert np.array_equal(w0, w1), "replicas diverged"
    # single-process reference: both shards' gradients, summed, one scaled ADAM step
    refs = [_engine(0, kind), _engine(G, kind)]
    for r, e in enumerate(refs):
        _play(e, G, r * G)
    grads = [torch.zeros(refs[0].grad_count(), dtype=torch.float32, device="cuda") for _ in refs]
    for t in range(1, STEPS + 1):
        for e, g in zip(refs, grads):
            e.learner_grad_sampled_dev(B, t, g.data_ptr())
            e.sync()
        assert np.array_equal(grads[0].cpu().numpy(), g0[t - 1]) and np.array_equal(grads[1].cpu().numpy(), g1[t - 1])
        tot = grads[0] + grads[1]
        torch.cuda.synchronize()
        for e in refs:
            e.learner_apply_dev(tot.data_ptr(), 0.5, _eta(kind, t))
            e.sync()
    ref_w = np.concatenate([refs[0].get_weights(n) for n in range(3)])
    assert np.array_equal(ref_w, w0), "the DP update differs from sum-then-scale of the shards' gradients"
    # sharded self-play = one engine with all 2G games
    full = _engine(0, kind)
    _play(full, 2 * G, 0)
    ln, board, player = full.selfplay_slots()
    assert np.array_equal(ln, np.concatenate([res[0][2], res[1][2]]))
    assert np.array_equal(board, np.concatenate([res[0][3], res[1][3]]))
    assert np.array_equal(player, np.concatenate([res[0][4], res[1][4]]))
    for e in refs + [full]:
        e.close()
