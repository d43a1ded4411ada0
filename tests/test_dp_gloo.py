"""Multi-process (world_size 2, gloo, CPU) tests of the data-parallel paths:
(1) the learner's gradient exchange (sum all-reduce, scale 1/world) keeps the
replicas bit-identical to the single-process ref_semantics update;
(2) self-play sharding by game_offset = rank * G reproduces the unsharded
search (games are independent; no data-path collective)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import dataclasses
    import ctypes
    import torch
    import torch.distributed as dist
    import _mzpkg
    _mzpkg.load()
    from muzero_jl_amd.config import to_c_config, to_c_ffhp, cos_schedule
    from muzero_jl_amd.games import tictactoe as ttt
    from muzero_jl_amd.learning import reduce_mean_grad
    from muzero_jl_amd.networks import init_nets
    from oracle import Oracle, lib
    from conftest import random_positions
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nets = init_nets(ttt.conf, ttt.hyper, seed=8)
    theta = np.concatenate(nets)
    # (1) gradient exchange: every rank's ref_semantics gradient is 2θ
    L = lib()
    m = np.zeros_like(theta)
    v = np.zeros_like(theta)
    bp = np.array([0.9, 0.999])
    for t in range(1, 4):
        g = torch.from_numpy(theta * np.float32(2))
        reduce_mean_grad(g, world, dist.all_reduce)
        assert np.array_equal(g.numpy(), theta * np.float32(2))   # exact for power-of-two world
        L.ora_adam_2theta(theta.ctypes.data_as(ctypes.c_void_p), m.ctypes.data_as(ctypes.c_void_p),
                          v.ctypes.data_as(ctypes.c_void_p), theta.size, bp.ctypes.data_as(ctypes.c_void_p),
                          cos_schedule(t))
        bp = bp * np.array([0.9, 0.999])
    gathered = [torch.zeros(theta.size) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(theta).to(torch.float32))
    same = all(torch.equal(gathered[0], x) for x in gathered)
    # (2) sharded search
    conf = dataclasses.replace(ttt.conf, num_iters=8)
    o = Oracle(to_c_config(conf), to_c_ffhp(ttt.hyper), seed=3)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
    G = 4
    obs, legal, tp = random_positions(G * world, 55)
    sl = slice(rank * G, (rank + 1) * G)
    _, _, act = o.mcts_search(obs[sl], legal[sl], tp[sl], rng_step=9, game_offset=rank * G)
    acts = [torch.zeros(G, dtype=torch.int32) for _ in range(world)]
    dist.all_gather(acts, torch.from_numpy(act))
    if rank == 0:
        _, _, full = o.mcts_search(obs, legal, tp, rng_step=9, game_offset=0)
        q.put((same, np.array_equal(torch.cat(acts).numpy(), full), theta.copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_dp_and_sharding():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    same, shard_ok, theta = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert same, "replicas diverged"
    assert shard_ok, "sharded search differs from the unsharded one"
