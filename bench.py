"""bench.py — MCTS node-expansions/s (+ learner steps/s) on MI355X.

Workload (default, BASELINE.json configs[1]): TicTacToe FC net (games/
tictactoe/params.jl hyper, 74,881 fp32 params, random glorot init), 512
concurrent games per GPU, 50 simulations per move.  One step = one batched
run_mcts + select_action over the 512 games (a single search-kernel launch)
from real TicTacToe positions already resident in HBM; each step uses a fresh
RNG step key.  `--net resnet` measures configs[2] instead: the ResNet path
(Constructors.jl ResNetHP, 2 blocks x 64 filters) on 2048 games, the search
being a root launch + 50 x (tree step, network launch) + a final tree step;
its roofline is the network kernel's, timed by the engine's own HIP events on
the launch stream.  Multi-GPU: games shard across ranks (no data-path
collective) -> "scaling": "weak"; the learner leg all-reduces its gradient
bucket over RCCL.

Prints ONE JSON line on rank 0.
"""
import argparse
import glob
import dataclasses
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _self_launch():
    """`--gpus N` (N > 1) without a torch.distributed launcher (WORLD_SIZE
    unset): start N fresh child processes of this script, one rank per GPU,
    with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT
    set, and exit with their status.  This runs before torch or libmz is
    imported, so the parent never touches the GPU; the children inherit
    stdout, and rank 0 prints the one JSON line.  If a rank fails, the others
    are terminated (by their own Popen handles) and its exit code is
    returned.  Returns None when there is nothing to launch."""
    import socket
    import subprocess
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args()
    if a.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


if __name__ == "__main__":
    _rc = _self_launch()
    if _rc is not None:
        sys.exit(_rc)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before libmz: one shared HIP runtime)
import torch.distributed as dist  # noqa: E402

import _mzpkg  # noqa: E402

_mzpkg.load()
from muzero_jl_amd.abi import ENV_ATARI, ENV_CONNECT4, ENV_TICTACTOE, Engine  # noqa: E402
from muzero_jl_amd.config import cos_schedule, to_c_config, to_c_ffhp, to_c_resnet_hp  # noqa: E402
from muzero_jl_amd.games import atari_synth as atari  # noqa: E402
from muzero_jl_amd.games import connect4 as c4  # noqa: E402
from muzero_jl_amd.games import tictactoe as ttt  # noqa: E402
from muzero_jl_amd.networks import init_nets, net_macs  # noqa: E402
from muzero_jl_amd.selfplay import random_positions  # noqa: E402

METRIC = "self-play MCTS node-expansions/sec + train steps/sec, TicTacToe FC net, 1-8 GPU"
PEAK_F32 = 157.3                     # TFLOP/s, MI355X_MICROARCH.md (f32 MFMA = f32 vector peak)


def cpu_baseline(conf, hyper, nets, obs, legal, tp, budget_s=10.0, resnet=False, batch=32, threads=1):
    """The oracle (C restatement of the reference semantics) on a bounded
    sample of the same workload: `batch`-game batches of the same positions,
    the same sims/move, for `budget_s` of wall time on `threads` host threads
    (one Oracle instance each; ctypes releases the GIL during the search)."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    counts = [0] * threads
    batch = min(batch, obs.shape[0])     # fewer bench games than one batch: search them all, count what ran

    def worker(w):
        o = Oracle(to_c_config(conf), to_c_resnet_hp(hyper) if resnet else to_c_ffhp(hyper), seed=1)
        for n, wt in enumerate(nets):
            o.set_weights(n, wt)
        step = w
        while time.perf_counter() - t0 < budget_s:
            i = (step * batch) % (obs.shape[0] - batch + 1)
            o.mcts_search(obs[i:i + batch], legal[i:i + batch], tp[i:i + batch], exploration=True, rng_step=step)
            counts[w] += batch
            step += threads

    t0 = time.perf_counter()
    ts = [threading.Thread(target=worker, args=(w,)) for w in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    n_games = sum(counts)
    return dict(value=n_games * conf.num_iters / dt, unit="node-expansions/s", cores=threads, kind="port",
                sample=f"{n_games} games x {conf.num_iters} sims ({batch}-game batches of the bench positions), "
                       f"oracle/mz_oracle.c on {threads} host thread{'s' if threads > 1 else ''}, {dt:.1f} s",
                **host_cpu())


def host_cpu():
    """The host the CPU baseline ran on: logical CPUs of the machine
    (os.cpu_count: the whole box, not this job's share), the CPUs this
    process may run on, and the CPU model (/proc/cpuinfo)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return dict(host_cpus=os.cpu_count(), host_cpus_allowed=affinity, cpu_model=model)


def pmc_record(kernel, line=None):
    """(HBM bytes per launch, source file, counters) of `kernel` ("a+b": the
    sum over a launch pair) from the committed PMC summaries — profiles/pmc_*.json
    of tools/pmc_summary.py and profiles/pmc2_*.json of tools/pmc_kernels.py
    (FETCH_SIZE x2 for the 16 B/lane image reads, per MI355X_MICROARCH.md, +
    WRITE_SIZE).  The latest round wins, and among pmc2 summaries the bench
    line's own (`line` in the file name: default / resnet / atari — the same
    kernel runs different nets there).  These are the committed figures of a
    separate --pmc run of this command, not a measurement of this run: the
    line names the file (`traffic_source`).  (None, None, {}) if none."""
    if "+" in kernel:
        parts = [pmc_record(k, line) for k in kernel.split("+")]
        if any(p[0] is None for p in parts):
            return None, None, {}
        return sum(p[0] for p in parts), " + ".join(p[1] for p in parts), {}
    found = (None, None, {})
    if line:
        for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", f"pmc2_*_{line}.json"))):
            with open(pmc) as f:
                rec = json.load(f).get("kernels", {}).get(kernel)
            if rec and "hbm_bytes_per_launch_fetch_x2" in rec:
                found = (rec["hbm_bytes_per_launch_fetch_x2"], os.path.relpath(pmc, ROOT), rec)
        if found[0] is not None:
            return found
    for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        with open(pmc) as f:
            rec = json.load(f)
        if rec.get("kernel") == kernel:
            found = (rec.get("hbm_bytes_per_launch"), os.path.relpath(pmc, ROOT), rec)
    for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc2_*.json"))):
        with open(pmc) as f:
            rec = json.load(f).get("kernels", {}).get(kernel)
        if rec and "hbm_bytes_per_launch_fetch_x2" in rec:
            found = (rec["hbm_bytes_per_launch_fetch_x2"], os.path.relpath(pmc, ROOT), rec)
    return found


def bound_of(kernel, rec):
    """"mfma" for the kernels built on f32 MFMA; "valu" for the VALU-only FC
    small kernels (their PMC shows SQ_INSTS_MFMA = 0): the peak is the same
    157.3 TFLOP/s f32 vector rate, and what actually limits them is latency
    (the share of wave cycles parked is `wait_any_frac`)."""
    if rec.get("SQ_INSTS_MFMA") == 0.0 or kernel.startswith(("mz_search_small", "mz_learn_small")):
        return "valu"
    return "mfma"


def workload(game, resnet, G, S):
    if game is atari:
        return (f"synthetic Atari-like 84x84x4 observations, ResNet with the Learning.jl:175-187 downsampler "
                f"(84->6, then 2 blocks x 64 filters), 18 actions, {G} games/GPU x {S} sims/move (configs[4])")
    if game is c4:
        return (f"Connect4 6x7 {'ResNet-8 (4 blocks x 64 filters, 3x3)' if resnet else 'FC'}, {G} games/GPU x "
                f"{S} sims/move" + (" (configs[3]: 4096 games = 512/GPU x 8)" if resnet else ""))
    if resnet:
        return f"TicTacToe ResNet (2 blocks x 64 filters, 3x3), {G} games/GPU x {S} sims/move (configs[2])"
    cfg = "configs[0]-style single game" if G == 1 else "configs[1]" if (G, S) == (512, 50) else "TicTacToe FC"
    return f"TicTacToe FC (params.jl hyper), {G} games/GPU x {S} sims/move ({cfg})"


def replica_check(eng, world, leg):
    """DP replicas stay bit-identical (Learning.jl:395-397 on every rank): a
    digest of every rank's flat parameters (all three nets, Flux order) is
    all-gathered and must agree; a mismatch fails the run before the JSON line."""
    import hashlib
    h = hashlib.sha256()
    for n in range(3):
        h.update(np.ascontiguousarray(eng.get_weights(n)).tobytes())
    d = torch.tensor([int.from_bytes(h.digest()[:7], "little")], dtype=torch.int64)
    if dist.get_backend() == "nccl":                    # (RCCL gathers device tensors)
        d = d.cuda()
    got = [torch.zeros_like(d) for _ in range(world)]
    dist.all_gather(got, d)
    vals = [int(x.item()) for x in got]
    assert all(v == vals[0] for v in vals), f"{leg}: replicas diverged (parameter digests {vals})"
    REPLICA_CHECKS.append(leg)


REPLICA_CHECKS = []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--game", choices=["tictactoe", "connect4", "atari"], default="tictactoe")
    ap.add_argument("--net", choices=["fc", "resnet"], default="fc")
    ap.add_argument("--games", type=int, default=None,
                    help="games per GPU (tictactoe: fc 512, resnet 2048; connect4, atari: 512)")
    ap.add_argument("--pipeline-moves", type=int, default=20,
                    help="timed moves of the device self-play loop (0 = skip that leg)")
    ap.add_argument("--sims", type=int, default=None, help="sims per move (default 50; atari 200)")
    ap.add_argument("--learner-steps", type=int, default=50)
    ap.add_argument("--learner-chunk", type=int, default=64,
                    help="one GPU: consecutive ref_semantics learner steps per mz_learner_train_multi_dev call "
                         "(1..256, sub-chunks of 16; 1 = the one-step form only)")
    ap.add_argument("--batch", type=int, default=None,
                    help="learner batch size (default conf.batch_size = 32; SURVEY §8d config 3 also names 2048)")
    ap.add_argument("--train-moves", type=int, default=20,
                    help="timed moves of the actor-learner loop mz_train_run (0 = skip that leg)")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host threads of the oracle baseline (the box's CPU share for one GPU is 16)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--search-only", action="store_true",
                    help="the search leg only (no self-play pipeline, learner or actor-learner legs): the command "
                         "whose rocprof kernel stats cover the timed searches alone")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="(tests) ranks join a gloo group, all-reduce their rank ids on the CPU and rank 0 prints "
                         "one JSON line; no GPU call")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE = {world}"
    if args.launcher_selftest:
        if world > 1:
            dist.init_process_group("gloo")
        t = torch.tensor([float(rank + 1)])
        if world > 1:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"n_gpus": world, "rank_sum": float(t.item()), "pid": os.getpid()}), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    # one rank per GPU over RCCL ("nccl").  MZ_DIST_BACKEND=gloo with more ranks
    # than GPUs rehearses the N > 1 path on a one-GPU box (ranks share device
    # local % #GPUs; gloo all-reduces the CUDA gradient through the host)
    backend = os.environ.get("MZ_DIST_BACKEND", "nccl")
    local = local % torch.cuda.device_count() if backend != "nccl" else local
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    stream = torch.cuda.Stream(device=dev)        # non-null stream shared with libmz (events see it)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream

    game = {"connect4": c4, "atari": atari}.get(args.game, ttt)
    resnet = args.net == "resnet" or game is atari          # configs[4] is the downsampling ResNet
    S = args.sims or (200 if game is atari else 50)
    conf = dataclasses.replace(game.conf, num_iters=S)
    hyper = game.resnet_hyper if resnet else game.hyper
    A = len(conf.action_space)
    G = args.games or (2048 if resnet and game is ttt else 512)
    nets = init_nets(conf, hyper, seed=1234)              # identical replicas on every rank
    eng = Engine(conf, hyper, device=local, max_games=G, rng_seed=1)
    for n, w in enumerate(nets):
        eng.set_weights(n, w)

    if game is atari:                                     # synthetic observations, every action legal, 1 player
        obs = atari.observations(G, seed=rank)
        legal = np.ones((G, A), bool)
        tp = np.ones(G, np.int32)
    else:
        env_cls = c4.BatchedConnect4 if game is c4 else ttt.BatchedTicTacToe
        obs, legal, tp = random_positions(env_cls, G, seed=100 + rank, max_plies=6 if game is ttt else 16)
    # raw pointers cross the ABI: row-major (C-contiguous) device copies
    d_obs = torch.from_numpy(np.ascontiguousarray(obs, np.float32)).to(dev)
    d_legal = torch.from_numpy(np.ascontiguousarray(legal, np.uint8)).to(dev)
    d_tp = torch.from_numpy(np.ascontiguousarray(tp, np.int32)).to(dev)
    d_cv = torch.empty((G, A), dtype=torch.float32, device=dev)
    d_rv = torch.empty(G, dtype=torch.float32, device=dev)
    d_act = torch.empty(G, dtype=torch.int32, device=dev)

    def step(k):
        eng.mcts_search_dev(G, d_obs.data_ptr(), d_legal.data_ptr(), d_tp.data_ptr(), d_cv.data_ptr(),
                            d_rv.data_ptr(), d_act.data_ptr(), exploration=True, rng_step=k,
                            game_offset=rank * G, temperature=1.0, stream=sp)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the timed region carries no per-launch events: an event pair around every
    # launch puts marker packets between the searches (~14 us per step measured
    # against the rocprof kernel time); the per-launch duration for the roofline
    # comes from a second, instrumented pass of the same K launches below
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for k in range(args.steps):
        evs[k][0].record(stream)
        step(args.warmup + k)
        evs[k][1].record(stream)
    torch.cuda.synchronize()
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    if resnet:
        # the dominant kernel is the network launch (S per search): time it
        # with the engine's events on the launch stream over 3 more searches
        eng.debug_enable(2)
        eng.debug_kernel_time()
        for k in range(3):
            step(args.warmup + args.steps + k)
        torch.cuda.synchronize()
        t_ms, n_l = eng.debug_kernel_time()
        eng.debug_enable(0)
        kern_ms = t_ms / n_l
    eng.sync()
    acts = d_act.cpu().numpy()
    bad = np.flatnonzero(~legal[np.arange(G), acts - 1])
    assert len(bad) == 0, f"illegal action selected in games {bad[:8]} (actions {acts[bad[:8]]})"

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # ---- device self-play pipeline: the whole move loop on the
    # device — observation/stacked planes, search, env step, GameHistory and
    # replay-shard append — G games per rank, timed like the search leg
    pipe = None
    env_kind = ENV_ATARI if game is atari else ENV_CONNECT4 if game is c4 else ENV_TICTACTOE
    # replay shard: the config's capacity (Atari: 2G games of <= max_moves + 1 frames, 7 KB each)
    cap = max(G, min(conf.replay_buffer_size, 2 * G) if game is atari else conf.replay_buffer_size)
    eng.selfplay_init(env_kind, G, cap)
    mv = 1 << 20                                          # move counter (RNG step keys)
    if args.pipeline_moves > 0 and not args.search_only:
        for _ in range(3):
            eng.selfplay_move(mv, game_offset=rank * G, stream=sp)
            mv += 1
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tp0 = time.perf_counter()
        for _ in range(args.pipeline_moves):
            eng.selfplay_move(mv, game_offset=rank * G, stream=sp)
            mv += 1
        torch.cuda.synchronize()
        tpl = torch.tensor([time.perf_counter() - tp0], dtype=torch.float64, device=dev)
        eng.sync()
        if world > 1:
            dist.all_reduce(tpl, op=dist.ReduceOp.MAX)
        tpl = float(tpl.item())
        pipe = {"moves_per_s": round(world * G * args.pipeline_moves / tpl, 1),
                "node_expansions_per_s": round(world * G * S * args.pipeline_moves / tpl, 1),
                "ms_per_move": round(tpl / args.pipeline_moves * 1e3, 4), "moves": args.pipeline_moves}
    torch.cuda.synchronize()                              # (replay_counts syncs only libmz's own stream)
    while not args.search_only and eng.replay_counts()[1] == 0:   # the learner needs finished games
        eng.selfplay_move(mv, game_offset=rank * G, stream=sp)
        mv += 1
        torch.cuda.synchronize()
    if pipe is not None:
        pipe["replay"] = dict(zip(("num_played_games", "num_played_steps", "total_samples"),
                                  (int(x) for x in eng.replay_counts()[0])))

    # ---- learner leg: ref_semantics learner step at B = batch_size (32) on
    # batches sampled on the device from this rank's replay shard (§8f-2),
    # gradient bucket all-reduced over RCCL when world > 1
    B, K = args.batch or conf.batch_size, conf.num_unroll_steps
    # the global batch B is split over the ranks, each drawing B/world samples from its own shard
    Br = B // world + (1 if rank < B % world else 0)
    learner_sps = lstep_ms = lkern = learner_1step = None
    multi = None
    if not args.search_only:
        grad = torch.empty(eng.grad_count(), dtype=torch.float32, device=dev)
        losses = torch.empty(8, dtype=torch.float32, device=dev)

        def lstep(k):
            if world == 1:                                  # get_batch + unroll, losses + ADAM: one launch (FC)
                eng.learner_train_dev(B, k + 1, cos_schedule(k + 1), losses.data_ptr(), stream=sp)
                return
            # get_batch fused into the unroll (B/world samples of this rank's shard); the data term of ∇
            # exchanged, 2θ added by apply
            eng.learner_grad_sampled_dev(Br, k + 1, grad.data_ptr(), losses.data_ptr(), stream=sp)
            dist.all_reduce(grad)
            eng.learner_apply_dev(grad.data_ptr(), 1.0 / world, cos_schedule(k + 1), stream=sp)

        for k in range(5):
            lstep(k)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tl0 = time.perf_counter()
        for k in range(args.learner_steps):
            lstep(5 + k)
        torch.cuda.synchronize()
        tl = torch.tensor([time.perf_counter() - tl0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tl, op=dist.ReduceOp.MAX)
        learner_1step = learner_sps = args.learner_steps / float(tl.item())
        eng.sync()                                          # a device fault of the leg fails the run here
        # per-step device time: events around each step on the launch stream, in
        # a separate loop (recording events between steps adds host work)
        nev = 20
        lev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nev)]
        for k in range(nev):
            lev[k][0].record(stream)
            lstep(5 + args.learner_steps + k)
            lev[k][1].record(stream)
        torch.cuda.synchronize()
        lstep_ms = float(np.mean([a.elapsed_time(b) for a, b in lev]))
        tnext = 5 + args.learner_steps + nev + 1           # the next learner step number
        # the learner's dominant kernel: FC world 1 = the whole step is one launch
        # (mz_learn_small*), timed by the events around it; ResNet = the unroll
        # (chain + predictions, the pair mz_learner_variant names), timed by the engine's events on its launch stream
        if resnet:
            eng.debug_enable(4)
            eng.debug_kernel_time()
            for k in range(5):
                lstep(tnext - 1 + k)
            tnext += 5
            torch.cuda.synchronize()
            t_ms, n_l = eng.debug_kernel_time()
            eng.debug_enable(0)
            lkern, lkern_ms = eng.learner_variant(), t_ms / n_l
        else:
            # world 1: the whole step is one launch (mz_learn_small1 / _small2 by batch size, as the engine
            # records it); world > 1: unroll, all-reduce and ADAM are separate launches (no single kernel)
            lkern = eng.learner_variant() if world == 1 else None
            lkern_ms = lstep_ms
        # L consecutive steps per launch pair (mz_learner_train_multi_dev; ref_semantics, Q11: the
        # update does not read the data and PER-off batches are keyed by the step): the headline learner
        # number; the one-step form above stays in the line (learner_steps_per_s_1step).  World > 1: every
        # rank runs the same update on B/world samples of its own shard (the data term of ∇ is zero in
        # ref_semantics, so no gradient crosses the ranks) and the per-step losses are averaged over the
        # ranks once per call
        if args.learner_chunk > 1:
            L = args.learner_chunk
            lm = torch.empty((L, 8), dtype=torch.float32, device=dev)

            def lchunk(t0):
                eng.learner_train_multi_dev(Br, t0, [cos_schedule(t0 + i) for i in range(L)], lm.data_ptr(),
                                            stream=sp)
                if world > 1:
                    dist.all_reduce(lm)
                    lm.div_(world)

            for _ in range(2):
                lchunk(tnext)
                tnext += L
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            nch = max(4, (args.learner_steps * 8 + L - 1) // L)
            tm0 = time.perf_counter()
            for _ in range(nch):
                lchunk(tnext)
                tnext += L
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            tm = torch.tensor([time.perf_counter() - tm0], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(tm, op=dist.ReduceOp.MAX)
            tm = float(tm.item())
            eng.sync()
            mev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
            for a, b in mev:
                a.record(stream)
                lchunk(tnext)
                tnext += L
                b.record(stream)
            torch.cuda.synchronize()
            chunk_ms = float(np.mean([a.elapsed_time(b) for a, b in mev]))
            eng.debug_enable(4)                             # the unroll launches alone (engine events)
            eng.debug_kernel_time()
            for _ in range(5):
                lchunk(tnext)
                tnext += L
            torch.cuda.synchronize()
            t_ms, n_l = eng.debug_kernel_time()
            eng.debug_enable(0)
            # the unroll launch(es): FC mz_learn_multi*, ResNet the mz_runroll_* kernels of the variant
            parts = eng.learner_variant().split("+")
            lkern = "+".join(k for k in parts if k.startswith("mz_runroll")) if resnet else parts[-1]
            lkern_ms = t_ms / n_l
            learner_sps = nch * L / tm
            lstep_ms = chunk_ms / L
            multi = {"steps_per_call": L, "steps_per_unroll_launch": 5 * L / n_l,
                     "learner_steps_per_s": round(learner_sps, 1), "call_ms": round(chunk_ms, 5),
                     "unroll_launch_ms": round(lkern_ms, 5), "kernels": eng.learner_variant(),
                     "steps_timed": nch * L}
        if world > 1:                                       # the DP replicas must still be bit-identical
            replica_check(eng, world, "learner")

    # ---- corrected-gradient learner (MZ_LEARN_CORRECTED; FC and ResNet nets): real
    # backprop through the unroll on MFMA; with world > 1 the exchanged
    # gradient is data-dependent
    corrected = None
    if args.learner_steps > 0 and not args.search_only:
        from muzero_jl_amd.abi import LEARN_CORRECTED, LEARN_REF_SEMANTICS
        eng.learner_set_mode(LEARN_CORRECTED)
        for k in range(3):
            lstep(1000 + k)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tc0 = time.perf_counter()
        ncs = max(10, args.learner_steps // 2)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for k in range(ncs):
            lstep(1003 + k)
        ev1.record(stream)
        torch.cuda.synchronize()
        tcs = torch.tensor([time.perf_counter() - tc0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tcs, op=dist.ReduceOp.MAX)
        f_fb = 3 * 2 * Br * (net_macs(conf, hyper, 0) + (K + 1) * net_macs(conf, hyper, 1) +
                            K * net_macs(conf, hyper, 2))     # forward + backward (dX, dW) ≈ 3x forward
        cms = ev0.elapsed_time(ev1) / ncs
        corrected = {"learner_steps_per_s": round(ncs / float(tcs.item()), 1), "step_ms": round(cms, 5),
                     "flop_per_step": f_fb, "tflops": round(f_fb / (cms * 1e-3) / 1e12, 4),
                     "frac": round(f_fb / (cms * 1e-3) / 1e12 / PEAK_F32, 5),
                     "kernels": (("mz_rp_sample + mz_dsbp_fwd + mz_rbp_sample + mz_dsbp_bwd + mz_dsbp_dw + "
                                  "mz_rbp_dw + mz_bp_fold + mz_adam_kernel") if game is atari else
                                 "mz_rp_sample + mz_rbp_sample + mz_rbp_dw + mz_bp_fold + mz_adam_kernel"
                                 if resnet else "mz_rp_sample + mz_bp_tile_lv%s + mz_bp_dw + mz_bp_fold + mz_adam_kernel"
                                 % ("" if hyper.use_batch_norm else "_nobn"))}
        eng.learner_set_mode(LEARN_REF_SEMANTICS)
        eng.sync()
        if world > 1:
            replica_check(eng, world, "learner_corrected")

    # ---- actor-learner loop (row a12, self_play! || learning!, Q16): self-play
    # moves with the actors' nets and one learner step per finished game, the
    # actors refreshed one checkpoint behind (mz_train_run).  World > 1: each rank
    # plays its own G games; per move the finished-game counts are summed over the
    # ranks and every rank takes that many learner steps on B/world samples of its
    # shard (mz_train_move -> all_reduce -> mz_train_learn), so the replicas stay
    # identical
    train = None
    if args.train_moves > 0 and not args.search_only:
        eng.selfplay_init(env_kind, G, cap)
        eng.train_init(Br)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)

        def train_moves(n, m0):
            if world == 1:
                return eng.train_run(n, move0=m0, game_offset=rank * G, stream=sp)
            tot = 0
            for m in range(n):
                cnt.fill_(eng.train_move(m0 + m, game_offset=rank * G, stream=sp))
                dist.all_reduce(cnt)
                st_ = eng.train_learn(int(cnt.item()), stream=sp)
                tot += st_[3]
            return st_[:3] + (tot,)

        train_moves(3, mv)
        mv += 3
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tt0 = time.perf_counter()
        st0 = train_moves(args.train_moves, mv)
        torch.cuda.synchronize()
        ttr = torch.tensor([time.perf_counter() - tt0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(ttr, op=dist.ReduceOp.MAX)
        ttr = float(ttr.item())
        eng.sync()
        mv += args.train_moves
        if world > 1:
            replica_check(eng, world, "train_loop")
        train = {"moves": args.train_moves, "ms_per_move": round(ttr / args.train_moves * 1e3, 4),
                 "node_expansions_per_s": round(world * G * S * args.train_moves / ttr, 1),
                 "learner_steps": st0[3], "learner_steps_per_s": round(st0[3] / ttr, 1),
                 "games_finished": st0[1], "actor_refreshes": st0[2],
                 "schedule": "mz_train_run: one self-play move of all games with the actors' nets, then one "
                             "learner step (B = batch_size, device get_batch) per finished game; actors take "
                             "the queued nets every checkpoint_interval steps; the learner steps of a move run "
                             "as one multi-step chunk across the refresh points" +
                             ("; world > 1: mz_train_move, the finished-game count all-reduced, mz_train_learn "
                              "with B/world samples per rank" if world > 1 else "")}

    if rank == 0:
        total_exp = world * G * S * args.steps
        value = total_exp / elapsed
        f_exp = 2 * (net_macs(conf, hyper, 1) + net_macs(conf, hyper, 2))   # prediction + dynamics
        f_root = 2 * (net_macs(conf, hyper, 0) + net_macs(conf, hyper, 1))  # representation + prediction
        # FC: one launch is the whole search; ResNet: one network launch = one
        # simulation's prediction + dynamics over the G games
        flop_launch = G * f_exp if resnet else G * S * f_exp + G * f_root
        achieved = flop_launch / (kern_ms * 1e-3) / 1e12
        # HBM bytes per launch from the committed PMC summary of THIS kernel
        # variant (tools/pmc_summary.py; latest round wins), else null
        variant = "mz_rsearch_nets" if resnet else eng.search_variant()
        pmc_line = "atari" if game is atari else "resnet" if resnet else "default" if game is ttt else None
        traffic, traffic_src, search_pmc = pmc_record(variant, pmc_line)
        # learner roofline (north_star: HBM GB/s and MFMA utilisation of the
        # learner): algorithmic FLOP of the unroll (2·B·(repr +
        # (K+1)·pred + K·dyn) MACs) + ADAM (~10 FLOP/param, FC one-launch step);
        # algorithmic bytes of the ADAM step = 28 B/param (θ, m, v read and
        # written, the image scatter; FC and ResNet alike), traffic from the
        # committed PMC summary of the same kernel
        lroof = None
        if lkern is not None:
            nparam = sum(int(x.size) for x in nets)
            f_unroll = 2 * Br * (net_macs(conf, hyper, 0) + (K + 1) * net_macs(conf, hyper, 1) +
                                K * net_macs(conf, hyper, 2))
            # ResNet: the timed launch pair is the unroll alone (ADAM runs in the loss kernel after it)
            lflop = f_unroll + (0 if resnet else 10 * nparam)
            # FC: the one-launch step's ADAM (28 B/param); ResNet: the unroll pair alone reads the weights
            # once (4 B/param), the batch's observations and actions, and writes value / reward / A logits
            # per (sample, step)
            lbytes = 28 * nparam if not resnet else \
                4 * nparam + 4 * Br * (obs.shape[1] + (K + 1)) + 4 * Br * (K + 1) * (A + 2)
            lbytes_step = 28 * nparam
            if multi:
                # mz_learn_multi*: L unrolls + loss terms per launch (the ADAM chain runs in mz_learn_chain):
                # each step reads its θ image (4 B/param), its batch (observations, actions, value / policy
                # targets, gradient_scale) and writes its read-outs and loss terms
                Lm = multi["steps_per_unroll_launch"]
                lflop = Lm * f_unroll
                lbytes = Lm * (4 * nparam + 4 * Br * (obs.shape[1] + 2 * (K + 1) + (K + 1) * A + 1) +
                               4 * Br * (K + 1) * (A + 4)) if not resnet else Lm * lbytes
                # (ResNet: the unroll launches per step as the one-step form; the losses run after them)
            lach = lflop / (lkern_ms * 1e-3) / 1e12
            ltraffic, ltraffic_src, lpmc = pmc_record(lkern, pmc_line)
            hbm_gbs = (ltraffic if ltraffic else lbytes) / (lkern_ms * 1e-3) / 1e9
            lroof = {"bound": bound_of(lkern, lpmc), "achieved": round(lach, 4), "peak": PEAK_F32,
                     "unit": "TFLOP/s", "frac": round(lach / PEAK_F32, 5), "traffic": ltraffic,
                     "traffic_source": ltraffic_src, "kernel": lkern,
                     "kernel_ms": round(lkern_ms, 5), "flop_per_launch": lflop,
                     "hbm_bytes_algorithmic": lbytes, "hbm_bytes_algorithmic_per_step": lbytes_step,
                     "hbm_GBps": round(hbm_gbs, 2), "hbm_frac": round(hbm_gbs / 8000.0, 5),
                     "mfma_util_chip": lpmc.get("mfma_util_chip")}
        cpu = cpu1 = None
        if world == 1 and not args.no_cpu:
            nt = max(1, min(args.cpu_threads, os.cpu_count() or 1))
            cpu = cpu_baseline(conf, hyper, nets, obs, legal, tp, args.cpu_budget, resnet,
                               batch=1 if game is atari else 32, threads=nt)
            cpu1 = cpu_baseline(conf, hyper, nets, obs, legal, tp, args.cpu_budget, resnet,
                                batch=1 if game is atari else 32, threads=1)
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "node-expansions/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": ("synthetic: 84x84x4 U[0,1) Philox observations for the timed searches, random glorot weights; "
                     "learner batches sampled on the device from the self-play shard of the synthetic Atari-like "
                     "env (games/atari_synth.py)" if game is atari else
                     f"synthetic: random-play {game.__name__.split('.')[-1]} positions, random glorot weights; "
                     "learner batches sampled on the device from the self-play replay shard"),
            "config": {"workload": workload(game, resnet, G, S),
                       "games_per_gpu": G, "sims_per_move": S, "global_games": G * world,
                       "parallelism": f"games sharded x{world}, learner dp{world} (global batch {B}, "
                                      f"{B // world}{'+' if B % world else ''} samples per rank)"},
            "learner_steps_per_s": round(learner_sps, 1) if learner_sps else None,
            "learner_steps_per_s_1step": round(learner_1step, 1) if learner_1step else None,
            "learner_multi": multi,
            "replica_checks": REPLICA_CHECKS if world > 1 else None,
            "learner_step_ms": round(lstep_ms, 5) if lstep_ms else None,
            "learner_roofline": lroof,
            "learner_corrected": corrected,
            "train_loop": train,
            "learner_config": {"batch_size": B, "batch_per_rank": Br, "num_unroll_steps": K, "mode": "ref_semantics",
                               "note": ("learner_steps_per_s is the multi-step form (learner_multi), valid because "
                                        "in ref_semantics the update θ <- ADAM(θ, 2θ) reads no data (Q11); "
                                        "learner_steps_per_s_1step is the one-step form, the rounds 1-4 metric"
                                        if multi else None),
                               "form": (f"mz_learner_train_multi_dev: {multi['steps_per_call']} consecutive steps "
                                        f"per call, {multi['steps_per_unroll_launch']:g} per unroll launch "
                                        f"({multi['kernels']}); the one-step form (mz_learner_train_dev) in "
                                        "learner_steps_per_s_1step" if multi else "one step per call"),
                               "batch_source": (("mz_learner_train_dev: one launch — unroll + losses, ADAM into the second "
                                 "image set, and step t+1's device get_batch + make_target into the other batch "
                                 "set (step t's was drawn by the previous launch)" if not resnet else
                                 "mz_learner_train_dev: device get_batch + make_target, ResNet unroll chain + "
                                 "predictions, losses with ADAM") if world == 1 else
                                "multi-step form: mz_learner_train_multi_dev on B/world samples of each rank's "
                                "shard, the per-step losses all-reduced once per call (the data term of the "
                                "gradient is zero in ref_semantics); one-step form and corrected mode: "
                                "mz_learner_grad_sampled_dev (device get_batch fused into the unroll) + RCCL "
                                "all-reduce + mz_learner_apply_dev")},
            "selfplay_pipeline": pipe,
            "roofline": {"bound": bound_of(variant, search_pmc), "achieved": round(achieved, 4), "peak": PEAK_F32,
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_F32, 5), "traffic": traffic,
                         "traffic_source": traffic_src, "kernel": variant, "kernel_ms": round(kern_ms, 4),
                         "flop_per_launch": flop_launch, "wait_any_frac": search_pmc.get("wait_any_frac"),
                         "mfma_util_chip": search_pmc.get("mfma_util_chip")},
            "cpu_baseline": cpu,
            "cpu_baseline_1thread": cpu1,    # the reference's single self-play worker (main.jl:2)
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
