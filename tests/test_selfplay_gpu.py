"""Device self-play and replay shard through the C ABI,
against the host driver (selfplay.BatchedSelfPlay over the same engine search
and the numpy envs) and the host ReplayBuffer: finished games, games in
progress, replay counters, FIFO eviction and get_batch/make_target samples,
bit for bit; then a learner step fed straight from the device batch."""
import dataclasses

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _env(kind):
    from muzero_jl_amd import abi
    from muzero_jl_amd.games import connect4, tictactoe
    if kind == "ttt":
        return tictactoe, tictactoe.BatchedTicTacToe, abi.ENV_TICTACTOE
    return connect4, connect4.BatchedConnect4, abi.ENV_CONNECT4


def _engines(mod, conf, hyper, G, seed=5):
    from muzero_jl_amd import abi
    from muzero_jl_amd.networks import init_nets
    nets = init_nets(conf, hyper, seed=seed + 100)
    out = []
    for _ in range(2):
        e = abi.Engine(conf, hyper, device=0, max_games=G, rng_seed=seed)
        for n, w in enumerate(nets):
            e.set_weights(n, w)
        out.append(e)
    return out


def _same_game(dev, host, osz):
    a, b = dev.as_arrays(), host.as_arrays()
    assert np.array_equal(a["observation"].reshape(-1, osz), b["observation"].reshape(-1, osz))
    for k in ("action", "reward", "to_play", "child_visits", "root_values"):
        assert np.array_equal(a[k], b[k]), k


def _play_both(kind, G, moves, cap, S=6, resnet=False, step0=100, temperature=1.0, thr=None):
    from muzero_jl_amd.selfplay import BatchedSelfPlay
    mod, env_cls, env_kind = _env(kind)
    conf = dataclasses.replace(mod.conf, num_iters=S, replay_buffer_size=cap, temperature_threshold=thr)
    hyper = mod.resnet_hyper if resnet else mod.hyper
    eh, ed = _engines(mod, conf, hyper, G)
    sp = BatchedSelfPlay(eh, env_cls, G, game_offset=7, step0=step0)
    ed.selfplay_init(env_kind, G, cap)
    for m in range(moves):
        sp.play_move(temperature)
        ed.selfplay_move(step0 + m, game_offset=7, temperature=temperature)
    return conf, sp, eh, ed


@pytest.mark.parametrize("kind,G,moves", [("ttt", 24, 13), ("c4", 12, 30)])
def test_device_selfplay_matches_host(kind, G, moves):
    conf, sp, eh, ed = _play_both(kind, G, moves, cap=8 * G)
    osz = int(np.prod(conf.observation_shape))
    counts, held = ed.replay_counts()
    assert counts[0] == len(sp.finished) and held == len(sp.finished) and held > 0
    assert counts[1] == sum(len(h.root_values) for h in sp.finished) == counts[2]
    for i, h in enumerate(sp.finished):
        _same_game(ed.replay_get_game(i), h, osz)
    ln, board, player = ed.selfplay_slots()
    assert np.array_equal(ln, [len(h.action_history) for h in sp.histories])
    assert np.array_equal(board, sp.env.board.astype(np.uint8)) and np.array_equal(player, sp.env.player)
    eh.close(); ed.close()


@pytest.mark.parametrize("kind,resnet", [("ttt", False), ("ttt", True), ("c4", False)])
def test_temperature_threshold_matches_host(kind, resnet):
    """conf.temperature_threshold (SelfPlay.jl:344-346): once a game has
    recorded that many moves it plays at temperature 0 — per slot on the
    device (mz_sp_prepare writes each slot's temperature), per game on the
    host; finished games and games in progress agree move for move."""
    G, thr = 16, 2
    conf, sp, eh, ed = _play_both(kind, G, 14, cap=8 * G, S=5, resnet=resnet, thr=thr)
    osz = int(np.prod(conf.observation_shape))
    counts, held = ed.replay_counts()
    assert counts[0] == len(sp.finished) > 0
    for i, h in enumerate(sp.finished):
        _same_game(ed.replay_get_game(i), h, osz)
    ln, board, _ = ed.selfplay_slots()
    assert np.array_equal(ln, [len(h.action_history) for h in sp.histories])
    assert np.array_equal(board, sp.env.board.astype(np.uint8))
    eh.close(); ed.close()


def test_device_selfplay_resnet_matches_host():
    conf, sp, eh, ed = _play_both("ttt", 16, 11, cap=64, S=4, resnet=True)
    counts, held = ed.replay_counts()
    assert counts[0] == len(sp.finished) > 0
    for i, h in enumerate(sp.finished):
        _same_game(ed.replay_get_game(i), h, 27)
    eh.close(); ed.close()


def test_replay_fifo_and_sample_match_host():
    """cap = G: the FIFO evicts; counters, held games and samples follow the
    host ReplayBuffer fed the same finished games in the same order."""
    from muzero_jl_amd.replay_buffer import ReplayBuffer
    G = 16
    conf, sp, eh, ed = _play_both("ttt", G, 30, cap=G)
    rb = ReplayBuffer(conf, seed=5)
    for h in sp.finished:
        rb.save_game(h)
    counts, held = ed.replay_counts()
    assert len(sp.finished) > G                                  # eviction happened
    assert (counts[0], counts[1], counts[2]) == (rb.num_played_games, rb.num_played_steps, rb.total_samples)
    assert held == len(rb) == G
    for i, (gid, h) in enumerate(rb.buffer.items()):
        _same_game(ed.replay_get_game(i), h, 27)
    for step in (1, 2, 77):
        B = 40
        conf_b = dataclasses.replace(conf, batch_size=B)
        rb.conf = conf_b
        idx_h, bh = rb.get_batch(step)
        b, idx_d = ed.replay_sample(B, step, index=True)
        bd = ed.batch_to_host(b)
        assert [tuple(x) for x in idx_d] == [tuple(x) for x in idx_h]
        for k in bh:
            assert np.array_equal(bd[k], bh[k]), (step, k)
    eh.close(); ed.close()


def test_learner_step_from_device_batch():
    """mz_replay_sample -> mz_learner_grad_dev/apply: same losses and weights as
    mz_learner_step on the host-assembled batch of the same samples."""
    import torch
    from muzero_jl_amd.config import cos_schedule
    from muzero_jl_amd.replay_buffer import ReplayBuffer
    G = 16
    conf, sp, eh, ed = _play_both("ttt", G, 12, cap=64)
    rb = ReplayBuffer(dataclasses.replace(conf, batch_size=32), seed=5)
    for h in sp.finished:
        rb.save_game(h)
    for step in (1, 2, 3):
        _, bh = rb.get_batch(step)
        lh = eh.learner_step(bh, cos_schedule(step))
        b, _ = ed.replay_sample(32, step)
        grad = torch.empty(ed.grad_count(), dtype=torch.float32, device="cuda")
        losses = torch.empty(8, dtype=torch.float32, device="cuda")
        ed.learner_grad_dev([b.observation, b.actions, b.target_values, b.target_rewards, b.target_policies,
                             b.gradient_scale], 32, grad.data_ptr(), losses.data_ptr())
        ed.learner_apply_dev(grad.data_ptr(), 1.0, cos_schedule(step))
        ed.sync()
        assert np.array_equal(losses.cpu().numpy()[:6], lh)
        for n in range(3):
            assert np.array_equal(ed.get_weights(n), eh.get_weights(n))
    eh.close(); ed.close()


def test_selfplay_rejects_bad_setup(ttt):
    from muzero_jl_amd import abi
    from muzero_jl_amd.abi import MzError
    e = abi.Engine(ttt.conf, ttt.hyper, device=0, max_games=8, rng_seed=1)
    with pytest.raises(MzError, match="Connect4 needs"):
        e.selfplay_init(abi.ENV_CONNECT4, 8, 8)
    with pytest.raises(MzError, match="replay_games"):
        e.selfplay_init(abi.ENV_TICTACTOE, 8, 4)
    with pytest.raises(MzError, match="mz_selfplay_init first"):
        e.selfplay_move(0)
    e.selfplay_init(abi.ENV_TICTACTOE, 8, 8)
    with pytest.raises(MzError, match="empty"):
        e.replay_sample(4, 1)
    e.close()


def _device_pair(kind, G, moves, cap, resnet=False):
    """Two engines with the same weights whose device self-play fills
    identical replay shards."""
    mod, _, env_kind = _env(kind)
    conf = dataclasses.replace(mod.conf, num_iters=6, replay_buffer_size=cap)
    e1, e2 = _engines(mod, conf, mod.resnet_hyper if resnet else mod.hyper, G)
    for e in (e1, e2):
        e.selfplay_init(env_kind, G, cap)
        for m in range(moves):
            e.selfplay_move(100 + m, game_offset=7)
    return e1, e2


@pytest.mark.parametrize("kind,resnet,B", [("ttt", False, 32), ("ttt", False, 40), ("c4", False, 24),
                                           ("ttt", False, 1100), ("ttt", True, 32)])
def test_fused_learner_matches_separate_calls(kind, resnet, B):
    """mz_learner_train_dev (sampling fused into the unroll, ADAM into the loss
    kernel) and mz_learner_grad_sampled_dev + apply == mz_replay_sample +
    mz_learner_grad_dev + mz_learner_apply_dev, bit for bit: losses, weights."""
    import torch
    from muzero_jl_amd.config import cos_schedule
    e1, e2 = _device_pair(kind, 16, 14 if kind == "ttt" else 30, cap=64, resnet=resnet)
    assert e1.replay_counts()[0][0] > 0
    grad = torch.empty(e1.grad_count(), dtype=torch.float32, device="cuda")
    l1 = torch.empty(8, dtype=torch.float32, device="cuda")
    l2 = torch.empty(8, dtype=torch.float32, device="cuda")
    for step in (1, 2, 3, 4):
        eta = cos_schedule(step)
        b, _ = e1.replay_sample(B, step)
        e1.learner_grad_dev([b.observation, b.actions, b.target_values, b.target_rewards, b.target_policies,
                             b.gradient_scale], B, grad.data_ptr(), l1.data_ptr())
        e1.learner_apply_dev(grad.data_ptr(), 1.0, eta)
        if step % 2:
            e2.learner_train_dev(B, step, eta, l2.data_ptr())
        else:
            g2 = torch.empty_like(grad)
            e2.learner_grad_sampled_dev(B, step, g2.data_ptr(), l2.data_ptr())
            e2.learner_apply_dev(g2.data_ptr(), 1.0, eta)
        e1.sync(); e2.sync()
        assert np.array_equal(l1.cpu().numpy()[:6], l2.cpu().numpy()[:6]), step
        for n in range(3):
            assert np.array_equal(e1.get_weights(n), e2.get_weights(n)), (step, n)
    e1.close(); e2.close()


@pytest.mark.parametrize("kind,B", [("ttt", 32), ("ttt", 40), ("c4", 24)])
def test_batch_prefetch_matches_in_place_sampling(kind, B, monkeypatch):
    """The one-launch learner samples step t+1's batch during step t (the
    other batch set); a prefetched set is used only while the shard, the step
    and B still match.  Runs with the prefetch and with MZ_NO_BATCH_PREFETCH=1
    stay bit-identical across every way the match can break: consecutive steps
    (prefetch used), a step gap, a self-play move storing games, a separate
    mz_replay_sample (refills set 0), a split learner step, a batch size change."""
    import torch
    from muzero_jl_amd.config import cos_schedule
    mod, _, env_kind = _env(kind)
    moves = 14 if kind == "ttt" else 30
    e1, e2 = _device_pair(kind, 16, moves, cap=64)
    l1 = torch.empty(8, dtype=torch.float32, device="cuda")
    l2 = torch.empty(8, dtype=torch.float32, device="cuda")
    grad = torch.empty(e1.grad_count(), dtype=torch.float32, device="cuda")
    plan = [("t", 1), ("t", 2), ("t", 3), ("t", 5), ("t", 6), ("move", 0), ("t", 7), ("t", 8), ("sample", 9),
            ("t", 9), ("t", 10), ("split", 11), ("t", 12), ("t", 13), ("B", 14), ("t", 15), ("t", 16)]
    for eng, lo, pf in ((e1, l1, False), (e2, l2, True)):
        if pf:
            monkeypatch.delenv("MZ_NO_BATCH_PREFETCH", raising=False)
        else:
            monkeypatch.setenv("MZ_NO_BATCH_PREFETCH", "1")
        b_cur = B
        for op, step in plan:
            if op == "t":
                eng.learner_train_dev(b_cur, step, cos_schedule(step), lo.data_ptr())
            elif op == "move":
                eng.selfplay_move(100 + moves, game_offset=7)
            elif op == "sample":
                eng.replay_sample(b_cur, step)
            elif op == "split":
                eng.learner_grad_sampled_dev(b_cur, step, grad.data_ptr(), lo.data_ptr())
                eng.learner_apply_dev(grad.data_ptr(), 1.0, cos_schedule(step))
            else:
                b_cur = B + 8
        eng.sync()
    monkeypatch.delenv("MZ_NO_BATCH_PREFETCH", raising=False)
    assert np.array_equal(l1.cpu().numpy()[:6], l2.cpu().numpy()[:6])
    for n in range(3):
        assert np.array_equal(e1.get_weights(n), e2.get_weights(n)), n
    e1.close(); e2.close()


@pytest.mark.parametrize("kind,opp,mzp", [("ttt", "random", 1), ("ttt", "random", 2), ("c4", "random", 2),
                                          ("ttt", "self", 1)])
def test_evaluation_play_matches_host(kind, opp, mzp):
    """competitive_play! on the device (mz_selfplay_mode(SP_EVAL)): random
    opponent moves, temperature 0, games tallied instead of saved — the same
    games as the host driver (BatchedSelfPlay(opponent=...)) move for move."""
    from muzero_jl_amd import abi
    from muzero_jl_amd.selfplay import BatchedSelfPlay, game_winner
    mod, env_cls, env_kind = _env(kind)
    G = 16
    conf = dataclasses.replace(mod.conf, num_iters=6, replay_buffer_size=64)
    eh, ed = _engines(mod, conf, mod.hyper, G)
    sp = BatchedSelfPlay(eh, env_cls, G, game_offset=7, step0=100, opponent=opp, muzero_player=mzp)
    ed.selfplay_init(env_kind, G, 64)
    ed.selfplay_mode(abi.SP_EVAL, abi.OPP_RANDOM if opp == "random" else abi.OPP_SELF, mzp)
    for m in range(14 if kind == "ttt" else 30):
        sp.play_move(0.0)
        ed.selfplay_move(100 + m, game_offset=7, temperature=0.0)
    name = "tictactoe" if kind == "ttt" else "connect4"
    t = [0, 0, 0, 0]
    for h in sp.finished:
        w = game_winner(name, h.reward_history[-1], h.to_play_history[-1])
        t[0] += 1
        t[3 if w == 0 else 1 if w == mzp else 2] += 1
    assert t[0] > 0 and ed.eval_results() == tuple(t)
    assert ed.replay_counts()[0][0] == 0                      # competitive_play! saves nothing
    ln, board, player = ed.selfplay_slots()
    assert np.array_equal(ln, [len(h.action_history) for h in sp.histories])
    assert np.array_equal(board, sp.env.board.astype(np.uint8)) and np.array_equal(player, sp.env.player)
    ed.selfplay_mode(abi.SP_TRAIN)                             # back to self_play!: finished games are saved
    for m in range(12):
        ed.selfplay_move(200 + m, game_offset=7)
    assert ed.replay_counts()[0][0] > 0
    with pytest.raises(abi.MzError, match="muzero_player"):
        ed.selfplay_mode(abi.SP_EVAL, abi.OPP_RANDOM, 3)
    eh.close(); ed.close()


def _per_engines(G, moves, cap, host=True):
    from muzero_jl_amd.selfplay import BatchedSelfPlay
    mod, env_cls, env_kind = _env("ttt")
    conf = dataclasses.replace(mod.conf, num_iters=6, replay_buffer_size=cap, PER=True, PER_alpha=1)
    e1, e2 = _engines(mod, conf, mod.hyper, G)
    sp = BatchedSelfPlay(e1, env_cls, G, game_offset=7, step0=100) if host else None
    e2.selfplay_init(env_kind, G, cap)
    if not host:
        e1.selfplay_init(env_kind, G, cap)
    for m in range(moves):
        if host:
            sp.play_move()
        else:
            e1.selfplay_move(100 + m, game_offset=7)
        e2.selfplay_move(100 + m, game_offset=7)
    return conf, sp, e1, e2


def _np_losses(pv, pp, tv, tpol, gs, w):
    """Learning.jl:261-288 with PER weights, in f64 (ref_semantics: the
    policy term is Q11's mean_j(CE_j)·mean_i(w_i/g_i) broadcast)."""
    B = pv.shape[0]
    vl = np.mean(((pv.astype(np.float64) - tv) ** 2).sum(1) / gs * w)
    lp = np.log(np.exp(pp.astype(np.float64)).sum(-1, keepdims=True))
    ce = -(tpol * (pp - lp)).sum((1, 2))
    return vl, ce.sum() * (w / gs.astype(np.float64)).sum() / (B * B)


def test_per_replay_matches_host():
    """PER on the device shard == the host ReplayBuffer mirror: initial
    priorities (save_game), prioritized get_batch with its importance weights,
    the weighted losses, and update_priorities! after each learner step."""
    import torch
    from muzero_jl_amd.replay_buffer import ReplayBuffer
    conf, sp, eh, ed = _per_engines(16, 30, cap=24)
    rb = ReplayBuffer(conf, seed=5)
    for h in sp.finished:
        rb.save_game(h)
    assert ed.replay_counts()[1] == len(rb) == 24 and len(sp.finished) > 24     # the FIFO evicted

    def same_priorities():
        for i, (gid, h) in enumerate(rb.buffer.items()):
            pr, gp = ed.replay_get_priorities(i)
            assert np.array_equal(pr, h.priorities) and np.float32(gp) == h.game_priority, i

    same_priorities()
    B = 40
    rb.conf = dataclasses.replace(conf, batch_size=B)
    grad = torch.empty(ed.grad_count(), dtype=torch.float32, device="cuda")
    losses = torch.empty(8, dtype=torch.float32, device="cuda")
    for step in (1, 2, 3):
        idx_h, bh = rb.get_batch(step)
        b, idx_d = ed.replay_sample(B, step, index=True)
        bd = ed.batch_to_host(b)
        assert [tuple(x) for x in idx_d] == [tuple(x) for x in idx_h]
        for k in bh:
            assert np.array_equal(bd[k], bh[k]), (step, k)
        assert bh["weights"].max() == 1.0
        ed.learner_grad_dev([b.observation, b.actions, b.target_values, b.target_rewards, b.target_policies,
                             b.gradient_scale, b.weights], B, grad.data_ptr(), losses.data_ptr())
        pv, pp, _ = ed.debug_unroll(B)
        lo = losses.cpu().numpy()
        vl, pl = _np_losses(pv, pp, bh["target_values"], bh["target_policies"], bh["gradient_scale"],
                            bh["weights"])
        np.testing.assert_allclose([lo[0], lo[2]], [vl, pl], rtol=1e-4, atol=1e-6)
        ed.replay_update_priorities()
        rb.update_priorities(idx_h, pv, bh["target_values"])
        same_priorities()
    eh.close(); ed.close()


def test_per_fused_learner_matches_separate_calls():
    """With PER, mz_learner_train_dev (weights, losses, priority update fused)
    == replay_sample + grad_dev(weights) + update_priorities + apply."""
    import torch
    from muzero_jl_amd.config import cos_schedule
    conf, _, e1, e2 = _per_engines(16, 20, cap=64, host=False)
    B = 32
    grad = torch.empty(e1.grad_count(), dtype=torch.float32, device="cuda")
    l1 = torch.empty(8, dtype=torch.float32, device="cuda")
    l2 = torch.empty(8, dtype=torch.float32, device="cuda")
    for step in (1, 2, 3):
        eta = cos_schedule(step)
        b, _ = e1.replay_sample(B, step)
        e1.learner_grad_dev([b.observation, b.actions, b.target_values, b.target_rewards, b.target_policies,
                             b.gradient_scale, b.weights], B, grad.data_ptr(), l1.data_ptr())
        e1.replay_update_priorities()
        e1.learner_apply_dev(grad.data_ptr(), 1.0, eta)
        e2.learner_train_dev(B, step, eta, l2.data_ptr())
        e1.sync(); e2.sync()
        assert np.array_equal(l1.cpu().numpy()[:6], l2.cpu().numpy()[:6]), step
        held = e1.replay_counts()[1]
        for i in range(held):
            p1, g1 = e1.replay_get_priorities(i)
            p2, g2 = e2.replay_get_priorities(i)
            assert np.array_equal(p1, p2) and g1 == g2
        for n in range(3):
            assert np.array_equal(e1.get_weights(n), e2.get_weights(n)), (step, n)
    e1.close(); e2.close()


def test_per_host_save_game_priorities():
    """mz_replay_save_game with PER: the initial priorities of host-played games
    (save_game, ReplayBuffer.jl:136-143) equal the host mirror's."""
    from muzero_jl_amd import abi
    from muzero_jl_amd.replay_buffer import ReplayBuffer
    from muzero_jl_amd.selfplay import BatchedSelfPlay
    mod, env_cls, env_kind = _env("ttt")
    conf = dataclasses.replace(mod.conf, num_iters=4, replay_buffer_size=8, PER=True, PER_alpha=2)
    e1, e2 = _engines(mod, conf, mod.hyper, 8)
    sp = BatchedSelfPlay(e1, env_cls, 8, step0=3)
    for _ in range(24):
        sp.play_move()
    e2.selfplay_init(env_kind, 8, 8)
    rb = ReplayBuffer(conf, seed=1)
    for h in sp.finished:
        e2.replay_save_game(h)
        rb.save_game(h)
    assert len(rb) == e2.replay_counts()[1] > 0
    for i, h in enumerate(rb.buffer.values()):
        pr, gp = e2.replay_get_priorities(i)
        assert np.array_equal(pr, h.priorities) and np.float32(gp) == h.game_priority
    e1.close(); e2.close()


def test_dp_rccl_world1_matches_single_gpu():
    """The C-ABI data-parallel learner (mz_dp_unique_id / mz_dp_init /
    mz_learner_train_dp: grad + RCCL all-reduce + apply(1/world)) on a
    one-rank communicator equals mz_learner_train_dev, bit for bit."""
    import torch
    from muzero_jl_amd import abi
    from muzero_jl_amd.config import cos_schedule
    e1, e2 = _device_pair("ttt", 16, 14, cap=64)
    with pytest.raises(abi.MzError, match="mz_dp_init first"):
        e2.dp_allreduce()
    e2.dp_init(0, 1, abi.Engine.dp_unique_id())
    l1 = torch.empty(8, dtype=torch.float32, device="cuda")
    l2 = torch.empty(8, dtype=torch.float32, device="cuda")
    for step in (1, 2, 3):
        eta = cos_schedule(step)
        e1.learner_train_dev(32, step, eta, l1.data_ptr())
        e2.learner_train_dp(32, step, eta, l2.data_ptr())
        e1.sync(); e2.sync()
        assert np.array_equal(l1.cpu().numpy()[:6], l2.cpu().numpy()[:6]), step
        for n in range(3):
            assert np.array_equal(e1.get_weights(n), e2.get_weights(n)), (step, n)
    e1.close(); e2.close()
