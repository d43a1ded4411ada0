"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker; never by the product package.
PARITY UNPINNED (see mz_oracle.c header): the Julia reference cannot run here.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_VP = ctypes.c_void_p
_lib = None


class OHist(ctypes.Structure):
    _fields_ = [("T", ctypes.c_int32), ("obs", _VP), ("actions", _VP), ("rewards", _VP),
                ("to_play", _VP), ("child_visits", _VP), ("root_values", _VP)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.ora_param_count.restype = ctypes.c_size_t
        L.ora_param_count.argtypes = [_VP, _VP, ctypes.c_int]
        L.ora_hidden_size.restype = ctypes.c_int
        L.ora_hidden_size.argtypes = [_VP, _VP]
        L.ora_net_forward.argtypes = [_VP, _VP, ctypes.c_int, _VP, _VP, ctypes.c_int, _VP, _VP]
        L.ora_mcts_search.restype = ctypes.c_int
        L.ora_mcts_search.argtypes = [_VP, _VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_int, _VP, _VP, _VP,
                                      ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float,
                                      _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP]
        L.ora_play_game.restype = ctypes.c_int
        L.ora_play_game.argtypes = [_VP, _VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_float, _VP, _VP, _VP, _VP, _VP, _VP]
        L.ora_ttt_step.argtypes = [_VP, _VP, ctypes.c_int, _VP, _VP, _VP]
        L.ora_stacked_obs.argtypes = [_VP, _VP, _VP, ctypes.c_int, _VP]
        L.ora_compute_target_value.restype = ctypes.c_float
        L.ora_compute_target_value.argtypes = [_VP, ctypes.POINTER(OHist), ctypes.c_int]
        L.ora_get_batch.argtypes = [_VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32,
                                    _VP, _VP, _VP, _VP, _VP, _VP, _VP]
        L.ora_unroll.argtypes = [_VP, _VP, _VP, _VP, _VP, ctypes.c_int, _VP, _VP, _VP, _VP, _VP]
        L.ora_losses.argtypes = [_VP, ctypes.c_int, _VP, _VP, _VP, _VP, _VP, _VP, _VP]
        L.ora_sqnorm.restype = ctypes.c_double
        L.ora_sqnorm.argtypes = [_VP, ctypes.c_size_t]
        L.ora_adam_2theta.argtypes = [_VP, _VP, _VP, ctypes.c_size_t, _VP, ctypes.c_double]
        L.ora_adam_grad.argtypes = [_VP, _VP, _VP, _VP, ctypes.c_size_t, _VP, ctypes.c_double]
        L.ora_cos_schedule.restype = ctypes.c_double
        L.ora_cos_schedule.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int]
        L.ora_learner_step.argtypes = [_VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_int, _VP, _VP, _VP,
                                       _VP, _VP, ctypes.c_double, _VP]
        L.ora_per_priority.restype = ctypes.c_float
        L.ora_per_priority.argtypes = [ctypes.c_float, ctypes.c_int]
        L.ora_per_categorical.restype = ctypes.c_int
        L.ora_per_categorical.argtypes = [_VP, ctypes.c_int, ctypes.c_double, _VP]
        L.ora_per_init.argtypes = [_VP, ctypes.POINTER(OHist), _VP, _VP]
        L.ora_get_batch_per.argtypes = [_VP, _VP, _VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                        ctypes.c_uint32] + [_VP] * 8
        L.ora_update_priorities.argtypes = [_VP, _VP, _VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, _VP, _VP, _VP]
        L.ora_learner_step_w.argtypes = [_VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_int, _VP, _VP, _VP,
                                         _VP, _VP, _VP, ctypes.c_double, _VP]
        L.ora_eval_play.restype = ctypes.c_int
        L.ora_eval_play.argtypes = [_VP, _VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                    _VP, _VP, _VP, _VP]
        L.ora_losses_w.argtypes = [_VP, ctypes.c_int, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP]
        L.ora_train_loop.restype = ctypes.c_int
        L.ora_train_loop.argtypes = [_VP, _VP] + [_VP] * 9 + [_VP, _VP, _VP, ctypes.c_uint64, ctypes.c_int,
                                                           ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                                           ctypes.c_uint32] + [_VP] * 13
        for n, r, a in [("ora_det_expf", ctypes.c_float, [ctypes.c_float]),
                        ("ora_det_tanhf", ctypes.c_float, [ctypes.c_float]),
                        ("ora_det_logf", ctypes.c_float, [ctypes.c_float]),
                        ("ora_det_exp", ctypes.c_double, [ctypes.c_double]),
                        ("ora_det_log", ctypes.c_double, [ctypes.c_double])]:
            getattr(L, n).restype = r
            getattr(L, n).argtypes = a
        L.ora_rng_u32.restype = ctypes.c_uint32
        L.ora_rng_u32.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L.ora_philox.argtypes = [ctypes.c_uint32] * 6 + [_VP]
        L.ora_dirichlet.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_float, _VP]
        L.ora_softmax.argtypes = [_VP, ctypes.c_int, _VP]
        L.ora_dot.restype = ctypes.c_float
        L.ora_dot.argtypes = [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, _VP]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(_VP)


def nethp(chp):
    """Tagged network hyper-parameters of the oracle (ora_nethp): FC or ResNet."""
    from muzero_jl_amd.config import MzFFHP, MzResNetHP   # registered by _mzpkg.load()

    class OraNetHP(ctypes.Structure):
        _fields_ = [("kind", ctypes.c_int32), ("ff", MzFFHP), ("rn", MzResNetHP)]

    o = OraNetHP()
    if isinstance(chp, MzResNetHP):
        o.kind, o.rn = 1, chp
    else:
        o.kind, o.ff = 0, chp
    return o


class Oracle:
    """The oracle bound to one (Config, FeedForwardHP | ResNetHP) and three flat weight vectors."""

    def __init__(self, cconf, chp, seed=0):
        self.L = lib()
        self.cconf = cconf
        self.chp = nethp(chp)
        self.seed = seed
        self.A = cconf.action_space_size
        self.H = self.L.ora_hidden_size(ctypes.byref(self.cconf), ctypes.byref(self.chp))
        # board of the dynamics action plane: the hidden state's
        self.plane = self.H // chp.num_filters if self.chp.kind == 1 else \
            cconf.observation_shape[0] * cconf.observation_shape[1]
        self.S = cconf.num_iters
        self.K = cconf.num_unroll_steps
        self.params = [np.zeros(self.param_count(i), np.float32) for i in range(3)]

    def _c(self):
        return ctypes.byref(self.cconf), ctypes.byref(self.chp)

    def param_count(self, net):
        c, h = self._c()
        return self.L.ora_param_count(c, h, net)

    def set_weights(self, net, flat):
        self.params[net] = np.ascontiguousarray(flat, dtype=np.float32).copy()

    def forward(self, net, x):
        c, h = self._c()
        x = np.ascontiguousarray(x, np.float32)
        n = x.shape[0]
        if net == 1:
            o0, o1 = np.empty((n, 1), np.float32), np.empty((n, self.A), np.float32)
        elif net == 2:
            o0, o1 = np.empty((n, self.H), np.float32), np.empty((n, 1), np.float32)
        else:
            o0, o1 = np.empty((n, self.H), np.float32), None
        self.L.ora_net_forward(c, h, net, _p(self.params[net]), _p(x), n, _p(o0), _p(o1))
        return (o0, o1) if o1 is not None else o0

    def mcts_search(self, obs, legal, to_play, exploration=True, rng_step=0, game_offset=0, temperature=1.0,
                    dump=False):
        c, h = self._c()
        obs = np.ascontiguousarray(obs, np.float32)
        G = obs.shape[0]
        legal = np.ascontiguousarray(legal, np.uint8)
        tp = np.ascontiguousarray(to_play, np.int32)
        cv = np.empty((G, self.A), np.float32)
        rv = np.empty(G, np.float32)
        act = np.empty(G, np.int32)
        stats = np.zeros(2, np.int64)
        tree = None
        if dump:
            S, A = self.S, self.A
            tree = dict(N=np.zeros((G, S + 1, A), np.int32), W=np.zeros((G, S + 1, A), np.float32),
                        P=np.zeros((G, S + 1, A), np.float32), R=np.zeros((G, S + 1, A), np.float32),
                        C=np.full((G, S + 1, A), -1, np.int32), to_play=np.zeros((G, S + 1), np.int32))
        t = tree or {}
        self.L.ora_mcts_search(c, h, _p(self.params[0]), _p(self.params[1]), _p(self.params[2]), self.seed, G,
                               _p(obs), _p(legal), _p(tp), int(exploration), rng_step & 0xffffffff, game_offset,
                               temperature, _p(cv), _p(rv), _p(act), _p(t.get("N")), _p(t.get("W")),
                               _p(t.get("P")), _p(t.get("R")), _p(t.get("C")), _p(t.get("to_play")), _p(stats))
        out = (cv, rv, act)
        if dump:
            return out + (tree, stats)
        return out

    def play_game(self, game_id=0, step0=0, temperature=1.0):
        c, h = self._c()
        M = self.cconf.max_moves + 1
        A = self.A
        obs = np.zeros((M, 27), np.float32)
        acts = np.zeros(M, np.int32)
        rew = np.zeros(M, np.float32)
        tp = np.zeros(M, np.int32)
        cv = np.zeros((M, A), np.float32)
        rv = np.zeros(M, np.float32)
        T = self.L.ora_play_game(c, h, _p(self.params[0]), _p(self.params[1]), _p(self.params[2]), self.seed,
                                 game_id, step0, temperature, _p(obs), _p(acts), _p(rew), _p(tp), _p(cv), _p(rv))
        return dict(observation=obs[:T].copy(), action=acts[:T].copy(), reward=rew[:T].copy(),
                    to_play=tp[:T].copy(), child_visits=cv[:T].copy(), root_values=rv[:T].copy())

    def unroll(self, obs, actions):
        c, h = self._c()
        B = obs.shape[0]
        K, A = self.K, self.A
        pv = np.empty((B, K + 1), np.float32)
        pp = np.empty((B, K + 1, A), np.float32)
        pr = np.empty((B, K + 1), np.float32)
        self.L.ora_unroll(c, h, _p(self.params[0]), _p(self.params[1]), _p(self.params[2]), B,
                          _p(np.ascontiguousarray(obs, np.float32)), _p(np.ascontiguousarray(actions, np.float32)),
                          _p(pv), _p(pp), _p(pr))
        return pv, pp, pr

    def learner_step_w(self, state, batch, eta, weights=None):
        """ora_learner_step_w: the ref_semantics step with PER importance weights."""
        c, h = self._c()
        a = {k: np.ascontiguousarray(batch[k], np.float32) for k in
             ("observation", "actions", "target_values", "target_policies", "gradient_scale")}
        w = None if weights is None else np.ascontiguousarray(weights, np.float32)
        losses = np.empty(6, np.float32)
        B = a["observation"].shape[0]
        self.L.ora_learner_step_w(c, h, _p(self.params[0]), _p(self.params[1]), _p(self.params[2]), _p(state["m"]),
                                  _p(state["v"]), _p(state["bp"]), B, _p(a["observation"]), _p(a["actions"]),
                                  _p(a["target_values"]), _p(a["target_policies"]), _p(a["gradient_scale"]), _p(w),
                                  eta, _p(losses))
        return losses

    def eval_play(self, G, moves, move0=0, game_offset=0, random_opponent=True, muzero_player=1, temperature=0.0):
        """ora_eval_play: competitive_play! for G lockstep TicTacToe slots ->
        (tally {games, MuZero wins, opponent wins, draws}, slot lens, boards, players)."""
        c, h = self._c()
        tally = np.zeros(4, np.int64)
        ln = np.zeros(G, np.int32)
        board = np.zeros((G, 27), np.uint8)
        player = np.zeros(G, np.int32)
        rc = self.L.ora_eval_play(c, h, _p(self.params[0]), _p(self.params[1]), _p(self.params[2]), self.seed, G,
                                  moves, move0, game_offset, int(random_opponent), muzero_player, temperature,
                                  _p(tally), _p(ln), _p(board), _p(player))
        assert rc == 0, "ora_eval_play: TicTacToe only"
        return tuple(int(x) for x in tally), ln, board, player

    def learner_state(self):
        n = sum(p.size for p in self.params)
        return dict(m=np.zeros(n, np.float32), v=np.zeros(n, np.float32), bp=np.array([0.9, 0.999]))

    def learner_step(self, state, batch, eta):
        c, h = self._c()
        a = {k: np.ascontiguousarray(batch[k], np.float32) for k in
             ("observation", "actions", "target_values", "target_policies", "gradient_scale")}
        losses = np.empty(6, np.float32)
        B = a["observation"].shape[0]
        self.L.ora_learner_step(c, h, _p(self.params[0]), _p(self.params[1]), _p(self.params[2]), _p(state["m"]),
                                _p(state["v"]), _p(state["bp"]), B, _p(a["observation"]), _p(a["actions"]),
                                _p(a["target_values"]), _p(a["target_policies"]), _p(a["gradient_scale"]),
                                eta, _p(losses))
        return losses


def train_loop(ora, G, cap, moves, move0=0, game_offset=0, state=None, t0=0):
    """ora_train_loop (oracle/mz_oracle.c): the actor–learner schedule of
    mz_train_run from fresh slots — ora.params are the learner's nets (updated
    in place); returns dict(t, counters, held games, slots, actor / queued
    nets, losses, state)."""
    c, h = ora._c()
    conf = ora.cconf
    A, Tm = ora.A, conf.max_moves + 1
    st = state or ora.learner_state()
    actor = [p.copy() for p in ora.params]
    queued = [p.copy() for p in ora.params]
    t = np.full(1, t0, np.int64)
    counters = np.zeros(3, np.int64)
    hT = np.zeros(cap, np.int32)
    hobs = np.zeros((cap, Tm, 27), np.float32)
    hact = np.zeros((cap, Tm), np.int32)
    hrew = np.zeros((cap, Tm), np.float32)
    htp = np.zeros((cap, Tm), np.int32)
    hcv = np.zeros((cap, Tm, A), np.float32)
    hrv = np.zeros((cap, Tm), np.float32)
    slen = np.zeros(G, np.int32)
    sboard = np.zeros((G, 27), np.uint8)
    splayer = np.zeros(G, np.int32)
    losses = np.zeros(6, np.float32)
    P = ora.params
    nh = ora.L.ora_train_loop(c, h, _p(P[0]), _p(P[1]), _p(P[2]), _p(actor[0]), _p(actor[1]), _p(actor[2]),
                              _p(queued[0]), _p(queued[1]), _p(queued[2]), _p(st["m"]), _p(st["v"]), _p(st["bp"]),
                              ora.seed, G, cap, moves, move0, game_offset, _p(t), _p(counters), _p(hT), _p(hobs),
                              _p(hact), _p(hrew), _p(htp), _p(hcv), _p(hrv), _p(slen), _p(sboard), _p(splayer),
                              _p(losses))
    assert nh >= 0, "ora_train_loop: TicTacToe only"
    held = [dict(observation=hobs[i, :hT[i]].copy(), action=hact[i, :hT[i]].copy(), reward=hrew[i, :hT[i]].copy(),
                 to_play=htp[i, :hT[i]].copy(), child_visits=hcv[i, :hT[i]].copy(), root_values=hrv[i, :hT[i]].copy())
            for i in range(nh)]
    return dict(t=int(t[0]), counters=counters, held=held, slot_len=slen, slot_board=sboard, slot_player=splayer,
                actor=actor, queued=queued, losses=losses, state=st)


class PerReplay:
    """The oracle's PER shard (ora_per_init / ora_get_batch_per /
    ora_update_priorities) over a list of held games (oldest first), game
    numbers first_id.. — the reference's intended PER reading."""

    def __init__(self, ora, histories, first_id):
        self.o = ora
        self.hist = histories
        self.first_id = first_id
        self.arr, self.keep = histories_to_c(histories)
        self.Tmax = ora.cconf.max_moves + 1
        n = len(histories)
        self.lens = np.array([len(h["action"]) for h in histories], np.int32)
        self.prio = np.zeros((n, self.Tmax), np.float32)
        self.gprio = np.zeros(n, np.float32)
        c, _ = ora._c()
        for i in range(n):
            ora.L.ora_per_init(c, ctypes.byref(self.arr[i]), _p(self.prio[i]),
                               self.gprio[i:i + 1].ctypes.data_as(ctypes.c_void_p))

    def get_batch(self, step, B):
        import dataclasses  # noqa: F401
        o = self.o
        cc = type(o.cconf)()
        ctypes.pointer(cc)[0] = o.cconf
        cc.batch_size = B
        K, A = o.K, o.A
        osz = self.hist[0]["observation"].shape[1]
        feat = (osz // 3) * (3 * (cc.stacked_observations + 1) + cc.stacked_observations)
        out = dict(observation=np.zeros((B, feat), np.float32), actions=np.zeros((B, K + 1), np.float32),
                   target_values=np.zeros((B, K + 1), np.float32), target_rewards=np.zeros((B, K + 1), np.float32),
                   target_policies=np.zeros((B, K + 1, A), np.float32), gradient_scale=np.zeros(B, np.float32),
                   weights=np.zeros(B, np.float32))
        idx = np.zeros((B, 2), np.int32)
        o.L.ora_get_batch_per(ctypes.byref(cc), self.arr, _p(self.prio), _p(self.gprio), len(self.hist), self.Tmax,
                              self.first_id, o.seed, step, _p(out["observation"]), _p(out["actions"]),
                              _p(out["target_values"]), _p(out["target_rewards"]), _p(out["target_policies"]),
                              _p(out["gradient_scale"]), _p(out["weights"]), _p(idx))
        return idx, out

    def update_priorities(self, idx, pv, tv):
        c, _ = self.o._c()
        B = idx.shape[0]
        self.o.L.ora_update_priorities(c, _p(self.prio), _p(self.gprio), _p(self.lens), len(self.hist), self.Tmax,
                                       self.first_id, B, _p(np.ascontiguousarray(idx, np.int32)),
                                       _p(np.ascontiguousarray(pv, np.float32)),
                                       _p(np.ascontiguousarray(tv, np.float32)))


def histories_to_c(histories):
    """list of dicts (observation (T,27), action, reward, to_play, child_visits (T,A), root_values)
    -> (array of OHist, keepalive)."""
    arr = (OHist * len(histories))()
    keep = []
    for i, hst in enumerate(histories):
        cols = [np.ascontiguousarray(hst["observation"], np.float32), np.ascontiguousarray(hst["action"], np.int32),
                np.ascontiguousarray(hst["reward"], np.float32), np.ascontiguousarray(hst["to_play"], np.int32),
                np.ascontiguousarray(hst["child_visits"], np.float32),
                np.ascontiguousarray(hst["root_values"], np.float32)]
        keep.append(cols)
        arr[i] = OHist(len(cols[1]), *[_p(x) for x in cols])
    return arr, keep
