"""ctypes binding of libmz (include/mz.h) — the Python side of the drop-in
boundary.  The Julia side a maintainer would add is in INTEGRATION.md.

The product path has no fallback: if libmz.so is missing or no HIP device is
present, `Engine(...)` raises.  Arrays crossing the ABI are numpy arrays in the
reference's column-major shapes, stored here as C-contiguous arrays whose LAST
axis is Julia's FIRST (e.g. Julia (A, G) == numpy (G, A)).
"""
import ctypes
import os

import numpy as np

from . import LIB_PATH
from .config import (MzConfig, MzFFHP, MzResNetHP, ResNetHP, hidden_size, stacked_features, to_c_config,
                     to_c_ffhp, to_c_resnet_hp)

NET_REPR, NET_PRED, NET_DYN = 0, 1, 2
ENV_TICTACTOE, ENV_CONNECT4, ENV_ATARI = 0, 1, 2
SP_TRAIN, SP_EVAL = 0, 1
TRAIN_LEARNER, TRAIN_ACTOR, TRAIN_QUEUED = 0, 1, 2
LEARN_REF_SEMANTICS, LEARN_CORRECTED = 0, 1
OPP_SELF, OPP_RANDOM = 0, 1

_lib = None

_F = ctypes.POINTER(ctypes.c_float)
_I = ctypes.POINTER(ctypes.c_int32)
_U8 = ctypes.POINTER(ctypes.c_uint8)
_VP = ctypes.c_void_p


class MzBatch(ctypes.Structure):
    _fields_ = [("batch_size", ctypes.c_int32), ("observation", _VP), ("actions", _VP),
                ("target_values", _VP), ("target_rewards", _VP), ("target_policies", _VP),
                ("gradient_scale", _VP), ("weights", _VP)]


# exported symbol -> (restype, argtypes); tests check every one is present
SIGNATURES = {
    "mz_engine_create": (ctypes.c_int, [ctypes.POINTER(MzConfig), ctypes.POINTER(MzFFHP), ctypes.c_int,
                                        ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(_VP)]),
    "mz_engine_create_resnet": (ctypes.c_int, [ctypes.POINTER(MzConfig), ctypes.POINTER(MzResNetHP), ctypes.c_int,
                                               ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(_VP)]),
    "mz_engine_destroy": (None, [_VP]),
    "mz_last_error": (ctypes.c_char_p, [_VP]),
    "mz_create_error": (ctypes.c_char_p, []),
    "mz_net_param_count": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]),
    "mz_weights_set": (ctypes.c_int, [_VP, ctypes.c_int, _VP, ctypes.c_size_t]),
    "mz_weights_get": (ctypes.c_int, [_VP, ctypes.c_int, _VP, ctypes.c_size_t]),
    "mz_net_forward": (ctypes.c_int, [_VP, ctypes.c_int, _VP, ctypes.c_int, _VP, _VP]),
    "mz_mcts_search": (ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP, ctypes.c_int, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_float, _VP, _VP, _VP]),
    "mz_mcts_search_dev": (ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP, ctypes.c_int, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_float, _VP, _VP, _VP, _VP]),
    "mz_debug_enable": (ctypes.c_int, [_VP, ctypes.c_int]),
    "mz_set_sync_stream": (ctypes.c_int, [_VP, _VP, ctypes.c_int]),
    "mz_debug_tree": (ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP, _VP, _VP, _VP]),
    "mz_debug_unroll": (ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP]),
    "mz_debug_kernel_time": (ctypes.c_int, [_VP, _VP, _VP]),
    "mz_learner_step": (ctypes.c_int, [_VP, ctypes.POINTER(MzBatch), ctypes.c_double, _VP]),
    "mz_grad_count": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_size_t)]),
    "mz_learner_grad_dev": (ctypes.c_int, [_VP, ctypes.POINTER(MzBatch), _VP, _VP, _VP]),
    "mz_learner_apply_dev": (ctypes.c_int, [_VP, _VP, ctypes.c_float, ctypes.c_double, _VP]),
    "mz_selfplay_init": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "mz_selfplay_move": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float, _VP]),
    "mz_dp_unique_id": (ctypes.c_int, [_VP]),
    "mz_dp_init": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, _VP]),
    "mz_dp_allreduce": (ctypes.c_int, [_VP, _VP, _VP]),
    "mz_learner_train_dp": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_uint32, ctypes.c_double, _VP, _VP]),
    "mz_selfplay_mode": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "mz_eval_results": (ctypes.c_int, [_VP, _VP]),
    "mz_replay_counts": (ctypes.c_int, [_VP, _VP, _VP]),
    "mz_replay_save_game": (ctypes.c_int, [_VP, ctypes.c_int32, _VP, _VP, _VP, _VP, _VP, _VP]),
    "mz_replay_sample": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_uint32, ctypes.POINTER(MzBatch), _VP, _VP]),
    "mz_learner_grad_sampled_dev": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_uint32, _VP, _VP, _VP]),
    "mz_learner_train_dev": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_uint32, ctypes.c_double, _VP, _VP]),
    "mz_learner_train_multi_dev": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int32,
                                                  ctypes.POINTER(ctypes.c_double), _VP, _VP, _VP]),
    "mz_debug_unroll_step": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, _VP, _VP, _VP]),
    "mz_replay_update_priorities": (ctypes.c_int, [_VP, _VP]),
    "mz_replay_get_priorities": (ctypes.c_int, [_VP, ctypes.c_int32, _VP, _VP]),
    "mz_replay_get_game": (ctypes.c_int, [_VP, ctypes.c_int32, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    "mz_selfplay_slots": (ctypes.c_int, [_VP, _VP, _VP, _VP]),
    "mz_learner_set_mode": (ctypes.c_int, [_VP, ctypes.c_int]),
    "mz_train_init": (ctypes.c_int, [_VP, ctypes.c_int32]),
    "mz_train_init_at": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_int64]),
    "mz_train_set_networks_path": (ctypes.c_int, [_VP, ctypes.c_char_p]),
    "mz_train_run": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32, _VP, _VP, _VP]),
    "mz_train_move": (ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_uint32, _VP, _VP]),
    "mz_train_learn": (ctypes.c_int, [_VP, ctypes.c_int64, _VP, _VP, _VP]),
    "mz_train_weights_get": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, _VP, ctypes.c_size_t]),
    "mz_checkpoint_save": (ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_int64]),
    "mz_checkpoint_load": (ctypes.c_int, [_VP, ctypes.c_char_p, _VP]),
    "mz_search_variant": (ctypes.c_char_p, [_VP]),
    "mz_learner_variant": (ctypes.c_char_p, [_VP]),
    "mz_sync": (ctypes.c_int, [_VP]),
}


def load_library(path=LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libmz.so not built at {path}: run __graft_entry__.build() "
                           "(there is no CPU fallback for the engine)")
    # torch's wheel ships its own libamdhip64.so.7 with the same soname as
    # /opt/rocm's: whichever loads first serves the whole process.  Loading
    # torch first (when present) makes libmz bind to torch's copy, so the
    # engine and torch streams / device tensors share one HIP runtime in any
    # import order; torch cannot initialise on the other copy.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    variant = bool(os.environ.get("MZ_LIB")) and path == os.environ.get("MZ_LIB")
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):
            continue                 # an older A/B variant library (MZ_LIB) without this entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _p(a):
    return None if a is None else a.ctypes.data_as(_VP)


_hip = None


def _copy_d2h(dst, src_ptr):
    """hipMemcpy device -> host (the HIP runtime libmz is linked against)."""
    global _hip
    if _hip is None:
        # by soname: the copy already loaded for libmz (torch's or /opt/rocm's,
        # whichever came first); a plain "libamdhip64.so" can load a second runtime
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipMemcpy.restype = ctypes.c_int
        _hip.hipMemcpy.argtypes = [_VP, _VP, ctypes.c_size_t, ctypes.c_int]
    rc = _hip.hipMemcpy(dst.ctypes.data_as(_VP), ctypes.c_void_p(src_ptr), dst.nbytes, 2)   # DeviceToHost
    if rc != 0:
        raise MzError(f"hipMemcpy failed ({rc})")


class MzError(RuntimeError):
    pass


class Engine:
    """One libmz handle = one GPU (SURVEY §8b conventions)."""

    def __init__(self, conf, hyper, device=0, max_games=512, rng_seed=0):
        lib = load_library()
        self.lib = lib
        self.conf = conf
        self.hyper = hyper
        self._cconf = to_c_config(conf)
        h = _VP()
        if isinstance(hyper, ResNetHP):        # row a14: the ResNet networks
            self._chp = to_c_resnet_hp(hyper)
            rc = lib.mz_engine_create_resnet(ctypes.byref(self._cconf), ctypes.byref(self._chp), device, max_games,
                                             rng_seed, ctypes.byref(h))
        else:
            self._chp = to_c_ffhp(hyper)
            rc = lib.mz_engine_create(ctypes.byref(self._cconf), ctypes.byref(self._chp), device, max_games,
                                      rng_seed, ctypes.byref(h))
        if rc != 0:
            raise MzError(f"mz_engine_create: {lib.mz_create_error().decode()}")
        self.h = h
        self.rng_seed = rng_seed
        self.max_games = max_games
        self.A = len(conf.action_space)
        self.H = hidden_size(conf, hyper)
        self.obs_feat = stacked_features(conf)

    def close(self):
        if getattr(self, "h", None):
            self.lib.mz_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise MzError(f"{what}: {self.lib.mz_last_error(self.h).decode()}")

    # ---- weights (Flux order per net)
    def param_count(self, net):
        n = ctypes.c_size_t()
        self._check(self.lib.mz_net_param_count(self.h, net, ctypes.byref(n)), "mz_net_param_count")
        return n.value

    def set_weights(self, net, flat):
        flat = np.ascontiguousarray(flat, dtype=np.float32)
        self._check(self.lib.mz_weights_set(self.h, net, _p(flat), flat.size), "mz_weights_set")

    def get_weights(self, net):
        out = np.empty(self.param_count(net), dtype=np.float32)
        self._check(self.lib.mz_weights_get(self.h, net, _p(out), out.size), "mz_weights_get")
        return out

    # ---- batched net forward (Flux Chain call)
    def forward(self, net, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        n = x.shape[0]
        if net == NET_PRED:
            o0 = np.empty((n, 1), np.float32)
            o1 = np.empty((n, self.A), np.float32)
        elif net == NET_DYN:
            o0 = np.empty((n, self.H), np.float32)
            o1 = np.empty((n, 1), np.float32)
        else:
            o0 = np.empty((n, self.H), np.float32)
            o1 = None
        self._check(self.lib.mz_net_forward(self.h, net, _p(x), n, _p(o0), _p(o1)), "mz_net_forward")
        return (o0, o1) if o1 is not None else o0

    # ---- batched run_mcts
    def mcts_search(self, obs, legal_mask, to_play, exploration=True, rng_step=0, game_offset=0,
                    temperature=1.0):
        obs = np.ascontiguousarray(obs, dtype=np.float32)
        G = obs.shape[0]
        legal = np.ascontiguousarray(legal_mask, dtype=np.uint8)
        tp = np.ascontiguousarray(to_play, dtype=np.int32)
        cv = np.empty((G, self.A), np.float32)
        rv = np.empty(G, np.float32)
        act = np.empty(G, np.int32)
        self._check(self.lib.mz_mcts_search(self.h, G, _p(obs), _p(legal), _p(tp), int(exploration),
                                            rng_step & 0xffffffff, game_offset, temperature,
                                            _p(cv), _p(rv), _p(act)), "mz_mcts_search")
        return cv, rv, act

    def mcts_search_dev(self, G, obs_ptr, legal_ptr, tp_ptr, cv_ptr, rv_ptr, act_ptr, exploration=True,
                        rng_step=0, game_offset=0, temperature=1.0, stream=None):
        self._check(self.lib.mz_mcts_search_dev(self.h, G, obs_ptr, legal_ptr, tp_ptr, int(exploration),
                                                rng_step & 0xffffffff, game_offset, temperature, cv_ptr,
                                                rv_ptr, act_ptr, stream), "mz_mcts_search_dev")

    def set_sync_stream(self, stream, narrow=True):
        """Narrow the host-synchronous calls' wait to `stream` + the handle's own (mz_set_sync_stream)."""
        self._check(self.lib.mz_set_sync_stream(self.h, stream, int(narrow)), "mz_set_sync_stream")

    def debug_enable(self, flags=1):
        self._check(self.lib.mz_debug_enable(self.h, flags), "mz_debug_enable")

    def debug_tree(self, G):
        S, A = self.conf.num_iters, self.A
        eN = np.empty((G, S + 1, A), np.int32)
        eW = np.empty((G, S + 1, A), np.float32)
        eP = np.empty((G, S + 1, A), np.float32)
        eR = np.empty((G, S + 1, A), np.float32)
        eC = np.empty((G, S + 1, A), np.int32)
        ntp = np.empty((G, S + 1), np.int32)
        self._check(self.lib.mz_debug_tree(self.h, G, _p(eN), _p(eW), _p(eP), _p(eR), _p(eC), _p(ntp)),
                    "mz_debug_tree")
        return dict(N=eN, W=eW, P=eP, R=eR, C=eC, to_play=ntp)

    def debug_kernel_time(self):
        """(summed ms, launches) of the timed network launches since the last call."""
        t, n = ctypes.c_double(), ctypes.c_int()
        self._check(self.lib.mz_debug_kernel_time(self.h, ctypes.byref(t), ctypes.byref(n)), "mz_debug_kernel_time")
        return t.value, n.value

    def debug_unroll(self, B):
        """Read-outs of the last learner unroll: values (B, K+1), policies
        (B, K+1, A) as probabilities, rewards (B, K+1)."""
        K1 = self.conf.num_unroll_steps + 1
        pv = np.empty((B, K1), np.float32)
        pp = np.empty((B, K1, self.A), np.float32)
        pr = np.empty((B, K1), np.float32)
        self._check(self.lib.mz_debug_unroll(self.h, B, _p(pv), _p(pp), _p(pr)), "mz_debug_unroll")
        return pv, pp, pr

    def debug_unroll_step(self, i, B):
        """debug_unroll of step step0 + i of the last learner_train_multi_dev."""
        K1 = self.conf.num_unroll_steps + 1
        pv = np.empty((B, K1), np.float32)
        pp = np.empty((B, K1, self.A), np.float32)
        pr = np.empty((B, K1), np.float32)
        self._check(self.lib.mz_debug_unroll_step(self.h, i, B, _p(pv), _p(pp), _p(pr)), "mz_debug_unroll_step")
        return pv, pp, pr

    # ---- learner
    def learner_step(self, batch, eta):
        """batch: dict with observation (B, F), actions (B, K+1), target_values (B, K+1),
        target_rewards (B, K+1), target_policies (B, K+1, A), gradient_scale (B) and,
        with PER, weights (B)."""
        arrs = {k: np.ascontiguousarray(batch[k], dtype=np.float32) for k in
                ("observation", "actions", "target_values", "target_rewards", "target_policies", "gradient_scale")}
        w = batch.get("weights")
        w = None if w is None else np.ascontiguousarray(w, dtype=np.float32)
        b = MzBatch(arrs["observation"].shape[0], _p(arrs["observation"]), _p(arrs["actions"]),
                    _p(arrs["target_values"]), _p(arrs["target_rewards"]), _p(arrs["target_policies"]),
                    _p(arrs["gradient_scale"]), _p(w))
        losses = np.empty(6, np.float32)
        self._check(self.lib.mz_learner_step(self.h, ctypes.byref(b), float(eta), _p(losses)), "mz_learner_step")
        return losses

    def grad_count(self):
        n = ctypes.c_size_t()
        self._check(self.lib.mz_grad_count(self.h, ctypes.byref(n)), "mz_grad_count")
        return n.value

    def learner_grad_dev(self, dev_batch_ptrs, B, grad_ptr, losses_ptr=None, stream=None):
        b = MzBatch(B, *dev_batch_ptrs)
        self._check(self.lib.mz_learner_grad_dev(self.h, ctypes.byref(b), grad_ptr, losses_ptr, stream),
                    "mz_learner_grad_dev")

    def learner_apply_dev(self, grad_ptr, grad_scale, eta, stream=None):
        self._check(self.lib.mz_learner_apply_dev(self.h, grad_ptr, grad_scale, float(eta), stream),
                    "mz_learner_apply_dev")

    # ---- device self-play + replay shard
    def selfplay_init(self, env_kind, G, replay_games):
        self._check(self.lib.mz_selfplay_init(self.h, env_kind, G, replay_games), "mz_selfplay_init")
        self.sp_G = G
        self.osz = int(np.prod(self.conf.observation_shape))
        if env_kind == ENV_ATARI:                      # one 84x84 frame per move in the records
            self.osz = int(self.conf.observation_shape[0] * self.conf.observation_shape[1])

    def selfplay_move(self, rng_step, game_offset=0, temperature=1.0, stream=None):
        self._check(self.lib.mz_selfplay_move(self.h, rng_step, game_offset, temperature, stream),
                    "mz_selfplay_move")

    def learner_set_mode(self, mode):
        """LEARN_REF_SEMANTICS (∇ = 2θ, quirk Q11) or LEARN_CORRECTED (backprop)."""
        self._check(self.lib.mz_learner_set_mode(self.h, mode), "mz_learner_set_mode")

    def train_init(self, batch_size, t0=0):
        """Actor–learner loop (self_play! ‖ learning!, Q16): actors and the
        queued nets start from the current weights (mz_train_init_at; t0 = the
        learner step to continue from, e.g. a loaded checkpoint's)."""
        self._check(self.lib.mz_train_init_at(self.h, batch_size, int(t0)), "mz_train_init_at")

    def train_set_networks_path(self, path):
        """conf.networks_path: periodic checkpoints <path>/<t>.safetensors past
        0.9 training_steps (Learning.jl:416-432); None = none."""
        self._check(self.lib.mz_train_set_networks_path(self.h, path.encode() if path else None),
                    "mz_train_set_networks_path")

    def train_run(self, moves, move0=0, game_offset=0, losses_ptr=None, stream=None):
        """`moves` self-play moves with the actors' nets, one learner step per
        finished game, actor refresh every checkpoint_interval steps; returns
        (t, num_played_games, actor refreshes, learner steps of this call)."""
        st = np.zeros(4, np.int64)
        self._check(self.lib.mz_train_run(self.h, moves, move0, game_offset, _p(st), losses_ptr, stream),
                    "mz_train_run")
        return tuple(int(x) for x in st)

    def train_move(self, move, game_offset=0, stream=None):
        """One self-play move of the actor-learner loop with the actors' nets; returns the games it saved
        (this rank's shard).  A data-parallel host sums that over the ranks and passes it to train_learn."""
        n = np.zeros(1, np.int64)
        self._check(self.lib.mz_train_move(self.h, move, game_offset, _p(n), stream), "mz_train_move")
        return int(n[0])

    def train_learn(self, steps, losses_ptr=None, stream=None):
        """`steps` learner steps (capped at training_steps) with the actor refreshes; returns
        (t, num_played_games, actor refreshes, learner steps of this call)."""
        st = np.zeros(4, np.int64)
        self._check(self.lib.mz_train_learn(self.h, int(steps), losses_ptr, _p(st), stream), "mz_train_learn")
        return tuple(int(x) for x in st)

    def train_weights(self, which, net):
        """Flux-order weights of the learner / actors / queued nets."""
        out = np.empty(self.param_count(net), np.float32)
        self._check(self.lib.mz_train_weights_get(self.h, which, net, _p(out), out.size), "mz_train_weights_get")
        return out

    def selfplay_mode(self, mode, opponent=OPP_SELF, muzero_player=1):
        """SP_TRAIN (self_play!) or SP_EVAL (competitive_play!: games tallied, not saved)."""
        self._check(self.lib.mz_selfplay_mode(self.h, mode, opponent, muzero_player), "mz_selfplay_mode")

    def eval_results(self):
        """(games finished, MuZero wins, opponent wins, draws) since selfplay_init."""
        out = np.zeros(4, np.int64)
        self._check(self.lib.mz_eval_results(self.h, _p(out)), "mz_eval_results")
        return tuple(int(x) for x in out)

    def replay_counts(self):
        """({num_played_games, num_played_steps, total_samples}, games held)."""
        c = np.zeros(3, np.int64)
        n = ctypes.c_int32()
        self._check(self.lib.mz_replay_counts(self.h, _p(c), ctypes.byref(n)), "mz_replay_counts")
        return c, n.value

    def replay_save_game(self, hist):
        """save_game of a host GameHistory (selfplay.GameHistory)."""
        a = hist.as_arrays()
        obs = np.ascontiguousarray(a["observation"], np.uint8)      # 0/1 planes, or frame bytes
        self._check(self.lib.mz_replay_save_game(
            self.h, len(a["action"]), _p(obs), _p(np.ascontiguousarray(a["action"], np.int32)),
            _p(np.ascontiguousarray(a["reward"], np.float32)), _p(np.ascontiguousarray(a["to_play"], np.int32)),
            _p(np.ascontiguousarray(a["child_visits"], np.float32)),
            _p(np.ascontiguousarray(a["root_values"], np.float32))), "mz_replay_save_game")

    def replay_get_game(self, i):
        """Game i of the shard (0 = oldest held) as a selfplay.GameHistory."""
        from .selfplay import GameHistory
        Tm = self.conf.max_moves + 1
        T = ctypes.c_int32()
        obs = np.zeros((Tm, self.osz), np.uint8)
        act = np.zeros(Tm, np.int32)
        rew = np.zeros(Tm, np.float32)
        tp = np.zeros(Tm, np.int32)
        cv = np.zeros((Tm, self.A), np.float32)
        rv = np.zeros(Tm, np.float32)
        self._check(self.lib.mz_replay_get_game(self.h, i, ctypes.byref(T), _p(obs), _p(act), _p(rew), _p(tp),
                                                _p(cv), _p(rv)), "mz_replay_get_game")
        n = T.value
        return GameHistory(observation_history=[o.astype(np.float32) for o in obs[:n]],
                           action_history=[int(x) for x in act[:n]], reward_history=[float(x) for x in rew[:n]],
                           to_play_history=[int(x) for x in tp[:n]], child_visits=[c for c in cv[:n]],
                           root_values=[float(x) for x in rv[:n]])

    def replay_sample(self, B, step, stream=None, index=False):
        """Device get_batch: returns (MzBatch of device pointers, index_batch (B, 2) or None)."""
        b = MzBatch()
        idx = np.zeros((B, 2), np.int32) if index else None
        self._check(self.lib.mz_replay_sample(self.h, B, step, ctypes.byref(b), _p(idx) if index else None, stream),
                    "mz_replay_sample")
        return b, idx

    def learner_grad_sampled_dev(self, B, step, grad_ptr, losses_ptr=None, stream=None):
        """replay_sample(B, step) + learner_grad_dev, the sampling fused into the unroll kernel."""
        self._check(self.lib.mz_learner_grad_sampled_dev(self.h, B, step, grad_ptr, losses_ptr, stream),
                    "mz_learner_grad_sampled_dev")

    def learner_train_dev(self, B, step, eta, losses_ptr=None, stream=None):
        """One GPU: replay_sample + learner_grad_dev + learner_apply_dev(scale 1) in two launches."""
        self._check(self.lib.mz_learner_train_dev(self.h, B, step, float(eta), losses_ptr, stream),
                    "mz_learner_train_dev")

    def learner_train_multi_dev(self, B, step0, etas, losses_ptr=None, theta_ptr=None, stream=None):
        """len(etas) consecutive learner_train_dev steps step0 .. step0+L-1 (ref_semantics FC: the ADAM
        chain in one launch, the L unrolls + losses side by side in a second); losses_ptr: [L][8] floats,
        theta_ptr: [L][nflat] floats (the parameters after each step), both optional device pointers."""
        e = np.ascontiguousarray(etas, dtype=np.float64)
        self._check(self.lib.mz_learner_train_multi_dev(self.h, B, step0, e.size,
                                                        e.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                                        losses_ptr, theta_ptr, stream), "mz_learner_train_multi_dev")

    # ---- data-parallel learner over RCCL through the C ABI
    @staticmethod
    def dp_unique_id():
        """128-byte RCCL id (rank 0; hand it to every rank out of band)."""
        lib = load_library()
        buf = (ctypes.c_uint8 * 128)()
        if lib.mz_dp_unique_id(buf) != 0:
            raise MzError("mz_dp_unique_id failed (librccl.so.1)")
        return bytes(buf)

    def dp_init(self, rank, world, uid):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        self._check(self.lib.mz_dp_init(self.h, rank, world, buf), "mz_dp_init")

    def dp_allreduce(self, grad_ptr=None, stream=None):
        self._check(self.lib.mz_dp_allreduce(self.h, grad_ptr, stream), "mz_dp_allreduce")

    def learner_train_dp(self, B, step, eta, losses_ptr=None, stream=None):
        """grad_sampled_dev + RCCL all-reduce + apply(1/world) in one call."""
        self._check(self.lib.mz_learner_train_dp(self.h, B, step, float(eta), losses_ptr, stream),
                    "mz_learner_train_dp")

    def batch_to_host(self, b):
        """Copy a device MzBatch (from replay_sample) into the host dict layout of ReplayBuffer.get_batch."""
        B, K1, A = b.batch_size, self.conf.num_unroll_steps + 1, self.A
        self.sync()
        out = {}
        for name, shape in (("observation", (B, self.obs_feat)), ("actions", (B, K1)), ("target_values", (B, K1)),
                            ("target_rewards", (B, K1)), ("target_policies", (B, K1, A)), ("gradient_scale", (B,))):
            a = np.empty(shape, np.float32)
            _copy_d2h(a, getattr(b, name))
            out[name] = a
        if b.weights:                                   # PER importance weights
            a = np.empty(B, np.float32)
            _copy_d2h(a, b.weights)
            out["weights"] = a
        return out

    def replay_update_priorities(self, stream=None):
        """PER update_priorities! of the last sampled batch from the last unroll's values."""
        self._check(self.lib.mz_replay_update_priorities(self.h, stream), "mz_replay_update_priorities")

    def replay_get_priorities(self, i):
        """(priorities (T,), game priority) of shard game i (0 = oldest held)."""
        T = self.replay_get_game(i).as_arrays()["action"].shape[0]
        pr = np.zeros(T, np.float32)
        gp = np.zeros(1, np.float32)
        self._check(self.lib.mz_replay_get_priorities(self.h, i, _p(pr), _p(gp)), "mz_replay_get_priorities")
        return pr, float(gp[0])

    def selfplay_slots(self):
        G = self.sp_G
        ln = np.zeros(G, np.int32)
        board = np.zeros((G, self.osz), np.uint8)
        pl = np.zeros(G, np.int32)
        self._check(self.lib.mz_selfplay_slots(self.h, _p(ln), _p(board), _p(pl)), "mz_selfplay_slots")
        return ln, board, pl

    # ---- checkpoints
    def checkpoint_save(self, path, training_step):
        self._check(self.lib.mz_checkpoint_save(self.h, os.fsencode(path), int(training_step)), "mz_checkpoint_save")

    def checkpoint_load(self, path):
        """Restores weights + ADAM state; returns the checkpoint's training step."""
        step = ctypes.c_int64()
        self._check(self.lib.mz_checkpoint_load(self.h, os.fsencode(path), ctypes.byref(step)), "mz_checkpoint_load")
        return step.value

    def search_variant(self):
        return self.lib.mz_search_variant(self.h).decode()

    def learner_variant(self):
        return self.lib.mz_learner_variant(self.h).decode()

    def sync(self):
        self._check(self.lib.mz_sync(self.h), "mz_sync")
