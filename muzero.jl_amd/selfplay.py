"""Self-play host driver — the Python mirror of src/SelfPlay.jl over libmz.

The search itself (run_mcts + select_action + store_search_stats!,
SelfPlay.jl:115-306) runs as one HIP kernel per move for the whole batch of
games; this module keeps the reference's game loop (play_game, :330-382),
the stacked observations (:128-149) and the GameHistory records
(Constructors.jl:6-16).  Games advance in lockstep; a finished slot is reset
and starts a new game (continuous batched self-play).  RNG step keys: the
global move counter `step` (unique per move across the run), game id = slot.
"""
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .config import stacked_features
from .rng import rng_below, rng_u32

MZ_RNG_OPPONENT = 7                                               # include/mz_detmath.h


def game_winner(env_name, last_reward, last_mover):
    """Winner of a finished game from its last move (0 = draw).  TicTacToe with
    Q14: the win test after a move looks at the plane of the player then to
    move, so a nonzero reward means 3 - mover holds a line; Connect4: the mover."""
    if last_reward == 0.0:
        return 0
    return 3 - last_mover if env_name == "tictactoe" else last_mover


def visit_softmax_temperature_fn(trained_steps: int) -> float:   # SelfPlay.jl:48-56
    if trained_steps < 500e3:
        return 1.0
    elif trained_steps < 750e3:
        return 0.5
    return 0.25


@dataclass
class GameHistory:                                               # Constructors.jl:6-16
    observation_history: List[np.ndarray] = field(default_factory=list)   # (W*H*C,) per move
    action_history: List[int] = field(default_factory=list)
    reward_history: List[float] = field(default_factory=list)
    to_play_history: List[int] = field(default_factory=list)
    child_visits: List[np.ndarray] = field(default_factory=list)          # (A,) per move
    root_values: List[float] = field(default_factory=list)
    reanalysed_predicted_root_values: Optional[list] = None
    priorities: Optional[np.ndarray] = None
    game_priority: Optional[float] = None

    def as_arrays(self):
        return dict(observation=np.array(self.observation_history, np.float32),
                    action=np.array(self.action_history, np.int32),
                    reward=np.array(self.reward_history, np.float32),
                    to_play=np.array(self.to_play_history, np.int32),
                    child_visits=np.array(self.child_visits, np.float32),
                    root_values=np.array(self.root_values, np.float32))


def frame_stack_obs(frames, index, n):
    """The frame-stacked observation at 1-based move `index` (games/atari_synth.py):
    frames index-n+1 .. index as the channels, zeros before move 1, bytes x f32(1/255)."""
    plane = np.asarray(frames[0]).size
    out = np.zeros(n * plane, np.float32)
    scale = np.float32(1.0) / np.float32(255.0)
    for c in range(n):
        s = index - n + 1 + c
        if s >= 1:
            out[c * plane:(c + 1) * plane] = np.asarray(frames[s - 1], np.uint8).astype(np.float32) * scale
    return out


def get_stacked_observations(obs_hist, action_hist, index, num_stacked, plane):
    """SelfPlay.jl:128-149 (Q15): [obs_t, (action plane, obs_{t-1}) ...], zeros before
    the first move; the action plane holds the raw action id.  `index` is 1-based."""
    parts = [np.asarray(obs_hist[index - 1], np.float32)]
    osz = parts[0].size
    for past in range(index - 1, index - num_stacked - 1, -1):
        if past >= 1:
            parts.append(np.full(plane, float(action_hist[past - 1]), np.float32))
            parts.append(np.asarray(obs_hist[past - 1], np.float32))
        else:
            parts.append(np.zeros(plane + osz, np.float32))
    return np.concatenate(parts)


class BatchedSelfPlay:
    """G TicTacToe games played in lockstep on one engine (one GPU)."""

    def __init__(self, engine, env_cls, G, game_offset=0, step0=0, opponent="self", muzero_player=1):
        """opponent "self" (self_play!, SelfPlay.jl:384-419) or "random": the
        player != muzero_player plays a uniform legal action
        (select_opponent_action, :311-325) — competitive_play! (:421-435)."""
        assert opponent in ("self", "random") and muzero_player in (1, 2)
        self.opponent = opponent
        self.muzero_player = muzero_player
        self.eng = engine
        self.conf = engine.conf
        self.G = G
        # keyed envs (games/atari_synth.py) draw from the engine's Philox streams
        self.env = (env_cls(G, seed=engine.rng_seed, game_offset=game_offset) if getattr(env_cls, "KEYED", False)
                    else env_cls(G))
        self.frame_stack = getattr(env_cls, "FRAME_STACK", 0)
        self.game_offset = game_offset
        self.step = step0
        self.plane = self.conf.observation_shape[0] * self.conf.observation_shape[1]
        self.histories = [GameHistory() for _ in range(G)]
        self.finished: List[GameHistory] = []

    def _stacked(self):
        c = self.conf
        out = np.empty((self.G, stacked_features(c)), np.float32)
        for g, h in enumerate(self.histories):
            if self.frame_stack:                         # the env's own frame stack (atari_synth)
                out[g] = frame_stack_obs(h.observation_history, len(h.observation_history), self.frame_stack)
                continue
            out[g] = get_stacked_observations(h.observation_history, h.action_history,
                                              len(h.observation_history), c.stacked_observations, self.plane)
        return out

    def play_move(self, temperature=1.0):
        """One move of every game (play_game's loop body, SelfPlay.jl:343-380)."""
        c = self.conf
        tp = self.env.player.copy()                                           # :351
        for g, h in enumerate(self.histories):
            h.observation_history.append(self.env.board[g].copy() if self.frame_stack else
                                         self.env.board[g].astype(np.float32))   # :352
        obs = self._stacked()                                                 # :355
        legal = self.env.legal_mask()
        cv, rv, act = self.eng.mcts_search(obs, legal, tp, exploration=True, rng_step=self.step,
                                           game_offset=self.game_offset, temperature=temperature)  # :359-360
        if c.temperature_threshold is not None:
            # :344-346: a game with >= temperature_threshold moves plays at temperature 0.
            # A game's search depends only on its own inputs and Philox keys (game id,
            # step), so the batch is searched again at 0 and those games take that action.
            moves = np.array([len(h.action_history) for h in self.histories])
            cold = moves >= c.temperature_threshold
            if cold.any() and temperature != 0.0:
                _, _, act0 = self.eng.mcts_search(obs, legal, tp, exploration=True, rng_step=self.step,
                                                  game_offset=self.game_offset, temperature=0.0)
                act = np.where(cold, act0, act)
        if self.opponent == "random":                                         # :357-362, :321
            for g in np.flatnonzero(tp != self.muzero_player):
                acts = np.flatnonzero(legal[g])
                if len(acts):
                    r = rng_u32(self.eng.rng_seed, MZ_RNG_OPPONENT, self.game_offset + int(g), self.step, 0)
                    act[g] = acts[rng_below(r, len(acts))] + 1
        reward, done = self.env.step(act)                                     # :366-368
        for g, h in enumerate(self.histories):                                # :375-379
            h.child_visits.append(cv[g])
            h.root_values.append(float(rv[g]))
            h.action_history.append(int(act[g]))
            h.reward_history.append(float(reward[g]))
            h.to_play_history.append(int(tp[g]))
        too_long = np.array([len(h.action_history) > c.max_moves for h in self.histories])
        ended = np.flatnonzero(done | too_long)
        for g in ended:
            self.finished.append(self.histories[g])
            self.histories[g] = GameHistory()
        if len(ended):
            if getattr(self.env, "KEYED", False):
                self.env.reset(ended, step=self.step)
            else:
                self.env.reset(ended)
        self.step += 1
        return ended

    def play_games(self, temperature=1.0):
        """Play every slot's current game to the end (no new games started);
        returns the histories in slot order."""
        results: List[Optional[GameHistory]] = [None] * self.G
        active = np.ones(self.G, bool)
        while active.any():
            n0 = len(self.finished)
            ended = self.play_move(temperature)
            for k, g in enumerate(ended):
                if active[g]:
                    results[g] = self.finished[n0 + k]
                    active[g] = False
        return results


def random_positions(env_cls, G, seed=0, max_plies=6):
    """Real positions for benchmarking (any env with [p1, p2, empty] board
    planes, stacked_observations = 1): random legal play from the initial
    board for 0..max_plies plies; returns stacked observations (G, F), legal
    masks (G, A) and to_play (G,).  Positions that ended are replaced by the
    initial board."""
    rng = np.random.default_rng(seed)
    env = env_cls(G)
    osz = env.board.shape[1]
    plane = osz // 3
    prev_obs = np.zeros((G, osz), np.float32)
    prev_act = np.zeros(G, np.int32)
    plies = rng.integers(0, max_plies + 1, G)
    alive = np.ones(G, bool)
    for t in range(max_plies):
        legal = env.legal_mask()
        go = (plies > t) & alive & legal.any(1)
        if not go.any():
            break
        # games not playing this ply take their first legal move and are restored below
        choice = np.array([rng.choice(np.flatnonzero(legal[g])) + 1 if go[g] else int(np.argmax(legal[g])) + 1
                           for g in range(G)], np.int32)
        before = env.board.astype(np.float32)
        saved = {k: v.copy() for k, v in vars(env).items() if isinstance(v, np.ndarray)}
        _, done = env.step(choice)
        for k, v in saved.items():                       # games not playing this ply keep their state
            getattr(env, k)[~go] = v[~go]
        prev_obs[go] = before[go]
        prev_act[go] = choice[go]
        ended = go & done
        if ended.any():
            env.reset(np.flatnonzero(ended))
            prev_obs[ended] = 0
            prev_act[ended] = 0
            alive &= ~ended
    cur = env.board.astype(np.float32)
    planes = np.repeat(prev_act[:, None].astype(np.float32), plane, axis=1)
    obs = np.concatenate([cur, planes, prev_obs], axis=1)
    return obs, env.legal_mask(), env.player.copy()
