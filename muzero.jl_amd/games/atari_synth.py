"""Synthetic Atari-like workload — BASELINE configs[4]: "Synthetic 84x84x4
Atari-like observations, conv repr+dynamics, 200 sims/move" (SURVEY §8d
config 5).  The reference ships no Atari game; its ResNet representation has
a `downsample` branch (src/Learning.jl:175-187) for exactly this input, so
this module is that branch's configuration:

* observations (84, 84, 4) f32 ~ U[0, 1) from a Philox stream (seed 0), the
  four channels read as four stacked grey frames (stacked_observations = 0,
  so the representation's input is the observation itself);
* 18 actions (the full Atari action set), one player, every action legal;
* ResNetHP with downsample = true: the downsampler takes 84x84 to 6x6
  (networks.resnet_board), then 64 filters, 2 residual blocks per tower.

The self-play data path (SelfPlay.jl:330-382 -> ReplayBuffer.jl:133-217) needs
an environment.  `BatchedAtariSynth` is a Philox-keyed stand-in with the shape
of a frame-stacked Atari game (same rules on the device, mz_selfplay.hip):

* state: a 32-bit key per game.  reset: key = u32(seed, ENV, game_offset +
  slot, step, ~0) — the global game id, so the ranks of a data-parallel job
  play different games (step = the move at which the slot restarts; ~0 for
  the initial games);
* frame(key): 84x84 bytes, column-major, the little-endian bytes of the words
  of Philox(c0 = j, c1 = key, c2 = 0, c3 = FRAME; seed), j = 0..440;
* step(a): (v0, v1, v2, _) = Philox(0, key, a, ENV; seed); reward 1 if
  below(v0, 18) == a - 1 else 0 (the mover's reward); terminal when
  v1 mod 128 == 0 (p = 1/128, "game over"), or past max_moves; key <- v2;
* observation at 1-based move index t: the frames of moves t-3 .. t as the
  four channels (newest last), zeros before move 1, each byte x as
  f32(x) * f32(1/255).  The history and the replay shard hold one frame per
  move (7,056 bytes), and the four-frame stack is rebuilt wherever an
  observation is needed (the env's own frame stacking, so
  stacked_observations = 0).
"""
import numpy as np

from ..config import Config, ResNetHP
from ..rng import philox_np, rng_below, rng_u32, _philox
from ..selfplay import frame_stack_obs  # noqa: F401  (the observation rule above)

W, H, C, A = 84, 84, 4, 18

conf = Config(
    observation_shape=(W, H, C),
    action_space=list(range(1, A + 1)),
    players=[1],
    stacked_observations=0,
    num_workers=1,
    max_moves=1000,                 # episodes end by the env (p = 1/128 per move) or here
    num_unroll_steps=5,
    td_steps=10,
    PER=False,
    opponent="none",
    training_steps=10000,
    batch_size=32,
    num_iters=200,
)

resnet_hyper = ResNetHP(
    num_blocks=2, depth_representation=0, num_filters=64, conv_kernel_size=(3, 3),
    hidden_state_size=6 * 6 * 64, representation_output_size=(6, 6, 64), depth_policy=1, depth_value=1,
    num_second_head_filters=2, num_first_head_filters=1, batch_norm_momentum=0.6, downsample=True,
    width_hidden=64, reward_activation="tanh")


def observations(G, seed=0, step=0):
    """(G, 84*84*4) column-major (W,H,C) observations ~ U[0,1) f32 from Philox(seed), advanced per step."""
    bg = np.random.Philox(key=seed)
    bg = bg.advance(step * ((G * W * H * C + 1) // 2 + 1)) if step else bg
    return np.random.Generator(bg).random((G, W * H * C), dtype=np.float32)


MZ_RNG_ENV, MZ_RNG_FRAME = 8, 9                  # include/mz_detmath.h
FRAME = W * H
FRAME_SCALE = np.float32(1.0) / np.float32(255.0)


def frame(seed, key):
    """The 84x84 frame bytes of env key `key`."""
    seed = int(seed)
    w = philox_np(np.arange(FRAME // 16), int(key), 0, MZ_RNG_FRAME, seed & 0xFFFFFFFF, seed >> 32)
    return np.stack(w, axis=1).astype("<u4").view(np.uint8).reshape(FRAME)


class BatchedAtariSynth:
    """G synthetic Atari-like games stepped together (the device env's rules)."""
    FRAME_STACK = C
    KEYED = True

    def __init__(self, G, seed=0, game_offset=0):
        self.G = G
        self.seed = int(seed)
        self.game_offset = int(game_offset)
        self.board = np.zeros((G, FRAME), np.uint8)       # the current frame
        self.player = np.ones(G, np.int32)
        self.key = np.zeros(G, np.uint32)
        self.reset(np.arange(G))

    def reset(self, idx, step=None):
        s = 0xFFFFFFFF if step is None else int(step)
        for g in np.atleast_1d(idx):
            self.key[g] = rng_u32(self.seed, MZ_RNG_ENV, self.game_offset + int(g), s, 0xFFFFFFFF)
            self.board[g] = frame(self.seed, self.key[g])

    def legal_mask(self):
        return np.ones((self.G, A), bool)

    def step(self, actions):
        """actions 1-based (G,); returns (reward for the mover, done)."""
        reward = np.zeros(self.G, np.float32)
        done = np.zeros(self.G, bool)
        for g in range(self.G):
            a = int(actions[g])
            v0, v1, v2, _ = _philox(0, int(self.key[g]), a, MZ_RNG_ENV, self.seed & 0xFFFFFFFF, self.seed >> 32)
            reward[g] = 1.0 if rng_below(v0, A) == a - 1 else 0.0
            done[g] = (v1 & 127) == 0
            self.key[g] = v2
            self.board[g] = frame(self.seed, v2)
        return reward, done
