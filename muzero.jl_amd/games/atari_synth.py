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
"""
import numpy as np

from ..config import Config, ResNetHP

W, H, C, A = 84, 84, 4, 18

conf = Config(
    observation_shape=(W, H, C),
    action_space=list(range(1, A + 1)),
    players=[1],
    stacked_observations=0,
    num_workers=1,
    max_moves=27000,
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
