"""Config / FeedForwardHP / ResNetHP with the reference's field names and
defaults (src/Constructors.jl:18-90), plus their ctypes mirrors of the
`mz_config` / `mz_ffhp` PODs of include/mz.h."""
import ctypes
import math
from dataclasses import dataclass, field
from typing import Optional, Tuple

ACT_IDENTITY, ACT_RELU, ACT_TANH = 0, 1, 2


@dataclass
class Config:                                   # Constructors.jl:18-52
    observation_shape: Tuple[int, int, int]
    action_space: list
    players: list
    stacked_observations: int
    num_workers: int
    max_moves: int
    num_iters: int
    num_unroll_steps: int
    td_steps: int
    PER: bool
    training_steps: int
    batch_size: int
    seed: int = 1337
    muzero_player: int = 1
    opponent: str = "expert"
    intermediate_rewards: bool = False
    selfplay_on_gpu: bool = False
    temperature_threshold: Optional[int] = None
    dirichlet_α: float = 0.25
    exploration_ϵ: float = 0.25
    pb_c_base: int = 19652
    pb_c_init: float = 1.25
    discount: float = 0.997
    replay_buffer_size: int = 10000
    PER_alpha: int = 1
    results_path: str = "./results"
    networks_path: str = "./networks"
    checkpoint_interval: int = 10
    value_loss_weight: float = 0.25


@dataclass
class FeedForwardHP:                            # Constructors.jl:62-75
    width_hidden: int
    depth_representation: int
    depth_prediction: int
    depth_dynamics: int
    depth_policy: int
    depth_value: int
    depth_reward: int
    depth_state_head: int
    hidden_state_size: int
    reward_activation: str = "tanh"
    use_batch_norm: bool = False
    batch_norm_momentum: float = 0.6


@dataclass
class ResNetHP:                                 # Constructors.jl:77-90 (path not runnable in the reference, Q12)
    num_blocks: int
    depth_representation: int
    num_filters: int
    conv_kernel_size: Tuple[int, int]
    hidden_state_size: int
    representation_output_size: Optional[tuple]
    depth_policy: int
    depth_value: int
    num_second_head_filters: int = 2
    num_first_head_filters: int = 1
    batch_norm_momentum: float = 0.6
    downsample: bool = False
    # read by the reference's ResNet heads (Learning.jl:203,235) but never
    # declared in ResNetHP (Q12): the intended architecture's Dense width
    width_hidden: int = 64
    reward_activation: object = "tanh"


class MzConfig(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_int32), ("observation_shape", ctypes.c_int32 * 3),
        ("action_space_size", ctypes.c_int32), ("players", ctypes.c_int32),
        ("stacked_observations", ctypes.c_int32), ("muzero_player", ctypes.c_int32),
        ("intermediate_rewards", ctypes.c_int32), ("num_workers", ctypes.c_int32),
        ("selfplay_on_gpu", ctypes.c_int32), ("max_moves", ctypes.c_int32),
        ("temperature_threshold", ctypes.c_int32), ("dirichlet_alpha", ctypes.c_float),
        ("exploration_eps", ctypes.c_float), ("pb_c_base", ctypes.c_int32),
        ("pb_c_init", ctypes.c_float), ("discount", ctypes.c_float), ("num_iters", ctypes.c_int32),
        ("replay_buffer_size", ctypes.c_int32), ("num_unroll_steps", ctypes.c_int32),
        ("td_steps", ctypes.c_int32), ("PER", ctypes.c_int32), ("PER_alpha", ctypes.c_int32),
        ("training_steps", ctypes.c_int32), ("batch_size", ctypes.c_int32),
        ("checkpoint_interval", ctypes.c_int32), ("value_loss_weight", ctypes.c_float),
    ]


class MzFFHP(ctypes.Structure):
    _fields_ = [
        ("width_hidden", ctypes.c_int32), ("depth_representation", ctypes.c_int32),
        ("depth_prediction", ctypes.c_int32), ("depth_dynamics", ctypes.c_int32),
        ("depth_policy", ctypes.c_int32), ("depth_value", ctypes.c_int32),
        ("depth_reward", ctypes.c_int32), ("depth_state_head", ctypes.c_int32),
        ("use_batch_norm", ctypes.c_int32), ("batch_norm_momentum", ctypes.c_float),
        ("hidden_state_size", ctypes.c_int32), ("reward_activation", ctypes.c_int32),
    ]


class MzResNetHP(ctypes.Structure):
    _fields_ = [
        ("num_blocks", ctypes.c_int32), ("num_filters", ctypes.c_int32),
        ("conv_kernel_size", ctypes.c_int32 * 2), ("num_second_head_filters", ctypes.c_int32),
        ("num_first_head_filters", ctypes.c_int32), ("batch_norm_momentum", ctypes.c_float),
        ("downsample", ctypes.c_int32), ("depth_policy", ctypes.c_int32), ("depth_value", ctypes.c_int32),
        ("width_hidden", ctypes.c_int32), ("reward_activation", ctypes.c_int32),
    ]


_ACTS = {"identity": ACT_IDENTITY, "relu": ACT_RELU, "tanh": ACT_TANH, None: ACT_IDENTITY}


def to_c_config(c: Config) -> MzConfig:
    m = MzConfig()
    m.seed = c.seed
    for i in range(3):
        m.observation_shape[i] = c.observation_shape[i]
    if list(c.action_space) != list(range(1, len(c.action_space) + 1)):
        raise ValueError("action_space must be 1:n")
    if list(c.players) != list(range(1, len(c.players) + 1)):
        raise ValueError("players must be 1:n")
    m.action_space_size = len(c.action_space)
    m.players = len(c.players)
    m.stacked_observations = c.stacked_observations
    m.muzero_player = c.muzero_player
    m.intermediate_rewards = int(c.intermediate_rewards)
    m.num_workers = c.num_workers
    m.selfplay_on_gpu = int(c.selfplay_on_gpu)
    m.max_moves = c.max_moves
    m.temperature_threshold = -1 if c.temperature_threshold is None else c.temperature_threshold
    m.dirichlet_alpha = c.dirichlet_α
    m.exploration_eps = c.exploration_ϵ
    m.pb_c_base = c.pb_c_base
    m.pb_c_init = c.pb_c_init
    m.discount = c.discount
    m.num_iters = c.num_iters
    m.replay_buffer_size = c.replay_buffer_size
    m.num_unroll_steps = c.num_unroll_steps
    m.td_steps = c.td_steps
    m.PER = int(c.PER)
    m.PER_alpha = c.PER_alpha
    m.training_steps = c.training_steps
    m.batch_size = c.batch_size
    m.checkpoint_interval = c.checkpoint_interval
    m.value_loss_weight = c.value_loss_weight
    return m


def to_c_ffhp(h: FeedForwardHP) -> MzFFHP:
    m = MzFFHP()
    for f in ("width_hidden", "depth_representation", "depth_prediction", "depth_dynamics",
              "depth_policy", "depth_value", "depth_reward", "depth_state_head", "hidden_state_size"):
        setattr(m, f, getattr(h, f))
    m.use_batch_norm = int(h.use_batch_norm)
    m.batch_norm_momentum = h.batch_norm_momentum
    act = h.reward_activation
    if callable(act):
        act = act.__name__
    m.reward_activation = _ACTS[act]
    return m


def to_c_resnet_hp(h: ResNetHP) -> MzResNetHP:
    m = MzResNetHP()
    for f in ("num_blocks", "num_filters", "num_second_head_filters", "num_first_head_filters",
              "depth_policy", "depth_value", "width_hidden"):
        setattr(m, f, getattr(h, f))
    m.conv_kernel_size[0], m.conv_kernel_size[1] = h.conv_kernel_size
    m.batch_norm_momentum = h.batch_norm_momentum
    m.downsample = int(bool(h.downsample))
    act = h.reward_activation
    if callable(act):
        act = act.__name__
    m.reward_activation = _ACTS[act]
    return m


def hidden_size(conf: Config, hyper) -> int:
    """Hidden-state floats: FeedForwardHP.hidden_state_size, or W*H*num_filters
    on the hidden board (after the downsampler when ResNetHP.downsample)."""
    if isinstance(hyper, ResNetHP):
        from .networks import resnet_board
        W, H = resnet_board(conf, hyper)
        return W * H * hyper.num_filters
    return hyper.hidden_state_size


def stacked_features(c: Config) -> int:
    """indim of init_representation (Learning.jl:88)."""
    w, h, ch = c.observation_shape
    return w * h * (ch * (c.stacked_observations + 1) + c.stacked_observations)


def cos_schedule(t: int, λ0: float = 1e-4, λ1: float = 1e-1, period: int = 10) -> float:
    """ParameterSchedulers 0.2.3 Cos(λ0, λ1, period) under Stateful, t = 1, 2, ...
    (Learning.jl:319, 382): |λ0-λ1|·(1+cos(2π(t-1)/period))/2 + min(λ0, λ1)."""
    rng = abs(λ0 - λ1)
    off = min(λ0, λ1)
    a = 6.283185307179586 * float(t - 1) / float(period)
    return rng * (1.0 + math.cos(a)) / 2.0 + off
