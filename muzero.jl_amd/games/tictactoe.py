"""TicTacToe AbstractEnv (games/tictactoe/game.jl) and its params
(games/tictactoe/params.jl), with the reference's exact rules (quirk Q14).

Board = BitArray (3,3,3) with planes [player 1, player 2, empty], stored as a
flat 27-vector in Julia's column-major order (cell + 9*plane); action a in 1..9
is CartesianIndices((3,3))[a] = cell a-1.  `is_win` checks the plane of the
player TO MOVE (game.jl:102-115); the walk-built state table labels any such
line winner=1 and terminates on it or on a full board (game.jl:117-147).
"""
import numpy as np

from ..config import Config, FeedForwardHP, ResNetHP

LINES = np.array([[0, 3, 6], [1, 4, 7], [2, 5, 8], [0, 1, 2], [3, 4, 5], [6, 7, 8], [0, 4, 8], [6, 4, 2]])

# games/tictactoe/params.jl:2-16
conf = Config(
    observation_shape=(3, 3, 3),
    action_space=list(range(1, 10)),
    players=[1, 2],
    stacked_observations=1,
    num_workers=2,
    max_moves=9,
    num_unroll_steps=5,
    td_steps=5,
    PER=False,
    opponent="human",
    training_steps=10000,
    batch_size=32,
    num_iters=10,
)

# games/tictactoe/params.jl:18-29
hyper = FeedForwardHP(
    width_hidden=64,
    depth_representation=3,
    depth_prediction=3,
    depth_dynamics=3,
    depth_policy=1,
    depth_value=1,
    depth_reward=1,
    depth_state_head=3,
    hidden_state_size=27,
    reward_activation="tanh",
)

# BASELINE config 3: the ResNet networks (intended architecture, SURVEY §2.1
# Q12; the reference ships no ResNet config): 3x3 representation convs,
# 64 filters, 2 residual blocks per tower, 1x1 convs in prediction / dynamics.
resnet_hyper = ResNetHP(
    num_blocks=2, depth_representation=0, num_filters=64, conv_kernel_size=(3, 3),
    hidden_state_size=3 * 3 * 64, representation_output_size=(3, 3, 64), depth_policy=1, depth_value=1,
    num_second_head_filters=2, num_first_head_filters=1, batch_norm_momentum=0.6, downsample=False,
    width_hidden=64, reward_activation="tanh")


class TicTacToe:
    """RLBase-style single environment (game.jl:3-100)."""

    def __init__(self):
        self.board = np.zeros(27, dtype=bool)
        self.board[18:] = True
        self.player = 1

    def reset(self):                                      # RLBase.reset! (:15-20)
        self.board[:] = False
        self.board[18:] = True
        self.player = 1
        return self.board

    def current_player(self):                             # :54
        return self.player

    def _line_to_move(self):
        pl = self.board[9 * (self.player - 1): 9 * self.player]
        return bool(np.any(pl[LINES].all(axis=1)))

    def legal_action_space_mask(self, p=None):            # :37-43
        if self._line_to_move():
            return np.zeros(9, dtype=bool)
        return self.board[18:].copy()

    def legal_action_space(self, p=None):                 # :35 findall(mask), 1-based
        return [i + 1 for i in np.flatnonzero(self.legal_action_space_mask(p))]

    def __call__(self, action):                           # env(action) (:45-52)
        c = action - 1
        self.board[18 + c] = False
        self.board[9 * (self.player - 1) + c] = True
        self.player = (self.player % 2) + 1
        return self.board

    def is_terminated(self):                              # :85 via the state table
        return (not self.board[18:].any()) or self._line_to_move()

    def reward(self, player):                             # :87-100
        if not self.is_terminated():
            return 0
        if not self._line_to_move():
            return 0
        return 1 if player == 1 else -1


class BatchedTicTacToe:
    """G independent TicTacToe games stepped together (numpy), for the batched
    self-play driver; same rules as TicTacToe."""

    def __init__(self, G):
        self.G = G
        self.board = np.zeros((G, 27), dtype=bool)
        self.player = np.ones(G, dtype=np.int32)
        self.reset_all()

    def reset_all(self):
        self.board[:] = False
        self.board[:, 18:] = True
        self.player[:] = 1

    def reset(self, idx):
        self.board[idx] = False
        self.board[idx, 18:] = True
        self.player[idx] = 1

    def _line_to_move(self):
        G = self.G
        off = 9 * (self.player - 1)
        cells = off[:, None, None] + LINES[None, :, :]
        vals = self.board[np.arange(G)[:, None, None], cells]
        return vals.all(axis=2).any(axis=1)

    def legal_mask(self):
        win = self._line_to_move()
        m = self.board[:, 18:].copy()
        m[win] = False
        return m

    def step(self, actions):
        """actions 1-based (G,); returns (reward for the mover, done)."""
        G = self.G
        mover = self.player.copy()
        c = actions - 1
        r = np.arange(G)
        self.board[r, 18 + c] = False
        self.board[r, 9 * (self.player - 1) + c] = True
        self.player = (self.player % 2) + 1
        win = self._line_to_move()
        full = ~self.board[:, 18:].any(axis=1)
        done = full | win
        reward = np.where(done & win, np.where(mover == 1, 1.0, -1.0), 0.0).astype(np.float32)
        return reward, done
