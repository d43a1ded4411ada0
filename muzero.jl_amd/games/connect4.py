"""Connect4 env — the "Connect4-style 6x7 board (new AbstractGame env)" of
BASELINE configs[3].  The reference ships no Connect4, so this module defines
it, on the same AbstractEnv surface as games/tictactoe.py (game.jl:3-100):

Board = BitArray (6,7,3) with planes [player 1, player 2, empty], stored as a
flat 126-vector in column-major order: cell (w, h) = w + 6h with w the row
(0 = bottom) and h the column, plane offset 42·plane.  Action a in 1..7 drops
a stone in column a-1 onto its lowest empty row.  Standard rules: four in a
row (vertical, horizontal or diagonal) through the stone just played wins, a
full board is a draw.  reward(env, p) is +1 for the winner, so the reward
recorded for a move (SelfPlay.jl:366-368, reward of the mover) is +1 for a
winning move and 0 otherwise.  No legal actions once the game is over.
The device env (mz_selfplay.hip) implements the same rules; the tests pin one
against the other.
"""
import numpy as np

from ..config import Config, FeedForwardHP, ResNetHP

W, H = 6, 7
CELLS = W * H

conf = Config(
    observation_shape=(W, H, 3),
    action_space=list(range(1, H + 1)),
    players=[1, 2],
    stacked_observations=1,
    num_workers=2,
    max_moves=CELLS,
    num_unroll_steps=5,
    td_steps=10,
    PER=False,
    opponent="human",
    training_steps=10000,
    batch_size=32,
    num_iters=50,
)

# the FC networks of games/tictactoe/params.jl:18-29 on this board (the FC
# path reshapes h to the observation, so hidden_state_size = 6·7·3)
hyper = FeedForwardHP(
    width_hidden=64, depth_representation=3, depth_prediction=3, depth_dynamics=3, depth_policy=1, depth_value=1,
    depth_reward=1, depth_state_head=3, hidden_state_size=3 * CELLS, reward_activation="tanh")

# BASELINE configs[3]: "ResNet-8" read as 8 conv layers in the representation
# tower (4 residual blocks), 64 filters, 3x3 kernels
resnet_hyper = ResNetHP(
    num_blocks=4, depth_representation=0, num_filters=64, conv_kernel_size=(3, 3),
    hidden_state_size=CELLS * 64, representation_output_size=(W, H, 64), depth_policy=1, depth_value=1,
    num_second_head_filters=2, num_first_head_filters=1, batch_norm_momentum=0.6, downsample=False,
    width_hidden=64, reward_activation="tanh")

_DIRS = ((1, 0), (0, 1), (1, 1), (1, -1))


def _wins(stones, w, h):
    """Four in a row of `stones` (bool[CELLS]) through (w, h)."""
    for dw, dh in _DIRS:
        n = 1
        for s in (1, -1):
            ww, hh = w + s * dw, h + s * dh
            while 0 <= ww < W and 0 <= hh < H and stones[ww + W * hh]:
                n += 1
                ww += s * dw
                hh += s * dh
        if n >= 4:
            return True
    return False


class BatchedConnect4:
    """G independent Connect4 games stepped together; same rules as the device env."""

    def __init__(self, G):
        self.G = G
        self.board = np.zeros((G, 3 * CELLS), dtype=bool)
        self.player = np.ones(G, dtype=np.int32)
        self.over = np.zeros(G, dtype=bool)
        self.reset_all()

    def reset_all(self):
        self.reset(np.arange(self.G))

    def reset(self, idx):
        self.board[idx] = False
        self.board[idx, 2 * CELLS:] = True
        self.player[idx] = 1
        self.over[idx] = False

    def legal_mask(self):
        top = self.board[:, 2 * CELLS + (W - 1) + W * np.arange(H)]       # top cell of each column empty
        return np.ascontiguousarray(top & ~self.over[:, None])          # (G, A) row-major for the ABI

    def step(self, actions):
        """actions 1-based (G,); returns (reward for the mover, done)."""
        reward = np.zeros(self.G, np.float32)
        done = np.zeros(self.G, bool)
        for g in range(self.G):
            h = int(actions[g]) - 1
            empty = self.board[g, 2 * CELLS:]
            w = next(r for r in range(W) if empty[r + W * h])
            p = self.player[g]
            cell = w + W * h
            self.board[g, 2 * CELLS + cell] = False
            self.board[g, (p - 1) * CELLS + cell] = True
            win = _wins(self.board[g, (p - 1) * CELLS:p * CELLS], w, h)
            full = not self.board[g, 2 * CELLS:].any()
            done[g] = win or full
            reward[g] = 1.0 if win else 0.0
            self.over[g] = done[g]
            self.player[g] = 3 - p
        return reward, done
