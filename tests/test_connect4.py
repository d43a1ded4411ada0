"""Connect4 env rules (BASELINE configs[3]'s new env, games/connect4.py): the
host env that the device env (mz_selfplay.hip) is pinned against."""
import numpy as np


def _play(env, moves):
    out = []
    for a in moves:
        out.append(env.step(np.array([a], np.int32)))
    return out


def test_vertical_win_and_legal_after():
    from muzero_jl_amd.games.connect4 import BatchedConnect4
    env = BatchedConnect4(1)
    res = _play(env, [1, 2, 1, 2, 1, 2, 1])
    assert all(not d[0] for _, d in res[:-1])
    r, d = res[-1]
    assert d[0] and r[0] == 1.0
    assert not env.legal_mask().any()                       # no moves once the game is over


def test_horizontal_and_diagonal_wins():
    from muzero_jl_amd.games.connect4 import BatchedConnect4
    env = BatchedConnect4(1)
    r, d = _play(env, [1, 1, 2, 2, 3, 3, 4])[-1]             # player 1: bottom row, columns 1-4
    assert d[0] and r[0] == 1.0
    env = BatchedConnect4(1)
    # player 2 wins a rising diagonal: (0,1)(1,2)(2,3)(3,4) in (row, column)
    r, d = _play(env, [1, 2, 3, 3, 4, 4, 5, 4, 5, 5, 1, 5])[-1]
    assert d[0] and r[0] == 1.0 and env.player[0] == 1


def test_full_column_is_illegal_and_board_planes():
    from muzero_jl_amd.games.connect4 import BatchedConnect4, CELLS, W
    env = BatchedConnect4(1)
    _play(env, [3, 3, 3, 3, 3, 3])                          # column 3 full, alternating, no line
    m = env.legal_mask()[0]
    assert not m[2] and m.sum() == 6
    b = env.board[0]
    assert b[:CELLS].sum() == 3 and b[CELLS:2 * CELLS].sum() == 3 and b[2 * CELLS:].sum() == CELLS - 6
    assert all(b[(k % 2) * CELLS + k + W * 2] for k in range(6))   # stones stacked from the bottom row up


def test_reset_subset():
    from muzero_jl_amd.games.connect4 import BatchedConnect4
    env = BatchedConnect4(3)
    env.step(np.array([1, 2, 3], np.int32))
    env.reset(np.array([1]))
    assert env.board[1, 84:].all() and env.player[1] == 1 and env.player[0] == 2
