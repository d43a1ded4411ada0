"""Diagnostic: run N multi-step learner chunks of length L (argv) on a TicTacToe FC engine
with a filled replay shard, for rocprofv3 kernel stats of mz_learn_chain / mz_learn_multi*."""
import dataclasses
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _mzpkg  # noqa: E402

_mzpkg.load()
from muzero_jl_amd import abi  # noqa: E402
from muzero_jl_amd.config import cos_schedule  # noqa: E402
from muzero_jl_amd.games import tictactoe as ttt  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402

L, N = int(sys.argv[1]), int(sys.argv[2]) if len(sys.argv) > 2 else 50
conf = dataclasses.replace(ttt.conf, num_iters=10)
e = abi.Engine(conf, ttt.hyper, device=0, max_games=64, rng_seed=1)
for n, w in enumerate(init_nets(conf, ttt.hyper, seed=3)):
    e.set_weights(n, w)
e.selfplay_init(abi.ENV_TICTACTOE, 64, 256)
for m in range(12):
    e.selfplay_move(m)
lm = torch.zeros((L, 8), dtype=torch.float32, device="cuda")
t = 1
for _ in range(N):
    e.learner_train_multi_dev(32, t, [cos_schedule(t + i) for i in range(L)], lm.data_ptr())
    t += L
e.sync()
print("ok", L, N, e.learner_variant())
