"""muzero.jl_amd — MI355X-native MuZero self-play + learner hot path.

Python host mirror of deveshjawla/MuZero.jl's plugin surface (Config /
FeedForwardHP, the TicTacToe AbstractEnv, run_mcts / play_game / self_play!,
the ReplayBuffer and learning!) over the C ABI of libmz (include/mz.h), whose
kernels are hand-written HIP for gfx950.  Load via `_mzpkg.load()`.
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# MZ_LIB: an A/B variant of the library (tools/build_variants.py); default the in-tree build
LIB_PATH = os.environ.get("MZ_LIB") or os.path.join(PKG_DIR, "lib", "libmz.so")
