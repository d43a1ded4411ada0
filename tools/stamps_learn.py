"""Diagnostic: phase ticks of the one-launch learner step (mz_learn_small*,
mz_learner_train_dev) from the -DMZ_STAMPS build (libmz_stamps.so): per unroll
workgroup the unroll phases, the whole unroll and the loss terms.  Shares only."""
import ctypes
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime)
import _mzpkg  # noqa: E402

pkg = _mzpkg.load()
from muzero_jl_amd import abi  # noqa: E402
from muzero_jl_amd.config import cos_schedule  # noqa: E402
from muzero_jl_amd.games import tictactoe as ttt  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402

PHASES = ["setup", "repr", "sim gather", "step inputs", "8 stages", "raw writes", "unroll total", "loss terms"]


def main():
    abi._lib = None
    L = abi.load_library(os.path.join(pkg.PKG_DIR, "lib", os.environ.get("STAMPS_LIB", "libmz_stamps.so")))
    L.mz_debug_stamps.restype = ctypes.c_int
    L.mz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    conf = dataclasses.replace(ttt.conf, num_iters=8)
    B = int(os.environ.get("B", conf.batch_size))
    eng = abi.Engine(conf, ttt.hyper, device=0, max_games=512, rng_seed=1)
    for n, w in enumerate(init_nets(conf, ttt.hyper, seed=1234)):
        eng.set_weights(n, w)
    eng.selfplay_init(abi.ENV_TICTACTOE, 64, 256)
    for m in range(12):
        eng.selfplay_move(m)
    for k in range(4):
        eng.learner_train_dev(B, k + 1, cos_schedule(k + 1))
    eng.sync()
    out = np.zeros((B, 8), np.uint64)
    assert L.mz_debug_stamps(eng.h, out.ctypes.data_as(ctypes.c_void_p), B) == 0
    med = np.median(out.astype(np.float64), axis=0)
    print(f"one-launch learner B={B}: median ticks per unroll workgroup")
    for i, p in enumerate(PHASES):
        print(f"  {p:13s} {med[i]:10.0f}")
    eng.close()


if __name__ == "__main__":
    main()
