"""Diagnostic: per-phase ticks of the learner unroll kernel (mz_unroll_small*)
from the -DMZ_STAMPS build made by tools/stamps.py.  Shares only."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime)
import _mzpkg  # noqa: E402

pkg = _mzpkg.load()
from muzero_jl_amd import abi  # noqa: E402
from muzero_jl_amd.games import tictactoe as ttt  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402

PHASES = ["setup", "repr", "sim gather", "step inputs", "8 stages", "raw writes"]


def main():
    lib = os.path.join(pkg.PKG_DIR, "lib", "libmz_stamps.so")
    abi._lib = None
    L = abi.load_library(lib)
    L.mz_debug_stamps.restype = ctypes.c_int
    L.mz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    conf, hyper = ttt.conf, ttt.hyper
    B, K, A = conf.batch_size, conf.num_unroll_steps, len(conf.action_space)
    eng = abi.Engine(conf, hyper, device=0, max_games=512, rng_seed=1)
    for n, w in enumerate(init_nets(conf, hyper, seed=1234)):
        eng.set_weights(n, w)
    rng = np.random.default_rng(0)
    feat = eng.obs_feat if hasattr(eng, "obs_feat") else 63
    batch = dict(observation=(rng.random((B, feat)) < 0.4).astype(np.float32),
                 actions=rng.integers(1, A + 1, (B, K + 1)).astype(np.float32),
                 target_values=rng.standard_normal((B, K + 1)).astype(np.float32),
                 target_rewards=np.zeros((B, K + 1), np.float32),
                 target_policies=np.full((B, K + 1, A), 1.0 / A, np.float32),
                 gradient_scale=np.full(B, float(K), np.float32))
    for k in range(3):
        eng.learner_step(batch, 1e-3)
    out = np.zeros((B, 8), np.uint64)
    assert L.mz_debug_stamps(eng.h, out.ctypes.data_as(ctypes.c_void_p), B) == 0
    out = out[out.sum(1) > 0].astype(np.float64)
    med = np.median(out, axis=0)
    print(f"unroll B={B} K={K}: median ticks per workgroup ({len(out)} blocks)")
    for i, p in enumerate(PHASES):
        print(f"  {p:12s} {med[i]:10.0f}")
    print("  total       ", np.median(out.sum(1)))


if __name__ == "__main__":
    main()
