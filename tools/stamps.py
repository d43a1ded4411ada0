"""Diagnostic: per-phase cycle breakdown of the search kernels from a separate
-DMZ_STAMPS build (libmz_stamps.so).  Shares only; never quote its run time."""
import ctypes
import dataclasses
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import _mzpkg  # noqa: E402

pkg = _mzpkg.load()
from muzero_jl_amd import abi, build as mzbuild  # noqa: E402
from muzero_jl_amd.games import tictactoe as ttt  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402
from muzero_jl_amd.selfplay import random_positions  # noqa: E402

PHASES = ["root", "select", "gather", "nets", "expand", "backup", "recomp", "-"]


def main():
    lib = os.path.join(pkg.PKG_DIR, "lib", "libmz_stamps.so")
    srcs = [os.path.join(pkg.PKG_DIR, "csrc", s) for s in mzbuild.SOURCES]
    if "--no-build" not in sys.argv:
        extra = os.environ.get("STAMPS_DEFS", "").split()
        subprocess.run(["/opt/rocm/bin/hipcc"] + mzbuild.FLAGS + ["-DMZ_STAMPS"] + extra + ["-shared", "-o", lib] + srcs,
                       check=True)
    abi._lib = None
    L = abi.load_library(lib)
    L.mz_debug_stamps.restype = ctypes.c_int
    L.mz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    G = int(os.environ.get("G", "512"))
    S = int(os.environ.get("S", "50"))
    conf = dataclasses.replace(ttt.conf, num_iters=S)
    eng = abi.Engine(conf, ttt.hyper, device=0, max_games=G, rng_seed=1)
    for n, w in enumerate(init_nets(conf, ttt.hyper, seed=1234)):
        eng.set_weights(n, w)
    obs, legal, tp = random_positions(ttt.BatchedTicTacToe, G, seed=100)
    for k in range(3):
        eng.mcts_search(obs, legal, tp, rng_step=k)
    out = np.zeros((G, 8), np.uint64)
    assert L.mz_debug_stamps(eng.h, out.ctypes.data_as(ctypes.c_void_p), G) == 0
    var = eng.search_variant()
    nb = -(-G // int(var.split("small")[1][0])) if "small" in var else G
    wv = out[nb:2 * nb].astype(np.float64) if 2 * nb <= G else None   # per-wave post-network phase (small*)
    out = out[:nb]
    out = out[out.sum(1) > 0]
    print("variant", var, "blocks", len(out))
    if wv is not None and wv.sum() > 0:
        med = np.median(wv, axis=0)
        print(f"  post-network phase per wave, per sim: wave 0 backup {med[0] / S:.0f}, wave 2 expand "
              f"{med[1] / S:.0f}, wave 3 h' store {med[2] / S:.0f} (ticks)")
    levels = out[:, 7].astype(np.float64)
    out[:, 7] = 0
    tot = out.sum(1).astype(np.float64)
    med = np.median(out.astype(np.float64), axis=0)
    print(f"G={G} S={S}: median cycles per workgroup (s_memtime ticks, 100 MHz ref? see note)")
    for i, p in enumerate(PHASES[:7]):
        print(f"  {p:8s} {med[i]:12.0f}  per-sim {med[i] / S:10.1f}  share {med[i] / np.median(tot):6.3f}")
    print("  total   ", np.median(tot))
    print(f"  select levels per sim (max over the workgroup's games): {np.median(levels) / S:.2f}; "
          f"ticks per level {med[1] / np.median(levels):.1f}")


if __name__ == "__main__":
    main()
