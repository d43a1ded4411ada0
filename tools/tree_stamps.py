"""Diagnostic: phase ticks (s_memtime) of the LDS-cached ResNet tree step
(mz_rsearch_tree_lds*), workgroup 0, every 4th simulation of one search, from
a separate -DMZ_STAMPS build (libmz_stamps.so).  Workload: the Atari-like
configs[4] (GAME=atari, default) or TicTacToe ResNet (GAME=ttt)."""
import ctypes
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import _mzpkg  # noqa: E402

pkg = _mzpkg.load()
from muzero_jl_amd import abi, build as mzbuild  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402

PH = ["copy issue", "copy wait", "expand", "backup", "recompute", "write-back", "select", "gather"]


def main():
    lib = os.path.join(pkg.PKG_DIR, "lib", "libmz_stamps.so")
    if "--no-build" not in sys.argv:
        mzbuild.build(out=lib, objdir=os.path.join(pkg.PKG_DIR, "lib", "obj_stamps"), extra=["-DMZ_STAMPS"])
    abi._lib = None
    L = abi.load_library(lib)
    L.mz_debug_stamps.restype = ctypes.c_int
    L.mz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    G = int(os.environ.get("G", "512"))
    if os.environ.get("GAME", "atari") == "atari":
        from muzero_jl_amd.games import atari_synth as gm
        conf, hyper = gm.conf, gm.resnet_hyper
        obs = gm.observations(G)
        legal = np.ones((G, len(conf.action_space)), bool)
        tp = np.ones(G, np.int32)
    else:
        from muzero_jl_amd.games import tictactoe as gm
        from muzero_jl_amd.selfplay import random_positions
        conf, hyper = gm.conf, gm.resnet_hyper
        obs, legal, tp = random_positions(gm.BatchedTicTacToe, G, seed=100)
    eng = abi.Engine(conf, hyper, device=0, max_games=G, rng_seed=1)
    for n, w in enumerate(init_nets(conf, hyper, seed=1234)):
        eng.set_weights(n, w)
    for k in range(2):
        eng.mcts_search(obs, legal, tp, rng_step=k)
    out = np.zeros(512 * 8, np.uint64)
    assert L.mz_debug_stamps(eng.h, out.ctypes.data_as(ctypes.c_void_p), 512) == 0
    st = out[1024:].astype(np.int64).reshape(-1, 16)
    print("s     " + " ".join(f"{p:>11s}" for p in PH) + "       total")
    for i in range(st.shape[0]):
        r = st[i]
        if not r[0]:
            continue
        prev, cells = r[0], []
        for k in range(1, 9):
            if r[k]:
                cells.append(f"{r[k] - prev:11d}")
                prev = r[k]
            else:
                cells.append(f"{'-':>11s}")
        print(f"{4 * i:4d}  " + " ".join(cells) + f" {prev - r[0]:11d}  moved {r[10]} depth {r[11]} D {r[12]}")
    eng.close()


if __name__ == "__main__":
    main()
