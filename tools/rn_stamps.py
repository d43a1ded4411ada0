"""Diagnostic: per-layer ticks (s_memtime) of the ResNet network kernel, from
a separate -DMZ_STAMPS build (libmz_stamps.so): for nets workgroups (0, pred)
and (0, dyn) of simulation 0, per wave, the compute span of each layer (or
run of 1x1 layers) and the wait at its barrier.  Shares only."""
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


def main():
    lib = os.path.join(pkg.PKG_DIR, "lib", "libmz_stamps.so")
    srcs = [os.path.join(pkg.PKG_DIR, "csrc", s) for s in mzbuild.SOURCES]
    if "--no-build" not in sys.argv:
        subprocess.run(["/opt/rocm/bin/hipcc"] + mzbuild.FLAGS + ["-DMZ_STAMPS", "-shared", "-o", lib] + srcs, check=True)
    if "--build-only" in sys.argv:
        return
    abi._lib = None
    L = abi.load_library(lib)
    L.mz_debug_stamps.restype = ctypes.c_int
    L.mz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    G = int(os.environ.get("G", "2048"))
    conf = dataclasses.replace(ttt.conf, num_iters=4)
    eng = abi.Engine(conf, ttt.resnet_hyper, device=0, max_games=G, rng_seed=1)
    for n, w in enumerate(init_nets(conf, ttt.resnet_hyper, seed=1234)):
        eng.set_weights(n, w)
    obs, legal, tp = random_positions(ttt.BatchedTicTacToe, G, seed=100)
    for k in range(2):
        eng.mcts_search(obs, legal, tp, rng_step=k)
    out = np.zeros(256 * 8, np.uint64)
    assert L.mz_debug_stamps(eng.h, out.ctypes.data_as(ctypes.c_void_p), 256) == 0
    for y, name in ((0, "pred"), (1, "dyn")):
        st = out[y * 1024:y * 1024 + 768].reshape(12, 64).astype(np.int64)
        t0 = st[:, 63].min()
        print(f"== {name}: per layer [compute end - previous barrier exit | barrier wait] ticks, waves 0..11")
        prev = st[:, 63].copy()
        for i in range(31):
            if not st[:, 2 * i].any():
                continue
            comp = st[:, 2 * i] - prev
            wait = st[:, 2 * i + 1] - st[:, 2 * i]
            prev = st[:, 2 * i + 1].copy()
            print(f"  layer {i:2d}: " + " ".join(f"{c:6d}|{w:<6d}" for c, w in zip(comp, wait)))
            d = out[y * 1024 + 768 + 8 * i: y * 1024 + 768 + 8 * i + 4].astype(np.int64)
            if d.all():
                print(f"      wave 0 unit 0: operands {d[1] - d[0]}  chunks {d[2] - d[1]}  epilogue {d[3] - d[2]}")
        last = max(2 * i + 1 for i in range(31) if st[:, 2 * i].any())
        k0 = st[:, 60].min()
        print(f"  staging {t0 - k0}  layers {st[:, last].max() - t0}  outputs {st[:, 61].max() - st[:, last].max()}"
              f"  kernel (start -> outputs staged) {st[:, 61].max() - k0} ticks")
    eng.close()


if __name__ == "__main__":
    main()
