"""Diagnostic: per-layer ticks (s_memtime) of the ResNet learner chain kernel
(mz_runroll_chain), from a separate -DMZ_STAMPS build (libmz_stamps.so): for
chain workgroup 0, per wave, the compute span of each layer of the
representation and of the first dynamics step, and the wait at its barrier.
usage: python tools/rn_chain_stamps.py [--no-build] [--game atari]"""
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


def show(st, name, dbg=None):
    st = st.reshape(8, 64).astype(np.int64)
    st = st[st[:, 63] != 0]                # waves that ran (mz_runroll_chain_r has 4)
    t0 = st[:, 63].min()
    print(f"== {name}: per layer [compute end - previous barrier exit | barrier wait] ticks, waves 0..{len(st) - 1}")
    prev = st[:, 63].copy()
    tot_c = tot_w = 0
    for i in range(31):
        if not st[:, 2 * i].any():
            continue
        comp = st[:, 2 * i] - prev
        wait = st[:, 2 * i + 1] - st[:, 2 * i]
        prev = st[:, 2 * i + 1].copy()
        tot_c += comp.max()
        tot_w += (st[:, 2 * i + 1].max() - st[:, 2 * i].max())
        print(f"  layer {i:2d}: " + " ".join(f"{c:6d}|{w:<6d}" for c, w in zip(comp, wait)))
        if dbg is not None and dbg[i, 0]:
            d = dbg[i].astype(np.int64)
            bx = st[0, 2 * i - 1] if i > 0 else st[0, 63]
            print(f"      wave 0 unit 0: entry {d[0] - bx}  operands {d[1] - d[0]}  chunks {d[2] - d[1]}"
                  f"  epilogue {d[3] - d[2]}  -> layer end {st[0, 2 * i] - d[3]}")
    last = max(2 * i + 1 for i in range(31) if st[:, 2 * i].any())
    print(f"  total {st[:, last].max() - t0} ticks")


def main():
    lib = os.path.join(pkg.PKG_DIR, "lib", "libmz_stamps.so")
    srcs = [os.path.join(pkg.PKG_DIR, "csrc", s) for s in mzbuild.SOURCES]
    if "--no-build" not in sys.argv:
        subprocess.run(["/opt/rocm/bin/hipcc"] + mzbuild.FLAGS + ["-DMZ_STAMPS", "-shared", "-o", lib] + srcs,
                       check=True)
    if "--build-only" in sys.argv:
        return
    abi._lib = None
    L = abi.load_library(lib)
    L.mz_debug_stamps.restype = ctypes.c_int
    L.mz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    conf = ttt.conf
    hyper = ttt.resnet_hyper
    eng = abi.Engine(conf, hyper, device=0, max_games=512, rng_seed=1)
    for n, w in enumerate(init_nets(conf, hyper, seed=1234)):
        eng.set_weights(n, w)
    B, K, A = conf.batch_size, conf.num_unroll_steps, len(conf.action_space)
    rng = np.random.default_rng(0)
    obs = (rng.random((B, 3 * 3 * 7)) < 0.3).astype(np.float32)     # (3, 3, 7) stacked planes
    tpol = rng.random((B, K + 1, A)).astype(np.float32)
    batch = dict(observation=obs, actions=rng.integers(1, A + 1, (B, K + 1)).astype(np.float32),
                 target_values=rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
                 target_rewards=np.zeros((B, K + 1), np.float32),
                 target_policies=tpol / tpol.sum(-1, keepdims=True),
                 gradient_scale=rng.integers(1, K + 1, B).astype(np.float32))
    for k in range(3):
        eng.learner_step(batch, 1e-4)
    out = np.zeros(512 * 8, np.uint64)
    assert L.mz_debug_stamps(eng.h, out.ctypes.data_as(ctypes.c_void_p), 512) == 0
    show(out[:512], "representation", out[1024:1024 + 31 * 8].reshape(31, 8))
    show(out[512:1024], "dynamics (step 1)", out[1536:1536 + 31 * 8].reshape(31, 8))
    eng.close()


if __name__ == "__main__":
    main()
