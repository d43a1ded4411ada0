"""Diagnostic: timeline of one mz_runroll_fused_r launch (ResNet learner, B = 32)
from the -DMZ_STAMPS build (libmz_stamps.so, built on the CPU host by
tools/build_all.sh): per block s_memrealtime (100 MHz) at start, at its input's
publish (items) / the chain's last publish (chain blocks), and at the end.
usage: python tools/rn_fused_stamps.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import _mzpkg  # noqa: E402

pkg = _mzpkg.load()
from muzero_jl_amd import abi  # noqa: E402
from muzero_jl_amd.games import tictactoe as ttt  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402


def main():
    L = abi.load_library(os.path.join(pkg.PKG_DIR, "lib", "libmz_stamps.so"))
    L.mz_debug_stamps.restype = ctypes.c_int
    L.mz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    conf, hyper = ttt.conf, ttt.resnet_hyper
    eng = abi.Engine(conf, hyper, device=0, max_games=512, rng_seed=1)
    for n, w in enumerate(init_nets(conf, hyper, seed=1234)):
        eng.set_weights(n, w)
    B, K, A = conf.batch_size, conf.num_unroll_steps, len(conf.action_space)
    rng = np.random.default_rng(0)
    obs = (rng.random((B, 3 * 3 * 7)) < 0.3).astype(np.float32)
    tpol = rng.random((B, K + 1, A)).astype(np.float32)
    batch = dict(observation=obs, actions=rng.integers(1, A + 1, (B, K + 1)).astype(np.float32),
                 target_values=rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
                 target_rewards=np.zeros((B, K + 1), np.float32),
                 target_policies=tpol / tpol.sum(-1, keepdims=True),
                 gradient_scale=rng.integers(1, K + 1, B).astype(np.float32))
    for _ in range(4):
        eng.learner_step(batch, 1e-4)
    print("variant", eng.learner_variant() if hasattr(eng, "learner_variant") else "?")
    out = np.zeros(512 * 8, np.uint64)
    assert L.mz_debug_stamps(eng.h, out.ctypes.data_as(ctypes.c_void_p), 512) == 0
    n_l2 = int(os.environ.get("N_L2", "0"))
    nb = B + n_l2 + 3 * B * K
    st = out[2048:2048 + 4 * nb].reshape(nb, 4).astype(np.int64)
    t0 = st[:, 0].min()
    us = lambda x: (x - t0) / 100.0          # 100 MHz ticks -> us
    ch = st[:B]
    print(f"chain: start {us(ch[:, 0]).min():.1f}-{us(ch[:, 0]).max():.1f}  last publish max {us(ch[:, 1]).max():.1f}"
          f"  end max {us(ch[:, 2]).max():.1f} us")
    it = st[B + n_l2:]
    for s in range(K):
        for rw in (0, 1, 2):
            g = it[(s * 3 + rw) * B:(s * 3 + rw + 1) * B]
            print(f"step {s} {('value ', 'policy', 'reward')[rw]}: start {us(g[:, 0]).min():6.1f}-{us(g[:, 0]).max():6.1f}"
                  f"  input {us(g[:, 1]).min():6.1f}-{us(g[:, 1]).max():6.1f}  end {us(g[:, 2]).min():6.1f}-"
                  f"{us(g[:, 2]).max():6.1f}  run {np.mean(g[:, 2] - g[:, 1]) / 100:5.1f} us")
    eng.close()


if __name__ == "__main__":
    main()
