"""Diagnostic (stamp build, MZ_LIB=libmz_stamps.so): per-layer ticks of the
configs[4] downsampler for item 0 of a 32-item mz_net_forward(representation)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _mzpkg  # noqa: E402

_mzpkg.load()
from muzero_jl_amd import abi  # noqa: E402
from muzero_jl_amd.games import atari_synth as at  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
e = abi.Engine(at.conf, at.resnet_hyper, device=0, max_games=max(n, 64), rng_seed=1)
for k, w in enumerate(init_nets(at.conf, at.resnet_hyper, seed=3)):
    e.set_weights(k, w)
x = at.observations(n, seed=1)
for _ in range(3):
    e.forward(0, x)
out = np.zeros(8 * 8, np.uint64)
e.sync()
rc = e.lib.mz_debug_stamps(e.h, out.ctypes.data_as(abi._VP), 8)
assert rc == 0, e.lib.mz_last_error(e.h)
nl = 20
t = out[:nl + 1].astype(np.int64)
start = t[nl]
prev = start
for i in range(nl):
    print(f"layer {i:2d}: {int(t[i] - prev):7d} ticks")
    prev = t[i]
print("total", int(t[nl - 1] - start), "ticks")
