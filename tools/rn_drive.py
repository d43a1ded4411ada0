"""Drive the ResNet search (configs[2] shape) for profiling: N searches of G
games x S sims on device buffers; prints the network kernel's mean time from
the engine's HIP events.  Used under rocprofv3 (kernel trace / PMC passes)."""
import argparse
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _mzpkg  # noqa: E402

_mzpkg.load()
from muzero_jl_amd.abi import Engine  # noqa: E402
from muzero_jl_amd.games import tictactoe as ttt  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402
from muzero_jl_amd.selfplay import random_positions  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=2048)
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--n", type=int, default=3)
    ap.add_argument("--warm", type=int, default=4, help="untimed searches first (clocks settle)")
    ap.add_argument("--lib", default=None, help="a libmz variant to load instead of the default")
    args = ap.parse_args()
    if args.lib:
        from muzero_jl_amd import abi
        abi._lib = None
        abi.load_library(args.lib)
    conf = dataclasses.replace(ttt.conf, num_iters=args.sims)
    G = args.games
    eng = Engine(conf, ttt.resnet_hyper, device=0, max_games=G, rng_seed=1)
    for n, w in enumerate(init_nets(conf, ttt.resnet_hyper, seed=1234)):
        eng.set_weights(n, w)
    obs, legal, tp = random_positions(ttt.BatchedTicTacToe, G, seed=100)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (obs, legal.astype(np.uint8), tp.astype(np.int32))]
    cv = torch.empty((G, 9), dtype=torch.float32, device=dev)
    rv = torch.empty(G, dtype=torch.float32, device=dev)
    act = torch.empty(G, dtype=torch.int32, device=dev)
    for k in range(args.warm):
        eng.mcts_search_dev(G, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), cv.data_ptr(), rv.data_ptr(),
                            act.data_ptr(), exploration=True, rng_step=100 + k, game_offset=0, temperature=1.0)
    eng.debug_enable(2)
    for k in range(args.n):
        eng.mcts_search_dev(G, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), cv.data_ptr(), rv.data_ptr(),
                            act.data_ptr(), exploration=True, rng_step=k, game_offset=0, temperature=1.0)
    eng.sync()
    t, n = eng.debug_kernel_time()
    print(f"nets kernel {t / n * 1e3:.1f} us over {n} launches")
    eng.close()


if __name__ == "__main__":
    main()
