"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference (Julia) cannot run in this image, so these vectors
pin the oracle's restatement against regressions and feed the GPU parity
tests; they are inputs + expected outputs only.  Run: python tests/golden/make_golden.py
"""
import dataclasses
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import _mzpkg  # noqa: E402

_mzpkg.load()
from muzero_jl_amd.config import to_c_config, to_c_ffhp  # noqa: E402
from muzero_jl_amd.games import tictactoe as ttt  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402
from oracle import Oracle  # noqa: E402
from conftest import random_positions  # noqa: E402


def main():
    nets = init_nets(ttt.conf, ttt.hyper, seed=2024)
    # weights are regenerated from the seed (numpy PCG64 is stable); keep a checksum
    out = {"weights_sum": np.array([float(np.sum(w.astype(np.float64))) for w in nets])}
    rng = np.random.default_rng(2024)
    base = Oracle(to_c_config(ttt.conf), to_c_ffhp(ttt.hyper), seed=42)
    for n, w in enumerate(nets):
        base.set_weights(n, w)
    for net, feat in [(0, 63), (1, 27), (2, 36)]:
        x = rng.standard_normal((8, feat)).astype(np.float32)
        out[f"fwd{net}_x"] = x
        r = base.forward(net, x)
        out[f"fwd{net}_y0"], out[f"fwd{net}_y1"] = (r, np.zeros(0, np.float32)) if net == 0 else r
    for S in (10, 25):
        conf = dataclasses.replace(ttt.conf, num_iters=S)
        o = Oracle(to_c_config(conf), to_c_ffhp(ttt.hyper), seed=42)
        for n, w in enumerate(nets):
            o.set_weights(n, w)
        obs, legal, tp = random_positions(16, 100 + S)
        cv, rv, act = o.mcts_search(obs, legal, tp, exploration=True, rng_step=S, game_offset=3)
        out.update({f"s{S}_obs": obs, f"s{S}_legal": legal.astype(np.uint8), f"s{S}_tp": tp,
                    f"s{S}_cv": cv, f"s{S}_rv": rv, f"s{S}_act": act})
    g = base.play_game(game_id=5, step0=11)
    for k, v in g.items():
        out[f"game_{k}"] = v
    np.savez_compressed(os.path.join(HERE, "oracle_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "oracle_golden.npz"))


if __name__ == "__main__":
    main()
