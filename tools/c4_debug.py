"""Diagnostic: Connect4 ResNet search at the bench size; games whose chosen
action is illegal are re-run alone through the oracle (same game id)."""
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import _mzpkg  # noqa: E402

_mzpkg.load()
from muzero_jl_amd import abi  # noqa: E402
from muzero_jl_amd.config import to_c_config, to_c_resnet_hp  # noqa: E402
from muzero_jl_amd.games import connect4  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402
from muzero_jl_amd.selfplay import random_positions  # noqa: E402
from oracle import Oracle  # noqa: E402

G, S = int(os.environ.get("G", "512")), int(os.environ.get("S", "50"))
conf = dataclasses.replace(connect4.conf, num_iters=S)
hyper = connect4.resnet_hyper
nets = init_nets(conf, hyper, seed=1234)
eng = abi.Engine(conf, hyper, device=0, max_games=G, rng_seed=1)
for n, w in enumerate(nets):
    eng.set_weights(n, w)
obs, legal, tp = random_positions(connect4.BatchedConnect4, G, seed=100, max_plies=16)
eng.debug_enable(1)
for step in range(int(os.environ.get("STEPS", "13"))):
    cv, rv, act = eng.mcts_search(obs, legal, tp, exploration=True, rng_step=step, game_offset=0, temperature=1.0)
    bad = np.flatnonzero(~legal[np.arange(G), act - 1])
    print("step", step, "illegal games:", bad[:20], "count", len(bad))
    if len(bad):
        break
tree = eng.debug_tree(G)
for g in bad[:3]:
    print("game", g, "legal", legal[g].astype(int), "act", act[g], "cv", np.round(cv[g], 3))
    print("  root N", tree["N"][g, 0], "root P", np.round(tree["P"][g, 0], 3))
    o = Oracle(to_c_config(conf), to_c_resnet_hp(hyper), seed=1)
    for n, w in enumerate(nets):
        o.set_weights(n, w)
    cv2, rv2, act2, _, _ = o.mcts_search(obs[g:g + 1], legal[g:g + 1], tp[g:g + 1], exploration=True, rng_step=step,
                                         game_offset=g, temperature=1.0, dump=True)
    print("  oracle act", act2, "cv", np.round(cv2[0], 3), "rv", rv2, "gpu rv", rv[g])
