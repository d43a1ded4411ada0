"""Diagnostic: the bench's Connect4 ResNet search sequence (device buffers on a
torch stream, steps 0..6, then 7..9 with the network-launch events), legality
checked after every search."""
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import _mzpkg  # noqa: E402

_mzpkg.load()
from muzero_jl_amd import abi  # noqa: E402
from muzero_jl_amd.games import connect4  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402
from muzero_jl_amd.selfplay import random_positions  # noqa: E402

G, S = 512, 50
conf = dataclasses.replace(connect4.conf, num_iters=S)
hyper = connect4.resnet_hyper
dev = torch.device("cuda", 0)
stream = torch.cuda.Stream(device=dev)
torch.cuda.set_stream(stream)
sp = stream.cuda_stream if os.environ.get("OWN_STREAM") is None else None
eng = abi.Engine(conf, hyper, device=0, max_games=G, rng_seed=1)
for n, w in enumerate(init_nets(conf, hyper, seed=1234)):
    eng.set_weights(n, w)
obs, legal, tp = random_positions(connect4.BatchedConnect4, G, seed=100, max_plies=16)
d = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (obs, legal.astype(np.uint8), tp.astype(np.int32))]
cv = torch.empty((G, 7), dtype=torch.float32, device=dev)
rv = torch.empty(G, dtype=torch.float32, device=dev)
act = torch.empty(G, dtype=torch.int32, device=dev)
for k in range(10):
    if k == 7 and os.environ.get("NO_EVENTS") is None:
        eng.debug_enable(2)
    eng.mcts_search_dev(G, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), cv.data_ptr(), rv.data_ptr(),
                        act.data_ptr(), exploration=True, rng_step=k, game_offset=0, temperature=1.0, stream=sp)
    torch.cuda.synchronize()
    a = act.cpu().numpy()
    bad = np.flatnonzero(~legal[np.arange(G), a - 1])
    c = cv.cpu().numpy()
    print("step", k, "illegal", bad[:8], "cv rows summing to 0:", int((np.abs(c.sum(1) - 1) > 1e-3).sum()),
          "nan rv:", int(np.isnan(rv.cpu().numpy()).sum()))

# same step through the host-buffer API, and the oracle on the offending game
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from muzero_jl_amd.config import to_c_config, to_c_resnet_hp  # noqa: E402
from oracle import Oracle  # noqa: E402
k = 0
eng.mcts_search_dev(G, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), cv.data_ptr(), rv.data_ptr(),
                    act.data_ptr(), exploration=True, rng_step=k, game_offset=0, temperature=1.0, stream=sp)
torch.cuda.synchronize()
a_dev, c_dev = act.cpu().numpy(), cv.cpu().numpy()
c_h, r_h, a_h = eng.mcts_search(obs, legal, tp, exploration=True, rng_step=k, game_offset=0, temperature=1.0)
diff = np.flatnonzero((a_h != a_dev) | np.any(c_h != c_dev, axis=1))
print("host vs dev differing games:", diff[:10], len(diff))
for g in np.flatnonzero(~legal[np.arange(G), a_dev - 1])[:2]:
    print("game", g, "legal", legal[g].astype(int), "tp", tp[g], "dev act", a_dev[g], "cv", np.round(c_dev[g], 3))
    print("   host act", a_h[g], "cv", np.round(c_h[g], 3))
    print("   obs cur empty plane", obs[g, 84:126].astype(int))
    o = Oracle(to_c_config(conf), to_c_resnet_hp(hyper), seed=1)
    for n, w in enumerate(init_nets(conf, hyper, seed=1234)):
        o.set_weights(n, w)
    c2, r2, a2, _, _ = o.mcts_search(obs[g:g + 1], legal[g:g + 1], tp[g:g + 1], exploration=True, rng_step=k,
                                     game_offset=g, temperature=1.0, dump=True)
    print("   oracle act", a2, "cv", np.round(c2[0], 3))
