"""Diagnostic: level-end cycles (s_memtime) of tile 0 of the corrected FC
learner's mz_bp_tile_lv (NET=fc, default: TicTacToe FC at batch_size 32,
K = 5, the default bench's corrected leg), or application-end cycles of sample
0 of the ResNet corrected learner's mz_rbp_sample (NET=resnet, GAME=ttt or
connect4), from the -DMZ_STAMPS build (libmz_stamps.so, built by
tools/tree_stamps.py)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import _mzpkg  # noqa: E402

pkg = _mzpkg.load()
from muzero_jl_amd import abi  # noqa: E402
from muzero_jl_amd.networks import init_nets  # noqa: E402
from muzero_jl_amd.games import tictactoe, connect4  # noqa: E402


def main():
    import torch
    abi._lib = None
    L = abi.load_library(os.path.join(pkg.PKG_DIR, "lib", "libmz_stamps.so"))
    L.mz_debug_stamps.restype = ctypes.c_int
    L.mz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    resnet = os.environ.get("NET", "fc") == "resnet"
    gm = connect4 if os.environ.get("GAME", "ttt") == "connect4" else tictactoe
    conf, hyper = gm.conf, (gm.resnet_hyper if resnet else gm.hyper)
    B, K = conf.batch_size, conf.num_unroll_steps
    eng = abi.Engine(conf, hyper, device=0, max_games=8, rng_seed=1)
    A, feat = len(conf.action_space), eng.obs_feat
    for n, w in enumerate(init_nets(conf, hyper, seed=1)):
        eng.set_weights(n, w)
    eng.learner_set_mode(abi.LEARN_CORRECTED)
    rng = np.random.default_rng(0)
    tpol = rng.random((B, K + 1, A)).astype(np.float32)
    arrs = [(rng.random((B, feat)) < 0.4).astype(np.float32), rng.integers(1, A + 1, (B, K + 1)).astype(np.float32),
            rng.uniform(-1, 1, (B, K + 1)).astype(np.float32), rng.uniform(-1, 1, (B, K + 1)).astype(np.float32),
            tpol / tpol.sum(-1, keepdims=True), np.ones(B, np.float32)]
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs] + [None]
    grad = torch.zeros(eng.grad_count(), dtype=torch.float32, device="cuda")
    losses = torch.zeros(8, dtype=torch.float32, device="cuda")
    for _ in range(3):
        eng.learner_grad_dev([t.data_ptr() if t is not None else None for t in dev], B, grad.data_ptr(),
                             losses.data_ptr())
    eng.sync()
    out = np.zeros(1024, np.uint64)
    assert L.mz_debug_stamps(eng.h, out.ctypes.data_as(ctypes.c_void_p), 128) == 0
    st = out.astype(np.int64)
    if resnet:
        assert st[0] > 0, "no stamps: the ResNet corrected learner did not run"
        n = int(np.argmax(st[1:] == 0))           # forward ends + heads, then backward
        na = (n - 1) // 2 if n > 2 else 0
        fw, hd, bw = st[1:1 + na], st[1 + na], st[2 + na:2 + 2 * na]
        print(f"apps {na}: forward {fw[-1] - st[0]} cycles, heads {hd - fw[-1]}, backward {bw[0] - hd} "
              f"(reverse order: last app first)")
        d = np.diff(np.concatenate([[st[0]], fw]))
        print("forward per app:", " ".join(map(str, d)))
        d = np.diff(np.concatenate([[hd], bw[::-1]]))
        print("backward per app (in backward order):", " ".join(map(str, d)))
        eng.close()
        return
    t0 = st[0]
    fw = [st[2 + i] for i in range(254) if st[2 + i] > 0]
    bw = [st[256 + i] for i in range(512) if st[256 + i] > 0]
    print(f"forward levels {len(fw)}: {fw[-1] - t0} cycles; heads {st[1] - fw[-1]}; backward levels {len(bw)}: "
          f"{bw[-1] - st[1]} cycles")
    prev = t0
    print("forward per level:", " ".join(str(x - p) for p, x in zip([t0] + fw[:-1], fw)))
    print("backward per level:", " ".join(str(x - p) for p, x in zip([st[1]] + bw[:-1], bw)))
    eng.close()


if __name__ == "__main__":
    main()
