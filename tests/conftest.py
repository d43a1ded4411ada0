import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import _mzpkg  # noqa: E402

_mzpkg.load()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libmz.so")


@pytest.fixture(scope="session")
def ttt():
    from muzero_jl_amd.games import tictactoe
    return tictactoe


@pytest.fixture(scope="session")
def nets(ttt):
    from muzero_jl_amd.networks import init_nets
    return init_nets(ttt.conf, ttt.hyper, seed=11)


def random_positions(G, seed=0, A=9, feat=63, p_legal=0.6):
    rng = np.random.default_rng(seed)
    obs = (rng.random((G, feat)) < 0.35).astype(np.float32)
    obs[:, 27:36] = rng.integers(0, 10, (G, 1)).astype(np.float32)   # action plane (raw id, Q15)
    legal = rng.random((G, A)) < p_legal
    legal[np.arange(G), rng.integers(0, A, G)] = True
    tp = rng.integers(1, 3, G).astype(np.int32)
    return obs, legal, tp
