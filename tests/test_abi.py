"""The C-ABI library loads and exports every symbol include/mz.h declares (no
compute calls: runs without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "mz.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(mz_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    names = _declared()
    for n in ("mz_engine_create", "mz_mcts_search", "mz_mcts_search_dev", "mz_net_forward",
              "mz_learner_step", "mz_learner_grad_dev", "mz_learner_apply_dev", "mz_weights_set"):
        assert n in names


def test_libmz_exports_every_declared_symbol():
    import _mzpkg
    pkg = _mzpkg.load()
    if not os.path.exists(pkg.LIB_PATH):
        from muzero_jl_amd import build
        build.build()
    lib = ctypes.CDLL(pkg.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    from muzero_jl_amd import abi
    for n in abi.SIGNATURES:
        assert n in _declared(), f"abi.py binds {n} which mz.h does not declare"


def test_engine_fails_loudly_without_gpu(ttt):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from muzero_jl_amd.abi import Engine, MzError
    with pytest.raises(MzError):
        Engine(ttt.conf, ttt.hyper, device=0, max_games=4)


def test_create_validates_config(ttt):
    import dataclasses
    from muzero_jl_amd.abi import Engine, MzError
    bad = dataclasses.replace(ttt.hyper, hidden_state_size=20)
    with pytest.raises(MzError, match="hidden_state_size|GPU"):
        Engine(ttt.conf, bad, device=0, max_games=4)
