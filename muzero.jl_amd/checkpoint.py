"""Checkpoints — Python side of mz_checkpoint_save / _load.

The reference writes each net with Julia's `serialize` to
"$(step)_<net>.bin" (src/Learning.jl:424-431) and reads it back with
`deserialize` (games/tictactoe/play.jl:12-14); that format is unreadable
outside Julia.  A libmz checkpoint is one safetensors file (layout in
muzero.jl_amd/csrc/mz_checkpoint.cpp): tensor "<net>.<i>" is the i-th array of
Flux.params(<net>) with the Julia array's column-major bytes and the Julia
shape reversed, so `arr.transpose()` of the numpy array is the Julia array
(and `permutedims(arr, reverse(1:ndims(arr)))` in Julia undoes SafeTensors.jl's
row-major view); plus "adam.m", "adam.v", "adam.beta_pow" and metadata.

Loading uses safetensors' numpy loader only (no pickle, nothing executed).
"""
import json

import numpy as np

from .config import ResNetHP
from .networks import layer_specs, param_count, resnet_specs

NETS = ("representation", "prediction", "dynamics")
FORMAT = "libmz-checkpoint-1"


def param_table(conf, hyper, net):
    """[(name, julia_shape, offset in the net's flat vector)] in Flux.params order
    (mz_param_table in the engine)."""
    out, off, i = [], 0, 0

    def add(shape):
        nonlocal off, i
        out.append((f"{NETS[net]}.{i}", tuple(shape), off))
        off += int(np.prod(shape))
        i += 1

    if isinstance(hyper, ResNetHP):
        for op in resnet_specs(conf, hyper, net):
            if op["kind"] == "pool":                      # MeanPool: no params
                continue
            if op["kind"] == "conv":
                add((op["kw"], op["kh"], op["cin"], op["cout"]))
                add((op["cout"],))
                if op["bn"]:
                    add((op["cout"],))                    # BatchNorm β
                    add((op["cout"],))                    # BatchNorm γ
            else:
                add((op["cout"], op["cin"]))
                add((op["cout"],))
    else:
        for _, fin, fout, _, bn in layer_specs(conf, hyper, net, True):
            add((fout, fin))
            add((fout,))
            if bn:                                        # make_dense's BatchNorm: β, γ
                add((fout,))
                add((fout,))
    assert off == param_count(conf, hyper, net)
    return out


def flux_arrays(conf, hyper, net, flat):
    """The net's Flux.params arrays (Julia shapes, column-major order) from its flat vector."""
    flat = np.asarray(flat, np.float32)
    return [flat[o:o + int(np.prod(s))].reshape(s, order="F") for _, s, o in param_table(conf, hyper, net)]


def write(path, conf, hyper, nets, training_step=0, adam=None):
    """Write a checkpoint from host arrays: nets = three flat vectors; adam =
    (m, v, beta_pow) over the nets back to back, or None for a fresh optimiser."""
    from safetensors.numpy import save_file
    tensors = {}
    for net in range(3):
        flat = np.asarray(nets[net], np.float32)
        for name, shape, off in param_table(conf, hyper, net):
            n = int(np.prod(shape))
            tensors[name] = np.ascontiguousarray(flat[off:off + n].reshape(shape[::-1]))
    n = sum(param_count(conf, hyper, k) for k in range(3))
    m, v, bp = adam if adam is not None else (np.zeros(n, np.float32), np.zeros(n, np.float32),
                                             np.array([0.9, 0.999]))
    tensors["adam.m"] = np.asarray(m, np.float32)
    tensors["adam.v"] = np.asarray(v, np.float32)
    tensors["adam.beta_pow"] = np.asarray(bp, np.float64)
    kind = "resnet" if isinstance(hyper, ResNetHP) else "fc"
    save_file(tensors, path, metadata={"format": FORMAT, "network": kind, "training_step": str(int(training_step)),
                                       "config": json.dumps({"observation_shape": list(conf.observation_shape),
                                                             "action_space_size": len(conf.action_space)})})


def read(path):
    """(tensors dict of numpy arrays, metadata dict) — safetensors' numpy loader."""
    from safetensors import safe_open
    with safe_open(path, framework="numpy") as f:
        meta = f.metadata() or {}
        tensors = {k: f.get_tensor(k) for k in f.keys()}
    return tensors, meta


def nets_from(tensors, conf, hyper):
    """The three flat parameter vectors (engine / mz_weights_set order) of a checkpoint."""
    out = []
    for net in range(3):
        parts = []
        for name, shape, _ in param_table(conf, hyper, net):
            a = tensors[name]
            if tuple(a.shape) != tuple(shape[::-1]):
                raise ValueError(f"{name}: shape {a.shape}, expected {shape[::-1]}")
            parts.append(np.ascontiguousarray(a, np.float32).ravel())
        out.append(np.concatenate(parts))
    return out
