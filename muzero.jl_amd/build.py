"""Build libmz.so (hand-written HIP for gfx950) in-tree with hipcc.

Each source compiles to its own object in parallel (a source is rebuilt when
it, or any header, is newer than its object); the objects link into
muzero.jl_amd/lib/libmz.so."""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

from . import PKG_DIR, LIB_PATH

SOURCES = ["mz_engine.hip", "mz_search.hip", "mz_small.hip", "mz_nets.hip", "mz_resnet.hip", "mz_selfplay.hip",
           "mz_downsample.hip", "mz_checkpoint.cpp", "mz_backprop.hip"]
HEADERS = ["mz_internal.h", "mz_mlp_device.h", "mz_tree_device.h", "mz_small_params.h", "mz_resnet_params.h",
           "mz_selfplay_params.h", "mz_ckpt_iface.h", "mz_replay_device.h", "mz_learner_device.h",
           "mz_backprop_params.h", "mz_st_header.h"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
         # the numerics contract (include/mz_detmath.h): no FP contraction, IEEE
         # division/sqrt, f32 denormals kept (hipcc defaults for the last two)
         "-ffp-contract=off", "-fno-fast-math", "-Wno-unused-result",
         # the SLP vectorizer packs the small kernel's per-game fmaf chains into
         # v_pk_fma_f32 with each resident weight duplicated into a register
         # pair (2x the weight registers -> spills); scalar fmaf keeps 1x
         "-fno-slp-vectorize"]


def build(force=False, verbose=False, jobs=None, out=None, objdir=None, extra=()):
    """out / objdir / extra: a variant library (A/B experiments, tools/ab_default.sh)."""
    csrc = os.path.join(PKG_DIR, "csrc")
    inc = os.path.join(os.path.dirname(PKG_DIR), "include")
    lib_path = out or LIB_PATH
    objdir = objdir or os.path.join(os.path.dirname(LIB_PATH), "obj")
    srcs = [os.path.join(csrc, s) for s in SOURCES]
    hdrs = [os.path.join(csrc, h) for h in HEADERS] + [os.path.join(inc, f) for f in ("mz.h", "mz_detmath.h")]
    missing = [f for f in srcs + hdrs if not os.path.exists(f)]
    if missing:                      # a dropped source would link into a library with undefined symbols
        raise FileNotFoundError(f"libmz sources missing: {missing}")
    hdr_t = max(os.path.getmtime(d) for d in hdrs)
    os.makedirs(objdir, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or not os.path.exists(o) or os.path.getmtime(o) < max(hdr_t, os.path.getmtime(s)):
            todo.append((s, o))

    def compile_one(so):
        s, o = so
        cmd = [hipcc] + FLAGS + list(extra) + ["-c", "-o", o + ".tmp", s]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(o + ".tmp", o)

    if todo:
        with ThreadPoolExecutor(jobs or min(len(todo), os.cpu_count() or 4, 16)) as ex:
            list(ex.map(compile_one, todo))
    if todo or not os.path.exists(lib_path) or os.path.getmtime(lib_path) < max(os.path.getmtime(o) for o in objs):
        cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-Wl,--no-undefined", "-o", lib_path + ".tmp"] + \
            objs + ["-ldl"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(lib_path + ".tmp", lib_path)
    return lib_path
