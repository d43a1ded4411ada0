"""Build libmz.so (hand-written HIP for gfx950) in-tree with hipcc."""
import os
import subprocess

from . import PKG_DIR, LIB_PATH

SOURCES = ["mz_engine.hip", "mz_search.hip", "mz_small.hip", "mz_nets.hip", "mz_resnet.hip", "mz_selfplay.hip",
           "mz_downsample.hip", "mz_checkpoint.cpp"]
HEADERS = ["mz_internal.h", "mz_mlp_device.h", "mz_tree_device.h", "mz_small_params.h", "mz_resnet_params.h",
           "mz_selfplay_params.h", "mz_ckpt_iface.h", "mz_replay_device.h", "mz_learner_device.h"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
         # the numerics contract (include/mz_detmath.h): no FP contraction, IEEE
         # division/sqrt, f32 denormals kept (hipcc defaults for the last two)
         "-ffp-contract=off", "-fno-fast-math", "-Wno-unused-result",
         # the SLP vectorizer packs the small kernel's per-game fmaf chains into
         # v_pk_fma_f32 with each resident weight duplicated into a register
         # pair (2x the weight registers -> spills); scalar fmaf keeps 1x
         "-fno-slp-vectorize"]


def build(force=False, verbose=False):
    csrc = os.path.join(PKG_DIR, "csrc")
    inc = os.path.join(os.path.dirname(PKG_DIR), "include")
    srcs = [os.path.join(csrc, s) for s in SOURCES]
    deps = srcs + [os.path.join(csrc, h) for h in HEADERS] + \
        [os.path.join(inc, f) for f in ("mz.h", "mz_detmath.h")]
    if not force and os.path.exists(LIB_PATH):
        t = os.path.getmtime(LIB_PATH)
        if all(os.path.getmtime(d) <= t for d in deps):
            return LIB_PATH
    os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc] + FLAGS + ["-o", LIB_PATH + ".tmp"] + srcs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH
