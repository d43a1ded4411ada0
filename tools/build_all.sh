#!/bin/bash
# Build libmz.so and the -DMZ_STAMPS diagnostic variant (tools/stamps.py) in-tree, incrementally.
cd "$(dirname "$0")/.." && python - <<'PY'
import os, sys
sys.path.insert(0, os.getcwd())
import _mzpkg
pkg = _mzpkg.load()
from muzero_jl_amd import build as b
b.build()
lib = os.path.join(pkg.PKG_DIR, "lib")
b.build(out=os.path.join(lib, "libmz_stamps.so"), objdir=os.path.join(lib, "obj_stamps"), extra=["-DMZ_STAMPS"])
print("built")
PY
