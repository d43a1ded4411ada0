#!/bin/bash
# A/B of compile-time variants of the ResNet layer code: builds
# lib/libmz_ab_<i>.so per "-D..." set in $VARIANTS (';'-separated) and times
# the network kernel of each with tools/rn_drive.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
i=0
IFS=';' read -ra VS <<< "${VARIANTS:-}"
for v in "" "${VS[@]}"; do
  lib="$R/muzero.jl_amd/lib/libmz_ab_$i.so"
  if [ ! -f "$lib" ]; then
    python - "$lib" $v <<'PY' || exit 1
import subprocess, sys, os
sys.path.insert(0, os.getcwd())
import _mzpkg; _mzpkg.load()
from muzero_jl_amd import build as b
srcs = [os.path.join(os.getcwd(), "muzero.jl_amd", "csrc", s) for s in b.SOURCES]
subprocess.run(["/opt/rocm/bin/hipcc"] + b.FLAGS + sys.argv[2:] + ["-o", sys.argv[1]] + srcs, check=True)
PY
  fi
  echo -n "[$v] "; timeout -k 10 120 python tools/rn_drive.py --lib "$lib" || exit 1
  i=$((i+1))
done
