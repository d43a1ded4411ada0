#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && export TMPDIR=/tmp
MZ_LIB=$R/muzero.jl_amd/lib/libmz_stamps.so timeout -k 10 120 python tools/ds_stamps.py 32 2>&1 | grep -v amdgpu.ids
