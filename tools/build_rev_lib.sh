#!/bin/bash
# Build libmz.so of a git revision into muzero.jl_amd/lib/libmz_<name>.so (A/B baselines: MZ_LIB=...).
# Usage: tools/build_rev_lib.sh <rev> <name>
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" archive "$1" muzero.jl_amd/csrc include | tar -x -C "$T"
cd "$T"
ls muzero.jl_amd/csrc/*.hip muzero.jl_amd/csrc/*.cpp | xargs -P 8 -I{} /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC \
  -std=c++17 -ffp-contract=off -fno-fast-math -Wno-unused-result -fno-slp-vectorize -Iinclude -c {} -o {}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/muzero.jl_amd/lib/libmz_$2.so" muzero.jl_amd/csrc/*.o -ldl
rm -rf "$T"
echo "built $R/muzero.jl_amd/lib/libmz_$2.so from $1"
