#!/bin/bash
# ResNet network-kernel study: parity, the network kernel timed, and one SQ
# PMC pass (counters averaged over the mz_rsearch_nets dispatches).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_resnet_gpu.py -x -q > gpurun_out/rn.log 2>&1 || { tail -30 gpurun_out/rn.log; exit 1; }
tail -1 gpurun_out/rn.log
timeout -k 10 120 python tools/rn_drive.py || exit 1
[ -n "$NOPMC" ] && exit 0
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES"}
cd /tmp && export TMPDIR=/tmp
for mode in nets; do
  rm -rf "$R/gpurun_out/pmc_$mode"
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d "$R/gpurun_out/pmc_$mode" -o run -- \
      python "$R/tools/rn_drive.py" --n 1 > "$R/gpurun_out/pmc_$mode.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_$mode.log"; exit 1; }
done
python - "$R" <<'PY'
import csv, glob, os, sys, collections
R = sys.argv[1]
for mode in ("nets",):
    tot = collections.defaultdict(float); n = collections.defaultdict(int)
    for f in glob.glob(os.path.join(R, "gpurun_out", f"pmc_{mode}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Kernel_Name"].startswith("mz_rsearch_nets"):
                tot[row["Counter_Name"]] += float(row["Counter_Value"]); n[row["Counter_Name"]] += 1
    print(mode, {k: f"{v / max(n[k], 1):.4g}" for k, v in sorted(tot.items())})
PY
