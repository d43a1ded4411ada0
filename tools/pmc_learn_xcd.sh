#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of mz_learn_small1 with the XCD-affine placement (MZ_LEARN_XCD=1)
# and without, each counter in its own rocprofv3 pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/lxp && export TMPDIR=/tmp
O=$R/gpurun_out/lxp
B="--no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 50"
for v in xcd plain; do
  if [ $v = xcd ]; then export MZ_LEARN_XCD=1; else unset MZ_LEARN_XCD; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 180 rocprofv3 --pmc $c --output-format csv -d $O/${v}_$c -o run -- python bench.py $B > $O/${v}_$c.log 2>&1 || { echo FAILED $v $c; tail -5 $O/${v}_$c.log; exit 1; }
  done
  python - "$O" "$v" <<'PY'
import csv, glob, sys
o, v = sys.argv[1], sys.argv[2]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = []
    for f in glob.glob(f"{o}/{v}_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Kernel_Name", "").startswith("mz_learn_small1"):
                vals.append(float(r["Counter_Value"]))
    print(v, c, "dispatches", len(vals), "mean KB", round(sum(vals) / max(1, len(vals)), 1))
PY
done
