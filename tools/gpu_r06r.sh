#!/bin/bash
# Round 6, verdict item 4: where mz_rsearch_nets' HBM bytes go on configs[2].  Traffic model per launch
# (G = 2048, H = 576 floats): x_pred read by both workgroups of a tile (2 x 4.72 MB), the dynamics trunk
# hand-off to the prediction workgroup's reward head (rew_split: 4.72 MB written + 4.72 MB read), h' stored
# (4.72 MB), weights (~0.93 MB per XCD).  Measured: FETCH_SIZE / WRITE_SIZE passes and kernel time with and
# without the hand-off (MZ_RN_NO_RSPLIT=1: the reward head on the dynamics workgroup).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6r && export TMPDIR=/tmp
O=$R/gpurun_out/r6r
B="--net resnet --steps 4 --warmup 1 --no-cpu --search-only"
run() {  # name, command...
  local n=$1; shift
  timeout -k 10 240 "$@" > $O/$n.log 2>&1 || { echo "FAILED $n"; tail -20 $O/$n.log; exit 1; }
}
for v in split nosplit; do
  if [ $v = nosplit ]; then export MZ_RN_NO_RSPLIT=1; else unset MZ_RN_NO_RSPLIT; fi
  run kt_$v rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python bench.py $B
  run fetch_$v rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$v -o run -- python bench.py $B
  run write_$v rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$v -o run -- python bench.py $B
  python tools/pmc_kernels.py $O/pmc_$v.json "MZ_RN_NO_RSPLIT=$([ $v = nosplit ] && echo 1) python bench.py $B" $O/fetch_$v $O/write_$v -- mz_rsearch_nets mz_rsearch_tree_lds mz_rsearch_root > /dev/null || exit 1
  echo "$v $(grep '^{' $O/kt_$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['roofline'].get('traffic'))")"
  grep -E "mz_rsearch" $O/kt_$v/run_kernel_stats.csv | cut -d, -f1-4
  python -c "import json; d=json.load(open('$O/pmc_$v.json'))['kernels']; [print(k, v['FETCH_SIZE'], v['WRITE_SIZE'], v['hbm_bytes_per_launch_fetch_x2']) for k, v in d.items()]"
done
