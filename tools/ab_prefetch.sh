set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pf_t.log 2>&1 || { tail -40 gpurun_out/pf_t.log; exit 1; }
tail -2 gpurun_out/pf_t.log
for n in off on off on; do
  if [ $n = off ]; then export MZ_NO_BATCH_PREFETCH=1; else unset MZ_NO_BATCH_PREFETCH; fi
  timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 --pipeline-moves 10 --train-moves 20 > gpurun_out/pf_b_$n.log 2>&1 || { tail -20 gpurun_out/pf_b_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/pf_b_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp/s', round(d['value']/1e6,2), 'learner', d['learner_steps_per_s'], d['learner_roofline']['kernel_ms'], 'loop', d['train_loop']['learner_steps_per_s'], round(d['train_loop']['node_expansions_per_s']/1e6,2))")"
done
