set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py tests/test_atari_gpu.py tests/test_bench_sizes_gpu.py tests/test_selfplay_gpu.py -x -q --timeout 120 --timeout-method thread -k "learner or fused or configs3" > gpurun_out/rt.log 2>&1 || { tail -30 gpurun_out/rt.log; exit 1; }
tail -1 gpurun_out/rt.log
for ng in 1 2 4 16; do
  MZ_RN_NG_LEARN=$ng timeout -k 10 200 python bench.py --net resnet --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 > gpurun_out/rb_$ng.log 2>&1 || { tail -20 gpurun_out/rb_$ng.log; exit 1; }
  echo "ng=$ng $(tail -1 gpurun_out/rb_$ng.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['learner_steps_per_s'], d['learner_roofline']['kernel_ms'])")"
done
MZ_RUNROLL_FUSED=1 timeout -k 10 200 python bench.py --net resnet --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 > gpurun_out/rb_f.log 2>&1 || exit 1
echo "fused $(tail -1 gpurun_out/rb_f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['learner_steps_per_s'], d['learner_roofline']['kernel_ms'])")"
