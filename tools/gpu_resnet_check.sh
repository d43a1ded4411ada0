set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --game atari --no-cpu > gpurun_out/bench_atari.log 2>&1 || { tail -20 gpurun_out/bench_atari.log; exit 1; }
tail -1 gpurun_out/bench_atari.log
timeout -k 10 300 python bench.py --net resnet --no-cpu > gpurun_out/bench_resnet.log 2>&1 || { tail -20 gpurun_out/bench_resnet.log; exit 1; }
tail -1 gpurun_out/bench_resnet.log
