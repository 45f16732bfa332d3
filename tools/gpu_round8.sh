set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench4.err; exit 1; }
cat gpurun_out/bench4.json
timeout -k 10 300 python tools/reverify_bench.py --reps 2 --slots 3 --slot-mib 1024 > gpurun_out/reverify_b.json 2> gpurun_out/reverify.err || { echo REVERIFY_FAIL; tail -20 gpurun_out/reverify.err; exit 1; }
cat gpurun_out/reverify_b.json
