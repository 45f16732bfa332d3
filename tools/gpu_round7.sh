set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_loop_harness.py -x -q -s > gpurun_out/pytest_loop.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_loop.log; exit 1; }
grep pieces gpurun_out/pytest_loop.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench3.err; exit 1; }
cat gpurun_out/bench3.json
