set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
nproc > gpurun_out/env.txt; grep -m1 'model name' /proc/cpuinfo >> gpurun_out/env.txt; echo "OMP=$OMP_NUM_THREADS" >> gpurun_out/env.txt
python -c "import os; print(len(os.sched_getaffinity(0)))" >> gpurun_out/env.txt
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o check -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof.log 2>&1 || { echo PROF_FAIL; tail -30 $R/gpurun_out/prof.log; exit 1; }
find $R/gpurun_out/prof -name '*stats*'
