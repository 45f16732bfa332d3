set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/reverify_bench.py --reps 3 --slots 3 --slot-mib 1024 > gpurun_out/reverify_c.json 2> gpurun_out/reverify.err || { echo REVERIFY_FAIL; tail -20 gpurun_out/reverify.err; exit 1; }
cat gpurun_out/reverify_c.json
timeout -k 10 300 python tools/reverify_bench.py --reps 3 --slots 4 --slot-mib 512 > gpurun_out/reverify_d.json 2>> gpurun_out/reverify.err || { echo REVERIFY_FAIL; tail -20 gpurun_out/reverify.err; exit 1; }
cat gpurun_out/reverify_d.json
