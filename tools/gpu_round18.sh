set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/ab_ragged_vs_uniform.py > gpurun_out/rvu.json 2> gpurun_out/rvu.err || { echo FAIL; tail -20 gpurun_out/rvu.err; exit 1; }
cat gpurun_out/rvu.json
timeout -k 10 300 python tools/ragged_bench.py --variants 1,2 > gpurun_out/ragged2.json 2>> gpurun_out/rvu.err && cat gpurun_out/ragged2.json
timeout -k 10 300 python tools/reverify_bench.py --reps 3 --slots 3 --slot-mib 1024 > gpurun_out/reverify_e.json 2>> gpurun_out/rvu.err && cat gpurun_out/reverify_e.json
