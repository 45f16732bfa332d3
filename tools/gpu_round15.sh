set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench6.json 2> gpurun_out/bench6.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench6.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench6.json'));print(d['value'], d['roofline']['achieved'], d['roofline']['kernel_ms'])"
