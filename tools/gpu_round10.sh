set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "async or host_batches or verify_files or seeding or known" > gpurun_out/pytest_e2e.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_e2e.log; exit 1; }
tail -1 gpurun_out/pytest_e2e.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench5.json'));print(d['value'],d['e2e'])"
