set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/ragged_bench.py > gpurun_out/ragged.json 2> gpurun_out/ragged.err || { echo RAGGED_FAIL; tail -20 gpurun_out/ragged.err; exit 1; }
cat gpurun_out/ragged.json
timeout -k 10 400 python tools/reverify_bench.py > gpurun_out/reverify.json 2> gpurun_out/reverify.err || { echo REVERIFY_FAIL; tail -20 gpurun_out/reverify.err; exit 1; }
cat gpurun_out/reverify.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --same-device --no-cpu-baseline --no-e2e > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err || { echo BENCH2_FAIL; tail -30 gpurun_out/bench_2rank.err; exit 1; }
cat gpurun_out/bench_2rank.json
