set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "uniform or config2" > gpurun_out/pytest_ab.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_ab.log; exit 1; }
tail -2 gpurun_out/pytest_ab.log
timeout -k 10 300 python tools/ab_uniform.py --variants 1,2 > gpurun_out/ab1.json 2> gpurun_out/ab1.err || { echo AB_FAIL; tail -20 gpurun_out/ab1.err; exit 1; }
cat gpurun_out/ab1.json
timeout -k 10 300 python tools/ab_uniform.py --variants 1,2 --pieces 131072 --piece-len 131072 > gpurun_out/ab2.json 2>> gpurun_out/ab1.err && cat gpurun_out/ab2.json
timeout -k 10 300 python tools/ab_uniform.py --variants 1,2 --pieces 8192 --piece-len 2097152 > gpurun_out/ab3.json 2>> gpurun_out/ab1.err && cat gpurun_out/ab3.json
