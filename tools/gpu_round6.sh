set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_loop_harness.py -x -q -s > gpurun_out/pytest_loop.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_loop.log; exit 1; }
tail -3 gpurun_out/pytest_loop.log
