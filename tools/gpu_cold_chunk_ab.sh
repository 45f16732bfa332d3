set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/coldchunk
timeout -k 10 300 python -u -m pytest tests/test_gpu_reverify_shard.py tests/test_gpu_layouts.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/coldchunk/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/coldchunk/pytest.log; exit 1; }
tail -2 gpurun_out/coldchunk/pytest.log
timeout -k 10 600 python -u tools/reverify_ab.py --reps 3 --cold-reps 6 --configs "cold1m=;cold_off=VX_VERIFY_COLD_CHUNK=0" > gpurun_out/coldchunk/ab_cold_chunk.jsonl 2> gpurun_out/coldchunk/ab.err || { echo AB_FAIL; tail -20 gpurun_out/coldchunk/ab.err; exit 1; }
tail -3 gpurun_out/coldchunk/ab.err
