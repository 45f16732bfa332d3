# Parallel stage copies for unregistered host batches: tests, then config 3
# from plain memory (tools/e2e_ragged.py --unregistered) and the registered
# rows for reference.
set -o pipefail
mkdir -p gpurun_out/e2e3
O=gpurun_out/e2e3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_batch or submit_errors or random_mix or gather_batch or scattered or strided or streaming or two_contexts" > $O/pytest_stage.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_stage.log; exit 1; }
tail -1 $O/pytest_stage.log
timeout -k 10 200 python -u tools/e2e_ragged.py --unregistered --reps 3 >> $O/stage.jsonl 2>> $O/stage.err || { echo FAIL; tail -5 $O/stage.err; exit 1; }
timeout -k 10 200 python -u tools/e2e_ragged.py --unregistered --reps 3 --scale 0.125 >> $O/stage.jsonl 2>> $O/stage.err || { echo FAIL; tail -5 $O/stage.err; exit 1; }
timeout -k 10 200 python -u tools/e2e_ragged.py >> $O/stage.jsonl 2>> $O/stage.err || { echo FAIL; tail -5 $O/stage.err; exit 1; }
cat $O/stage.jsonl
