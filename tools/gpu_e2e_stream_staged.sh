# Unregistered host batches with long pieces stream chunks through the pinned
# stages: tests, then config 3 from plain memory at full and 1/8 scale, and a
# 1,024 x 2 MiB plain-memory batch (tools/e2e_ragged.py --unregistered).
set -o pipefail
mkdir -p gpurun_out/e2e3
O=gpurun_out/e2e3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_batch or submit_errors or random_mix or gather_batch or scattered or strided or streaming or two_contexts or pieces_over or config5" > $O/pytest_sstream.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_sstream.log; exit 1; }
tail -1 $O/pytest_sstream.log
for sc in 1.0 0.125; do
  timeout -k 10 200 python -u tools/e2e_ragged.py --unregistered --reps 3 --scale $sc >> $O/sstream.jsonl 2>> $O/sstream.err || { echo FAIL; tail -5 $O/sstream.err; exit 1; }
done
timeout -k 10 200 python -u tools/e2e_ragged.py --scale 0.125 >> $O/sstream.jsonl 2>> $O/sstream.err || { echo FAIL; tail -5 $O/sstream.err; exit 1; }
cat $O/sstream.jsonl
