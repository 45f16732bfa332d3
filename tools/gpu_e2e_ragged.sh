# config 3 from host memory (tools/e2e_ragged.py): longest-first host batches
# (VX_BATCH_SORT=1, default) against caller order (0), registered and plain.
set -o pipefail
mkdir -p gpurun_out/e2e3
O=gpurun_out/e2e3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_batches or random_mix or gather_batch or scattered or strided or pool_growth" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0 1; do
  VX_BATCH_SORT=$v timeout -k 10 200 python -u tools/e2e_ragged.py >> $O/ab_sort.jsonl 2>> $O/ab.err || { echo FAIL; tail -5 $O/ab.err; exit 1; }
done
for v in 1 0; do
  VX_BATCH_SORT=$v timeout -k 10 200 python -u tools/e2e_ragged.py --scale 0.125 >> $O/ab_sort.jsonl 2>> $O/ab.err || { echo FAIL; tail -5 $O/ab.err; exit 1; }
done
VX_BATCH_SORT=1 timeout -k 10 200 python -u tools/e2e_ragged.py --unregistered --reps 1 >> $O/ab_sort.jsonl 2>> $O/ab.err || { echo FAIL; tail -5 $O/ab.err; exit 1; }
cat $O/ab_sort.jsonl
