#!/bin/bash
# bench.py's own GPU tests, then one default bench run (the driver's form), under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-bench_check}
mkdir -p $OUT
bash tools/gpu_tests.sh ${1:-bench_check} tests/test_bench.py || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1])
print('value', d['value'], 'clock', d['roofline']['valu']['clock_run'].get('GHz_mean'))
for k in ('cpu_baseline','ragged','e2e','e2e_async','e2e_contiguous','reverify','reverify_cold'):
    print(k, d.get(k, {}).get('value', d.get(k)), d.get(k, {}).get('bound', ''))
print(json.dumps(d['e2e_async'].get('paced'), indent=0)[:3000])
"
