#!/bin/bash
# Full GPU suite, smoke(), then one default bench run (the driver's form), under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-check_all}
mkdir -p $OUT
bash tools/gpu_tests.sh ${1:-check_all} || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1])
c=d['roofline']['valu']['clock_run']
print('value', d['value'], 'frac', d['roofline']['frac'], 'clock', c.get('GHz_mean'), c.get('one_wave_issue_at_run_clock',{}).get('frac'))
for k in ('cpu_baseline','ragged','e2e','e2e_async','e2e_contiguous','reverify','reverify_cold'):
    v=d.get(k,{}); print(k, v.get('value', v.get('error')), (v.get('cpu_pool') or {}).get('value'))
"
