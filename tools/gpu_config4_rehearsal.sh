#!/bin/bash
# Config 4's shape on the one GPU: 8 gloo ranks x 65,536 x 256 KiB (128 GiB of HBM),
# every rank's identity and clock, and the full-size config-5 re-verify split over
# the 8 ranks (reverify_multi).  A rehearsal of the driver's N=8 line, not a rate.
set -o pipefail
OUT=gpurun_out/${1:-config4}
mkdir -p $OUT
timeout -k 10 900 python -u bench.py --gpus 8 --same-device --dist-backend gloo > $OUT/bench_8rank.json 2> $OUT/bench_8rank.err || { echo REHEARSAL_FAIL; tail -30 $OUT/bench_8rank.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench_8rank.json').read().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'world', d['world_size'], 'distinct', d['ranks']['distinct_devices'], 'clock', d['ranks']['clock_GHz'])
rm=d.get('reverify_multi',{}); print('reverify_multi', {k: rm.get(k,{}).get('value') for k in ('warm','cold')}, rm.get('error'), rm.get('io_threads_per_rank'))
"
