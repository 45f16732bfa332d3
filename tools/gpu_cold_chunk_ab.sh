#!/bin/bash
# Cold re-verify (file evicted before every call) with the default 256 KiB
# rounds against vx_config.verify_cold_chunk = 512 KiB / 1 MiB, alternating;
# then the chunk-schedule parity tests (the ramp now also covers pieces of
# exactly two chunks).
set -o pipefail
OUT=gpurun_out/${1:-cold_chunk_ab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "chunk_schedule or chunked" \
  --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TEST_FAIL; tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python -u tools/reverify_ab.py --cold-reps 8 --cold-only --no-cpu \
  --configs "c256k=;c512k=verify_cold_chunk=524288;c1m=verify_cold_chunk=1048576" > $OUT/ab.jsonl 2> $OUT/ab.err \
  || { echo AB_FAIL; tail -5 $OUT/ab.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); c=d.get('cold') or []
    print(d['config'], sorted(c)[len(c)//2] if c else None, c, [t.get('chunk_bytes') for t in d.get('cold_tr',[])][:1], [round(t.get('tail_ms',0),1) for t in d.get('cold_tr',[])])"
