#!/bin/bash
# Round-4 first probe on the 1-GPU box: the sysfs GPU count against torch's
# (each in its own process), the refusal path of a plain `bench.py --gpus 2`,
# the clock stamps in a short config-2 run, and a 2-rank gloo rehearsal with
# the per-rank device identity.
set -o pipefail
OUT=gpurun_out/r04_probe
mkdir -p $OUT
python3 -c "
from vortex_amd import topology
import json
print(json.dumps({'visible': topology.visible_gpus(), 'kfd': topology.kfd_gpus(), 'cap': topology.visibility_cap(),
                  'hip_mapped_after_count': topology.hip_runtime_mapped()}))" > $OUT/topology.json 2>&1 &&
timeout -k 10 120 python3 -c "
import torch, json
print(json.dumps({'torch_count': torch.cuda.device_count()}))" > $OUT/torch_count.json 2>&1 &&
ls -la /dev/dri > $OUT/dev_dri.txt 2>&1
env | grep -E 'VISIBLE|ORDINAL' > $OUT/env_visible.txt
timeout -k 10 120 python3 bench.py --gpus 2 --pieces 1024 --steps 2 --warmup 1 > $OUT/plain2.out 2> $OUT/plain2.err
echo "plain --gpus 2 rc=$?" >> $OUT/plain2.err
timeout -k 10 180 python3 -u bench.py --steps 20 --warmup 10 --no-e2e --no-ragged --no-reverify --no-cpu-baseline \
    > $OUT/bench_c2.json 2> $OUT/bench_c2.err &&
timeout -k 10 240 python3 -u bench.py --gpus 2 --same-device --dist-backend gloo --pieces 1024 --steps 3 --warmup 1 \
    --no-e2e --no-ragged --no-reverify --no-cpu-baseline > $OUT/gloo2.json 2> $OUT/gloo2.err
echo "done rc=$?"
