#!/bin/bash
# Kernel trace of the config-2 steps only: per-dispatch times of the warm-up and
# the timed steps (does the clock hold into the timed region?).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-trace_ramp}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-e2e --no-reverify --no-ragged > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $OUT/trace.log; exit 1; }
python3 $R/tools/trace_timed_avg.py --timed 20 $OUT/trace/bench_kernel_trace.csv
