# Where the lane kernel's non-VALU cycles go: instruction cache and the wait
# counters, on the bench workload.  Writes gpurun_out/icache/.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/icache
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/icache/p1 -o p1 -- python3 $R/bench.py --steps 3 --warmup 0 --no-cpu-baseline --no-e2e > $R/gpurun_out/icache/p1.log 2>&1 || { echo PMC_FAIL; tail -20 $R/gpurun_out/icache/p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_IFETCH_LEVEL --output-format csv -d $R/gpurun_out/icache/p2 -o p2 -- python3 $R/bench.py --steps 3 --warmup 0 --no-cpu-baseline --no-e2e > $R/gpurun_out/icache/p2.log 2>&1 || { echo PMC_FAIL; tail -20 $R/gpurun_out/icache/p2.log; exit 1; }
echo OK
