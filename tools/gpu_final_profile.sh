# Round-end evidence: bench line + rocprofv3 kernel stats + PMC traffic for the
# hot kernel, all from the same binary.  Writes gpurun_out/${OUT:-final}/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/${OUT:-final}
timeout -k 10 400 python bench.py > gpurun_out/${OUT:-final}/bench.json 2> gpurun_out/${OUT:-final}/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/${OUT:-final}/bench.err; exit 1; }
cat gpurun_out/${OUT:-final}/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${OUT:-final}/trace -o bench -- python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-e2e --no-reverify > $R/gpurun_out/${OUT:-final}/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $R/gpurun_out/${OUT:-final}/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${OUT:-final}/pmc_fetch -o fetch -- python3 $R/bench.py --steps 3 --warmup 0 --no-cpu-baseline --no-e2e --no-ragged --no-reverify > $R/gpurun_out/${OUT:-final}/pmc_fetch.log 2>&1 || { echo PMC_FAIL; tail -20 $R/gpurun_out/${OUT:-final}/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/${OUT:-final}/pmc_sq -o sq -- python3 $R/bench.py --steps 3 --warmup 0 --no-cpu-baseline --no-e2e --no-ragged --no-reverify > $R/gpurun_out/${OUT:-final}/pmc_sq.log 2>&1 || { echo PMC_FAIL; tail -20 $R/gpurun_out/${OUT:-final}/pmc_sq.log; exit 1; }
grep -h sha1 $R/gpurun_out/${OUT:-final}/trace/bench_kernel_stats.csv
