set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_uniform.py --variants 1,2 --pieces 32768 > gpurun_out/ab4.json 2> gpurun_out/ab.err && cat gpurun_out/ab4.json
timeout -k 10 300 python tools/ab_uniform.py --variants 1,2 --pieces 16384 > gpurun_out/ab5.json 2>> gpurun_out/ab.err && cat gpurun_out/ab5.json
timeout -k 10 300 python tools/ab_uniform.py --variants 1,2 --pieces 1387 --piece-len 2097152 > gpurun_out/ab6.json 2>> gpurun_out/ab.err && cat gpurun_out/ab6.json
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err && cat gpurun_out/bench2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc1 -o fetch -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc1.log 2>&1 || { echo PMC1_FAIL; tail -20 $R/gpurun_out/pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc2 -o sq -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc2.log 2>&1 || { echo PMC2_FAIL; tail -20 $R/gpurun_out/pmc2.log; exit 1; }
ls -R $R/gpurun_out/pmc1 $R/gpurun_out/pmc2 | head
