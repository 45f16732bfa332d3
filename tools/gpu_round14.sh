set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_uniform.py --variants 1,8,9,10 --rounds 8 > gpurun_out/ab_fence.json 2> gpurun_out/ab.err || { echo AB_FAIL; tail -20 gpurun_out/ab.err; exit 1; }
cat gpurun_out/ab_fence.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc4 -o sq -- python3 $R/tools/ab_uniform.py --variants 1,8,9,10 --rounds 1 --reps 1 > $R/gpurun_out/pmc4.log 2>&1 || { echo PMC_FAIL; tail -20 $R/gpurun_out/pmc4.log; exit 1; }
echo done
