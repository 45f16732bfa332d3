# Chain-bound split kernel (1,024 x 4 MiB pieces: 16 pairs of waves, 65,537
# blocks per lane): clock and instruction mix, to tell issue-bound from
# stalled.  Writes gpurun_out/pmc_split/.
#   /usr/local/graft/bin/gpurun --timeout 600 -- bash tools/gpu_pmc_split.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_split
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
W="$R/tools/ab_uniform.py --pieces 1024 --piece-len 4194304 --variants 2 --rounds 1 --reps 2"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $W > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o p1 -- python3 $W > $O/p1.log 2>&1 || { echo PMC1_FAIL; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAVE_CYCLES --output-format csv -d $O/p2 -o p2 -- python3 $W > $O/p2.log 2>&1 || { echo PMC2_FAIL; tail -20 $O/p2.log; exit 1; }
echo OK
