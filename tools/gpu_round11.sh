set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/e2etrace -o e2e -- python3 $R/tools/e2e_probe.py > $R/gpurun_out/e2etrace.log 2>&1 || { echo FAIL; tail -20 $R/gpurun_out/e2etrace.log; exit 1; }
tail -2 $R/gpurun_out/e2etrace.log
