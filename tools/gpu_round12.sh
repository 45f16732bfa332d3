set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for q in 4 8 16; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 tools/e2e_probe.py > gpurun_out/e2e_q$q.json 2>gpurun_out/e2e.err || { echo FAIL; tail gpurun_out/e2e.err; exit 1; }
echo "q=$q $(cat gpurun_out/e2e_q$q.json)"
done
