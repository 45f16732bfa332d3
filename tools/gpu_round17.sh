set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_ragged_vs_uniform.py > gpurun_out/rvu.json 2> gpurun_out/rvu.err || { echo FAIL; tail -20 gpurun_out/rvu.err; exit 1; }
cat gpurun_out/rvu.json
timeout -k 10 300 python tools/ab_ragged_vs_uniform.py --pieces 1387 > gpurun_out/rvu2.json 2>> gpurun_out/rvu.err && cat gpurun_out/rvu2.json
