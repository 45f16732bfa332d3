set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_uniform.py --variants 2,11 --pieces 8192 --piece-len 2097152 --rounds 4 > gpurun_out/ab_op1.json 2> gpurun_out/ab.err || { echo AB_FAIL; tail -20 gpurun_out/ab.err; exit 1; }
cat gpurun_out/ab_op1.json
timeout -k 10 300 python tools/ab_uniform.py --variants 2,11 --pieces 16384 --rounds 6 > gpurun_out/ab_op2.json 2>> gpurun_out/ab.err && cat gpurun_out/ab_op2.json
timeout -k 10 300 python tools/ragged_bench.py --variants 2,11 > gpurun_out/ragged_op.json 2>> gpurun_out/ab.err && cat gpurun_out/ragged_op.json
