set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_uniform.py --variants 1,6 --rounds 6 > gpurun_out/ab_alias.json 2> gpurun_out/ab.err || { echo AB_FAIL; tail -20 gpurun_out/ab.err; exit 1; }
cat gpurun_out/ab_alias.json
