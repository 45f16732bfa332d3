set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 120 ./tools/native/h2d_probe > gpurun_out/h2d_probe.json 2>&1 || { echo PROBE_FAIL; cat gpurun_out/h2d_probe.json; exit 1; }
cat gpurun_out/h2d_probe.json
