# Measurement sweep used for DESIGN.md (one gpurun call):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_measure.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/measure
O=gpurun_out/measure
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python tools/ab_uniform.py --variants 1,2 --rounds 6 > $O/ab_uniform.json 2> $O/err.log && cat $O/ab_uniform.json
timeout -k 10 300 python tools/ab_uniform.py --variants 1,2 --pieces 8192 --piece-len 2097152 --rounds 3 > $O/ab_uniform_2MiB.json 2>> $O/err.log && cat $O/ab_uniform_2MiB.json
timeout -k 10 300 python tools/ab_ragged_vs_uniform.py > $O/ab_ragged_vs_uniform.json 2>> $O/err.log && cat $O/ab_ragged_vs_uniform.json
timeout -k 10 300 python tools/ragged_bench.py > $O/ragged.json 2>> $O/err.log && cat $O/ragged.json
timeout -k 10 300 python tools/reverify_bench.py --reps 3 --slots 3 --slot-mib 1024 > $O/reverify.json 2>> $O/err.log && cat $O/reverify.json
timeout -k 10 200 python3 tools/e2e_probe.py > $O/e2e.json 2>> $O/err.log && cat $O/e2e.json
timeout -k 10 120 ./tools/native/h2d_probe > $O/h2d_probe.json 2>> $O/err.log && cat $O/h2d_probe.json
