# Power/clock while the config-2 kernel runs back to back.
#   /usr/local/graft/bin/gpurun --timeout 300 -- bash tools/gpu_power_probe.sh
# Read-only telemetry (amd-smi metric / rocm-smi); changes no GPU setting.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/power
O=gpurun_out/power
timeout -k 5 30 amd-smi static -g 0 --limit --clock > $O/static.txt 2>&1
timeout -k 5 30 amd-smi metric -g 0 -p -c -t > $O/idle.txt 2>&1
timeout -k 10 90 python tools/power_load.py --seconds 15 > $O/load.jsonl 2> $O/load.err &
P=$!
sleep 4
for i in 1 2 3 4 5 6 7 8; do
  date +%s.%N >> $O/busy.txt
  timeout -k 5 20 amd-smi metric -g 0 -p -c -t >> $O/busy.txt 2>&1
  sleep 0.5
done
timeout -k 5 20 rocm-smi --showpower --showclocks >> $O/rocm_smi_busy.txt 2>&1
wait $P
RC=$?
cat $O/load.jsonl
exit $RC
