# Ragged split A/B with the box identity and clock/power sampled during the run.
#   /usr/local/graft/bin/gpurun --timeout 600 -- bash tools/gpu_ragged_clock.sh [variants]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/rclock
O=gpurun_out/rclock
hostname > $O/host.txt
timeout -k 5 30 amd-smi static -g 0 --asic --board > $O/asic.txt 2>&1
timeout -k 10 300 python tools/ragged_bench.py --variants ${1:-3,4} --rounds 4 > $O/ragged.json 2> $O/err &
P=$!
sleep 6
for i in 1 2 3 4 5 6; do timeout -k 5 20 amd-smi metric -g 0 -p -c >> $O/busy.txt 2>&1; sleep 1; done
wait $P
RC=$?
grep -m1 -i "serial" $O/asic.txt; cat $O/host.txt
grep -E "SOCKET_POWER|^ +CLK:" $O/busy.txt | head -12
cat $O/ragged.json
exit $RC
