set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/wide_ab
python3 -c "import oracle; open('/tmp/exp2m.bin','wb').write(oracle.pool_digest_synth(0x5EED00AA, 0, 97, 2097152, last_index=96, last_len=1179648, threads=16))" || exit 1
for rep in 1 2; do
  for v in prewide widesplit; do
    cp tools/ab/libvortex_amd_$v.so vortex_amd/libvortex_amd.so
    echo -n "{\"v\": \"$v\", \"async2m\": " >> gpurun_out/wide_ab/out.jsonl
    timeout -k 10 120 ./tools/native/async_probe 2097152 1024 16 512 2 | tr -d '\n' >> gpurun_out/wide_ab/out.jsonl || exit 1
    echo -n ", \"loop2m\": " >> gpurun_out/wide_ab/out.jsonl
    timeout -k 10 120 ./tests/native/loop_harness /tmp/exp2m.bin 97 2097152 1179648 0x5EED00AA 32 4 50 | tail -1 | tr -d '\n' >> gpurun_out/wide_ab/out.jsonl || exit 1
    echo "}" >> gpurun_out/wide_ab/out.jsonl
  done
done
cp tools/ab/libvortex_amd_widesplit.so vortex_amd/libvortex_amd.so
cat gpurun_out/wide_ab/out.jsonl
