#!/bin/bash
# A/B of the engine's H2D ordering policies (VX_H2D_MODE, vx_engine.hip
# chain_h2d) on the host e2e probe and the config-5 re-verify.
set -e
mkdir -p gpurun_out/h2d_modes
for rep in 1 2; do
  for m in 0 1 2 3; do
    VX_H2D_MODE=$m timeout -k 10 120 python tools/e2e_probe.py > gpurun_out/h2d_modes/e2e_m${m}_r${rep}.json 2>/dev/null
  done
done
for m in 0 1 2 3; do
  VX_H2D_MODE=$m timeout -k 10 300 python tools/reverify_bench.py --reps 3 > gpurun_out/h2d_modes/reverify_m${m}.json 2>/dev/null
done
