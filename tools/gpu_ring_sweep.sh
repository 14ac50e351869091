#!/bin/bash
# Staging ring depth x window size sweep of the end-to-end C2 leg and the files leg
# (DESIGN.md 4.5): gpurun --timeout 1200 -- 'bash tools/gpu_ring_sweep.sh'
mkdir -p gpurun_out/ring_sweep
for rep in 1 2; do
  for nw in 3 4; do
    for mb in 256 512 1024; do
      out=gpurun_out/ring_sweep/e2e_w${nw}_mb${mb}_r${rep}.log
      KRK_STAGING_WINDOWS=$nw KRK_WINDOW_MB=$mb timeout -k 10 200 python bench.py --e2e-only --no-cpu-baseline > $out 2>&1 || { echo "failed $out"; exit 1; }
      echo "e2e w=$nw mb=$mb rep=$rep $(grep -o '"end_to_end": {"value": [0-9.]*' $out)"
    done
  done
done
for nw in 3 4; do
  for mb in 512 1024; do
    out=gpurun_out/ring_sweep/files_w${nw}_mb${mb}.log
    KRK_STAGING_WINDOWS=$nw KRK_WINDOW_MB=$mb timeout -k 10 300 python bench.py --workload files --steps 2 --warmup 1 --no-cpu-baseline > $out 2>&1 || { echo "failed $out"; exit 1; }
    echo "files w=$nw mb=$mb $(grep -o '"value": [0-9.]*' $out | head -1)"
  done
done
