#!/bin/bash
# Round-2 experiment, measured and dropped: the LDS-DMA CRC variants
# 19-22 it selects are no longer in crc32_pieces.hip.
# CRC variants 19 / 20 (LDS-DMA nt staging): parity, then the CRC-alone rate on the C2
# (4 MiB pieces) and C4 (256 KiB pieces) shapes against the default (16), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-19 20}; do
  KRK_CRC_VARIANT=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_full_size.py tests/test_gpu_windowed.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/glds_parity_v$v.log 2>&1 || { echo "parity v$v failed"; tail -30 gpurun_out/glds_parity_v$v.log; exit 1; }
  echo "parity v$v: $(tail -1 gpurun_out/glds_parity_v$v.log)"
done
: > gpurun_out/glds_probe.jsonl
for rep in 1 2; do
  for v in 16 ${VARIANTS:-19 20}; do
    timeout -k 10 200 python tools/probe_perf.py --variant $v --crc-spec 32:100:4096,22:20480:256 --sha none > gpurun_out/glds_v$v.log 2>&1 || { tail -5 gpurun_out/glds_v$v.log; exit 1; }
    sed "s/^{/{\"variant\": $v, /" gpurun_out/glds_v$v.log >> gpurun_out/glds_probe.jsonl
  done
done
cut -c1-230 gpurun_out/glds_probe.jsonl
