#!/bin/bash
# CRC variant 18 (R4 tables, 24 KiB LDS: co-resident beside a two-pair SHA-256 workgroup):
# parity, then C3 and the CRC-alone rate against the default (16).  Measured in round 2
# and dropped; the variant is no longer in crc32_pieces.hip.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
KRK_CRC_VARIANT=18 timeout -k 10 300 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_windowed.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/crc18_parity.log 2>&1 || { tail -20 gpurun_out/crc18_parity.log; exit 1; }
tail -1 gpurun_out/crc18_parity.log
for v in 16 18; do
  KRK_CRC_VARIANT=$v timeout -k 10 200 python tools/probe_perf.py --variant $v --crc-spec 16:100:4096 --sha none > gpurun_out/crc18_alone_v$v.log 2>&1 || exit 1
  cat gpurun_out/crc18_alone_v$v.log
done
for v in 18 16; do
  KRK_CRC_VARIANT=$v timeout -k 10 600 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/crc18_c3_v$v.log 2>&1 || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/crc18_c3_v$v.log').read().strip().splitlines()[-1]);print('C3 v$v', d['value'], d['ms_per_step'], d['kernels'])"
done
