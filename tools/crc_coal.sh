#!/bin/bash
# Coalesced layout with byte-addressable tables: parity for 12, then timing of 7 / 12
# and the load-only diagnostics 11 (strided) / 13 (coalesced) at the same occupancy.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
KRK_CRC_VARIANT=12 timeout -k 10 300 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_digest_metainfo.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/crc_parity_v12.log 2>&1
rc=$?; tail -3 gpurun_out/crc_parity_v12.log >&2
[ $rc -ne 0 ] && exit $rc
for v in 7 12 11 13 7 12 11 13; do
  echo "variant $v" >> gpurun_out/crc_coal_probe.log
  timeout -k 10 200 python tools/probe_perf.py --variant $v --crc-gb 16 --sha none >> gpurun_out/crc_coal_probe.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/crc_coal_probe.log >&2; exit $rc; }
done
cat gpurun_out/crc_coal_probe.log >&2
