#!/bin/bash
# Nontemporal-load CRC variants: parity for 9, then timing of 7 / 9 and the load-only 11 / 10.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
KRK_CRC_VARIANT=9 timeout -k 10 300 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_digest_metainfo.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/crc_parity_v9.log 2>&1
rc=$?; tail -3 gpurun_out/crc_parity_v9.log >&2
[ $rc -ne 0 ] && exit $rc
for v in 7 9 11 10 7 9; do
  timeout -k 10 200 python tools/probe_perf.py --variant $v --crc-gb 16 --sha none >> gpurun_out/crc_nt_probe.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/crc_nt_probe.log >&2; exit $rc; }
done
for v in 7 9 11 10; do
  timeout -k 10 200 python tools/probe_perf.py --variant $v --crc-spec 20:20480:256 --sha none >> gpurun_out/crc_nt_probe_c4.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/crc_nt_probe_c4.log >&2; exit $rc; }
done
cat gpurun_out/crc_nt_probe.log gpurun_out/crc_nt_probe_c4.log >&2
