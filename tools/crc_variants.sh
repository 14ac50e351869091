cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
set -o pipefail
for v in 7 8 5 2 3 0 1; do
  echo "=== parity variant $v" >&2
  KRK_CRC_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_digest_metainfo.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/crc_parity_v$v.log 2>&1
  rc=$?; tail -3 gpurun_out/crc_parity_v$v.log >&2
  if [ $rc -ne 0 ]; then echo "stop rc=$rc" >&2; exit $rc; fi
done
for v in 7 8 5 0 1 2 3; do
  echo "=== probe variant $v" >&2
  timeout -k 10 200 python tools/probe_perf.py --variant $v --crc-gb 16 --sha none > gpurun_out/crc_probe_v$v.log 2>&1
  rc=$?; cat gpurun_out/crc_probe_v$v.log >&2
  if [ $rc -ne 0 ]; then echo "stop rc=$rc" >&2; exit $rc; fi
done
