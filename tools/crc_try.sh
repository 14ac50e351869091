set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 16 17; do
  KRK_CRC_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_full_size.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/crc_parity_v$v.log 2>&1 || { echo "parity v$v failed"; tail -20 gpurun_out/crc_parity_v$v.log; exit 1; }
  tail -1 gpurun_out/crc_parity_v$v.log
done
for rep in 1 2; do for v in 7 16 17; do
  timeout -k 10 200 python tools/probe_perf.py --variant $v --crc-spec 32:100:4096,22:20480:256 --sha none > gpurun_out/crc_probe_v${v}_$rep.log 2>&1 || exit 1
  echo v$v rep$rep; cat gpurun_out/crc_probe_v${v}_$rep.log
done; done
for v in 7 16; do
  timeout -k 10 200 python tools/probe_perf.py --variant $v --c2 > gpurun_out/crc_c2split_v$v.log 2>&1 || exit 1
  echo c2split v$v; cat gpurun_out/crc_c2split_v$v.log
done
