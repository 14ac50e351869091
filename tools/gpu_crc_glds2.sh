# Round-2 experiment, measured and dropped: the LDS-DMA CRC variants
# 19-22 it selects are no longer in crc32_pieces.hip.
cd /root/repo; mkdir -p gpurun_out; : > gpurun_out/glds2.jsonl
KRK_CRC_VARIANT=22 timeout -k 10 300 python -u -m pytest tests/test_gpu_pieces.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/glds_parity_v22.log 2>&1; tail -1 gpurun_out/glds_parity_v22.log
for v in 16 19 21 22; do
  timeout -k 10 200 python tools/probe_perf.py --variant $v --crc-spec 32:100:4096 --sha none > gpurun_out/glds2_v$v.log 2>&1 || { tail -5 gpurun_out/glds2_v$v.log; exit 1; }
  sed "s/^{/{\"variant\": $v, /" gpurun_out/glds2_v$v.log >> gpurun_out/glds2.jsonl
done
cut -c1-200 gpurun_out/glds2.jsonl
