#!/bin/bash
# Eight-lane SHA-256 plan: parity, plan sweep (+ diagnostic consumer-only), C2 bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_digest_metainfo.py -k "sha_launch_plans" > gpurun_out/sha8_pytest.log 2>&1 || { tail -30 gpurun_out/sha8_pytest.log; exit 1; }
tail -2 gpurun_out/sha8_pytest.log
for p in 5 2; do
  timeout -k 10 240 python -u tools/probe_perf.py --crc-gb 0 --sha-plan $p --sha "1000:16,1000:16" \
      > gpurun_out/sha8_probe_p$p.log 2>&1 || { tail -20 gpurun_out/sha8_probe_p$p.log; exit 1; }
  echo "plan $p"; cat gpurun_out/sha8_probe_p$p.log
done
KRK_LIB_PATH=kraken_amd/lib/diag/libkraken_hip.so timeout -k 10 240 python -u tools/probe_perf.py --crc-gb 0 --sha-plan 108 --sha "1000:16,1000:16" \
      > gpurun_out/sha8_probe_p108.log 2>&1 || { tail -20 gpurun_out/sha8_probe_p108.log; exit 1; }
echo "plan 108 (diag consumer only)"; cat gpurun_out/sha8_probe_p108.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/sha8_bench.log 2>&1 || { tail -30 gpurun_out/sha8_bench.log; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/sha8_bench.log') if l.startswith('{')][0])
print('C2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['issue_bound'].get('achieved_per_stream_MBps'), d['roofline_crc']['achieved'], d['end_to_end']['value'])"
