#!/bin/bash
# Eight-lane SHA-256: parity of the production build, then consumer variants
# (experiment builds kraken_amd/lib/var_*) on C2-shaped streams.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
      tests/test_gpu_digest_metainfo.py -k "sha or digester" > gpurun_out/sha8_pytest.log 2>&1 || { tail -30 gpurun_out/sha8_pytest.log; exit 1; }
  tail -2 gpurun_out/sha8_pytest.log
fi
out=gpurun_out/sha8var.jsonl; : > $out
for v in prod ${VARS-} prod; do  # VARS: names of `make var` builds
  lib=kraken_amd/lib/var_$v/libkraken_hip.so; [ $v = prod ] && lib=kraken_amd/lib/libkraken_hip.so
  KRK_LIB_PATH=$lib timeout -k 10 120 python -u tools/probe_perf.py --crc-gb 0 --sha-plan ${PLAN:-5} --sha "1000:16,1000:16" \
      > gpurun_out/sha8var_$v.log 2>&1 || { tail -20 gpurun_out/sha8var_$v.log; exit 1; }
  sed "s/^{/{\"build\": \"$v\", /" gpurun_out/sha8var_$v.log >> $out
done
cut -c1-160 $out
[ "${BENCH:-1}" = 1 ] || exit 0
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/sha8_bench.log 2>&1 || { tail -30 gpurun_out/sha8_bench.log; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/sha8_bench.log') if l.startswith('{')][0])
r=d['roofline']; ib=r['issue_bound']
print('C2', d['value'], d['ms_per_step'], r['avg_launch_ms'], ib.get('achieved_per_stream_MBps'), ib.get('ceiling_per_stream_MBps'), ib.get('frac'), ib.get('fetch_bound',{}).get('frac'), ib.get('clock_mhz'), d['roofline_crc']['achieved'], d['end_to_end']['value'])"
