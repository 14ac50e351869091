#!/bin/bash
# A/B on one box: two-lane consumer pipelined (production) vs rounds2 (var_sha2old build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/sha2p_ab.jsonl
for rep in 1 2 3; do
  for v in prod old; do
    lib=kraken_amd/lib/libkraken_hip.so; [ $v = old ] && lib=kraken_amd/lib/var_sha2old/libkraken_hip.so
    for p in 2 4; do
      KRK_LIB_PATH=$lib timeout -k 10 200 python tools/probe_perf.py --sha-plan $p --crc-gb 0 --sha 8192:4,16384:2 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
      sed "s/^{/{\"build\": \"$v\", \"plan\": $p, /" gpurun_out/ab.log >> gpurun_out/sha2p_ab.jsonl
    done
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/sha2p_ab.jsonl"):
    r = json.loads(l)
    d[(r["build"], r["plan"], r["streams"])].append(r["per_stream_MBps"])
for k in sorted(d): print(k, [round(x, 2) for x in d[k]])
PY
