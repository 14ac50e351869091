#!/bin/bash
# A/B of the submission engine's launch depth and first-launch coalescing on the native
# 256-digester harness (tests/native/digesters): interleaved passes, 5 rounds each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/engine_ab.jsonl
: > $out
for pass in 1 2; do
  for cfg in "3 30000 3000" "6 30000 3000" "6 10000 3000" "6 10000 1000"; do
    set -- $cfg
    KRK_ENGINE_INFLIGHT=$1 KRK_SHA_COALESCE_US=$2 KRK_SHA_QUIET_US=$3 timeout -k 10 120 tests/native/digesters 256 16 5 \
      > gpurun_out/eab.log 2>&1 || { echo "rc=$? for $cfg"; tail -3 gpurun_out/eab.log; exit 1; }
    grep '^{' gpurun_out/eab.log | sed "s/^{/{\"inflight\": $1, \"coalesce_us\": $2, \"quiet_us\": $3, \"pass\": $pass, /" >> $out
  done
done
python3 - <<'EOF'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/engine_ab.jsonl")]
by = collections.defaultdict(list)
for r in rows:
    if r["round"] > 0:
        by[(r["inflight"], r["coalesce_us"], r["quiet_us"])].append(r["GBps"])
for k, v in by.items():
    v = sorted(v)
    print(k, "median %.2f min %.2f max %.2f" % (v[len(v) // 2], v[0], v[-1]), v)
EOF
