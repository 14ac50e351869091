#!/bin/bash
# Zero-copy slots vs H2D-first, and a smaller pinned pool, on the 256-digester harness.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/engine_zc.jsonl
: > $out
for pass in 1 2; do
  for cfg in "zc 1 4096" "h2d 0 4096" "zc_pool512 1 512"; do
    set -- $cfg
    KRK_SHA_ZERO_COPY=$2 KRK_SLOT_POOL_MB=$3 timeout -k 10 120 tests/native/digesters 256 16 8 > gpurun_out/ezc.log 2>&1 || { echo "rc=$? for $cfg"; tail -3 gpurun_out/ezc.log; exit 1; }
    grep '^{' gpurun_out/ezc.log | sed "s/^{/{\"cfg\": \"$1\", \"pass\": $pass, /" >> $out
  done
done
python3 - <<'P'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/engine_zc.jsonl")]
by = collections.defaultdict(list)
for r in rows:
    if r["round"] > 0:
        by[r["cfg"]].append(r["GBps"])
for k, v in by.items():
    v = sorted(v)
    print(k, "median %.2f min %.2f max %.2f" % (v[len(v) // 2], v[0], v[-1]), v)
P
