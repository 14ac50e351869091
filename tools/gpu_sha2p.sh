#!/bin/bash
# Two-lane pipelined blocks (block2p): parity of every SHA plan, the windowed C3 path,
# then the per-stream rate at the two-lane stream counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_digest_metainfo.py tests/test_gpu_windowed.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "sha or digest or windowed or chunk" > gpurun_out/sha2p_parity.log 2>&1 || { tail -30 gpurun_out/sha2p_parity.log; exit 1; }
tail -1 gpurun_out/sha2p_parity.log
: > gpurun_out/sha2p_probe.jsonl
for p in 2 4; do
  timeout -k 10 200 python tools/probe_perf.py --sha-plan $p --crc-gb 0 --sha 8192:4,16384:2 >> gpurun_out/sha2p_probe.jsonl 2>&1 || exit 1
done
cut -c1-200 gpurun_out/sha2p_probe.jsonl
