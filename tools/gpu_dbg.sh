#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for v in prod noc1 noc2 noc12; do
  lib=kraken_amd/lib/var_$v/libkraken_hip.so; [ $v = prod ] && lib=kraken_amd/lib/libkraken_hip.so
  echo "== $v"; KRK_LIB_PATH=$lib timeout -k 10 120 python -u tools/sha_empty_probe.py || exit 1
done
