#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_full_size.py -k c1 > gpurun_out/c1test.log 2>&1 || { tail -30 gpurun_out/c1test.log; exit 1; }
tail -3 gpurun_out/c1test.log
./tools/gpu_r02.sh bc4 bc5 bc5r bf1
