#!/bin/bash
# Which earlier GPU test file leaves the state under which the C3 host-lane windowed test
# fails (it passes alone, fails after the whole suite)?  One pytest process per file:
# the file's tests, then the lane test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LANE='tests/test_gpu_windowed.py::test_windowed_c3_matches_one_shot_and_oracle[1-200-lane2]'
for f in ${FILES:-tests/test_gpu_*.py}; do
  [ "$f" = tests/test_gpu_windowed.py ] && continue
  timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu "$f" "$LANE" \
    > "gpurun_out/bisect_$(basename $f .py).log" 2>&1
  rc=$?
  echo "$f rc=$rc $(tail -1 gpurun_out/bisect_$(basename $f .py).log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
done
