#!/bin/bash
# Round-3 closing GPU pass: the whole GPU suite, smoke, the default bench line, the C5 regen
# and C1/c5regen_digest lines, and the end-to-end copy-thread A/B.  Each step under its own
# limit; stop at the first crash / timeout / GPU fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r03.sh test smoke bench bc5r || exit $?
bash tools/e2e_share_ab.sh
