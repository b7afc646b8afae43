#!/bin/bash
# round-4 GPU session (final evidence at HEAD): C5 A/B against the library
# before the round's edge-tile and LDS changes (tools/r04_session_y.sh), then
# the checkpoint sequence (suite, smoke, default bench, traces, share proxy:
# tools/r04_session_s.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r04_session_s.sh || exit 1
bash tools/r04_session_y.sh || exit 1
echo "final session done"
