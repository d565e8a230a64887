#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for e in 0 1 2; do EXTRA=$e timeout -k 10 200 python -u probe/step_floor.py 2>/dev/null || exit 1; done
