#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MATH=fp16x3 bash scripts/conv_pmc.sh icnv5 fwd i5f && MATH=fp16x3 bash scripts/conv_pmc.sh icnv5 wgrad i5w && MATH=fp16x3 bash scripts/conv_pmc.sh big3x3 fwd b3f
