#!/bin/bash
# fp16x3 conv micro-benchmark (all shapes) + PMC HBM traffic of the config-2 step in fp16x3 (round 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/conv_micro.py --math fp16x3 --reps 20 > gpurun_out/r02d_micro.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/r02d_micro.log
[ $rc -eq 0 ] || exit $rc
bash scripts/pmc.sh r02 config2 fp16x3 8
rc=$?; echo "pmc rc=$rc"; cat gpurun_out/pmc_config2_fp16x3_b8.json | head -50
