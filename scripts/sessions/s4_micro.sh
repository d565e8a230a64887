set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SH=${SH:-cnv1b,cnv2b,icnv1,icnv2,icnv3}
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  echo "== $name ($vars)"
  env $vars timeout -k 10 120 python3 scripts/conv_micro.py --math bf16x6r --shapes $SH --modes ${MODES:-fwd,dgrad} --reps 20 2>/dev/null | grep -v "^=="
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
true
