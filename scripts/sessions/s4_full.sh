set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/full_tests.log 2>&1; rc=$?; tail -3 gpurun_out/full_tests.log; grep FAILED gpurun_out/full_tests.log | head; [ $rc -le 1 ] || exit $rc
bash scripts/sessions/s4_micro.sh "d:X=1"
bash scripts/ab_env.sh "halo:X=1" "nohalo:TDE_HALO=0"
