set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/s4b_gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s4b_gpu_tests.log; [ $rc -le 1 ] || exit $rc
bash scripts/round_profile.sh r01s4
