# Round 6: the whole GPU suite as the driver runs it (one process, -x), then smoke.  Usage: r06_tests.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06}
timeout -k 10 1000 python -u -m pytest tests -x -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_${tag}.txt 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests_${tag}.txt
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${tag}.txt 2>&1
echo "smoke rc=$?"; tail -3 gpurun_out/smoke_${tag}.txt
exit $rc
