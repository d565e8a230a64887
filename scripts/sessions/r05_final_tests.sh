set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_final.txt 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests_final.txt
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.txt 2>&1
echo "smoke rc=$?"; tail -3 gpurun_out/smoke_final.txt
exit $rc
