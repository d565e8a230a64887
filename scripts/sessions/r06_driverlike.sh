# Round 6: the GPU suite exactly as the driver runs it (one process, -x, no per-test timeout plugin), then smoke.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06}
timeout -k 10 900 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider > gpurun_out/gpu_tests_${tag}_driverlike.txt 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_${tag}_driverlike.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${tag}.txt 2>&1; rc=$?
tail -2 gpurun_out/smoke_${tag}.txt; exit $rc
