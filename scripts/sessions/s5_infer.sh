set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_inference.py > gpurun_out/s5_infer_tests.log 2>&1; rc=$?; tail -5 gpurun_out/s5_infer_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/infer_bench.py > gpurun_out/s5_infer_bench.json 2> gpurun_out/s5_infer_bench.err || exit $?
cat gpurun_out/s5_infer_bench.err | grep -v amdgpu.ids
