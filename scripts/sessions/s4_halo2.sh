set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "conv" > gpurun_out/halo_kern.log 2>&1; rc=$?; tail -3 gpurun_out/halo_kern.log; [ $rc -le 1 ] || exit $rc
bash scripts/sessions/s4_micro.sh "halo:X=1" "nohalo:TDE_HALO=0"
