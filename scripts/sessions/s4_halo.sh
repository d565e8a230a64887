set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "conv" > gpurun_out/halo_kern.log 2>&1; rc=$?; tail -15 gpurun_out/halo_kern.log; [ $rc -le 1 ] || exit $rc
bash scripts/ab_env.sh "halo:X=1" "nohalo:TDE_HALO=0" "halo_nw4:TDE_HALO_NW=4"
timeout -k 10 200 python3 scripts/layer_profile.py --top 30 > gpurun_out/layers_halo.txt 2>&1; head -25 gpurun_out/layers_halo.txt
