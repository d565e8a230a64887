set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/head_micro.py > gpurun_out/head_r05n_pf1.txt 2>&1 || exit $?
TDE_RWK_PF=0 timeout -k 10 300 python -u scripts/head_micro.py > gpurun_out/head_r05n_pf0.txt 2>&1 || exit $?
TDE_HEAD_RWK=0 timeout -k 10 300 python -u scripts/head_micro.py > gpurun_out/head_r05n_tiled.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k head > gpurun_out/tests_r05n.log 2>&1
