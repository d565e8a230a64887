set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/psw_tests.txt 2>&1 || { tail -30 gpurun_out/psw_tests.txt; exit 1; }
tail -2 gpurun_out/psw_tests.txt
bash scripts/ab_env.sh "psw:TDE_PSW_MINM=8192" "nopsw:TDE_PSW_MINM=0" "psw2:TDE_PSW_MINM=8192" "nopsw2:TDE_PSW_MINM=0"
for n in psw nopsw psw2 nopsw2; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'])" gpurun_out/abe_$n.json; done
