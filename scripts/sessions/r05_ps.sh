set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "pixel_shuffle or bwd_fused or deconv or ring_presplit" > gpurun_out/ps_tests.txt 2>&1 || { tail -30 gpurun_out/ps_tests.txt; exit 1; }
tail -2 gpurun_out/ps_tests.txt
AB_BENCH_ARGS="" bash scripts/ab_env.sh "ps7:TDE_PS_MAXK=7" "ps3:TDE_PS_MAXK=3" "ps7nobwd:TDE_PS_BWD=0" "ps7b:TDE_PS_MAXK=7" "ps3b:TDE_PS_MAXK=3"
for n in ps7 ps3 ps7nobwd ps7b ps3b; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'])" gpurun_out/abe_$n.json; done
