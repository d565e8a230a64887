# Round 6: TDE_BN_MAXCH 256 vs 1024 on config 2 (the secondary workload most sensitive to it in round 2) and the BN /
# trainer GPU tests under 256.  Usage: r06_bnchunk_c2.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
tag=${1:-r06zf}
TDE_BN_MAXCH=256 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_trainers.py -x -q --timeout 150 --timeout-method thread > gpurun_out/tests_${tag}.txt 2>&1 || { tail -30 gpurun_out/tests_${tag}.txt; exit 1; }
tail -2 gpurun_out/tests_${tag}.txt
n=0
for v in "base:" "ch256:TDE_BN_MAXCH=256" "base:" "ch256:TDE_BN_MAXCH=256"; do
  n=$((n+1)); name=${v%%:*}; vars=${v#*:}
  env $vars timeout -k 10 300 python -u bench.py --workload config2 --steps 50 --warmup 10 --no-secondary --no-cpu-baseline > gpurun_out/bench_${tag}_${name}_$n.json 2> gpurun_out/bench_${tag}_${name}_$n.err || { tail -20 gpurun_out/bench_${tag}_${name}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/bench_${tag}_${name}_$n.json "config2 $name"
done
