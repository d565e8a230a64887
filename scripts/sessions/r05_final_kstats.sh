set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_final_c4" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 100 --warmup 20 > gpurun_out/prof_final_c4.log 2>&1 || { tail -5 gpurun_out/prof_final_c4.log; exit 1; }
tail -c 300 gpurun_out/prof_final_c4.log
