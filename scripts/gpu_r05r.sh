set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/pmc_step.sh r05final config4 fp16x3 8 || exit $?
cp gpurun_out/pmc_config4_fp16x3_b8.json profiles/pmc_config4_fp16x3_b8.json || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r05_final.json 2> gpurun_out/bench_r05_final.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_final -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/prof_r05_final.log 2>&1
