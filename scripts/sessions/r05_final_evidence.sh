set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/pmc_step.sh r05final2 config4 fp16x3 8 || exit $?
cp gpurun_out/pmc_config4_fp16x3_b8.json profiles/pmc_config4_fp16x3_b8.json
timeout -k 10 400 python3 bench.py --graph-spans gpurun_out/spans_final.json > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -5 gpurun_out/bench_final.err; exit 1; }
cat gpurun_out/bench_final.json
python3 scripts/spans_table.py gpurun_out/spans_final.json 80 > gpurun_out/spans_final.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_final" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_final.log 2>&1 || { tail -5 gpurun_out/prof_final.log; exit 1; }
ls gpurun_out/prof_final
