set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "adam" > gpurun_out/sum_adam.txt 2>&1 || { tail -20 gpurun_out/sum_adam.txt; exit 1; }
tail -2 gpurun_out/sum_adam.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ddp.py > gpurun_out/sum_ddp.txt 2>&1 || { tail -20 gpurun_out/sum_ddp.txt; exit 1; }
tail -2 gpurun_out/sum_ddp.txt
for i in 1 2; do
for x in auto on; do
timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --exchange $x > gpurun_out/sum_bench_${x}_$i.json 2> gpurun_out/sum_bench_${x}_$i.err || { tail -5 gpurun_out/sum_bench_${x}_$i.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['config'].get('hip_graph'), d['config'].get('graph_segment_cuts'))" gpurun_out/sum_bench_${x}_$i.json
done
done
