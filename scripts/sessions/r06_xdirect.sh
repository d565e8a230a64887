# Round 6: the exchange over direct RCCL communicators (tf_depth_estimation_amd/rccl.py): the RCCL GPU tests, then
# the world-1 exchange benches (segments inline with 256 / 64 MB buckets, graph mode).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06e}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_ddp_world2.py -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests_${tag}_ddp.txt 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_${tag}_ddp.txt; [ $rc -ne 0 ] && exit $rc
for v in "segments 256" "segments 64" "graph 256"; do
  set -- $v
  timeout -k 10 300 python3 bench.py --exchange on --exchange-mode $1 --bucket-mb $2 --no-cpu-baseline --no-secondary --steps 60 --warmup 15 > gpurun_out/bench_${tag}_x$1_b$2.json 2> gpurun_out/bench_${tag}_x$1_b$2.err || { tail -5 gpurun_out/bench_${tag}_x$1_b$2.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['config']['grad_exchange'], d['config']['graph_segment_cuts'])" gpurun_out/bench_${tag}_x$1_b$2.json
done
echo done
