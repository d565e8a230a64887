set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/s5l_gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s5l_gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5l_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/s5l_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/s5l_bench.json 2> gpurun_out/s5l_bench.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/s5l_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'], d['depth_l1_vs_ref']['worst_max_rel'])"
