set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/s5_loss_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s5_loss_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
for w in config2 config4; do timeout -k 10 300 python bench.py --workload $w --steps 100 --warmup 20 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['value'], d['ms_per_step'])" || exit 1; done
