set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 900 --timeout-method thread tests/test_golden.py -m gpu > gpurun_out/tests_r05q_golden.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r05q.log 2>&1
