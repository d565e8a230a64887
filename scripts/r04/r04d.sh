#!/bin/bash
# Round 4: single-kernel BatchNorm up to 8192 rows per group (1024-thread blocks): BN / conv+BN / trainer tests,
# then the bench line, then split-K block-target A/B on config 4 (TDE_SPLIT_TARGET 256 / 384 vs the default 512).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_nets.py tests/test_gpu_fullsize.py -k "bn or fused or grouped or config4 or config2" > gpurun_out/tests_r04d.log 2>&1
rc=$?; tail -5 gpurun_out/tests_r04d.log; echo "[r04d] tests rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --graph-spans gpurun_out/spans_r04d.json > gpurun_out/bench_r04d.json 2> gpurun_out/bench_r04d.err
rc=$?; echo "[r04d] bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_r04d.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_r04d.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'frac',r['frac'],'busy',r['conv_ms_per_step'],'sum',r['sum_of_call_spans_ms']);print(d['secondary'])"
for t in 256 384 512; do
  TDE_SPLIT_TARGET=$t timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/ab_r04d_split$t.json 2>/dev/null
  rc=$?; [ $rc -ne 0 ] && { echo "split $t rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/ab_r04d_split$t.json'));print('split $t', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
exit 0
