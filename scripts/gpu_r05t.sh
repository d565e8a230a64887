set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u probe/step_timeline.py gpurun_out/timeline_r05t.txt > gpurun_out/timeline_r05t.log 2>&1
