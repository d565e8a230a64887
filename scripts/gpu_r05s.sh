set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/pmc_step.sh r05bytes config4 fp16x3 8 || exit $?
cp gpurun_out/pmc_config4_fp16x3_b8.json gpurun_out/pmc_r05bytes.json
