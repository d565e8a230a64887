# Round 6 closing evidence: PMC traffic refresh (three counter passes; copied into profiles/ so the bench line's
# roofline.traffic reads it), then the driver-form GPU suite, smoke, the default bench line with graph spans, the
# inference timing, the world-1 exchange line and the rocprofv3 kernel-trace summary.  Usage: r06_final.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06z}
bash scripts/pmc_step.sh $tag config4 fp16x3 || exit 1
cp gpurun_out/pmc_config4_fp16x3_b8.json profiles/pmc_config4_fp16x3_b8.json
python3 -c "import json; d=json.load(open('profiles/pmc_config4_fp16x3_b8.json')); print('pmc', d.get('label'), {k: round(v.get('hbm_gb', 0), 2) for k, v in d.get('families', {}).items()} if isinstance(d.get('families'), dict) else '')"
bash scripts/sessions/r06_evidence.sh $tag
