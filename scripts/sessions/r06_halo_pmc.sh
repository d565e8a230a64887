# Round 6: SQ counters of the halo forward / data-gradient kernel on config-4 shapes.  Usage: r06_halo_pmc.sh TAG
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06r}
timeout -k 10 120 python -u scripts/conv_micro.py --math fp16x3 --modes fwd,dgrad --reps 30 \
  --shapes cnv1b_b16,icnv1_b16,icnv2_b16,cnv2b_b16,icnv3_b16 2>&1 | grep -v amdgpu.ids
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d "$PWD/gpurun_out/halopmc_${tag}_$i" -o run --output-format csv \
    -- python3 scripts/conv_micro.py --math fp16x3 --modes fwd --reps 5 --shapes cnv1b_b16,icnv2_b16 \
    > gpurun_out/halopmc_${tag}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/halopmc_${tag}_$i.log; exit $rc; }
done
python3 scripts/kernel_pmc.py gpurun_out/halopmc_${tag}_1 gpurun_out/halopmc_${tag}_2 --filter halo_conv_kernel | tee gpurun_out/halopmc_${tag}.txt
