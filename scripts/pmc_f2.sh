#!/usr/bin/env bash
# PMC passes over the F2 probe (one counter group per run)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmcf2
export TMPDIR=/tmp
i=0
for g in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum" "SQ_WAIT_ANY SQ_INSTS_FLAT SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g -d gpurun_out/pmcf2/p$i -o run --output-format csv -- python3 -u tools/probe_f2.py 1 > gpurun_out/pmcf2/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmcf2/p$i.log; }
done
ls -R gpurun_out/pmcf2 | head -30
