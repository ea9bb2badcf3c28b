#!/usr/bin/env bash
# PMC passes over the F1 probe (one counter group per run): where k_fq_nlpos's waves wait
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmcf1
export TMPDIR=/tmp
i=0
for g in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum" \
         "SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $g -d gpurun_out/pmcf1/p$i -o run --output-format csv -- python3 -u tools/probe_f1.py > gpurun_out/pmcf1/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmcf1/p$i.log; exit 1; }
done
find gpurun_out/pmcf1 -name "*.csv" | head -20
