#!/usr/bin/env bash
# PMC passes over the F2 probe (one counter group per rocprofv3 run; probe args passed through,
# e.g. "1 16000000 97 128" for one length class)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-f2}
P=gpurun_out/pmc_$TAG
mkdir -p $P
i=0
for g in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_SALU" \
         "SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g -d $P/p$i -o run --output-format csv -- python3 -u tools/probe_f2.py "$@" > $P/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $P/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $P
