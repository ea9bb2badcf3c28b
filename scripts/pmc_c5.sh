#!/usr/bin/env bash
# C5 counter PMC passes (one counter group per rocprofv3 run) over tools/c5_only.py (uniform 2^24),
# summarised by tools/pmc_c5_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
P=gpurun_out/pmc_c5
run() { name=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" -d $P/$name -o run --output-format csv -- python3 tools/c5_only.py 24 0 3 > $P.$name.log 2>&1 || { echo "pass $name failed"; exit 1; }; }
mkdir -p $P
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
# traffic of the C5 variants: FETCH_SIZE / WRITE_SIZE passes only
for v in "U20 20 0" "zipf1.1_U24 24 1.1" "zipf1.1_U20 20 1.1"; do
  set -- $v
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$P/var_$1/$(echo $c | tr A-Z a-z | cut -d_ -f1)
    timeout -s KILL 90 rocprofv3 --pmc $c -d $d -o run --output-format csv -- python3 tools/c5_only.py $2 $3 3 > $P.var_$1.$c.log 2>&1 || { echo "variant pass $1 $c failed"; exit 1; }
  done
done
echo DONE
