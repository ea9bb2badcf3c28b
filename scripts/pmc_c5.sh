set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c5/fetch -o run --output-format csv -- python3 tools/c5_only.py > gpurun_out/pmc_c5_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_c5/write -o run --output-format csv -- python3 tools/c5_only.py > gpurun_out/pmc_c5_write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR -d gpurun_out/pmc_c5/sq -o run --output-format csv -- python3 tools/c5_only.py > gpurun_out/pmc_c5_sq.log 2>&1 || exit 1
echo DONE
