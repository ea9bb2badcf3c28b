set -u
export TMPDIR=/tmp
for v in base det; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/abp/$v -o run --output-format csv -- tools/tune_counter_$v 125000000 10 24 0 > gpurun_out/abp/$v.log 2>&1 || exit 1
done
echo DONE
