set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/c5p
for cfg in "24 0" "24 1.1" "20 0" "20 1.1"; do
  set -- $cfg
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5p/u$1_z$2 -o run --output-format csv -- python3 tools/c5_only.py $1 $2 10 > gpurun_out/c5p/u$1_z$2.log 2>&1 || exit 1
done
echo DONE
