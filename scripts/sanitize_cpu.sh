#!/usr/bin/env bash
# Host-code sanitizers: the Cython front with the host C++ codec (csrc/host_codec.h), the
# C oracle and the CPU-baseline port, built with -fsanitize=address,undefined into build/asan/ (the
# in-tree builds are untouched), then the CPU test suite run against those builds with the ASan/UBSan
# runtimes preloaded (python itself is not instrumented; leak checking is off for CPython).
#   scripts/sanitize_cpu.sh [pytest args]      (container only; needs no GPU)
set -eu
cd "$(dirname "$0")/.."
OUT=build/asan
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined -g -O1"
rm -rf $OUT
mkdir -p $OUT/shortseq_amd $OUT/oracle
gcc $SAN -fPIC -std=c11 -march=x86-64-v3 -shared oracle/ss_oracle.c oracle/ref_harness.c -o $OUT/oracle/liboracle.so
g++ $SAN -fPIC -std=c++17 -march=x86-64-v3 -mbmi2 -mpopcnt -fopenmp -shared oracle/cpu_baseline.cpp -o $OUT/oracle/libcpubaseline.so
cp oracle/*.py $OUT/oracle/
python3 -m cython -3 --cplus --module-name shortseq_amd._shortseq -I shortseq_amd/csrc shortseq_amd/csrc/_shortseq.pyx \
    -o $OUT/_shortseq.cpp > /dev/null
PYINC=$(python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
EXT=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
g++ $SAN -std=c++17 -fPIC -shared -mbmi2 -mpopcnt -march=x86-64-v3 -fno-strict-aliasing -w -I"$PYINC" \
    -I shortseq_amd/csrc -I include $OUT/_shortseq.cpp -ldl -o $OUT/shortseq_amd/_shortseq$EXT
cp shortseq_amd/*.py $OUT/shortseq_amd/
ln -s "$PWD/shortseq_amd/lib" $OUT/shortseq_amd/lib          # the HIP library (device code) as built
[ -d oracle/_ref ] && ln -s "$PWD/oracle/_ref" $OUT/oracle/_ref   # the reference build (fuzz test)
PRE="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
# the sanitized builds are the ones the tests import
LD_PRELOAD="$PRE" ASAN_OPTIONS=detect_leaks=0 python3 -c "
import sys; sys.path[:0] = ['$OUT', '$OUT/oracle']
import shortseq_amd._shortseq as m, oracle
assert '$OUT' in m.__file__ and '$OUT' in oracle.LIB_PATH, (m.__file__, oracle.LIB_PATH)
print('sanitized builds:', m.__file__, oracle.LIB_PATH)"
LD_PRELOAD="$PRE" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 SHORTSEQ_TEST_ROOT=$PWD/$OUT \
    python3 -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@"
