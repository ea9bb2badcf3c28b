#!/usr/bin/env bash
# build tools/tune_counter_<name> with -D knobs:  scripts/build_tune_counter.sh name -DKNOB=V ...
set -eu
name=$1; shift
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include "$@" tools/tune_counter.hip \
  shortseq_amd/csrc/ss_codec.hip shortseq_amd/csrc/ss_runtime.hip -o tools/tune_counter_$name
