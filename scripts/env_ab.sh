#!/usr/bin/env bash
# The same command under two settings of one environment variable, interleaved in separate processes:
#   scripts/env_ab.sh <rounds> <VAR> <value_a> <value_b> <cmd...>     (last output line of each run)
set -o pipefail
rounds=$1 var=$2 a=$3 b=$4; shift 4
for r in $(seq 1 "$rounds"); do
  for v in "$a" "$b"; do
    echo "== round $r $var=$v: $(env "$var=$v" timeout -k 10 300 "$@" 2>&1 | tail -2 | tr '\n' ' ')"
  done
done
