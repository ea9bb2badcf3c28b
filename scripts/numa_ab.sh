#!/usr/bin/env bash
# The same command with the process on the GPU's NUMA node's CPUs and on another node's:
#   scripts/numa_ab.sh <rounds> <cmd...>     (last output line of each run, to stdout)
set -o pipefail
rounds=$1; shift
node=-1
for d in /sys/class/drm/card*/device; do
  [ "$(cat $d/vendor 2>/dev/null)" = "0x1002" ] && node=$(cat $d/numa_node) && break
done
local_cpus=$(cat /sys/devices/system/node/node$node/cpulist 2>/dev/null)
other=$(ls -d /sys/devices/system/node/node[0-9]* | grep -v "node$node\$" | head -1)
other_cpus=$(cat $other/cpulist 2>/dev/null)
echo "gpu node $node: local $local_cpus, other $(basename $other): $other_cpus"
for r in $(seq 1 "$rounds"); do
  for w in local other; do
    c=$local_cpus; [ $w = other ] && c=$other_cpus
    echo "== round $r $w: $(timeout -k 10 300 taskset -c $c "$@" 2>&1 | tail -1)"
  done
done
