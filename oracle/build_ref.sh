#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY — builds the *unmodified* reference (AlexTate/ShortSeq) from its own
# Cython sources where they lie under /root/reference, with outputs only into oracle/_ref/.
# Used to (1) generate the golden fixtures under tests/golden/ and (2) validate the C restatement
# in oracle/ss_oracle.c.  Nothing under shortseq_amd/ imports or links this.
#
# Recipe: cython (the reference's own translator, present in the image) -> g++ with the reference's
# flags from setup.py:16-23, except -march=native -> -march=x86-64-v3 so the objects are portable.
# No reference file is copied; the package __init__.py under _ref is our own empty file (we import
# submodules directly), so the reference's __init__.py is never duplicated.
set -euo pipefail
REF=${REF_ROOT:-/root/reference}/shortseq
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$HERE/_ref
if [ ! -d "$REF" ]; then echo "reference not present; skipping _ref build" >&2; exit 0; fi
mkdir -p "$OUT/build" "$OUT/shortseq"
: > "$OUT/shortseq/__init__.py"
PYINC=$(python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
EXT=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
for m in util short_seq_64 short_seq_192 short_seq_var short_seq fast_read counter; do
  so="$OUT/shortseq/$m$EXT"
  if [ -f "$so" ] && [ "$so" -nt "$REF/$m.pyx" ]; then continue; fi
  cython -3 --cplus "$REF/$m.pyx" -o "$OUT/build/$m.cpp" >/dev/null
  g++ -shared -fPIC -O3 -std=c++20 -mbmi2 -mpopcnt -march=x86-64-v3 -w -I"$PYINC" \
      "$OUT/build/$m.cpp" -o "$so"
done
echo "reference built into $OUT"
