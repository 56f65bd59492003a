#!/usr/bin/env bash
# ORACLE — TEST INFRASTRUCTURE ONLY.
# Builds the REFERENCE's own log-uniform sampler (C++ + Cython binding) from the
# sources where they lie under /root/reference, writing outputs ONLY into oracle/_ref/.
# Used by tests/golden/make_goldens.py to pin oracle/log_uniform_oracle.c and the
# product sampler.  Nothing from /root/reference is copied into the repository;
# oracle/_ref/ is git-ignored.  Needs: cython (image has 3.2.x), g++, numpy headers.
# The reference's shipped log_uniform.cpp / cpython-36 .so are NOT used.
set -euo pipefail
REF=${REF:-/root/reference/U2GNN_pytorch/log_uniform}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
mkdir -p "$OUT"
if [ ! -f "$REF/log_uniform.pyx" ]; then
  echo "reference sources not present at $REF; skipping _ref build" >&2
  exit 0
fi
PY=${PYTHON:-python3}
EXT=$($PY -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
PYINC=$($PY -c 'import sysconfig; print(sysconfig.get_paths()["include"])')
NPINC=$($PY -c 'import numpy; print(numpy.get_include())')
# Cython output goes to oracle/_ref, never next to the .pyx (reference is read-only)
$PY -m cython --cplus -3 -o "$OUT/log_uniform_gen.cpp" "$REF/log_uniform.pyx"
g++ -O2 -std=c++11 -fPIC -shared -w -I"$REF" -I"$PYINC" -I"$NPINC" \
    "$OUT/log_uniform_gen.cpp" "$REF/Log_Uniform_Sampler.cpp" \
    -o "$OUT/log_uniform$EXT"
echo "built $OUT/log_uniform$EXT"
