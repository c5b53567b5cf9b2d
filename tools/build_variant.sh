#!/bin/bash
# Tuning build of the whole library under extra compiler flags (every source, so struct layouts
# agree), linked to <out.so>:  tools/build_variant.sh <out.so> -DNAME=value ...
set -e
cd "$(dirname "$0")/.."
out=$1; shift
FLAGS=$(python -c "from shadow_amd import build as B; print(' '.join(B.FLAGS))")
SRCS=$(python -c "from shadow_amd import build as B; print(' '.join(B.SRC))")
tmp=$(mktemp -d)
objs=""
for s in $SRCS; do
  o=$tmp/$(basename $s).o
  /opt/rocm/bin/hipcc $FLAGS "$@" -c $s -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -L/opt/rocm/lib -lrccl -ldl -lpthread -o $out
rm -rf $tmp
