#!/bin/bash
# Tuning build: the library with one source compiled under -D<MACRO>, linked to the other
# objects of the normal build:  tools/build_prof.sh <MACRO> <source in csrc/> <out.so>
set -e
cd "$(dirname "$0")/.."
python -c "from shadow_amd import build as B; B.build()" > /dev/null
FLAGS=$(python -c "from shadow_amd import build as B; print(' '.join(B.FLAGS))")
objs=$(ls shadow_amd/build/obj/*.o | grep -v "/$2.o")
/opt/rocm/bin/hipcc $FLAGS -D$1 -c shadow_amd/csrc/$2 -o /tmp/prof_$2.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC /tmp/prof_$2.o $objs -L/opt/rocm/lib -lrccl -ldl -lpthread -o $3
