#!/bin/bash
# relay_stamp_v6 phase clocks (wave 0 of every workgroup, -DSHD_STAMP_PROF builds in ablibs/)
cd "$(dirname "$0")/.."
for lib in "$@"; do
  echo "== $lib"
  SHD_ACCEL_LIB=$PWD/ablibs/$lib.so timeout -k 10 120 python3 tools/stamp_prof.py 5 2>&1 | tail -13 || exit 3
done
