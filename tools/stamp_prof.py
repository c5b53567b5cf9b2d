"""Phase breakdown of relay_stamp_v6 (tuning build with -DSHD_STAMP_PROF).

Build:  hipcc <build.py FLAGS> -DSHD_STAMP_PROF <SRC> -o tools/libshd_prof.so
Run:    SHD_ACCEL_LIB=tools/libshd_prof.so python tools/stamp_prof.py [rounds]
Prints shader clocks per phase summed over workgroups, per round and per workgroup.
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [sys.argv[0], sys.argv[1] if len(sys.argv) > 1 else "5"]
import relay_only  # noqa: E402
from shadow_amd import _native  # noqa: E402

relay_only.main()
lib = C.CDLL(_native.LIB_PATH)
out = (C.c_ulonglong * 12)()
assert lib.shd_debug_stamp_prof(out, 0) == 0
names = ["group setup", "rows issue+wait", "rows stage", "chunk barrier", "scan", "stores",
         "run update", "tail", "idx (owner map)", "load issue", "decide(wait)", "-"]
tot = sum(out)
for n, v in zip(names, out):
    print(f"{n:18s} {v:16d}  {100.0 * v / max(tot, 1):5.1f}%")
