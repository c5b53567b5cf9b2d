"""Per-wave timeline of the relay's K0 draws (tuning build with -DSHD_STAMP_PROF).

Build:  tools/build_prof.sh SHD_STAMP_PROF relay.hip tools/libshd_k0prof.so
Run:    SHD_ACCEL_LIB=tools/libshd_k0prof.so python tools/k0_prof.py
Prints the waves' start spread, lifetimes (100 MHz clock) and shader clocks per phase.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.argv = [sys.argv[0], "3"]
import relay_only  # noqa: E402
from shadow_amd import _native  # noqa: E402

relay_only.main()
lib = C.CDLL(_native.LIB_PATH)
buf = (C.c_ulonglong * (4096 * 5))()
assert lib.shd_debug_k0_prof(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 5).astype(np.int64)
a = a[a[:, 3] > 0]
t0 = a[:, 3].min()
st, en = (a[:, 3] - t0) / 100.0, (a[:, 4] - t0) / 100.0
print(f"waves={len(a)} span={en.max():.2f}us start p50/p90/max={np.percentile(st, 50):.2f}/{np.percentile(st, 90):.2f}/"
      f"{st.max():.2f}us life p50/max={np.median(en - st):.2f}/{(en - st).max():.2f}us")
for i, n in enumerate(["setup (loads)", "draws", "transpose + stores"]):
    print(f"  {n:20s} p50 {np.median(a[:, i]):8.0f} clk  max {a[:, i].max():8.0f}")
