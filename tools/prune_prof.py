"""Per-workgroup phase timeline of prune_rows on C2 (tuning build with -DSHD_SSSP_PROF).

Build:  tools/build_prof.sh SHD_SSSP_PROF routing.hip tools/libshd_sssp_prof.so
Run:    SHD_ACCEL_LIB=tools/libshd_sssp_prof.so python tools/prune_prof.py [shape ...]
Per shape (SHD_PRUNE_SHAPE): shader clocks per phase (median over workgroups, thread 0) and the
100 MHz start/end timeline of the workgroups relative to the first start.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import prepare, run_rows  # noqa: E402
from shadow_amd import _native, synth  # noqa: E402
from shadow_amd.routing import Engine  # noqa: E402

eng = Engine(0)
n = prepare(eng, synth.complete_graph(1000, 1))
lat = torch.empty((n, n), dtype=torch.int64, device="cuda")
loss = torch.empty((n, n), dtype=torch.float32, device="cuda")
lib = C.CDLL(_native.LIB_PATH)
buf = (C.c_ulonglong * (4096 * 8))()
names = ["row load + max", "histogram", "boundary bin", "detour selection", "2-hop tests", "list write"]
for shape in (sys.argv[1:] or ["0"]):
    eng.set_knob("PRUNE_SHAPE", int(shape))
    for rep in range(4):
        run_rows(eng, 0, 0, n, lat, loss)
    torch.cuda.synchronize()
    assert lib.shd_debug_prune_prof(buf, 0) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8)[:n].astype(np.int64)
    st, en = a[:, 6] - a[:, 6].min(), a[:, 7] - a[:, 6].min()
    print(f"shape={shape} span={en.max() / 100:.2f}us start p50/p90/max={np.percentile(st, 50) / 100:.2f}/"
          f"{np.percentile(st, 90) / 100:.2f}/{st.max() / 100:.2f}us dur p50/max={np.median(en - st) / 100:.2f}/"
          f"{(en - st).max() / 100:.2f}us")
    for k, nm in enumerate(names):
        print(f"   {nm:18s} p50 {np.median(a[:, k]):8.0f} clk  max {a[:, k].max():8.0f}")
