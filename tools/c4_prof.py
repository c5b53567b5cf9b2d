"""Phase breakdown of the SSSP kernels on a BA graph (C4 rows: global labels; C3: LDS labels),
from a tuning build with -DSHD_SSSP_PROF.

Build:  tools/build_prof.sh SHD_SSSP_PROF routing.hip tools/libshd_sssp_prof.so
Run:    SHD_ACCEL_LIB=tools/libshd_sssp_prof.so python tools/c4_prof.py [rows] [c4|c3] [algo]
"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import prepare, run_rows  # noqa: E402
from shadow_amd import _native, synth  # noqa: E402
from shadow_amd.routing import Engine  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
graph = sys.argv[2] if len(sys.argv) > 2 else "c4"
algo = int(sys.argv[3]) if len(sys.argv) > 3 else 3
eng = Engine(0)
n = prepare(eng, synth.barabasi_albert(50_000, 4, 3) if graph == "c4" else synth.barabasi_albert(10_000, 3, 2))
lat = torch.empty((rows, n), dtype=torch.int64, device="cuda")
loss = torch.empty((rows, n), dtype=torch.float32, device="cuda")
lib = C.CDLL(_native.LIB_PATH)
out = (C.c_ulonglong * 8)()
run_rows(eng, algo, 0, rows, lat, loss)
assert lib.shd_debug_sssp_prof(out, 1) == 0
run_rows(eng, algo, 0, rows, lat, loss)
torch.cuda.synchronize()
assert lib.shd_debug_sssp_prof(out, 0) == 0
rw = out[7]   # (row, wave) pairs
print(f"rows={rows} row-waves={rw} sweeps/row={out[5] / max(rw, 1):.2f} expanded/row-wave={out[6] / max(rw, 1):.1f} "
      f"ms_main={eng.last_info()['ms_main']:.3f}")
tot = sum(out[:5])
for k, name in enumerate(["init", "scan", "relax (flush)", "sweep end (reduce+barrier)", "output"]):
    print(f"{name:28s} {out[k] / max(rw, 1):12.0f} clk/row-wave  {100.0 * out[k] / max(tot, 1):5.1f}%")
