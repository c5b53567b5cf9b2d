"""Phase breakdown of the padded-list SSSP kernel (C2; tuning build with -DSHD_SSSP_PROF).

Build:  tools/build_prof.sh SHD_SSSP_PROF routing.hip tools/libshd_sssp_prof.so
Run:    SHD_ACCEL_LIB=tools/libshd_sssp_prof.so python tools/sssp_prof.py [builds]
Prints shader clocks per phase summed over waves, per wave and row (one wave's share of a row).
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

builds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
eng = Engine(0)
# PROBE_GRAPH=c3: the 10k-node BA graph (AUTO = delta buckets, the 1024-thread LDS kernel)
c3 = os.environ.get("PROBE_GRAPH") == "c3"
n = prepare(eng, synth.barabasi_albert(10_000, 3, 2) if c3 else synth.complete_graph(1000, 1))
lat = torch.empty((n, n), dtype=torch.int64, device="cuda")
loss = torch.empty((n, n), dtype=torch.float32, device="cuda")
lib = C.CDLL(_native.LIB_PATH)
out = (C.c_ulonglong * 8)()
run_rows(eng, 0, 0, n, lat, loss)
assert lib.shd_debug_sssp_prof(out, 1) == 0
for _ in range(builds):
    run_rows(eng, 0, 0, n, lat, loss)
torch.cuda.synchronize()
assert lib.shd_debug_sssp_prof(out, 0) == 0
waves = out[7]
print(f"builds={builds} waves={waves} sweeps/row={out[5] / max(waves, 1):.2f} expanded/wave={out[6] / max(waves, 1):.1f} "
      f"ms_main={eng.last_info()['ms_main']:.4f}")
tot = sum(out[:5])
for k, name in enumerate(["init", "scan", "relax (flush)", "sweep end (reduce+barrier)", "output"]):
    print(f"{name:28s} {out[k] / max(waves, 1):10.0f} clk/wave  {100.0 * out[k] / max(tot, 1):5.1f}%")
