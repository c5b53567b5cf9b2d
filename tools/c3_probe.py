"""Tuning probe for C3 (10k-node BA m=3): time the full DELTA build under env overrides and
print a checksum of the table:  SHD_SSSP_GLOBAL=1 SHD_SSSP_REORDER=1 python tools/c3_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import prepare, run_rows  # noqa: E402
from shadow_amd import _native as N  # noqa: E402
from shadow_amd import synth  # noqa: E402
from shadow_amd.routing import Engine  # noqa: E402

eng = Engine(0)
el = synth.barabasi_albert(10_000, 3, 2)
n = prepare(eng, el)
lat = torch.empty((n, n), dtype=torch.int64, device="cuda")
loss = torch.empty((n, n), dtype=torch.float32, device="cuda")
for rep in range(3):
    t0 = time.perf_counter()
    run_rows(eng, N.ALGO_DELTA, 0, n, lat, loss)
    dt = time.perf_counter() - t0
i = eng.last_info()
h = (int(lat.sum().item()), int(loss.view(torch.int32).to(torch.int64).sum().item()))
print(f"C3 DELTA ms_main={i['ms_main']:.2f} wall={dt * 1e3:.2f} sum={h} "
      f"env={ {k: v for k, v in os.environ.items() if k.startswith('SHD_')} }", flush=True)
