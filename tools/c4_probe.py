"""Tuning probe for the C4 global-label SSSP: time a row range of the 50k-node BA graph under
env overrides, e.g.  SHD_SSSP_STATS=1 python tools/c4_probe.py 0 4096 1,3  (algos)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import prepare, run_rows  # noqa: E402
from shadow_amd import synth  # noqa: E402
from shadow_amd.routing import Engine  # noqa: E402

rb, re = int(sys.argv[1]), int(sys.argv[2])
algos = [int(a) for a in sys.argv[3].split(",")]
eng = Engine(0)
el = synth.barabasi_albert(50_000, 4, 3)
n = prepare(eng, el)
lat = torch.empty((re - rb, n), dtype=torch.int64, device="cuda")
loss = torch.empty((re - rb, n), dtype=torch.float32, device="cuda")
ref = None
for algo in algos:
    for rep in range(2):
        t0 = time.perf_counter()
        run_rows(eng, algo, rb, re, lat, loss)
        dt = time.perf_counter() - t0
    i = eng.last_info()
    h = (int(lat.sum().item()), int(loss.view(torch.int32).to(torch.int64).sum().item()))
    ref = ref or h
    print(f"algo={algo} rows={re-rb} ms_main={i['ms_main']:.2f} wall={dt*1e3:.2f} per_row_us={i['ms_main']*1e3/(re-rb):.1f} "
          f"same={h == ref} hash={h} env={ {k: v for k, v in os.environ.items() if k.startswith('SHD_')} }", flush=True)
