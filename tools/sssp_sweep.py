"""Tuning sweep for the SSSP kernel (G, block, delta) on a config; prints kernel ms per setting.
Settings change only speed: every run is checked bit-identical to the first."""
import ctypes as C
import itertools
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(cfg, algo, reps=5):
    from shadow_amd import _native as N
    from shadow_amd import synth
    from shadow_amd.routing import Engine, NetworkGraph
    el = synth.CONFIGS[cfg]()
    g = NetworkGraph(el.node_ids, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed)
    n = g.n_nodes
    rows = int(os.environ.get("ROWS", n))
    used = np.arange(n, dtype=np.uint32)
    eng = Engine(0)
    err = N.Error()
    cg = g._cgraph()
    N.check(eng.lib.shd_routing_prepare(eng.ctx, C.byref(cg), N.ptr(used), n, 0, C.byref(err)), "prep")
    import torch
    lat = torch.empty((rows, n), dtype=torch.int64, device="cuda")
    loss = torch.empty((rows, n), dtype=torch.float32, device="cuda")
    ts = []
    for _ in range(reps):
        N.check(eng.lib.shd_routing_run(eng.ctx, algo, 0, rows, N.ptr(lat), N.ptr(loss), C.byref(err)), "run")
        info = eng.last_info()
        ts.append((info["ms_main"], info["ms_total"], info["ms_minplus"]))
    h = int(np.frombuffer(lat.cpu().numpy().tobytes(), np.uint8).astype(np.uint64).sum() * 31 +
            np.frombuffer(loss.cpu().numpy().tobytes(), np.uint8).astype(np.uint64).sum())
    ts = np.array(ts[1:])
    print(f"RESULT cfg={cfg} algo={algo} G={os.environ.get('SHD_SSSP_G','auto')} "
          f"block={os.environ.get('SHD_SSSP_BLOCK','256')} delta={os.environ.get('SHD_SSSP_DELTA','auto')} "
          f"main_ms={ts[:,0].mean():.3f} total_ms={ts[:,1].mean():.3f} minplus_ms={ts[:,2].mean():.3f} "
          f"kept={info['arcs_kept']} hash={h}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2:
        one(sys.argv[1], int(sys.argv[2]))
        sys.exit(0)
    cfg = os.environ.get("CFG", "c2")
    grid = os.environ.get("GRID", "")
    runs = []
    for spec in grid.split(";"):
        if spec.strip():
            env = dict(kv.split("=") for kv in spec.split(","))
            runs.append(env)
    for env in runs:
        algo = env.pop("algo", "0")
        e = dict(os.environ, **env)
        subprocess.run([sys.executable, __file__, cfg, algo], env=e, check=False)
