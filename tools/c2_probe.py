"""Tuning probe for the C2 build: time every engine / knob combination on the 1k-node complete
graph (tables checked identical).  SHD_SSSP_STATS=1 prints sweeps and expansions."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import prepare, run_rows  # noqa: E402
from shadow_amd import synth  # noqa: E402
from shadow_amd.routing import Engine  # noqa: E402

eng = Engine(0)
GRAPH = os.environ.get("PROBE_GRAPH", "c2")   # c2: 1k complete graph; c3: 10k-node BA m=3
el = synth.complete_graph(1000, 1) if GRAPH == "c2" else synth.barabasi_albert(10_000, 3, 2)
# PROBE_PERM (layout experiments; tables then differ from the unpermuted graph's by the relabelling):
# "random" relabels the nodes at random; "spread" deals the nodes in descending degree order to
# the 16 waves' bitmap words of the 1024-thread LDS kernel (word k belongs to wave k mod 16), so
# the hubs -- the first nodes of a BA graph -- no longer all sit in the first waves' words
PERM = os.environ.get("PROBE_PERM", "")
if PERM:
    V = el.n_nodes
    if PERM == "random":
        p = np.random.default_rng(1).permutation(V)
    else:
        deg = np.bincount(el.src, minlength=V) + np.bincount(el.dst, minlength=V)
        r2n = np.argsort(-deg, kind="stable")           # rank -> node
        NW = 16
        r = np.arange(V)
        q = r // NW
        pos = ((q // 32) * NW + r % NW) * 32 + q % 32   # rank -> position (may pass V: compact below)
        order = np.argsort(pos, kind="stable")          # ranks in position order
        p = np.empty(V, np.int64)
        p[r2n[order]] = np.arange(V)                    # node -> new index
    el = synth.EdgeList(el.node_ids, p[el.src].astype(el.src.dtype), p[el.dst].astype(el.dst.dtype),
                        el.latency_ns, el.packet_loss, el.directed)
n = prepare(eng, el)
lat = torch.empty((n, n), dtype=torch.int64, device="cuda")
loss = torch.empty((n, n), dtype=torch.float32, device="cuda")
ref = None
for spec in sys.argv[1:]:           # "algo[:ENV=val,ENV=val]"
    algo, _, envs = spec.partition(":")
    for kv in filter(None, envs.split(",")):
        k, v = kv.split("=")
        eng.set_knob(k, int(v))   # knobs are per context (read from the env only at shd_open)
    ms = []
    for rep in range(8 if GRAPH == "c2" else 3):
        run_rows(eng, int(algo), 0, n, lat, loss)
        ms.append(eng.last_info()["ms_main"])
    h = (int(lat.sum().item()), int(loss.view(torch.int32).to(torch.int64).sum().item()))
    ref = ref or h
    i = eng.last_info()
    print(f"{spec:40s} main_us={np.median(ms) * 1e3:7.1f} total_us={i['ms_total'] * 1e3:7.1f} kept={i['arcs_kept']} "
          f"same={h == ref}", flush=True)
    for kv in filter(None, envs.split(",")):
        eng.set_knob(kv.split("=")[0], None)
