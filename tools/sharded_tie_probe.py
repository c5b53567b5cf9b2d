"""Diagnostic (round 4, open item): statuses of a sharded C5-style round whose sends all share
one instant, two in-process ranks, against corc.relay_round."""
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import corc  # noqa: E402
from shadow_amd import dist as D  # noqa: E402
from shadow_amd import synth  # noqa: E402
from shadow_amd.routing import Engine  # noqa: E402

H, NN, P = 2000, 40, 150_000
el = synth.complete_graph(NN, 8)
code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False,
                                  np.arange(NN, dtype=np.uint32))
host_node, rng0 = synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1)
start = 10**9
b = synth.packet_batch(H, P, start, start + 10**6, seed=7)
b.send_time[:] = start
rd = (start + 10**6, start + 10**12, 0)
o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                     np.zeros(H, np.uint64), *rd)
engines = [Engine(0), Engine(0)]
D.comm_init_local(engines)
rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
outs = [None, None]


def run(i):
    r = rels[i]
    a, z = int(b.src_off[r.lo]), int(b.src_off[r.hi])
    off = (b.src_off[r.lo:r.hi + 1] - b.src_off[r.lo]).astype(np.uint32)
    outs[i] = r.round(off, b.send_time[a:z], b.dst_host[a:z], b.payload[a:z], rd)


ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
for t in ts:
    t.start()
for t in ts:
    t.join()
for i, r in enumerate(rels):
    a, z = int(b.src_off[r.lo]), int(b.src_off[r.hi])
    st = outs[i][0]
    bad = np.nonzero(st != o["status"][a:z])[0]
    print(f"rank {i}: hosts [{r.lo},{r.hi}) sends {z - a} mismatches {len(bad)}", flush=True)
    if len(bad):
        k = bad[:8]
        hosts = np.searchsorted(b.src_off, a + k, side="right") - 1
        print("  idx", (a + k).tolist(), "gpu", st[k].tolist(), "ref", o["status"][a + k].tolist(),
              "host", hosts.tolist(), "first send of host", b.src_off[hosts].tolist(), flush=True)
    print("  reductions gpu", outs[i][2:], "ref", (o["min_deliver"], o["min_latency"], o["n_sent"]), flush=True)
