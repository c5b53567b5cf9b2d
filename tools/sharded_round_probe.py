"""Cost of the sharded relay round's exchange at full C5 on one GPU: two in-process ranks
(shd_comm_init_local, two contexts on cuda:0, one host thread each) run shd_relay_round_sharded
on their halves of the same batch, against one context running the whole batch through the same
entry point at world size 1.  Both ranks share the device, so their local work adds up to about
the single context's; what the two-rank round costs beyond it is the exchange between ranks: the sizing
all-to-all and its host sync, the 24-byte event packing, the exchange and the per-destination
merge of the two senders' runs.  Prints ms per round for both (median of the timed rounds), and
first the plain device round (shd_relay_round_device) on the same batch, the baseline of the
sharded entry point's fixed cost (PROBE_RCCL=1: the world-1 leg over RCCL instead of the
in-process communicator).  Every timed round ends with a device synchronize.  Under
`rocprofv3 --kernel-trace --memory-copy-trace`, tools/r06_shard_trace.py splits the trace into
the three legs' rounds and prints one round's phases.

    python tools/sharded_round_probe.py [rounds]
"""
import os
import statistics
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import corc  # noqa: E402
from shadow_amd import _native as N  # noqa: E402
from shadow_amd import dist as D  # noqa: E402
from shadow_amd import synth  # noqa: E402
from shadow_amd.routing import Engine  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    H, NN, P = 100_000, 1000, 10_000_000
    el = synth.complete_graph(NN, 1)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False,
                                      np.arange(NN, dtype=np.uint32))
    assert code == "OK"
    host_node, rng0 = synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1)
    start = synth.SIM_START + 10**9
    b = synth.packet_batch(H, P, start, start + 10**6, seed=4)
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()  # noqa: E731

    # ---- the plain device round (shd_relay_round_device), same box, same batch: the baseline the
    #      sharded entry point's fixed cost is measured against
    from shadow_amd.relay import Relay
    e0 = Engine(0)
    N.check(e0.lib.shd_relay_set_counters(e0.ctx, int(os.environ.get("PROBE_COUNTERS", "0"))), "set_counters")
    r0 = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=e0)
    d0 = [dev(b.src_off, np.int32), dev(b.send_time, np.int64), dev(b.dst_host, np.int32), dev(b.payload, np.int32)]
    bufs = r0.device_buffers(P)
    t_plain = []
    for k in range(rounds + 2):
        d0[1].add_(10**6)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r0.round_device(*d0, start + (k + 2) * 10**6, start + 10**12, 0, bufs)
        torch.cuda.synchronize()
        if k >= 2:
            t_plain.append((time.perf_counter() - t0) * 1e3)
    e0.close()
    del d0, bufs

    # ---- one context, the whole batch (the sharded entry point at world size 1)
    e1 = Engine(0)
    if os.environ.get("PROBE_RCCL"):   # the world-1 leg over RCCL (the transport of the driver's N > 1 runs)
        D.comm_init_rccl(e1)
    else:
        D.comm_init_local([e1])
    one = D.ShardedRelay(e1, host_node, rng0, np.zeros(H, np.uint64), lat, loss)
    counters = int(os.environ.get("PROBE_COUNTERS", "0"))   # the bench's relay leg runs without them
    N.check(e1.lib.shd_relay_set_counters(e1.ctx, counters), "set_counters")
    d1 = [dev(b.src_off, np.int32), dev(b.send_time, np.int64), dev(b.dst_host, np.int32), dev(b.payload, np.int32)]
    st1 = torch.empty(P, dtype=torch.uint8, device="cuda")
    t_one = []
    for k in range(rounds + 2):
        d1[1].add_(10**6)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        one.round_device(*d1, (start + (k + 2) * 10**6, start + 10**12, 0), st1)
        torch.cuda.synchronize()
        if k >= 2:
            t_one.append((time.perf_counter() - t0) * 1e3)
    p1 = one.last_pipeline()
    e1.close()

    # ---- two in-process ranks on the same GPU, each its half of the sources
    engines = [Engine(0), Engine(0)]
    D.comm_init_local(engines)
    rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
    for e in engines:
        N.check(e.lib.shd_relay_set_counters(e.ctx, counters), "set_counters")
    parts = []
    for r in rels:
        a, z = int(b.src_off[r.lo]), int(b.src_off[r.hi])
        off = (b.src_off[r.lo:r.hi + 1] - b.src_off[r.lo]).astype(np.uint32)
        parts.append(([dev(off, np.int32), dev(b.send_time[a:z], np.int64), dev(b.dst_host[a:z], np.int32),
                       dev(b.payload[a:z], np.int32)], torch.empty(max(z - a, 1), dtype=torch.uint8, device="cuda")))
    t_two = []
    for k in range(rounds + 2):
        for d, _ in parts:
            d[1].add_(10**6)
        torch.cuda.synchronize()
        rd = (start + (k + 2) * 10**6, start + 10**12, 0)
        ths = [threading.Thread(target=lambda i=i: rels[i].round_device(*parts[i][0], rd, parts[i][1]))
               for i in range(2)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        torch.cuda.synchronize()
        if k >= 2:
            t_two.append((time.perf_counter() - t0) * 1e3)
    p2 = [r.last_pipeline() for r in rels]
    for e in engines:
        e.close()
    m0, m1, m2 = statistics.median(t_plain), statistics.median(t_one), statistics.median(t_two)
    print(f"plain device round (shd_relay_round_device): {m0:.3f} ms; world-1 fixed cost {m1 - m0:.3f} ms", flush=True)
    print(f"one context (world 1), whole C5 round: {m1:.3f} ms; two in-process ranks on the same GPU (halves + "
          f"exchange + merge): {m2:.3f} ms; sharded-path overhead {m2 - m1:.3f} ms per round; pipelines "
          f"{p1} / {p2} (SHD_RELAY_SHARD_X24={os.environ.get('SHD_RELAY_SHARD_X24', '')})", flush=True)


if __name__ == "__main__":
    main()
