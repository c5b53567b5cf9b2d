"""The drop-in flush alone (for tracing): C5 on the C2 table, 16 pinned stages, rounds with 16- and
12-byte events.   python tools/flush_probe.py [rounds]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import ctypes as C

    import bench
    from shadow_amd import _native as N
    from shadow_amd import synth
    from shadow_amd.relay import PinnedStages
    from shadow_amd.routing import Engine, NetworkGraph
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    eng = Engine(0)
    el = synth.complete_graph(1000, 1)
    g = NetworkGraph(el.node_ids, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed)
    t = g.compute_shortest_paths(np.arange(1000, dtype=np.uint32), eng)
    H, P, start, runahead, b, host_node, rng0 = bench.relay_inputs()
    N.check(eng.lib.shd_relay_setup(eng.ctx, H, N.ptr(host_node), 1000, N.ptr(t.lat), N.ptr(t.loss), N.ptr(rng0),
                                    N.ptr(np.zeros(H, np.uint64))), "relay_setup")
    N.check(eng.lib.shd_relay_set_counters(eng.ctx, 0), "set_counters")
    time_base = int(b.send_time.min())
    st = synth.stage_round(b, 16, time_base, seed=11)
    ps = PinnedStages.pinned(eng.lib, st.run_host, st.run_count, st.sends)
    st2 = bench.torch_pinned_u8((P + 3) // 4)
    ev_off = bench.torch_pinned_u8((H + 1) * 4)
    evs = bench.torch_pinned_u8(P * 16)
    sb = bench.torch_pinned_u8(H * 8)
    rnd = N.Round(start + runahead, start + 10**12, 0)
    for eb in (16, 12, 16, 12):
        out = N.FlushOut(st2.data_ptr(), ev_off.data_ptr(), evs.data_ptr(), sb.data_ptr(), 0, 0, 0, 0, eb)
        ms = []
        for _ in range(rounds):
            t0 = time.perf_counter()
            N.check(eng.lib.shd_relay_flush(eng.ctx, ps.array, len(ps.stages), time_base, C.byref(rnd), C.byref(out)),
                    "flush")
            ms.append((time.perf_counter() - t0) * 1e3)
        print(f"event_bytes {eb}: ms per round {np.median(ms):.3f} ({', '.join(f'{x:.2f}' for x in ms)})", flush=True)
    ps.free()


if __name__ == "__main__":
    main()
