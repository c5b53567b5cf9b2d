"""Why the relay round measures slower inside the bench's equeue leg than in its own leg: the same
C5 round timed host-side (a) back to back, (b) after a torch update of the send times + device
sync, (c) with shd_equeue_advance between rounds, (d) both, as the equeue leg does."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from shadow_amd import _native as N
    from shadow_amd import synth
    from shadow_amd.routing import Engine, NetworkGraph
    eng = Engine(0)
    el = synth.complete_graph(1000, 1)
    g = NetworkGraph(el.node_ids, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed)
    t = g.compute_shortest_paths(np.arange(1000, dtype=np.uint32), eng)
    rl = bench.relay_leg(eng, 1, 0, 1, 0, t.lat, t.loss)
    H, P = rl["H"], rl["P"]
    N.check(eng.lib.shd_relay_setup(eng.ctx, H, N.ptr(rl["host_node"]), 1000, N.ptr(t.lat), N.ptr(t.loss),
                                    N.ptr(rl["rng0"]), N.ptr(np.zeros(H, np.uint64))), "relay_setup")
    N.check(eng.lib.shd_equeue_setup(eng.ctx, H), "equeue_setup")
    st = torch.empty(P, dtype=torch.uint8, device="cuda")
    ev = [torch.empty(H + 1, dtype=torch.int32, device="cuda"), torch.empty(P, dtype=torch.int64, device="cuda"),
          torch.empty(P, dtype=torch.int32, device="cuda"), torch.empty(P, dtype=torch.int64, device="cuda"),
          torch.empty(P, dtype=torch.int32, device="cuda")]
    out = N.RelayOut(N.ptr(st).value, *(N.ptr(x).value for x in ev), 0, 0, 0)
    qo = N.EqueueOut()
    b = rl["batch"]
    d = [bench._dev(b.src_off, np.int32), bench._dev(b.send_time, np.int64), bench._dev(b.dst_host, np.int32),
         bench._dev(b.payload, np.int32)]
    t_base = d[1].clone()
    start = rl["start"]
    for mode in ("back_to_back", "update", "advance", "update+advance", "back_to_back"):
        times = []
        for k in range(8):
            if "update" in mode:
                d[1].copy_(t_base + k * 10**6)
                torch.cuda.synchronize()
            batch = N.Batch(P, *(N.ptr(x).value for x in d), None)
            rnd = N.Round(start + 10**6, start + 10**12, 0)
            t0 = time.perf_counter()
            N.check(eng.lib.shd_relay_round_device(eng.ctx, C.byref(batch), C.byref(rnd), C.byref(out)), "relay")
            times.append(time.perf_counter() - t0)
            if "advance" in mode:
                N.check(eng.lib.shd_equeue_advance(eng.ctx, C.byref(out), start + 2 * 10**6, C.byref(qo)), "adv")
            start += 10**6
        print(f"{mode:16s} relay ms per round (last 4): {np.mean(times[4:]) * 1e3:.3f}  all: "
              f"{' '.join(f'{x * 1e3:.3f}' for x in times)}", flush=True)


if __name__ == "__main__":
    main()
