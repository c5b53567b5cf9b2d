"""C5 relay rounds feeding the device event queues (bench's equeue leg alone, for profiling)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    import bench
    from shadow_amd import synth
    from shadow_amd.routing import Engine, NetworkGraph
    eng = Engine(0)
    el = synth.complete_graph(1000, 1)
    g = NetworkGraph(el.node_ids, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed)
    t = g.compute_shortest_paths(np.arange(1000, dtype=np.uint32), eng)
    rl = bench.relay_leg(eng, 1, 0, 1, 0, t.lat, t.loss)   # one relay round: the leg's inputs
    r = bench.equeue_leg(eng, rl, t.lat, t.loss)
    print(r, flush=True)


if __name__ == "__main__":
    main()
