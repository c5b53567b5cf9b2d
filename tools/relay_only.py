"""Run C5 relay rounds only (for profiling): python tools/relay_only.py [rounds] [counters 0/1]."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (one HIP runtime; see shadow_amd/_native.py)
    import bench
    from shadow_amd import synth
    from shadow_amd.routing import Engine
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    counters = len(sys.argv) > 2 and sys.argv[2] == "1"
    eng = Engine(0)
    el = synth.complete_graph(1000, 1)
    from shadow_amd.routing import NetworkGraph
    g = NetworkGraph(el.node_ids, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed)
    t = g.compute_shortest_paths(np.arange(1000, dtype=np.uint32), eng)
    r = bench.relay_leg(eng, 1, 0, rounds, 1, t.lat, t.loss, counters=counters)
    print("ms_per_round", r["ms_per_step"], flush=True)


if __name__ == "__main__":
    main()
