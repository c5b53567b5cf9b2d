"""Time the native GML loader (shd_gml_parse) against the oracle's Python restatement on the
C4 graph written out as GML text (50k nodes, ~200k edges + self-loops).

  python tools/gml_bench.py [nodes] [m]     (defaults: 50000 4 = BASELINE config C4)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def gml_text(el) -> str:
    lines = ["graph [", "  directed 0"]
    for i in el.node_ids:
        lines += ["  node [", f"    id {int(i)}", '    host_bandwidth_up "1 Gbit"',
                  '    host_bandwidth_down "1 Gbit"', "  ]"]
    for a, b, lat, p in zip(el.src, el.dst, el.latency_ns, el.packet_loss):
        lines += ["  edge [", f"    source {int(el.node_ids[a])}", f"    target {int(el.node_ids[b])}",
                  f'    latency "{int(lat) // 1000} us"', f"    packet_loss {float(p)!r}", "  ]"]
    return "\n".join(lines + ["]", ""])


def main():
    from oracle.gml import parse_network_graph
    from shadow_amd import synth
    from shadow_amd.routing import NetworkGraph
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    el = synth.barabasi_albert(n, m, 3)
    text = gml_text(el)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        g = NetworkGraph.parse(text)
        ts.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    o = parse_network_graph(text)
    t_py = time.perf_counter() - t0
    assert g.edge_latency_ns.tolist() == [e.latency_ns for e in o.edges]
    assert np.array_equal(g.edge_packet_loss, np.asarray([e.packet_loss for e in o.edges], np.float32))
    mb = len(text.encode()) / 1e6
    print(f"GML {n} nodes {len(g.edge_src)} edges, {mb:.1f} MB: native {min(ts) * 1e3:.1f} ms "
          f"({mb / min(ts):.0f} MB/s, incl. numpy copies), python oracle {t_py * 1e3:.0f} ms, "
          f"identical arrays")


if __name__ == "__main__":
    main()
