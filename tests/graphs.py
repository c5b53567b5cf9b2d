"""Test helpers: graphs from the oracle's GML parser / synthetic generators as engine inputs."""
import numpy as np

from oracle.gml import parse_network_graph

KAT_SHORTEST_PATH = """graph [
                  directed {directed}
                  node [
                    id 0
                  ]
                  node [
                    id 1
                  ]
                  node [
                    id 2
                  ]
                  edge [
                    source 0
                    target 0
                    latency "3333 ns"
                  ]
                  edge [
                    source 1
                    target 1
                    latency "5555 ns"
                  ]
                  edge [
                    source 2
                    target 2
                    latency "7777 ns"
                  ]
                  edge [
                    source 0
                    target 1
                    latency "3 ns"
                  ]
                  edge [
                    source 1
                    target 0
                    latency "5 ns"
                  ]
                  edge [
                    source 0
                    target 2
                    latency "7 ns"
                  ]
                  edge [
                    source 2
                    target 1
                    latency "11 ns"
                  ]
                ]"""
"""Graph text of the reference KAT ``test_shortest_path`` (src/main/network/graph/mod.rs:566-613)."""


def oracle_graph_arrays(g):
    """oracle NetworkGraph -> (node_ids, src, dst, lat, loss, directed)."""
    return (np.asarray(g.node_ids, np.uint32),
            np.asarray([e.source for e in g.edges], np.uint32),
            np.asarray([e.target for e in g.edges], np.uint32),
            np.asarray([e.latency_ns for e in g.edges], np.uint64),
            np.asarray([e.packet_loss for e in g.edges], np.float32),
            g.directed)


def engine_graph_from_gml(text):
    from shadow_amd.routing import NetworkGraph
    ids, s, d, l, p, directed = oracle_graph_arrays(parse_network_graph(text))
    return NetworkGraph(ids, s, d, l, p, directed)


def engine_graph_from_edges(el):
    from shadow_amd.routing import NetworkGraph
    return NetworkGraph(el.node_ids, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed)


def random_graph(rng, n, p_edge, directed, max_ms=20, loss_max=0.3, ties=True, self_loops=True,
                 connected=True):
    """Small random graph with forced ties (integer-ms latencies from a small range)."""
    src, dst = [], []
    for a in range(n):
        for b in range(n):
            if a == b or (not directed and b < a):
                continue
            if rng.random() < p_edge:
                src.append(a); dst.append(b)
    if connected:  # a ring (both directions if directed) guarantees reachability
        for a in range(n):
            b = (a + 1) % n
            if n > 1:
                src.append(a); dst.append(b)
                if directed:
                    src.append(b); dst.append(a)
    if self_loops:
        for a in range(n):
            src.append(a); dst.append(a)
    m = len(src)
    hi = max_ms if ties else 10**6
    lat = rng.integers(1, hi + 1, size=m).astype(np.uint64) * np.uint64(1_000_000 if ties else 1)
    loss = rng.uniform(0, loss_max, size=m).astype(np.float32)
    # some exact-zero and exact-one losses
    z = rng.random(m)
    loss[z < 0.05] = np.float32(0.0)
    order = rng.permutation(m)
    return (np.arange(n, dtype=np.uint32), np.asarray(src, np.uint32)[order],
            np.asarray(dst, np.uint32)[order], lat[order], loss[order], directed)


def gml_text(node_ids, src, dst, lat_ns, loss, directed=False):
    """GML text of an edge list (node indices -> ids), one key per line as the reference's grammar
    wants (a newline after every '[' and value); latencies in ns, losses as float literals."""
    out = ["graph [\n", f"  directed {int(directed)}\n"]
    for i in node_ids:
        out.append(f"  node [\n    id {int(i)}\n  ]\n")
    for a, b, lt, pl in zip(src, dst, lat_ns, loss):
        out.append("  edge [\n    source %d\n    target %d\n    latency \"%d ns\"\n    packet_loss %r\n  ]\n"
                   % (int(node_ids[a]), int(node_ids[b]), int(lt), float(pl)))
    out.append("]\n")
    return "".join(out)
