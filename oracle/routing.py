"""Routing build restated in Python (test infrastructure only; pure-Python loops: small graphs).

Restates ``src/main/network/graph/mod.rs``:
  * ``PathProperties`` Add / PartialOrd / Default (:298-333): latency u64 add, loss left fold
    ``1f32 - (1f32 - p) * (1f32 - e)`` in binary32, lexicographic (latency, loss) order;
  * ``compute_shortest_paths`` (:185-230) over petgraph 0.6.3 ``algo::dijkstra`` (lazy-deletion
    binary heap, strict ``<`` improvement, visited set), used-node filter, self-loop diagonal,
    ``assert_eq!(paths.len(), n^2)``;
  * ``get_direct_paths`` (:232-254) and ``get_edge_weight`` (:258-295) error rules;
  * ``IpAssignment`` (:354-422), ``RoutingInfo`` (:430-479).
"""
from __future__ import annotations

import heapq

import numpy as np

from .gml import NetworkGraph

F1 = np.float32(1.0)


class RoutingError(Exception):
    """Mirrors the reference's ``Err`` / panic outcomes with a machine-readable code."""

    def __init__(self, code: str, a=None, b=None, msg: str = ""):
        super().__init__(msg or f"{code} {a} {b}")
        self.code, self.a, self.b = code, a, b


def fold(p: np.float32, e: np.float32) -> np.float32:
    """Loss part of ``PathProperties::add`` (graph/mod.rs:324-333), binary32, no FMA."""
    return np.float32(F1 - np.float32(np.float32(F1 - np.float32(p)) * np.float32(F1 - np.float32(e))))


def path_add(a, b):
    """``PathProperties + PathProperties`` -> (latency_ns, loss)."""
    return (a[0] + b[0], fold(a[1], b[1]))


def adjacency(g: NetworkGraph):
    """petgraph ``edges(node)``: directed -> outgoing; undirected -> every incident edge once."""
    adj = [[] for _ in range(g.n_nodes)]
    for e in g.edges:
        adj[e.source].append((e.target, e.latency_ns, e.packet_loss))
        if not g.directed and e.target != e.source:
            adj[e.target].append((e.source, e.latency_ns, e.packet_loss))
    return adj


def dijkstra(adj, start: int):
    """petgraph 0.6.3 ``algo::dijkstra(graph, start, None, cost)`` -> {node: (lat, loss)}."""
    scores = {start: (0, np.float32(0.0))}
    visited = set()
    heap = [(0, np.float32(0.0), start)]
    while heap:
        lat, loss, node = heapq.heappop(heap)
        if node in visited:
            continue
        for (nxt, elat, eloss) in adj[node]:
            if nxt in visited:
                continue
            cand = (lat + elat, fold(loss, eloss))
            old = scores.get(nxt)
            if old is None or cand < old:          # strict lexicographic improvement
                scores[nxt] = cand
                heapq.heappush(heap, (cand[0], cand[1], nxt))
        visited.add(node)
    return scores


def edge_weight(g: NetworkGraph, src: int, dst: int):
    """``get_edge_weight`` (graph/mod.rs:258-295): exactly one edge src->dst ({src,dst})."""
    found = []
    for e in g.edges:
        if (e.source == src and e.target == dst) or (
                not g.directed and e.source == dst and e.target == src):
            found.append(e)
    sid, did = g.node_ids[src], g.node_ids[dst]
    if not found:
        raise RoutingError("NO_EDGE", sid, did, f"No edge connecting node {sid} to {did}")
    if len(found) > 1:
        raise RoutingError("MULTI_EDGE", sid, did,
                           f"More than one edge connecting node {sid} to {did}")
    return (found[0].latency_ns, found[0].packet_loss)


def compute_shortest_paths(g: NetworkGraph, nodes):
    """``compute_shortest_paths`` (graph/mod.rs:185-230) -> {(src_idx, dst_idx): (lat, loss)}."""
    adj = adjacency(g)
    used = set(nodes)
    paths = {}
    for src in nodes:
        for dst, p in dijkstra(adj, src).items():
            if dst in used:
                paths[(src, dst)] = p
    for n in nodes:
        assert paths[(n, n)] == (0, np.float32(0.0))
        paths[(n, n)] = edge_weight(g, n, n)
    if len(paths) != len(nodes) ** 2:
        missing = next((a, b) for a in nodes for b in nodes if (a, b) not in paths)
        raise RoutingError("UNREACHABLE", g.node_ids[missing[0]], g.node_ids[missing[1]],
                           "assertion failed: paths.len() == nodes.len().pow(2)")
    return paths


def get_direct_paths(g: NetworkGraph, nodes):
    """``get_direct_paths`` (graph/mod.rs:232-254): the single edge per ordered pair, no fold."""
    return {(s, d): edge_weight(g, s, d) for s in nodes for d in nodes}


def table(paths: dict, nodes):
    """Dense row-major (lat u64[n,n], loss f32[n,n]) in ``nodes`` order (the build's layout)."""
    n = len(nodes)
    lat = np.zeros((n, n), np.uint64)
    loss = np.zeros((n, n), np.float32)
    for i, s in enumerate(nodes):
        for j, d in enumerate(nodes):
            lat[i, j], loss[i, j] = paths[(s, d)]
    return lat, loss


class IpAssignment:
    """``IpAssignment`` (graph/mod.rs:354-422): explicit IPs, then 11.0.0.1.. skipping .0/.255."""

    def __init__(self):
        self.map = {}
        self.last = (11 << 24)

    @staticmethod
    def _inc(addr: int) -> int:
        while True:
            addr = (addr + 1) & 0xFFFFFFFF
            if addr & 0xFF not in (0, 255):
                return addr

    def assign(self, node_id: int) -> int:
        while True:
            ip = self._inc(self.last)
            self.last = ip
            if ip not in self.map:
                self.map[ip] = node_id
                return ip

    def assign_ip(self, node_id: int, ip: int):
        if ip in self.map:
            raise RoutingError("IP_ASSIGNED", ip, None, "IP address has already been assigned")
        self.map[ip] = node_id

    def get_node(self, ip: int):
        return self.map.get(ip)

    def get_nodes(self):
        return set(self.map.values())


def smallest_latency_ns(lat: np.ndarray) -> int:
    """``RoutingInfo::get_smallest_latency_ns`` (graph/mod.rs:476-478): min over all n^2."""
    return int(lat.min())
