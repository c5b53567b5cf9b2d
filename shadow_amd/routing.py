"""Host-side mirror of the reference's routing-build interface, running on the MI355X engine.

Mirrors (FlyearthR/shadow ``src/main/network/graph/mod.rs``):
  * ``NetworkGraph`` (:115-183) with ``node_id_to_index`` / ``node_index_to_id``,
    ``compute_shortest_paths`` (:185-230) and ``get_direct_paths`` (:232-254);
  * ``PathProperties`` as a ``(latency_ns, packet_loss)`` pair (:298-342);
  * ``RoutingInfo`` (:430-479): ``path``, ``increment_packet_count`` (device counters),
    ``get_smallest_latency_ns``;
  * ``generate_routing_info`` (``src/main/core/sim_config.rs:424-461``);
  * ``NetworkGraph.parse`` (:136-183) and ``load_network_graph`` (:481-520) over the native
    GML loader (``shd_gml_parse``; host code, no GPU).
Errors keep the reference's messages: ``Err(..)`` results raise :class:`NetGraphError`; the
reference's ``assert_eq!`` panic on an unreachable pair raises :class:`RoutingPanic`.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


class NetGraphError(Exception):
    """``NetGraphError`` (graph/mod.rs:20): the build returned ``Err``."""


class RoutingPanic(AssertionError):
    """The reference panics here (``assert_eq!(paths.len(), nodes.len().pow(2))``)."""


class Engine:
    """One engine context per GPU (``shd_open``)."""

    def __init__(self, device: int = 0):
        self.lib = N.load()
        st = C.c_int32(0)
        self.ctx = self.lib.shd_open(device, C.byref(st))
        if not self.ctx:
            raise N.ShdError(st.value, f"shd_open(device={device})")
        self.device = device

    def close(self):
        if self.ctx:
            self.lib.shd_close(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_stream(self, stream_handle: int | None):
        N.check(self.lib.shd_set_stream(self.ctx, C.c_void_p(stream_handle) if stream_handle else None),
                "shd_set_stream")

    def last_info(self) -> dict:
        info = N.RoutingInfo()
        N.check(self.lib.shd_routing_last_info(self.ctx, C.byref(info)), "shd_routing_last_info")
        return {k: getattr(info, k) for k, _ in N.RoutingInfo._fields_}

    def smallest_latency_ns(self) -> int:
        v = C.c_uint64(0)
        N.check(self.lib.shd_routing_smallest_latency(self.ctx, C.byref(v)), "smallest_latency")
        return v.value


_default_engine = None


def default_engine() -> Engine:
    global _default_engine
    if _default_engine is None:
        _default_engine = Engine(0)
    return _default_engine


class PathTable:
    """Dense used-node table (row-major in ``nodes`` order): the build's output layout."""

    def __init__(self, graph: "NetworkGraph", nodes, lat: np.ndarray, loss: np.ndarray,
                 row_begin: int = 0):
        self.graph = graph
        self.nodes = list(nodes)
        self.lat = lat
        self.loss = loss
        self.row_begin = row_begin
        self._col = {n: j for j, n in enumerate(self.nodes)}

    def __getitem__(self, key):
        s, d = key
        i = self._col[s] - self.row_begin
        j = self._col[d]
        return int(self.lat[i, j]), np.float32(self.loss[i, j])

    def __len__(self):
        return self.lat.size

    def to_dict(self):
        """``HashMap<(NodeIndex, NodeIndex), PathProperties>`` as the reference returns it."""
        out = {}
        for i in range(self.lat.shape[0]):
            s = self.nodes[self.row_begin + i]
            for j, d in enumerate(self.nodes):
                out[(s, d)] = (int(self.lat[i, j]), np.float32(self.loss[i, j]))
        return out


class NetworkGraph:
    """A parsed network graph: node GML ids and edges (by node index, GML order)."""

    def __init__(self, node_ids, edge_src, edge_dst, edge_latency_ns, edge_packet_loss,
                 directed: bool = False):
        self.node_ids = np.ascontiguousarray(node_ids, np.uint32)
        self.edge_src = np.ascontiguousarray(edge_src, np.uint32)
        self.edge_dst = np.ascontiguousarray(edge_dst, np.uint32)
        self.edge_latency_ns = np.ascontiguousarray(edge_latency_ns, np.uint64)
        self.edge_packet_loss = np.ascontiguousarray(edge_packet_loss, np.float32)
        self.directed = bool(directed)
        self._id_to_index = {int(v): i for i, v in enumerate(self.node_ids)}

    @classmethod
    def parse(cls, graph_text) -> "NetworkGraph":
        """``NetworkGraph::parse`` (graph/mod.rs:136-183) through the native loader.

        Raises :class:`NetGraphError` with the reference's message on any GML or validation
        error, :class:`RoutingPanic` for an edge latency beyond u64 ns (the reference's
        ``convert(Nano).unwrap()``, :338)."""
        lib = N.load()
        data = graph_text.encode() if isinstance(graph_text, str) else bytes(graph_text)
        h = C.c_void_p()
        msg = C.create_string_buffer(1024)
        st = lib.shd_gml_parse(data, len(data), C.byref(h), msg, len(msg))
        if st != N.SHD_OK:
            text = msg.value.decode("utf-8", "replace")
            if N.STATUS_NAMES.get(st) == "LATENCY_OVERFLOW":
                raise RoutingPanic(text)
            raise NetGraphError(text)
        try:
            v = N.Graph()
            N.check(lib.shd_gml_graph(h, C.byref(v)), "shd_gml_graph")

            def arr(p, n, ct, dt):
                if n == 0:
                    return np.zeros(0, dt)
                return np.ctypeslib.as_array(C.cast(p, C.POINTER(ct)), shape=(n,)).astype(dt, copy=True)
            g = cls(arr(v.node_ids, v.n_nodes, C.c_uint32, np.uint32),
                    arr(v.edge_src, v.n_edges, C.c_uint32, np.uint32),
                    arr(v.edge_dst, v.n_edges, C.c_uint32, np.uint32),
                    arr(v.edge_latency_ns, v.n_edges, C.c_uint64, np.uint64),
                    arr(v.edge_packet_loss, v.n_edges, C.c_float, np.float32), bool(v.directed))
            down = np.empty(v.n_nodes, np.uint64)
            up = np.empty(v.n_nodes, np.uint64)
            N.check(lib.shd_gml_node_bandwidth(h, N.ptr(down), N.ptr(up)), "shd_gml_node_bandwidth")
            g.bandwidth_down_bps, g.bandwidth_up_bps = down, up   # UINT64_MAX = not given
            return g
        finally:
            lib.shd_gml_free(h)

    @property
    def n_nodes(self) -> int:
        return len(self.node_ids)

    def node_id_to_index(self, gml_id: int):
        return self._id_to_index.get(int(gml_id))

    def node_index_to_id(self, index: int):
        return int(self.node_ids[index]) if 0 <= index < self.n_nodes else None

    def _cgraph(self) -> N.Graph:
        return N.Graph(self.n_nodes, len(self.edge_src), N.ptr(self.edge_src).value,
                       N.ptr(self.edge_dst).value, N.ptr(self.edge_latency_ns).value,
                       N.ptr(self.edge_packet_loss).value, N.ptr(self.node_ids).value,
                       int(self.directed))

    def _build(self, nodes, mode, algo, engine, rows):
        eng = engine or default_engine()
        used = np.ascontiguousarray(nodes, np.uint32)
        n = len(used)
        rb, re = (0, n) if rows is None else rows
        lat = np.zeros((re - rb, n), np.uint64)
        loss = np.zeros((re - rb, n), np.float32)
        err = N.Error()
        g = self._cgraph()
        st = eng.lib.shd_routing_build(eng.ctx, C.byref(g), N.ptr(used), n, mode, algo, rb, re,
                                       N.ptr(lat), N.ptr(loss), C.byref(err))
        if st in (1, 2):
            what = "No edge connecting" if st == 1 else "More than one edge connecting"
            raise NetGraphError(f"{what} node {err.node_a} to {err.node_b}")
        if st == 3:
            raise RoutingPanic(f"assertion failed: paths.len() == nodes.len().pow(2) "
                               f"(no path from node {err.node_a} to {err.node_b})")
        N.check(st, "shd_routing_build", err)
        return PathTable(self, list(used), lat, loss, rb)

    def compute_shortest_paths(self, nodes, engine: Engine | None = None,
                               algo: int = N.ALGO_AUTO, rows=None) -> PathTable:
        """``NetworkGraph::compute_shortest_paths`` (graph/mod.rs:185-230)."""
        return self._build(nodes, N.ROUTE_SHORTEST, algo, engine, rows)

    def get_direct_paths(self, nodes, engine: Engine | None = None, rows=None) -> PathTable:
        """``NetworkGraph::get_direct_paths`` (graph/mod.rs:232-254)."""
        return self._build(nodes, N.ROUTE_DIRECT, N.ALGO_AUTO, engine, rows)


class RoutingInfo:
    """``RoutingInfo<u32>`` keyed by GML node ids (graph/mod.rs:430-479)."""

    def __init__(self, table: PathTable):
        self.table = table
        g = table.graph
        self._idx = {int(g.node_ids[n]): n for n in table.nodes}
        self.packet_counts = {}

    def path(self, start: int, end: int):
        s, e = self._idx.get(start), self._idx.get(end)
        if s is None or e is None:
            return None
        return self.table[(s, e)]

    def increment_packet_count(self, start: int, end: int):
        k = (start, end)
        self.packet_counts[k] = min(self.packet_counts.get(k, 0) + 1, (1 << 64) - 1)

    def get_smallest_latency_ns(self):
        return int(self.table.lat.min()) if self.table.lat.size else None


def generate_routing_info(graph: NetworkGraph, nodes, use_shortest_paths: bool = True,
                          engine: Engine | None = None) -> RoutingInfo:
    """``generate_routing_info`` (sim_config.rs:424-461): ``nodes`` are GML ids of used nodes."""
    idx = [graph.node_id_to_index(n) for n in nodes]
    table = (graph.compute_shortest_paths(idx, engine) if use_shortest_paths
             else graph.get_direct_paths(idx, engine))
    return RoutingInfo(table)


def load_network_graph(path: str) -> str:
    """``load_network_graph`` (graph/mod.rs:481-520) for a GML file source: the text of `path`,
    xz-decompressed when it ends in ``.xz`` (the reference's ``compression: xz``; Python's
    lzma stands in for lzma-rs), decoded as strict UTF-8 like ``String::from_utf8``."""
    import lzma
    if path.endswith(".xz"):
        with lzma.open(path, "rb") as f:
            raw = f.read()
    else:
        with open(path, "rb") as f:
            raw = f.read()
    try:
        return raw.decode("utf-8")
    except UnicodeDecodeError as e:
        raise NetGraphError(f"invalid utf-8: {e}") from None
