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

    def set_knob(self, name: str, value: int | None):
        """Tuning / testing knob of this context (knobs.h; None or < 0: the built-in default).
        Knobs start from the SHD_<name> environment variables, read once when the engine opens."""
        v = -1 if value is None else int(value)
        N.check(self.lib.shd_set_knob(self.ctx, name.encode(), v), f"shd_set_knob({name})")

    def get_knob(self, name: str) -> int | None:
        v = C.c_int64(0)
        N.check(self.lib.shd_get_knob(self.ctx, name.encode(), C.byref(v)), f"shd_get_knob({name})")
        return None if v.value < 0 else v.value

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
        return cls._from_handle(lib, h)

    @classmethod
    def _from_handle(cls, lib, h) -> "NetworkGraph":
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
        self._raise(st, err)
        return PathTable(self, list(used), lat, loss, rb)

    def compute_shortest_paths(self, nodes, engine: Engine | None = None,
                               algo: int = N.ALGO_AUTO, rows=None) -> PathTable:
        """``NetworkGraph::compute_shortest_paths`` (graph/mod.rs:185-230)."""
        return self._build(nodes, N.ROUTE_SHORTEST, algo, engine, rows)

    def get_direct_paths(self, nodes, engine: Engine | None = None, rows=None) -> PathTable:
        """``NetworkGraph::get_direct_paths`` (graph/mod.rs:232-254)."""
        return self._build(nodes, N.ROUTE_DIRECT, N.ALGO_AUTO, engine, rows)

    def compute_next_hops(self, nodes, engine: Engine | None = None, algo: int = N.ALGO_AUTO, rows=None,
                          shortest: bool = True):
        """The table plus next hops (``shd_routing_run_next_hops``; the reference keeps none).
        Returns (PathTable, next_hop[r, n] node indices): next_hop(s, d) is the node after s on
        the lowest-index tight-predecessor chain of d; next_hop(s, s) = s."""
        import torch
        eng = engine or default_engine()
        used = np.ascontiguousarray(nodes, np.uint32)
        n = len(used)
        rb, re = (0, n) if rows is None else rows
        err = N.Error()
        g = self._cgraph()
        st = eng.lib.shd_routing_prepare(eng.ctx, C.byref(g), N.ptr(used), n,
                                         N.ROUTE_SHORTEST if shortest else N.ROUTE_DIRECT, C.byref(err))
        self._raise(st, err)
        lat = torch.empty((re - rb, n), dtype=torch.int64, device="cuda")
        loss = torch.empty((re - rb, n), dtype=torch.float32, device="cuda")
        nh = torch.empty((re - rb, n), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        st = eng.lib.shd_routing_run_next_hops(eng.ctx, algo, rb, re, N.ptr(lat), N.ptr(loss), N.ptr(nh),
                                               C.byref(err))
        self._raise(st, err)
        t = PathTable(self, list(used), lat.cpu().numpy().view(np.uint64), loss.cpu().numpy(), rb)
        return t, nh.cpu().numpy().view(np.uint32)

    @staticmethod
    def _raise(st, err):
        if st in (1, 2):
            what = "No edge connecting" if st == 1 else "More than one edge connecting"
            raise NetGraphError(f"{what} node {err.node_a} to {err.node_b}")
        if st == 3:
            raise RoutingPanic(f"assertion failed: paths.len() == nodes.len().pow(2) "
                               f"(no path from node {err.node_a} to {err.node_b})")
        N.check(st, "routing", err)


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

    def latency_ns(self, start: int, end: int):
        """``WorkerShared::latency`` / ``worker_getLatency`` (worker.rs:529-536, 660-670)."""
        p = self.path(start, end)
        return None if p is None else p[0]

    def reliability(self, start: int, end: int):
        """``WorkerShared::reliability`` (worker.rs:538-543): ``1.0f32 - packet_loss``."""
        p = self.path(start, end)
        return None if p is None else np.float32(np.float32(1.0) - p[1])


class IpAssignmentError(Exception):
    """``IpPreviouslyAssignedError`` (graph/mod.rs:343-351) with the caller's context
    (sim_config.rs:407-409)."""


def assign_ips(node_gml_ids, ips=None, host_names=None):
    """``assign_ips`` (sim_config.rs:399-420) over ``IpAssignment`` (graph/mod.rs:354-422), in the
    native host code (``shd_assign_ips``).  ``node_gml_ids[h]`` is host h's network node id (hosts
    in HostId order), ``ips[h]`` its configured IPv4 address as an int (0 / None = none),
    ``host_names[h]`` its name (for the error context; the host's index when absent).
    Returns (ip per host, used node ids ascending = IpAssignment::get_nodes, each host's column
    in that list = the relay's host -> node map)."""
    lib = N.load()
    ids = np.ascontiguousarray(node_gml_ids, np.uint32)
    n = len(ids)
    ip_in = None if ips is None else np.ascontiguousarray([int(x or 0) for x in ips], np.uint32)
    ip_out = np.zeros(n, np.uint32)
    used = np.zeros(max(n, 1), np.uint32)
    col = np.zeros(max(n, 1), np.uint32)
    n_used = C.c_uint32(0)
    bad = C.c_uint32(0)
    st = lib.shd_assign_ips(n, N.ptr(ids), N.ptr(ip_in), N.ptr(ip_out), N.ptr(used), C.byref(n_used),
                            N.ptr(col), C.byref(bad))
    if st == 5 and ip_in is not None and n:
        h = bad.value
        ip = ip_in[h]
        name = host_names[h] if host_names is not None else str(h)
        # anyhow context over IpPreviouslyAssignedError ("{:#}"): the reference's two messages
        raise IpAssignmentError(f"Failed to assign IP address {ip >> 24}.{(ip >> 16) & 255}.{(ip >> 8) & 255}."
                                f"{ip & 255} for host '{name}' to node '{ids[h]}': IP address has already been "
                                f"assigned")
    N.check(st, "shd_assign_ips")
    return ip_out, used[:n_used.value].copy(), col[:n].copy()


def generate_routing_info(graph: NetworkGraph, nodes, use_shortest_paths: bool = True,
                          engine: Engine | None = None) -> RoutingInfo:
    """``generate_routing_info`` (sim_config.rs:424-461): ``nodes`` are GML ids of used nodes."""
    idx = [graph.node_id_to_index(n) for n in nodes]
    table = (graph.compute_shortest_paths(idx, engine) if use_shortest_paths
             else graph.get_direct_paths(idx, engine))
    return RoutingInfo(table)


def load_network_graph(path: str, compression: str | None = None) -> NetworkGraph:
    """``load_network_graph`` (graph/mod.rs:481-511) + ``NetworkGraph::parse`` for a GML file
    source, natively (``shd_gml_load``): ``compression="xz"`` (the reference's
    ``compression: xz``, read_xz :482-494) decompresses through the system liblzma; the text must
    be strict UTF-8 (``String::from_utf8``)."""
    lib = N.load()
    h = C.c_void_p()
    msg = C.create_string_buffer(1024)
    st = lib.shd_gml_load(path.encode(), 1 if compression == "xz" else 0, C.byref(h), msg, len(msg))
    if st != N.SHD_OK:
        text = msg.value.decode("utf-8", "replace")
        if N.STATUS_NAMES.get(st) == "LATENCY_OVERFLOW":
            raise RoutingPanic(text)
        raise NetGraphError(text)
    return NetworkGraph._from_handle(lib, h)
