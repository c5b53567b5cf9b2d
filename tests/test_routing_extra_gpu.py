"""GPU tests of the routing build's remaining interfaces:
  * next hops (north star; the reference keeps none) against the C oracle's
    restatement of the engine's definition (lowest-index tight predecessor chain), every engine,
    tie-heavy graphs, the wide-latency path, direct mode and used-node subsets;
  * generate_routing_info (sim_config.rs:424-461) over the native assign_ips / IpAssignment
    (sim_config.rs:399-420, graph/mod.rs:354-422), keyed by GML ids, against the Python
    restatement of compute_shortest_paths;
  * RoutingInfo::path / worker_getLatency lookups on the resident table (shd_routing_lookup,
    graph/mod.rs:446-448, worker.rs:660-670) and get_smallest_latency_ns (graph/mod.rs:476-478).
"""
import ctypes as C

import numpy as np
import pytest

from oracle import corc
from oracle import routing as R
from oracle.gml import parse_network_graph
from tests.graphs import engine_graph_from_edges, gml_text, random_graph

pytestmark = pytest.mark.gpu


def _oracle_nh(n, s, d, l, p, directed, used, shortest=True):
    code, lat, loss, _ = corc.routing(n, s, d, l, p, directed, used, shortest=shortest)
    assert code == "OK"
    return lat, loss, corc.next_hops(n, s, d, l, p, directed, used, lat, loss)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("algo", [0, 1, 2, 3, 4])
def test_next_hops_random_graphs(engine, seed, algo):
    from shadow_amd.routing import NetworkGraph
    rng = np.random.default_rng(5000 + seed)
    n = int(rng.integers(2, 250))
    ids, s, d, l, p, directed = random_graph(rng, n, float(rng.uniform(0.01, 0.3)), bool(seed % 2),
                                             max_ms=int(rng.integers(2, 12)))
    used = rng.permutation(n).astype(np.uint32)
    lat, loss, nh = _oracle_nh(n, s, d, l, p, directed, used)
    t, gnh = NetworkGraph(ids, s, d, l, p, directed).compute_next_hops(used, engine, algo=algo)
    assert np.array_equal(t.lat, lat)
    assert np.array_equal(t.loss.view(np.uint32), loss.view(np.uint32))
    assert np.array_equal(gnh, nh)
    # every next hop is a neighbour of the source (an arc s -> hop exists)
    arcs = set(zip(s.tolist(), d.tolist())) | (set() if directed else set(zip(d.tolist(), s.tolist())))
    for i in range(0, n, max(1, n // 7)):
        src = int(used[i])
        for j in range(n):
            h = int(gnh[i, j])
            assert h == src if int(used[j]) == src else (src, h) in arcs


def test_next_hops_c2_rows_and_subset(engine):
    """C2 (1k-node complete graph, pruned engine) rows; a used subset gives the same hops as the
    full build's columns (labels do not depend on the used set)."""
    from shadow_amd import synth
    el = synth.complete_graph(1000, 1)
    used = np.arange(1000, dtype=np.uint32)
    lat, loss, nh = _oracle_nh(1000, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    g = engine_graph_from_edges(el)
    t, gnh = g.compute_next_hops(used, engine)
    assert np.array_equal(gnh, nh) and np.array_equal(t.lat, lat)
    sub = np.random.default_rng(2).choice(1000, size=300, replace=False).astype(np.uint32)
    _, snh = g.compute_next_hops(sub, engine)
    assert np.array_equal(snh, nh[np.ix_(sub, sub)])


def test_next_hops_wide_and_direct(engine):
    from shadow_amd import synth
    from shadow_amd.routing import NetworkGraph
    rng = np.random.default_rng(7)
    ids, s, d, l, p, directed = random_graph(rng, 60, 0.05, False)
    l = (l // np.uint64(1_000_000)) * np.uint64(900_000_000)   # paths >= 2^32 ns: u64 kernels
    used = np.arange(60, dtype=np.uint32)
    lat, loss, nh = _oracle_nh(60, s, d, l, p, directed, used)
    t, gnh = NetworkGraph(ids, s, d, l, p, directed).compute_next_hops(used, engine)
    assert engine.last_info()["wide_latency"] == 1
    assert np.array_equal(t.lat, lat) and np.array_equal(gnh, nh)
    el = synth.complete_graph(50, 4)
    used = np.random.default_rng(1).permutation(50).astype(np.uint32)
    t, gnh = engine_graph_from_edges(el).compute_next_hops(used, engine, shortest=False)
    assert np.array_equal(gnh, np.tile(used, (50, 1)))


def test_generate_routing_info_over_ip_assignment(engine):
    """Hosts on a graph with non-contiguous GML ids; some with configured addresses.  The table
    over IpAssignment::get_nodes(), keyed by GML ids, against the restatement."""
    from shadow_amd.routing import NetworkGraph, assign_ips, generate_routing_info
    rng = np.random.default_rng(11)
    n = 40
    ids, s, d, l, p, directed = random_graph(rng, n, 0.1, False, max_ms=9)
    gml_ids = (np.arange(n, dtype=np.uint32) * 7 + 3)           # ids 3, 10, 17, ...
    g = NetworkGraph(gml_ids, s, d, l, p, directed)
    host_node = rng.choice(gml_ids[: n // 2], size=300).astype(np.uint32)   # half the nodes own hosts
    cfg = [0] * 300
    for h in range(0, 300, 17):
        cfg[h] = (10 << 24) | (h + 1)
    ip, used_gml, col = assign_ips(host_node, cfg)
    o = R.IpAssignment()
    for h in range(300):
        if cfg[h]:
            o.assign_ip(int(host_node[h]), cfg[h])
    for h in range(300):
        if not cfg[h]:
            assert o.assign(int(host_node[h])) == int(ip[h])
    assert set(used_gml.tolist()) == o.get_nodes()
    ri = generate_routing_info(g, used_gml.tolist(), True, engine)
    og = parse_network_graph(gml_text(gml_ids, s, d, l, p))
    idx = [og.id_to_index[int(x)] for x in used_gml]
    paths = R.compute_shortest_paths(og, idx)
    for a in used_gml.tolist():
        for b in used_gml.tolist():
            lat_w, loss_w = paths[(og.id_to_index[a], og.id_to_index[b])]
            got = ri.path(a, b)
            assert got[0] == lat_w and np.float32(got[1]).view(np.uint32) == np.float32(loss_w).view(np.uint32)
            assert ri.latency_ns(a, b) == lat_w
    # the relay's host -> node map is the host's column in the used list
    assert np.array_equal(used_gml[col], host_node)
    assert ri.path(gml_ids[-1], gml_ids[0]) is None or gml_ids[-1] in used_gml


def test_resident_table_lookups(engine):
    from shadow_amd import _native as N
    from shadow_amd import synth
    el = synth.barabasi_albert(3000, 2, 5)
    used = np.random.default_rng(4).permutation(3000)[:700].astype(np.uint32)
    code, lat, loss, _ = corc.routing(3000, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    g = engine_graph_from_edges(el)
    g.compute_shortest_paths(used, engine)                    # full build: the table stays resident
    rng = np.random.default_rng(9)
    for _ in range(200):
        i, j = (int(x) for x in rng.integers(0, 700, size=2))
        lv, pv = C.c_uint64(0), C.c_float(0)
        N.check(engine.lib.shd_routing_lookup(engine.ctx, i, j, C.byref(lv), C.byref(pv)), "lookup")
        assert lv.value == int(lat[i, j]) and np.float32(pv.value).view(np.uint32) == loss[i, j].view(np.uint32)
    assert engine.smallest_latency_ns() == int(lat.min())
    st = engine.lib.shd_routing_lookup(engine.ctx, 700, 0, C.byref(C.c_uint64()), C.byref(C.c_float()))
    assert st == 5   # out of range: SHD_ERR_INVALID
    # batched: 100k pairs in one gather
    rows = rng.integers(0, 700, 100_000).astype(np.uint32)
    cols = rng.integers(0, 700, 100_000).astype(np.uint32)
    bl, bp = np.zeros(100_000, np.uint64), np.zeros(100_000, np.float32)
    N.check(engine.lib.shd_routing_lookup_batch(engine.ctx, 100_000, N.ptr(rows), N.ptr(cols), N.ptr(bl), N.ptr(bp)),
            "lookup_batch")
    assert np.array_equal(bl, lat[rows, cols]) and np.array_equal(bp.view(np.uint32), loss[rows, cols].view(np.uint32))
    # the host mirror: single lookups are host reads, identical answers
    N.check(engine.lib.shd_routing_mirror(engine.ctx, 1), "mirror")
    for k in range(0, 100_000, 997):
        lv, pv = C.c_uint64(0), C.c_float(0)
        N.check(engine.lib.shd_routing_lookup(engine.ctx, int(rows[k]), int(cols[k]), C.byref(lv), C.byref(pv)),
                "lookup")
        assert lv.value == int(bl[k]) and np.float32(pv.value).view(np.uint32) == bp[k].view(np.uint32)
    bl2 = np.zeros(100_000, np.uint64)
    N.check(engine.lib.shd_routing_lookup_batch(engine.ctx, 100_000, N.ptr(rows), N.ptr(cols), N.ptr(bl2), None),
            "lookup_batch (mirror)")
    assert np.array_equal(bl2, bl)
    # a new build drops the mirror with the resident table it copied
    g.compute_shortest_paths(used, engine)
    N.check(engine.lib.shd_routing_lookup(engine.ctx, 3, 4, C.byref(lv), C.byref(pv)), "lookup")
    assert lv.value == int(lat[3, 4])
    N.check(engine.lib.shd_routing_mirror(engine.ctx, 0), "mirror off")


def test_kernel_timing_sampling(engine):
    """shd_routing_set_timing: the dominant kernel is timed on every `every`-th build only
    (ms_main = -1 on the others, 0 = never); the tables are the same either way."""
    from shadow_amd import synth
    el = synth.complete_graph(200, 5)
    g = engine_graph_from_edges(el)
    used = np.arange(200, dtype=np.uint32)
    ref = g.compute_shortest_paths(used, engine)
    try:
        engine.lib.shd_routing_set_timing(engine.ctx, 3)
        seen = []
        for _ in range(6):
            t = g.compute_shortest_paths(used, engine)
            seen.append(engine.last_info()["ms_main"])
            assert np.array_equal(t.lat, ref.lat) and np.array_equal(t.loss.view(np.uint32), ref.loss.view(np.uint32))
        assert [m >= 0 for m in seen] == [True, False, False, True, False, False]
        assert all(m > 0 for m in seen[::3])
        engine.lib.shd_routing_set_timing(engine.ctx, 0)
        g.compute_shortest_paths(used, engine)
        assert engine.last_info()["ms_main"] == -1
    finally:
        engine.lib.shd_routing_set_timing(engine.ctx, 1)
