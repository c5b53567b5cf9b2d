"""GPU parity tests of the routing build: HIP engine vs golden fixtures and the CPU oracle.
Bit-exact latencies and loss bits; error codes and the GML ids they name."""
import json
import os

import numpy as np
import pytest

from oracle import corc
from tests.graphs import KAT_SHORTEST_PATH, engine_graph_from_edges, engine_graph_from_gml, random_graph

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
ALGOS = [0, 1, 2, 3, 4]


def _graph(case):
    from shadow_amd.routing import NetworkGraph
    return NetworkGraph(case["node_ids"], case["src"], case["dst"], case["lat"],
                        np.asarray(case["loss_bits"], np.uint32).view(np.float32), case["directed"])


def _assert_table(t, lat, loss_bits):
    assert np.array_equal(t.lat, np.asarray(lat, np.uint64))
    assert np.array_equal(t.loss.view(np.uint32), np.asarray(loss_bits, np.uint32))


@pytest.mark.parametrize("directed", [True, False])
def test_reference_kat_shortest_path(engine, directed):
    """The reference's own test_shortest_path (graph/mod.rs:562-649) through the engine."""
    g = engine_graph_from_gml(KAT_SHORTEST_PATH.format(directed=int(directed)))
    n0, n1, n2 = (g.node_id_to_index(i) for i in (0, 1, 2))
    sp = g.compute_shortest_paths([n0, n1, n2], engine)
    lat = lambda a, b: sp[(a, b)][0]  # noqa: E731
    assert lat(n0, n0) == 3333 and lat(n1, n1) == 5555 and lat(n2, n2) == 7777
    assert lat(n0, n1) == 3 and lat(n0, n2) == 7
    if directed:
        assert (lat(n1, n0), lat(n1, n2), lat(n2, n0), lat(n2, n1)) == (5, 12, 16, 11)
    else:
        assert (lat(n1, n0), lat(n1, n2), lat(n2, n0), lat(n2, n1)) == (3, 10, 7, 10)


@pytest.mark.parametrize("algo", ALGOS)
def test_golden_routing_cases(engine, algo):
    from shadow_amd.routing import NetGraphError, RoutingPanic
    for case in json.load(open(os.path.join(GOLD, "routing_cases.json"))):
        g = _graph(case)
        exp = case["expect"]
        build = (lambda: g.compute_shortest_paths(case["used"], engine, algo=algo)) \
            if case["mode"] == "shortest" else (lambda: g.get_direct_paths(case["used"], engine))
        if exp["status"] == "OK":
            _assert_table(build(), exp["lat"], exp["loss_bits"])
        elif exp["status"] == "UNREACHABLE":
            with pytest.raises(RoutingPanic, match=f"node {exp['a']} to {exp['b']}"):
                build()
        else:
            word = "No edge" if exp["status"] == "NO_EDGE" else "More than one edge"
            with pytest.raises(NetGraphError, match=f"{word} connecting node {exp['a']} to {exp['b']}"):
                build()


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("algo", ALGOS)
def test_random_graphs_vs_c_oracle(engine, seed, algo):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(2, 300))
    ids, s, d, l, p, directed = random_graph(rng, n, float(rng.uniform(0.005, 0.3)), bool(seed % 2),
                                             max_ms=int(rng.integers(2, 50)))
    n_used = int(rng.integers(1, n + 1))
    used = rng.choice(n, size=n_used, replace=False).astype(np.uint32)
    code, lat, loss, _ = corc.routing(n, s, d, l, p, directed, used)
    assert code == "OK"
    from shadow_amd.routing import NetworkGraph
    t = NetworkGraph(ids, s, d, l, p, directed).compute_shortest_paths(used, engine, algo=algo)
    _assert_table(t, lat, loss.view(np.uint32))


@pytest.mark.parametrize("algo", [0, 4])
def test_wide_latency_fallback(engine, algo):
    """Path latencies >= 2^32 ns take the u64 kernels; still bit-exact."""
    rng = np.random.default_rng(7)
    ids, s, d, l, p, directed = random_graph(rng, 60, 0.05, False)
    l = (l // np.uint64(1_000_000)) * np.uint64(900_000_000)   # up to 18 s per edge
    used = np.arange(60, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(60, s, d, l, p, directed, used)
    assert code == "OK" and lat.max() > 2**32
    from shadow_amd.routing import NetworkGraph
    t = NetworkGraph(ids, s, d, l, p, directed).compute_shortest_paths(used, engine, algo=algo)
    _assert_table(t, lat, loss.view(np.uint32))
    assert engine.last_info()["wide_latency"] == 1


@pytest.fixture(scope="module")
def c2_case():
    from shadow_amd import synth
    el = synth.complete_graph(1000, 1)
    used = np.arange(1000, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(1000, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    return el, used, lat, loss


@pytest.mark.parametrize("algo", ALGOS)
def test_c2_full_bit_exact(engine, c2_case, algo):
    """BASELINE config 2 (1k-node complete graph) against the C restatement."""
    el, used, lat, loss = c2_case
    t = engine_graph_from_edges(el).compute_shortest_paths(used, engine, algo=algo)
    _assert_table(t, lat, loss.view(np.uint32))
    assert engine.smallest_latency_ns() == int(lat.min())


@pytest.mark.parametrize("group", ["", "8", "4"])
def test_c2_repeated_runs_bit_exact(engine, c2_case, group, knob):
    """Prepare once, run several builds: from the second on the engine knows the pruned arc count,
    so AUTO picks the padded-list kernel (sssp_lds_group<..., 8>) -- the C2 headline kernel, which
    a single shd_routing_build never reaches (its first run sizes the lane groups on the unpruned
    degree).  Every build against the C restatement; also with the lane-group width forced."""
    import ctypes as C

    import torch

    from shadow_amd import _native as N
    if group:
        knob("SSSP_G", int(group))
    # the dense-CSR prune (no dense_build) and the dense_build one
    knob("PRUNE_DENSE_BUILD", 1 if group == "4" else 0)
    el, used, lat, loss = c2_case
    g = engine_graph_from_edges(el)._cgraph()
    err = N.Error()
    N.check(engine.lib.shd_routing_prepare(engine.ctx, C.byref(g), N.ptr(used), len(used), N.ROUTE_SHORTEST,
                                           C.byref(err)), "prepare", err)
    n = len(used)
    dl = torch.empty((n, n), dtype=torch.int64, device="cuda")
    dp = torch.empty((n, n), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for _ in range(3):
        N.check(engine.lib.shd_routing_run(engine.ctx, N.ALGO_AUTO, 0, n, N.ptr(dl), N.ptr(dp), C.byref(err)),
                "shd_routing_run", err)
        assert engine.last_info()["algo_used"] == N.ALGO_PRUNED
        assert np.array_equal(dl.cpu().numpy().view(np.uint64), lat)
        assert np.array_equal(dp.cpu().numpy().view(np.uint32), loss.view(np.uint32))


def test_c3_rows_bit_exact(engine):
    """BASELINE config 3 (10k-node BA graph): a row slice against the C restatement."""
    from shadow_amd import synth
    el = synth.barabasi_albert(10_000, 3, 2)
    used = np.arange(10_000, dtype=np.uint32)
    rows = used[:64]
    code, lat, loss, _ = corc.routing(10_000, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    g = engine_graph_from_edges(el)
    for algo in (1, 3, 4):
        t = g.compute_shortest_paths(used, engine, algo=algo, rows=(0, 64))
        _assert_table(t, lat[:64], loss[:64].view(np.uint32))
        t = g.compute_shortest_paths(used, engine, algo=algo, rows=(5000, 5100))
        _assert_table(t, lat[5000:5100], loss[5000:5100].view(np.uint32))
    del rows


@pytest.mark.parametrize("spread", [1, 0])
def test_c3_spread_order_used_subset(engine, knob, spread):
    """The 1024-thread LDS kernel on its wave-spread relabelled CSR (prepare_spread, default for
    C3-like graphs) against the C restatement, with a used set that is neither every node nor in
    index order, so the relabelled ids of the used columns carry the table's column order."""
    from shadow_amd import synth
    el = synth.barabasi_albert(10_000, 3, 2)
    used = np.random.default_rng(3).permutation(10_000)[:7_000].astype(np.uint32)
    knob("SSSP_NO_SPREAD", 1 - spread)
    g = engine_graph_from_edges(el)
    for lo, hi in ((0, 64), (6_900, 7_000)):
        code, lat, loss, _ = corc.routing(10_000, el.src, el.dst, el.latency_ns, el.packet_loss, False, used,
                                          rows=(lo, hi))
        assert code == "OK"
        for algo in (0, 1):
            t = g.compute_shortest_paths(used, engine, algo=algo, rows=(lo, hi))
            _assert_table(t, lat, loss.view(np.uint32))


def test_direct_paths_c2(engine):
    from shadow_amd import synth
    el = synth.complete_graph(300, 9)
    used = np.random.default_rng(1).permutation(300).astype(np.uint32)
    code, lat, loss, _ = corc.routing(300, el.src, el.dst, el.latency_ns, el.packet_loss, False, used,
                                      shortest=False)
    assert code == "OK"
    t = engine_graph_from_edges(el).get_direct_paths(used, engine)
    _assert_table(t, lat, loss.view(np.uint32))


def test_row_shards_concatenate(engine):
    from shadow_amd import synth
    el = synth.complete_graph(257, 3)
    used = np.arange(257, dtype=np.uint32)
    g = engine_graph_from_edges(el)
    full = g.compute_shortest_paths(used, engine)
    parts = [g.compute_shortest_paths(used, engine, rows=(a, min(a + 64, 257))) for a in range(0, 257, 64)]
    assert np.array_equal(np.concatenate([p.lat for p in parts]), full.lat)
    assert np.array_equal(np.concatenate([p.loss for p in parts]).view(np.uint32), full.loss.view(np.uint32))


@pytest.mark.parametrize("algo", ALGOS)
def test_negative_zero_loss_and_parallel_edges(engine, algo):
    """'packet_loss -0.0' passes the reference's range check; parallel arcs of equal latency."""
    rng = np.random.default_rng(42)
    ids, s, d, l, p, directed = random_graph(rng, 80, 0.3, False, max_ms=6)
    k = len(s) // 3
    s = np.concatenate([s, s[:k]]); d = np.concatenate([d, d[:k]])
    l = np.concatenate([l, l[:k]]); p = np.concatenate([p, rng.uniform(0, 0.3, k).astype(np.float32)])
    p[rng.random(len(p)) < 0.2] = np.float32(-0.0)
    loops = s == d
    keep = ~loops | (np.cumsum(loops) <= 80)          # exactly one self-loop per node
    s, d, l, p = s[keep], d[keep], l[keep], p[keep]
    used = np.arange(80, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(80, s, d, l, p, directed, used)
    assert code == "OK"
    from shadow_amd.routing import NetworkGraph
    t = NetworkGraph(ids, s, d, l, p, directed).compute_shortest_paths(used, engine, algo=algo)
    _assert_table(t, lat, loss.view(np.uint32))


def test_blocked_closure_padding_and_directed(engine):
    """Blocked min-plus on sizes that are not tile multiples (padding rows/columns), directed
    graphs, and both tile shapes; the closure time is reported."""
    from shadow_amd.routing import NetworkGraph
    for n, tile, directed in ((65, "64", True), (200, "128", False), (130, "64", False)):
        rng = np.random.default_rng(n)
        ids, s, d, l, p, _ = random_graph(rng, n, 0.08, directed, max_ms=20)
        used = rng.permutation(n).astype(np.uint32)
        code, lat, loss, _ = corc.routing(n, s, d, l, p, directed, used)
        assert code == "OK"
        engine.set_knob("FW_TILE", int(tile))
        try:
            t = NetworkGraph(ids, s, d, l, p, directed).compute_shortest_paths(used, engine, algo=4)
        finally:
            engine.set_knob("FW_TILE", None)
        _assert_table(t, lat, loss.view(np.uint32))
        info = engine.last_info()
        assert info["algo_used"] == 4 and info["ms_minplus"] > 0


@pytest.mark.parametrize("algo", [1, 3])
def test_global_label_kernel_large_graph(engine, algo):
    """V = 25k nodes: 8-byte labels no longer fit the LDS, so the global-label kernel runs.
    200 used nodes spread over the graph; every pair against the C restatement."""
    from shadow_amd import synth
    el = synth.barabasi_albert(25_000, 2, 17)
    used = np.random.default_rng(5).choice(25_000, size=200, replace=False).astype(np.uint32)
    code, lat, loss, _ = corc.routing(25_000, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    t = engine_graph_from_edges(el).compute_shortest_paths(used, engine, algo=algo)
    _assert_table(t, lat, loss.view(np.uint32))


def _tie_heavy_ba(n, m, seed, directed):
    """BA graph with integer-ms latencies in [1, 6] (many equal-latency paths, so the loss
    tie-break decides); directed: every undirected edge becomes two arcs with their own draws."""
    from shadow_amd import synth
    el = synth.barabasi_albert(n, m, seed)
    rng = np.random.default_rng(seed + 100)
    s, d = el.src.copy(), el.dst.copy()
    if directed:
        keep = s != d
        s = np.concatenate([s, d[keep]])
        d = np.concatenate([d, el.src[keep]])
    lat = rng.integers(1, 7, size=len(s)).astype(np.uint64) * np.uint64(1_000_000)
    loss = rng.uniform(0, 0.2, size=len(s)).astype(np.float32)
    loss[rng.random(len(s)) < 0.1] = np.float32(0.0)
    return el.node_ids, s, d, lat, loss, directed


@pytest.mark.parametrize("directed", [False, True])
@pytest.mark.parametrize("slots", ["2", "1"])
def test_global_label_kernel_claimed_rows(engine, directed, slots, knob):
    """Every row of a 3,000-node tie-heavy graph on the persistent global-label kernel, built as
    C4 is (locality order + LDS labels for the hubs, SHD_SSSP_REORDER=1).  The grid holds
    slots x n_cu (256 CUs: 512 or 256) slots, so rows past it -- most of the table -- are taken
    from the row counter (sssp_global_group's dynamic claiming), and every one of them is compared
    against the C restatement (graph/mod.rs:185-230)."""
    from shadow_amd.routing import NetworkGraph
    knob("SSSP_GLOBAL", 1)
    knob("SSSP_REORDER", 1)
    knob("SSSP_SLOTS", int(slots))
    n = 3000
    ids, s, d, l, p, directed = _tie_heavy_ba(n, 3, 31 + int(slots), directed)
    used = np.arange(n, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(n, s, d, l, p, directed, used)
    assert code == "OK"
    g = NetworkGraph(ids, s, d, l, p, directed)
    for algo in (1, 3):
        t = g.compute_shortest_paths(used, engine, algo=algo)
        assert engine.last_info()["algo_used"] == algo
        _assert_table(t, lat, loss.view(np.uint32))


@pytest.mark.parametrize("reserve", [32, 255])
def test_global_label_kernel_claimed_rows_reserved_slots(engine, knob, reserve):
    """The grid every C4 build at N >= 2 runs from its second chunk on (shd_routing_run_sharded
    leaves SHD_SHARD_RESERVE_SLOTS = 32 slots unlaunched while the previous chunk is exchanged):
    2 x n_cu - reserve slots (capped at half), so the row counter hands out more rows per slot.
    Every row of a 3,000-node tie-heavy graph against the C restatement."""
    from shadow_amd.routing import NetworkGraph
    knob("SSSP_GLOBAL", 1)
    knob("SSSP_REORDER", 1)
    knob("SSSP_RESERVE", reserve)
    n = 3000
    ids, s, d, l, p, directed = _tie_heavy_ba(n, 3, 57, False)
    used = np.random.default_rng(11).permutation(n).astype(np.uint32)
    code, lat, loss, _ = corc.routing(n, s, d, l, p, directed, used)
    assert code == "OK"
    t = NetworkGraph(ids, s, d, l, p, directed).compute_shortest_paths(used, engine, algo=3)
    assert engine.last_info()["algo_used"] == 3
    _assert_table(t, lat, loss.view(np.uint32))


def test_global_label_kernel_claimed_rows_sub_range(engine, knob):
    """A row range that does not start at 0 (a rank's shard): claimed rows are offset by
    row_begin + grid, so rows [1000, 2900) of a 3,000-node graph, every one compared."""
    from shadow_amd.routing import NetworkGraph
    knob("SSSP_GLOBAL", 1)
    knob("SSSP_REORDER", 1)
    n = 3000
    ids, s, d, l, p, directed = _tie_heavy_ba(n, 2, 77, False)
    used = np.random.default_rng(3).permutation(n).astype(np.uint32)
    rows = (1000, 2900)
    code, lat, loss, _ = corc.routing(n, s, d, l, p, directed, used, rows=rows)
    assert code == "OK"
    t = NetworkGraph(ids, s, d, l, p, directed).compute_shortest_paths(used, engine, algo=3, rows=rows)
    _assert_table(t, lat, loss.view(np.uint32))


@pytest.mark.parametrize("seed", range(4))
def test_global_label_kernel_forced(engine, seed, knob):
    """The global-label kernel on small tie-heavy graphs (forced with SHD_SSSP_GLOBAL=1)."""
    knob("SSSP_GLOBAL", 1)
    rng = np.random.default_rng(2000 + seed)
    n = int(rng.integers(2, 300))
    ids, s, d, l, p, directed = random_graph(rng, n, float(rng.uniform(0.005, 0.3)), bool(seed % 2),
                                             max_ms=int(rng.integers(2, 50)))
    used = rng.permutation(n).astype(np.uint32)
    code, lat, loss, _ = corc.routing(n, s, d, l, p, directed, used)
    assert code == "OK"
    from shadow_amd.routing import NetworkGraph
    for algo in (1, 3):
        t = NetworkGraph(ids, s, d, l, p, directed).compute_shortest_paths(used, engine, algo=algo)
        _assert_table(t, lat, loss.view(np.uint32))



def _complete(n, mode, seed):
    from shadow_amd import synth
    el = synth.complete_graph(n, seed)
    rng = np.random.default_rng(seed)
    arcs = el.src != el.dst
    if mode == "const":      # every arc ties: each row's boundary bin holds all of it (slow selection)
        el.latency_ns[arcs] = np.uint64(5 * synth.MS)
    elif mode == "few":      # three latencies: heavy ties, > 64 candidates in the boundary bin
        el.latency_ns[arcs] = rng.integers(1, 4, size=int(arcs.sum())).astype(np.uint64) * np.uint64(synth.MS)
    elif mode == "wide":     # ns-granular latencies over four decades (bins from the global max)
        el.latency_ns[arcs] = rng.integers(1_000, 10_000_000, size=int(arcs.sum())).astype(np.uint64)
    return el


@pytest.mark.parametrize("n,mode", [(2, "rand"), (5, "rand"), (33, "rand"), (63, "const"), (64, "few"),
                                    (65, "rand"), (130, "few"), (257, "wide"), (513, "rand"), (777, "few")])
@pytest.mark.parametrize("dense_build", [0, 1])
@pytest.mark.parametrize("shape", [None, 0])
def test_prune_complete_graphs(engine, knob, n, mode, dense_build, shape):
    """The k-nearest 2-hop prune on complete graphs (the dense-CSR and the dense_build inputs)
    against the C restatement: the sorted-detour kernel (default; its fast and slow detour
    selections -- ties put > 64 candidates in the boundary bin) and the round-4 kernel
    (SHD_PRUNE_SHAPE=0); odd sizes exercise the LDS layout's alignment."""
    knob("PRUNE_SHAPE", shape)
    knob("PRUNE_DENSE_BUILD", dense_build)
    el = _complete(n, mode, 11 + n)
    used = np.arange(n, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(n, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    t = engine_graph_from_edges(el).compute_shortest_paths(used, engine, algo=2)
    _assert_table(t, lat, loss.view(np.uint32))
    assert engine.last_info()["algo_used"] == 2


@pytest.mark.parametrize("which", [0, 1, 2])
def test_sssp_kernels_within_register_budget(engine, which):
    """The SSSP kernels sit at the register budgets their residency needs (two 512-thread slots
    per CU for C4's global-label kernel, four 256-thread workgroups for C2's, one 1024-thread
    workgroup for C3's: <= 128 VGPRs each); one register more halves C4's residency (round 5: a
    null check in the shared row code did, C4 rows 0-4095 17.3 -> 27.2 ms)."""
    import ctypes as C
    lib = engine.lib
    lib.shd_debug_kernel_vgprs.restype = C.c_int
    n = lib.shd_debug_kernel_vgprs(which)
    assert 0 < n <= 128, n


@pytest.mark.parametrize("n", [3000, 4096])
def test_prune_large_complete_graph_matches_unpruned(engine, knob, n):
    """The sorted-detour prune at sizes whose LDS stage is ~100-140 KB (3000 nodes, and 4096 =
    kPruneMaxV): its tables against the unpruned LDS engine's (algo 1) on the same graph --
    exact either way."""
    from shadow_amd import synth
    el = synth.complete_graph(n, 5)
    used = np.arange(n, dtype=np.uint32)
    g = engine_graph_from_edges(el)
    ref = g.compute_shortest_paths(used, engine, algo=1)
    knob("PRUNE_SHAPE", None)
    t = g.compute_shortest_paths(used, engine, algo=2)
    assert engine.last_info()["algo_used"] == 2
    assert np.array_equal(t.lat, ref.lat)
    assert np.array_equal(t.loss.view(np.uint32), ref.loss.view(np.uint32))
