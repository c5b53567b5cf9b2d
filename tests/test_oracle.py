"""CPU tests: pin the oracle (test infrastructure) to the reference's known answers, published
algorithm vectors and independent cross-checks; check the committed golden fixtures."""
import itertools
import json
import os

import networkx as nx
import numpy as np
import pytest

from oracle import corc
from oracle import relay as OR
from oracle import rng as RNG
from oracle import routing as R
from oracle.gml import GmlError, ONE_GBIT_SWITCH_GRAPH, decimal_to_f32, parse_network_graph, parse_time
from tests.graphs import KAT_SHORTEST_PATH, random_graph

GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ------------------------------------------------------------------ reference known answers
@pytest.mark.parametrize("directed", [True, False])
def test_kat_shortest_path(directed):
    """graph/mod.rs:562-649 test_shortest_path."""
    g = parse_network_graph(KAT_SHORTEST_PATH.format(directed=int(directed)))
    n0, n1, n2 = (g.id_to_index[i] for i in (0, 1, 2))
    sp = R.compute_shortest_paths(g, [n0, n1, n2])
    lat = lambda a, b: sp[(a, b)][0]  # noqa: E731
    if directed:
        want = {(n0, n0): 3333, (n0, n1): 3, (n0, n2): 7, (n1, n0): 5, (n1, n1): 5555,
                (n1, n2): 12, (n2, n0): 16, (n2, n1): 11, (n2, n2): 7777}
    else:
        want = {(n0, n0): 3333, (n0, n1): 3, (n0, n2): 7, (n1, n0): 3, (n1, n1): 5555,
                (n1, n2): 10, (n2, n0): 7, (n2, n1): 10, (n2, n2): 7777}
    for k, v in want.items():
        assert lat(*k) == v


def test_kat_path_add():
    """graph/mod.rs:517-531 test_path_add."""
    p3 = R.path_add((23, np.float32(0.35)), (11, np.float32(0.85)))
    assert p3[0] == 34
    assert abs(p3[1] - 0.9025) < 0.01
    # binary32 bits of the left fold, not a decimal approximation
    assert np.float32(p3[1]).view(np.uint32) == np.float32(
        np.float32(1) - np.float32(np.float32(1) - np.float32(0.35)) * np.float32(np.float32(1) - np.float32(0.85))
    ).view(np.uint32)


@pytest.mark.parametrize("target,ok", [(2, False), (3, True)])
def test_kat_nonexistent_id(target, ok):
    """graph/mod.rs:533-559 test_nonexistent_id."""
    text = f"""graph [
                node [
                  id 1
                ]
                node [
                  id 3
                ]
                edge [
                  source 1
                  target {target}
                  latency "1 ns"
                ]
            ]"""
    if ok:
        parse_network_graph(text)
    else:
        with pytest.raises(GmlError):
            parse_network_graph(text)


def test_kat_units_time():
    """units.rs:584-640 test_parse_string (Time part)."""
    S, M, MS, US = 10**9, 60 * 10**9, 10**6, 10**3
    for txt, want in [("10", (10, S)), ("10 s", (10, S)), ("10s", (10, S)), ("10   s", (10, S)),
                      ("10sec", (10, S)), ("10  m", (10, M)), ("10  min", (10, M)),
                      ("10 ms", (10, MS)), ("10 μs", (10, US)), ("10 millisecond", (10, MS)),
                      ("10 milliseconds", (10, MS))]:
        assert parse_time(txt) == want
    for bad in ("-10 ms", "abc 10 ms", "10.5 ms", "10 abc"):
        with pytest.raises(GmlError):
            parse_time(bad)


def test_gml_value_rules():
    base = """graph [
  node [
    id 0
  ]
  edge [
    source 0
    target 0
    latency "1 ms"
{extra}  ]
]"""
    g = parse_network_graph(base.format(extra=""))
    assert g.edges[0].packet_loss == np.float32(0.0) and g.edges[0].latency_ns == 10**6
    with pytest.raises(GmlError, match="not a float"):       # ints are tried before floats
        parse_network_graph(base.format(extra="    packet_loss 0\n"))
    with pytest.raises(GmlError, match="range"):
        parse_network_graph(base.format(extra="    packet_loss 1.5\n"))
    with pytest.raises(GmlError, match="must not be 0"):
        parse_network_graph(base.replace('"1 ms"', '"0 ms"').format(extra=""))
    g = parse_network_graph(base.format(extra="    packet_loss 0.1\n    jitter \"5 ms\"\n"))
    assert g.edges[0].packet_loss == np.float32(0.1)
    g = parse_network_graph(ONE_GBIT_SWITCH_GRAPH)
    assert g.edges[0].latency_ns == 10**6 and not g.directed


def test_decimal_to_f32_correct_rounding():
    rng = np.random.default_rng(5)
    for _ in range(2000):
        x = float(rng.uniform(0, 1))
        s = repr(x)
        assert decimal_to_f32(s) == np.float32(x) or abs(float(decimal_to_f32(s)) - x) <= abs(float(np.float32(x)) - x)
    # a value whose f64 rounding lands on an f32 tie (double rounding would differ)
    assert decimal_to_f32("1.00000005960464477539062500001").view(np.uint32) == 0x3F800001
    assert decimal_to_f32("0.25") == np.float32(0.25)


# ------------------------------------------------------------------ independent cross-checks
def _oracle_graph(arr):
    from tests.golden.make_golden import to_oracle_graph
    return to_oracle_graph(*arr)


@pytest.mark.parametrize("seed", range(8))
def test_latency_matches_networkx(seed):
    rng = np.random.default_rng(seed)
    arr = random_graph(rng, int(rng.integers(3, 30)), 0.3, bool(seed % 2))
    g = _oracle_graph(arr)
    ids, s, d, l, p, directed = arr
    G = nx.DiGraph() if directed else nx.Graph()
    G.add_nodes_from(range(len(ids)))
    for a, b, w in zip(s, d, l):
        if a == b:
            continue
        if G.has_edge(int(a), int(b)):
            w = min(int(w), G[int(a)][int(b)]["weight"])
        G.add_edge(int(a), int(b), weight=int(w))
    used = list(range(len(ids)))
    sp = R.compute_shortest_paths(g, used)
    dist = dict(nx.all_pairs_dijkstra_path_length(G))
    for a in used:
        for b in used:
            if a != b:
                assert sp[(a, b)][0] == dist[a][b]


@pytest.mark.parametrize("seed", range(10))
def test_loss_matches_bruteforce_simple_paths(seed):
    """Lexicographic min over all simple paths of the left-fold cost (walks never win)."""
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(3, 7))
    arr = random_graph(rng, n, 0.6, bool(seed % 2), max_ms=4, loss_max=0.6)
    g = _oracle_graph(arr)
    adj = R.adjacency(g)
    sp = R.compute_shortest_paths(g, list(range(n)))

    def best(src, dst):
        out = None
        stack = [(src, (0, np.float32(0.0)), {src})]
        while stack:
            u, cost, seen = stack.pop()
            if u == dst:
                out = cost if out is None or cost < out else out
                continue
            for v, el, ep in adj[u]:
                if v not in seen:
                    stack.append((v, (cost[0] + el, R.fold(cost[1], ep)), seen | {v}))
        return out

    for a, b in itertools.product(range(n), repeat=2):
        if a != b:
            want = best(a, b)
            got = sp[(a, b)]
            assert got[0] == want[0] and np.float32(got[1]).view(np.uint32) == np.float32(want[1]).view(np.uint32)


def test_left_fold_is_not_segment_composition():
    """composing segments differs from the left fold, so FW loss would be wrong."""
    rng = np.random.default_rng(0)
    e = rng.uniform(0, 0.05, size=(20000, 3)).astype(np.float32)
    left = [R.fold(R.fold(R.fold(np.float32(0), a), b), c) for a, b, c in e[:2000]]
    comp = [R.fold(R.fold(R.fold(np.float32(0), a), np.float32(0)), R.fold(R.fold(np.float32(0), b), c))
            for a, b, c in e[:2000]]
    assert sum(x != y for x, y in zip(left, comp)) > 100


# ------------------------------------------------------------------ RNG vectors
def test_rng_published_vectors():
    # SipHash-2-4 reference vectors (key 00..0f), the core shared with SipHash-1-3
    k0, k1 = 0x0706050403020100, 0x0F0E0D0C0B0A0908
    assert RNG.siphash(b"", k0, k1, 2, 4) == 0x726FDB47DD0E0E31
    assert RNG.siphash(bytes([0]), k0, k1, 2, 4) == 0x74F839C593DC67FD
    # rand_xoshiro Xoshiro256PlusPlus reference test (seed state [1,2,3,4])
    x = RNG.Xoshiro256PlusPlus([1, 2, 3, 4])
    assert [x.next_u64() for _ in range(10)] == [
        41943041, 58720359, 3588806011781223, 3591011842654386, 9228616714210784205,
        9973669472204895162, 14011001112246962877, 12406186145184390807,
        15849039046786891736, 10450023813501588000]
    # rand_xoshiro SplitMix64 reference test
    s = RNG.SplitMix64(1477776061723855037)
    assert [s.next_u64() for _ in range(4)] == [1985237415132408290, 2979275885539914483,
                                                 13511426838097143398, 8488337342461049707]


def test_rng_golden_fixture_reproduces():
    gold = json.load(open(os.path.join(GOLD, "rng_vectors.json")))
    for seed, v in gold["xoshiro_from_seed"].items():
        x = RNG.Xoshiro256PlusPlus.seed_from_u64(int(seed))
        assert [str(a) for a in x.state()] == v["state"]
        assert [str(x.next_u64()) for _ in range(8)] == v["next"]
    for gs, names in gold["host_seed"].items():
        for nm, want in names.items():
            assert str(RNG.host_seed(int(gs), nm)) == want


def test_synth_host_rng_matches_oracle():
    from shadow_amd import synth
    st = synth.host_rng_states(300, global_seed=3)
    for h in (0, 7, 299):
        assert [int(v) for v in st[h]] == RNG.host_rng_state(3, f"host{h:06d}")


# ------------------------------------------------------------------ golden fixtures
def test_routing_golden_reproduces():
    from tests.golden.make_golden import routing_cases
    assert routing_cases() == json.load(open(os.path.join(GOLD, "routing_cases.json")))


def test_relay_golden_reproduces():
    from tests.golden.make_golden import relay_cases
    assert relay_cases() == json.load(open(os.path.join(GOLD, "relay_cases.json")))


# ------------------------------------------------------------------ C restatement == Python
@pytest.mark.parametrize("seed", range(6))
def test_c_oracle_routing_matches_python(seed):
    rng = np.random.default_rng(300 + seed)
    arr = random_graph(rng, int(rng.integers(2, 40)), 0.3, bool(seed % 2))
    ids, s, d, l, p, directed = arr
    used = list(range(len(ids)))
    lat, loss = R.table(R.compute_shortest_paths(_oracle_graph(arr), used), used)
    for variant in (corc.TIDY, corc.FAITHFUL):
        code, clat, closs, _ = corc.routing(len(ids), s, d, l, p, directed, used, variant=variant)
        assert code == "OK"
        assert np.array_equal(clat, lat)
        assert np.array_equal(closs.view(np.uint32), loss.view(np.uint32))


def test_c_oracle_errors_match_python():
    for case in json.load(open(os.path.join(GOLD, "routing_cases.json"))):
        ids = np.asarray(case["node_ids"], np.uint32)
        loss = np.asarray(case["loss_bits"], np.uint32).view(np.float32)
        code, lat, lo, (a, b) = corc.routing(len(ids), case["src"], case["dst"], case["lat"], loss,
                                             case["directed"], case["used"],
                                             shortest=case["mode"] == "shortest")
        exp = case["expect"]
        assert code == exp["status"], case["name"]
        if code == "OK":
            assert lat.tolist() == exp["lat"], case["name"]
            assert lo.view(np.uint32).tolist() == exp["loss_bits"], case["name"]
        else:
            assert (int(ids[a]), int(ids[b])) == (exp["a"], exp["b"]), case["name"]


def test_c_oracle_relay_matches_golden():
    for case in json.load(open(os.path.join(GOLD, "relay_cases.json"))):
        rng_state = np.asarray([[int(v) for v in r] for r in case["rng"]], np.uint64).reshape(-1, 4)
        nid = np.asarray([int(v) for v in case["next_id"]], np.uint64)
        loss = np.asarray(case["loss_bits"], np.uint32).view(np.float32)
        r = corc.relay_round(np.asarray(case["src_off"], np.uint32),
                             np.asarray([int(v) for v in case["send_time"]], np.uint64),
                             np.asarray(case["dst_host"], np.uint32), np.asarray(case["payload"], np.uint32),
                             np.asarray(case["host_node"], np.uint32), np.asarray(case["lat"], np.uint64),
                             loss, rng_state, nid, int(case["round_end"]), int(case["sim_end"]),
                             int(case["bootstrap_end"]))
        e = case["expect"]
        assert r["status"].tolist() == e["status"], case["name"]
        ev = r["events"]
        assert ev["off"].tolist() == e["ev_off"]
        got = [[str(t), int(s), str(q), int(pk)] for t, s, q, pk in
               zip(ev["deliver"].tolist(), ev["src"].tolist(), ev["seq"].tolist(), ev["pkt"].tolist())]
        assert got == e["ev"], case["name"]
        assert str(r["min_deliver"]) == e["min_deliver"] and str(r["min_latency"]) == e["min_latency"]
        assert [[str(v) for v in row] for row in rng_state.tolist()] == e["rng"]
        assert [str(v) for v in nid.tolist()] == e["next_id"]


def test_relay_window_helpers():
    assert OR.next_window(100, 10, 1000) == (100, 110)
    assert OR.next_window(995, 10, 1000) == (995, 1000)
    assert OR.next_window(1000, 10, 1000) is None
    assert OR.runahead(None, 5, 1_000_000) == 1_000_000
    assert OR.runahead(2_000_000, 5, 1_000_000) == 2_000_000


@pytest.mark.parametrize("seed", range(4))
def test_c_oracle_row_range_matches_full(seed):
    """orc_shortest_paths_rows (the checker for C4 row slices) against the full build."""
    rng = np.random.default_rng(300 + seed)
    n = int(rng.integers(20, 200))
    ids, s, d, l, p, directed = random_graph(rng, n, 0.08, bool(seed % 2), max_ms=20)
    used = rng.permutation(n).astype(np.uint32)
    code, lat, loss, _ = corc.routing(n, s, d, l, p, directed, used)
    assert code == "OK"
    for rb, re in ((0, 1), (3, 17), (n - 5, n)):
        for variant in (corc.TIDY, corc.FAITHFUL):
            c2, l2, p2, _ = corc.routing(n, s, d, l, p, directed, used, variant=variant, rows=(rb, re))
            assert c2 == "OK"
            assert np.array_equal(l2, lat[rb:re])
            assert np.array_equal(p2.view(np.uint32), loss[rb:re].view(np.uint32))


@pytest.mark.parametrize("seed", range(4))
def test_native_assign_ips_matches_ip_assignment(seed):
    """shd_assign_ips (host code) against the IpAssignment restatement (graph/mod.rs:354-422,
    sim_config.rs:399-420): configured addresses first, then 11.0.0.1.. skipping .0/.255 and
    every address already taken."""
    from shadow_amd.routing import IpAssignmentError, assign_ips
    rng = np.random.default_rng(40 + seed)
    n = int(rng.integers(1, 700))
    ids = rng.choice([3, 7, 11, 200, 4096, 99999], size=n).astype(np.uint32)
    ips = [0] * n
    k = n // 4
    picks = rng.choice(np.arange(1, 600), size=k, replace=seed % 2 == 1)   # odd seeds: repeats
    for h, a in zip(rng.choice(n, size=k, replace=False), picks):
        ips[h] = (11 << 24) + int(a)      # inside the automatic range: assign() must skip them
    o = R.IpAssignment()
    want = [0] * n
    dup = None
    for h in range(n):
        if ips[h]:
            try:
                o.assign_ip(int(ids[h]), ips[h])
                want[h] = ips[h]
            except R.RoutingError:
                dup = h
                break
    if dup is not None:
        with pytest.raises(IpAssignmentError, match="already been assigned"):
            assign_ips(ids, ips)
        ip = ips[dup]
        names = [f"host{h}" for h in range(n)]
        want_msg = (f"Failed to assign IP address 11.{(ip >> 16) & 255}.{(ip >> 8) & 255}.{ip & 255} for host "
                    f"'host{dup}' to node '{ids[dup]}': IP address has already been assigned")
        with pytest.raises(IpAssignmentError) as e:   # sim_config.rs:407-409 context + graph/mod.rs:349
            assign_ips(ids, ips, host_names=names)
        assert str(e.value) == want_msg
        return
    for h in range(n):
        if not ips[h]:
            want[h] = o.assign(int(ids[h]))
    ip_out, used, col = assign_ips(ids, ips)
    assert ip_out.tolist() == want
    assert all((ip & 0xFF) not in (0, 255) for ip in ip_out.tolist())
    assert used.tolist() == sorted(o.get_nodes())
    assert np.array_equal(used[col], ids)
