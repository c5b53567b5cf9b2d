"""Generate the committed golden fixtures from the CPU oracle (run in the build container).

    python tests/golden/make_golden.py

Fixtures are data only (inputs + expected outputs).  Routing cases include the reference's own
known-answer graphs (src/main/network/graph/mod.rs:562-649), the built-in 1_gbit_switch graph
(configuration.rs:1314-1327) and the lossy test graph (src/test/tcp/tcp-blocking-lossy.yaml),
all parsed by the oracle GML restatement, plus seeded random graphs with forced ties.
The relay fixtures are parity-unpinned (no reference vector exists): they record the oracle's
restatement of send_packet on seeded batches.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import relay as OR  # noqa: E402
from oracle import rng as RNG  # noqa: E402
from oracle import routing as R  # noqa: E402
from oracle.gml import NetworkGraph, Edge, ONE_GBIT_SWITCH_GRAPH, parse_network_graph  # noqa: E402
from graphs import KAT_SHORTEST_PATH, oracle_graph_arrays, random_graph  # noqa: E402

LOSSY_GRAPH = """graph [
  directed 0
  node [
    id 0
    host_bandwidth_down "81920 Kibit"
    host_bandwidth_up "81920 Kibit"
  ]
  edge [
    source 0
    target 0
    latency "50 ms"
    packet_loss 0.25
  ]
]"""
"""Data from src/test/tcp/tcp-blocking-lossy.yaml:5-19 (inline graph)."""


def f32_bits(a):
    return np.asarray(a, np.float32).view(np.uint32).tolist()


def to_oracle_graph(ids, s, d, l, p, directed):
    edges = [Edge(int(a), int(b), int(x), np.float32(y)) for a, b, x, y in zip(s, d, l, p)]
    return NetworkGraph(directed=bool(directed), node_ids=[int(v) for v in ids], edges=edges,
                        id_to_index={int(v): i for i, v in enumerate(ids)})


def routing_case(name, arrays, used, mode):
    ids, s, d, l, p, directed = arrays
    g = to_oracle_graph(*arrays)
    case = dict(name=name, node_ids=[int(v) for v in ids], src=[int(v) for v in s],
                dst=[int(v) for v in d], lat=[int(v) for v in l], loss_bits=f32_bits(p),
                directed=bool(directed), used=[int(u) for u in used], mode=mode)
    try:
        paths = (R.compute_shortest_paths(g, used) if mode == "shortest"
                 else R.get_direct_paths(g, used))
        lat, loss = R.table(paths, used)
        case["expect"] = dict(status="OK", lat=lat.tolist(), loss_bits=loss.view(np.uint32).tolist())
    except R.RoutingError as e:
        case["expect"] = dict(status=e.code, a=e.a, b=e.b)
    return case


def routing_cases():
    cases = []
    for directed in (1, 0):
        g = parse_network_graph(KAT_SHORTEST_PATH.format(directed=directed))
        cases.append(routing_case(f"kat_shortest_path_directed{directed}", oracle_graph_arrays(g),
                                  [0, 1, 2], "shortest"))
    for name, text in (("one_gbit_switch", ONE_GBIT_SWITCH_GRAPH), ("tcp_lossy", LOSSY_GRAPH)):
        g = parse_network_graph(text)
        for mode in ("shortest", "direct"):
            cases.append(routing_case(f"{name}_{mode}", oracle_graph_arrays(g), [0], mode))
    rng = np.random.default_rng(20241015)
    for k in range(24):
        n = int(rng.integers(2, 25))
        directed = bool(k % 2)
        arr = random_graph(rng, n, float(rng.uniform(0.1, 0.6)), directed)
        n_used = int(rng.integers(1, n + 1))
        used = sorted(rng.choice(n, size=n_used, replace=False).tolist())
        if k % 3 == 0:
            rng.shuffle(used)
        cases.append(routing_case(f"random{k}", arr, used, "shortest"))
    # unused transit nodes, parallel edges with equal latency and different loss
    ids = np.arange(4, dtype=np.uint32)
    s = np.array([0, 1, 2, 3, 0, 1, 0, 2, 0], np.uint32)
    d = np.array([0, 1, 2, 3, 2, 3, 3, 3, 2], np.uint32)
    l = np.array([5, 5, 5, 5, 10, 10, 30, 20, 10], np.uint64)
    p = np.array([0.5, 0, 0.25, 0.1, 0.2, 0.3, 0.0, 0.1, 0.05], np.float32)
    cases.append(routing_case("parallel_edges_transit", (ids, s, d, l, p, False), [0, 1, 3], "shortest"))
    # error cases
    cases.append(routing_case("missing_self_loop", (ids, s[1:], d[1:], l[1:], p[1:], False), [0, 1], "shortest"))
    s2 = np.append(s, 1).astype(np.uint32); d2 = np.append(d, 1).astype(np.uint32)
    l2 = np.append(l, 7).astype(np.uint64); p2 = np.append(p, 0.5).astype(np.float32)
    cases.append(routing_case("two_self_loops", (ids, s2, d2, l2, p2, False), [0, 1, 2], "shortest"))
    s3 = np.array([0, 1, 2, 0], np.uint32); d3 = np.array([0, 1, 2, 1], np.uint32)
    cases.append(routing_case("unreachable", (ids[:3], s3, d3, np.array([1, 1, 1, 4], np.uint64),
                                              np.zeros(4, np.float32), True), [0, 1, 2], "shortest"))
    cases.append(routing_case("unreachable_directed_back", (ids[:3], s3, d3,
                                                            np.array([1, 1, 1, 4], np.uint64),
                                                            np.zeros(4, np.float32), True), [0, 1], "shortest"))
    # direct mode on a small complete graph, and its error cases
    n = 6
    iu, ju = np.triu_indices(n, 1)
    sc = np.concatenate([np.arange(n), iu]).astype(np.uint32)
    dc = np.concatenate([np.arange(n), ju]).astype(np.uint32)
    lc = rng.integers(1, 100, size=len(sc)).astype(np.uint64) * np.uint64(1000)
    pc = rng.uniform(0, 0.1, size=len(sc)).astype(np.float32)
    arr = (np.arange(n, dtype=np.uint32), sc, dc, lc, pc, False)
    cases.append(routing_case("direct_complete", arr, list(range(n)), "direct"))
    cases.append(routing_case("shortest_complete", arr, list(range(n)), "shortest"))
    cases.append(routing_case("direct_missing", (arr[0], sc[:-1], dc[:-1], lc[:-1], pc[:-1], False),
                              list(range(n)), "direct"))
    cases.append(routing_case("direct_multi", (arr[0], np.append(sc, 2).astype(np.uint32),
                                               np.append(dc, 4).astype(np.uint32),
                                               np.append(lc, 5).astype(np.uint64),
                                               np.append(pc, 0).astype(np.float32), False),
                              list(range(n)), "direct"))
    # GML ids that are not 0..n-1 (error messages report GML ids)
    ids_g = np.array([10, 20, 30], np.uint32)
    cases.append(routing_case("gml_ids_missing_loop", (ids_g, np.array([0, 1, 0], np.uint32),
                                                       np.array([0, 1, 2], np.uint32),
                                                       np.array([1, 1, 3], np.uint64),
                                                       np.zeros(3, np.float32), False), [0, 1, 2], "shortest"))
    return cases


def rng_vectors():
    out = {"xoshiro_from_seed": {}, "gen_f64": {}, "host_seed": {}}
    for seed in (0, 1, 2, (1 << 64) - 1):
        x = RNG.Xoshiro256PlusPlus.seed_from_u64(seed)
        out["xoshiro_from_seed"][str(seed)] = {"state": [str(v) for v in x.state()],
                                              "next": [str(x.next_u64()) for _ in range(8)]}
        y = RNG.Xoshiro256PlusPlus.seed_from_u64(seed)
        out["gen_f64"][str(seed)] = [y.gen_f64().hex() for _ in range(8)]
    names = ["host000000", "host000001", "host099999", "lossy.tcpserver.echo",
             "lossy.tcpclient.echo", "server", "client1", ""]
    for gs in (1, 2, 12345):
        out["host_seed"][str(gs)] = {nm: str(RNG.host_seed(gs, nm)) for nm in names}
    return out


def relay_cases():
    from shadow_amd import synth
    cases = []
    rng = np.random.default_rng(77)
    for k in range(6):
        n_nodes = int(rng.integers(2, 12))
        arr = random_graph(rng, n_nodes, 0.5, bool(k % 2), max_ms=5, loss_max=0.5)
        g = to_oracle_graph(*arr)
        used = list(range(n_nodes))
        lat, loss = R.table(R.compute_shortest_paths(g, used), used)
        if k == 2:
            loss[0, 1] = np.float32(1.0)  # always-drop path
        n_hosts = int(rng.integers(2, 60))
        host_node = rng.integers(0, n_nodes, size=n_hosts).astype(np.uint32)
        n_pk = int(rng.integers(0, 3000)) if k else 0
        start = 1_000_000_000
        runahead = 1_000_000
        b = synth.packet_batch(n_hosts, max(n_pk, 1), start, start + runahead, seed=100 + k)
        if n_pk == 0:
            b = synth.PacketBatch(np.zeros(n_hosts + 1, np.uint32), np.zeros(0, np.uint64),
                                  np.zeros(0, np.uint32), np.zeros(0, np.uint32))
        round_end = start + runahead
        sim_end = start + (runahead * 3) // 4 if k == 3 else start + 10 * runahead
        boot_end = start + runahead // 2 if k == 4 else 0
        rng_state = synth.host_rng_states(n_hosts, global_seed=k + 1)
        next_id = rng.integers(0, 1000, size=n_hosts).astype(np.uint64)
        src = np.repeat(np.arange(n_hosts), np.diff(b.src_off)).astype(np.uint32)
        r = OR.relay_round(b.send_time, src, b.dst_host, b.payload, host_node, lat, loss,
                           rng_state, next_id, round_end, sim_end, boot_end)
        ev_off = [0]
        ev = []
        for h in range(n_hosts):
            e = r.events.get(h, [])
            ev.extend(e)
            ev_off.append(len(ev))
        cases.append(dict(
            name=f"relay{k}", n_nodes=n_nodes, lat=lat.tolist(), loss_bits=loss.view(np.uint32).tolist(),
            host_node=host_node.tolist(), rng=[[str(v) for v in row] for row in rng_state.tolist()],
            next_id=[str(v) for v in next_id.tolist()], src_off=b.src_off.tolist(),
            send_time=[str(v) for v in b.send_time.tolist()], dst_host=b.dst_host.tolist(),
            payload=b.payload.tolist(), round_end=str(round_end), sim_end=str(sim_end),
            bootstrap_end=str(boot_end),
            expect=dict(status=r.status.tolist(), ev_off=ev_off,
                        ev=[[str(t), s_, str(q), pk] for (t, s_, q, pk) in ev],
                        min_deliver=str(r.min_deliver), min_latency=str(r.min_latency),
                        rng=[[str(v) for v in row] for row in r.rng_state.tolist()],
                        next_id=[str(v) for v in r.next_event_id.tolist()])))
    return cases


def main():
    with open(os.path.join(HERE, "routing_cases.json"), "w") as f:
        json.dump(routing_cases(), f)
    with open(os.path.join(HERE, "rng_vectors.json"), "w") as f:
        json.dump(rng_vectors(), f, indent=1)
    with open(os.path.join(HERE, "relay_cases.json"), "w") as f:
        json.dump(relay_cases(), f)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
