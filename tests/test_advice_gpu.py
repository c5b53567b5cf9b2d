"""GPU tests of the engine's state rules: per-path packet counters count a round once and only
when it commits; a relay on the resident table stops when that table is rebuilt; zero-latency
edges are rejected as ShadowEdge::try_from rejects them (graph/mod.rs:107)."""
import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


def _setup(H, NN, P, seed, start=10**9, ra=10**6):
    from shadow_amd import synth
    el = synth.complete_graph(NN, seed)
    used = np.arange(NN, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    b = synth.packet_batch(H, P, start, start + ra, seed=seed)
    return el, lat, loss, synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1), b


def _want_counts(NN, host_node, b, status):
    src = np.repeat(np.arange(len(b.src_off) - 1), np.diff(b.src_off))
    sent = status == 2
    want = np.zeros((NN, NN), np.uint64)
    np.add.at(want, (host_node[src[sent]], host_node[b.dst_host[sent]]), 1)
    return want


@pytest.mark.parametrize("pipe", [7, 3])
def test_failed_round_does_not_count(engine, pipe, monkeypatch):
    from shadow_amd._native import ShdError
    from shadow_amd.relay import Relay
    monkeypatch.setenv("SHD_RELAY_FORCE_V3", "1" if pipe == 3 else "0")
    H, NN = 2000, 40
    _, lat, loss, host_node, rng0, b = _setup(H, NN, 100_000, 21)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    bad = b.dst_host.copy()
    bad[::997] = H + 3
    with pytest.raises(ShdError, match="NO_HOST"):
        rl.round(b.src_off, b.send_time, bad, b.payload, 10**9 + 10**6, 10**12, 0)
    assert not rl.packet_counts().any()
    # a drawing send after a skipped one (sim_end inside the round, send times going backwards)
    sim_end = 10**9 + 5 * 10**5
    t = b.send_time.copy()
    h = int(np.argmax(np.diff(b.src_off) > 3))
    a0 = int(b.src_off[h])
    t[a0], t[a0 + 1] = np.uint64(sim_end + 5), np.uint64(sim_end - 5)
    with pytest.raises(ShdError, match="INVALID"):
        rl.round(b.src_off, t, b.dst_host, b.payload, 10**9 + 10**6, sim_end, 0)
    assert not rl.packet_counts().any()
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, 10**9 + 10**6, 10**12, 0)
    assert rl.last_pipeline() == pipe
    assert np.array_equal(rl.packet_counts(), _want_counts(NN, host_node, b, r.status))


def test_wide_offset_rerun_counts_once(engine):
    """Sends far past round_end give deliver offsets >= 2^32: the narrow pipeline's round is
    redone on the 64-bit pipeline, and the counters see the round once."""
    from shadow_amd.relay import Relay
    H, NN = 500, 20
    start = 3 * 2**32
    _, lat, loss, host_node, rng0, b = _setup(H, NN, 30_000, 9, start=start)
    rd = (10**9, 2**62, 0)
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                         rng0.copy(), np.zeros(H, np.uint64), *rd)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, *rd)
    assert rl.last_pipeline() == 1
    assert np.array_equal(r.status, o["status"])
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), o["events"][k]), k
    assert np.array_equal(rl.packet_counts(), _want_counts(NN, host_node, b, r.status))
    r2 = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, *rd)
    assert np.array_equal(rl.packet_counts(), _want_counts(NN, host_node, b, r.status) +
                          _want_counts(NN, host_node, b, r2.status))


def test_relay_on_resident_table_invalidated_by_rebuild(engine):
    from shadow_amd._native import ShdError
    from shadow_amd.relay import Relay
    from tests.graphs import engine_graph_from_edges
    H, NN = 300, 30
    el, lat, loss, host_node, rng0, b = _setup(H, NN, 20_000, 4)
    g = engine_graph_from_edges(el)
    used = np.arange(NN, dtype=np.uint32)
    g.compute_shortest_paths(used, engine)           # full build -> resident table
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), engine=engine)   # NULL tables: resident
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                         rng0.copy(), np.zeros(H, np.uint64), 10**9 + 10**6, 10**12, 0)
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, 10**9 + 10**6, 10**12, 0)
    assert np.array_equal(r.ev_deliver, o["events"]["deliver"])
    g.compute_shortest_paths(used[:10], engine)      # rebuilds the resident table
    with pytest.raises(ShdError, match="STATE"):
        rl.round(b.src_off, b.send_time, b.dst_host, b.payload, 10**9 + 10**6, 10**12, 0)


def test_zero_latency_edge_rejected(engine):
    from shadow_amd._native import ShdError
    from shadow_amd.routing import NetworkGraph
    g = NetworkGraph([0, 1], [0, 1, 0], [0, 1, 1], [5, 5, 0], [0.0, 0.0, 0.0], False)
    with pytest.raises(ShdError, match="INVALID"):
        g.compute_shortest_paths([0, 1], engine)
