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
def test_failed_round_does_not_count(engine, pipe, knob):
    from shadow_amd._native import ShdError
    from shadow_amd.relay import Relay
    knob("RELAY_FORCE_V3", 1 if pipe == 3 else 0)
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


def test_round_window_without_device_queues():
    """A caller that keeps the relay's events in its own queues (no shd_equeue_setup) and reports
    their heads as its next event time: shd_round_window must count each relay output's earliest
    deliver time for the window right after that round only, so the window keeps moving forward
    (controller.rs:86-111, manager.rs:455-464) -- round after round against the restatement, with
    the dynamic runahead (runahead.rs:43-115) fed by every round's min latency.  A fresh engine:
    the session engine may hold device queues from other tests."""
    from oracle.relay import EventQueues, RunaheadState, next_window
    from shadow_amd import synth
    from shadow_amd.relay import Relay
    from shadow_amd.rounds import Runahead, next_window as eng_window
    from shadow_amd.routing import Engine
    H, NN, P = 3000, 40, 60_000
    _, lat, loss, host_node, rng0, _ = _setup(H, NN, 1000, 41)
    U64 = 2**64 - 1
    with Engine(0) as eng:
        rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=eng)
        min_possible = int(lat.min())
        Runahead(eng, True, min_possible)
        ora = RunaheadState(True, min_possible)
        q = EventQueues(H)
        end_time = 10**9 + 500 * 10**6
        ws, we = 10**9, 10**9 + ora.get()
        starts = []
        for rnd in range(6):
            for h in range(H):   # every host executes its events below the window end
                q.pop_until(h, we)
            b = synth.packet_batch(H, P, ws, we, seed=300 + rnd)
            r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, we, end_time, 0)
            if r.min_latency != U64:
                ora.update_lowest_used_latency(r.min_latency)
            for d in range(H):
                for t, s, sq, p in r.events_for(d):
                    q.push(d, t, s, sq, (rnd << 32) | p)
            heads = [q.next_event_time(h) for h in range(H)]
            heads = [x for x in heads if x is not None]
            cpu_next = min(heads) if heads else None
            want = next_window(min(cpu_next if cpu_next is not None else U64, r.min_deliver), ora.get(), end_time)
            got = eng_window(eng, cpu_next, end_time)
            assert got == want, (rnd, got, want)
            ws, we = want
            starts.append(ws)
        assert starts == sorted(starts) and starts[-1] > starts[0]


def test_lent_batch_slot_refuses_larger_rounds(engine):
    """shd_equeue_batch_buffers lends a slot of max_events events: a relay round of more packets
    into that slot is refused before any kernel runs (it could write past the slot), and the same
    round into a slot large enough goes through and is adopted."""
    import torch
    from shadow_amd import synth
    from shadow_amd._native import ShdError
    from shadow_amd.equeue import EventQueues
    from shadow_amd.relay import Relay
    H, NN, P = 1000, 30, 20_000
    _, lat, loss, host_node, rng0, b = _setup(H, NN, P, 43)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    q = EventQueues(engine, H)
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()  # noqa: E731
    d = [dev(b.src_off, np.int32), dev(b.send_time, np.int64), dev(b.dst_host, np.int32), dev(b.payload, np.int32)]
    st = torch.empty(P, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    small = q.batch_buffers(P // 2)
    small.status = st.data_ptr()
    with pytest.raises(ShdError, match="INVALID"):
        rl.round_device_into(*d, 10**9 + 10**6, 10**12, 0, small)
    big = q.batch_buffers(P)
    big.status = st.data_ptr()
    out = rl.round_device_into(*d, 10**9 + 10**6, 10**12, 0, big)
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                         rng0.copy(), np.zeros(H, np.uint64), 10**9 + 10**6, 10**12, 0)
    assert out.n_sent == int((o["status"] == 2).sum())
    p = q.popped(q.advance_device(out, 2**63))
    assert np.array_equal(p.deliver, o["events"]["deliver"])
    assert np.array_equal(p.seq, o["events"]["seq"])
