"""GPU parity of the device-resident destination event queues against the
EventQueue restatement (oracle/relay.py: BinaryHeap per host, event.rs order, the pop loop of
Host::execute host.rs:697-706).  Path latencies (1-300 ms) exceed the 50 ms window, so events
stay pending across several rounds before they are popped."""
import numpy as np
import pytest

from oracle import corc
from oracle.relay import EventQueues as OracleQueues

pytestmark = pytest.mark.gpu


def _check(p, oq, H, window_end):
    for h in range(H):
        want = oq.pop_until(h, window_end)
        got = p.events_for(h)
        assert got == [(t, s, q, g) for t, s, q, g in want], h
    n_pending = sum(len(q) for q in oq.q)
    assert p.n_pending == n_pending
    heads = [oq.next_event_time(h) for h in range(H)]
    heads = [x for x in heads if x is not None]
    assert p.next_time == (min(heads) if heads else 2**64 - 1)


MERGE_KNOBS = {"sort": {}, "search": {"EQ_SEARCH_ONLY": 1}, "merge16": {"EQ_WAVE_MERGE": 0}}


@pytest.mark.parametrize("merge", list(MERGE_KNOBS))
@pytest.mark.parametrize("chance_mode,H,P", [(False, 3000, 120_000), (True, 3000, 120_000), (False, 40, 40_000)])
def test_queues_across_rounds_vs_oracle(engine, chance_mode, H, P, merge, knob):
    """H=3000: ~40 popped events per host and round, some hosts past the 16-lane merge's LDS
    stage (64); H=40: ~1000, past both stages (64 / 160), so the global-search path is the one
    checked.  merge: eqr_merge ranking staged hosts by a wave sort (default) or by searches
    alone, or eqr_merge16 (four hosts a wave)."""
    for k, v in MERGE_KNOBS[merge].items():
        knob(k, v)
    from shadow_amd import synth
    from shadow_amd.equeue import EventQueues
    from shadow_amd.relay import Relay
    NN = 60
    el = synth.complete_graph(NN, 31)
    used = np.arange(NN, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    host_node = synth.c5_host_nodes(H, NN)
    rng0 = synth.host_rng_states(H, 1)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    q = EventQueues(engine, H)
    oq = OracleQueues(H)
    orng, onid = rng0.copy(), np.zeros(H, np.uint64)
    start, win = 10**9, 50 * 10**6
    for rnd in range(6):
        b = synth.packet_batch(H, P, start, start + win, seed=70 + rnd)
        chance = np.random.default_rng(rnd).random(b.n) if chance_mode else None
        r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, start + win, start + 10**12, 0,
                     chance=chance)
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid,
                             start + win, start + 10**12, 0, chance=chance)
        ev = o["events"]
        for d in range(H):
            for k in range(int(ev["off"][d]), int(ev["off"][d + 1])):
                oq.push(d, ev["deliver"][k], ev["src"][k], ev["seq"][k], (rnd << 32) | int(ev["pkt"][k]))
        # the next round's window: [start + win, start + 2 win)
        p = q.advance(r.ev_off, r.ev_deliver, r.ev_src, r.ev_seq, r.ev_pkt, window_end=start + 2 * win)
        _check(p, oq, H, start + 2 * win)
        assert p.n_pending > 0 and len(p.deliver) > 0
        start += win
    # no new batch: drain what is left in two windows
    for w_end in (start + 3 * win, 2**63):
        p = q.advance(window_end=w_end)
        _check(p, oq, H, w_end)
    assert p.n_pending == 0 and p.next_time == 2**64 - 1


def test_empty_queues_and_empty_batch(engine):
    from shadow_amd.equeue import EventQueues
    q = EventQueues(engine, 5)
    p = q.advance(window_end=10)
    assert p.n_pending == 0 and len(p.deliver) == 0 and p.off.tolist() == [0] * 6
    p = q.advance(np.zeros(6, np.uint32), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                  np.zeros(0, np.uint64), np.zeros(0, np.uint32), window_end=10)
    assert p.n_pending == 0 and p.next_time == 2**64 - 1
    # equal delivery times: (src, seq) decides, across batches
    off = np.array([0, 0, 3, 3, 3, 3], np.uint32)
    p = q.advance(off, np.array([20, 20, 30], np.uint64), np.array([1, 4, 0], np.uint32),
                  np.array([7, 2, 9], np.uint64), np.array([0, 1, 2], np.uint32), window_end=15)
    assert len(p.deliver) == 0 and p.n_pending == 3 and p.next_time == 20
    p = q.advance(off, np.array([20, 25, 40], np.uint64), np.array([1, 0, 0], np.uint32),
                  np.array([6, 1, 2], np.uint64), np.array([5, 6, 7], np.uint32), window_end=31)
    # batch numbers count every batch handed over (the empty one above was batch 0)
    assert p.events_for(1) == [(20, 1, 6, (2 << 32) | 5), (20, 1, 7, 1 << 32), (20, 4, 2, (1 << 32) | 1),
                               (25, 0, 1, (2 << 32) | 6), (30, 0, 9, (1 << 32) | 2)]
    assert p.n_pending == 1 and p.next_time == 40


def test_run_compaction_and_pending_vs_oracle(engine, knob):
    """5 ms windows against 1-300 ms path latencies: no stored run drains for many rounds, so the
    8-run limit (EQ_MAX_RUNS knob) compacts the runs (from round 9 on), and pending() -- a compaction itself --
    returns every host's queue in EventQueue order, as the oracle's heaps hold it."""
    knob("EQ_MAX_RUNS", 8)
    from shadow_amd import synth
    from shadow_amd.equeue import EventQueues
    from shadow_amd.relay import Relay
    H, P, NN = 500, 20_000, 60
    el = synth.complete_graph(NN, 31)
    used = np.arange(NN, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    host_node = synth.c5_host_nodes(H, NN)
    rng0 = synth.host_rng_states(H, 1)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    q = EventQueues(engine, H)
    oq = OracleQueues(H)
    orng, onid = rng0.copy(), np.zeros(H, np.uint64)
    start, win = 10**9, 5 * 10**6
    for rnd in range(12):
        b = synth.packet_batch(H, P, start, start + win, seed=90 + rnd)
        r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, start + win, start + 10**12, 0)
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid,
                             start + win, start + 10**12, 0)
        ev = o["events"]
        for d in range(H):
            for k in range(int(ev["off"][d]), int(ev["off"][d + 1])):
                oq.push(d, ev["deliver"][k], ev["src"][k], ev["seq"][k], (rnd << 32) | int(ev["pkt"][k]))
        p = q.advance(r.ev_off, r.ev_deliver, r.ev_src, r.ev_seq, r.ev_pkt, window_end=start + 2 * win)
        _check(p, oq, H, start + 2 * win)
        if rnd in (3, 10):
            off, d, s, sq, t = q.pending()
            for h in range(H):
                a, e = int(off[h]), int(off[h + 1])
                got = list(zip(d[a:e].tolist(), s[a:e].tolist(), sq[a:e].tolist(), t[a:e].tolist()))
                assert got == sorted(oq.q[h]), h
        start += win
    assert p.n_pending > 0


def _cmp_popped(p, op):
    assert p.n_pending == op["n_pending"] and p.next_time == op["next_time"]
    assert np.array_equal(p.off, op["off"])
    assert np.array_equal(p.deliver, op["deliver"])
    assert np.array_equal(p.src, op["src"])
    assert np.array_equal(p.seq, op["seq"])
    assert np.array_equal(p.tag, op["tag"])


@pytest.mark.parametrize("merge,max_runs", [(m, 8) for m in MERGE_KNOBS] + [("sort", 3), ("sort", 12)])
@pytest.mark.parametrize("adopt", [True, False])
def test_adopted_batches_vs_c_queues(engine, adopt, merge, max_runs, knob):
    """The relay writes each round straight into the slot shd_equeue_batch_buffers hands out and
    the advance adopts it as a stored run (no copy) -- or, adopt=False, into the caller's own
    device arrays (copied).  5 ms windows over 1-300 ms paths for 14 rounds: the run limit
    (EQ_MAX_RUNS knob: 8, or 3 -- a compaction nearly every round -- or the default 12) forces
    partial compactions (the runs holding the fewest pending events) from then on.  Every
    popped event, the pending count and the next time against the C EventQueues; then pending()
    against the heaps' contents.  merge: as in test_queues_across_rounds_vs_oracle."""
    for k, v in MERGE_KNOBS[merge].items():
        knob(k, v)
    knob("EQ_MAX_RUNS", max_runs)
    import torch
    from shadow_amd import synth
    from shadow_amd.equeue import EventQueues
    from shadow_amd.relay import Relay
    H, P, NN = 2000, 60_000, 60
    el = synth.complete_graph(NN, 31)
    used = np.arange(NN, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    host_node = synth.c5_host_nodes(H, NN)
    rng0 = synth.host_rng_states(H, 1)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    q = EventQueues(engine, H)
    oq = corc.EventQueues(H)
    orng, onid = rng0.copy(), np.zeros(H, np.uint64)
    bufs = rl.device_buffers(P)
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()  # noqa: E731
    start, win = 10**9, 5 * 10**6
    for rnd in range(14):
        b = synth.packet_batch(H, P, start, start + win, seed=300 + rnd)
        d = [dev(b.src_off, np.int32), dev(b.send_time, np.int64), dev(b.dst_host, np.int32), dev(b.payload, np.int32)]
        torch.cuda.synchronize()
        if adopt:
            out = q.batch_buffers(P)
            out.status = N_ptr(bufs["status"])
            rl.round_device_into(*d, start + win, start + 10**12, 0, out)
        else:
            out = rl.round_device(*d, start + win, start + 10**12, 0, bufs)
        corc.relay_round_eq(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid,
                            start + win, start + 10**12, 0, queues=oq, batch_no=rnd)
        p = q.popped(q.advance_device(out, start + 2 * win))
        _cmp_popped(p, oq.pop(start + 2 * win))
        start += win
    off, dl, sr, sq, tg = q.pending()
    op = oq.pending()
    for k, v in (("off", off), ("deliver", dl), ("src", sr), ("seq", sq), ("tag", tg)):
        assert np.array_equal(v, op[k]), k


def N_ptr(t):
    return t.data_ptr()


def test_c5_scale_rounds_vs_c_queues(engine):
    """BASELINE config 5 at full size: 100k hosts x 10M packets per round on the C2 table (1-300
    ms paths), 1 ms windows for 4 rounds -- the queues then hold ~40M pending events in up to 5
    runs -- and a drain in two windows.  Every popped event of every host, the pending count and
    the next event time are compared with the C restatement of the per-host EventQueues
    (oracle/c/equeue.c: push_packet_to_host into each destination's heap during the relay round,
    then the pop loop of Host::execute, host.rs:697-706)."""
    from shadow_amd import synth
    from shadow_amd.equeue import EventQueues
    from shadow_amd.relay import Relay
    import torch
    H, P = 100_000, 10_000_000
    el = synth.complete_graph(1000, 1)
    used = np.arange(1000, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(1000, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    host_node = synth.c5_host_nodes(H, 1000)
    rng0 = synth.host_rng_states(H, 1)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    q = EventQueues(engine, H)
    oq = corc.EventQueues(H)
    orng, onid = rng0.copy(), np.zeros(H, np.uint64)
    bufs = rl.device_buffers(P)
    start, win, end = synth.SIM_START + 10**9, 10**6, synth.SIM_START + 10**12
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()  # noqa: E731
    for rnd in range(4):
        b = synth.packet_batch(H, P, start, start + win, seed=140 + rnd)
        d = [dev(b.src_off, np.int32), dev(b.send_time, np.int64), dev(b.dst_host, np.int32),
             dev(b.payload, np.int32)]
        torch.cuda.synchronize()
        out = rl.round_device(*d, start + win, end, 0, bufs)
        o = corc.relay_round_eq(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid,
                                start + win, end, 0, queues=oq, batch_no=rnd, threads=corc.max_threads())
        assert out.n_sent == o["n_sent"] and out.min_deliver == o["min_deliver"]
        p = q.popped(q.advance_device(out, start + 2 * win))
        op = oq.pop(start + 2 * win, threads=corc.max_threads())
        _cmp_popped(p, op)
        assert p.n_pending > 10_000_000 * rnd
        start += win
        del d
    for w_end in (start + 100 * win, 2**63):
        p = q.popped(q.advance_device(None, w_end))
        _cmp_popped(p, oq.pop(w_end, threads=corc.max_threads()))
    assert p.n_pending == 0


def test_c5_scale_adopted_rounds_with_compaction_vs_c_queues(engine, knob):
    """The bench's path at full C5 size for 12 rounds: each round's relay output is written into the
    slot shd_equeue_batch_buffers lends and adopted as a stored run; 1 ms windows over 1-300 ms
    paths keep every run alive, so from round 9 on an 8-run limit (EQ_MAX_RUNS knob; the default
    12 would compact once) forces the partial compactions (the runs holding the fewest pending
    events merged into one) at ~40-100M pending events.  Every popped event, the pending count and
    the next time against the C EventQueues, then a drain."""
    knob("EQ_MAX_RUNS", 8)
    from shadow_amd import synth
    from shadow_amd.equeue import EventQueues
    from shadow_amd.relay import Relay
    import torch
    H, P = 100_000, 10_000_000
    el = synth.complete_graph(1000, 1)
    used = np.arange(1000, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(1000, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    host_node = synth.c5_host_nodes(H, 1000)
    rng0 = synth.host_rng_states(H, 1)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    q = EventQueues(engine, H)
    oq = corc.EventQueues(H)
    orng, onid = rng0.copy(), np.zeros(H, np.uint64)
    st = torch.empty(P, dtype=torch.uint8, device="cuda")
    start, win, end = synth.SIM_START + 10**9, 10**6, synth.SIM_START + 10**12
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()  # noqa: E731
    for rnd in range(12):
        b = synth.packet_batch(H, P, start, start + win, seed=240 + rnd)
        d = [dev(b.src_off, np.int32), dev(b.send_time, np.int64), dev(b.dst_host, np.int32),
             dev(b.payload, np.int32)]
        torch.cuda.synchronize()
        out = q.batch_buffers(P)
        out.status = st.data_ptr()
        rl.round_device_into(*d, start + win, end, 0, out)
        o = corc.relay_round_eq(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid,
                                start + win, end, 0, queues=oq, batch_no=rnd, threads=corc.max_threads())
        assert out.n_sent == o["n_sent"] and out.min_deliver == o["min_deliver"]
        p = q.popped(q.advance_device(out, start + 2 * win))
        op = oq.pop(start + 2 * win, threads=corc.max_threads())
        _cmp_popped(p, op)
        start += win
        del d
    assert p.n_pending > 40_000_000   # ~4 rounds of events stay pending (1-300 ms paths)
    for w_end in (start + 150 * win, 2**63):
        p = q.popped(q.advance_device(None, w_end))
        _cmp_popped(p, oq.pop(w_end, threads=corc.max_threads()))
    assert p.n_pending == 0
