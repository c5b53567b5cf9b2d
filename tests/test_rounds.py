"""CPU tests of the round bookkeeping: the window arithmetic of the library (shd_window_compute,
no GPU needed) against the restatement of controller.rs:86-111 / runahead.rs:43-115, and the C
restatement of the per-host EventQueues (oracle/c/equeue.c) against the Python one."""
import numpy as np
import pytest

from oracle import corc
from oracle.relay import EMUTIME_MAX, EventQueues, RunaheadState, next_window

U64_MAX = 2**64 - 1


@pytest.mark.parametrize("min_next,ra,end", [
    (10**9, 10**6, 10**12),                   # plain window
    (10**9, 10**6, 10**9 + 5),                # end_time cuts it
    (10**9, 10**6, 10**9),                    # empty: stop
    (None, 10**6, 10**12),                    # no next event: EmulatedTime::MAX -> stop
    (U64_MAX, 10**6, U64_MAX),                # None at the ABI, with an end past MAX
    (EMUTIME_MAX - 10, 10**6, U64_MAX),       # checked_add past EMUTIME_MAX -> MAX
    (EMUTIME_MAX - 10, 5, U64_MAX),           # sum == EMUTIME_MAX - 5: fits
    (2**64 - 3, 1, U64_MAX),                  # sum == EMUTIME_MAX exactly
    (0, 1, 1),
])
def test_window_compute_matches_controller(min_next, ra, end):
    from shadow_amd.rounds import window_compute
    assert window_compute(min_next, ra, end) == next_window(min_next, ra, end)


def test_window_compute_random():
    from shadow_amd.rounds import window_compute
    rng = np.random.default_rng(3)
    for _ in range(500):
        m = int(rng.integers(0, 2**63)) * int(rng.integers(1, 3))
        ra = int(rng.integers(1, 2**40))
        end = int(rng.integers(0, 2**63)) * 2
        assert window_compute(m, ra, end) == next_window(m, ra, end)


def test_runahead_restatement():
    """Runahead::get / update_lowest_used_latency (runahead.rs:43-115)."""
    r = RunaheadState(True, 5_000_000, None)
    assert r.get() == 5_000_000
    r.update_lowest_used_latency(7_000_000)
    assert r.get() == 7_000_000          # the used latency replaces the possible one, even if larger
    r.update_lowest_used_latency(3_000_000)
    r.update_lowest_used_latency(4_000_000)
    assert r.get() == 3_000_000
    c = RunaheadState(True, 5_000_000, 10_000_000)
    c.update_lowest_used_latency(1_000_000)
    assert c.get() == 10_000_000         # the config is a lower bound
    s = RunaheadState(False, 5_000_000, None)
    s.update_lowest_used_latency(1_000_000)
    assert s.get() == 5_000_000          # not dynamic: never updated


def test_c_event_queues_match_python_heaps():
    """oracle/c/equeue.c against oracle/relay.py's heapq queues: random batches with unique
    (src, seq) keys and many equal delivery times, pushed and popped across 10 windows."""
    rng = np.random.default_rng(0)
    H = 64
    cq, pq = corc.EventQueues(H), EventQueues(H)
    seq = 0
    w_prev = 0
    for b in range(10):
        cnt = rng.integers(0, 25, H)
        off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
        n = int(off[-1])
        d = (rng.integers(0, 6, n) * 5 + w_prev).astype(np.uint64)   # ties on time
        s = rng.integers(0, H, n).astype(np.uint32)
        q = (np.arange(n) + seq).astype(np.uint64)                  # unique ids
        rng.shuffle(q)
        seq += n
        pk = np.arange(n, dtype=np.uint32)
        cq.push_batch(off, d, s, q, pk, b)
        for h in range(H):
            for k in range(off[h], off[h + 1]):
                pq.push(h, d[k], s[k], q[k], (b << 32) | int(pk[k]))
        w = w_prev + 12
        o = cq.pop(w)
        for h in range(H):
            want = pq.pop_until(h, w)
            a, e = int(o["off"][h]), int(o["off"][h + 1])
            got = list(zip(o["deliver"][a:e].tolist(), o["src"][a:e].tolist(), o["seq"][a:e].tolist(),
                           o["tag"][a:e].tolist()))
            assert got == [tuple(x) for x in want], h
        assert o["n_pending"] == sum(len(x) for x in pq.q)
        heads = [pq.next_event_time(h) for h in range(H)]
        heads = [x for x in heads if x is not None]
        assert o["next_time"] == (min(heads) if heads else U64_MAX)
        w_prev = w
    p = cq.pending()
    for h in range(H):
        a, e = int(p["off"][h]), int(p["off"][h + 1])
        assert list(zip(p["deliver"][a:e].tolist(), p["src"][a:e].tolist(), p["seq"][a:e].tolist(),
                        p["tag"][a:e].tolist())) == sorted(pq.q[h])


def test_c_event_queues_refuse_time_going_backwards():
    """EventQueue::pop asserts that time never moves backwards (event_queue.rs:36-40)."""
    q = corc.EventQueues(1)
    q.push_batch(np.array([0, 1], np.uint32), np.array([10], np.uint64), np.zeros(1, np.uint32),
                 np.zeros(1, np.uint64), np.zeros(1, np.uint32), 0)
    q.pop(11)
    q.push_batch(np.array([0, 1], np.uint32), np.array([5], np.uint64), np.zeros(1, np.uint32),
                 np.ones(1, np.uint64), np.zeros(1, np.uint32), 1)
    with pytest.raises(AssertionError):
        q.pop(11)


def test_relay_into_c_queues_matches_relay_then_push():
    """orc_relay_round_eq (push_packet_to_host during the round) leaves the same queues as the
    round's sorted events pushed afterwards."""
    from shadow_amd import synth
    H, NN = 300, 20
    el = synth.complete_graph(NN, 2)
    used = np.arange(NN, dtype=np.uint32)
    _, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    host_node = synth.c5_host_nodes(H, NN)
    rng0 = synth.host_rng_states(H, 1)
    b = synth.packet_batch(H, 20_000, 10**9, 10**9 + 10**6, seed=5)
    qa, qb = corc.EventQueues(H), corc.EventQueues(H)
    o1 = corc.relay_round_eq(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                             np.zeros(H, np.uint64), 10**9 + 10**6, 10**12, 0, queues=qa, batch_no=3)
    o2 = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                          np.zeros(H, np.uint64), 10**9 + 10**6, 10**12, 0)
    ev = o2["events"]
    qb.push_batch(ev["off"], ev["deliver"], ev["src"], ev["seq"], ev["pkt"], 3)
    assert o1["n_sent"] == o2["n_sent"] and np.array_equal(o1["status"], o2["status"])
    pa, pb = qa.pending(), qb.pending()
    for k in ("off", "deliver", "src", "seq", "tag"):
        assert np.array_equal(pa[k], pb[k]), k
