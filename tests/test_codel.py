"""CoDel router queue: the reference's own unit tests (codel_queue.rs:332-540) against the
oracle restatement (CPU), then the GPU engine against the oracle (bit-exact fates and states)."""
import math

import numpy as np
import pytest

from oracle import codel as O

START = 1000 * 10**6 + 946684800 * 10**9   # mock_time_millis(1000): SIMULATION_START + 1 s
ONE = 10**6


def test_ref_empty():
    q = O.CoDelQueue()
    assert len(q) == 0 and q.pop(START) is None


def test_ref_push_pop_simple():
    q = O.CoDelQueue()
    for i in range(1, 11):
        assert len(q) == i - 1
        q.push(i, 1500, START)
        assert len(q) == i
    for i in range(1, 11):
        assert len(q) == 10 - i + 1
        assert q.pop(START) is not None
        assert len(q) == 10 - i
    assert q.pop(START) is None


def test_ref_control_law():
    for i in range(2):
        assert O.apply_control_law(START, i) - START == O.INTERVAL
    for i in range(2, 20):
        assert O.apply_control_law(START, i) - START == round(O.INTERVAL / math.sqrt(i))


def test_ref_interval():
    q = O.CoDelQueue()
    for k in range(5):
        q.push(k, 1500, START)
    assert q.total_bytes_stored > O.MTU and q.interval_end is None
    T, I = O.TARGET, O.INTERVAL
    assert q._process_standing_delay(START + T - ONE, T - ONE) is False and q.interval_end is None
    assert q._process_standing_delay(START + T, T) is False and q.interval_end == START + T + I
    assert q._process_standing_delay(START + T + I, T + I) is True and q.interval_end == START + T + I
    assert q._process_standing_delay(START + T + 2 * I, T + 2 * I) is True
    assert q._process_standing_delay(START + T + 2 * I, ONE) is False and q.interval_end is None


def test_ref_mode():
    T, I = O.TARGET, O.INTERVAL
    q = O.CoDelQueue()
    for k in range(6):
        q.push(k, 1500, START)
    assert q.mode == O.STORE
    q.pop(START + T - ONE); assert len(q) == 5 and q.mode == O.STORE
    q.pop(START + T); assert len(q) == 4 and q.mode == O.STORE
    q.pop(START + T + I - ONE); assert len(q) == 3 and q.mode == O.STORE
    q.pop(START + T + I); assert len(q) == 1 and q.mode == O.DROP
    for k in range(3):
        q.push(10 + k, 1500, START + T + 2 * I - ONE)
    q.pop(START + T + 2 * I)
    assert q.mode == O.STORE


def test_ref_drop_empty():
    q = O.CoDelQueue()
    q.mode = O.DROP
    q.pop(START)
    assert q.mode == O.STORE


def test_ref_drop_many():
    T, I = O.TARGET, O.INTERVAL
    end = 1000000 * 10**6 + 946684800 * 10**9
    q = O.CoDelQueue()
    for k in range(20):
        q.push(k, 1500, START)
    q.pop(START + T)
    assert len(q) == 19 and q.current_drop_count == 0 and q.previous_drop_count == 0
    assert not q._was_dropping_recently(START + T) and q.mode == O.STORE
    q.pop(START + T + I)
    assert len(q) == 17 and q.current_drop_count == 1 and q.previous_drop_count == 1
    assert q.drop_next is not None and q._was_dropping_recently(START + T + I) and q.mode == O.DROP
    assert q._should_drop(end)
    q.pop(end)
    assert len(q) == 1 and q.current_drop_count == 16 and q.mode == O.STORE


# ------------------------------------------------------------------ GPU engine vs oracle
def _random_ops(rng, n_hosts, per_host, pid0=0):
    off, times, sizes, pkts = [0], [], [], []
    pid = pid0
    for h in range(n_hosts):
        t = START + int(rng.integers(0, 10**9))
        n = int(rng.integers(0, per_host + 1))
        for _ in range(n):
            t += int(rng.choice([0, rng.integers(0, 3 * ONE), rng.integers(0, 60 * ONE), rng.integers(0, 400 * ONE)]))
            if rng.random() < float(rng.choice([0.35, 0.5, 0.65])):
                times.append(t); sizes.append(int(rng.choice([1500, 60, 1200, int(rng.integers(1, 3000))])))
                pkts.append(pid); pid += 1
            else:
                times.append(t); sizes.append(O.U64_MAX & 0xFFFFFFFF); pkts.append(0)
        off.append(len(times))
    return (np.array(off, np.uint32), np.array(times, np.uint64), np.array(sizes, np.uint32),
            np.array(pkts, np.uint32), pid)


def _oracle_fate(fate_dict, n_ids):
    out = np.zeros(n_ids, np.uint64)
    for p, (k, kind) in fate_dict.items():
        out[p] = (k << 2) | kind
    return out


@pytest.mark.gpu
def test_reference_scenarios_on_gpu(engine):
    """drop_many and mode (codel_queue.rs) as op batches on one host; the state after each pop
    matches the reference's assertions."""
    from shadow_amd.codel import CoDelQueues, POP
    T, I = O.TARGET, O.INTERVAL
    q = CoDelQueues(engine, 1, 64)
    end = 1000000 * 10**6 + 946684800 * 10**9
    pushes = [(START, 1500, k) for k in range(20)]
    off = np.array([0, 20], np.uint32)
    q.run(off, [t for t, _, _ in pushes], [s for _, s, _ in pushes], [p for _, _, p in pushes])
    for now, want in ((START + T, dict(len=19, current_drop_count=0, previous_drop_count=0, mode=0)),
                      (START + T + I, dict(len=17, current_drop_count=1, previous_drop_count=1, mode=1)),
                      (end, dict(len=1, current_drop_count=16, mode=0))):
        q.run(np.array([0, 1], np.uint32), [now], [POP], [0])
        st = q.state(0)
        for k, v in want.items():
            assert st[k] == v, (now, k, st)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_random_batches_vs_oracle(engine, seed):
    """Many hosts, several batches in a row (state carried on the device), bit-exact pop results,
    packet fates and final queue states."""
    from shadow_amd.codel import CoDelQueues
    rng = np.random.default_rng(500 + seed)
    n_hosts = int(rng.integers(1, 300))
    q = CoDelQueues(engine, n_hosts, 512)
    queues = None
    pid = 0
    for _ in range(3):
        off, t, sz, pk, pid2 = _random_ops(rng, n_hosts, 60, pid)
        n_ids = max(pid2, 1)
        queues, pop_ref, fate_ref = O.run_ops(n_hosts, off, t, sz, pk, queues)
        pop_out, fate = q.run(off, t, sz, pk, n_ids=n_ids)
        assert pop_out.tolist() == [int(x) for x in pop_ref]
        assert np.array_equal(fate, _oracle_fate(fate_ref, n_ids))
        pid = pid2
    for h in range(n_hosts):
        st, r = q.state(h), queues[h]
        assert (st["len"], st["mode"], st["interval_end"], st["drop_next"], st["current_drop_count"],
                st["previous_drop_count"], st["total_bytes_stored"]) == \
               (len(r), r.mode, r.interval_end, r.drop_next, r.current_drop_count,
                r.previous_drop_count, r.total_bytes_stored)


@pytest.mark.gpu
def test_capacity_overflow_reported(engine):
    from shadow_amd.codel import CoDelQueues
    from shadow_amd._native import ShdError
    q = CoDelQueues(engine, 2, 4)
    off = np.array([0, 5, 5], np.uint32)
    with pytest.raises(ShdError, match="INVALID"):
        q.run(off, [START] * 5, [1500] * 5, list(range(5)))
    # the overflowing batch left the queues undefined: no further batch until set up again
    with pytest.raises(ShdError, match="STATE"):
        q.run(off, [START] * 5, [1500] * 5, list(range(5)))
    q2 = CoDelQueues(engine, 2, 8)
    pop, _ = q2.run(off, [START] * 5, [1500] * 5, list(range(5)))
    assert (pop == 0xFFFFFFFF).all()


@pytest.mark.parametrize("seed", range(4))
def test_c_restatement_matches_python_oracle(seed):
    """oracle/c/queues.c (the bench's multi-core CPU baseline) against oracle/codel.py on one
    fresh batch: pop results and packet fates bit for bit."""
    from oracle import corc
    rng = np.random.default_rng(700 + seed)
    n_hosts = int(rng.integers(1, 400))
    off, t, sz, pk, pid = _random_ops(rng, n_hosts, 80)
    n_ids = max(pid, 1)
    _, pop_ref, fate_ref = O.run_ops(n_hosts, off, t, sz, pk)
    pop, fate = corc.codel_run(n_hosts, off, t, sz, pk, n_ids)
    assert pop.tolist() == [int(x) for x in pop_ref]
    assert np.array_equal(fate, _oracle_fate(fate_ref, n_ids))
