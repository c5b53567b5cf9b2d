"""Token-bucket relays: the reference's own unit tests (token_bucket.rs:160-277) against the
oracle restatement (CPU), then the GPU engine against the oracle (bit-exact statuses, values and
bucket states, state carried across batches)."""
import numpy as np
import pytest

from oracle import token_bucket as O

MS = 10**6


def mock_time_millis(ms):
    """network/mod.rs:20-23: SIMULATION_START + ms."""
    return O.SIM_START + ms * MS


def test_ref_new_invalid_args():
    now = mock_time_millis(1000)
    for args in ((0, 1, 1), (1, 0, 1), (1, 1, 0)):
        with pytest.raises(ValueError):
            O.TokenBucket(*args, now)


def test_ref_new_valid_args():
    now = mock_time_millis(1000)
    for itv in (1, MS, 1000 * MS):
        O.TokenBucket(1, 1, itv, now)
    tb = O.TokenBucket(54321, 12345, 1000 * MS, now)
    assert (tb.capacity, tb.refill_increment, tb.refill_interval) == (54321, 12345, 1000 * MS)


def test_ref_refill_after_one_interval():
    interval, capacity, increment = 10 * MS, 100, 10
    now = mock_time_millis(1000)
    tb = O.TokenBucket(capacity, increment, interval, now)
    assert tb.balance == capacity
    assert tb.conforming_remove(capacity, now)[0]
    assert tb.balance == 0
    for i in range(1, capacity // increment + 1):
        ok, v = tb.conforming_remove(0, now + interval * i)
        assert ok and v == tb.balance == increment * i


def test_ref_refill_after_multiple_intervals():
    now = mock_time_millis(1000)
    tb = O.TokenBucket(100, 10, 10 * MS, now)
    assert tb.conforming_remove(100, now)[0] and tb.balance == 0
    ok, v = tb.conforming_remove(0, now + 50 * MS)
    assert ok and v == tb.balance == 50


def test_ref_capacity_limit():
    now = mock_time_millis(1000)
    tb = O.TokenBucket(100, 10, 10 * MS, now)
    assert tb.conforming_remove(100, now)[0] and tb.balance == 0
    ok, v = tb.conforming_remove(0, now + 60 * 1000 * MS)
    assert ok and v == tb.balance == 100


def test_ref_remove_error():
    now = mock_time_millis(1000)
    tb = O.TokenBucket(100, 10, 125 * MS, now)
    assert tb.conforming_remove(100, now) == (True, 0)
    assert tb.conforming_remove(50, now) == (False, 125 * 5 * MS)
    assert tb.conforming_remove(50, mock_time_millis(1000 + 10)) == (False, (125 * 5 - 10) * MS)


def test_create_token_bucket():
    """relay/mod.rs:291-302: 1 ms refills of max(1, Bps / 1000), capacity + MTU burst."""
    assert O.create_token_bucket(125_000_000) == (125_000 + 1500, 125_000, MS)
    assert O.create_token_bucket(999) == (1 + 1500, 1, MS)


def _random_batch(rng, n_relays, per, t0, span, flags_p=0.1):
    counts = rng.integers(0, 2 * per + 1, n_relays)
    off = np.zeros(n_relays + 1, np.uint32)
    off[1:] = np.cumsum(counts)
    n = int(off[-1])
    time = np.empty(n, np.uint64)
    for r in range(n_relays):
        a, b = int(off[r]), int(off[r + 1])
        time[a:b] = np.sort(rng.integers(t0, t0 + span, b - a)).astype(np.uint64)
    size = rng.choice([0, 66, 1448, 1514, 9000], n).astype(np.uint32)
    flags = (rng.random(n) < flags_p).astype(np.uint8)
    return off, time, size, flags


def _setup(rng, n_relays, t0):
    caps, incs, itvs = [], [], []
    for r in range(n_relays):
        kind = r % 4
        if kind == 0:
            c, i, v = 0, 0, 0                                   # unlimited relay
        elif kind == 1:
            c, i, v = O.create_token_bucket(int(rng.integers(1, 10**7)))
        else:
            c, i, v = int(rng.integers(1, 20000)), int(rng.integers(1, 3000)), int(rng.integers(1, 5 * MS))
        caps.append(c); incs.append(i); itvs.append(v)
    return np.array(caps, np.uint64), np.array(incs, np.uint64), np.array(itvs, np.uint64)


@pytest.mark.gpu
def test_gpu_reference_remove_error_sequence(engine):
    """test_remove_error replayed through the engine on one relay."""
    from shadow_amd.tbucket import BLOCKED, FORWARDED, SKIPPED, TokenBuckets
    now = mock_time_millis(1000)
    tb = TokenBuckets(engine, [100], [10], [125 * MS], [now])
    st, v = tb.run([0, 1], [now], [100])
    assert st.tolist() == [FORWARDED] and v.tolist() == [0]
    st, v = tb.run([0, 2], [now, mock_time_millis(1010)], [50, 50])
    # the block makes the relay Pending until now + 625 ms: the next attempt is not made
    assert st.tolist() == [BLOCKED, SKIPPED]
    assert v.tolist() == [625 * MS, now + 625 * MS]
    s = tb.state(0)
    assert s["balance"] == 0 and s["pending_until"] == now + 625 * MS and s["last_refill"] == now


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_random_batches_vs_oracle(engine, seed):
    from shadow_amd.tbucket import TokenBuckets
    rng = np.random.default_rng(seed)
    R = 700
    t0 = O.SIM_START + 5 * 10**9
    caps, incs, itvs = _setup(rng, R, t0)
    tb = TokenBuckets(engine, caps, incs, itvs, t0)
    buckets = [None if c == 0 else O.TokenBucket(int(c), int(i), int(v), t0)
               for c, i, v in zip(caps, incs, itvs)]
    pending = [0] * R
    t = t0
    for _ in range(4):
        off, time, size, flags = _random_batch(rng, R, 30, t, 20 * MS)
        st, val = tb.run(off, time, size, flags)
        ost, oval = O.relay_run(buckets, pending, off, time, size, flags)
        assert st.tolist() == ost
        assert val.tolist() == oval
        t += 20 * MS
    for r in range(0, R, 37):
        s = tb.state(r)
        b = buckets[r]
        if b is not None:
            assert (s["balance"], s["last_refill"]) == (b.balance, b.last_refill)
        assert s["pending_until"] == pending[r]


@pytest.mark.gpu
def test_gpu_invalid_setup_and_time_before_refill(engine):
    from shadow_amd import _native as N
    from shadow_amd.tbucket import TokenBuckets
    with pytest.raises(N.ShdError):
        TokenBuckets(engine, [100, 5], [10, 0], [MS, MS], [0, 0])
    now = mock_time_millis(1000)
    tb = TokenBuckets(engine, [100], [10], [MS], [now])
    with pytest.raises(N.ShdError):
        tb.run([0, 1], [now - 1], [10])    # duration_since before last_refill: the reference panics


@pytest.mark.parametrize("seed", [4, 5, 6])
def test_c_restatement_matches_python_oracle(seed):
    """oracle/c/queues.c (the bench's multi-core CPU baseline) against oracle/token_bucket.py."""
    from oracle import corc
    rng = np.random.default_rng(seed)
    R = 900
    t0 = O.SIM_START + 5 * 10**9
    caps, incs, itvs = _setup(rng, R, t0)
    buckets = [None if c == 0 else O.TokenBucket(int(c), int(i), int(v), t0) for c, i, v in zip(caps, incs, itvs)]
    off, time, size, flags = _random_batch(rng, R, 40, t0, 30 * MS)
    ost, oval = O.relay_run(buckets, [0] * R, off, time, size, flags)
    st, val, panics = corc.tb_run(caps, incs, itvs, np.full(R, t0, np.uint64), off, time, size, flags)
    assert panics == 0
    assert st.tolist() == ost and val.tolist() == oval
