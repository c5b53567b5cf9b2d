"""shd_relay_flush -- the drop-in round barrier: worker threads' staging buffers (per-thread runs of
12-byte sends with the CPU's top-32-bit draws) grouped on the device, 2-bit statuses and 16-byte
events back.  Against the C restatement of send_packet in CPU-chance mode (worker.rs:328-413, the
f64 chance of each send = the same u64 draw >> 11 * 2^-53), round after round."""
import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


def _case(H, NN, seed):
    from shadow_amd import synth
    el = synth.complete_graph(NN, seed)
    used = np.arange(NN, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    return lat, loss, synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1)


def _host_of_send(st):
    """The staging's own knowledge: the source host of every send in stage order."""
    return np.concatenate([np.repeat(np.asarray(h, np.uint32), np.asarray(c, np.int64))
                           for h, c in zip(st.run_host, st.run_count)])


def _check(fr, o, st, nid_before, round_end):
    inv = np.empty(len(st.stage_of_send), np.int64)
    inv[st.stage_of_send] = np.arange(len(st.stage_of_send))
    assert np.array_equal(fr.status, o["status"][st.stage_of_send])
    ev = o["events"]
    assert np.array_equal(fr.ev_off, ev["off"])
    assert fr.n_sent == o["n_sent"] == len(fr.events)
    e = fr.events
    if e.shape[1] == 3:   # 12-byte events {deliver_off, seq_off, send}: the source from the send's run
        e = np.stack([e[:, 0], _host_of_send(st)[e[:, 2]], e[:, 1], e[:, 2]], axis=1)
    assert np.array_equal(e[:, 0].astype(np.uint64), ev["deliver"] - np.uint64(round_end))
    assert np.array_equal(e[:, 1], ev["src"])
    assert np.array_equal(e[:, 2].astype(np.uint64) + fr.seq_base[e[:, 1]], ev["seq"])
    assert np.array_equal(e[:, 3].astype(np.int64), inv[ev["pkt"].astype(np.int64)])
    assert np.array_equal(fr.seq_base, nid_before)
    assert (fr.min_deliver, fr.min_latency) == (o["min_deliver"], o["min_latency"])


@pytest.mark.parametrize("n_threads,pinned,event_bytes,pinned_out,copy",
                         [(1, False, 16, False, 0), (16, False, 16, False, 0), (1, True, 16, False, 0),
                          (16, True, 16, False, 0), (16, True, 12, False, 0), (16, True, 16, True, 0),
                          (16, True, 12, True, 0), (16, True, 16, True, 1)])
def test_flush_rounds_vs_c_oracle(engine, knob, n_threads, pinned, event_bytes, pinned_out, copy):
    """Pinned staging is read where it lies and pinned outputs are written where they lie (zero-copy)
    unless the FLUSH_COPY knob asks for the copies; pageable buffers are always copied."""
    from shadow_amd import synth
    from shadow_amd.relay import PinnedStages, Relay
    H, NN, P = 20_000, 200, 1_000_000
    lat, loss, host_node, rng0 = _case(H, NN, 21)
    knob("FLUSH_COPY", copy)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    onid = np.zeros(H, np.uint64)
    start, ra = 10**9, 10**6
    for rnd in range(3):
        b = synth.packet_batch(H, P, start, start + ra, seed=60 + rnd)
        st = synth.stage_round(b, n_threads, start, seed=rnd)
        chance = (st.draw64 >> np.uint64(11)).astype(np.float64) * 2.0**-53
        nid_before = onid.copy()
        boot = start + ra // 2 if rnd == 0 else 0
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                             onid, start + ra, start + 100 * ra, boot, chance=chance)
        ps = PinnedStages.pinned(engine.lib, st.run_host, st.run_count, st.sends) if pinned else None
        try:
            fr = rl.flush(st.run_host, st.run_count, st.sends, start, start + ra, start + 100 * ra, boot, pinned=ps,
                          event_bytes=event_bytes, pinned_out=pinned_out)
        finally:
            if ps is not None:
                ps.free()
        _check(fr, o, st, nid_before, start + ra)
        start += ra
    rng, nid = rl.host_state()
    assert np.array_equal(rng, rng0)          # the device streams were not used: the CPU drew
    assert np.array_equal(nid, onid)          # event ids advanced by the sent packets


def test_flush_many_hosts_runs(engine):
    """600k hosts with about one send each (a host has one run: the staging contract), so the scans
    of the run counts and of the per-host counts span more than 64 tiles of 8192 -- the look-back's
    second window (scan.h) -- and the round takes the radix pipeline (more hosts than pipeline 7's
    2^18)."""
    from shadow_amd import synth
    from shadow_amd.relay import Relay
    H, NN, P = 600_000, 200, 650_000
    lat, loss, host_node, rng0 = _case(H, NN, 23)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    start, ra = 10**9, 10**6
    b = synth.packet_batch(H, P, start, start + ra, seed=71)
    st = synth.stage_round(b, 4, start, seed=5)
    assert sum(len(h) for h in st.run_host) > 64 * 8192
    chance = (st.draw64 >> np.uint64(11)).astype(np.float64) * 2.0**-53
    onid = np.zeros(H, np.uint64)
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                         onid, start + ra, start + 100 * ra, 0, chance=chance)
    fr = rl.flush(st.run_host, st.run_count, st.sends, start, start + ra, start + 100 * ra, 0)
    _check(fr, o, st, np.zeros(H, np.uint64), start + ra)


def test_flush_then_device_draws_round(engine):
    """A flush round (CPU draws) followed by a device-drawn round: ids carry over, the device
    streams start where they were."""
    from shadow_amd import synth
    from shadow_amd.relay import Relay
    H, NN, P = 5000, 60, 200_000
    lat, loss, host_node, rng0 = _case(H, NN, 5)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    onid = np.zeros(H, np.uint64)
    b = synth.packet_batch(H, P, 10**9, 10**9 + 10**6, seed=1)
    st = synth.stage_round(b, 8, 10**9, seed=2)
    chance = (st.draw64 >> np.uint64(11)).astype(np.float64) * 2.0**-53
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(), onid,
                         10**9 + 10**6, 10**12, 0, chance=chance)
    fr = rl.flush(st.run_host, st.run_count, st.sends, 10**9, 10**9 + 10**6, 10**12, 0)
    assert np.array_equal(fr.status, o["status"][st.stage_of_send])
    b2 = synth.packet_batch(H, P, 10**9 + 10**6, 10**9 + 2 * 10**6, seed=2)
    orng = rng0.copy()
    o2 = corc.relay_round(b2.src_off, b2.send_time, b2.dst_host, b2.payload, host_node, lat, loss, orng, onid,
                          10**9 + 2 * 10**6, 10**12, 0)
    r2 = rl.round(b2.src_off, b2.send_time, b2.dst_host, b2.payload, 10**9 + 2 * 10**6, 10**12, 0)
    assert np.array_equal(r2.status, o2["status"])
    assert np.array_equal(r2.ev_seq, o2["events"]["seq"])
    rng, nid = rl.host_state()
    assert np.array_equal(rng, orng) and np.array_equal(nid, onid)


def test_flush_rejects_bad_staging(engine):
    from shadow_amd import synth
    from shadow_amd._native import ShdError
    from shadow_amd.relay import Relay
    H, NN, P = 2000, 30, 50_000
    lat, loss, host_node, rng0 = _case(H, NN, 9)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    b = synth.packet_batch(H, P, 10**9, 10**9 + 10**6, seed=3)
    st = synth.stage_round(b, 4, 10**9, seed=4)
    args = (10**9, 10**9 + 10**6, 10**12, 0)
    # one host in two threads' buffers
    rh = [h.copy() for h in st.run_host]
    rh[1][0] = rh[0][0]
    with pytest.raises(ShdError, match="INVALID"):
        rl.flush(rh, st.run_count, st.sends, *args)
    # a run of a host the relay does not have
    rh = [h.copy() for h in st.run_host]
    rh[2][3] = H + 5
    with pytest.raises(ShdError, match="NO_HOST"):
        rl.flush(rh, st.run_count, st.sends, *args)
    # runs that do not cover the stage's records
    rc = [c.copy() for c in st.run_count]
    rc[0][0] += 1
    with pytest.raises(ShdError, match="INVALID"):
        rl.flush(st.run_host, rc, st.sends, *args)
    # a destination outside the hosts
    sd = [s.copy() for s in st.sends]
    sd[3][7, 1] = (sd[3][7, 1] & np.uint32(0x80000000)) | np.uint32(H + 1)
    with pytest.raises(ShdError, match="NO_HOST"):
        rl.flush(st.run_host, st.run_count, sd, *args)
    # nothing was committed: the next good flush matches a fresh oracle round
    onid = np.zeros(H, np.uint64)
    chance = (st.draw64 >> np.uint64(11)).astype(np.float64) * 2.0**-53
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(), onid,
                         10**9 + 10**6, 10**12, 0, chance=chance)
    fr = rl.flush(st.run_host, st.run_count, st.sends, *args)
    _check(fr, o, st, np.zeros(H, np.uint64), 10**9 + 10**6)


@pytest.mark.parametrize("path", ["bins", "x24", "bins-pinned"])
def test_flush_two_ranks_vs_c_oracle(engine, knob, path):
    """shd_relay_flush under a two-rank communicator: both ranks get the same 16 stages (every
    thread's buffer mixes both ranks' hosts); each keeps its own hosts' runs.  The OR of the ranks'
    statuses, each rank's destinations' events (relative ids, sends in stage order) and the reduced
    round outputs against the C restatement in CPU-chance mode, three rounds; both exchange forms."""
    import threading

    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.routing import Engine
    H, NN, P = 6000, 60, 400_000
    lat, loss, host_node, rng0 = _case(H, NN, 13)
    engines = [Engine(0), Engine(0)]
    try:
        for e in engines:
            knob("RELAY_SHARD_X24", 1 if path == "x24" else 0, eng=e)
        D.comm_init_local(engines)
        rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
        onid = np.zeros(H, np.uint64)
        start, ra = 10**9, 10**6
        for rnd in range(3):
            b = synth.packet_batch(H, P, start, start + ra, seed=70 + rnd)
            st = synth.stage_round(b, 16, start, seed=10 + rnd)
            chance = (st.draw64 >> np.uint64(11)).astype(np.float64) * 2.0**-53
            nid_before = onid.copy()
            boot = start + ra // 2 if rnd == 0 else 0
            o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                                 onid, start + ra, start + 100 * ra, boot, chance=chance)
            res, errs = [None, None], []
            from shadow_amd.relay import PinnedStages
            ps = PinnedStages.pinned(engines[0].lib, st.run_host, st.run_count, st.sends) if path == "bins-pinned" else None

            def go(i):
                try:   # (both ranks read the same pinned stages in place)
                    res[i] = rels[i].flush(st.run_host, st.run_count, st.sends, start, start + ra, start + 100 * ra, boot,
                                           pinned=ps)
                except BaseException as ex:   # noqa: BLE001
                    errs.append(ex)
            ts = [threading.Thread(target=go, args=(i,)) for i in range(2)]
            for t in ts:
                t.start()
            for t in ts:
                t.join(timeout=300)
            if ps is not None:
                ps.free()
            assert not errs, errs
            assert [r.last_pipeline() for r in rels] == ([7, 7] if path == "x24" else [8, 8])
            inv = np.empty(len(st.stage_of_send), np.int64)
            inv[st.stage_of_send] = np.arange(len(st.stage_of_send))
            assert np.array_equal(res[0].status | res[1].status, o["status"][st.stage_of_send])
            seq_base = np.zeros(H, np.uint64)
            for r, fr in zip(rels, res):
                seq_base[r.lo:r.hi] = fr.seq_base[r.lo:r.hi]
            assert np.array_equal(seq_base, nid_before)
            ev = o["events"]
            for r, fr in zip(rels, res):
                s0, s1 = int(ev["off"][r.lo]), int(ev["off"][r.hi])
                assert np.array_equal(fr.ev_off, (ev["off"][r.lo:r.hi + 1] - ev["off"][r.lo]).astype(np.uint32))
                e = fr.events
                assert len(e) == s1 - s0
                assert np.array_equal(e[:, 0].astype(np.uint64), ev["deliver"][s0:s1] - np.uint64(start + ra))
                assert np.array_equal(e[:, 1], ev["src"][s0:s1])
                assert np.array_equal(e[:, 2].astype(np.uint64) + seq_base[e[:, 1]], ev["seq"][s0:s1])
                assert np.array_equal(e[:, 3].astype(np.int64), inv[ev["pkt"][s0:s1].astype(np.int64)])
                assert (fr.min_deliver, fr.min_latency, fr.n_sent) == (o["min_deliver"], o["min_latency"], o["n_sent"])
            start += ra
        for r in rels:
            rng, nid = r.host_state()
            assert np.array_equal(rng[r.lo:r.hi], rng0[r.lo:r.hi])   # the CPU drew
            assert np.array_equal(nid[r.lo:r.hi], onid[r.lo:r.hi])
    finally:
        for e in engines:
            e.close()
