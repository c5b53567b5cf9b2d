"""ctypes front end of the C restatement (oracle/c/oracle.c) -- test infrastructure only."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

TIDY, FAITHFUL = 0, 1
CODES = {0: "OK", 1: "NO_EDGE", 2: "MULTI_EDGE", 3: "UNREACHABLE", 4: "NOMEM"}


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", os.path.join(_HERE, "c")])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        P = C.c_void_p
        _lib.orc_shortest_paths.restype = C.c_int
        _lib.orc_shortest_paths.argtypes = [C.c_uint32, C.c_uint32, P, P, P, P, C.c_int, P,
                                            C.c_uint32, C.c_int, C.c_int, P, P, P, P]
        _lib.orc_shortest_paths_rows.restype = C.c_int
        _lib.orc_shortest_paths_rows.argtypes = [C.c_uint32, C.c_uint32, P, P, P, P, C.c_int, P,
                                                 C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int,
                                                 P, P, P, P]
        _lib.orc_next_hops.restype = C.c_int
        _lib.orc_next_hops.argtypes = [C.c_uint32, C.c_uint32, P, P, P, P, C.c_int, P, C.c_uint32, C.c_uint32,
                                       C.c_uint32, P, P, C.c_int, P]
        _lib.orc_codel_run.restype = None
        _lib.orc_codel_run.argtypes = [C.c_uint32, P, P, P, P, P, P, C.c_uint32, C.c_int]
        _lib.orc_tb_run.restype = C.c_int64
        _lib.orc_tb_run.argtypes = [C.c_uint32, P, P, P, P, P, P, P, P, P, P, C.c_int]
        _lib.orc_direct_paths.restype = C.c_int
        _lib.orc_direct_paths.argtypes = [C.c_uint32, C.c_uint32, P, P, P, P, C.c_int, P,
                                          C.c_uint32, P, P, P, P]
        _lib.orc_relay_round.restype = C.c_int64
        _lib.orc_relay_round.argtypes = [C.c_uint32, P, P, P, P, P, P, C.c_uint32, P, P, P, P,
                                         C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, P, P, P,
                                         P, P, P, P, P, P, P]
        _lib.orc_relay_round_eq.restype = C.c_int64
        _lib.orc_relay_round_eq.argtypes = [C.c_uint32, P, P, P, P, P, P, C.c_uint32, P, P, P, P,
                                            C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, P, P, P,
                                            P, P, P, C.c_uint64]
        _lib.orc_eq_new.restype = P
        _lib.orc_eq_new.argtypes = [C.c_uint32]
        _lib.orc_eq_free.restype = None
        _lib.orc_eq_free.argtypes = [P]
        _lib.orc_eq_push_batch.restype = C.c_int
        _lib.orc_eq_push_batch.argtypes = [P, P, P, P, P, P, C.c_uint64, C.c_int]
        _lib.orc_eq_pop.restype = C.c_int64
        _lib.orc_eq_pop.argtypes = [P, C.c_uint64, P, P, P, P, P, P, P, C.c_int]
        _lib.orc_eq_pending.restype = C.c_uint64
        _lib.orc_eq_pending.argtypes = [P, P, P, P, P, P]
        _lib.orc_max_threads.restype = C.c_int
        _lib.orc_xoshiro_seed.argtypes = [C.c_uint64, P]
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def routing(n_nodes, es, ed, el, ep, directed, used, shortest=True, variant=TIDY, threads=0,
            rows=None):
    """Returns (code, lat[r,n] u64, loss[r,n] f32, (err_a, err_b)); ``rows = (rb, re)`` builds
    only source rows [rb, re) of the used-node table (r = re - rb; default: all n rows)."""
    es = np.ascontiguousarray(es, np.uint32); ed = np.ascontiguousarray(ed, np.uint32)
    el = np.ascontiguousarray(el, np.uint64); ep = np.ascontiguousarray(ep, np.float32)
    used = np.ascontiguousarray(used, np.uint32)
    n = len(used)
    rb, re = (0, n) if rows is None else (int(rows[0]), int(rows[1]))
    lat = np.zeros((re - rb, n), np.uint64); loss = np.zeros((re - rb, n), np.float32)
    ea = np.zeros(1, np.uint32); eb = np.zeros(1, np.uint32)
    if shortest:
        rc = lib().orc_shortest_paths_rows(n_nodes, len(es), _p(es), _p(ed), _p(el), _p(ep),
                                           int(directed), _p(used), n, rb, re, variant, threads,
                                           _p(lat), _p(loss), _p(ea), _p(eb))
    else:
        rc = lib().orc_direct_paths(n_nodes, len(es), _p(es), _p(ed), _p(el), _p(ep),
                                    int(directed), _p(used), n, _p(lat), _p(loss), _p(ea), _p(eb))
    return CODES[rc], lat, loss, (int(ea[0]), int(eb[0]))


def next_hops(n_nodes, es, ed, el, ep, directed, used, lat, loss, rows=None, threads=0):
    """Next hops of table rows (the engine's definition; see oracle.c).  ``used`` must list every
    node; ``lat``/``loss`` are the rows [rb, re) of the table the oracle built."""
    used = np.ascontiguousarray(used, np.uint32)
    n = len(used)
    rb, re = (0, n) if rows is None else (int(rows[0]), int(rows[1]))
    out = np.zeros((re - rb, n), np.uint32)
    rc = lib().orc_next_hops(n_nodes, len(es), _p(np.ascontiguousarray(es, np.uint32)),
                             _p(np.ascontiguousarray(ed, np.uint32)), _p(np.ascontiguousarray(el, np.uint64)),
                             _p(np.ascontiguousarray(ep, np.float32)), int(directed), _p(used), n, rb, re,
                             _p(np.ascontiguousarray(lat, np.uint64)), _p(np.ascontiguousarray(loss, np.float32)),
                             threads, _p(out))
    assert rc == 0, "next_hops: used must list every node"
    return out


def relay_round(src_off, send_time, dst_host, payload, host_node, lat, loss, rng, next_id,
                round_end, sim_end, bootstrap_end, chance=None, threads=0, want_events=True):
    """C restatement of one relay round.  rng [H,4] and next_id [H] are updated in place."""
    n = len(send_time)
    H = len(src_off) - 1
    status = np.zeros(n, np.uint8); deliver = np.zeros(n, np.uint64); seq = np.zeros(n, np.uint64)
    mind = np.zeros(1, np.uint64); minl = np.zeros(1, np.uint64)
    out = None
    if want_events:
        out = dict(off=np.zeros(H + 1, np.uint32), deliver=np.zeros(n, np.uint64),
                   src=np.zeros(n, np.uint32), seq=np.zeros(n, np.uint64), pkt=np.zeros(n, np.uint32))
    nn = lat.shape[0]
    n_sent = lib().orc_relay_round(
        H, _p(np.ascontiguousarray(src_off, np.uint32)), _p(np.ascontiguousarray(send_time, np.uint64)),
        _p(np.ascontiguousarray(dst_host, np.uint32)), _p(np.ascontiguousarray(payload, np.uint32)),
        _p(None if chance is None else np.ascontiguousarray(chance, np.float64)),
        _p(np.ascontiguousarray(host_node, np.uint32)), nn, _p(np.ascontiguousarray(lat, np.uint64)),
        _p(np.ascontiguousarray(loss, np.float32)), _p(rng), _p(next_id), round_end, sim_end,
        bootstrap_end, threads, _p(status), _p(deliver), _p(seq), _p(mind), _p(minl),
        _p(out["off"]) if out else None, _p(out["deliver"]) if out else None,
        _p(out["src"]) if out else None, _p(out["seq"]) if out else None,
        _p(out["pkt"]) if out else None)
    if out:
        for k in ("deliver", "src", "seq", "pkt"):
            out[k] = out[k][:n_sent]
    return dict(status=status, deliver=deliver, seq=seq, min_deliver=int(mind[0]),
                min_latency=int(minl[0]), n_sent=int(n_sent), events=out)


def max_threads():
    return lib().orc_max_threads()


def codel_run(n_hosts, off, time, size, pkt, n_ids, threads=0):
    """C restatement of a CoDel batch on fresh queues -> (pop_out u32[n_ops], fate u64[n_ids])."""
    n = len(time)
    pop = np.zeros(n, np.uint32)
    fate = np.zeros(n_ids, np.uint64)
    lib().orc_codel_run(n_hosts, _p(np.ascontiguousarray(off, np.uint32)), _p(np.ascontiguousarray(time, np.uint64)),
                        _p(np.ascontiguousarray(size, np.uint32)), _p(np.ascontiguousarray(pkt, np.uint32)),
                        _p(pop), _p(fate), n_ids, threads)
    return pop, fate


def tb_run(capacity, increment, interval, last_refill, off, time, size, flags, threads=0):
    """C restatement of a token-bucket batch on fresh buckets -> (status u8, value u64, panics)."""
    n = len(time)
    st = np.zeros(n, np.uint8)
    val = np.zeros(n, np.uint64)
    a = [np.ascontiguousarray(x, np.uint64) for x in (capacity, increment, interval, last_refill)]
    k = lib().orc_tb_run(len(a[0]), *(_p(x) for x in a), _p(np.ascontiguousarray(off, np.uint32)),
                         _p(np.ascontiguousarray(time, np.uint64)), _p(np.ascontiguousarray(size, np.uint32)),
                         _p(np.ascontiguousarray(flags, np.uint8)), _p(st), _p(val), threads)
    return st, val, int(k)


class EventQueues:
    """C restatement of the per-host EventQueues (oracle/c/equeue.c: event_queue.rs:10-49,
    push_packet_to_host worker.rs:619-629, the pop loop of Host::execute host.rs:697-706)."""

    def __init__(self, n_hosts: int):
        self.n_hosts = int(n_hosts)
        self.h = lib().orc_eq_new(self.n_hosts)
        assert self.h, "orc_eq_new"

    def close(self):
        if self.h:
            lib().orc_eq_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:   # noqa: BLE001 -- interpreter shutdown
            pass

    def push_batch(self, off, deliver, src, seq, pkt, batch_no: int, threads=0):
        rc = lib().orc_eq_push_batch(self.h, _p(np.ascontiguousarray(off, np.uint32)),
                                     _p(np.ascontiguousarray(deliver, np.uint64)),
                                     _p(np.ascontiguousarray(src, np.uint32)), _p(np.ascontiguousarray(seq, np.uint64)),
                                     _p(np.ascontiguousarray(pkt, np.uint32)), int(batch_no), threads)
        assert rc == 0, "orc_eq_push_batch: out of memory"

    def pop(self, window_end: int, threads=0, want=True):
        """Every host's events below window_end -> dict(off, deliver, src, seq, tag, n_pending,
        next_time); next_time is 2**64-1 when every queue is empty."""
        npend, head = np.zeros(1, np.uint64), np.zeros(1, np.uint64)
        if not want:
            n = lib().orc_eq_pop(self.h, int(window_end), None, None, None, None, None, _p(npend), _p(head), threads)
            assert n >= 0, "EventQueue::pop: time moved backwards"
            return dict(n_popped=int(n), n_pending=int(npend[0]), next_time=int(head[0]))
        # the popped events land in per-host buffers first; two calls would pop twice, so size the
        # outputs by everything that could pop (all pending events)
        cap = int(lib().orc_eq_pending(self.h, None, None, None, None, None))
        off = np.zeros(self.n_hosts + 1, np.uint32)
        d = np.zeros(cap, np.uint64); s = np.zeros(cap, np.uint32)
        q = np.zeros(cap, np.uint64); t = np.zeros(cap, np.uint64)
        n = lib().orc_eq_pop(self.h, int(window_end), _p(off), _p(d), _p(s), _p(q), _p(t), _p(npend), _p(head),
                             threads)
        assert n >= 0, "EventQueue::pop: time moved backwards"
        return dict(off=off, deliver=d[:n], src=s[:n], seq=q[:n], tag=t[:n], n_popped=int(n),
                    n_pending=int(npend[0]), next_time=int(head[0]))

    def pending(self):
        n = int(lib().orc_eq_pending(self.h, None, None, None, None, None))
        off = np.zeros(self.n_hosts + 1, np.uint32)
        d = np.zeros(n, np.uint64); s = np.zeros(n, np.uint32)
        q = np.zeros(n, np.uint64); t = np.zeros(n, np.uint64)
        lib().orc_eq_pending(self.h, _p(off), _p(d), _p(s), _p(q), _p(t))
        return dict(off=off, deliver=d, src=s, seq=q, tag=t)


def relay_round_eq(src_off, send_time, dst_host, payload, host_node, lat, loss, rng, next_id,
                   round_end, sim_end, bootstrap_end, queues: EventQueues, batch_no: int, chance=None, threads=0):
    """One relay round whose sent packets are pushed into persistent C queues (the reference's
    push_packet_to_host).  rng / next_id are updated in place."""
    n = len(send_time)
    H = len(src_off) - 1
    status = np.zeros(n, np.uint8); deliver = np.zeros(n, np.uint64); seq = np.zeros(n, np.uint64)
    mind = np.zeros(1, np.uint64); minl = np.zeros(1, np.uint64)
    n_sent = lib().orc_relay_round_eq(
        H, _p(np.ascontiguousarray(src_off, np.uint32)), _p(np.ascontiguousarray(send_time, np.uint64)),
        _p(np.ascontiguousarray(dst_host, np.uint32)), _p(np.ascontiguousarray(payload, np.uint32)),
        _p(None if chance is None else np.ascontiguousarray(chance, np.float64)),
        _p(np.ascontiguousarray(host_node, np.uint32)), lat.shape[0], _p(np.ascontiguousarray(lat, np.uint64)),
        _p(np.ascontiguousarray(loss, np.float32)), _p(rng), _p(next_id), round_end, sim_end, bootstrap_end,
        threads, _p(status), _p(deliver), _p(seq), _p(mind), _p(minl), queues.h, int(batch_no))
    return dict(status=status, deliver=deliver, seq=seq, min_deliver=int(mind[0]), min_latency=int(minl[0]),
                n_sent=int(n_sent))
