"""Host-side mirror of the destination event queues (``EventQueue`` per host,
``src/main/core/work/event_queue.rs:10-49``; ``push_packet_to_host``, ``worker.rs:619-629``;
the pop loop of ``Host::execute``, ``host.rs:697-706``) kept on the MI355X engine.

``EventQueues(engine, n_hosts)``; ``advance(batch, window_end)`` merges a round's relay output
(device arrays) into the pending queues and returns, per host, every event with
``deliver < window_end`` in EventQueue order; the rest stays pending on the device.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native as N


@dataclass
class Popped:
    off: np.ndarray        # u32 [n_hosts + 1]
    deliver: np.ndarray    # u64
    src: np.ndarray        # u32
    seq: np.ndarray        # u64
    tag: np.ndarray        # u64: (batch number << 32) | packet index in that batch
    n_pending: int
    next_time: int         # earliest pending deliver time, 2**64-1 when none

    def events_for(self, h: int):
        a, b = int(self.off[h]), int(self.off[h + 1])
        return list(zip(self.deliver[a:b].tolist(), self.src[a:b].tolist(), self.seq[a:b].tolist(),
                        self.tag[a:b].tolist()))


class EventQueues:
    """``n_hosts`` = all hosts.  Under an engine communicator of > 1 ranks the queues hold this
    rank's destination shard [lo, hi) (shd_shard_range), and every per-host array -- a batch's
    ev_off, the popped ``off`` -- covers those hi - lo hosts (``self.n_local``)."""

    def __init__(self, engine, n_hosts: int):
        self.eng = engine
        self.n_hosts = int(n_hosts)
        w, r = C.c_int32(0), C.c_int32(0)
        N.check(engine.lib.shd_comm_info(engine.ctx, C.byref(w), C.byref(r)), "shd_comm_info")
        lo, hi = C.c_uint32(0), C.c_uint32(self.n_hosts)
        if w.value > 1:
            N.check(engine.lib.shd_shard_range(self.n_hosts, w.value, r.value, C.byref(lo), C.byref(hi)),
                    "shd_shard_range")
        self.lo, self.hi = lo.value, hi.value
        self.n_local = self.hi - self.lo
        N.check(engine.lib.shd_equeue_setup(engine.ctx, self.n_hosts), "shd_equeue_setup")

    def batch_buffers(self, max_events: int) -> N.RelayOut:
        """Engine-owned device arrays for the next relay output (``shd_equeue_batch_buffers``):
        pass them as that round's output and then to ``advance_device``, which adopts the batch
        without copying it.  The caller sets ``status`` before the relay call."""
        out = N.RelayOut()
        N.check(self.eng.lib.shd_equeue_batch_buffers(self.eng.ctx, int(max_events), C.byref(out)),
                "shd_equeue_batch_buffers")
        return out

    def advance_device(self, d_batch: N.RelayOut | None, window_end: int) -> N.EqueueOut:
        out = N.EqueueOut()
        N.check(self.eng.lib.shd_equeue_advance(self.eng.ctx, C.byref(d_batch) if d_batch is not None else None,
                                                int(window_end), C.byref(out)), "shd_equeue_advance")
        return out

    def advance(self, ev_off=None, deliver=None, src=None, seq=None, pkt=None, *, window_end: int) -> Popped:
        """Host arrays of one round's events grouped by destination (or none) -> popped events."""
        batch = None
        keep = []
        if ev_off is not None:
            import torch
            n = len(deliver)
            dev = lambda a, np_dt, dt: torch.from_numpy(np.ascontiguousarray(a, np_dt).view(dt)).cuda()  # noqa: E731
            keep = [dev(ev_off, np.uint32, np.int32), dev(deliver, np.uint64, np.int64),
                    dev(src, np.uint32, np.int32), dev(seq, np.uint64, np.int64), dev(pkt, np.uint32, np.int32)]
            batch = N.RelayOut(None, *(N.ptr(t).value for t in keep), 0, 0, n, len(ev_off) - 1, n)
        out = self.advance_device(batch, window_end)
        del keep
        return self.popped(out)

    def popped(self, out: N.EqueueOut) -> Popped:
        n = out.n_popped
        off = np.zeros(self.n_local + 1, np.uint32)
        d = np.zeros(n, np.uint64); s = np.zeros(n, np.uint32)
        q = np.zeros(n, np.uint64); t = np.zeros(n, np.uint64)
        N.check(self.eng.lib.shd_equeue_copy_popped(self.eng.ctx, N.ptr(off), N.ptr(d), N.ptr(s), N.ptr(q),
                                                    N.ptr(t)), "shd_equeue_copy_popped")
        return Popped(off, d, s, q, t, out.n_pending, out.next_time)

    def pending(self):
        n = C.c_uint64(0)
        N.check(self.eng.lib.shd_equeue_pending(self.eng.ctx, None, None, None, None, None, C.byref(n)),
                "shd_equeue_pending")
        k = n.value
        off = np.zeros(self.n_local + 1, np.uint32)
        d = np.zeros(k, np.uint64); s = np.zeros(k, np.uint32)
        q = np.zeros(k, np.uint64); t = np.zeros(k, np.uint64)
        N.check(self.eng.lib.shd_equeue_pending(self.eng.ctx, N.ptr(off), N.ptr(d), N.ptr(s), N.ptr(q), N.ptr(t),
                                                C.byref(n)), "shd_equeue_pending")
        return off, d, s, q, t
