"""Host-side mirror of the reference's CoDel router queue (``CoDelQueue``,
src/main/network/router/codel_queue.rs:60-330), batched over hosts on the MI355X engine.

``CoDelQueues(engine, n_hosts, capacity)`` keeps one queue per host on the device;
``run(host_off, time, size, pkt)`` replays a batch of push / pop operations grouped by host
(``size == POP`` marks a pop) and returns, per operation, the packet a pop dequeued and, per
packet, when it left the queue (dequeued or dropped).  No CPU fallback: without the native
library or a gfx950 GPU every call raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N

POP = 0xFFFFFFFF
STORE, DROP = 0, 1


class CoDelQueues:
    def __init__(self, engine, n_hosts: int, capacity: int = 4096):
        self.eng = engine
        self.n_hosts = int(n_hosts)
        N.check(engine.lib.shd_codel_setup(engine.ctx, self.n_hosts, int(capacity)), "shd_codel_setup")
        self._ids = 1   # packets still queued may come out of any later batch

    def run(self, host_off, time, size, pkt, n_ids: int | None = None):
        """Returns (pop_out[n_ops] u32, fate[n_ids] u64: (op << 2) | 1 dequeued / 2 dropped,
        0 = untouched).  Host arrays in, host arrays out."""
        import torch
        host_off = np.ascontiguousarray(host_off, np.uint32)
        time = np.ascontiguousarray(time, np.uint64)
        size = np.ascontiguousarray(size, np.uint32)
        pkt = np.ascontiguousarray(pkt, np.uint32)
        assert len(host_off) == self.n_hosts + 1 and int(host_off[-1]) == len(time) == len(size) == len(pkt)
        if np.any(size != POP):
            self._ids = max(self._ids, int(pkt[size != POP].max()) + 1)
        if n_ids is None:
            n_ids = self._ids
        dev = lambda a, dt: torch.from_numpy(a.view(dt)).cuda()  # noqa: E731
        d_off, d_time = dev(host_off, np.int32), dev(time, np.int64)
        d_size, d_pkt = dev(size, np.int32), dev(pkt, np.int32)
        pop_out = torch.empty(max(len(time), 1), dtype=torch.int32, device="cuda")
        fate = torch.zeros(max(n_ids, 1), dtype=torch.int64, device="cuda")
        ops = N.CodelOps(len(time), N.ptr(d_off).value, N.ptr(d_time).value, N.ptr(d_size).value,
                         N.ptr(d_pkt).value)
        st = self.eng.lib.shd_codel_run_device(self.eng.ctx, C.byref(ops), N.ptr(pop_out), N.ptr(fate),
                                               int(n_ids))
        torch.cuda.synchronize()
        N.check(st, "shd_codel_run_device")
        return (pop_out.cpu().numpy().view(np.uint32)[: len(time)].copy(),
                fate.cpu().numpy().view(np.uint64)[:n_ids].copy())

    def state(self, host: int) -> dict:
        s = N.CodelState()
        N.check(self.eng.lib.shd_codel_get_state(self.eng.ctx, int(host), C.byref(s)), "shd_codel_get_state")
        return {"len": s.len, "mode": s.mode,
                "interval_end": s.interval_end if s.has_interval_end else None,
                "drop_next": s.drop_next if s.has_drop_next else None,
                "current_drop_count": s.current_drop_count, "previous_drop_count": s.previous_drop_count,
                "total_bytes_stored": s.total_bytes_stored}
