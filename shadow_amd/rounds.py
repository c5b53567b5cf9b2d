"""Host-side mirror of the round bookkeeping kept in the engine: ``Runahead``
(``src/main/core/scheduler/runahead.rs:12-115``) and the next scheduling window
(``SimController::manager_finished_current_round``, ``controller.rs:86-111``).

``Runahead(engine, dynamic, min_possible_latency_ns, min_runahead_config_ns)`` mirrors
``Runahead::new`` (``manager.rs:246-251``); committed relay rounds update it on the device side
(``update_lowest_used_latency``, ``worker.rs:380``).  ``next_window(engine, cpu_next, end_time)``
is the manager's end-of-round step: the minimum over the caller's own next event time, the pending
destination queues and the last relay output not yet merged, reduced over every rank of the
engine's communicator.
"""
from __future__ import annotations

import ctypes as C

from . import _native as N

EMUTIME_MAX = (1 << 64) - 2      # EmulatedTime::MAX
NONE = (1 << 64) - 1             # "no event" (Option::None) at the ABI


class Runahead:
    def __init__(self, engine, dynamic: bool, min_possible_latency_ns: int = 0,
                 min_runahead_config_ns: int | None = None):
        self.eng = engine
        N.check(engine.lib.shd_runahead_setup(engine.ctx, 1 if dynamic else 0, int(min_possible_latency_ns),
                                              int(min_runahead_config_ns or 0)), "shd_runahead_setup")

    def get(self) -> int:
        """``Runahead::get`` (runahead.rs:43-56)."""
        r = C.c_uint64(0)
        N.check(self.eng.lib.shd_runahead_get(self.eng.ctx, C.byref(r)), "shd_runahead_get")
        return r.value


def next_window(engine, cpu_next_event_time: int | None, end_time: int):
    """(start, end) of the next round, or None when the simulation stops (controller.rs:92-111).
    Collective under an engine communicator of > 1 ranks."""
    s, e, run = C.c_uint64(0), C.c_uint64(0), C.c_int32(0)
    N.check(engine.lib.shd_round_window(engine.ctx, NONE if cpu_next_event_time is None else int(cpu_next_event_time),
                                        int(end_time), C.byref(s), C.byref(e), C.byref(run)), "shd_round_window")
    return (s.value, e.value) if run.value else None


def window_compute(min_next_event_time: int | None, runahead: int, end_time: int):
    """The window arithmetic alone (``shd_window_compute``; no GPU needed)."""
    lib = N.load()
    s, e, run = C.c_uint64(0), C.c_uint64(0), C.c_int32(0)
    N.check(lib.shd_window_compute(NONE if min_next_event_time is None else int(min_next_event_time), int(runahead),
                                   int(end_time), C.byref(s), C.byref(e), C.byref(run)), "shd_window_compute")
    return (s.value, e.value) if run.value else None
