"""Per-round inter-host packet relay restated in Python (test infrastructure only).

Restates, per staged send, ``Worker::send_packet`` (``src/main/core/worker.rs:328-413``):
  1. ``is_completed = now >= sim_end`` -> return: no RNG draw, no event, no status (:334-341);
  2. ``reliability = (1.0f32 - loss) as f64`` (``WorkerShared::reliability`` :538-543);
  3. ``chance = src_host.rng.gen::<f64>()`` -- one draw per non-completed send (:365);
  4. drop iff ``!bootstrapping && chance >= reliability && payload_size > 0`` (:370-378);
  5. ``deliver = max(now + latency, round_end)`` (:398-402); next-event min (:406);
     ``update_lowest_used_latency(latency)`` (:382);
  6. event key ``(deliver, Packet, src_host_id, src_host_event_id)`` pushed to the destination's
     queue; the event id is the source host's counter (``host.rs:580-584``) consumed only by
     sent packets (``Event::new_packet``, ``event.rs:20-31``).
Event order inside a destination queue: ``event.rs:84-155`` (time, then Packet<Local, then
src host id, then src event id).  Round reductions: ``worker.rs:314-322``,
``manager.rs:430-435,459-464``.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .rng import Xoshiro256PlusPlus

ST_SKIPPED = 0      # is_completed: send_packet returned before any effect
ST_DROPPED = 1      # PDS_INET_DROPPED
ST_SENT = 2         # PDS_INET_SENT, event pushed


@dataclass
class RelayResult:
    status: np.ndarray          # u8 per packet
    deliver: np.ndarray         # u64 per packet (0 unless SENT)
    seq: np.ndarray             # u64 per packet (event id; 0 unless SENT)
    rng_state: np.ndarray       # u64 [n_hosts, 4] after the round
    next_event_id: np.ndarray   # u64 [n_hosts] after the round
    events: dict                # dst_host -> list of (deliver, src_host, seq, pkt_idx), sorted
    min_deliver: int            # u64::MAX if nothing sent
    min_latency: int            # u64::MAX if nothing sent
    path_counts: dict           # (src_node, dst_node) -> count  (RoutingInfo counters)


U64_MAX = (1 << 64) - 1


def relay_round(send_time, src_host, dst_host, payload, host_node, lat, loss,
                rng_state, next_event_id, round_end, sim_end, bootstrap_end, chance=None):
    """Apply ``send_packet`` to every staged packet of one round, in batch order.

    ``lat``/``loss`` are the dense used-node table (row-major, ``host_node`` indexes it).
    Packets of one source host must appear in that host's send order (any interleaving of
    hosts is allowed).  ``chance`` (f64 per packet) replaces the device-side draw when the CPU
    drew at send time.
    """
    n = len(send_time)
    rngs = [Xoshiro256PlusPlus([int(v) for v in st]) for st in rng_state]
    eid = [int(v) for v in next_event_id]
    status = np.zeros(n, np.uint8)
    deliver = np.zeros(n, np.uint64)
    seq = np.zeros(n, np.uint64)
    events = {}
    counts = {}
    min_deliver = U64_MAX
    min_latency = U64_MAX
    one = np.float32(1.0)
    for i in range(n):
        now = int(send_time[i])
        if now >= sim_end:
            continue
        s, d = int(src_host[i]), int(dst_host[i])
        sn, dn = int(host_node[s]), int(host_node[d])
        reliability = float(np.float32(one - np.float32(loss[sn, dn])))
        c = float(chance[i]) if chance is not None else rngs[s].gen_f64()
        bootstrapping = now < bootstrap_end
        if (not bootstrapping) and c >= reliability and int(payload[i]) > 0:
            status[i] = ST_DROPPED
            continue
        delay = int(lat[sn, dn])
        min_latency = min(min_latency, delay)
        counts[(sn, dn)] = counts.get((sn, dn), 0) + 1
        t = now + delay
        if t < round_end:
            t = round_end
        status[i] = ST_SENT
        deliver[i] = t
        seq[i] = eid[s]
        eid[s] += 1
        min_deliver = min(min_deliver, t)
        events.setdefault(d, []).append((t, s, int(seq[i]), i))
    for d in events:
        events[d].sort(key=lambda ev: (ev[0], ev[1], ev[2]))
    return RelayResult(status, deliver, seq,
                       np.array([r.state() for r in rngs], np.uint64).reshape(-1, 4),
                       np.array(eid, np.uint64), events, min_deliver, min_latency, counts)


EMUTIME_MAX = U64_MAX - 1   # EmulatedTime::MAX (emulated_time.rs:27,47)


def next_window(min_next_event_time, runahead: int, end_time: int):
    """``SimController::manager_finished_current_round`` (controller.rs:86-111).  ``None`` as the
    minimum is the manager's ``unwrap_or(EmulatedTime::MAX)`` (manager.rs:459-464);
    ``checked_add`` fails past ``EMUTIME_MAX`` (``from_c_emutime``) and then gives ``MAX``."""
    assert runahead != 0
    start = EMUTIME_MAX if min_next_event_time is None else min(int(min_next_event_time), EMUTIME_MAX)
    end = start + runahead
    if end > EMUTIME_MAX:
        end = EMUTIME_MAX
    stop = min(end, end_time)
    return (start, stop) if start < stop else None


def runahead(min_used_latency, min_possible_latency: int, runahead_config) -> int:
    """``Runahead::get`` (runahead.rs:43-56); ``runahead_config`` None is ``ZERO``."""
    r = min_possible_latency if min_used_latency is None else min_used_latency
    return max(r, runahead_config or 0)


class RunaheadState:
    """``Runahead`` with ``update_lowest_used_latency`` (runahead.rs:58-115): the lowest latency of
    every sent packet, kept only when dynamic."""

    def __init__(self, dynamic: bool, min_possible_latency: int, runahead_config=None):
        assert min_possible_latency > 0
        self.dynamic, self.min_possible, self.cfg = dynamic, min_possible_latency, runahead_config
        self.min_used = None

    def update_lowest_used_latency(self, latency: int):
        assert latency > 0
        if self.dynamic and (self.min_used is None or latency < self.min_used):
            self.min_used = latency

    def get(self) -> int:
        return runahead(self.min_used, self.min_possible, self.cfg)


class EventQueues:
    """Per-host packet ``EventQueue`` (``src/main/core/work/event_queue.rs:10-49``): a min-heap
    of ``Reverse(Event)`` ordered by (time, Packet before Local, src host id, src event id)
    (``event.rs:84-155``; only packet events here), fed by ``push_packet_to_host``
    (``worker.rs:619-629``) and drained by ``Host::execute``'s pop loop: every event whose time is
    below the window end, in order (``host.rs:697-706``).  ``pop`` asserts time never goes
    backwards, as ``EventQueue::pop`` does (``event_queue.rs:36-40``)."""

    def __init__(self, n_hosts: int):
        import heapq
        self._hq = heapq
        self.q = [[] for _ in range(n_hosts)]
        self.last = [0] * n_hosts

    def push(self, dst: int, deliver: int, src: int, seq: int, tag):
        self._hq.heappush(self.q[dst], (int(deliver), int(src), int(seq), tag))

    def push_round(self, events: dict, batch_no: int):
        """A round's events (``RelayResult.events``: dst -> [(deliver, src, seq, pkt)])."""
        for d, evs in events.items():
            for t, s, q, p in evs:
                self.push(d, t, s, q, (batch_no << 32) | int(p))

    def next_event_time(self, h: int):
        return self.q[h][0][0] if self.q[h] else None

    def pop_until(self, h: int, window_end: int):
        out = []
        while self.q[h] and self.q[h][0][0] < window_end:
            ev = self._hq.heappop(self.q[h])
            assert ev[0] >= self.last[h], "EventQueue::pop: time moved backwards"
            self.last[h] = ev[0]
            out.append(ev)
        return out

    def pending(self, h: int):
        return sorted(self.q[h])
