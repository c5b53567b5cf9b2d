"""CoDel router queue, restated from the reference (test infrastructure only).

Restates ``src/main/network/router/codel_queue.rs:19-330`` (FlyearthR/shadow): TARGET 10 ms,
INTERVAL 100 ms, LIMIT unbounded, MTU 1500 (``definitions.h:124``); ``push``, ``pop`` with the
store/drop modes, ``codel_pop`` (RFC 8289 ``dodequeue``), ``process_standing_delay``,
``should_drop``, ``was_dropping_recently`` and ``apply_control_law``
(``time + round(INTERVAL / sqrt(count))`` in f64, saturating).  Times are EmulatedTime ns (u64);
``None`` options are kept as ``None``.  Packets are opaque ids with a total size in bytes.
"""
from __future__ import annotations

import math
from collections import deque

TARGET = 10_000_000
INTERVAL = 100_000_000
MTU = 1500
U64_MAX = (1 << 64) - 1
STORE, DROP = 0, 1


def _sat_add(a: int, b: int) -> int:
    return min(a + b, U64_MAX)


def _sat_sub(a: int, b: int) -> int:
    return max(a - b, 0)


def apply_control_law(time: int, count: int) -> int:
    """codel_queue.rs:272-286."""
    sqrt_count = 1.0 if count == 0 else math.sqrt(float(count))
    div = float(INTERVAL) / sqrt_count
    r = math.floor(div)                  # f64::round: half away from zero (div > 0 here)
    if div - r >= 0.5:
        r += 1
    return _sat_add(time, int(r))


class CoDelQueue:
    def __init__(self):
        self.elements = deque()        # (pkt, size, enqueue_ts)
        self.total_bytes_stored = 0
        self.mode = STORE
        self.interval_end = None
        self.drop_next = None
        self.current_drop_count = 0
        self.previous_drop_count = 0
        self.dropped = []              # packets dropped, in order

    def __len__(self):
        return len(self.elements)

    def push(self, pkt, size: int, now: int):
        """codel_queue.rs:291-306 (LIMIT = usize::MAX: never full)."""
        self.total_bytes_stored += size
        self.elements.append((pkt, size, now))

    def pop(self, now: int):
        """codel_queue.rs:125-147."""
        item = self._codel_pop(now)
        if item is None:
            self.mode = STORE
            return None
        pkt, ok_to_drop = item
        if not ok_to_drop:
            self.mode = STORE
            return pkt
        if self.mode == STORE:
            return self._drop_from_store_mode(now, pkt)
        return self._drop_from_drop_mode(now, pkt)

    def _drop_from_store_mode(self, now, pkt):
        """codel_queue.rs:149-170."""
        self.dropped.append(pkt)
        nxt = self._codel_pop(now)
        self.mode = DROP
        delta = _sat_sub(self.current_drop_count, self.previous_drop_count)
        self.current_drop_count = delta if (self._was_dropping_recently(now) and delta > 1) else 1
        self.drop_next = apply_control_law(now, self.current_drop_count)
        self.previous_drop_count = self.current_drop_count
        return None if nxt is None else nxt[0]

    def _drop_from_drop_mode(self, now, pkt):
        """codel_queue.rs:172-198."""
        item = (pkt, True)
        while item is not None and self.mode == DROP and self._should_drop(now):
            self.dropped.append(item[0])
            self.current_drop_count += 1
            item = self._codel_pop(now)
            if item is not None and item[1]:
                self.drop_next = apply_control_law(self.drop_next, self.current_drop_count)
            else:
                self.mode = STORE
        return None if item is None else item[0]

    def _codel_pop(self, now):
        """codel_queue.rs:201-223 (dodequeue)."""
        if not self.elements:
            self.interval_end = None
            return None
        pkt, size, ts = self.elements.popleft()
        self.total_bytes_stored = _sat_sub(self.total_bytes_stored, size)
        standing = _sat_sub(now, ts)
        return pkt, self._process_standing_delay(now, standing)

    def _process_standing_delay(self, now, standing):
        """codel_queue.rs:227-255."""
        if standing < TARGET or self.total_bytes_stored <= MTU:
            self.interval_end = None
            return False
        if self.interval_end is not None:
            return now >= self.interval_end
        self.interval_end = _sat_add(now, INTERVAL)
        return False

    def _should_drop(self, now):
        return self.drop_next is not None and now >= self.drop_next

    def _was_dropping_recently(self, now):
        return self.drop_next is not None and _sat_sub(now, self.drop_next) < INTERVAL * 16


def run_ops(n_hosts: int, host_off, time, size, pkt, queues=None):
    """Batch form used by the engine: per host, its ops in order (size == 0xFFFFFFFF: pop).
    Returns (queues, pop_out, fate) with fate: pkt -> (op index, 1 dequeued | 2 dropped)."""
    POP = 0xFFFFFFFF
    if queues is None:
        queues = [CoDelQueue() for _ in range(n_hosts)]
    pop_out = [POP] * len(time)
    fate = {}
    for h in range(n_hosts):
        q = queues[h]
        for k in range(int(host_off[h]), int(host_off[h + 1])):
            if int(size[k]) == POP:
                before = len(q.dropped)
                got = q.pop(int(time[k]))
                for d in q.dropped[before:]:
                    fate[d] = (k, 2)
                if got is not None:
                    pop_out[k] = got
                    fate[got] = (k, 1)
            else:
                q.push(int(pkt[k]), int(size[k]), int(time[k]))
    return queues, pop_out, fate
