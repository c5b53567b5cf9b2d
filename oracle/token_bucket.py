"""Token-bucket relay rate limiting, restated from the reference (test infrastructure only).

Restates ``src/main/network/relay/token_bucket.rs:6-157`` (FlyearthR/shadow): ``new_inner``
(None unless capacity, refill increment and refill interval are all non-zero), ``lazy_refill``
(whole elapsed refill intervals, tokens ``increment.saturating_mul(n)``, balance clamped to the
capacity, ``last_refill`` advanced by ``interval * n``), ``conforming_remove`` (the balance after
the removal, or the duration to the refill boundary after which the removal would conform) and
``compute_conforming_duration``; ``create_token_bucket`` (``relay/mod.rs:291-302``: 1 ms refill
interval, ``max(1, bytes_per_second / 1000)`` tokens per refill, capacity = that + CONFIG_MTU
1500, ``definitions.h:124``).

The batch replay (``relay_run``) restates the parts of ``Relay::forward_until_blocked``
(``relay/mod.rs:200-287``) and its Idle / Pending state (``:112-160``) that touch the bucket: a
packet that is local or sent while bootstrapping is forwarded without the bucket
(``:224-229``); a relay without a bucket (``RateLimit::Unlimited``) forwards everything; a
removal that does not conform blocks the relay until ``now + duration`` (``forward_later``),
and attempts before that time are not made (the relay is Pending).  Times are EmulatedTime ns.
"""
from __future__ import annotations

U64_MAX = (1 << 64) - 1
SIMTIME_MAX = 17500059273709551614           # simulation_time.rs:377
EMUTIME_MAX = U64_MAX - 1                    # emulated_time.rs:27
SIM_START = 946684800 * 1_000_000_000        # EmulatedTime::SIMULATION_START (emulated_time.rs:34)
MTU = 1500
MS = 1_000_000

FORWARDED, BLOCKED, SKIPPED = 0, 1, 2
EXEMPT = 1   # op flag: local packet or bootstrapping (no tokens taken)


class ReferencePanic(Exception):
    """Where the reference would panic (an unwrap on an out-of-range time)."""


def _simtime(v: int) -> int:
    """SimulationTime::from_c_simtime(v).unwrap() (simulation_time.rs:36-47)."""
    if v > SIMTIME_MAX:
        raise ReferencePanic("SimulationTime out of range")
    return v


def simtime_sat_mul(t: int, k: int) -> int:
    """SimulationTime::saturating_mul (simulation_time.rs:145-148)."""
    p = t * k
    return SIMTIME_MAX if p > U64_MAX else _simtime(p)


def simtime_sat_add(a: int, b: int) -> int:
    """SimulationTime::saturating_add (simulation_time.rs:135-138)."""
    s = a + b
    return SIMTIME_MAX if s > U64_MAX else _simtime(s)


def emutime_sat_add(t: int, d: int) -> int:
    """EmulatedTime::saturating_add (emulated_time.rs:95-108)."""
    s = t + d
    return EMUTIME_MAX if s > EMUTIME_MAX else s


def create_token_bucket(bytes_per_second: int) -> tuple[int, int, int]:
    """relay/mod.rs:291-302 -> (capacity, refill_increment, refill_interval_ns)."""
    refill = max(1, bytes_per_second // 1000)
    return refill + MTU, refill, MS


class TokenBucket:
    def __init__(self, capacity: int, refill_increment: int, refill_interval: int, last_refill: int):
        """new_inner (token_bucket.rs:37-60); ValueError where the reference returns None."""
        if not (capacity > 0 and refill_increment > 0 and refill_interval > 0):
            raise ValueError("token bucket needs a positive capacity, increment and interval")
        self.capacity = capacity
        self.balance = capacity
        self.refill_increment = refill_increment
        self.refill_interval = refill_interval
        self.last_refill = last_refill

    def lazy_refill(self, now: int) -> int:
        """token_bucket.rs:127-157; returns the span to the next refill."""
        if now < self.last_refill:
            raise ReferencePanic("duration_since: now before last_refill")
        span = now - self.last_refill
        if span >= self.refill_interval:
            n = span // self.refill_interval
            tokens = min(self.refill_increment * n, U64_MAX)         # u64::saturating_mul
            self.balance = min(min(self.balance + tokens, U64_MAX), self.capacity)
            inc = simtime_sat_mul(self.refill_interval, n)
            self.last_refill = emutime_sat_add(self.last_refill, inc)
            if now < self.last_refill:
                raise ReferencePanic("duration_since: now before last_refill")
            span = now - self.last_refill
        return self.refill_interval - span

    def compute_conforming_duration(self, decrement: int, next_refill_span: int) -> int:
        """token_bucket.rs:94-120."""
        req = max(decrement - self.balance, 0)
        n = req // self.refill_increment + (1 if req % self.refill_increment else 0)
        if n == 0:
            return 0
        if n == 1:
            return next_refill_span
        return simtime_sat_add(next_refill_span, simtime_sat_mul(self.refill_interval, n - 1))

    def conforming_remove(self, decrement: int, now: int) -> tuple[bool, int]:
        """token_bucket.rs:75-86: (True, balance) or (False, duration until conforming)."""
        nxt = self.lazy_refill(now)
        if self.balance >= decrement:
            self.balance -= decrement
            return True, self.balance
        return False, self.compute_conforming_duration(decrement, nxt)


def relay_run(buckets, pending, host_off, time, size, flags):
    """Replay a batch of forwarding attempts grouped by relay (each relay's in time order).

    ``buckets[r]`` is a TokenBucket or None (unlimited); ``pending[r]`` the time until which the
    relay is blocked (0: idle).  Returns (status list, value list): FORWARDED with the balance
    after the removal (U64_MAX without a bucket; the unchanged balance for an exempt packet),
    BLOCKED with the duration until the removal conforms, SKIPPED with the pending deadline.
    Mutates ``buckets`` and ``pending``."""
    n = len(time)
    status, value = [0] * n, [0] * n
    for r in range(len(host_off) - 1):
        tb = buckets[r]
        for k in range(int(host_off[r]), int(host_off[r + 1])):
            now = int(time[k])
            if now < pending[r]:
                status[k], value[k] = SKIPPED, pending[r]
            elif tb is None:
                status[k], value[k] = FORWARDED, U64_MAX
            elif int(flags[k]) & EXEMPT:
                status[k], value[k] = FORWARDED, tb.balance
            else:
                ok, v = tb.conforming_remove(int(size[k]), now)
                if ok:
                    status[k], value[k] = FORWARDED, v
                else:
                    status[k], value[k] = BLOCKED, v
                    pending[r] = emutime_sat_add(now, v)
    return status, value
