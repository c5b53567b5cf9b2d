"""Host RNG streams and seed derivation (test infrastructure only).

Restated (published algorithms; crates absent from /root/reference, versions from
``src/Cargo.lock``):
  * rand_xoshiro 0.6.0 ``SplitMix64`` and ``Xoshiro256PlusPlus::{seed_from_u64, next_u64}``;
  * rand 0.8.5 ``Standard`` f64: ``(next_u64 >> 11) as f64 * 2^-53``;
  * std ``DefaultHasher`` (SipHash-1-3, k0 = k1 = 0); ``<str as Hash>::hash`` writes the bytes
    then ``write_u8(0xff)``.
Call sites restated: ``src/main/core/sim_config.rs:49-53`` (global seed ->
``randomness_for_seed_calc``), ``:223-244`` (host seed = randomness ^ hash(hostname)),
``src/main/host/host.rs:218`` (host RNG = ``seed_from_u64(node_seed)``),
``src/main/core/worker.rs:365`` (one ``gen::<f64>()`` per non-completed send).

Parity note: the reference holds no known-answer vector for any of these streams; the
restatement is checked against the algorithms' published test vectors only (parity unpinned).
"""
from __future__ import annotations

M64 = (1 << 64) - 1


def rotl(x: int, k: int) -> int:
    return ((x << k) | (x >> (64 - k))) & M64


class SplitMix64:
    def __init__(self, seed: int):
        self.x = seed & M64

    def next_u64(self) -> int:
        self.x = (self.x + 0x9E3779B97F4A7C15) & M64
        z = self.x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)


class Xoshiro256PlusPlus:
    def __init__(self, s):
        self.s = [v & M64 for v in s]

    @classmethod
    def seed_from_u64(cls, seed: int) -> "Xoshiro256PlusPlus":
        # rand_xoshiro: SplitMix64::seed_from_u64(seed) then from_rng -> fill 32 bytes LE
        sm = SplitMix64(seed)
        return cls([sm.next_u64() for _ in range(4)])

    def next_u64(self) -> int:
        s = self.s
        res = (rotl((s[0] + s[3]) & M64, 23) + s[0]) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = rotl(s[3], 45)
        return res

    def gen_f64(self) -> float:
        return (self.next_u64() >> 11) * (1.0 / (1 << 53))

    def state(self):
        return list(self.s)


def siphash(data: bytes, k0: int = 0, k1: int = 0, c_rounds: int = 1, d_rounds: int = 3) -> int:
    """SipHash-c-d (default 1-3 as Rust's DefaultHasher)."""
    v0 = k0 ^ 0x736F6D6570736575
    v1 = k1 ^ 0x646F72616E646F6D
    v2 = k0 ^ 0x6C7967656E657261
    v3 = k1 ^ 0x7465646279746573

    def rnd(v0, v1, v2, v3):
        v0 = (v0 + v1) & M64; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32)
        v2 = (v2 + v3) & M64; v3 = rotl(v3, 16); v3 ^= v2
        v0 = (v0 + v3) & M64; v3 = rotl(v3, 21); v3 ^= v0
        v2 = (v2 + v1) & M64; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32)
        return v0, v1, v2, v3

    n = len(data)
    tail_len = n % 8
    for off in range(0, n - tail_len, 8):
        m = int.from_bytes(data[off:off + 8], "little")
        v3 ^= m
        for _ in range(c_rounds):
            v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
        v0 ^= m
    b = ((n & 0xFF) << 56) | int.from_bytes(data[n - tail_len:], "little")
    v3 ^= b
    for _ in range(c_rounds):
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    v0 ^= b
    v2 ^= 0xFF
    for _ in range(d_rounds):
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    return v0 ^ v1 ^ v2 ^ v3


def hostname_hash(name: str) -> int:
    """``DefaultHasher`` over ``name.hash()`` = SipHash-1-3(bytes ++ 0xFF), zero keys."""
    return siphash(name.encode("utf-8") + b"\xff")


def randomness_for_seed_calc(seed: int) -> int:
    """``Xoshiro256PlusPlus::seed_from_u64(seed).gen::<u64>()`` (sim_config.rs:49-53)."""
    return Xoshiro256PlusPlus.seed_from_u64(seed).next_u64()


def host_seed(global_seed: int, hostname: str) -> int:
    """Host seed (sim_config.rs:223-244): randomness_for_seed_calc ^ hash(hostname)."""
    return randomness_for_seed_calc(global_seed) ^ hostname_hash(hostname)


def host_rng_state(global_seed: int, hostname: str):
    """Initial 4x u64 Xoshiro256++ state of a host's RNG (host.rs:218)."""
    return Xoshiro256PlusPlus.seed_from_u64(host_seed(global_seed, hostname)).state()
