"""CPU oracle for the Shadow routing build and per-round packet relay.

TEST INFRASTRUCTURE ONLY.  This package restates, in plain Python/numpy (and in C under
``oracle/c``), the arithmetic of the reference's two hot paths so that the HIP product path
can be checked bit-for-bit.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker / the timed
CPU baseline.  The product path (``shadow_amd``) never imports, links or calls it.

Reference: FlyearthR/shadow (Shadow 3.0.0) at /root/reference.  Every function cites the
reference file:line it restates.  Third-party arithmetic restated from published algorithms
(absent from the reference tree, versions pinned by ``src/Cargo.lock``):
  * petgraph 0.6.3 ``algo::dijkstra``       (lazy-deletion binary-heap Dijkstra)
  * rand 0.8.5 ``Standard`` for f64/u64     (``(next_u64 >> 11) * 2^-53``)
  * rand_xoshiro 0.6.0 Xoshiro256++ / SplitMix64 ``seed_from_u64``
  * std ``DefaultHasher`` = SipHash-1-3 with zero keys; ``str::hash`` appends 0xFF
  * nom 7.1.3 combinators used by ``src/lib/gml-parser``

Pinning (see DESIGN.md "Oracle"): the routing restatement is pinned by the reference's own
known-answer tests (``src/main/network/graph/mod.rs:517-649``) and the units tests
(``src/main/core/support/units.rs:584-640``) and cross-checked against networkx Dijkstra and
brute-force path enumeration.  The RNG / SipHash streams and the relay event order have no
known-answer vector anywhere in the reference: those parts are **parity unpinned** (checked
only against published algorithm test vectors for SipHash-2-4 / SplitMix64 / Xoshiro256++).
"""
