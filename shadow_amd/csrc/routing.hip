// Routing build on gfx950: lexicographic (latency, loss) shortest paths into the dense
// used-node table, and the direct-path mode.
//
// Reference semantics (FlyearthR/shadow src/main/network/graph/mod.rs):
//   compute_shortest_paths :185-230 -- one petgraph Dijkstra per used source; the result of
//     each is the lexicographic minimum over walks of the LEFT-FOLDED path cost (latency u64
//     add; loss 1f32-(1f32-p)*(1f32-e), edge on the right).  Every non-loop edge strictly
//     increases latency and the fold is monotone, so the minimum is a unique fixed point: any
//     label-correcting relaxation that always appends one edge on the right converges to the
//     same bits as Dijkstra.  That is what the kernels below do (never segment composition,
//     which is not associative in f32 -- SURVEY F2).
//   diagonal := the node's single self-loop edge, raw loss (:212-219); unreachable -> panic
//     (:221); get_direct_paths :232-254 with get_edge_weight :258-295.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_ext.h>

#include "ctx.h"

namespace shd {

// ------------------------------------------------------------------------------------------
// Kernel 1: batched per-source SSSP, one workgroup per source row, labels in LDS.
// Label = packed u64 key (lat32 << 32 | f32 loss bits); ds_min_rtn_u64 keeps the lexicographic
// minimum exactly.  Active set = LDS bitmap; sweeps until a sweep improves nothing.
// Arcs are 16-byte AoS records {dst, lat32,
// q = 1f32 - loss bits, 0} so one dwordx4 load fetches an arc; a group of G lanes relaxes one
// active node's arcs together (G ~ average degree), so a node costs one load latency instead
// of `degree` dependent ones.  64/G nodes are in flight per wave, NW waves per source.
// ------------------------------------------------------------------------------------------
// delta = bucket width in ns for delta-stepping (SHD_ALGO_DELTA): a sweep only expands active
// nodes whose latency is <= (min active latency + delta), which keeps the expansion order close
// to Dijkstra's and cuts re-expansions.  delta = 0xFFFFFFFF expands every active node (plain
// chaotic Bellman-Ford).  Both converge to the same unique fixed point.
// Label loads: labels in LDS are read at workgroup scope; labels in global memory (kernel 1b)
// at agent scope, which bypasses the CU's L1 -- the L2 atomics never update it.
template <bool GLAB>
__device__ __forceinline__ uint64_t ld_lab(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED,
                             GLAB ? __HIP_MEMORY_SCOPE_AGENT : __HIP_MEMORY_SCOPE_WORKGROUP);
}

// delta-stepping bucket of a latency for the global-label kernel's LDS bucket bytes: any
// estimate works (it only orders the expansions), so a float multiply, saturating at 255
// The byte holds the latency in steps of delta / kBktSub: the sweeps schedule by byte >>
// kBktShift (delta-wide buckets) while the relax filter compares whole bytes, kBktSub times finer.
constexpr uint32_t kBktShift = 0, kBktSub = 1u << kBktShift;   // shift 2 (4x finer filter) measured no faster on C4
__device__ __forceinline__ uint8_t bucket_of(uint32_t lat, float inv_delta) {
    return (uint8_t)fminf(255.0f, (float)lat * inv_delta);
}

template <int G, int R, bool CACHE, bool GLAB>
__device__ __forceinline__ void relax_node(uint32_t u, uint32_t gl, uint64_t* lab, uint32_t* bits,
                                           uint32_t scratch, const uint2* rng, const uint32_t* offl,
                                           const uint32_t* __restrict__ abeg,
                                           const uint32_t* __restrict__ aend,
                                           const uint4* __restrict__ arcs, bool& ovf, bool& dirty,
                                           uint8_t* bkt, float inv_delta, uint32_t& mnext) {
    const uint64_t ku = ld_lab<GLAB>(&lab[u]);
    const uint32_t lu = key_lat(ku);
    const float qu = one_minus(key_loss(ku));
    const uint2 r = CACHE ? rng[u] : offl ? make_uint2(offl[u], offl[u + 1]) : make_uint2(abeg[u], aend[u]);
    for (uint32_t k0 = r.x + gl; k0 < r.y; k0 += G * R) {
        // R arc loads, then R label atomics, all issued back to back: the loads are clamped into
        // the node's range and the atomics are unconditional (a dead slot carries the +inf key,
        // which min leaves unchanged, aimed at the lane's own scratch label so no two lanes
        // collide), so no branch splits them and each group waits for one load and one LDS
        // round trip per R arcs instead of R of each
        uint4 a[R];
        bool live[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const uint32_t k = k0 + i * G;
            live[i] = k < r.y;
            a[i] = arcs[live[i] ? k : r.y - 1];
        }
        uint64_t cand[R], old[R];
        uint32_t tgt[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const uint32_t cl = lu + a[i].y;
            const bool ok = live[i] && a[i].y != kLat32Inf && cl >= lu && cl != kLat32Inf;
            if (live[i] && a[i].y != kLat32Inf && !ok) ovf = true;   // leaves u32: wide rerun
            cand[i] = ok ? pack_key(cl, fold_q(qu, __uint_as_float(a[i].z))) : kKeyInf;
            tgt[i] = ok ? a[i].x : scratch;
        }
        // global labels: they only decrease, so a candidate not below the label read now cannot
        // improve it; the read filters the device-scope atomics (few relaxations improve a label)
        if constexpr (GLAB) {   // global labels: no scratch slots, skip dead slots instead
            uint64_t cur[R];
#pragma unroll
            for (int i = 0; i < R; ++i) cur[i] = cand[i] != kKeyInf ? ld_lab<GLAB>(&lab[a[i].x]) : 0ull;
#pragma unroll
            for (int i = 0; i < R; ++i)
                old[i] = cand[i] < cur[i]
                             ? atomicMin(reinterpret_cast<unsigned long long*>(&lab[a[i].x]), (unsigned long long)cand[i])
                             : cur[i];
        } else {   // LDS labels: unconditional atomics, one LDS round trip for the R arcs (a
                   // filtering read first measured slower: C2 172 -> 205 us, C3 11.2 -> 13.5 ms)
#pragma unroll
            for (int i = 0; i < R; ++i)
                old[i] = atomicMin(reinterpret_cast<unsigned long long*>(&lab[tgt[i]]), (unsigned long long)cand[i]);
        }
        uint32_t imp = 0;
#pragma unroll
        for (int i = 0; i < R; ++i) imp |= (cand[i] < old[i] ? 1u : 0u) << i;
        if (imp) {
            dirty = true;
#pragma unroll
            for (int i = 0; i < R; ++i)
                if ((imp >> i) & 1u) {
                    uint32_t key = key_lat(cand[i]);
                    if (bkt) {
                        const uint8_t bk = bucket_of(key, inv_delta);
                        bkt[a[i].x] = bk;
                        key = bk >> kBktShift;
                    }
                    atomicOr(&bits[a[i].x >> 5], 1u << (a[i].x & 31));
                    mnext = min(mnext, key);
                }
        }
    }
}

// Padded arc lists (pruned dense graphs, prune_rows): every node's list is a multiple of
// kArcPad slots, the tail filled with no-op arcs {scratch label V + i, lat 0, q 0} whose
// candidate (lu, 1.0f) meets a scratch label holding 0.  The group then loads its G x R slots
// at immediate offsets from one address, with no clamp, liveness test or per-arc select, and
// the u32 overflow test is one compare per node: a label above lat_guard (2^32 - 2 - the
// largest arc latency) flags the build for the wide rerun before any add can wrap.  The
// kernel is issue-bound (C2 PMC: VALU pipe ~70% busy), so these per-arc instructions are the
// cost that matters.
constexpr uint32_t kArcPad = 64;
template <int G, int R, bool CACHE>
__device__ __forceinline__ void relax_node_pad(uint32_t u, uint32_t gl, uint64_t* lab, uint32_t* bits,
                                               const uint2* rng, const uint32_t* __restrict__ abeg,
                                               const uint32_t* __restrict__ aend,
                                               const uint4* __restrict__ arcs, uint32_t lat_guard,
                                               bool& ovf, bool& dirty, uint32_t& mnext) {
    static_assert(kArcPad % (G * R) == 0, "a padded list holds whole G x R steps");
    const uint64_t ku = lab[u];
    const uint32_t lu = key_lat(ku);
    if (lu > lat_guard) ovf = true;
    const float qu = one_minus(key_loss(ku));
    const uint2 r = CACHE ? rng[u] : make_uint2(abeg[u], aend[u]);
    for (uint32_t k0 = r.x; k0 < r.y; k0 += G * R) {
        const uint4* ap = arcs + k0 + gl;
        uint4 a[R];
#pragma unroll
        for (int i = 0; i < R; ++i) a[i] = ap[i * G];
        uint64_t cand[R], old[R];
#pragma unroll
        for (int i = 0; i < R; ++i) cand[i] = pack_key(lu + a[i].y, fold_q(qu, __uint_as_float(a[i].z)));
        // (a plain read first and the atomic only for a better candidate measured slower: C2 SSSP
        // 61 -> 66 us)
#pragma unroll
        for (int i = 0; i < R; ++i)
            old[i] = atomicMin(reinterpret_cast<unsigned long long*>(&lab[a[i].x]), (unsigned long long)cand[i]);
        uint32_t imp = 0;
#pragma unroll
        for (int i = 0; i < R; ++i) imp |= (cand[i] < old[i] ? 1u : 0u) << i;
        if (imp) {
            dirty = true;
#pragma unroll
            for (int i = 0; i < R; ++i)
                if ((imp >> i) & 1u) {
                    atomicOr(&bits[a[i].x >> 5], 1u << (a[i].x & 31));
                    mnext = min(mnext, key_lat(cand[i]));
                }
        }
    }
}

// LDS kernels on unpadded lists: a queued node of more than kHubDeg arcs is relaxed by its whole
// wave (sssp_row).  C3 (BA m = 3, 10k nodes), full build on one box: off 8.80-8.85 ms, 16: 7.27,
// 32: 7.02, 64: 7.18, 128: 7.62 (SHD_SSSP_HUB; 0 = off)
constexpr uint32_t kHubDeg = 32;
constexpr uint32_t kQCap = 64;   // per-wave expansion queue: flushed at kQCap, one scan step adds <= 64
constexpr uint32_t kQStride = kQCap + 64;
constexpr uint32_t kFlatWords = 257;   // per-wave scratch of expand_flat: pre[65], beg, lat, q [64]
constexpr int kFlatR = 8;              // arcs per lane per round of expand_flat

// Global labels: expand up to 64 queued nodes at once, edge-parallel.  The nodes' arc ranges
// are laid end to end (a wave prefix sum of the degrees) and every lane takes kFlatR arcs of
// the concatenation, so a round of the wave issues 64 x kFlatR independent arc loads, label
// reads and atomics -- one chain of global round trips per ~512 relaxations instead of one per
// node group.  The owner of an arc is the last node whose prefix is <= its position.  BA and
// internet-like graphs mix hubs and low-degree nodes; this keeps every lane busy on both.
template <bool GLAB>
__device__ __forceinline__ void expand_flat(const uint32_t* q, uint32_t qn, uint32_t lane, uint64_t* lab,
                                            uint32_t* bits, const uint2* rng, const uint32_t* __restrict__ abeg,
                                            const uint32_t* __restrict__ aend, const uint4* __restrict__ arcs,
                                            uint32_t* fx, bool& ovf, bool& dirty, uint8_t* bkt, float inv_delta,
                                            uint32_t scratch, uint32_t& mnext, const uint32_t* offl = nullptr) {
    uint32_t* pre = fx;          // [65]
    uint32_t* beg = fx + 65;     // [64]
    uint32_t* nl = fx + 129;     // [64] latency of the node's label
    uint32_t* nq = fx + 193;     // [64] q = 1f32 - loss of the node's label
    for (uint32_t c0 = 0; c0 < qn; c0 += 64) {
        const uint32_t cn = min(64u, qn - c0);
        uint32_t deg = 0, b = 0;
        uint64_t ku = kKeyInf;
        if (lane < cn) {
            const uint32_t u = q[c0 + lane];
            const uint2 r = rng ? rng[u] : offl ? make_uint2(offl[u], offl[u + 1]) : make_uint2(abeg[u], aend[u]);
            b = r.x;
            deg = r.y - b;
            ku = ld_lab<GLAB>(&lab[u]);
        }
        uint32_t incl = deg;
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const uint32_t T = __shfl(incl, 63);
        pre[lane] = incl - deg;
        beg[lane] = b;
        nl[lane] = key_lat(ku);
        nq[lane] = __float_as_uint(one_minus(key_loss(ku)));
        if (lane == 0) pre[64] = T;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t t0 = 0; t0 < T; t0 += 64 * kFlatR) {
            uint4 a[kFlatR];
            uint32_t lu[kFlatR];
            float qu[kFlatR];
            bool live[kFlatR];
#pragma unroll
            for (int r = 0; r < kFlatR; ++r) {
                const uint32_t t = t0 + r * 64 + lane;
                live[r] = t < T;
                const uint32_t tc = min(t, T - 1);   // dead slots load the last arc (in bounds)
                uint32_t lo = 0, hi = 64;   // last j with pre[j] <= tc (zero-degree nodes are skipped)
#pragma unroll
                for (int it = 0; it < 6; ++it) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (pre[mid] <= tc) lo = mid; else hi = mid;
                }
                lu[r] = nl[lo];
                qu[r] = __uint_as_float(nq[lo]);
                a[r] = arcs[beg[lo] + (tc - pre[lo])];
            }
            uint64_t cand[kFlatR], cur[kFlatR];
#pragma unroll
            for (int r = 0; r < kFlatR; ++r) {
                const uint32_t cl = lu[r] + a[r].y;
                const bool ok = live[r] && a[r].y != kLat32Inf && cl >= lu[r] && cl != kLat32Inf;
                if (live[r] && a[r].y != kLat32Inf && !ok) ovf = true;   // leaves u32: wide rerun
                cand[r] = ok ? pack_key(cl, fold_q(qu[r], __uint_as_float(a[r].z))) : kKeyInf;
            }
            if constexpr (GLAB) {
                // bucket-byte filter: bkt[v] >= the bucket of v's label (it is written only by a
                // relaxation that just lowered the label, and the label only falls further), so
                // a candidate in a higher bucket cannot improve it -- skip its global label read
                // (most relaxations of a sparse graph fail; the byte is in LDS)
                if (bkt) {
#pragma unroll
                    for (int r = 0; r < kFlatR; ++r)
                        if (cand[r] != kKeyInf && bucket_of(key_lat(cand[r]), inv_delta) > bkt[a[r].x]) cand[r] = kKeyInf;
                }
#pragma unroll
                for (int r = 0; r < kFlatR; ++r) cur[r] = cand[r] != kKeyInf ? ld_lab<true>(&lab[a[r].x]) : 0ull;
#pragma unroll
                for (int r = 0; r < kFlatR; ++r) {
                    // labels only decrease: a candidate not below the label read now cannot improve it
                    if (cand[r] < cur[r]) {
                        const uint64_t old =
                            atomicMin(reinterpret_cast<unsigned long long*>(&lab[a[r].x]), (unsigned long long)cand[r]);
                        if (cand[r] < old) {
                            dirty = true;
                            if (bkt) {
                                const uint8_t bk = bucket_of(key_lat(cand[r]), inv_delta);
                                bkt[a[r].x] = bk;
                                mnext = min(mnext, (uint32_t)(bk >> kBktShift));
                            }
                            atomicOr(&bits[a[r].x >> 5], 1u << (a[r].x & 31));
                        }
                    }
                }
            } else {   // LDS labels: unconditional atomics (dead slots hit the lane's scratch label)
#pragma unroll
                for (int r = 0; r < kFlatR; ++r)
                    cur[r] = atomicMin(reinterpret_cast<unsigned long long*>(&lab[cand[r] != kKeyInf ? a[r].x : scratch]),
                                       (unsigned long long)cand[r]);
                uint32_t imp = 0;
#pragma unroll
                for (int r = 0; r < kFlatR; ++r) imp |= (cand[r] < cur[r] ? 1u : 0u) << r;
                if (imp) {
                    dirty = true;
#pragma unroll
                    for (int r = 0; r < kFlatR; ++r)
                        if ((imp >> r) & 1u) {
                            atomicOr(&bits[a[r].x >> 5], 1u << (a[r].x & 31));
                            mnext = min(mnext, key_lat(cand[r]));
                        }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// expand_flat for the global-label kernel on compact arcs: {dst, lat} (8 B) per arc, q = 1f32 -
// loss in a side array read only by the relaxations that survive the bucket-byte filter.  Most
// relaxations of a sparse graph fail, so the arc stream a sweep reads halves and (C4: 400k arcs,
// 3.2 MB) fits one XCD's L2.
__device__ __forceinline__ void expand_flat8(const uint32_t* q, uint32_t qn, uint32_t lane, uint64_t* lab,
                                             uint32_t* bits, const uint32_t* __restrict__ abeg,
                                             const uint32_t* __restrict__ aend, const uint2* __restrict__ arcs8,
                                             const float* __restrict__ aq, uint32_t* fx, bool& ovf, bool& dirty,
                                             uint8_t* bkt, float inv_delta, uint32_t& mnext, uint64_t* llab,
                                             uint32_t kl, uint32_t* wmin) {
    uint32_t* pre = fx;          // [65]
    uint32_t* beg = fx + 65;     // [64]
    uint32_t* nl = fx + 129;     // [64] latency of the node's label
    uint32_t* nq = fx + 193;     // [64] q = 1f32 - loss of the node's label
    for (uint32_t c0 = 0; c0 < qn; c0 += 64) {
        const uint32_t cn = min(64u, qn - c0);
        uint32_t deg = 0, b = 0;
        uint64_t ku = kKeyInf;
        if (lane < cn) {
            const uint32_t u = q[c0 + lane];
            b = abeg[u];
            deg = aend[u] - b;
            ku = u < kl ? llab[u] : ld_lab<true>(&lab[u]);
        }
        uint32_t incl = deg;
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const uint32_t T = __shfl(incl, 63);
        pre[lane] = incl - deg;
        beg[lane] = b;
        nl[lane] = key_lat(ku);
        nq[lane] = __float_as_uint(one_minus(key_loss(ku)));
        if (lane == 0) pre[64] = T;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t t0 = 0; t0 < T; t0 += 64 * kFlatR) {
            uint2 a[kFlatR];
            uint32_t lu[kFlatR], k[kFlatR], cl[kFlatR];
            float qu[kFlatR];
            bool ok[kFlatR], sure[kFlatR];
            // (every round issues all kFlatR slots: skipping a short last round's empty slots
            // behind wave-uniform branches measured slower, C4 rows 0-4095 17.2 -> 18.2 ms)
#pragma unroll
            for (int r = 0; r < kFlatR; ++r) {
                const uint32_t t = t0 + r * 64 + lane;
                ok[r] = t < T;
                const uint32_t tc = min(t, T - 1);   // dead slots load the last arc (in bounds)
                uint32_t lo = 0, hi = 64;   // last j with pre[j] <= tc (zero-degree nodes are skipped)
#pragma unroll
                for (int it = 0; it < 6; ++it) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (pre[mid] <= tc) lo = mid; else hi = mid;
                }
                lu[r] = nl[lo];
                qu[r] = __uint_as_float(nq[lo]);
                k[r] = beg[lo] + (tc - pre[lo]);
                a[r] = arcs8[k[r]];
            }
#pragma unroll
            for (int r = 0; r < kFlatR; ++r) {
                cl[r] = lu[r] + a[r].y;
                const bool fit = cl[r] >= lu[r] && cl[r] != kLat32Inf;
                if (ok[r] && !fit) ovf = true;   // leaves u32: wide rerun
                // bucket-byte filter (see expand_flat): a higher bucket cannot improve the label;
                // a strictly lower one surely does (bkt >= the label's bucket), so its atomic
                // goes out without the filtering read -- one global round trip less on the
                // flush's chain (C4 rows 0-4095: 19.3 -> 17.6 ms)
                const uint32_t bq = bucket_of(cl[r], inv_delta), bv = bkt[a[r].x];
                ok[r] = ok[r] && fit && bq <= bv;
                sure[r] = bq < bv;
            }
            uint64_t cur[kFlatR];
            float qa[kFlatR];
#pragma unroll
            for (int r = 0; r < kFlatR; ++r) {
                cur[r] = !ok[r] ? 0ull : a[r].x < kl ? llab[a[r].x] : sure[r] ? kKeyInf : ld_lab<true>(&lab[a[r].x]);
                qa[r] = ok[r] ? aq[k[r]] : 0.0f;
            }
#pragma unroll
            for (int r = 0; r < kFlatR; ++r) {
                if (!ok[r]) continue;
                const uint64_t cand = pack_key(cl[r], fold_q(qu[r], qa[r]));
                // labels only decrease: a candidate not below the label read now cannot improve it
                if (cand < cur[r]) {
                    // the hottest nodes' labels live in LDS (kl, locality order: highest degree
                        // first), the rest in the slot's global row
                    const uint64_t old =
                        a[r].x < kl ? atomicMin(reinterpret_cast<unsigned long long*>(&llab[a[r].x]), (unsigned long long)cand)
                                    : atomicMin(reinterpret_cast<unsigned long long*>(&lab[a[r].x]), (unsigned long long)cand);
                    if (cand < old) {
                        dirty = true;
                        const uint8_t bk = (uint8_t)bucket_of(cl[r], inv_delta);
                        bkt[a[r].x] = bk;
                        mnext = min(mnext, (uint32_t)(bk >> kBktShift));
                        atomicOr(&bits[a[r].x >> 5], 1u << (a[r].x & 31));
                        // after the bit (sssp_row's word scan relies on this order): a release,
                        // so neither the compiler nor the LDS queue lets the minimum go first
                        if (wmin)
                            __hip_atomic_fetch_min(&wmin[a[r].x >> 5], (uint32_t)(bk >> kBktShift), __ATOMIC_RELEASE,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

#ifdef SHD_SSSP_PROF
// tuning builds only (tools/sssp_prof.py): shader clocks per phase of the padded-list kernel,
// summed over waves: init, bitmap scan, relaxation (flush), sweep end (reduce + barrier), output
__device__ unsigned long long g_sssp_prof[8];
#define SS_MARK(slot) do { if (true) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    ss_acc[slot] += t_ - ss_t; ss_t = t_; } } while (0)
// prune_rows: shader clocks per phase summed over workgroups (thread 0): row load + max, histogram,
// boundary bin, detour selection, 2-hop tests, list write; [6] first start, [7] last end (100 MHz)
__device__ unsigned long long g_prune_prof[4096 * 8];   // per workgroup (row u < 4096)
#define PR_MARK(slot) do { if (threadIdx.x == 0) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    pr_acc[slot] += t_ - pr_t; pr_t = t_; } } while (0)
#else
#define SS_MARK(slot) do { } while (0)
#define PR_MARK(slot) do { } while (0)
#endif

// One source row: init, sweeps until nothing improves, emit the used columns.
// FASTG (global labels): flat expansion + bucket bytes + one-barrier delta sweeps only (C4)
template <int BLOCK, int G, int R, bool CACHE, bool GLAB, int PADR = 0, bool FASTG = false, bool FLATL = false>
__device__ __forceinline__ void sssp_row(
    uint64_t* lab, uint32_t* bits, uint32_t* ctl, uint32_t* wq, uint2* rng,
    const uint32_t* __restrict__ abeg, const uint32_t* __restrict__ aend,
    const uint4* __restrict__ arcs, uint32_t V, const uint32_t* __restrict__ used,
    uint32_t n_used, uint32_t row, size_t orow, const uint64_t* __restrict__ diag_lat,
    const float* __restrict__ diag_loss, uint64_t* __restrict__ out_lat,
    float* __restrict__ out_loss, uint32_t* __restrict__ flags,
    unsigned long long* __restrict__ unreach, uint32_t delta,
    unsigned long long* __restrict__ stats, const uint32_t* __restrict__ seed_lat,
    uint32_t seed_stride, uint8_t* bkt, uint32_t* flat, uint32_t* nh_out, uint32_t* pred,
    uint32_t lat_guard, const uint2* __restrict__ arcs8 = nullptr, const float* __restrict__ aq = nullptr,
    uint32_t* offl = nullptr, uint64_t* llab = nullptr, uint32_t kl = 0, uint32_t* wmin = nullptr,
    uint32_t hub_deg = 0) {
    // bkt (global labels + delta-stepping): per node, the bucket of the latency that last
    // activated it, in LDS, so choosing a sweep's nodes reads no global label
    constexpr uint32_t NW = BLOCK / 64, NG = 64 / G;
    const uint32_t W = (V + 31) >> 5;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t grp = lane / G, gl = lane % G;
    uint32_t* q = wq + wave * kQStride;
    // (LDS kernels: nullptr = every node used, in index order; the global-label kernel always
    // passes the array -- a runtime check there cost the one VGPR above 128 that halves its
    // residency: C4 rows 0-4095 17.3 -> 27.2 ms)
    uint32_t src;
    if constexpr (GLAB) src = used[row];
    else src = used ? used[row] : row;
#ifdef SHD_SSSP_PROF
    uint64_t ss_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ss_t = __builtin_amdgcn_s_memtime();
#endif
    // PADR kernels run only delta-stepping with one-barrier sweeps and no seed (launch_group)
    const bool use_delta = PADR != 0 || FASTG || delta != kLat32Inf;
    // bucket bytes count steps of delta / kBktSub (global labels); the LDS kernels do not use them
    const float inv_delta = use_delta ? (float)kBktSub / (float)delta : 0.0f;
    // the ordering key of an active node: its bucket byte, or its label's latency
    auto act_key = [&](uint32_t v) -> uint32_t {
        // LDS labels: the latency half only, a 4-byte read (C3 DELTA 6.86 -> 6.79 ms; the 64-bit
        // atomics write both halves at once, so the half read is always one label's latency)
        if constexpr (!GLAB && !FASTG)
            if (!bkt)
                return __hip_atomic_load(reinterpret_cast<const uint32_t*>(&lab[v]) + 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
        return FASTG || bkt ? (uint32_t)(bkt[v] >> kBktShift) : key_lat(ld_lab<GLAB>(&lab[v]));
    };

    // seed_lat (blocked path): labels start at (final latency, +inf loss) so only the loss
    // part can still improve, and only through tight arcs
    const uint32_t* seed = PADR == 0 && seed_lat ? seed_lat + (size_t)src * seed_stride : nullptr;
    for (uint32_t v = tid; v < V; v += BLOCK) {
        uint64_t l0 = kKeyInf;
        if (seed) {
            const uint32_t d = seed[v];
            if (d != kLat32Inf) l0 = ((uint64_t)d << 32) | 0xFFFFFFFFull;
        }
        if (GLAB) {
            if (v == src) l0 = 0;   // PathProperties::default() = (0 ns, 0.0)
            if (v < kl) llab[v] = l0;
            else __hip_atomic_store(&lab[v], l0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            lab[v] = l0;
        }
        if (CACHE) rng[v] = make_uint2(abeg[v], aend[v]);
        else if (offl) offl[v] = abeg[v];
    }
    for (uint32_t w = tid; w < W; w += BLOCK) bits[w] = 0;
    if (wmin)   // per bitmap word, a lower bound of its active nodes' bucket keys (none: +inf)
        for (uint32_t w = tid; w < W; w += BLOCK) wmin[w] = w == (src >> 5) ? 0u : kLat32Inf;
    if (bkt)   // unreached: the top bucket (the relax filter never skips against it)
        for (uint32_t w = tid; w < (V + 3) / 4; w += BLOCK) reinterpret_cast<uint32_t*>(bkt)[w] = 0xFFFFFFFFu;
    if (offl && tid == 0) offl[V] = aend[V - 1];   // CSR: aend == abeg + 1
    if (!GLAB && tid < 64) lab[V + tid] = 0;   // scratch labels: no candidate improves them
    // global labels: every storing wave drains its stores before the barrier, so the L2 holds
    // them before any wave's atomics
    if (GLAB) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // One-barrier sweeps (LDS labels + delta-stepping): the next sweep's bucket floor is the
    // minimum over the nodes still active after this one -- those the selection skipped, and
    // those a relaxation just improved -- gathered while the sweep runs, so no separate scan
    // and only one barrier per sweep.  Three rotating accumulators ctl[1..3]: sweep k writes
    // slot k%3, all read it after the barrier, and sweep k resets slot (k+1)%3, whose last
    // readers passed the barrier of sweep k-1.  A floor taken from a node that the same sweep
    // then expands is only lower than needed: the next sweep selects less, never wrongly.
    const bool fused = PADR != 0 || FASTG || (use_delta && (!GLAB || bkt));
    if (tid == 0) {
        if (!GLAB) lab[src] = 0;  // PathProperties::default() = (0 ns, 0.0)
        bits[src >> 5] = 1u << (src & 31);
        if (bkt) bkt[src] = 0;
        if (fused) ctl[1] = ctl[2] = ctl[3] = kLat32Inf;
    }
    if (fused) __syncthreads();
    SS_MARK(0);
    bool ovf = false;
    uint32_t expanded = 0, sweeps = 0;
    uint32_t slot = 0;   // fused: this sweep's accumulator, ctl[1 + slot]
    for (;;) {
        uint32_t thr = kLat32Inf;
        uint32_t mnext = kLat32Inf;   // fused: lowest latency active after this sweep (this lane)
        if (fused) {
            const uint32_t lo = sweeps == 0 ? 0u : ctl[1 + (slot + 2) % 3];
            if (lo == kLat32Inf) break;  // no active node anywhere
            if (tid == 0) ctl[1 + (slot + 1) % 3] = kLat32Inf;
            thr = bkt ? lo : lo + delta < lo ? kLat32Inf - 1 : lo + delta;
        } else {
            if (tid == 0) {
                ctl[0] = 0;
                ctl[1] = kLat32Inf;
            }
            __syncthreads();
        }
        if (use_delta && !fused) {
            uint32_t m = kLat32Inf;
            for (uint32_t widx = lane * NW + wave; widx < W; widx += NW * 64) {   // lane per word
                const uint32_t word = __hip_atomic_load(&bits[widx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                for (uint32_t mm = word; mm; mm &= mm - 1) m = min(m, act_key(widx * 32 + __builtin_ctz(mm)));
            }
            for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o));
            if (lane == 0 && m != kLat32Inf) atomicMin(&ctl[1], m);
            __syncthreads();
            const uint32_t lo = ctl[1];
            if (lo == kLat32Inf) break;  // no active node anywhere
            thr = bkt ? lo : lo + delta < lo ? kLat32Inf - 1 : lo + delta;
        }
        bool dirty = false;
        uint32_t qn = 0;  // wave-uniform queue length
        // expand the queued nodes: NG nodes per step, G lanes each (or edge-parallel, global labels)
        auto flush = [&]() {
            SS_MARK(1);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            expanded += qn;
            if constexpr (GLAB) {
                if constexpr (FASTG) {
                    expand_flat8(q, qn, lane, lab, bits, abeg, aend, arcs8, aq, flat + wave * kFlatWords, ovf, dirty,
                                 bkt, inv_delta, mnext, llab, kl, wmin);
                } else if (flat) {
                    expand_flat<GLAB>(q, qn, lane, lab, bits, nullptr, abeg, aend, arcs, flat + wave * kFlatWords,
                                      ovf, dirty, bkt, inv_delta, V + lane, mnext);
                } else {
                    for (uint32_t t = 0; t < qn; t += NG) {
                        const uint32_t qi = t + grp;
                        if (qi < qn)
                            relax_node<G, R, CACHE, GLAB>(q[qi], gl, lab, bits, V + lane, rng, offl, abeg, aend, arcs,
                                                          ovf, dirty, bkt, inv_delta, mnext);
                    }
                }
            } else if constexpr (FLATL) {   // LDS labels, edge-parallel (sparse graphs with hubs)
                expand_flat<false>(q, qn, lane, lab, bits, CACHE ? rng : nullptr, abeg, aend, arcs,
                                   flat + wave * kFlatWords, ovf, dirty, nullptr, inv_delta, V + lane, mnext, offl);
            } else {
                if constexpr (PADR == 0 && !GLAB) {
                    // hubs (sparse power-law graphs, C3): a queued node of more than hub_deg arcs is
                    // relaxed by the whole wave first, 128 arcs per step, instead of by one lane group
                    // that the other groups of the wave -- and the sweep's other waves at its
                    // barrier -- would wait for
                    if (hub_deg) {
                        for (uint32_t t0 = 0; t0 < qn; t0 += 64) {
                            const uint32_t qi = t0 + lane;
                            const uint32_t u = qi < qn ? q[qi] : 0xFFFFFFFFu;
                            uint32_t deg = 0;
                            if (u != 0xFFFFFFFFu) {
                                const uint2 r = CACHE ? rng[u] : offl ? make_uint2(offl[u], offl[u + 1])
                                                                      : make_uint2(abeg[u], aend[u]);
                                deg = r.y - r.x;
                            }
                            uint64_t big = __ballot(deg > hub_deg);
                            while (big) {   // wave-uniform
                                const uint32_t b = (uint32_t)__ffsll((unsigned long long)big) - 1u;
                                big &= big - 1ull;
                                relax_node<64, 2, CACHE, GLAB>((uint32_t)__shfl((int)u, (int)b), lane, lab, bits,
                                                               V + lane, rng, offl, abeg, aend, arcs, ovf, dirty,
                                                               bkt, inv_delta, mnext);
                            }
                            if (deg > hub_deg) q[qi] = 0xFFFFFFFFu;   // done: the group pass skips it
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
                }
                for (uint32_t t = 0; t < qn; t += NG) {
                    const uint32_t qi = t + grp;
                    if (qi >= qn) continue;
                    if constexpr (PADR != 0) {   // padded lists: a whole 64-slot list per group step
                        relax_node_pad<G, PADR, CACHE>(q[qi], gl, lab, bits, rng, abeg, aend, arcs, lat_guard,
                                                       ovf, dirty, mnext);
                    } else {
                        const uint32_t u = q[qi];
                        if (u != 0xFFFFFFFFu)
                            relax_node<G, R, CACHE, GLAB>(u, gl, lab, bits, V + lane, rng, offl, abeg, aend, arcs,
                                                          ovf, dirty, bkt, inv_delta, mnext);
                    }
                }
            }
            qn = 0;
            __builtin_amdgcn_wave_barrier();
            SS_MARK(2);
        };
        // scan form: padded-list kernels (dense graphs, V <= kPruneMaxV) only the small-bitmap
        // one, global-label kernels (large V) only the lane-per-word one, so each kernel carries
        // one loop (fewer registers)
        // (plain chaotic sweeps, no delta, keep the word-per-step form: C3 SSSP 11.2 ms against
        // 17.4 with lane-per-word, whose frontier there is dense)
#ifndef SHD_SCAN_WORDSTEP   // (tuning A/B: the LDS kernels back on the word-per-step / lane-per-word scans)
        constexpr int kScan = GLAB ? 2 : 3;   // 3 nibbles (LDS labels), 2 lane per word (global labels)
#else
        constexpr int kScan = PADR != 0 ? 1 : GLAB ? 2 : 0;
#endif
        const bool lane_scan = kScan == 2 || (kScan == 0 && use_delta && W > NW * 16);
        // (plain chaotic sweeps on an unpruned graph keep the word-per-step form: C2 SSSP 2.65 ms
        // against 2.95 with nibbles; the seeded loss pass of the blocked engine takes nibbles)
        if (kScan == 3 && (use_delta || seed)) {
            // bits in parallel (LDS labels; C2: 32 words over 4 waves, C3: 313 over 16): a wave
            // takes 8 of its words at once, each lane 4 bits of one, so the key reads of all 8
            // words are in flight together -- one LDS round trip per 256 bits instead of one per
            // word step (the word-per-step form used half the lanes, one word at a time; the
            // lane-per-word form walked a word's bits one dependent read after another)
            for (uint32_t k0 = 0;; k0 += 8) {
                const bool more = k0 * NW + wave < W;   // wave-uniform
                const uint32_t widx = (k0 + (lane >> 3)) * NW + wave, nb = (lane & 7) * 4;
                uint32_t sel4 = 0;
                if (more && widx < W) {
                    const uint32_t word = __hip_atomic_load(&bits[widx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    const uint32_t nib = (word >> nb) & 0xFu;
                    uint32_t key[4];
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i)
                        key[i] = (nib >> i) & 1u ? (use_delta ? act_key(widx * 32 + nb + i) : 0u) : kLat32Inf;
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        if (!((nib >> i) & 1u)) continue;   // (thr is +inf in plain chaotic sweeps)
                        if (key[i] <= thr) sel4 |= 1u << i;
                        else mnext = min(mnext, key[i]);
                    }
                    // words are owned by one wave; other waves only set bits: clearing is exact
                    if (sel4) atomicAnd(&bits[widx], ~(sel4 << nb));
                }
#pragma unroll
                for (uint32_t i = 0; i < 4; ++i) {
                    const bool has = (sel4 >> i) & 1u;
                    const uint64_t bal = __ballot(has);
                    if (bal == 0) continue;   // wave-uniform
                    if (has) q[qn + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = widx * 32 + nb + i;
                    qn += (uint32_t)__popcll(bal);
                    if (qn >= kQCap) flush();
                }
                if (!more) {
                    if (qn > 0) flush();
                    break;
                }
            }
        } else if (!lane_scan) {
            // small bitmap (C2: 32 words over 4 waves): a word per wave step, lane per bit
            for (uint32_t widx = wave;; widx += NW) {
                const bool more = widx < W;
                if (more) {
                    const uint32_t word = __hip_atomic_load(&bits[widx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (word != 0) {  // wave-uniform
                        bool sel = lane < 32 && ((word >> lane) & 1u);
                        if (use_delta && sel) {
                            const uint32_t key = act_key(widx * 32 + lane);
                            sel = key <= thr;
                            if (!sel) mnext = min(mnext, key);
                        }
                        const uint32_t mask = (uint32_t)__ballot(sel);
                        if (mask) {
                            // words are owned by one wave; other waves only set bits: clearing is exact
                            if (lane == 0) atomicAnd(&bits[widx], ~mask);
                            if (sel) q[qn + __popc(mask & ((1u << lane) - 1u))] = widx * 32 + lane;
                            qn += __popc(mask);
                        }
                    }
                }
                if (qn >= kQCap || (!more && qn > 0)) flush();
                if (!more) break;
            }
        }
        if (lane_scan) {
        // Lane per bitmap word: a wave reads 64 words at once, each lane picks its word's selected
        // nodes (bits clear first; other waves only set bits in a word this lane owns, so the
        // atomicAnd is exact), then the selected nodes enter the queue one per lane per step.  A
        // sweep's frontier is sparse (C4: about one active node per word), so this reads the
        // bitmap 64x faster than a word per wave step with half the lanes idle (C4 DELTA, 4096
        // rows: 50.8 -> 38.7 ms).  Words are dealt round-robin (word k*NW + wave to lane k).
        for (uint32_t k0 = 0;; k0 += 64) {
            const bool more = k0 * NW + wave < W;   // wave-uniform: the wave has words in this batch
            const uint32_t widx = (k0 + lane) * NW + wave;
            uint32_t rem = 0;           // this lane's selected nodes not yet queued
            // Per-word minimum (wmin, global labels): a word whose active nodes all lie above
            // the threshold is skipped on one LDS read instead of one bucket-byte read per active
            // node -- most active nodes of a sparse graph wait many sweeps for their bucket.
            // The scanning lane owns the word: it resets wmin, then reads the bits and puts the
            // keys of those it leaves back; a relaxation sets the bit first and lowers wmin
            // after, so every set bit is either seen by that read or lowers wmin afterwards.
            bool scan_word = more && widx < W;
            if (scan_word && wmin) {
                const uint32_t m = __hip_atomic_load(&wmin[widx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (m > thr) {
                    mnext = min(mnext, m);
                    scan_word = false;
                } else {   // an acquire: the bits below are read after the reset, never before
                    (void)__hip_atomic_exchange(&wmin[widx], kLat32Inf, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            if (scan_word) {
                const uint32_t word = __hip_atomic_load(&bits[widx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (word) {
                    uint32_t selm = word;
                    if (use_delta) {
                        selm = 0;
                        uint32_t rest = kLat32Inf;
                        for (uint32_t mm = word; mm; mm &= mm - 1) {
                            const uint32_t b = __builtin_ctz(mm);
                            const uint32_t key = act_key(widx * 32 + b);
                            if (key <= thr) selm |= 1u << b;
                            else rest = min(rest, key);
                        }
                        mnext = min(mnext, rest);
                        if (wmin && rest != kLat32Inf) atomicMin(&wmin[widx], rest);
                    }
                    if (selm) atomicAnd(&bits[widx], ~selm);
                    rem = selm;
                }
            }
            for (;;) {
                const uint64_t bal = __ballot(rem != 0);
                if (more && bal == 0) break;   // this batch of words is queued
                if (rem) {
                    q[qn + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = widx * 32 + __builtin_ctz(rem);
                    rem &= rem - 1;
                }
                qn += (uint32_t)__popcll(bal);
                if (qn < kQCap && (more || qn == 0)) {
                    if (more) continue;
                    break;
                }
                flush();
                if (!more && bal == 0) break;
            }
            if (!more) break;
        }
        }
        ++sweeps;
        SS_MARK(1);
        if (fused) {
            for (int o = 32; o > 0; o >>= 1) mnext = min(mnext, (uint32_t)__shfl_xor((int)mnext, o));
            if (lane == 0 && mnext != kLat32Inf) atomicMin(&ctl[1 + slot], mnext);
            __syncthreads();
            SS_MARK(3);
            slot = slot == 2 ? 0 : slot + 1;
        } else if (!use_delta) {
            if (dirty) ctl[0] = 1;
            __syncthreads();
            const bool again = ctl[0] != 0;
            __syncthreads();
            if (!again) break;
        } else {
            __syncthreads();
        }
    }
    if (ovf) atomicOr(&flags[0], 1u);
    if (stats && lane == 0) {
        atomicAdd(&stats[0], (unsigned long long)expanded);
        if (wave == 0) atomicAdd(&stats[1], (unsigned long long)sweeps);
    }
    if (nh_out) {
        // Next hops (north star; the reference keeps none).  pred(v) = the lowest node
        // index u with an arc u -> v that is tight for the final labels (key(u) (+) arc == key(v),
        // bit for bit); every label is reached through such an arc (the fold is monotone), and
        // latency strictly grows along it, so the pred chain of any reached node ends at the
        // source.  next hop(src, d) = the node after src on d's pred chain.  pred lives where
        // the arc-range cache was (LDS kernel) or in a global scratch row (global labels).
        __syncthreads();
        for (uint32_t v = tid; v < V; v += BLOCK) pred[v] = 0xFFFFFFFFu;
        if (GLAB) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (uint32_t u = tid; u < V; u += BLOCK) {
            const uint64_t ku = ld_lab<GLAB>(&lab[u]);
            if (ku == kKeyInf) continue;
            const uint32_t lu = key_lat(ku);
            const float qu = one_minus(key_loss(ku));
            const uint32_t e = aend[u];
            for (uint32_t k = abeg[u]; k < e; ++k) {
                const uint4 a = arcs[k];
                const uint32_t cl = lu + a.y;
                if (a.x == u || a.y == kLat32Inf || cl < lu || cl == kLat32Inf) continue;
                if (pack_key(cl, fold_q(qu, __uint_as_float(a.z))) == ld_lab<GLAB>(&lab[a.x]))
                    atomicMin(&pred[a.x], u);
            }
        }
        if (GLAB) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (uint32_t j = tid; j < n_used; j += BLOCK) {
            const uint32_t v = GLAB || used ? used[j] : j;
            uint32_t nh = 0xFFFFFFFFu;
            if (v == src) {
                nh = src;
            } else {
                uint32_t w = v, pw = GLAB ? __hip_atomic_load(&pred[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : pred[w];
                for (uint32_t hop = 0; hop < V && pw != src && pw != 0xFFFFFFFFu; ++hop) {
                    w = pw;
                    pw = GLAB ? __hip_atomic_load(&pred[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : pred[w];
                }
                if (pw == src) nh = w;
            }
            __builtin_nontemporal_store(nh, &nh_out[orow + j]);
        }
    }
#ifndef SHD_OUT_SINGLE   // (tuning A/B: one column per iteration)
    constexpr uint32_t kOut = 4;   // columns per thread per iteration: their loads in flight together
#else
    constexpr uint32_t kOut = 1;
#endif
    for (uint32_t j0 = tid; j0 < n_used; j0 += kOut * BLOCK) {
        uint32_t uj[kOut];
        uint64_t k[kOut];
#pragma unroll
        for (uint32_t i = 0; i < kOut; ++i) {
            const uint32_t j = j0 + i * BLOCK;
            uj[i] = j < n_used ? (GLAB || used ? used[j] : j) : 0u;
        }
#pragma unroll
        for (uint32_t i = 0; i < kOut; ++i) {
            const uint32_t j = j0 + i * BLOCK;
            k[i] = j < n_used && j != row ? (uj[i] < kl ? llab[uj[i]] : ld_lab<GLAB>(&lab[uj[i]])) : 0ull;
        }
#pragma unroll
        for (uint32_t i = 0; i < kOut; ++i) {
            const uint32_t j = j0 + i * BLOCK;
            if (j >= n_used) break;
            uint64_t l;
            float p;
            if (j == row) {
                l = diag_lat[j];
                p = diag_loss[j];
            } else if (k[i] == kKeyInf) {
                atomicMin(unreach, (unsigned long long)((uint64_t)row * n_used + j));
                l = ~0ull;
                p = 0.0f;
            } else {
                l = key_lat(k[i]);
                p = key_loss(k[i]);
            }
            // the table is written once and never read here: non-temporal stores keep it from
            // evicting the label rows (C4: 600 KB of table per source row) from L2 / Infinity Cache
            __builtin_nontemporal_store(l, &out_lat[orow + j]);
            __builtin_nontemporal_store(p, &out_loss[orow + j]);
        }
    }
#ifdef SHD_SSSP_PROF
    SS_MARK(4);
    if (lane == 0) {
        for (int k = 0; k < 5; ++k) atomicAdd(&g_sssp_prof[k], (unsigned long long)ss_acc[k]);
        atomicAdd(&g_sssp_prof[5], (unsigned long long)sweeps);
        atomicAdd(&g_sssp_prof[6], (unsigned long long)expanded);
        atomicAdd(&g_sssp_prof[7], 1ull);
    }
#endif
}

// Kernel 1: one workgroup per source row, labels (8 B/node) and the arc ranges in LDS.
// PADR = 8: padded arc lists (prune_rows), relax_node_pad with 8 arcs per lane per step.
template <int BLOCK, int G, int R, bool CACHE, int PADR, bool FLATL = false>
__global__ __launch_bounds__(BLOCK) void sssp_lds_group(
    const uint32_t* __restrict__ abeg, const uint32_t* __restrict__ aend,
    const uint4* __restrict__ arcs, uint32_t V, const uint32_t* __restrict__ used,
    uint32_t n_used, uint32_t row_begin, const uint64_t* __restrict__ diag_lat,
    const float* __restrict__ diag_loss, uint64_t* __restrict__ out_lat,
    float* __restrict__ out_loss, uint32_t* __restrict__ flags,
    unsigned long long* __restrict__ unreach, uint32_t delta,
    unsigned long long* __restrict__ stats, const uint32_t* __restrict__ seed_lat,
    uint32_t seed_stride, uint32_t* __restrict__ nh_out, uint32_t lat_guard, uint32_t use_offl,
    uint32_t flat_off, uint32_t hub_deg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr uint32_t NW = BLOCK / 64;
    uint32_t* flat = FLATL ? reinterpret_cast<uint32_t*>(smem + flat_off) : nullptr;   // expand_flat scratch
    uint64_t* lab = reinterpret_cast<uint64_t*>(smem);   // V labels + 64 per-lane scratch labels
    const uint32_t W = (V + 31) >> 5;
    uint32_t* bits = reinterpret_cast<uint32_t*>(lab + V + 64);
    uint32_t* ctl = bits + W;            // [0] dirty  [1..3] min active latency
    uint32_t* wq = ctl + 4;              // per-wave queue (kQStride node ids)
    // [V] arc range {beg, end}, 8-byte aligned after the queues
    const uint32_t rng_off =
        (((uint32_t)((wq + NW * kQStride) - reinterpret_cast<uint32_t*>(smem)) * 4u) + 7u) & ~7u;
    uint2* rng = reinterpret_cast<uint2*>(smem + rng_off);
    // !CACHE on a plain CSR (aend == abeg + 1): the offsets alone, 4 B/node, in LDS (use_offl);
    // next hops' pred[V] then follows them
    uint32_t* offl = !CACHE && use_offl ? reinterpret_cast<uint32_t*>(smem + rng_off) : nullptr;
    uint32_t* pred = offl ? offl + V + 1 : reinterpret_cast<uint32_t*>(smem + rng_off);
    sssp_row<BLOCK, G, R, CACHE, false, PADR, false, FLATL>(lab, bits, ctl, wq, rng, abeg, aend, arcs, V, used, n_used,
                                              row_begin + blockIdx.x, (size_t)blockIdx.x * n_used,
                                              diag_lat, diag_loss, out_lat, out_loss, flags, unreach,
                                              delta, stats, seed_lat, seed_stride, nullptr, flat, nh_out,
                                              pred, lat_guard, nullptr, nullptr, offl, nullptr, 0u, nullptr,
                                              hub_deg);
}

// Kernel 1b: labels in global memory, for graphs whose labels do not fit the LDS (C4: 50k
// nodes = 400 KB per source).  A persistent grid of slots: slot b owns the label array
// glab[b*V, (b+1)*V) and walks rows row_begin + b, + gridDim.x, ...; the bitmap and the queues
// stay in LDS (V/8 bytes).
// (Two slots per CU need <= 128 VGPRs at BLOCK = 512; the kernel sits at exactly 128, so any
// added live value halves its residency -- check .vgpr_count after changes to sssp_row.  A
// waves-per-EU launch bound keeps the count but schedules worse: C4 rows 0-4095 17.4 -> 18.5 ms.)
template <int BLOCK, int G, int R, bool FASTG>
__global__ __launch_bounds__(BLOCK) void sssp_global_group(
    const uint32_t* __restrict__ abeg, const uint32_t* __restrict__ aend,
    const uint4* __restrict__ arcs, uint32_t V, const uint32_t* __restrict__ used,
    uint32_t n_used, uint32_t row_begin, uint32_t row_end, const uint64_t* __restrict__ diag_lat,
    const float* __restrict__ diag_loss, uint64_t* __restrict__ out_lat,
    float* __restrict__ out_loss, uint32_t* __restrict__ flags,
    unsigned long long* __restrict__ unreach, uint32_t delta,
    unsigned long long* __restrict__ stats, uint64_t* __restrict__ glab, uint32_t use_bkt, uint32_t use_flat,
    uint32_t* __restrict__ nh_out, uint32_t* __restrict__ gpred, const uint2* __restrict__ arcs8,
    const float* __restrict__ aq, uint32_t kl, uint32_t* __restrict__ row_ctr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint32_t s_next;
    const uint32_t W = (V + 31) >> 5;
    uint32_t* bits = reinterpret_cast<uint32_t*>(smem);
    uint32_t* ctl = bits + W;
    uint32_t* wq = ctl + 4;
    uint32_t* flat = use_flat ? wq + (BLOCK / 64) * kQStride : nullptr;
    uint8_t* bkt = use_bkt ? reinterpret_cast<uint8_t*>(wq + (BLOCK / 64) * (kQStride + (use_flat ? kFlatWords : 0)))
                           : nullptr;
    uint64_t* lab = glab + (size_t)blockIdx.x * V;
    // FASTG with use_flat bit 1: the per-word minimum keys (W words) after the bucket bytes
    uint32_t* wmin = FASTG && use_bkt && (use_flat & 2u) ? reinterpret_cast<uint32_t*>(bkt + ((V + 3) / 4) * 4) : nullptr;
    // kl > 0 (FASTG, no next hops): the labels of nodes [0, kl) in LDS after the bucket bytes (and wmin)
    uint64_t* llab = nullptr;
    if (FASTG && kl) {
        const unsigned char* end = wmin ? reinterpret_cast<unsigned char*>(wmin + W) : bkt + ((V + 3) / 4) * 4;
        const size_t at = ((size_t)(end - smem) + 7) & ~(size_t)7;
        llab = reinterpret_cast<uint64_t*>(smem + at);
    }
    // row_ctr (zeroed before the launch): after its first row a slot takes the next unclaimed row,
    // so the grid drains together instead of waiting for the slot whose fixed rows ran longest
    uint32_t row = row_begin + blockIdx.x;
    while (row < row_end) {
        sssp_row<BLOCK, G, R, false, true, 0, FASTG>(lab, bits, ctl, wq, nullptr, abeg, aend, arcs, V, used,
                                           n_used, row, (size_t)(row - row_begin) * n_used,
                                           diag_lat, diag_loss, out_lat, out_loss, flags, unreach,
                                           delta, stats, nullptr, 0, bkt, flat, nh_out,
                                           gpred ? gpred + (size_t)blockIdx.x * V : nullptr, 0u, arcs8, aq, nullptr,
                                           llab, FASTG ? kl : 0u, wmin);
        __syncthreads();   // the next row re-initialises labels and bitmap
        if (row_ctr) {
            if (threadIdx.x == 0) s_next = row_begin + gridDim.x + atomicAdd(row_ctr, 1u);
            __syncthreads();
            row = s_next;
        } else {
            row += gridDim.x;
        }
    }
}

__global__ __launch_bounds__(256) void arcs_pack(const uint32_t* __restrict__ dst,
                                                 const uint32_t* __restrict__ lat,
                                                 const float* __restrict__ loss,
                                                 uint4* __restrict__ out, uint2* __restrict__ out8,
                                                 float* __restrict__ outq, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float q = one_minus(loss[i]);
    out[i] = make_uint4(dst[i], lat[i], __float_as_uint(q), 0u);
    out8[i] = make_uint2(dst[i], lat[i]);   // compact arcs of the global-label kernel
    outq[i] = q;
}

// compact arcs only (the locality-ordered copy of the global-label kernel)
__global__ __launch_bounds__(256) void arcs_pack8(const uint32_t* __restrict__ dst, const uint32_t* __restrict__ lat,
                                                  const float* __restrict__ loss, uint2* __restrict__ out8,
                                                  float* __restrict__ outq, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    out8[i] = make_uint2(dst[i], lat[i]);
    outq[i] = one_minus(loss[i]);
}

// ------------------------------------------------------------------------------------------
// Dense-graph arc pruning (SHD_ALGO_PRUNED).  An arc (u,v) lies on no shortest-latency path if
// some 2-hop detour u->x->v is STRICTLY shorter; such arcs cannot change any lexicographic
// label (the latency part is decided first and every tight path avoids them), so the SSSP
// below runs on the surviving arcs only and still reproduces the reference's bits.  x ranges
// over the K lowest-latency neighbours of u (any subset is sound; the nearest catch almost
// all: C2 keeps ~49 of 999 arcs per node with K = 32).  Ties (detour == arc) are kept.
// ------------------------------------------------------------------------------------------
// per-build flags (one launch instead of three memsets): [0,16) overflow / misc = 0,
// [16,24) first unreachable pair = ~0, [24,64) = 0 (stats counters at 32)
__global__ __launch_bounds__(64) void flags_init(uint32_t* __restrict__ f) {
    const uint32_t t = threadIdx.x;
    if (t < 16) f[t] = (t == 4 || t == 5) ? 0xFFFFFFFFu : 0u;
}

// One workgroup per row u: the row's arc keys (parallel arcs folded by a lexicographic LDS
// atomicMin) built in LDS and written once as the latency row Wl and the loss row Wp -- one
// pass instead of init + global-atomic scatter + a latency-extract pass (C2: 16 -> 7 us); the
// prune reads its own row's latencies from Wl and the loss only of the arcs it keeps, so the
// 8-byte key row is not written (round 3).
// (A u16 latency row rounded up -- sound for the prune, half the gathered bytes -- measured
// slower: prune_rows 32 -> 57 us, the decode outweighing the bytes.)
__global__ __launch_bounds__(256) void dense_build(const uint32_t* __restrict__ off,
                                                   const uint32_t* __restrict__ adst,
                                                   const uint32_t* __restrict__ alat,
                                                   const float* __restrict__ aloss, uint32_t V,
                                                   float* __restrict__ Wp, uint32_t* __restrict__ Wl,
                                                   uint32_t* __restrict__ cursor, uint32_t* __restrict__ flags) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t* rowk = reinterpret_cast<uint64_t*>(smem);
    const uint32_t u = blockIdx.x, tid = threadIdx.x;
    for (uint32_t v = tid; v < V; v += 256) rowk[v] = kKeyInf;
    if (u == 0 && tid == 0) *cursor = 0;   // prune_rows' output cursor
    if (u == 0 && tid < 16) flags[tid] = (tid == 4 || tid == 5) ? 0xFFFFFFFFu : 0u;   // as flags_init
    __syncthreads();
    for (uint32_t k = off[u] + tid; k < off[u + 1]; k += 256)
        atomicMin(reinterpret_cast<unsigned long long*>(&rowk[adst[k]]), (unsigned long long)pack_key(alat[k], aloss[k]));
    __syncthreads();
    const size_t base = (size_t)u * V;
    for (uint32_t v = tid; v < V; v += 256) {
        const uint64_t k = rowk[v];
        Wp[base + v] = key_loss(k);
        Wl[base + v] = key_lat(k);
    }
}

// DCSR (complete graphs without parallel arcs, PreparedGraph::dense_rows): the arc CSR is the
// dense matrix itself -- node x's arcs are every other node in index order, so the latency of
// (x, v) is Wl[x (V - 1) + v - (v > x)] and (x, x) has none -- and the prune reads it directly:
// no dense_build pass, no V x V matrices (the CSR's latency and loss arrays are Wl and Wp).
// Block 0 then also resets the build flags (dense_build's job otherwise).
template <bool DCSR>
__device__ __forceinline__ uint32_t dense_lat(const uint32_t* __restrict__ Wl, uint32_t V, uint32_t x, uint32_t v) {
    if constexpr (DCSR) return v == x ? kLat32Inf : Wl[(size_t)x * (V - 1) + v - (v > x ? 1u : 0u)];
    else return Wl[(size_t)x * V + v];
}

template <int BLOCK, int K, bool DCSR = false, int VB = 4, int KB = 8, bool CMP = false, int PB = 8>
__global__ __launch_bounds__(BLOCK) void prune_rows(
    const uint32_t* __restrict__ Wl, const float* __restrict__ Wp, uint32_t V,
    uint32_t* __restrict__ pbeg, uint32_t* __restrict__ pend, uint4* __restrict__ parcs,
    uint32_t* __restrict__ cursor, uint32_t* __restrict__ flags, uint32_t shg = 0xFFFFFFFFu) {
    // Detour nodes x: ~K of u's lowest-latency neighbours, chosen by a 256-bin latency histogram
    // (every node in the bins below the K-th smallest latency's bin, then nodes of that bin in
    // index order up to K).  Any set of detour nodes is sound -- it only decides how many arcs
    // are dropped -- so this replaces a full bitonic sort of the row (55 barrier stages) by
    // three passes over it.
    // CMP (round 5, the K = 32 default; C2 prune 24.4 -> 15.6 us): the detours are the K
    // smallest (latency, index) pairs in ascending order, ranked in LDS by all waves; the first
    // batch tests every arc against the KB nearest, skipping detours no shorter than the arc; its
    // survivors (~11 % of a C2 row) are packed and tested one lane each against the rest, PB at a
    // time, stopping at the first detour no shorter than the arc -- instead of every wave
    // carrying a few live lanes through every batch.  The row's losses come in with its
    // latencies, so the kept arcs read them from LDS.
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint4* kept = reinterpret_cast<uint4*>(smem);      // V staged arcs
    uint32_t* cnt = reinterpret_cast<uint32_t*>(kept + V);   // [0] kept [1] base [2] max [3] below-bin
    uint32_t* hist = cnt + 8;                          // 256 bins
    uint32_t* selx = hist + 256;                       // K detour nodes
    uint32_t* sela = selx + K;                         // their latencies
    uint32_t* row = sela + K;                          // u's exact arc latencies
    uint16_t* binv = reinterpret_cast<uint16_t*>(row + V);   // bin per node (0xFFFF: no arc)
    uint2* live2 = reinterpret_cast<uint2*>((reinterpret_cast<uintptr_t>(binv + V) + 7) & ~(uintptr_t)7);   // CMP: first-batch survivors
    uint64_t* cand = reinterpret_cast<uint64_t*>(live2 + V);   // CMP: <= 64 detour candidates
    uint32_t* rk = reinterpret_cast<uint32_t*>(cand + 64);        // and their ranks
    float* prow = reinterpret_cast<float*>(rk + 64);              // CMP: u's arc losses
    const uint32_t u = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
#ifdef SHD_SSSP_PROF
    uint64_t pr_acc[6] = {0, 0, 0, 0, 0, 0}, pr_t = __builtin_amdgcn_s_memtime();
    const uint64_t pr_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    if (DCSR && u == 0 && tid < 16) flags[tid] = (tid == 4 || tid == 5) ? 0xFFFFFFFFu : 0u;   // as flags_init
    uint32_t mx = 0;
    for (uint32_t v = tid; v < V; v += BLOCK) {
        const uint32_t w = dense_lat<DCSR>(Wl, V, u, v);
        row[v] = w;
        if (w != kLat32Inf) mx = max(mx, w);
        if constexpr (CMP) {   // the row's losses ride the same memory trip (kept arcs read them)
            if (w != kLat32Inf) prow[v] = Wp[DCSR ? (size_t)u * (V - 1) + v - (v > u ? 1u : 0u) : (size_t)u * V + v];
        }
    }
    for (uint32_t i = tid; i < 256; i += BLOCK) hist[i] = 0;
    if (tid < 8) cnt[tid] = 0;
    if (CMP && tid < 64) rk[tid] = 0;
    uint32_t sh;
    if (CMP && shg != 0xFFFFFFFFu) {   // bins from the graph's largest arc latency (host): one barrier
        __syncthreads();
        sh = shg;
    } else {
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        __syncthreads();
        if (lane == 0) atomicMax(&cnt[2], mx);
        __syncthreads();
        const uint32_t bits = 32u - (uint32_t)__clz((int)max(cnt[2], 1u));
        sh = bits > 8 ? bits - 8 : 0;
    }
    PR_MARK(0);
    for (uint32_t v = tid; v < V; v += BLOCK) {
        const uint32_t w = row[v];
        binv[v] = w != kLat32Inf ? (uint16_t)(w >> sh) : (uint16_t)0xFFFF;
        if (w != kLat32Inf) atomicAdd(&hist[w >> sh], 1u);
    }
    __syncthreads();
    PR_MARK(1);
    if (tid < 64) {   // wave 0: the bin holding the K-th smallest latency
        uint32_t c[4], sum = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            c[i] = hist[tid * 4 + i];
            sum += c[i];
        }
        uint32_t incl = sum;
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        uint32_t run = incl - sum, bsel = 256, below = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (bsel == 256 && run + c[i] >= (uint32_t)K) {
                bsel = tid * 4 + i;
                below = run;
            }
            run += c[i];
        }
        const uint64_t m = __ballot(bsel != 256);
        if (m) {
            const uint32_t first = (uint32_t)__ffsll((unsigned long long)m) - 1u;
            const uint32_t b = __shfl((int)bsel, first), bl = __shfl((int)below, first);
            if (tid == 0) {
                cnt[4] = b;
                cnt[3] = bl;
            }
        } else if (tid == 0) {
            cnt[4] = 256;      // fewer than K finite entries: take them all
            cnt[3] = 0;
        }
        if (tid == 0) {
            cnt[5] = 0;        // slots below the bin
            cnt[6] = 0;        // slots in the bin
        }
    }
    __syncthreads();
    PR_MARK(2);
    // CMP: the detours are the K smallest (latency, index) pairs in ascending order.  Fast path:
    // the bins below and the boundary bin hold at most 64 candidates -- collect them, and wave 0
    // sorts them in registers; otherwise the index-order boundary scan below, then a rank sort.
    bool sel_done = false;
    if constexpr (CMP && K <= 64) {
        const uint32_t bsel = cnt[4];
        const uint32_t ncand = bsel < 256 ? cnt[3] + hist[bsel] : (uint32_t)K;
        if (ncand <= 64) {
            // rank sort: wave p compares every candidate with its share of the others
            for (uint32_t v = tid; v < V; v += BLOCK) {
                if (binv[v] <= bsel) {   // (no arc: 0xFFFF, above every bin)
                    const uint32_t sl = atomicAdd(&cnt[5], 1u);
                    cand[sl] = (uint64_t)row[v] << 32 | v;
                }
            }
            __syncthreads();
            const uint32_t n = cnt[5];
            constexpr uint32_t per = 64 / (BLOCK / 64);
            if (lane < n) {
                const uint64_t ki = cand[lane];
                const uint32_t j0 = (tid >> 6) * per;
                uint32_t r = 0;
#pragma unroll
                for (uint32_t jj = 0; jj < per; ++jj)
                    r += j0 + jj < n && cand[j0 + jj] < ki ? 1u : 0u;
                if (r) atomicAdd(&rk[lane], r);
            }
            __syncthreads();
            if (tid < 64) {
                if (lane < n) {
                    const uint32_t r = rk[lane];
                    if (r < (uint32_t)K) {
                        const uint64_t k = cand[lane];
                        selx[r] = (uint32_t)k;
                        sela[r] = (uint32_t)(k >> 32);
                    }
                } else if (lane < (uint32_t)K) {   // unused slots: no detour
                    selx[lane] = 0u;
                    sela[lane] = kLat32Inf;
                }
                if (tid == 0) {
                    cnt[0] = 0;
                    cnt[7] = 0;
                }
            }
            sel_done = true;
        }
    }
    if (!sel_done) {   // every node of the bins below; then wave 0 takes the boundary bin in index order, so
        // the detour set (and with it the kept-arc count) is the same on every run
        const uint32_t bsel = cnt[4], below = cnt[3];
        for (uint32_t v = tid; v < V; v += BLOCK) {
            if (binv[v] < bsel) {
                const uint32_t sl = atomicAdd(&cnt[5], 1u);
                selx[sl] = v;
                sela[sl] = row[v];
            }
        }
        if (tid < 64 && bsel < 256) {
            uint32_t taken = 0;
            for (uint32_t v0 = 0; v0 < V && below + taken < (uint32_t)K; v0 += 64) {
                const uint32_t v = v0 + lane;
                const bool hit = v < V && binv[v] == bsel;
                const uint64_t m = __ballot(hit);
                const uint32_t sl = below + taken + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (hit && sl < (uint32_t)K) {
                    selx[sl] = v;
                    sela[sl] = row[v];
                }
                taken += (uint32_t)__popcll(m);
            }
            if (tid == 0) cnt[6] = taken;
        }
        __syncthreads();
        const uint32_t nsel = min((uint32_t)K, cnt[5] + cnt[6]);
        for (uint32_t j = nsel + tid; j < (uint32_t)K; j += BLOCK) {   // unused slots: no detour
            selx[j] = 0u;
            sela[j] = kLat32Inf;
        }
        if (tid == 0) cnt[0] = 0;
        if constexpr (CMP) {   // detours in ascending latency (ties by index): wave 0 ranks them
            __syncthreads();
            uint32_t* tx = hist;   // the histogram is spent; K <= 128 pairs fit its 256 words
            uint32_t* ta = hist + K;
            if (tid < 64) {
                for (uint32_t i = lane; i < (uint32_t)K; i += 64) {
                    const uint32_t ai = sela[i], xi = selx[i];
                    uint32_t r = 0;
                    for (uint32_t j = 0; j < (uint32_t)K; ++j) {
                        const uint32_t aj = sela[j], xj = selx[j];
                        r += aj < ai || (aj == ai && (xj < xi || (xj == xi && j < i))) ? 1u : 0u;
                    }
                    tx[r] = xi;
                    ta[r] = ai;
                }
            }
            __syncthreads();
            for (uint32_t j = tid; j < (uint32_t)K; j += BLOCK) {
                selx[j] = tx[j];
                sela[j] = ta[j];
            }
            if (tid == 0) cnt[7] = 0;   // survivors of the first batch
        }
    }
    __syncthreads();
    PR_MARK(3);
    // 2-hop test of every arc of u: each thread tests VB arcs at once against batches of KB
    // detours (VB x KB loads in flight), and a lane stops loading for an arc as soon as a
    // strictly shorter detour is found -- most arcs of a dense row fall to the first batch
    for (uint32_t v0 = tid; v0 < V; v0 += BLOCK * VB) {
        uint32_t w[VB], z[VB];
#pragma unroll
        for (int i = 0; i < VB; ++i) {
            const uint32_t v = v0 + i * BLOCK;
            w[i] = v < V ? row[v] : kLat32Inf;
            z[i] = kLat32Inf;
        }
        for (int j0 = 0; j0 < (CMP ? KB : K); j0 += KB) {
            bool any = false;
#pragma unroll
            for (int i = 0; i < VB; ++i) any |= w[i] != kLat32Inf && w[i] <= z[i];
            if (!any) break;
            uint32_t as[KB], bv[VB][KB], xs[KB];
            size_t xb[KB];
#pragma unroll
            for (int j = 0; j < KB; ++j) {
                as[j] = sela[j0 + j];
                xs[j] = selx[j0 + j];
                xb[j] = (size_t)xs[j] * (DCSR ? V - 1 : V);
            }
#pragma unroll
            for (int i = 0; i < VB; ++i) {
                const uint32_t v = v0 + i * BLOCK;
                const bool live = w[i] != kLat32Inf && w[i] <= z[i];
#pragma unroll
                for (int j = 0; j < KB; ++j) {
                    if constexpr (CMP)   // sorted detours: one no shorter than the arc cannot beat it
                        bv[i][j] = live && as[j] < w[i] && v != xs[j]
                                       ? Wl[xb[j] + v - (DCSR && v > xs[j] ? 1u : 0u)]
                                       : kLat32Inf;
                    else if constexpr (DCSR)   // (x, x) has no arc; past the diagonal the row is shifted by one
                        bv[i][j] = live && as[j] != kLat32Inf && v != xs[j] ? Wl[xb[j] + v - (v > xs[j] ? 1u : 0u)]
                                                                            : kLat32Inf;
                    else
                        bv[i][j] = live && as[j] != kLat32Inf ? Wl[xb[j] + v] : kLat32Inf;
                }
            }
#pragma unroll
            for (int i = 0; i < VB; ++i)
#pragma unroll
                for (int j = 0; j < KB; ++j) {
                    const uint32_t t = as[j] + bv[i][j];
                    if (as[j] != kLat32Inf && bv[i][j] != kLat32Inf && t >= as[j]) z[i] = min(z[i], t);
                }
        }
#pragma unroll
        for (int i = 0; i < VB; ++i) {
            if (w[i] == kLat32Inf || w[i] > z[i]) continue;
            const uint32_t v = v0 + i * BLOCK;
            if constexpr (CMP) {   // survivors of the first batch: the rest of the detours below
                if (K > KB && w[i] > sela[KB]) {
                    const uint32_t li = atomicAdd(&cnt[7], 1u);
                    live2[li] = make_uint2(v, w[i]);
                    continue;
                }
            }
            const uint32_t slot = atomicAdd(&cnt[0], 1u);
            const size_t at = DCSR ? (size_t)u * (V - 1) + v - (v > u ? 1u : 0u) : (size_t)u * V + v;
            kept[slot] = make_uint4(v, w[i], __float_as_uint(one_minus(CMP ? prow[v] : Wp[at])), 0u);
        }
    }
    if constexpr (CMP && K > KB) {
        // the first batch's survivors, packed: one lane per arc over the remaining detours in
        // batches of 8 (a wave's loads are all live instead of a few lanes of every wave)
        __syncthreads();
        const uint32_t nl = cnt[7];
        for (uint32_t i = tid; i < nl; i += BLOCK) {
            const uint2 e = live2[i];
            const uint32_t v = e.x, wv = e.y;
            uint32_t z = kLat32Inf;
            for (int j0 = KB; j0 < K && wv <= z && sela[j0] < wv; j0 += PB) {
                uint32_t as[PB], bq[PB];
#pragma unroll
                for (int j = 0; j < PB; ++j) {
                    as[j] = j0 + j < K ? sela[j0 + j] : kLat32Inf;
                    const uint32_t x = j0 + j < K ? selx[j0 + j] : 0u;
                    bq[j] = as[j] < wv && v != x
                                ? Wl[(size_t)x * (DCSR ? V - 1 : V) + v - (DCSR && v > x ? 1u : 0u)]
                                : kLat32Inf;
                }
#pragma unroll
                for (int j = 0; j < PB; ++j) {
                    const uint32_t t = as[j] + bq[j];
                    if (as[j] != kLat32Inf && bq[j] != kLat32Inf && t >= as[j]) z = min(z, t);
                }
            }
            if (wv > z) continue;
            const uint32_t slot = atomicAdd(&cnt[0], 1u);
            kept[slot] = make_uint4(v, wv, __float_as_uint(one_minus(prow[v])), 0u);
        }
    }
    __syncthreads();
    PR_MARK(4);
    // each list is padded to kArcPad slots with no-op arcs for relax_node_pad (scratch label
    // V + i, lat 0, q 0: candidate (lu, 1.0f) against a scratch label holding 0).  Row u's list
    // starts at u * roundup(V, kArcPad): the 1000 workgroups of C2 finish together, and one
    // shared cursor (rows packed in arrival order) serialised their atomics at the end of the
    // kernel; the slots a sweep touches are the same lines either way.
    const uint32_t n = cnt[0], np = (n + kArcPad - 1) / kArcPad * kArcPad;
#ifdef SHD_PRUNE_CURSOR   // (tuning A/B: rows packed by one atomic cursor)
    if (tid == 0) cnt[1] = atomicAdd(cursor, np);
    __syncthreads();
    const uint32_t at = cnt[1];
#else
    const uint32_t at = u * ((V + kArcPad - 1) / kArcPad * kArcPad);
#endif
    for (uint32_t i = tid; i < np; i += BLOCK)
        parcs[at + i] = i < n ? kept[i] : make_uint4(V + (i & 63u), 0u, 0u, 0u);
    if (tid == 0) {
        pbeg[u] = at;
        pend[u] = at + n;
    }
#ifdef SHD_SSSP_PROF
    PR_MARK(5);
    if (tid == 0 && u < 4096) {
        for (int k = 0; k < 6; ++k) g_prune_prof[u * 8 + k] = pr_acc[k];
        g_prune_prof[u * 8 + 6] = pr_t0;
        g_prune_prof[u * 8 + 7] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// ------------------------------------------------------------------------------------------
// Kernel 2 (wide fallback): u64 latencies, labels in global memory, pull-form Jacobi rounds
// over in-arcs.  Used only when some path latency reaches 2^32-1 ns (or V exceeds the LDS).
// One launch = one round for a batch of sources; grid (ceil(V/256), n_src).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sssp_wide_round(
    const uint32_t* __restrict__ in_off, const uint32_t* __restrict__ in_src,
    const uint64_t* __restrict__ in_lat, const float* __restrict__ in_q, uint32_t V,
    const uint64_t* __restrict__ a_lat, const float* __restrict__ a_loss,
    uint64_t* __restrict__ b_lat, float* __restrict__ b_loss, uint32_t* __restrict__ changed,
    uint32_t* __restrict__ flags) {
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    const size_t s = blockIdx.y;
    if (v >= V) return;
    const uint64_t* al = a_lat + s * V;
    const float* ap = a_loss + s * V;
    uint64_t bl = al[v];
    float bp = ap[v];
    bool ch = false;
    for (uint32_t k = in_off[v]; k < in_off[v + 1]; ++k) {
        const uint32_t u = in_src[k];
        const uint64_t lu = al[u];
        if (lu == ~0ull) continue;
        const uint64_t cl = lu + in_lat[k];
        if (cl < lu || cl == ~0ull) {
            atomicOr(&flags[1], 1u);  // exceeds u64: LATENCY_OVERFLOW
            continue;
        }
        const float cp = fold_q(one_minus(ap[u]), in_q[k]);
        if (cl < bl || (cl == bl && cp < bp)) {
            bl = cl;
            bp = cp;
            ch = true;
        }
    }
    b_lat[s * V + v] = bl;
    b_loss[s * V + v] = bp;
    if (ch) changed[0] = 1;
}

__global__ void wide_init(uint64_t* lat, float* loss, uint32_t V, const uint32_t* used,
                          uint32_t row0) {
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    const size_t s = blockIdx.y;
    if (v >= V) return;
    const bool is_src = used[row0 + s] == v;
    lat[s * V + v] = is_src ? 0ull : ~0ull;
    loss[s * V + v] = 0.0f;
}

__global__ void wide_emit(const uint64_t* __restrict__ lat, const float* __restrict__ loss,
                          uint32_t V, const uint32_t* __restrict__ used, uint32_t n_used,
                          uint32_t row0, uint32_t out_row0, const uint64_t* __restrict__ diag_lat,
                          const float* __restrict__ diag_loss, uint64_t* __restrict__ out_lat,
                          float* __restrict__ out_loss, unsigned long long* __restrict__ unreach) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    const size_t s = blockIdx.y;
    if (j >= n_used) return;
    const uint32_t row = row0 + (uint32_t)s;
    uint64_t l;
    float p;
    if (j == row) {
        l = diag_lat[j];
        p = diag_loss[j];
    } else {
        l = lat[s * V + used[j]];
        p = loss[s * V + used[j]];
        if (l == ~0ull) atomicMin(unreach, (unsigned long long)((uint64_t)row * n_used + j));
    }
    const size_t o = (size_t)(out_row0 + s) * n_used + j;
    out_lat[o] = l;
    out_loss[o] = p;
}

// next hops on the wide path: pred(v) = lowest in-neighbour u whose final label extended by
// the arc equals v's label bit for bit (see sssp_row), then the walk back to the source
__global__ void wide_pred(const uint32_t* __restrict__ in_off, const uint32_t* __restrict__ in_src,
                          const uint64_t* __restrict__ in_lat, const float* __restrict__ in_q, uint32_t V,
                          const uint64_t* __restrict__ la, const float* __restrict__ pa,
                          const uint32_t* __restrict__ used, uint32_t row0, uint32_t* __restrict__ pred) {
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    const size_t s = blockIdx.y;
    if (v >= V) return;
    const uint64_t* al = la + s * V;
    const float* ap = pa + s * V;
    uint32_t best = 0xFFFFFFFFu;
    const uint64_t lv = al[v];
    if (v != used[row0 + s] && lv != ~0ull) {
        const uint32_t pv = __float_as_uint(ap[v]);
        for (uint32_t k = in_off[v]; k < in_off[v + 1]; ++k) {
            const uint32_t u = in_src[k];
            const uint64_t lu = al[u];
            if (u == v || u >= best || lu == ~0ull) continue;
            const uint64_t cl = lu + in_lat[k];
            if (cl < lu || cl != lv) continue;
            if (__float_as_uint(fold_q(one_minus(ap[u]), in_q[k])) == pv) best = u;
        }
    }
    pred[s * V + v] = best;
}

__global__ void wide_next_hop(const uint32_t* __restrict__ pred, uint32_t V, const uint32_t* __restrict__ used,
                              uint32_t n_used, uint32_t row0, uint32_t out_row0, uint32_t* __restrict__ out) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    const size_t s = blockIdx.y;
    if (j >= n_used) return;
    const uint32_t src = used[row0 + s], v = used[j];
    const uint32_t* pr = pred + s * V;
    uint32_t nh = 0xFFFFFFFFu;
    if (v == src) {
        nh = src;
    } else {
        uint32_t w = v, pw = pr[w];
        for (uint32_t hop = 0; hop < V && pw != src && pw != 0xFFFFFFFFu; ++hop) {
            w = pw;
            pw = pr[w];
        }
        if (pw == src) nh = w;
    }
    out[(size_t)(out_row0 + s) * n_used + j] = nh;
}

__global__ void direct_next_hop(const uint32_t* __restrict__ used, uint32_t n_used, uint32_t rb, uint32_t rows,
                                uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < (uint64_t)rows * n_used) out[i] = used[i % n_used];   // the one edge's far end (graph/mod.rs:232-254)
    (void)rb;
}

__global__ void arcs_q(const float* __restrict__ loss, float* __restrict__ q, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) q[i] = one_minus(loss[i]);
}

// ------------------------------------------------------------------------------------------
// Direct-path mode: count edges per ordered used pair, keep the edge's raw (lat, loss);
// the first pair (src-major in `used` order) without exactly one edge is the error.
// ------------------------------------------------------------------------------------------
__global__ void direct_scatter(const uint32_t* __restrict__ es, const uint32_t* __restrict__ ed,
                               const uint64_t* __restrict__ el, const float* __restrict__ ep,
                               uint32_t E, int directed, const int32_t* __restrict__ col,
                               uint32_t n_used, uint32_t* __restrict__ cnt,
                               uint64_t* __restrict__ tl, float* __restrict__ tp) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= E) return;
    const int32_t a = col[es[i]], b = col[ed[i]];
    if (a < 0 || b < 0) return;
    size_t c = (size_t)a * n_used + b;
    atomicAdd(&cnt[c], 1u);
    tl[c] = el[i];
    tp[c] = ep[i];
    if (!directed && a != b) {
        c = (size_t)b * n_used + a;
        atomicAdd(&cnt[c], 1u);
        tl[c] = el[i];
        tp[c] = ep[i];
    }
}

__global__ void direct_check(const uint32_t* __restrict__ cnt, uint64_t nn,
                             unsigned long long* __restrict__ first_bad) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < nn && cnt[i] != 1u) atomicMin(first_bad, (unsigned long long)i);
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
struct HostGraph {
    uint32_t V = 0;
    std::vector<uint32_t> off, dst;      // out-CSR without self-loops (petgraph edges(node))
    std::vector<uint64_t> lat;
    std::vector<float> loss;
    std::vector<uint64_t> diag_lat;      // per used index
    std::vector<float> diag_loss;
    uint64_t max_arc_lat = 0, min_arc_lat = 0;
    double sum_arc_lat = 0;
};

// Locality order for the global-label kernel (graphs whose labels leave the LDS, C4): nodes
// renumbered in breadth-first order from the highest-degree nodes, so a node's neighbours get
// nearby numbers -- the label reads and memory-side label atomics of one wave's relaxations then
// share cache lines instead of hitting one line each.  Only that kernel's copies are renumbered
// (offsets, compact arcs, the used list); results are indexed by used position, so the table is
// unchanged.  Next hops (lowest-index tie-break in GML order) run on the original numbering.
static shd_status prepare_reordered(shd_ctx* ctx, const HostGraph& H, const uint32_t* used, uint32_t n_used);
static shd_status prepare_spread(shd_ctx* ctx, const HostGraph& H, const uint32_t* used, uint32_t n_used);

static uint32_t gml_id(const shd_graph* g, uint32_t idx) {
    return g->node_ids ? g->node_ids[idx] : idx;
}

static shd_status set_err(shd_error* err, shd_status st, uint32_t a, uint32_t b) {
    if (err) {
        err->code = st;
        err->node_a = a;
        err->node_b = b;
    }
    return st;
}

static shd_status validate(const shd_graph* g, const uint32_t* used, uint32_t n_used) {
    if (!g || !used || n_used == 0) return SHD_ERR_INVALID;
    if (g->n_edges && (!g->edge_src || !g->edge_dst || !g->edge_latency_ns || !g->edge_packet_loss))
        return SHD_ERR_INVALID;
    for (uint32_t i = 0; i < g->n_edges; i++) {
        if (g->edge_src[i] >= g->n_nodes || g->edge_dst[i] >= g->n_nodes) return SHD_ERR_INVALID;
        // ShadowEdge::try_from rejects latency 0 (graph/mod.rs:107); the kernels rely on every
        // arc strictly increasing latency (unique fixed point = Dijkstra's pop-order result)
        if (g->edge_latency_ns[i] == 0) return SHD_ERR_INVALID;
        const float p = g->edge_packet_loss[i];
        if (!(p >= 0.0f && p <= 1.0f)) return SHD_ERR_INVALID;  // ShadowEdge::try_from range
    }
    std::vector<uint8_t> seen(g->n_nodes, 0);
    for (uint32_t i = 0; i < n_used; i++) {
        if (used[i] >= g->n_nodes || seen[used[i]]) return SHD_ERR_INVALID;
        seen[used[i]] = 1;
    }
    return SHD_OK;
}

// Self-loop rule (graph/mod.rs:212-219 via get_edge_weight): exactly one per used node, first
// offender in `used` order.  Fills the diagonal values.
static shd_status diag_from_self_loops(const shd_graph* g, const uint32_t* used, uint32_t n_used,
                                       HostGraph& H, shd_error* err) {
    std::vector<uint32_t> cnt(g->n_nodes, 0), first(g->n_nodes, 0);
    for (uint32_t i = 0; i < g->n_edges; i++) {
        if (g->edge_src[i] != g->edge_dst[i]) continue;
        const uint32_t v = g->edge_src[i];
        if (cnt[v]++ == 0) first[v] = i;
    }
    H.diag_lat.resize(n_used);
    H.diag_loss.resize(n_used);
    for (uint32_t j = 0; j < n_used; j++) {
        const uint32_t v = used[j];
        if (cnt[v] == 0) return set_err(err, SHD_ERR_NO_EDGE, gml_id(g, v), gml_id(g, v));
        if (cnt[v] > 1) return set_err(err, SHD_ERR_MULTI_EDGE, gml_id(g, v), gml_id(g, v));
        H.diag_lat[j] = g->edge_latency_ns[first[v]];
        H.diag_loss[j] = g->edge_packet_loss[first[v]];
    }
    return SHD_OK;
}

static void build_csr(const shd_graph* g, bool reverse, HostGraph& H) {
    const uint32_t V = g->n_nodes;
    H.V = V;
    H.off.assign(V + 1, 0);
    for (uint32_t i = 0; i < g->n_edges; i++) {
        const uint32_t a = g->edge_src[i], b = g->edge_dst[i];
        if (a == b) continue;  // a self-loop never improves a label (latency > 0)
        H.off[(reverse && g->directed ? b : a) + 1]++;
        if (!g->directed) H.off[b + 1]++;
    }
    for (uint32_t v = 0; v < V; v++) H.off[v + 1] += H.off[v];
    const size_t A = H.off[V];
    H.dst.resize(A);
    H.lat.resize(A);
    H.loss.resize(A);
    std::vector<uint32_t> fill(H.off.begin(), H.off.end() - 1);
    H.max_arc_lat = 0;
    H.min_arc_lat = ~0ull;
    for (uint32_t i = 0; i < g->n_edges; i++) {
        const uint32_t a = g->edge_src[i], b = g->edge_dst[i];
        if (a == b) continue;
        const uint64_t l = g->edge_latency_ns[i];
        const float p = g->edge_packet_loss[i] + 0.0f;  // -0.0 -> +0.0: same fold, ordered bits
        H.max_arc_lat = std::max(H.max_arc_lat, l);
        H.min_arc_lat = std::min(H.min_arc_lat, l);
        H.sum_arc_lat += l;
        auto put = [&](uint32_t from, uint32_t to) {
            const uint32_t k = fill[from]++;
            H.dst[k] = to;
            H.lat[k] = l;
            H.loss[k] = p;
        };
        if (g->directed) {
            if (reverse) put(b, a); else put(a, b);
        } else {
            put(a, b);
            put(b, a);
        }
    }
    // each node's arcs in destination order (stable: parallel arcs keep GML order).  The kernels
    // do not depend on the order; a complete graph's CSR then IS its dense matrix without the
    // diagonal, which the prune reads directly (dense_rows)
    std::vector<uint32_t> idx;
    for (uint32_t u = 0; u < V; ++u) {
        const uint32_t b0 = H.off[u], b1 = H.off[u + 1];
        bool sorted = true;
        for (uint32_t k = b0 + 1; k < b1 && sorted; ++k) sorted = H.dst[k - 1] <= H.dst[k];
        if (sorted) continue;
        idx.resize(b1 - b0);
        for (uint32_t k = 0; k < b1 - b0; ++k) idx[k] = b0 + k;
        std::stable_sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return H.dst[x] < H.dst[y]; });
        std::vector<uint32_t> d2(b1 - b0);
        std::vector<uint64_t> l2(b1 - b0);
        std::vector<float> p2(b1 - b0);
        for (uint32_t k = 0; k < b1 - b0; ++k) {
            d2[k] = H.dst[idx[k]];
            l2[k] = H.lat[idx[k]];
            p2[k] = H.loss[idx[k]];
        }
        std::copy(d2.begin(), d2.end(), H.dst.begin() + b0);
        std::copy(l2.begin(), l2.end(), H.lat.begin() + b0);
        std::copy(p2.begin(), p2.end(), H.loss.begin() + b0);
    }
}

// every node's arc list is exactly the other V - 1 nodes in index order (a complete graph with no
// parallel arcs): the CSR is the dense latency / loss matrix without its diagonal
static bool csr_is_dense(const HostGraph& H) {
    const uint32_t V = H.V;
    if (V < 2 || H.dst.size() != (size_t)V * (V - 1)) return false;
    for (uint32_t u = 0; u < V; ++u) {
        if (H.off[u] != (size_t)u * (V - 1)) return false;
        for (uint32_t k = 0; k + 1 < V; ++k)
            if (H.dst[H.off[u] + k] != k + (k >= u ? 1u : 0u)) return false;
    }
    return true;
}

template <class T>
static shd_status upload(DevBuf& b, const std::vector<T>& v, hipStream_t s) {
    SHD_TRY(b.ensure(std::max<size_t>(v.size(), 1) * sizeof(T)));
    if (!v.empty()) SHD_HIP(hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
    return SHD_OK;
}

// one pinned read-back of the build flags (overflow word, first unreachable pair) and one sync
static shd_status read_flags(shd_ctx* ctx) {
    return readback(ctx, ctx->stream, 0, ctx->g_flags.p, 24);
}
static bool flag_ovf(const shd_ctx* ctx) { return (uint32_t)ctx->h_pin[0] != 0; }

// the first unreachable pair of the last read_flags (the reference panics there, graph/mod.rs:221)
static shd_status check_unreach(shd_ctx* ctx, shd_error* err) {
    PreparedGraph& P = ctx->prep;
    const unsigned long long bad = ctx->h_pin[2];
    if (bad != ~0ull) {
        const uint32_t r = (uint32_t)(bad / P.n_used), c = (uint32_t)(bad % P.n_used);
        return set_err(err, SHD_ERR_UNREACHABLE, P.node_ids[P.used[r]], P.node_ids[P.used[c]]);
    }
    return SHD_OK;
}

static shd_status reset_flags(shd_ctx* ctx) {
    SHD_TRY(ctx->g_flags.ensure(64));
    flags_init<<<1, 64, 0, ctx->stream>>>(ctx->g_flags.as<uint32_t>());
    SHD_HIP(hipGetLastError());
    return SHD_OK;
}

// Wide path: u64 latency, global labels, Jacobi rounds over in-arcs; batches of sources.
static shd_status run_wide(shd_ctx* ctx, uint32_t rb, uint32_t re, uint64_t* d_lat, float* d_loss,
                           shd_error* err) {
    PreparedGraph& P = ctx->prep;
    shd_graph g = P.view();
    HostGraph R;
    build_csr(&g, /*reverse=*/true, R);
    hipStream_t s = ctx->stream;
    DevBuf w_off, w_src, w_lat, w_loss, w_q;
    SHD_TRY(upload(w_off, R.off, s));
    SHD_TRY(upload(w_src, R.dst, s));
    SHD_TRY(upload(w_lat, R.lat, s));
    SHD_TRY(upload(w_loss, R.loss, s));
    SHD_TRY(w_q.ensure(std::max<size_t>(R.loss.size(), 1) * 4));
    if (!R.loss.empty())
        arcs_q<<<div_up(R.loss.size(), 256), 256, 0, s>>>(w_loss.as<float>(), w_q.as<float>(), R.loss.size());
    const uint32_t V = R.V, n_used = P.n_used;
    const uint32_t batch = std::max<uint32_t>(
        1, std::min<uint32_t>(re - rb, (uint32_t)((1ull << 30) / (24ull * V))));
    DevBuf la, pa, lb, pb, ch, pr;
    if (ctx->nh_out) SHD_TRY(pr.ensure((size_t)batch * V * 4));
    SHD_TRY(la.ensure((size_t)batch * V * 8));
    SHD_TRY(lb.ensure((size_t)batch * V * 8));
    SHD_TRY(pa.ensure((size_t)batch * V * 4));
    SHD_TRY(pb.ensure((size_t)batch * V * 4));
    SHD_TRY(ch.ensure(4));
    for (uint32_t r0 = rb; r0 < re; r0 += batch) {
        const uint32_t nb = std::min(batch, re - r0);
        dim3 gv(div_up(V, 256), nb);
        wide_init<<<gv, 256, 0, s>>>(la.as<uint64_t>(), pa.as<float>(), V, ctx->g_used.as<uint32_t>(), r0);
        for (;;) {
            SHD_HIP(hipMemsetAsync(ch.p, 0, 4, s));
            sssp_wide_round<<<gv, 256, 0, s>>>(w_off.as<uint32_t>(), w_src.as<uint32_t>(),
                                               w_lat.as<uint64_t>(), w_q.as<float>(), V,
                                               la.as<uint64_t>(), pa.as<float>(), lb.as<uint64_t>(),
                                               pb.as<float>(), ch.as<uint32_t>(), ctx->g_flags.as<uint32_t>());
            uint32_t changed = 0;
            SHD_HIP(hipMemcpyAsync(&changed, ch.p, 4, hipMemcpyDeviceToHost, s));
            SHD_HIP(hipStreamSynchronize(s));
            std::swap(la, lb);
            std::swap(pa, pb);
            if (!changed) break;
        }
        dim3 ge(div_up(n_used, 256), nb);
        if (ctx->nh_out) {
            wide_pred<<<gv, 256, 0, s>>>(w_off.as<uint32_t>(), w_src.as<uint32_t>(), w_lat.as<uint64_t>(),
                                         w_q.as<float>(), V, la.as<uint64_t>(), pa.as<float>(),
                                         ctx->g_used.as<uint32_t>(), r0, pr.as<uint32_t>());
            wide_next_hop<<<ge, 256, 0, s>>>(pr.as<uint32_t>(), V, ctx->g_used.as<uint32_t>(), n_used, r0, r0 - rb,
                                             ctx->nh_out);
        }
        wide_emit<<<ge, 256, 0, s>>>(la.as<uint64_t>(), pa.as<float>(), V, ctx->g_used.as<uint32_t>(),
                                     n_used, r0, r0 - rb, ctx->g_diag_lat.as<uint64_t>(),
                                     ctx->g_diag_loss.as<float>(), d_lat, d_loss,
                                     reinterpret_cast<unsigned long long*>(ctx->g_flags.as<char>() + 16));
    }
    SHD_TRY(read_flags(ctx));
    if ((uint32_t)(ctx->h_pin[0] >> 32)) return set_err(err, SHD_ERR_LATENCY_OVERFLOW, 0, 0);
    ctx->info.wide_latency = 1;
    return check_unreach(ctx, err);
}

shd_status routing_prepare_impl(shd_ctx* ctx, const shd_graph* g, const uint32_t* used,
                                uint32_t n_used, uint32_t mode, shd_error* err) {
    if (err) *err = shd_error{SHD_OK, 0, 0};
    PreparedGraph& P = ctx->prep;
    P.ready = false;
    SHD_TRY(validate(g, used, n_used));
    if (mode != SHD_ROUTE_SHORTEST && mode != SHD_ROUTE_DIRECT) return SHD_ERR_INVALID;
    hipStream_t s = ctx->stream;
    P.mode = mode;
    P.reordered = false;
    P.spread = false;
    P.V = g->n_nodes;
    P.n_used = n_used;
    P.directed = g->directed != 0;
    P.used.assign(used, used + n_used);
    P.used_ident = n_used == g->n_nodes;
    for (uint32_t j = 0; j < n_used && P.used_ident; j++) P.used_ident = used[j] == j;
    P.node_ids.resize(g->n_nodes);
    for (uint32_t v = 0; v < g->n_nodes; v++) P.node_ids[v] = gml_id(g, v);
    P.es.assign(g->edge_src, g->edge_src + g->n_edges);
    P.ed.assign(g->edge_dst, g->edge_dst + g->n_edges);
    P.el.assign(g->edge_latency_ns, g->edge_latency_ns + g->n_edges);
    P.ep.assign(g->edge_packet_loss, g->edge_packet_loss + g->n_edges);
    SHD_TRY(upload(ctx->g_used, P.used, s));
    if (mode == SHD_ROUTE_DIRECT) {
        std::vector<int32_t> col(g->n_nodes, -1);
        for (uint32_t j = 0; j < n_used; j++) col[used[j]] = (int32_t)j;
        SHD_TRY(upload(ctx->d_es, P.es, s));
        SHD_TRY(upload(ctx->d_ed, P.ed, s));
        SHD_TRY(upload(ctx->d_el, P.el, s));
        SHD_TRY(upload(ctx->d_ep, P.ep, s));
        SHD_TRY(upload(ctx->d_col, col, s));
    } else {
        HostGraph H;
        SHD_TRY(diag_from_self_loops(g, used, n_used, H, err));
        SHD_TRY(upload(ctx->g_diag_lat, H.diag_lat, s));
        SHD_TRY(upload(ctx->g_diag_loss, H.diag_loss, s));
        build_csr(g, /*reverse=*/false, H);
        P.arcs = H.dst.size();
        P.dense_rows = csr_is_dense(H);
        P.max_arc_lat = H.max_arc_lat;
        P.narrow_arcs = H.max_arc_lat < kLat32Inf;
        P.mean_arc_lat = H.dst.empty() ? 1u
                         : (uint32_t)std::min<double>(kLat32Inf - 1, H.sum_arc_lat / H.dst.size());
        P.min_arc_lat = H.dst.empty() ? 1u : (uint32_t)std::min<uint64_t>(kLat32Inf - 1, std::max<uint64_t>(H.min_arc_lat, 1));
        if (P.narrow_arcs) {
            std::vector<uint32_t> l32(H.lat.begin(), H.lat.end());
            SHD_TRY(upload(ctx->g_off, H.off, s));
            SHD_TRY(upload(ctx->g_dst, H.dst, s));
            SHD_TRY(upload(ctx->g_lat, l32, s));
            SHD_TRY(upload(ctx->g_aux, H.loss, s));
            SHD_TRY(ctx->g_arc16.ensure(std::max<size_t>(H.loss.size(), 1) * 16));
            SHD_TRY(ctx->g_arc8.ensure(std::max<size_t>(H.loss.size(), 1) * 8));
            SHD_TRY(ctx->g_aq.ensure(std::max<size_t>(H.loss.size(), 1) * 4));
            if (!H.loss.empty())
                arcs_pack<<<div_up(H.loss.size(), 256), 256, 0, s>>>(
                    ctx->g_dst.as<uint32_t>(), ctx->g_lat.as<uint32_t>(), ctx->g_aux.as<float>(),
                    ctx->g_arc16.as<uint4>(), ctx->g_arc8.as<uint2>(), ctx->g_aq.as<float>(), H.loss.size());
            P.pruned_arcs = 0;
            P.tight_arcs = 0;
            SHD_TRY(prepare_reordered(ctx, H, used, n_used));
            SHD_TRY(prepare_spread(ctx, H, used, n_used));
        }
    }
    SHD_HIP(hipStreamSynchronize(s));
    P.ready = true;
    return SHD_OK;
}

static shd_status run_direct(shd_ctx* ctx, uint32_t rb, uint32_t re, uint64_t* d_lat,
                             float* d_loss, shd_error* err) {
    PreparedGraph& P = ctx->prep;
    hipStream_t s = ctx->stream;
    const uint32_t n_used = P.n_used;
    const uint64_t nn = (uint64_t)n_used * n_used;
    const uint32_t E = (uint32_t)P.es.size();
    DevBuf cnt, tl, tp;
    SHD_TRY(cnt.ensure(nn * 4));
    SHD_TRY(tl.ensure(nn * 8));
    SHD_TRY(tp.ensure(nn * 4));
    SHD_HIP(hipEventRecord(ctx->ev[2], s));
    SHD_HIP(hipMemsetAsync(cnt.p, 0, nn * 4, s));
    if (E)
        direct_scatter<<<div_up(E, 256), 256, 0, s>>>(
            ctx->d_es.as<uint32_t>(), ctx->d_ed.as<uint32_t>(), ctx->d_el.as<uint64_t>(),
            ctx->d_ep.as<float>(), E, P.directed, ctx->d_col.as<int32_t>(), n_used,
            cnt.as<uint32_t>(), tl.as<uint64_t>(), tp.as<float>());
    auto* bad_d = reinterpret_cast<unsigned long long*>(ctx->g_flags.as<char>() + 16);
    direct_check<<<div_up(nn, 256), 256, 0, s>>>(cnt.as<uint32_t>(), nn, bad_d);
    const size_t rows = re - rb;
    if (ctx->nh_out && rows)
        direct_next_hop<<<div_up((uint64_t)rows * n_used, 256), 256, 0, s>>>(ctx->g_used.as<uint32_t>(), n_used, rb,
                                                                             (uint32_t)rows, ctx->nh_out);
    SHD_HIP(hipMemcpyAsync(d_lat, tl.as<uint64_t>() + (size_t)rb * n_used, rows * n_used * 8,
                           hipMemcpyDeviceToDevice, s));
    SHD_HIP(hipMemcpyAsync(d_loss, tp.as<float>() + (size_t)rb * n_used, rows * n_used * 4,
                           hipMemcpyDeviceToDevice, s));
        unsigned long long bad = 0;
    SHD_HIP(hipMemcpyAsync(&bad, bad_d, 8, hipMemcpyDeviceToHost, s));
    uint32_t c = 0;
    SHD_HIP(hipStreamSynchronize(s));
    if (bad != ~0ull) {
        SHD_HIP(hipMemcpyAsync(&c, cnt.as<uint32_t>() + bad, 4, hipMemcpyDeviceToHost, s));
        SHD_HIP(hipStreamSynchronize(s));
        const uint32_t r = (uint32_t)(bad / n_used), q = (uint32_t)(bad % n_used);
        return set_err(err, c == 0 ? SHD_ERR_NO_EDGE : SHD_ERR_MULTI_EDGE, P.node_ids[P.used[r]],
                       P.node_ids[P.used[q]]);
    }
    return SHD_OK;
}

struct ArcView {
    const uint32_t *beg, *end;
    const uint4* arcs;
    uint64_t n_arcs;
    bool padded = false;   // lists padded to kArcPad slots with no-op arcs (prune_rows)
    const uint32_t* used = nullptr;   // a relabelled copy (prepare_spread): the used nodes' new ids
};

template <int BLOCK, int G, bool CACHE>
static void launch_group(shd_ctx* ctx, const ArcView& A, uint32_t rb, uint32_t re, size_t lds,
                         uint64_t* d_lat, float* d_loss, uint32_t delta, const uint32_t* seed,
                         uint32_t seed_stride, uint32_t use_offl) {
    PreparedGraph& P = ctx->prep;
    constexpr int R = G >= 32 ? 2 : G == 4 ? 2 : 4;   // arcs in flight per lane (R = 6, 8 at G = 8 measured slower on C2)
    // padded lists: labels stay below 2^32 - 1 while lu <= guard (0 = unpadded path)
    const uint64_t guard = (uint64_t)kLat32Inf - 1 - P.max_arc_lat;
    const uint32_t lat_guard =
        A.padded && delta != kLat32Inf && !seed && P.max_arc_lat < kLat32Inf - 1 &&
                ctx->knobs.get(K_SSSP_NO_PAD, 0) != 1
            ? (uint32_t)std::max<uint64_t>(guard, 1)
            : 0u;
    uint32_t* flags = ctx->g_flags.as<uint32_t>();
    auto* unreach = reinterpret_cast<unsigned long long*>(ctx->g_flags.as<char>() + 16);
    auto* stats = ctx->stats_on ? reinterpret_cast<unsigned long long*>(ctx->g_flags.as<char>() + 32) : nullptr;
    hipEvent_t e0 = ctx->time_now ? ctx->ev[2] : nullptr, e1 = ctx->time_now ? ctx->ev[3] : nullptr;
    const uint32_t* usedp = A.used ? A.used : P.used_ident ? nullptr : (const uint32_t*)ctx->g_used.as<uint32_t>();
    if constexpr (kArcPad % (G * 8) == 0) {
        if (lat_guard) {
            hipExtLaunchKernelGGL(sssp_lds_group<BLOCK, G, R, CACHE, 8>, dim3(re - rb), dim3(BLOCK), (uint32_t)lds,
                                  ctx->stream, e0, e1, 0u, A.beg, A.end, A.arcs, P.V, usedp, P.n_used, rb,
                                  (const uint64_t*)ctx->g_diag_lat.as<uint64_t>(),
                                  (const float*)ctx->g_diag_loss.as<float>(), d_lat, d_loss, flags, unreach, delta,
                                  stats, seed, seed_stride, ctx->nh_out, lat_guard, use_offl, 0u, 0u);
            return;
        }
    }
    // edge-parallel expansion (expand_flat) for sparse graphs whose hubs would idle a node
    // group's wave (SHD_SSSP_LFLAT=1), when its per-wave scratch fits beside the rest
    const size_t flat_off = (lds + 15) & ~(size_t)15, flat_bytes = (size_t)(BLOCK / 64) * kFlatWords * 4;
    const bool flatl = !A.padded && !seed && delta != kLat32Inf && ctx->knobs.get(K_SSSP_LFLAT, 0) == 1 &&
                       flat_off + flat_bytes <= ctx->max_lds;
    auto kern = flatl ? sssp_lds_group<BLOCK, G, R, CACHE, 0, true> : sssp_lds_group<BLOCK, G, R, CACHE, 0, false>;
    hipExtLaunchKernelGGL(kern, dim3(re - rb), dim3(BLOCK), (uint32_t)(flatl ? flat_off + flat_bytes : lds),
                          ctx->stream, e0, e1, 0u, A.beg, A.end, A.arcs, P.V, usedp, P.n_used, rb,
                          (const uint64_t*)ctx->g_diag_lat.as<uint64_t>(), (const float*)ctx->g_diag_loss.as<float>(),
                          d_lat, d_loss, flags, unreach, delta, stats, seed, seed_stride, ctx->nh_out, 0u,
                          use_offl, (uint32_t)flat_off, flatl ? 0u : ctx->knobs.get(K_SSSP_HUB, kHubDeg));
}

static size_t sssp_lds_bytes(uint32_t V, uint32_t block, bool cache) {
    // labels + bitmap + control + per-wave queues (+ arc ranges, 8-byte aligned)
    const size_t head = (size_t)(V + 64) * 8 + (size_t)((V + 31) / 32) * 4 + 16 + (block / 64) * kQStride * 4;
    return cache ? ((head + 7) & ~(size_t)7) + (size_t)V * 8 : head;
}

template <int BLOCK, bool CACHE>
static void launch_by_degree(shd_ctx* ctx, const ArcView& A, uint32_t rb, uint32_t re, uint64_t* d_lat,
                             float* d_loss, uint32_t delta, uint32_t G, const uint32_t* seed,
                             uint32_t ss) {
    const uint32_t V = ctx->prep.V;
    size_t lds = sssp_lds_bytes(V, BLOCK, CACHE);
    if (ctx->nh_out && !CACHE) lds = ((lds + 7) & ~(size_t)7) + (size_t)V * 4;   // pred[V]
    // no room for the {beg, end} cache: a plain CSR's offsets alone (4 B/node) when they fit
    // (C3, 10k nodes: every relaxation's arc range from LDS instead of two dependent loads)
    uint32_t use_offl = 0;
    if (!CACHE && A.end == A.beg + 1 && lds + (size_t)(V + 1) * 4 + 8 <= ctx->max_lds &&
        ctx->knobs.get(K_SSSP_NO_OFFL, 0) != 1) {
        lds = ((lds + 7) & ~(size_t)7) + (size_t)(V + 1) * 4;
        use_offl = 1;
    }
    switch (G) {
        case 64: launch_group<BLOCK, 64, CACHE>(ctx, A, rb, re, lds, d_lat, d_loss, delta, seed, ss, use_offl); break;
        case 32: launch_group<BLOCK, 32, CACHE>(ctx, A, rb, re, lds, d_lat, d_loss, delta, seed, ss, use_offl); break;
        case 16: launch_group<BLOCK, 16, CACHE>(ctx, A, rb, re, lds, d_lat, d_loss, delta, seed, ss, use_offl); break;
        case 8: launch_group<BLOCK, 8, CACHE>(ctx, A, rb, re, lds, d_lat, d_loss, delta, seed, ss, use_offl); break;
        default: launch_group<BLOCK, 4, CACHE>(ctx, A, rb, re, lds, d_lat, d_loss, delta, seed, ss, use_offl); break;
    }
}

static shd_status run_sssp(shd_ctx* ctx, const ArcView& A, uint32_t rb, uint32_t re,
                           uint64_t* d_lat, float* d_loss, uint32_t delta, bool* ovf,
                           const uint32_t* seed = nullptr, uint32_t ss = 0) {
    PreparedGraph& P = ctx->prep;
    hipStream_t s = ctx->stream;
    const double deg = (double)A.n_arcs / std::max<uint32_t>(P.V, 1);
    // G lanes x R arcs (R = 4 below G = 32) per node; measured best on C2 (pruned, ~48 arcs
    // per node) at G = 8 and on C3 (BA, ~6 arcs per node) at G = 4
    uint32_t G = deg >= 64 ? 16 : deg >= 24 ? 8 : 4;
    G = ctx->knobs.get(K_SSSP_G, G);          // tuning overrides (results are identical)
    // Workgroup shape: once a source's labels need most of the LDS, one 1024-thread workgroup
    // per CU (the LDS arc-range cache is dropped when it no longer fits).  Otherwise rows per CU
    // decide: with one row or fewer per CU the row's sweeps are the critical path and 16 waves
    // shorten them (C2, 125 rows: 71 us at 1024 threads vs 151 at 256); with ~4 rows per CU
    // the CU is full either way and 256 is best (196 vs 252 us).
    const size_t half = ctx->max_lds / 2;
    const uint32_t rows_per_cu = div_up(re - rb, (uint32_t)ctx->n_cu);
    uint32_t block = sssp_lds_bytes(P.V, 256, true) > half ? 1024
                     : rows_per_cu <= 1 ? 1024 : rows_per_cu <= 2 ? 512 : 256;
    block = ctx->knobs.get(K_SSSP_BLOCK, block);
    if (block != 256 && block != 512 && block != 1024) block = 256;
    // (edge-parallel expand_flat, as in the global-label kernel, measured slower here: the
    // kernel is issue-bound and the owner search costs more than the dead group slots; C2
    // 132 -> 197 us, so the LDS kernels keep node groups)
    const bool cache = sssp_lds_bytes(P.V, block, true) <= ctx->max_lds;
    // launch_group records ev[2] / ev[3] on the kernel's dispatch packet (hipExtLaunchKernel):
    // separate event markers around it cost ~6 us of queue gap each on C2
    if (block == 1024) {
        if (cache) launch_by_degree<1024, true>(ctx, A, rb, re, d_lat, d_loss, delta, G, seed, ss);
        else launch_by_degree<1024, false>(ctx, A, rb, re, d_lat, d_loss, delta, G, seed, ss);
    } else if (block == 512) {
        if (cache) launch_by_degree<512, true>(ctx, A, rb, re, d_lat, d_loss, delta, G, seed, ss);
        else launch_by_degree<512, false>(ctx, A, rb, re, d_lat, d_loss, delta, G, seed, ss);
    } else {
        if (cache) launch_by_degree<256, true>(ctx, A, rb, re, d_lat, d_loss, delta, G, seed, ss);
        else launch_by_degree<256, false>(ctx, A, rb, re, d_lat, d_loss, delta, G, seed, ss);
    }
    SHD_HIP(hipGetLastError());
    (void)ovf;   // the caller reads the overflow flag with read_flags()
    if (ctx->stats_on) {
        unsigned long long st[2];
        SHD_HIP(hipMemcpyAsync(st, ctx->g_flags.as<char>() + 32, 16, hipMemcpyDeviceToHost, s));
        SHD_HIP(hipStreamSynchronize(s));
        std::fprintf(stderr, "shd_sssp: rows=%u G=%u block=%u delta=%u expanded=%llu (%.2f per node) "
                     "sweeps=%llu (%.1f per row) arcs=%llu\n", re - rb, G, block, delta, st[0],
                     (double)st[0] / ((double)(re - rb) * P.V), st[1], (double)st[1] / (re - rb),
                     (unsigned long long)A.n_arcs);
    }
    return SHD_OK;
}

template <int BLOCK, int G>
static void launch_global(shd_ctx* ctx, const ArcView& A, uint32_t rb, uint32_t re, uint32_t grid,
                          size_t lds, uint64_t* d_lat, float* d_loss, uint32_t delta, uint32_t use_bkt,
                          uint32_t use_flat, uint32_t kl) {
    PreparedGraph& P = ctx->prep;
    constexpr int R = G >= 32 ? 2 : 4;
    // the events ride on the dispatch packet: the kernel's own duration, no marker gaps
    // flat + bucket bytes + delta (C4's configuration): the kernel without the other paths
    const bool fast = use_bkt && use_flat && delta != kLat32Inf;
    auto kern = fast ? sssp_global_group<BLOCK, G, R, true> : sssp_global_group<BLOCK, G, R, false>;
    // the locality-ordered copy (prepare_reordered) when it exists and no next hops are asked for
    const bool ro = fast && P.reordered && !ctx->nh_out && ctx->knobs.get(K_SSSP_NO_REORDER, 0) != 1;
    const uint32_t* beg = ro ? ctx->g_offr.as<uint32_t>() : A.beg;
    const uint32_t* end = ro ? ctx->g_offr.as<uint32_t>() + 1 : A.end;
    const uint32_t* usedp = ro ? ctx->g_usedr.as<uint32_t>() : ctx->g_used.as<uint32_t>();
    const uint2* a8 = ro ? ctx->g_arc8r.as<uint2>() : ctx->g_arc8.as<uint2>();
    const float* aqp = ro ? ctx->g_aqr.as<float>() : ctx->g_aq.as<float>();
    // dynamic row claiming (SHD_SSSP_DYN=0: fixed round-robin rows, for A/B)
    uint32_t* row_ctr = nullptr;
    if (ctx->knobs.get(K_SSSP_DYN, 1) != 0) {
        row_ctr = reinterpret_cast<uint32_t*>(ctx->g_flags.as<char>() + 48);
        (void)hipMemsetAsync(row_ctr, 0, 4, ctx->stream);
    }
    hipExtLaunchKernelGGL(
        kern, dim3(grid), dim3(BLOCK), (uint32_t)lds, ctx->stream,
        ctx->time_now ? ctx->ev[2] : nullptr, ctx->time_now ? ctx->ev[3] : nullptr, 0u,
        beg, end, A.arcs, P.V, usedp, P.n_used, rb, re,
        (const uint64_t*)ctx->g_diag_lat.as<uint64_t>(), (const float*)ctx->g_diag_loss.as<float>(), d_lat, d_loss,
        ctx->g_flags.as<uint32_t>(), reinterpret_cast<unsigned long long*>(ctx->g_flags.as<char>() + 16), delta,
        ctx->stats_on ? reinterpret_cast<unsigned long long*>(ctx->g_flags.as<char>() + 32) : nullptr,
        ctx->g_glab.as<uint64_t>(), use_bkt, use_flat, ctx->nh_out,
        ctx->nh_out ? ctx->g_pred.as<uint32_t>() : nullptr, a8, aqp, ro ? kl : 0u, row_ctr);
}

// Kernel 1b driver: labels in global memory (graphs whose labels exceed the LDS).
static shd_status run_sssp_global(shd_ctx* ctx, const ArcView& A, uint32_t rb, uint32_t re,
                                  uint64_t* d_lat, float* d_loss, uint32_t delta, bool* ovf) {
    PreparedGraph& P = ctx->prep;
    constexpr uint32_t BLOCK = 512;   // a 1024-thread single slot per CU: rows 0-4095 23.5 vs 19.1 ms
    const uint32_t W = (P.V + 31) / 32;
    // bitmap + control + per-wave queues (+ delta-stepping: one bucket byte per node, when it
    // fits beside the bitmap; else the sweeps read the active nodes' global labels)
    const uint32_t use_flat = ctx->knobs.get(K_SSSP_FLAT, 1) != 0;   // edge-parallel expansion
    size_t lds = (size_t)W * 4 + 16 + (BLOCK / 64) * (kQStride + (use_flat ? kFlatWords : 0)) * 4;
    if (lds > ctx->max_lds) return SHD_ERR_INVALID;   // bitmap of > ~1.2M nodes
    const size_t lds_bkt = lds + ((size_t)P.V + 3) / 4 * 4;
    const uint32_t use_bkt = delta != kLat32Inf && lds_bkt <= ctx->max_lds && ctx->knobs.get(K_SSSP_NO_BKT, 0) != 1;
    if (use_bkt) lds = lds_bkt;
    // the flat + bucket-byte kernel (FASTG) keeps a per-word minimum key beside the bitmap
    uint32_t flat_arg = use_flat;
    if (use_bkt && use_flat && delta != kLat32Inf && ctx->knobs.get(K_SSSP_WMIN, 1) != 0 && lds + (size_t)W * 4 <= ctx->max_lds) {
        lds += (size_t)W * 4;
        flat_arg |= 2u;
    }
    const uint32_t per_cu = std::max<uint32_t>(1, ctx->knobs.get(K_SSSP_SLOTS, 2));
    // labels of the first kl nodes (locality order: highest degree first) in the LDS left over by
    // per_cu slots per CU: their relaxations take LDS atomics instead of memory-side ones
    uint32_t kl = 0;
    if (use_bkt && use_flat && delta != kLat32Inf && P.reordered && !ctx->nh_out &&
        ctx->knobs.get(K_SSSP_NO_LDS_LABELS, 0) != 1) {
        const size_t room = ctx->max_lds / per_cu;
        if (room > lds + 64) kl = std::min<uint32_t>(std::min<uint32_t>(P.V, P.lds_labels), (uint32_t)((room - lds - 16) / 8)) & ~63u;
        if (kl) lds = ((lds + 7) & ~(size_t)7) + (size_t)kl * 8;
    }
    const uint32_t slots = (uint32_t)ctx->n_cu * per_cu;
    const uint32_t reserve = std::max(ctx->slot_reserve, ctx->knobs.get(K_SSSP_RESERVE, 0));   // env: tools/overlap_probe.py
    const uint32_t grid = std::min<uint32_t>(re - rb, slots - std::min(reserve, slots / 2));
    SHD_TRY(ctx->g_glab.ensure((size_t)grid * P.V * 8));
    if (ctx->nh_out) SHD_TRY(ctx->g_pred.ensure((size_t)grid * P.V * 4));
    const double deg = (double)A.n_arcs / std::max<uint32_t>(P.V, 1);
    const uint32_t G = ctx->knobs.get(K_SSSP_G, deg >= 64 ? 16 : deg >= 24 ? 8 : 4);
    switch (G) {
        case 16: launch_global<BLOCK, 16>(ctx, A, rb, re, grid, lds, d_lat, d_loss, delta, use_bkt, flat_arg, kl); break;
        case 8: launch_global<BLOCK, 8>(ctx, A, rb, re, grid, lds, d_lat, d_loss, delta, use_bkt, flat_arg, kl); break;
        default: launch_global<BLOCK, 4>(ctx, A, rb, re, grid, lds, d_lat, d_loss, delta, use_bkt, flat_arg, kl); break;
    }
    SHD_HIP(hipGetLastError());
    (void)ovf;   // the caller reads the overflow flag with read_flags()
    if (ctx->stats_on) {
        unsigned long long st[2];
        SHD_HIP(hipMemcpyAsync(st, ctx->g_flags.as<char>() + 32, 16, hipMemcpyDeviceToHost, ctx->stream));
        SHD_HIP(hipStreamSynchronize(ctx->stream));
        std::fprintf(stderr, "shd_sssp_global: rows=%u G=%u slots=%u delta=%u expanded=%llu (%.2f per node) "
                     "sweeps=%llu (%.1f per row)\n", re - rb, G, grid, delta, st[0],
                     (double)st[0] / ((double)(re - rb) * P.V), st[1], (double)st[1] / (re - rb));
    }
    return SHD_OK;
}

shd_status fw_latency(shd_ctx* ctx, uint32_t* D, uint32_t Vp, uint32_t T);
shd_status fw_tight(shd_ctx* ctx, const uint32_t* D, uint32_t Vp, uint32_t* pbeg, uint32_t* pend,
                    uint4* parcs, uint32_t* cursor);

// SHD_ALGO_BLOCKED (blocked.hip): latency closure by blocked min-plus, then the loss pass over
// the globally tight arcs with labels seeded from the closure rows.
static shd_status run_blocked(shd_ctx* ctx, uint32_t rb, uint32_t re, uint64_t* d_lat,
                              float* d_loss, bool* ovf) {
    PreparedGraph& P = ctx->prep;
    hipStream_t s = ctx->stream;
    const uint32_t V = P.V;
    const uint32_t T = ctx->knobs.get(K_FW_TILE, V > 2048 ? 128 : 64) == 128 ? 128 : 64;
    const uint32_t Vp = (V + T - 1) / T * T;
    SHD_TRY(ctx->g_fw.ensure((size_t)Vp * Vp * 4));
    SHD_TRY(ctx->g_prune_dst.ensure(std::max<uint64_t>(P.arcs, 1) * 16));
    SHD_TRY(ctx->g_prune_cnt.ensure((size_t)V * 8 + 16));
    uint32_t* D = ctx->g_fw.as<uint32_t>();
    uint32_t* pbeg = ctx->g_prune_cnt.as<uint32_t>();
    uint32_t* pend = pbeg + V;
    uint32_t* cursor = pend + V;
    SHD_HIP(hipEventRecord(ctx->ev[4], s));
    SHD_TRY(fw_latency(ctx, D, Vp, T));
    SHD_HIP(hipEventRecord(ctx->ev[5], s));
    SHD_TRY(fw_tight(ctx, D, Vp, pbeg, pend, ctx->g_prune_dst.as<uint4>(), cursor));
    if (P.tight_arcs == 0) {   // the kept-arc count steers the lane-group width (once per graph)
        uint32_t k = 0;
        SHD_HIP(hipMemcpyAsync(&k, cursor, 4, hipMemcpyDeviceToHost, s));
        SHD_HIP(hipStreamSynchronize(s));
        P.tight_arcs = std::max<uint32_t>(k, 1);
    }
    ArcView A{pbeg, pend, ctx->g_prune_dst.as<uint4>(), P.tight_arcs};
    SHD_TRY(run_sssp(ctx, A, rb, re, d_lat, d_loss, kLat32Inf, ovf, D, Vp));
    float ms = 0;
    SHD_HIP(hipEventSynchronize(ctx->ev[5]));
    (void)hipEventElapsedTime(&ms, ctx->ev[4], ctx->ev[5]);
    ctx->info.ms_minplus = ms;
    ctx->info.arcs_kept = P.tight_arcs;
    return SHD_OK;
}

constexpr uint32_t kPruneK = 32;
constexpr uint32_t kPruneMaxV = 4096;
constexpr uint32_t kBlockedMaxV = 16384;   // closure matrix <= 1 GiB

// Dense arc matrix + k-nearest 2-hop prune over all V rows -> pruned arc lists (row stride V).
static shd_status run_prune(shd_ctx* ctx, ArcView* out) {
    PreparedGraph& P = ctx->prep;
    hipStream_t s = ctx->stream;
    const uint32_t V = P.V;
    const uint64_t nn = (uint64_t)V * V;
    SHD_TRY(ctx->g_prune_dst.ensure((nn + (uint64_t)V * kArcPad) * 16));   // + list padding
    SHD_TRY(ctx->g_prune_cnt.ensure((size_t)V * 8 + 16));
    uint32_t* pbeg = ctx->g_prune_cnt.as<uint32_t>();
    uint32_t* pend = pbeg + V;
    uint32_t* cursor = pend + V;
    uint4* pa = ctx->g_prune_dst.as<uint4>();
    uint32_t* flags = ctx->g_flags.as<uint32_t>();
    const uint32_t Kr = ctx->knobs.get(K_PRUNE_K, kPruneK);   // tuning: detour nodes per row (same output tables)
    const uint32_t K = Kr >= 128 ? 128u : Kr >= 64 ? 64u : 32u;
    const size_t plds = (size_t)V * 22 + (8 + 256 + 2 * (size_t)K) * 4;
    // K = 32 (the default): the sorted-detour kernel (CMP) with the first batch's survivors
    // packed; SHD_PRUNE_SHAPE=0 keeps the round-4 kernel for A/B (same tables)
    const size_t plds_c = plds + 8 + (size_t)V * 12 + 64 * 12;   // + survivors (uint2 each), sort scratch, losses
    const bool legacy = ctx->knobs.get(K_PRUNE_SHAPE, 1) == 0;
    // bins from the graph's largest arc latency instead of each row's (SHD_PRUNE_SHAPE_SH=0: per row)
    const uint32_t gbits = 64u - (uint32_t)__builtin_clzll(std::max<uint64_t>(std::min<uint64_t>(P.max_arc_lat, kLat32Inf - 1), 1));
    const uint32_t shg = ctx->knobs.get(K_PRUNE_SHAPE_SH, 1) ? (gbits > 8 ? gbits - 8 : 0) : 0xFFFFFFFFu;
    if (P.dense_rows && !ctx->knobs.on(K_PRUNE_DENSE_BUILD)) {
        // the CSR is the dense matrix (complete graph, arcs in index order): prune straight from it
        const uint32_t* Wl = ctx->g_lat.as<uint32_t>();
        const float* Wp = ctx->g_aux.as<float>();
        if (K >= 128) prune_rows<256, 128, true><<<V, 256, plds, s>>>(Wl, Wp, V, pbeg, pend, pa, cursor, flags);
        else if (K >= 64) prune_rows<256, 64, true><<<V, 256, plds, s>>>(Wl, Wp, V, pbeg, pend, pa, cursor, flags);
        else if (legacy) prune_rows<256, 32, true><<<V, 256, plds, s>>>(Wl, Wp, V, pbeg, pend, pa, cursor, flags);
        else prune_rows<512, 32, true, 2, 8, true, 12><<<V, 512, plds_c, s>>>(Wl, Wp, V, pbeg, pend, pa, cursor, flags, shg);
    } else {
        SHD_TRY(ctx->g_dense.ensure(nn * 8));
        SHD_TRY(ctx->g_labels.ensure(nn * 4));
        float* Wp = ctx->g_dense.as<float>();   // the lexicographic-min arc's loss per pair (its latency: Wl)
        uint32_t* Wl = ctx->g_labels.as<uint32_t>();
        dense_build<<<V, 256, (size_t)V * 8, s>>>(ctx->g_off.as<uint32_t>(), ctx->g_dst.as<uint32_t>(),
                                                  ctx->g_lat.as<uint32_t>(), ctx->g_aux.as<float>(), V, Wp, Wl, cursor,
                                                  flags);
        if (K >= 128) prune_rows<256, 128><<<V, 256, plds, s>>>(Wl, Wp, V, pbeg, pend, pa, cursor, flags);
        else if (K >= 64) prune_rows<256, 64><<<V, 256, plds, s>>>(Wl, Wp, V, pbeg, pend, pa, cursor, flags);
        else if (legacy) prune_rows<256, 32><<<V, 256, plds, s>>>(Wl, Wp, V, pbeg, pend, pa, cursor, flags);
        else prune_rows<512, 32, false, 2, 8, true, 12><<<V, 512, plds_c, s>>>(Wl, Wp, V, pbeg, pend, pa, cursor, flags, shg);
    }
    SHD_HIP(hipGetLastError());
    *out = ArcView{pbeg, pend, ctx->g_prune_dst.as<uint4>(), 0, true};
    return SHD_OK;
}

static shd_status count_kept(shd_ctx* ctx, const ArcView& A) {
    std::vector<uint32_t> b(ctx->prep.V), e(ctx->prep.V);
    SHD_HIP(hipMemcpyAsync(b.data(), A.beg, b.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
    SHD_HIP(hipMemcpyAsync(e.data(), A.end, e.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    uint64_t k = 0;
    for (size_t i = 0; i < b.size(); i++) k += e[i] - b[i];
    ctx->info.arcs_kept = k;
    ctx->prep.pruned_arcs = k;
    return SHD_OK;
}

static size_t sssp_lds_bytes(uint32_t V, uint32_t block, bool cache);

static shd_status prepare_reordered(shd_ctx* ctx, const HostGraph& H, const uint32_t* used, uint32_t n_used) {
    PreparedGraph& P = ctx->prep;
    P.reordered = false;
    const uint32_t V = P.V;
    if (V == 0 || (sssp_lds_bytes(V, 1024, false) <= ctx->max_lds && ctx->knobs.get(K_SSSP_REORDER, 0) != 1) ||
        ctx->knobs.get(K_SSSP_NO_REORDER, 0) == 1)
        return SHD_OK;   // the LDS kernels take this graph
    hipStream_t s = ctx->stream;
    std::vector<uint32_t> deg(V), roots(V), ord, pi(V, 0xFFFFFFFFu);
    for (uint32_t v = 0; v < V; ++v) {
        deg[v] = H.off[v + 1] - H.off[v];
        roots[v] = v;
    }
    std::stable_sort(roots.begin(), roots.end(), [&](uint32_t a, uint32_t b) { return deg[a] > deg[b]; });
    ord.reserve(V);
    const uint32_t mode = ctx->knobs.get(K_REORDER_MODE, 0);   // tuning: 1 = degree order only
    // the K highest-degree nodes first: the global kernel keeps their labels in LDS (the LDS a
    // slot has left at 2 slots per CU, as run_sssp_global sizes it)
    {
        const size_t W = (V + 31) / 32;
        const size_t lds = W * 4 + 16 + 8 * (kQStride + kFlatWords) * 4 + ((size_t)V + 3) / 4 * 4;
        const size_t room = ctx->max_lds / 2;
        P.lds_labels = room > lds + 64 ? (uint32_t)std::min<size_t>(V, (room - lds - 16) / 8) & ~63u : 0u;
    }
    const uint32_t K = mode == 1 ? V : P.lds_labels;
    for (uint32_t i = 0; i < K && i < V; ++i) {
        pi[roots[i]] = (uint32_t)ord.size();
        ord.push_back(roots[i]);
    }
    {   // breadth-first from the hubs placed so far: their neighbours come next, together
        size_t head = 0;
        while (head < ord.size()) {
            const uint32_t u = ord[head++];
            for (uint32_t k = H.off[u]; k < H.off[u + 1]; ++k) {
                const uint32_t w = H.dst[k];
                if (pi[w] == 0xFFFFFFFFu) {
                    pi[w] = (uint32_t)ord.size();
                    ord.push_back(w);
                }
            }
        }
    }
    for (uint32_t r : roots) {   // breadth-first from each not yet numbered node, hubs first
        if (pi[r] != 0xFFFFFFFFu) continue;
        size_t head = ord.size();
        pi[r] = (uint32_t)ord.size();
        ord.push_back(r);
        while (head < ord.size()) {
            const uint32_t u = ord[head++];
            for (uint32_t k = H.off[u]; k < H.off[u + 1]; ++k) {
                const uint32_t w = H.dst[k];
                if (pi[w] == 0xFFFFFFFFu) {
                    pi[w] = (uint32_t)ord.size();
                    ord.push_back(w);
                }
            }
        }
    }
    const size_t A = H.dst.size();
    std::vector<uint32_t> offr(V + 1, 0), dstr(A), latr(A), usedr(n_used);
    std::vector<float> lossr(A);
    for (uint32_t i = 0; i < V; ++i) {
        const uint32_t u = ord[i];
        uint32_t at = offr[i];
        for (uint32_t k = H.off[u]; k < H.off[u + 1]; ++k, ++at) {
            dstr[at] = pi[H.dst[k]];
            latr[at] = (uint32_t)H.lat[k];
            lossr[at] = H.loss[k];
        }
        offr[i + 1] = at;
    }
    for (uint32_t j = 0; j < n_used; ++j) usedr[j] = pi[used[j]];
    SHD_TRY(upload(ctx->g_offr, offr, s));
    SHD_TRY(upload(ctx->g_usedr, usedr, s));
    DevBuf d_dst, d_lat, d_loss;
    SHD_TRY(upload(d_dst, dstr, s));
    SHD_TRY(upload(d_lat, latr, s));
    SHD_TRY(upload(d_loss, lossr, s));
    SHD_TRY(ctx->g_arc8r.ensure(std::max<size_t>(A, 1) * 8));
    SHD_TRY(ctx->g_aqr.ensure(std::max<size_t>(A, 1) * 4));
    if (A)
        arcs_pack8<<<div_up(A, 256), 256, 0, s>>>(d_dst.as<uint32_t>(), d_lat.as<uint32_t>(), d_loss.as<float>(),
                                                   ctx->g_arc8r.as<uint2>(), ctx->g_aqr.as<float>(), A);
    SHD_HIP(hipGetLastError());
    SHD_HIP(hipStreamSynchronize(s));   // the temporaries are freed on return
    P.reordered = true;
    return SHD_OK;
}

// Wave-spread relabelling for the 1024-thread LDS kernel (sparse graphs whose labels fill the
// LDS, C3).  Its bitmap word k belongs to wave k mod 16 for the whole build, so on a
// preferential-attachment graph -- hubs are the first nodes -- the first waves own every hub and
// the other waves wait for them at each sweep's barrier (24 % of the kernel).  The nodes are
// dealt in descending degree order to the 16 waves' words (rank r -> wave r mod 16), and the
// kernel runs on that copy of the CSR; the table is the same (labels are minima over paths, and
// the used columns keep their order: used[j] -> its new id).  C3 DELTA 6.79 -> 6.59 ms, tables
// identical (tools/c2_probe.py, SSSP_NO_SPREAD=1 alternated; a random relabelling: 7.05).  Not with next hops (the
// kernel would write relabelled ids) nor a seed (indexed by the original ids).
static shd_status prepare_spread(shd_ctx* ctx, const HostGraph& H, const uint32_t* used, uint32_t n_used) {
    PreparedGraph& P = ctx->prep;
    P.spread = false;
    const uint32_t V = P.V;
    constexpr uint32_t NW = 1024 / 64;
    const bool dense = V <= kPruneMaxV && P.arcs * 8 >= (uint64_t)V * V;   // the prune path instead
    if (V == 0 || dense || ctx->knobs.get(K_SSSP_NO_SPREAD, 0) == 1 ||
        sssp_lds_bytes(V, 1024, false) > ctx->max_lds ||          // global labels (C4)
        sssp_lds_bytes(V, 256, true) <= ctx->max_lds / 2)         // not the 1024-thread kernel
        return SHD_OK;
    hipStream_t s = ctx->stream;
    std::vector<uint32_t> deg(V), r2n(V);
    for (uint32_t v = 0; v < V; ++v) {
        deg[v] = H.off[v + 1] - H.off[v];
        r2n[v] = v;
    }
    std::stable_sort(r2n.begin(), r2n.end(), [&](uint32_t a, uint32_t b) { return deg[a] > deg[b]; });
    // rank r -> position ((q / 32) * NW + r mod NW) * 32 + q mod 32 (q = r / NW: the rank's place
    // among its wave's nodes), compacted to 0 .. V-1 in position order
    std::vector<uint64_t> pos(V);
    std::vector<uint32_t> byp(V);
    for (uint32_t r = 0; r < V; ++r) {
        const uint64_t q = r / NW;
        pos[r] = ((q / 32) * NW + r % NW) * 32 + q % 32;
        byp[r] = r;
    }
    std::stable_sort(byp.begin(), byp.end(), [&](uint32_t a, uint32_t b) { return pos[a] < pos[b]; });
    std::vector<uint32_t> pi(V), ord(V);   // node -> new id, new id -> node
    for (uint32_t i = 0; i < V; ++i) {
        ord[i] = r2n[byp[i]];
        pi[ord[i]] = i;
    }
    const size_t A = H.dst.size();
    std::vector<uint32_t> offs(V + 1, 0), dsts(A), lats(A), useds(n_used);
    std::vector<float> losss(A);
    for (uint32_t i = 0; i < V; ++i) {
        const uint32_t u = ord[i];
        uint32_t at = offs[i];
        for (uint32_t k = H.off[u]; k < H.off[u + 1]; ++k, ++at) {
            dsts[at] = pi[H.dst[k]];
            lats[at] = (uint32_t)H.lat[k];
            losss[at] = H.loss[k];
        }
        offs[i + 1] = at;
    }
    for (uint32_t j = 0; j < n_used; ++j) useds[j] = pi[used[j]];
    SHD_TRY(upload(ctx->g_offs, offs, s));
    SHD_TRY(upload(ctx->g_useds, useds, s));
    DevBuf d_dst, d_lat, d_loss, d_a8, d_q;
    SHD_TRY(upload(d_dst, dsts, s));
    SHD_TRY(upload(d_lat, lats, s));
    SHD_TRY(upload(d_loss, losss, s));
    SHD_TRY(ctx->g_arc16s.ensure(std::max<size_t>(A, 1) * 16));
    SHD_TRY(d_a8.ensure(std::max<size_t>(A, 1) * 8));
    SHD_TRY(d_q.ensure(std::max<size_t>(A, 1) * 4));
    if (A)
        arcs_pack<<<div_up(A, 256), 256, 0, s>>>(d_dst.as<uint32_t>(), d_lat.as<uint32_t>(), d_loss.as<float>(),
                                                  ctx->g_arc16s.as<uint4>(), d_a8.as<uint2>(), d_q.as<float>(), A);
    SHD_HIP(hipGetLastError());
    SHD_HIP(hipStreamSynchronize(s));   // the temporaries are freed on return
    P.spread = true;
    return SHD_OK;
}

// the dominant kernel's device time, when this build was timed (shd_routing_set_timing)
static float main_ms(shd_ctx* ctx) {
    // the read-back kernel (readback) can return before the runtime has seen the stop event
    // complete: wait for it, on timed builds only
    float ms = -1.0f;
    if (ctx->time_now && (hipEventSynchronize(ctx->ev[3]) != hipSuccess ||
                          hipEventElapsedTime(&ms, ctx->ev[2], ctx->ev[3]) != hipSuccess))
        ms = -1.0f;
    return ms;
}

shd_status routing_run_impl(shd_ctx* ctx, uint32_t algo, uint32_t rb, uint32_t re,
                            uint64_t* d_lat, float* d_loss, shd_error* err) {
    if (err) *err = shd_error{SHD_OK, 0, 0};
    PreparedGraph& P = ctx->prep;
    if (!P.ready) return SHD_ERR_STATE;
    if (re == 0) re = P.n_used;
    if (rb >= re || re > P.n_used) return SHD_ERR_INVALID;
    ctx->info = shd_routing_info{};
    ctx->info.arcs = P.arcs;
    ctx->info.arcs_kept = P.arcs;
    ctx->time_now = ctx->time_every != 0 && ctx->time_calls++ % ctx->time_every == 0;
    // labels + bitmap + queues (+ next hops: pred[V]) must fit the LDS for the LDS-label kernels
    const size_t lds = sssp_lds_bytes(P.V, 1024, false) + (ctx->nh_out ? (size_t)P.V * 4 + 8 : 0);
    const bool blocked = algo == SHD_ALGO_BLOCKED && P.narrow_arcs && lds <= ctx->max_lds && P.V <= kBlockedMaxV;
    const bool lds_path = !blocked && P.narrow_arcs && lds <= ctx->max_lds && ctx->knobs.get(K_SSSP_GLOBAL, 0) != 1;
    const bool dense = P.V <= kPruneMaxV && P.arcs * 8 >= (uint64_t)P.V * P.V;
    const bool prune = lds_path && P.mode != SHD_ROUTE_DIRECT &&
                       (algo == SHD_ALGO_PRUNED || ((algo == SHD_ALGO_AUTO || algo == SHD_ALGO_DELTA) && dense)) &&
                       P.V <= kPruneMaxV;
    SHD_TRY(ctx->g_flags.ensure(64));
    if (!prune) SHD_TRY(reset_flags(ctx));   // the prune path's dense_build (or prune_rows) resets them
    // wall time of the call (host clock): timing events between the build's kernels cost a
    // few microseconds of queue bubble each, so only the main kernel is bracketed by events
    const auto t_call = std::chrono::steady_clock::now();
    auto call_ms = [&] {
        return std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t_call).count();
    };
    if (P.mode == SHD_ROUTE_DIRECT) {
        shd_status st = run_direct(ctx, rb, re, d_lat, d_loss, err);
        float ms = 0;
        ms = call_ms();
        ctx->info.ms_total = ctx->info.ms_main = ms;
        return st;
    }
    if (blocked) {
        bool ovf = false;
        SHD_TRY(run_blocked(ctx, rb, re, d_lat, d_loss, &ovf));
        ctx->info.algo_used = SHD_ALGO_BLOCKED;
        SHD_TRY(read_flags(ctx));
        ovf = flag_ovf(ctx);
        float ms = 0, ms_main = 0;
        ms = call_ms();
        ms_main = main_ms(ctx);
        ctx->info.ms_total = ms;
        ctx->info.ms_main = ms_main;
        if (!ovf) {
            // an INF closure entry is unreachable OR >= 2^32-1 ns: let the u64 path decide
            const shd_status st = check_unreach(ctx, err);
            if (st != SHD_ERR_UNREACHABLE) return st;
            if (err) *err = shd_error{SHD_OK, 0, 0};
        }
        SHD_TRY(reset_flags(ctx));
        return run_wide(ctx, rb, re, d_lat, d_loss, err);
    }
    if (lds_path) {
        ArcView A{ctx->g_off.as<uint32_t>(), ctx->g_off.as<uint32_t>() + 1, ctx->g_arc16.as<uint4>(),
                  P.arcs};
        if (!prune && P.spread && !ctx->nh_out && ctx->knobs.get(K_SSSP_NO_SPREAD, 0) != 1) {   // prepare_spread
            A = ArcView{ctx->g_offs.as<uint32_t>(), ctx->g_offs.as<uint32_t>() + 1, ctx->g_arc16s.as<uint4>(), P.arcs};
            A.used = ctx->g_useds.as<uint32_t>();
        }
        if (prune) {
            SHD_TRY(run_prune(ctx, &A));
            // the kept-arc count steers the lane-group width: counted once per prepared graph,
            // before its first SSSP launch, so every build (the first too) runs the same kernel
            if (P.pruned_arcs == 0) SHD_TRY(count_kept(ctx, A));
            A.n_arcs = P.pruned_arcs;
        }
        bool ovf = false;
        // delta-stepping bucket width (env override for tuning).  SHD_ALGO_DELTA: the mean arc
        // latency x 1.5 (below).  AUTO on a pruned dense graph: the smallest arc latency (never pruned: every
        // detour has two arcs), floored at mean/256 so that a stray tiny arc cannot make the
        // sweep count explode -- a bucket no wider than every arc settles in one sweep, so each
        // node is expanded once (Dial order); the sweep jumps to the smallest active label, so
        // empty buckets cost nothing.  C2: 1 ms -> main kernel 172 -> 120 us, tables identical.
        // AUTO on a sparse graph: buckets of the mean arc latency (C3: 9.9 ms against 11.6 for
        // plain sweeps; 5 ms buckets 11.4, 2 ms 15.8)
        uint32_t delta = kLat32Inf;
        // (LDS labels: 1.5 x mean_arc_lat.  C3 with the hub relaxation, round 5, tools/c3_delta_sweep.sh:
        // 8 ms 7.85, 10 ms 7.38, 12.5 ms (1.0 x, the old default) 7.03, 16 ms 6.88, 20 ms 6.83-6.84,
        // 25 ms 7.02, 30 ms 7.17, 40 ms 7.64)
        if (algo == SHD_ALGO_DELTA || (algo == SHD_ALGO_AUTO && !prune && ctx->knobs.get(K_SSSP_NO_DELTA, 0) != 1))
            delta = ctx->knobs.get(K_SSSP_DELTA, (uint32_t)std::min<uint64_t>(kLat32Inf - 1, (uint64_t)P.mean_arc_lat * 3 / 2));
        else if (algo == SHD_ALGO_AUTO && prune && ctx->knobs.get(K_SSSP_NO_DELTA, 0) != 1)
            delta = ctx->knobs.get(K_SSSP_DELTA, std::max(P.min_arc_lat, P.mean_arc_lat / 256));
        SHD_TRY(run_sssp(ctx, A, rb, re, d_lat, d_loss, delta, &ovf));
        ctx->info.algo_used = algo == SHD_ALGO_DELTA ? SHD_ALGO_DELTA
                              : prune ? SHD_ALGO_PRUNED : delta != kLat32Inf ? SHD_ALGO_DELTA : SHD_ALGO_SSSP;
        SHD_TRY(read_flags(ctx));
        ovf = flag_ovf(ctx);
        float ms = 0, ms_main = 0;
        ms = call_ms();
        ms_main = main_ms(ctx);
        ctx->info.ms_total = ms;
        ctx->info.ms_main = ms_main;
        ctx->info.arcs_kept = prune ? P.pruned_arcs : P.arcs;
        if (!ovf) return check_unreach(ctx, err);
        SHD_TRY(reset_flags(ctx));  // some path latency >= 2^32-1 ns: redo with u64 labels
    }
    if (P.narrow_arcs && (lds > ctx->max_lds || ctx->knobs.get(K_SSSP_GLOBAL, 0) == 1)) {
        // labels exceed the LDS: global-label kernel (C4)
        bool ovf = false;
        // bucket width: 0.52 x mean_arc_lat, never below the smallest arc.  (mean_arc_lat is the
        // edge latencies' sum over the arc count: half the mean edge latency of an undirected
        // graph -- C4: 12.5 ms of 25 -- so this is 6.5 ms.)  Re-swept at the end of round 2 with
        // the LDS labels and locality order: rows 0-4095 (tools/c4_delta_sweep.sh) 3 ms 20.2 ms,
        // 4 ms 19.4, 5 ms 19.1, 6 ms 19.0, 8 ms 19.3, 10 ms 20.0, 15 ms 22.2; full builds
        // alternated on one box (tools/c4_full_ab.sh) 4 ms 232.3, 5 ms 229.0 / 229.2, 6 ms 228.4 -
        // 228.8, 7 ms 231.0, 10 ms 241.2 / 242.0.  Round 6 (tools/c4_full_ab.sh, alternated): 5 ms
        // 194.2-194.4, 6.5 ms 193.0-193.2, 8 ms 194.8 -> 0.52 x mean_arc_lat
        uint32_t delta = kLat32Inf;
        if (algo == SHD_ALGO_DELTA)
            delta = ctx->knobs.get(K_SSSP_DELTA, std::max(P.min_arc_lat, (uint32_t)(P.mean_arc_lat * 13ull / 25)));
        ArcView A{ctx->g_off.as<uint32_t>(), ctx->g_off.as<uint32_t>() + 1, ctx->g_arc16.as<uint4>(),
                  P.arcs};
        SHD_TRY(run_sssp_global(ctx, A, rb, re, d_lat, d_loss, delta, &ovf));
        ctx->info.algo_used = algo == SHD_ALGO_DELTA ? SHD_ALGO_DELTA : SHD_ALGO_SSSP;
        SHD_TRY(read_flags(ctx));
        ovf = flag_ovf(ctx);
        float ms = 0, ms_main = 0;
        ms = call_ms();
        ms_main = main_ms(ctx);
        ctx->info.ms_total = ms;
        ctx->info.ms_main = ms_main;
        if (!ovf) return check_unreach(ctx, err);
        SHD_TRY(reset_flags(ctx));
    }
    return run_wide(ctx, rb, re, d_lat, d_loss, err);
}

}  // namespace shd

// Test hook (not part of the ABI header): the vector registers of the shipped SSSP kernels,
// which sit at the budgets their residency needs (tests/test_routing_gpu.py): 0 = C4's global-
// label kernel (two 512-thread slots per CU: <= 128), 1 = C2's padded-list kernel (four 256-thread
// workgroups per CU: <= 128), 2 = C3's 1024-thread kernel (<= 128)
extern "C" int shd_debug_kernel_vgprs(int which) {
    hipFuncAttributes at{};
    const void* f = which == 0   ? reinterpret_cast<const void*>(&shd::sssp_global_group<512, 4, 4, true>)
                    : which == 1 ? reinterpret_cast<const void*>(&shd::sssp_lds_group<256, 8, 4, true, 8, false>)
                                 : reinterpret_cast<const void*>(&shd::sssp_lds_group<1024, 4, 2, false, 0, false>);
    return hipFuncGetAttributes(&at, f) == hipSuccess ? at.numRegs : -1;
}

#ifdef SHD_SSSP_PROF
extern "C" int shd_debug_sssp_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(shd::g_sssp_prof), sizeof(unsigned long long) * 8) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(shd::g_sssp_prof), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
extern "C" int shd_debug_prune_prof(unsigned long long* out, int reset) {   // 4096 x 8 words
    (void)reset;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(shd::g_prune_prof), sizeof(unsigned long long) * 4096 * 8) != hipSuccess;
}
#endif
