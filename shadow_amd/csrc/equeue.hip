// Device-resident destination event queues.
//
// Reference: every sent packet becomes Event::new_packet(deliver, src_host, src_event_id) pushed
// into the destination host's Mutex<EventQueue> (src/main/core/worker.rs:619-629), a
// BinaryHeap<Reverse<..>> ordered by (time, Packet before Local, src host id, src event id)
// (src/main/core/work/event.rs:84-155, event_queue.rs:28-48).  At the next round the host pops
// every event with time < window_end (src/main/host/host.rs:697-706), in that order; what
// remains waits for a later round (a latency longer than one window keeps an event pending for
// several rounds).  next_event_time() is the head's time (event_queue.rs:43-45).
//
// Here the pending packet events of all destinations of this GPU are a short list of RUNS, one
// per batch (the relay output of a round: per destination already in that order), each a CSR
// of per-host sorted events with a per-host cursor (its first unpopped event).  An advance
// (shd_equeue_advance) never rewrites the pending events: per host it finds every run's prefix
// below window_end (a binary search from the cursor), merges those prefixes and the batch's into
// the popped output -- the host's popped events staged in LDS and ranked by a wave sort of their
// deliver times (equal times: by searches, an event's rank being its index in its own run plus
// the number of smaller (time, src, seq) keys in each other run); no atomics, deterministic
// (keys are unique: (src, seq) never repeats) -- moves the cursors, and stores the
// batch's remainder as a new run.  A run whose events are all popped is dropped; when
// the run limit is reached (kEqMaxRuns, or the EQ_MAX_RUNS knob), half of them -- those holding
// the fewest pending events -- are first compacted into one (the same merge, every event).
// Traffic per advance ~ the batch (read + its remainder written) + the popped events (read +
// written), instead of every pending event read and written each round.
#include <cstdlib>
#include <algorithm>
#include <cstring>

#include "scan.h"
#include "wave.h"

namespace shd {

constexpr uint32_t kEqSrcMax = kEqMaxRuns + 1;   // the stored runs + the incoming batch

struct EqSrc {   // one source of an advance: a stored run (from its cursor) or the batch
    const uint32_t* off;       // [n_hosts + 1]
    const uint32_t* lo;        // stored run: per-host cursor; batch: nullptr (= off)
    uint32_t* cut;             // per host: first event not popped (eqr_count writes, eqr_merge reads)
    const uint64_t* deliver;
    const uint32_t* src;
    const uint64_t* seq;
    const uint64_t* tag;       // stored run
    const uint32_t* pkt;       // batch: tag = batch << 32 | pkt
    uint64_t batch;
};

struct EqSrcs {
    EqSrc s[kEqSrcMax];
    uint32_t n;
    int32_t b;   // index of the batch source, -1 without one
    // sources whose remainders [cut, end) are merged into the new run together with the batch's
    // (a compaction folded into the advance: those runs are dropped after it)
    uint32_t fold = 0;
};

__device__ __forceinline__ bool eq_less(uint64_t ta, uint32_t sa, uint64_t qa, uint64_t tb, uint32_t sb,
                                        uint64_t qb) {
    if (ta != tb) return ta < tb;
    if (sa != sb) return sa < sb;
    return qa < qb;
}

__device__ __forceinline__ uint32_t lower_bound_time(const uint64_t* t, uint32_t b, uint32_t e, uint64_t x) {
    while (b < e) {
        const uint32_t m = (b + e) >> 1;
        if (t[m] < x) b = m + 1; else e = m;
    }
    return b;
}

// lower_bound from the front: a run's popped prefix is short (C5: ~10 events per host and run),
// so probing b, b+1, b+3, b+7, ... finds the cut within a line or two of the cursor, where a
// plain bisection of the whole run touches a line per step
__device__ __forceinline__ uint32_t lower_bound_gallop(const uint64_t* t, uint32_t b, uint32_t e, uint64_t x) {
    if (b >= e || !(t[b] < x)) return b;
    uint32_t prev = b, step = 1;   // t[prev] < x
    while (step < e - prev && t[prev + step] < x) {
        prev += step;
        step <<= 1;
    }
    return lower_bound_time(t, prev + 1, min(e, prev + step), x);
}

// Q.next layout (one read-back per call): [0] unused, [1] popped, [2] kept batch events, [3] head
// time, [4 + k] events of source k left after the pop; then eqr_count's per-block partials
constexpr uint32_t kEqWords = 4 + kEqSrcMax;

// per host and source: the cut (first event at or past window_end); popped count per host, the
// batch's kept count per host, events left per source and the earliest kept deliver time.
// kEqLanes lanes per host, lane k on source k: the sources' binary searches run side by side.
constexpr uint32_t kEqLanes = 16;
static_assert(kEqSrcMax <= kEqLanes, "a lane per source");

constexpr uint32_t kEqCountBlocks = 2048;   // eqr_count's grid: per-block partials, no hot atomics
                                            // (full occupancy for its latency-bound searches: 1024 blocks 64 us, 2048 55)
constexpr uint32_t kEqCountBlocksMax = 4096;   // partials room (SHD_EQ_COUNT_BLOCKS: tuning)
constexpr uint32_t kEqPart = 1 + kEqSrcMax;  // partial words per block: head time, left per source

__global__ __launch_bounds__(256) void eqr_count(uint32_t n_hosts, EqSrcs S, uint64_t window_end,
                                                 uint32_t* __restrict__ pop, uint32_t* __restrict__ keep,
                                                 unsigned long long* __restrict__ part, uint2* __restrict__ ranges) {
    __shared__ unsigned long long s_w[4][kEqPart];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t total = ((uint64_t)n_hosts + 1) * kEqLanes;
    uint64_t head = ~0ull, rem_acc = 0;
    for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t - threadIdx.x < total;
         t += (uint64_t)gridDim.x * 256) {   // wave-uniform trip count (total is a multiple of 16)
        const uint32_t h = (uint32_t)(t / kEqLanes), k = (uint32_t)(t % kEqLanes);
        uint32_t np = 0;
        uint64_t rem = 0;
        if (h < n_hosts && k < S.n) {
            const EqSrc& q = S.s[k];
            const uint32_t lo = q.lo ? q.lo[h] : q.off[h], hi = q.off[h + 1];
            // a compaction (window_end = ~0) takes every event: one load confirms the run's last
            // event is below it, instead of a gallop across the whole run
            // (loading the first 8 or 16 times of the run at once and counting, instead of the
            // gallop's dependent loads, measured slower: C5 advance 0.37 / 0.45 ms against 0.35)
            const uint32_t m = window_end == ~0ull && lo < hi && q.deliver[hi - 1] < window_end
                                   ? hi
                                   : lower_bound_gallop(q.deliver, lo, hi, window_end);
            q.cut[h] = m;
            ranges[(size_t)h * kEqSrcMax + k] = make_uint2(lo, m);   // eqr_merge: one line per host
            np = m - lo;
            rem = hi - m;
            if (m < hi) head = q.deliver[m] < head ? q.deliver[m] : head;
        }
        // the new run's events of this host: the batch's remainder and the folded runs'
        uint32_t kp = h < n_hosts && k < S.n && ((int32_t)k == S.b || ((S.fold >> k) & 1u)) ? (uint32_t)rem : 0u;
        for (uint32_t o = kEqLanes / 2; o > 0; o >>= 1) {
            np += __shfl_xor(np, o);
            kp += __shfl_xor(kp, o);
        }
        if (h < n_hosts && k == 0) {
            pop[h] = np;
            keep[h] = kp;
        }
        if (h == n_hosts && k == 0) {
            pop[n_hosts] = 0;
            keep[n_hosts] = 0;
        }
        rem_acc += rem;   // lane k mod kEqLanes keeps source k's sum
    }
    for (uint32_t o = kEqLanes; o < 64; o <<= 1) rem_acc += __shfl_xor(rem_acc, o);
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t x = __shfl_xor(head, o);
        head = x < head ? x : head;
    }
    if (lane < kEqSrcMax) s_w[w][1 + lane] = rem_acc;
    if (lane == 0) s_w[w][0] = head;
    __syncthreads();
    if (threadIdx.x < kEqPart) {
        unsigned long long v = s_w[0][threadIdx.x];
        for (int ww = 1; ww < 4; ++ww) {
            const unsigned long long x = s_w[ww][threadIdx.x];
            v = threadIdx.x == 0 ? (x < v ? x : v) : v + x;
        }
        part[(size_t)blockIdx.x * kEqPart + threadIdx.x] = v;
    }
}

struct EqOut {
    uint64_t* deliver;
    uint32_t* src;
    uint64_t* seq;
    uint64_t* tag;
};

// One wave per host: every source's popped prefix [lo, cut) goes to its merged rank in the
// popped output: its index in its own prefix + the number of smaller events in each other
// prefix.  When the host's popped events fit kEqStage, the prefixes are staged in LDS (whole
// events, source after source, coalesced loads), every lane then takes one staged event and
// binary-searches the other prefixes in LDS; larger hosts search global memory source by
// source.  Then the batch's remainder [cut, end) is copied to the new run (in the same wave: a
// separate streaming kernel, alone or beside the merge on the side stream, measured slower).
#ifndef SHD_EQ_SEL
#define SHD_EQ_SEL 1   // staging: lane per staged event (0: source after source, for A/B)
#endif
// (an LDS table of the sources' arrays read by a per-lane source index, instead of the selects
// over every source's pointers, measured slower: C5 advance 0.395 against 0.377 ms)
constexpr uint32_t kEqStage = 160;   // 17.5 KB per 4-wave workgroup: 8 workgroups (32 waves) per CU

// u64 minimum / maximum over the wave
__device__ __forceinline__ uint64_t eq_wave_min64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t x = __shfl_xor(v, o);
        v = x < v ? x : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t eq_wave_max64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t x = __shfl_xor(v, o);
        v = x > v ? x : v;
    }
    return v;
}

// Rank a host's staged popped events by a wave sort instead of searches: (t - tmin) << 8 | staged
// index is a unique key, 32 bits when the deliver times span less than 2^24 ns (a window of up
// to ~16 ms: every normal pass), 64 bits otherwise (a compaction's whole runs), and a bitonic
// network over the wave (wave.h: one DPP / swizzle / permlane exchange per stage, 28 stages for
// 128 events) orders them -- a bisection per other source per event costs several times the
// VALU issue, which is what bounds the merge (~100 events per host on C5) -- and the events
// leave in rank order (coalesced stores).  Equal times, whose order needs (src, seq), return
// false: the caller's searches take the host.
template <int NPL>
__device__ __forceinline__ bool eq_sort_emit(uint32_t npop, uint32_t lane, const uint64_t* st, const uint32_t* ss,
                                             const uint64_t* sq, const uint64_t* sg, uint32_t po, EqOut popped) {
    static_assert(64 * NPL <= 256, "staged index in 8 key bits");
    uint64_t t[NPL], tmn = ~0ull, tmx = 0;
#pragma unroll
    for (int c = 0; c < NPL; ++c) {
        const uint32_t i = lane + 64u * c;
        t[c] = i < npop ? st[i] : 0ull;
        if (i < npop) {
            tmn = t[c] < tmn ? t[c] : tmn;
            tmx = t[c] > tmx ? t[c] : tmx;
        }
    }
    tmn = eq_wave_min64(tmn);
    tmx = eq_wave_max64(tmx);
    uint32_t idx[NPL];
    bool tie = false;   // equal times in sorted neighbours r, r + 1
    if (tmx - tmn < (1ull << 24)) {   // wave-uniform
        uint32_t k[NPL];
#pragma unroll
        for (int c = 0; c < NPL; ++c) {
            const uint32_t i = lane + 64u * c;   // npop < 256 here: no valid key reaches ~0u
            k[c] = i < npop ? ((uint32_t)(t[c] - tmn) << 8) | i : ~0u;
        }
        wave_bitonic32<NPL>(k, lane);
#pragma unroll
        for (int c = 0; c < NPL; ++c) {
            // (both shuffles with every lane active: a read of an inactive lane returns 0)
            const uint32_t down = (uint32_t)__shfl_down((int)k[c], 1);
            const uint32_t first = c + 1 < NPL ? (uint32_t)__shfl((int)k[c + 1 < NPL ? c + 1 : c], 0) : ~0u;
            const uint32_t nx = lane == 63 ? first : down;
            if (lane + 64u * c + 1 < npop && (nx >> 8) == (k[c] >> 8)) tie = true;
            idx[c] = k[c] & 0xFFu;
        }
    } else if (tmx - tmn < (1ull << 56)) {
        uint64_t k[NPL];
#pragma unroll
        for (int c = 0; c < NPL; ++c) {
            const uint32_t i = lane + 64u * c;
            k[c] = i < npop ? ((t[c] - tmn) << 8) | i : ~0ull;
        }
        wave_bitonic<NPL>(k, lane);
#pragma unroll
        for (int c = 0; c < NPL; ++c) {
            const uint64_t down = __shfl_down(k[c], 1);
            const uint64_t first = c + 1 < NPL ? __shfl(k[c + 1 < NPL ? c + 1 : c], 0) : ~0ull;
            const uint64_t nx = lane == 63 ? first : down;
            if (lane + 64u * c + 1 < npop && (nx >> 8) == (k[c] >> 8)) tie = true;
            idx[c] = (uint32_t)k[c] & 0xFFu;
        }
    } else {
        return false;
    }
    if (__ballot(tie) != 0) return false;
#pragma unroll
    for (int c = 0; c < NPL; ++c) {
        const uint32_t r = lane + 64u * c;
        if (r < npop) {
            const uint32_t i = idx[c];
            popped.deliver[po + r] = st[i];
            popped.src[po + r] = ss[i];
            popped.seq[po + r] = sq[i];
            popped.tag[po + r] = sg[i];
        }
    }
    return true;
}

// One host's merge (a wave): lane k < S.n holds source k's popped range [my_lo, my_m); po is the
// host's first popped slot, rb_no its first slot in the new run (a batch source only); sort_rank:
// rank staged hosts by eq_sort_emit first (SHD_EQ_SEARCH_ONLY=1: the searches alone).
template <uint32_t STAGE>
__device__ __forceinline__ void eq_merge_host(uint32_t h, uint32_t w, uint32_t lane, const EqSrcs& S, uint32_t my_lo,
                                              uint32_t my_m, uint32_t po, EqOut popped, EqOut nrun, uint32_t rb_no,
                                              uint32_t* __restrict__ nrun_cur, uint64_t (*s_t)[STAGE],
                                              uint64_t (*s_q)[STAGE], uint64_t (*s_g)[STAGE],
                                              uint32_t (*s_s)[STAGE], bool sort_rank) {
    const uint32_t cnt = my_m - my_lo;
    uint32_t incl = cnt;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    const uint32_t my_sb = incl - cnt, npop = __shfl(incl, 63);
    // every source's range as wave-uniform values (read while all lanes are active: a lane read
    // from inside the divergent loops below would see inactive lanes as 0)
    uint32_t u_lo[kEqSrcMax], u_c[kEqSrcMax], u_sb[kEqSrcMax];
#pragma unroll
    for (uint32_t k = 0; k < kEqSrcMax; ++k) {
        u_lo[k] = __builtin_amdgcn_readlane(my_lo, k);
        u_c[k] = __builtin_amdgcn_readlane(cnt, k);
        u_sb[k] = __builtin_amdgcn_readlane(my_sb, k);
    }
    // the batch remainder's first 128 events are loaded up front: their latency overlaps the
    // merge instead of following it (its cut is the batch range's end from eqr_count)
    uint32_t rb_m = 0, rb_e = 0;
    uint64_t pf_t[2] = {0, 0}, pf_q[2] = {0, 0};
    uint32_t pf_s[2] = {0, 0}, pf_p[2] = {0, 0};
    if (S.b >= 0) {
        const EqSrc& q = S.s[S.b];
#pragma unroll
        for (uint32_t k = 0; k < kEqSrcMax; ++k)
            if ((int32_t)k == S.b) rb_m = u_lo[k] + u_c[k];
        rb_e = q.off[h + 1];
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u) {
            const uint32_t j = rb_m + lane + 64 * u;
            if (j < rb_e) {
                pf_t[u] = q.deliver[j];
                pf_s[u] = q.src[j];
                pf_q[u] = q.seq[j];
                pf_p[u] = q.pkt[j];
            }
        }
    }
    if (npop <= STAGE) {
        uint64_t* st = s_t[w];
        uint64_t* sq = s_q[w];
        uint64_t* sg = s_g[w];
        uint32_t* ss = s_s[w];
#if SHD_EQ_SEL
        // lane i0 loads staged event i0 straight from its source (the source's arrays picked by
        // selects on wave-uniform values): every source's loads are in flight at once, instead
        // of one source's round trip after another
        for (uint32_t i0 = lane; i0 < npop; i0 += 64) {
            uint32_t at = u_lo[0] + i0;
            const uint64_t* dl = S.s[0].deliver;
            const uint64_t* qp = S.s[0].seq;
            const uint32_t* sp = S.s[0].src;
            const uint64_t* tp = S.s[0].tag;
            const uint32_t* pp = S.s[0].pkt;
            uint64_t bt = S.s[0].batch;
#pragma unroll
            for (uint32_t j = 1; j < kEqSrcMax; ++j) {
                if (j < S.n && u_sb[j] <= i0) {
                    at = u_lo[j] + (i0 - u_sb[j]);
                    dl = S.s[j].deliver;
                    qp = S.s[j].seq;
                    sp = S.s[j].src;
                    tp = S.s[j].tag;
                    pp = S.s[j].pkt;
                    bt = S.s[j].batch;
                }
            }
            st[i0] = dl[at];
            sq[i0] = qp[at];
            ss[i0] = sp[at];
            sg[i0] = tp ? tp[at] : ((bt << 32) | pp[at]);
        }
#else
        for (uint32_t k = 0; k < S.n; ++k) {
            const EqSrc& q = S.s[k];
            const uint32_t lo = u_lo[k], c = u_c[k], sb = u_sb[k];
            for (uint32_t i = lane; i < c; i += 64) {
                st[sb + i] = q.deliver[lo + i];
                sq[sb + i] = q.seq[lo + i];
                ss[sb + i] = q.src[lo + i];
                sg[sb + i] = q.tag ? q.tag[lo + i] : ((q.batch << 32) | q.pkt[lo + i]);
            }
        }
#endif
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        static_assert(STAGE <= 256, "staged index in 8 key bits");
        const bool sorted = sort_rank && npop > 1 &&
                            (npop <= 64    ? eq_sort_emit<1>(npop, lane, st, ss, sq, sg, po, popped)
                             : npop <= 128 ? eq_sort_emit<2>(npop, lane, st, ss, sq, sg, po, popped)
                                           : eq_sort_emit<4>(npop, lane, st, ss, sq, sg, po, popped));
        for (uint32_t i0 = sorted ? npop : lane; i0 < npop; i0 += 64) {
            uint32_t k = 0;   // staged event i0 belongs to source k: u_sb[k] <= i0 < u_sb[k + 1]
            for (uint32_t j = 1; j < S.n; ++j) k = u_sb[j] <= i0 ? j : k;
            const uint64_t t = st[i0], qq = sq[i0];
            const uint32_t sv = ss[i0];
            uint32_t rank = i0 - u_sb[k];
            for (uint32_t k2 = 0; k2 < S.n; ++k2) {
                if (k2 == k) continue;
                const uint32_t sb2 = u_sb[k2];
                uint32_t a = 0, b = u_c[k2];
                while (a < b) {
                    const uint32_t m = (a + b) >> 1, x = sb2 + m;
                    const uint64_t tm = st[x];
                    const bool less = tm != t ? tm < t : eq_less(tm, ss[x], sq[x], t, sv, qq);
                    if (less) a = m + 1; else b = m;
                }
                rank += a;
            }
            popped.deliver[po + rank] = t;
            popped.src[po + rank] = sv;
            popped.seq[po + rank] = qq;
            popped.tag[po + rank] = sg[i0];
        }
    } else {
        for (uint32_t k = 0; k < S.n; ++k) {
            const EqSrc& q = S.s[k];
            const uint32_t lo = u_lo[k], c = u_c[k];
            for (uint32_t i = lane; i < c; i += 64) {
                const uint64_t t = q.deliver[lo + i], qq = q.seq[lo + i];
                const uint32_t sv = q.src[lo + i];
                const uint64_t tg = q.tag ? q.tag[lo + i] : ((q.batch << 32) | q.pkt[lo + i]);
                uint32_t rank = i;
                for (uint32_t k2 = 0; k2 < S.n; ++k2) {
                    if (k2 == k) continue;
                    const EqSrc& r = S.s[k2];
                    const uint32_t lo2 = u_lo[k2];
                    uint32_t a = 0, b = u_c[k2];
                    while (a < b) {
                        const uint32_t m = (a + b) >> 1;
                        const uint64_t tm = r.deliver[lo2 + m];
                        const bool less = tm != t ? tm < t : eq_less(tm, r.src[lo2 + m], r.seq[lo2 + m], t, sv, qq);
                        if (less) a = m + 1; else b = m;
                    }
                    rank += a;
                }
                popped.deliver[po + rank] = t;
                popped.src[po + rank] = sv;
                popped.seq[po + rank] = qq;
                popped.tag[po + rank] = tg;
            }
        }
    }
    if (S.b >= 0) {   // the batch's remainder becomes the new run, whose cursor starts at its offset
        const EqSrc& q = S.s[S.b];
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u) {
            const uint32_t j = rb_m + lane + 64 * u;
            if (j < rb_e) {
                const uint32_t at = rb_no + (j - rb_m);
                nrun.deliver[at] = pf_t[u];
                nrun.src[at] = pf_s[u];
                nrun.seq[at] = pf_q[u];
                nrun.tag[at] = (q.batch << 32) | pf_p[u];
            }
        }
        for (uint32_t j = rb_m + 128 + lane; j < rb_e; j += 64) {
            const uint32_t at = rb_no + (j - rb_m);
            nrun.deliver[at] = q.deliver[j];
            nrun.src[at] = q.src[j];
            nrun.seq[at] = q.seq[j];
            nrun.tag[at] = (q.batch << 32) | q.pkt[j];
        }
        if (lane == 0) nrun_cur[h] = rb_no;
    }
}


// STAGE: staged events per host -- kEqStage on the normal passes (8 workgroups per CU), 256 on a
// compaction's (whole runs: ~100-250 pending per host on C5, sorted rather than searched in
// global memory)
// keep (a folded compaction's second launch): the sources in S.fold merge their remainders
// [cut, end) into `popped` = the new run at pop_off = its offsets, whose cursor starts there.
template <uint32_t STAGE>
__global__ __launch_bounds__(256) void eqr_merge(uint32_t n_hosts, EqSrcs S, const uint32_t* __restrict__ pop_off,
                                                 EqOut popped, EqOut nrun, const uint32_t* __restrict__ nrun_off,
                                                 uint32_t* __restrict__ nrun_cur, const uint2* __restrict__ ranges,
                                                 uint32_t sort_rank, uint32_t keep = 0) {
    __shared__ uint64_t s_t[4][STAGE], s_q[4][STAGE], s_g[4][STAGE];
    __shared__ uint32_t s_s[4][STAGE];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t h = blockIdx.x * 4 + w;
    if (h >= n_hosts) return;   // wave-uniform; the kernel has no workgroup barrier
    // lane k < S.n holds source k's popped range and its place in the LDS stage
    uint32_t my_lo = 0, my_m = 0;
    if (keep) {
        if (lane < S.n && ((S.fold >> lane) & 1u)) {
            my_lo = S.s[lane].cut[h];
            my_m = S.s[lane].off[h + 1];
        }
        eq_merge_host<STAGE>(h, w, lane, S, my_lo, my_m, pop_off[h], popped, EqOut{}, 0u, nullptr, s_t, s_q, s_g,
                             s_s, sort_rank != 0);
        if (lane == 0) nrun_cur[h] = pop_off[h];
        return;
    }
    if (lane < S.n) {   // eqr_count's (cursor, cut) pairs of this host: one line
        const uint2 r = ranges[(size_t)h * kEqSrcMax + lane];
        my_lo = r.x;
        my_m = r.y;
    }
    eq_merge_host<STAGE>(h, w, lane, S, my_lo, my_m, pop_off[h], popped, nrun, S.b >= 0 ? nrun_off[h] : 0u,
                         nrun_cur, s_t, s_q, s_g, s_s, sort_rank != 0);
}

// Sixteen lanes per host (EQ_WAVE_MERGE=0; tuning variant, NOT the default): for queues popping
// a few events per host and round, four hosts a wave put four hosts' load chains in flight in the
// slot a wave-per-host merge leaves mostly idle.  C5 pops ~100 per host (100k hosts, 9.9M events),
// past this kernel's 64-event stage, so most hosts take its global-search path: 525 us a launch
// against eqr_merge's 182.5 (rocprofv3 kernel trace, tools/equeue_only.py, round 4).  The same merge: lane l < S.n holds source l's range, popped events are staged in LDS
// (kEqStage16 a host; times, sources, sequence numbers -- the tags stay in the lanes' registers),
// each staged event's rank = its index in its source + a bisection per other source; a host
// popping more searches global memory; then the batch remainder goes to the new run.  The four
// groups of a wave share nothing in LDS but their own rows, so a wave barrier is the only sync.
constexpr uint32_t kEqG = 16;          // lanes per host
constexpr uint32_t kEqStage16 = 64;    // staged popped events per host (4 per lane)
constexpr uint32_t kEqPre16 = 4;       // batch remainder events per lane loaded up front
static_assert(kEqSrcMax <= kEqG, "a lane per source");

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(256) void eqr_merge16(uint32_t n_hosts, EqSrcs S, const uint32_t* __restrict__ pop_off,
                                                   EqOut popped, EqOut nrun, const uint32_t* __restrict__ nrun_off,
                                                   uint32_t* __restrict__ nrun_cur, const uint2* __restrict__ ranges) {
    __shared__ uint64_t s_t[16][kEqStage16], s_q[16][kEqStage16];
    __shared__ uint32_t s_s[16][kEqStage16];
    __shared__ uint32_t s_lo[16][kEqSrcMax], s_c[16][kEqSrcMax], s_sb[16][kEqSrcMax];
    const uint32_t g = threadIdx.x / kEqG, l = threadIdx.x % kEqG;
    const uint32_t h = blockIdx.x * 16 + g;
    const bool live = h < n_hosts;   // not wave-uniform: a dead group runs every loop zero times
    uint32_t lo = 0, m = 0, po = 0, rb_no = 0, rb_e = 0;
    if (live) {
        if (l < S.n) {
            const uint2 r = ranges[(size_t)h * kEqSrcMax + l];
            lo = r.x;
            m = r.y;
        }
        po = pop_off[h];
        if (S.b >= 0) {
            rb_no = nrun_off[h];
            rb_e = S.s[S.b].off[h + 1];
        }
    }
    const uint32_t cnt = m - lo;
    uint32_t incl = cnt;
    for (uint32_t o = 1; o < kEqG; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, kEqG);
        if (l >= o) incl += y;
    }
    const uint32_t npop = __shfl(incl, kEqG - 1, kEqG);
    if (l < kEqSrcMax) {
        s_lo[g][l] = lo;
        s_c[g][l] = cnt;
        s_sb[g][l] = incl - cnt;
    }
    wave_sync_lds();
    uint32_t u_lo[kEqSrcMax], u_c[kEqSrcMax], u_sb[kEqSrcMax];
#pragma unroll
    for (uint32_t k = 0; k < kEqSrcMax; ++k) {
        u_lo[k] = s_lo[g][k];
        u_c[k] = s_c[g][k];
        u_sb[k] = s_sb[g][k];
    }
    // the batch remainder [rb_m, rb_e): its first kEqPre16 x 16 events loaded before the merge
    uint32_t rb_m = rb_e;
    uint64_t pf_t[kEqPre16], pf_q[kEqPre16];
    uint32_t pf_s[kEqPre16], pf_p[kEqPre16];
    if (S.b >= 0) {
        const EqSrc& q = S.s[S.b];
        if (live) {
#pragma unroll
            for (uint32_t k = 0; k < kEqSrcMax; ++k)
                if ((int32_t)k == S.b) rb_m = u_lo[k] + u_c[k];
        }
#pragma unroll
        for (uint32_t u = 0; u < kEqPre16; ++u) {
            const uint32_t j = rb_m + l + kEqG * u;
            if (j < rb_e) {
                pf_t[u] = q.deliver[j];
                pf_s[u] = q.src[j];
                pf_q[u] = q.seq[j];
                pf_p[u] = q.pkt[j];
            }
        }
    }
    if (npop <= kEqStage16) {
        // staged event i = l + 16 u, straight from its source (pointer selects on group-uniform
        // values, every source's loads in flight at once); its tag stays in this lane
        uint64_t tg[kEqStage16 / kEqG];
        uint32_t ks[kEqStage16 / kEqG];
#pragma unroll
        for (uint32_t u = 0; u < kEqStage16 / kEqG; ++u) {
            const uint32_t i = l + kEqG * u;
            ks[u] = 0;
            if (i < npop) {
                uint32_t at = u_lo[0] + i, k = 0;
#pragma unroll
                for (uint32_t j = 1; j < kEqSrcMax; ++j)
                    if (j < S.n && u_sb[j] <= i) {
                        at = u_lo[j] + (i - u_sb[j]);
                        k = j;
                    }
                const uint64_t* dl = S.s[0].deliver;
                const uint64_t* qp = S.s[0].seq;
                const uint32_t* sp = S.s[0].src;
                const uint64_t* tp = S.s[0].tag;
                const uint32_t* pp = S.s[0].pkt;
                uint64_t bt = S.s[0].batch;
#pragma unroll
                for (uint32_t j = 1; j < kEqSrcMax; ++j)
                    if (j == k) {
                        dl = S.s[j].deliver;
                        qp = S.s[j].seq;
                        sp = S.s[j].src;
                        tp = S.s[j].tag;
                        pp = S.s[j].pkt;
                        bt = S.s[j].batch;
                    }
                ks[u] = k;
                s_t[g][i] = dl[at];
                s_q[g][i] = qp[at];
                s_s[g][i] = sp[at];
                tg[u] = tp ? tp[at] : ((bt << 32) | pp[at]);
            }
        }
        wave_sync_lds();
#pragma unroll
        for (uint32_t u = 0; u < kEqStage16 / kEqG; ++u) {
            const uint32_t i = l + kEqG * u;
            if (i >= npop) continue;
            const uint32_t k = ks[u];
            const uint64_t t = s_t[g][i], qq = s_q[g][i];
            const uint32_t sv = s_s[g][i];
            uint32_t rank = i - u_sb[k];
            for (uint32_t k2 = 0; k2 < S.n; ++k2) {
                if (k2 == k) continue;
                const uint32_t sb2 = u_sb[k2];
                uint32_t a = 0, b = u_c[k2];
                while (a < b) {
                    const uint32_t mid = (a + b) >> 1, x = sb2 + mid;
                    const uint64_t tm = s_t[g][x];
                    const bool less = tm != t ? tm < t : eq_less(tm, s_s[g][x], s_q[g][x], t, sv, qq);
                    if (less) a = mid + 1; else b = mid;
                }
                rank += a;
            }
            popped.deliver[po + rank] = t;
            popped.src[po + rank] = sv;
            popped.seq[po + rank] = qq;
            popped.tag[po + rank] = tg[u];
        }
    } else {
        for (uint32_t k = 0; k < S.n; ++k) {
            const EqSrc& q = S.s[k];
            const uint32_t lo1 = u_lo[k], c = u_c[k];
            for (uint32_t i = l; i < c; i += kEqG) {
                const uint64_t t = q.deliver[lo1 + i], qq = q.seq[lo1 + i];
                const uint32_t sv = q.src[lo1 + i];
                const uint64_t tg = q.tag ? q.tag[lo1 + i] : ((q.batch << 32) | q.pkt[lo1 + i]);
                uint32_t rank = i;
                for (uint32_t k2 = 0; k2 < S.n; ++k2) {
                    if (k2 == k) continue;
                    const EqSrc& r = S.s[k2];
                    const uint32_t lo2 = u_lo[k2];
                    uint32_t a = 0, b = u_c[k2];
                    while (a < b) {
                        const uint32_t mid = (a + b) >> 1;
                        const uint64_t tm = r.deliver[lo2 + mid];
                        const bool less =
                            tm != t ? tm < t : eq_less(tm, r.src[lo2 + mid], r.seq[lo2 + mid], t, sv, qq);
                        if (less) a = mid + 1; else b = mid;
                    }
                    rank += a;
                }
                popped.deliver[po + rank] = t;
                popped.src[po + rank] = sv;
                popped.seq[po + rank] = qq;
                popped.tag[po + rank] = tg;
            }
        }
    }
    if (S.b >= 0) {   // the batch's remainder becomes the new run, whose cursor starts at its offset
        const EqSrc& q = S.s[S.b];
#pragma unroll
        for (uint32_t u = 0; u < kEqPre16; ++u) {
            const uint32_t j = rb_m + l + kEqG * u;
            if (j < rb_e) {
                const uint32_t at = rb_no + (j - rb_m);
                nrun.deliver[at] = pf_t[u];
                nrun.src[at] = pf_s[u];
                nrun.seq[at] = pf_q[u];
                nrun.tag[at] = (q.batch << 32) | pf_p[u];
            }
        }
        for (uint32_t j = rb_m + kEqPre16 * kEqG + l; j < rb_e; j += kEqG) {
            const uint32_t at = rb_no + (j - rb_m);
            nrun.deliver[at] = q.deliver[j];
            nrun.src[at] = q.src[j];
            nrun.seq[at] = q.seq[j];
            nrun.tag[at] = (q.batch << 32) | q.pkt[j];
        }
        if (live && l == 0) nrun_cur[h] = rb_no;
    }
}

// the call's totals (popped, kept batch events, head time, left per source) from eqr_count's
// per-block partials, into one word array the host reads with one copy
__global__ __launch_bounds__(1024) void eq_totals(uint32_t n_hosts, uint32_t n_part, const uint32_t* __restrict__ pop_off,
                                                  const uint32_t* __restrict__ keep_off,
                                                  const unsigned long long* __restrict__ part,
                                                  unsigned long long* __restrict__ words,
                                                  unsigned long long* host_words, unsigned long long* marker) {
    __shared__ unsigned long long s_v[16][kEqPart];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // a thread takes whole partial records (independent loads), then one reduction per word
    unsigned long long v[kEqPart];
#pragma unroll
    for (uint32_t j = 0; j < kEqPart; ++j) v[j] = j == 0 ? ~0ull : 0ull;
    for (uint32_t b = threadIdx.x; b < n_part; b += 1024) {
#pragma unroll
        for (uint32_t j = 0; j < kEqPart; ++j) {
            const unsigned long long x = part[(size_t)b * kEqPart + j];
            v[j] = j == 0 ? (x < v[j] ? x : v[j]) : v[j] + x;
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < kEqPart; ++j) {
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long x = __shfl_xor(v[j], o);
            v[j] = j == 0 ? (x < v[j] ? x : v[j]) : v[j] + x;
        }
        if (lane == 0) s_v[w][j] = v[j];
    }
    __syncthreads();
    // host_words (the read-back in the same launch): the words go straight to the pinned host
    // words and the marker the host polls follows them (as rounds.hip readback_mark)
    unsigned long long* out = host_words ? host_words : words;
    if (threadIdx.x < kEqPart) {
        const uint32_t j = threadIdx.x;
        unsigned long long t = s_v[0][j];
        for (int ww = 1; ww < 16; ++ww) t = j == 0 ? (s_v[ww][j] < t ? s_v[ww][j] : t) : t + s_v[ww][j];
        if (j == 0) out[3] = t;
        else out[3 + j] = t;   // words[4 + k] = left of source k
    }
    if (threadIdx.x == 0) {
        out[1] = pop_off[n_hosts];
        out[2] = keep_off ? keep_off[n_hosts] : 0u;
    }
    if (host_words) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // every thread's words reach the host first
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(marker, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// a stored run's event arrays for n events (the ensure keeps growth headroom: slots are reused
// round after round)
// hint = false (shd_equeue_pending's full compaction, the whole pending set in one run): the
// growth neither takes nor raises the slots' shared capacity -- a hint raised to 1.5x every pending
// event would make every later slot growth that large (advisor, round 5: ~14x the largest run)
static shd_status eq_run_alloc(EqState& Q, EqRunBuf& r, uint32_t n_hosts, uint64_t n, bool hint = true) {
    // room for half as many again: the runs' sizes wander from round to round, and a regrowth
    // (hipFree + hipMalloc of ~0.5 GB of arrays) inside an advance cost ~0.3 ms (C5: 0.78 ms rounds);
    // and at least the largest capacity any slot has grown to, so the slots reach their steady
    // size in one growth each instead of several (the slots take turns as batch, remainder and
    // compaction runs of different sizes)
    const size_t m = std::max<uint64_t>(n, 1);
    if (r.deliver.bytes < m * 8 || r.src.bytes < m * 4 || r.seq.bytes < m * 8 || r.tag.bytes < m * 8) {
        const size_t g = hint ? std::max<size_t>(m + m / 2, Q.cap_hint) : m + m / 2;
        if (hint) Q.cap_hint = g;
        SHD_TRY(r.deliver.ensure(g * 8));
        SHD_TRY(r.src.ensure(g * 4));
        SHD_TRY(r.seq.ensure(g * 8));
        SHD_TRY(r.tag.ensure(g * 8));
    }
    SHD_TRY(r.off.ensure((size_t)(n_hosts + 1) * 4));
    SHD_TRY(r.deliver.ensure(m * 8));
    SHD_TRY(r.src.ensure(m * 4));
    SHD_TRY(r.seq.ensure(m * 8));
    SHD_TRY(r.tag.ensure(m * 8));
    r.has_pkt = false;
    r.fresh = false;
    return SHD_OK;
}

static EqOut eq_run_out(EqRunBuf& r) {
    return EqOut{r.deliver.as<uint64_t>(), r.src.as<uint32_t>(), r.seq.as<uint64_t>(), r.tag.as<uint64_t>()};
}

constexpr int kEqPinWord = 48;   // ctx->h_pin words [48, 48 + kEqWords)
static_assert(kEqPinWord + (int)kEqWords <= kPinMarker, "queue counts below the polled marker");

// One pass: per-host cuts at window_end, scans, the merge of every source's popped prefix into
// `out` at offsets out_off, and (nrun) the batch's remainder into a new run whose cursor goes to
// nrun_cur.  Returns with the counts in ctx->h_pin + kEqPinWord.
static shd_status eq_pass(shd_ctx* ctx, const EqSrcs& S, uint64_t window_end, uint32_t* out_off, EqOut out,
                          EqRunBuf* nrun, uint32_t* nrun_cur, uint64_t n_in, bool counts = true) {
    // S.fold: the batch's remainder (when there is one) and the folded runs' are merged into the
    // new run by a second merge launch; the first one then only pops
    EqState& Q = ctx->eq;
    hipStream_t s = ctx->stream;
    const uint32_t H = Q.n_hosts;
    unsigned long long* words = Q.next.as<unsigned long long>();
    unsigned long long* part = words + kEqWords;
    const EqOut nr = nrun ? eq_run_out(*nrun) : EqOut{};
    const uint32_t gx = ctx->knobs.get(K_EQ_COUNT_BLOCKS, 0);
    const uint32_t grid_max = gx >= 1 && gx <= kEqCountBlocksMax ? gx : kEqCountBlocks;
    const uint32_t nb = std::min<uint32_t>(grid_max, div_up(((uint64_t)H + 1) * kEqLanes, 256));
    SHD_TRY(Q.ranges.ensure((size_t)H * kEqSrcMax * 8));
    eqr_count<<<nb, 256, 0, s>>>(H, S, window_end, Q.pop_cnt.as<uint32_t>(), Q.keep_cnt.as<uint32_t>(), part,
                                 Q.ranges.as<uint2>());
    SHD_HIP(hipGetLastError());
    // the popped offsets and the new run's offsets: one hand-written look-back scan launch (scan.h)
    SHD_TRY(scan_excl2(Q.scan, Q.pop_cnt.as<uint32_t>(), out_off, nrun ? Q.keep_cnt.as<uint32_t>() : nullptr,
                       nrun ? nrun->off.as<uint32_t>() : nullptr, H + 1, s));
    if (n_in && S.fold) {
        EqSrcs SP = S, SK = S;
        SP.b = -1;   // no remainder copy: the keep launch merges the batch's with the folded runs'
        SP.fold = 0;
        SK.fold = S.fold | (S.b >= 0 ? 1u << S.b : 0u);
        SK.b = -1;
        const uint32_t srt = ctx->knobs.get(K_EQ_SEARCH_ONLY, 0) == 1 ? 0u : 1u;
        (window_end == ~0ull ? eqr_merge<256> : eqr_merge<kEqStage>)<<<div_up(H, 4), 256, 0, s>>>(
            H, SP, out_off, out, EqOut{}, nullptr, nullptr, Q.ranges.as<uint2>(), srt, 0u);
        eqr_merge<256><<<div_up(H, 4), 256, 0, s>>>(H, SK, nrun->off.as<uint32_t>(), nr, EqOut{}, nullptr, nrun_cur,
                                                     Q.ranges.as<uint2>(), srt, 1u);
    } else if (n_in) {
        if (ctx->knobs.get(K_EQ_WAVE_MERGE, 1) != 0)   // default: a wave a host (faster on C5, see eqr_merge16)
            (window_end == ~0ull ? eqr_merge<256> : eqr_merge<kEqStage>)<<<div_up(H, 4), 256, 0, s>>>(
                H, S, out_off, out, nr, nrun ? nrun->off.as<uint32_t>() : nullptr, nrun_cur, Q.ranges.as<uint2>(),
                ctx->knobs.get(K_EQ_SEARCH_ONLY, 0) == 1 ? 0u : 1u, 0u);
        else
            eqr_merge16<<<div_up(H, 16), 256, 0, s>>>(H, S, out_off, out, nr,
                                                      nrun ? nrun->off.as<uint32_t>() : nullptr, nrun_cur,
                                                      Q.ranges.as<uint2>());
    }
    SHD_HIP(hipGetLastError());
    if (!counts) return SHD_OK;   // (a compaction: what it moves is known on the host, nothing to wait for)
    if (ctx->spin_wait && ctx->knobs.get(K_SYNC_KERNEL, 1) != 0) {   // totals + read-back in one launch
        volatile unsigned long long* mark = ctx->h_pin + kPinMarker;
        *mark = 0;
        eq_totals<<<1, 1024, 0, s>>>(H, nb, out_off, nrun ? nrun->off.as<uint32_t>() : nullptr, part, words,
                                     ctx->h_pin + kEqPinWord, const_cast<unsigned long long*>(mark));
        SHD_HIP(hipGetLastError());
        return wait_marker(ctx, s);
    }
    eq_totals<<<1, 1024, 0, s>>>(H, nb, out_off, nrun ? nrun->off.as<uint32_t>() : nullptr, part, words, nullptr,
                                 nullptr);
    return readback(ctx, s, kEqPinWord, words, kEqWords * 8);
}

static uint32_t* eq_cursor(EqState& Q, int buf, int slot) {
    return Q.curs[buf].as<uint32_t>() + (size_t)slot * Q.n_hosts;
}

// the live runs as sources, from their cursors; cuts into the other cursor buffer.  pick
// (optional) selects a subset of the live slots.
static EqSrcs eq_sources(EqState& Q, int* slots, const bool* pick = nullptr) {
    EqSrcs S{};
    S.b = -1;
    for (int r = 0; r < kEqSlots; ++r) {
        EqRunBuf& R = Q.run[r];
        if (!R.live || (pick && !pick[r])) continue;
        slots[S.n] = r;
        // a run adopted by this call has no cursor yet: it starts at its offsets (lo = null)
        S.s[S.n++] = EqSrc{R.off.as<uint32_t>(), R.fresh ? nullptr : eq_cursor(Q, Q.ccur, r), eq_cursor(Q, 1 - Q.ccur, r),
                           R.deliver.as<uint64_t>(), R.src.as<uint32_t>(), R.seq.as<uint64_t>(),
                           R.has_pkt ? nullptr : R.tag.as<uint64_t>(), R.has_pkt ? R.pkt.as<uint32_t>() : nullptr,
                           R.batch};
    }
    return S;
}

static int eq_free_slot(const EqState& Q) {
    for (int r = 0; r < kEqSlots; ++r)
        if (!Q.run[r].live && r != Q.lend) return r;
    return -1;
}

// Pending events of several runs into one fresh run (cursor at its start); those runs are
// dropped, the others keep their cursors.  all = false: the half of the live runs holding the
// fewest pending events -- the oldest, mostly drained ones -- so a compaction forced by the run
// limit costs what those runs still hold, not every pending event (C5: runs drain over hundreds
// of rounds, the pending set is many rounds' worth).
static shd_status eq_compact(shd_ctx* ctx, bool all) {
    EqState& Q = ctx->eq;
    bool pick[kEqSlots] = {};
    int live[kEqSlots], nl = 0;
    for (int r = 0; r < kEqSlots; ++r)
        if (Q.run[r].live) live[nl++] = r;
    if (nl == 0) return SHD_OK;
    std::sort(live, live + nl, [&](int a, int b) { return Q.run[a].left < Q.run[b].left; });
    const int take = all ? nl : std::max(2, (nl + 1) / 2);
    uint64_t n = 0;
    for (int k = 0; k < take && k < nl; ++k) {
        pick[live[k]] = true;
        n += Q.run[live[k]].left;
    }
    int slots[kEqSrcMax];
    EqSrcs S = eq_sources(Q, slots, pick);
    if (S.n == 0) return SHD_OK;
    const int t = eq_free_slot(Q);
    EqRunBuf& T = Q.run[t];
    SHD_TRY(eq_run_alloc(Q, T, Q.n_hosts, n, !all));
    // every pending event of the picked runs moves (window ~0): n, known here, so inside an advance
    // the pass runs without its totals and read-back (the advance's own pass follows on the
    // stream).  The full compaction of shd_equeue_pending is not hot: it reads the totals back and
    // checks that exactly the n events the runs' counts promise were moved.
    SHD_TRY(eq_pass(ctx, S, ~0ull, T.off.as<uint32_t>(), eq_run_out(T), nullptr, nullptr, n, all));
    if (all && ctx->h_pin[kEqPinWord + 1] != n) return SHD_ERR_STATE;
    // the new run's cursor goes to the CURRENT cursor buffer: the runs left out keep theirs there
    SHD_HIP(hipMemcpyAsync(eq_cursor(Q, Q.ccur, t), T.off.p, (size_t)Q.n_hosts * 4, hipMemcpyDeviceToDevice,
                           ctx->stream));
    for (uint32_t k = 0; k < S.n; ++k) Q.run[slots[k]].live = false;
    T.live = n > 0;
    T.n = T.left = n;
    return SHD_OK;
}

}  // namespace shd

using namespace shd;

extern "C" {

shd_status shd_equeue_setup(shd_ctx* ctx, uint32_t n_total) {
    if (!ctx || n_total == 0) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    EqState& Q = ctx->eq;
    Q.ready = false;
    // under a communicator of > 1 ranks: this rank's destination shard (shd_relay_round_sharded's)
    uint32_t lo = 0, hi = n_total;
    if (ctx->comm && ctx->comm->size > 1) shard_range(n_total, ctx->comm->size, ctx->comm->rank, &lo, &hi);
    const uint32_t n_hosts = hi - lo;
    if (n_hosts == 0) return SHD_ERR_INVALID;
    for (int r = 0; r < kEqSlots; ++r) {
        Q.run[r].live = false;
        Q.run[r].n = Q.run[r].left = 0;
    }
    for (int k = 0; k < 2; ++k) SHD_TRY(Q.curs[k].ensure((size_t)kEqSlots * n_hosts * 4));
    Q.lend = -1;
    SHD_TRY(Q.bcut.ensure((size_t)n_hosts * 4));
    SHD_TRY(Q.pop_cnt.ensure((size_t)(n_hosts + 1) * 4));
    SHD_TRY(Q.keep_cnt.ensure((size_t)(n_hosts + 1) * 4));
    SHD_TRY(Q.pop_off.ensure((size_t)(n_hosts + 1) * 4));
    SHD_TRY(Q.next.ensure((kEqWords + (size_t)kEqCountBlocksMax * kEqPart) * 8));
    SHD_HIP(hipMemsetAsync(Q.pop_off.p, 0, (size_t)(n_hosts + 1) * 4, ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    Q.ccur = 0;
    Q.n_hosts = n_hosts;
    Q.host_lo = lo;
    Q.n_total = n_total;
    Q.head = ~0ull;
    Q.n_pending = 0;
    Q.n_popped = 0;
    Q.batches = 0;
    ctx->rnd.batch_min_deliver = ~0ull;   // new queues: no relay output is pending for them
    Q.ready = true;
    return SHD_OK;
}

shd_status shd_equeue_advance(shd_ctx* ctx, const shd_relay_out* d_batch, uint64_t window_end,
                              shd_equeue_out* out);

// the pending runs alone (an adopted batch is one of them by now)
static shd_status advance_runs(shd_ctx* ctx, uint64_t window_end, shd_equeue_out* out) {
    return shd_equeue_advance(ctx, nullptr, window_end, out);
}

shd_status shd_equeue_batch_buffers(shd_ctx* ctx, uint64_t max_events, shd_relay_out* out) {
    if (!ctx || !out) return SHD_ERR_INVALID;
    EqState& Q = ctx->eq;
    if (!Q.ready) return SHD_ERR_STATE;
    SHD_HIP(hipSetDevice(ctx->device));
    Q.lend = -1;
    const int t = eq_free_slot(Q);
    if (t < 0) return SHD_ERR_STATE;
    EqRunBuf& R = Q.run[t];
    const size_t m = std::max<uint64_t>(max_events, 1);
    SHD_TRY(R.off.ensure((size_t)(Q.n_hosts + 1) * 4));
    if (R.deliver.bytes < m * 8) {   // a growth takes the slots' largest capacity (eq_run_alloc)
        const size_t g = std::max<size_t>(m, Q.cap_hint);
        Q.cap_hint = g;
        SHD_TRY(R.deliver.ensure(g * 8));
        SHD_TRY(R.src.ensure(g * 4));
        SHD_TRY(R.seq.ensure(g * 8));
    }
    SHD_TRY(R.pkt.ensure(std::max<size_t>(m, R.deliver.bytes / 8) * 4));
    Q.lend = t;
    Q.lend_cap = m;   // the relay refuses a round of more events than this into the slot
    out->ev_off = R.off.as<uint32_t>();
    out->ev_deliver = R.deliver.as<uint64_t>();
    out->ev_src = R.src.as<uint32_t>();
    out->ev_seq = R.seq.as<uint64_t>();
    out->ev_pkt = R.pkt.as<uint32_t>();
    out->n_dst = Q.n_hosts;
    out->n_events = 0;
    return SHD_OK;
}

shd_status shd_equeue_advance(shd_ctx* ctx, const shd_relay_out* d_batch, uint64_t window_end,
                              shd_equeue_out* out) {
    if (!ctx || !out) return SHD_ERR_INVALID;
    EqState& Q = ctx->eq;
    if (!Q.ready) return SHD_ERR_STATE;
    const bool has_b = d_batch != nullptr;
    if (has_b && (!d_batch->ev_off || (d_batch->n_events && (!d_batch->ev_deliver || !d_batch->ev_src ||
                                                            !d_batch->ev_seq || !d_batch->ev_pkt))))
        return SHD_ERR_INVALID;
    if (has_b && Q.batches >= 0xFFFFFFFFull) return SHD_ERR_INVALID;   // tag bits exhausted
    // the batch must cover exactly these queues' hosts (ev_off has n_dst + 1 entries): a sharded
    // rank's relay output (n_dst = its shard) into queues set up for another host count would be
    // read past its end on the device
    if (has_b && d_batch->n_dst != Q.n_hosts) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    const uint32_t H = Q.n_hosts;
    const uint64_t n_b = has_b ? d_batch->n_events : 0;   // this context's events (a sharded round: received)
    const uint64_t n_in = Q.n_pending + n_b;
    if (n_in >= 0xFFFFFFFFull) return SHD_ERR_INVALID;   // 32-bit positions
    // adoption: a batch written into the slot shd_equeue_batch_buffers handed out becomes a stored
    // run as it is -- its cursor starts at its offsets, nothing of it is copied
    bool adopt = false;
    if (has_b && Q.lend >= 0) {
        EqRunBuf& L = Q.run[Q.lend];
        adopt = d_batch->ev_off == L.off.p && d_batch->ev_deliver == L.deliver.p && d_batch->ev_src == L.src.p &&
                d_batch->ev_seq == L.seq.p && d_batch->ev_pkt == L.pkt.p;
        if (adopt && (n_b * 8 > L.deliver.bytes || n_b * 4 > L.pkt.bytes)) return SHD_ERR_INVALID;
        if (!adopt) Q.lend = -1;   // the lent slot went unused: free again
    }
    int live = 0;
    for (int r = 0; r < kEqSlots; ++r) live += Q.run[r].live ? 1 : 0;
    const int max_runs = (int)std::min<int64_t>(std::max<int64_t>(ctx->knobs.get(K_EQ_MAX_RUNS, kEqMaxRuns), 2),
                                                kEqMaxRuns);
    if (has_b && n_b && live >= max_runs) {   // room for the batch's run
        // default: the compaction rides this advance's pass (the picked runs' remainders merge into
        // the new run, no pass of its own); SHD_EQ_FOLD=0: a compaction pass first (round 4)
        if (ctx->knobs.get(K_EQ_FOLD, 1) != 0) Q.fold_next = true;
        else SHD_TRY(eq_compact(ctx, false));
    }
    if (adopt) {
        const int t = Q.lend;
        EqRunBuf& R = Q.run[t];
        R.fresh = n_b > 0;   // the pass below reads its cursor from its offsets (no cursor copy)
        R.has_pkt = true;
        R.batch = Q.batches;
        R.n = R.left = n_b;
        R.live = n_b > 0;
        Q.lend = -1;
        ++Q.batches;
        Q.n_pending += n_b;
        ctx->rnd.batch_min_deliver = ~0ull;
        return advance_runs(ctx, window_end, out);
    }
    // the popped events: at most everything (headroom: the pending set creeps up at first)
    if (Q.ps.bytes < std::max<uint64_t>(n_in, 1) * 4) {
        const uint64_t cap = std::max<uint64_t>(n_in, 1) * 3 / 2 + 1;
        SHD_TRY(Q.pd.ensure(cap * 8));
        SHD_TRY(Q.ps.ensure(cap * 4));
        SHD_TRY(Q.pq.ensure(cap * 8));
        SHD_TRY(Q.pt.ensure(cap * 8));
    }
    int slots[kEqSrcMax];
    EqSrcs S = eq_sources(Q, slots);
    const uint32_t n_runs = S.n;
    // a folded compaction: the half of the runs holding the fewest pending events (as eq_compact)
    uint64_t n_fold = 0;
    if (Q.fold_next && n_runs >= 2) {
        int ord[kEqSrcMax];
        for (uint32_t k = 0; k < n_runs; ++k) ord[k] = (int)k;
        std::sort(ord, ord + n_runs, [&](int a, int b) { return Q.run[slots[a]].left < Q.run[slots[b]].left; });
        const uint32_t tk = ctx->knobs.get(K_EQ_FOLD_TAKE, 0);   // (tuning: runs folded; 0 = half)
        const uint32_t take = std::min<uint32_t>(n_runs, std::max<uint32_t>(2, tk ? tk : (n_runs + 1) / 2));
        for (uint32_t i = 0; i < take; ++i) {
            S.fold |= 1u << ord[i];
            n_fold += Q.run[slots[ord[i]]].left;
        }
    }
    Q.fold_next = false;
    EqRunBuf* nrun = nullptr;
    int t = -1;
    if (has_b) {
        S.b = (int32_t)S.n;
        S.s[S.n++] = EqSrc{d_batch->ev_off, nullptr, Q.bcut.as<uint32_t>(), d_batch->ev_deliver, d_batch->ev_src,
                           d_batch->ev_seq, nullptr, d_batch->ev_pkt, Q.batches};
    }
    if (has_b || S.fold) {   // the new run: the batch's remainder and / or the folded runs'
        t = eq_free_slot(Q);
        if (t < 0) return SHD_ERR_STATE;
        nrun = &Q.run[t];
        SHD_TRY(eq_run_alloc(Q, *nrun, H, n_b + n_fold));
    }
    const EqOut popped{Q.pd.as<uint64_t>(), Q.ps.as<uint32_t>(), Q.pq.as<uint64_t>(), Q.pt.as<uint64_t>()};
    SHD_TRY(eq_pass(ctx, S, window_end, Q.pop_off.as<uint32_t>(), popped, nrun,
                    nrun ? eq_cursor(Q, 1 - Q.ccur, t) : nullptr, n_in));
    const unsigned long long* wd = ctx->h_pin + kEqPinWord;
    const uint64_t n_pop = wd[1], n_keep = wd[2];
    uint64_t left = 0, into_new = 0;
    for (uint32_t k = 0; k < S.n; ++k) {
        left += wd[4 + k];
        if ((int32_t)k == S.b || ((S.fold >> k) & 1u)) into_new += wd[4 + k];
    }
    if (n_pop + left != n_in || (nrun && into_new != n_keep)) {   // batch ev_off / n_events disagree
        std::fprintf(stderr, "shd_equeue_advance: counts disagree: popped %llu + left %llu != in %llu "
                     "(pending %llu, batch %llu, runs %u, batch kept %llu vs %llu)\n",
                     (unsigned long long)n_pop, (unsigned long long)left, (unsigned long long)n_in,
                     (unsigned long long)Q.n_pending, (unsigned long long)n_b, n_runs,
                     has_b ? (unsigned long long)wd[4 + S.b] : 0ull, (unsigned long long)n_keep);
        return SHD_ERR_INVALID;
    }
    // commit: cursors moved to the cut buffer; drained runs dropped; the batch's remainder is a run
    for (uint32_t k = 0; k < n_runs; ++k) {
        EqRunBuf& R = Q.run[slots[k]];
        const bool folded = (S.fold >> k) & 1u;   // its remainder moved into the new run
        R.left = folded ? 0 : wd[4 + k];
        R.live = R.left > 0;
        R.fresh = false;   // its cursor is in the cut buffer now
    }
    if (nrun) {
        nrun->n = nrun->left = n_keep;
        nrun->live = n_keep > 0;
    }
    if (has_b) ++Q.batches;
    Q.ccur = 1 - Q.ccur;
    Q.n_pending = left;
    Q.n_popped = n_pop;
    out->off = Q.pop_off.as<uint32_t>();
    out->deliver = Q.pd.as<uint64_t>();
    out->src = Q.ps.as<uint32_t>();
    out->seq = Q.pq.as<uint64_t>();
    out->tag = Q.pt.as<uint64_t>();
    out->n_popped = n_pop;
    out->n_pending = left;
    out->next_time = wd[3];
    Q.head = wd[3];
    if (has_b) ctx->rnd.batch_min_deliver = ~0ull;   // merged: the queue heads carry it from now on
    return SHD_OK;
}

shd_status shd_equeue_copy_popped(shd_ctx* ctx, uint32_t* off, uint64_t* deliver, uint32_t* src,
                                  uint64_t* seq, uint64_t* tag) {
    if (!ctx) return SHD_ERR_INVALID;
    EqState& Q = ctx->eq;
    if (!Q.ready) return SHD_ERR_STATE;
    SHD_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint64_t n = Q.n_popped;
    if (off) SHD_HIP(hipMemcpyAsync(off, Q.pop_off.p, (size_t)(Q.n_hosts + 1) * 4, hipMemcpyDeviceToHost, s));
    if (n) {
        if (deliver) SHD_HIP(hipMemcpyAsync(deliver, Q.pd.p, n * 8, hipMemcpyDeviceToHost, s));
        if (src) SHD_HIP(hipMemcpyAsync(src, Q.ps.p, n * 4, hipMemcpyDeviceToHost, s));
        if (seq) SHD_HIP(hipMemcpyAsync(seq, Q.pq.p, n * 8, hipMemcpyDeviceToHost, s));
        if (tag) SHD_HIP(hipMemcpyAsync(tag, Q.pt.p, n * 8, hipMemcpyDeviceToHost, s));
    }
    SHD_HIP(hipStreamSynchronize(s));
    return SHD_OK;
}

// The pending queues as one CSR: the runs are compacted into one first (the queues' content and
// every later result are unchanged by a compaction).
shd_status shd_equeue_pending(shd_ctx* ctx, uint32_t* off, uint64_t* deliver, uint32_t* src,
                              uint64_t* seq, uint64_t* tag, uint64_t* n_pending) {
    if (!ctx) return SHD_ERR_INVALID;
    EqState& Q = ctx->eq;
    if (!Q.ready) return SHD_ERR_STATE;
    SHD_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint64_t n = Q.n_pending;
    if (n_pending) *n_pending = n;
    if (!off && !(n && (deliver || src || seq || tag))) return SHD_OK;
    SHD_TRY(eq_compact(ctx, true));
    int live = -1;
    for (int r = 0; r < kEqSlots; ++r)
        if (Q.run[r].live) live = r;
    if (off) {
        if (live >= 0) SHD_HIP(hipMemcpyAsync(off, Q.run[live].off.p, (size_t)(Q.n_hosts + 1) * 4, hipMemcpyDeviceToHost, s));
        else std::memset(off, 0, (size_t)(Q.n_hosts + 1) * 4);
    }
    if (n && live >= 0) {
        const EqRunBuf& R = Q.run[live];
        if (deliver) SHD_HIP(hipMemcpyAsync(deliver, R.deliver.p, n * 8, hipMemcpyDeviceToHost, s));
        if (src) SHD_HIP(hipMemcpyAsync(src, R.src.p, n * 4, hipMemcpyDeviceToHost, s));
        if (seq) SHD_HIP(hipMemcpyAsync(seq, R.seq.p, n * 8, hipMemcpyDeviceToHost, s));
        if (tag) SHD_HIP(hipMemcpyAsync(tag, R.tag.p, n * 8, hipMemcpyDeviceToHost, s));
    }
    SHD_HIP(hipStreamSynchronize(s));
    return SHD_OK;
}

}  // extern "C"
