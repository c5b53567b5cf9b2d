// Per-round inter-host packet relay on gfx950.
//
// Reference semantics, per staged send (FlyearthR/shadow src/main/core/worker.rs:328-413):
//   now >= sim_end -> nothing happens (no RNG draw, no status)                      :334-341
//   reliability = (1.0f32 - loss) as f64                                 WorkerShared :538-543
//   chance = src_host.rng.gen::<f64>() = (xoshiro256++ >> 11) * 2^-53                  :365
//   drop iff !bootstrapping && chance >= reliability && payload_size > 0              :370-378
//   deliver = max(now + latency, round_end); next-event-time min; lowest-used-latency  :380-406
//   event (deliver, Packet, src_host_id, src_host_event_id) into the dst queue  :408-411, 619-629
// Destination order = EventQueue pop order (core/work/event.rs:84-155): time, then src host id,
// then src event id.  Every event of round r has deliver >= round_end, so batching the whole
// round to the barrier (core/manager.rs:455-464) is exact.
//
// Pipelines (one stream plus a side stream for K0, one host sync per round):
//   7  K0 draws || bin histogram + scans; K1 stamp places every record into its destination
//      bin (32 destinations); K4 bin_sort_v7 sorts each bin in LDS (decoupled look-back for
//      the event offsets) and stores the events in order
//   3  K0; K1 stamp writes records by packet; K2 radix sort by destination; K3 offsets; K4
//      per-destination wave sort (fallback when a bin overflows pipeline 7's limits)
//   1  64-bit records (path latencies >= 2^32 ns)
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>


#include <vector>

#include "scan.h"
#include "wave.h"

namespace shd {

constexpr uint32_t kStSkipped = 0, kStDropped = 1, kStSent = 2;

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

struct Xoshiro {
    uint64_t s0, s1, s2, s3;
    __device__ __forceinline__ uint64_t next() {
        const uint64_t res = rotl64(s0 + s3, 23) + s0;
        const uint64_t t = s1 << 17;
        s2 ^= s0;
        s3 ^= s1;
        s1 ^= s2;
        s0 ^= s3;
        s2 ^= t;
        s3 = rotl64(s3, 45);
        return res;
    }
    // rand 0.8.5 Standard for f64: 53 high bits, multiply-based, [0, 1)
    __device__ __forceinline__ double gen_f64() {
        return (double)(next() >> 11) * (1.0 / 9007199254740992.0);
    }
};

// chance >= reliability (worker.rs:365-370) from the draw's top 32 bits h = draw >> 32, which is
// all K0 keeps (4 bytes per draw instead of 8).  chance = (draw >> 11) * 2^-53 exactly, so the
// test is draw >> 11 >= T = ceil(reliability * 2^53) (exact: a power-of-two scale).  With
// th = T >> 21 it is h >= th when T is a multiple of 2^21.  That always holds for a table loss
// in [0, 1]: reliability = 1f32 - loss is >= 2^-9 (then reliability * 2^53 = m * 2^(e + 30),
// e >= -9, a multiple of 2^21) or is 1 - loss for loss in [0.5, 1], a multiple of 2^-24 (T a
// multiple of 2^29).  For any other value h > th decides unless h == th, where the low bits
// would: `tie` is set and the round is redone on the 64-bit pipeline (its own exact draws).
// reliability <= 0 always drops, NaN never (as the f64 comparison).
__device__ __forceinline__ bool draw_drops(uint32_t h, double reliability, bool& tie) {
    if (!(reliability > 0.0)) return reliability <= 0.0;
    if (reliability >= 1.0) return false;   // chance < 1
    const uint64_t T = (uint64_t)ceil(reliability * 9007199254740992.0);
    const uint64_t th = T >> 21;
    const bool low = (T & 0x1FFFFFull) != 0;
    if (low && (uint64_t)h == th) tie = true;
    return (uint64_t)h >= th + (low ? 1u : 0u);
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o);
        v = w < v ? w : v;
    }
    return v;
}

struct RelayArgs {
    uint32_t n_hosts, n_nodes;
    uint32_t src_lo, n_src;    // source hosts of this context: [src_lo, src_lo + n_src)
    const uint32_t* src_off;   // [n_src + 1], host src_lo + k's sends are [src_off[k], src_off[k+1])
    const uint64_t* send_time;
    const uint32_t* dst_host;
    const uint32_t* payload;
    const double* chance;
    const uint32_t* draw_cpu;  // CPU-drawn top 32 bits of next_u64 per packet (shd_relay_flush), or null
    const uint32_t* host_node;
    const uint64_t* lat;
    const float* loss;
    const uint64_t* rng;       // host state at round start (read)
    const uint64_t* next_id;
    uint64_t* rng_out;         // host state after the round (written; committed on success)
    uint64_t* next_id_out;
    unsigned long long* counts;  // nullable
    uint64_t round_end, sim_end, bootstrap_end;
    uint8_t* status;
    uint64_t* deliver;
    uint64_t* seq;
    uint32_t* slot;
    uint32_t* dst_cnt;
    unsigned long long* red;     // [0] min deliver, [1] min latency, [2] n_sent, [3] bad dst
};

__global__ __launch_bounds__(256) void relay_stamp(RelayArgs a) {
    const uint32_t hl = blockIdx.x * 256 + threadIdx.x, h = a.src_lo + hl;
    uint64_t my_min_d = ~0ull, my_min_l = ~0ull, my_sent = 0;
    if (hl < a.n_src) {
        Xoshiro r{a.rng[4 * (size_t)h], a.rng[4 * (size_t)h + 1], a.rng[4 * (size_t)h + 2],
                  a.rng[4 * (size_t)h + 3]};
        uint64_t id = a.next_id[h];
        const uint32_t sn = a.host_node[h];
        const uint32_t i1 = a.src_off[hl + 1];
        for (uint32_t i = a.src_off[hl]; i < i1; ++i) {
            const uint64_t now = a.send_time[i];
            uint8_t st = kStSkipped;
            if (now < a.sim_end) {
                const uint32_t d = a.dst_host[i];
                if (d >= a.n_hosts) {  // "No host ID for dest address" (worker.rs:350-355)
                    atomicMin(&a.red[3], (unsigned long long)i);
                    a.status[i] = kStSkipped;
                    continue;
                }
                const size_t pi = (size_t)sn * a.n_nodes + a.host_node[d];
                const double reliability = (double)one_minus(a.loss[pi]);
                bool ge;
                if (a.draw_cpu) {   // the top 32 bits decide exactly for a table reliability (draw_drops)
                    bool tie = false;
                    ge = draw_drops(a.draw_cpu[i], reliability, tie);
                } else {
                    ge = (a.chance ? a.chance[i] : r.gen_f64()) >= reliability;
                }
                const bool boot = now < a.bootstrap_end;
                if (!boot && ge && a.payload[i] > 0) {
                    st = kStDropped;
                } else {
                    const uint64_t delay = a.lat[pi];
                    uint64_t t = now + delay;
                    if (t < a.round_end) t = a.round_end;
                    st = kStSent;
                    a.deliver[i] = t;
                    a.seq[i] = id++;
                    a.slot[i] = atomicAdd(&a.dst_cnt[d], 1u);
                    if (a.counts) atomicAdd(&a.counts[pi], 1ull);
                    my_min_d = t < my_min_d ? t : my_min_d;
                    my_min_l = delay < my_min_l ? delay : my_min_l;
                    ++my_sent;
                }
            }
            a.status[i] = st;
        }
        a.rng_out[4 * (size_t)h] = r.s0;
        a.rng_out[4 * (size_t)h + 1] = r.s1;
        a.rng_out[4 * (size_t)h + 2] = r.s2;
        a.rng_out[4 * (size_t)h + 3] = r.s3;
        a.next_id_out[h] = id;
    }
    my_min_d = wave_min_u64(my_min_d);
    my_min_l = wave_min_u64(my_min_l);
    for (int o = 32; o > 0; o >>= 1) my_sent += __shfl_xor(my_sent, o);
    if ((threadIdx.x & 63) == 0) {
        if (my_min_d != ~0ull) atomicMin(&a.red[0], (unsigned long long)my_min_d);
        if (my_min_l != ~0ull) atomicMin(&a.red[1], (unsigned long long)my_min_l);
        if (my_sent) atomicAdd(&a.red[2], (unsigned long long)my_sent);
    }
}

// Per-packet source host from the grouped offsets (binary search; hosts are few per packet).
__device__ __forceinline__ uint32_t owner_of(const uint32_t* off, uint32_t n_hosts, uint32_t i) {
    uint32_t lo = 0, hi = n_hosts;  // find h with off[h] <= i < off[h+1]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void relay_scatter(
    uint64_t n, uint32_t n_src, uint32_t src_lo, const uint32_t* __restrict__ src_off,
    const uint8_t* __restrict__ status, const uint32_t* __restrict__ dst_host,
    const uint32_t* __restrict__ slot, const uint64_t* __restrict__ deliver,
    const uint64_t* __restrict__ seq, const uint32_t* __restrict__ ev_off,
    uint64_t* __restrict__ ev_deliver, uint32_t* __restrict__ ev_src, uint64_t* __restrict__ ev_seq,
    uint32_t* __restrict__ ev_pkt) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n || status[i] != kStSent) return;
    const uint32_t pos = ev_off[dst_host[i]] + slot[i];
    ev_deliver[pos] = deliver[i];
    ev_src[pos] = src_lo + owner_of(src_off, n_src, (uint32_t)i);
    ev_seq[pos] = seq[i];
    ev_pkt[pos] = (uint32_t)i;
}

// Sort one destination's bucket by (deliver, src, seq) -- bitonic network in LDS.
constexpr uint32_t kV1Cap = 1024;

struct EvKey {
    uint64_t t;
    uint64_t sq;   // seq
    uint32_t src;
    uint32_t pkt;
};
__device__ __forceinline__ bool ev_less(const EvKey& a, const EvKey& b) {
    if (a.t != b.t) return a.t < b.t;
    if (a.src != b.src) return a.src < b.src;
    return a.sq < b.sq;
}

__global__ __launch_bounds__(256) void segment_sort(
    uint32_t n_hosts, const uint32_t* __restrict__ ev_off, uint64_t* __restrict__ ev_deliver,
    uint32_t* __restrict__ ev_src, uint64_t* __restrict__ ev_seq, uint32_t* __restrict__ ev_pkt,
    uint32_t* __restrict__ big) {
    __shared__ EvKey s[kV1Cap];
    const uint32_t d = blockIdx.x;
    const uint32_t b = ev_off[d], n = ev_off[d + 1] - b;
    if (n <= 1) return;
    if (n > kV1Cap) {
        if (threadIdx.x == 0) big[atomicAdd(&big[0], 1u) + 1] = d;
        return;
    }
    uint32_t P = 1;
    while (P < n) P <<= 1;
    for (uint32_t i = threadIdx.x; i < P; i += 256) {
        if (i < n)
            s[i] = EvKey{ev_deliver[b + i], ev_seq[b + i], ev_src[b + i], ev_pkt[b + i]};
        else
            s[i] = EvKey{~0ull, ~0ull, ~0u, ~0u};
    }
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < P; i += 256) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    EvKey x = s[i], y = s[l];
                    if (ev_less(y, x) == up) {
                        s[i] = y;
                        s[l] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < n; i += 256) {
        const EvKey e = s[i];
        ev_deliver[b + i] = e.t;
        ev_src[b + i] = e.src;
        ev_seq[b + i] = e.sq;
        ev_pkt[b + i] = e.pkt;
    }
}

// Oversized buckets (> kV1Cap events for one destination in one round): bottom-up merge
// sort of that bucket by one workgroup through a global scratch area.
__global__ __launch_bounds__(256) void segment_sort_big(
    const uint32_t* __restrict__ big, const uint32_t* __restrict__ ev_off,
    uint64_t* __restrict__ ev_deliver, uint32_t* __restrict__ ev_src, uint64_t* __restrict__ ev_seq,
    uint32_t* __restrict__ ev_pkt, EvKey* __restrict__ tmp) {
    const uint32_t d = big[1 + blockIdx.x];
    const uint32_t b = ev_off[d], n = ev_off[d + 1] - b;
    EvKey* A = tmp + b;  // this bucket's slice of the scratch (one EvKey per event)
    for (uint32_t i = threadIdx.x; i < n; i += 256)
        A[i] = EvKey{ev_deliver[b + i], ev_seq[b + i], ev_src[b + i], ev_pkt[b + i]};
    __syncthreads();
    // merge passes of run width w; each element finds its output rank by binary search in
    // the sibling run (keys are unique, so ranks never collide)
    for (uint32_t w = 1; w < n; w <<= 1) {
        // merge runs [i, i+w) and [i+w, i+2w) into ev_* arrays, then copy back
        for (uint32_t o = threadIdx.x; o < n; o += 256) {
            const uint32_t run = o / (2 * w), lo = run * 2 * w;
            const uint32_t mid = min(lo + w, n), hi = min(lo + 2 * w, n);
            // rank of element o within the merged output: binary search in the other run
            const EvKey x = A[o];
            uint32_t rank;
            if (o < mid) {
                uint32_t l = mid, h = hi;  // count of elements in right run strictly less
                while (l < h) {
                    const uint32_t m = (l + h) >> 1;
                    if (ev_less(A[m], x)) l = m + 1; else h = m;
                }
                rank = (o - lo) + (l - mid);
            } else {
                uint32_t l = lo, h = mid;  // count of elements in left run <= x (keys unique)
                while (l < h) {
                    const uint32_t m = (l + h) >> 1;
                    if (ev_less(x, A[m])) h = m; else l = m + 1;
                }
                rank = (o - mid) + (l - lo);
            }
            const uint32_t dst = b + lo + rank;
            ev_deliver[dst] = x.t;
            ev_src[dst] = x.src;
            ev_seq[dst] = x.sq;
            ev_pkt[dst] = x.pkt;
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < n; i += 256)
            A[i] = EvKey{ev_deliver[b + i], ev_seq[b + i], ev_src[b + i], ev_pkt[b + i]};
        __syncthreads();
    }
}

// ==========================================================================================
// Narrow pipeline (every path latency < 2^32 ns and every deliver - round_end < 2^32): 16-byte
// event records {deliver - round_end, src host, seq - seq_base[src], packet index}.
//   K0 relay_draws      lane per source host: its Xoshiro256++ stream (the only sequential work)
//   K1 relay_stamp_v5   workgroup per 64 source hosts (in source-node order), lane per send:
//                       coalesced loads, path lookup (LDS-staged rows), drop rule, deliver
//                       stamp, scan-based event ids, coalesced stores of status / key / record
//   K2 stable LSD radix sort of the records by destination (scan.h rs_hist / rs_scatter, 6-bit
//      digits) -- stable: the batch is in (source host, event id) order, so every
//      destination's run stays in that order
//   K3 bucket_offsets   lower bound of every destination in the sorted keys
//   K4 segment_sort_v4  wave per destination run: bitonic sort in registers of the unique key
//                       (deliver offset << 32 | position in the run); ties on the deliver time
//                       fall back to run order = (src host, event id) order
// ==========================================================================================
struct RelayArgs3 {
    uint32_t n_hosts, n_nodes;
    uint32_t src_lo, n_src;    // source hosts of this context: [src_lo, src_lo + n_src)
    const uint32_t* src_off;   // [n_src + 1], indexed by host - src_lo
    const uint64_t* send_time;
    const uint32_t* dst_host;
    const uint32_t* payload;
    const double* chance;
    uint32_t keep_rng;         // 1: the draws came from the CPU (shd_relay_flush): device streams untouched
    const uint32_t* host_node;
    const uint32_t* order;     // the n_src source host ids sorted by host_node (workgroup -> hosts)
    const uint2* path;         // {latency ns (u32), packet loss bits} per node pair
    const uint64_t* rng;
    const uint64_t* next_id;
    uint64_t* rng_out;
    uint64_t* next_id_out;
    unsigned long long* counts;
    uint64_t round_end, sim_end, bootstrap_end;
    uint32_t abs_seq;    // 1: every event id of the round fits 32 bits -> records hold absolute ids
    uint8_t* status;
    uint4* rec;          // per packet (valid when SENT)
    uint32_t* key;       // per packet: destination host if SENT, else n_hosts (sorts last)
    unsigned long long* red;   // [0] min deliver [1] min latency [2] n_sent [3] bad dst [4] wide
                               // [5] send-order violation [6] v7 bin overflow
    // v7 (destination-bin placement): the records of bin b written by stamp workgroup g start at
    // bin_base[b] + seg_pre[g * n_bins + b]
    const uint32_t* bin_base;
    const uint32_t* seg_pre;
    uint32_t n_bins;
    uint32_t gs;         // hosts per group of relay_stamp_v6 / relay_bin_hist (<= kS5Hosts)
    // v7 under a communicator (relay_round_sharded_v7): every rank's destinations [r * sh_per,
    // ...) start a fresh bin, so rank r's bins are [r * sh_bpr, ...) and the records bound for it
    // one contiguous slice; sh_mul = ceil(2^40 / sh_per).  sh_per = 0: bins of consecutive hosts.
    uint32_t sh_per, sh_bpr;
    uint64_t sh_mul;
};

#ifndef SHD_DRAW_SLICE
#define SHD_DRAW_SLICE 16
#endif
constexpr uint32_t kDrawSlice = SHD_DRAW_SLICE;   // draws per host per LDS transpose (16: 43 us vs 47 at 8 on C5)

// K0 relay_draws: the only sequential part of the relay -- every source host's Xoshiro256++
// stream (host.rs:218, worker.rs:365) -- as its own kernel: one lane per host (64 consecutive
// hosts per one-wave workgroup), staged through LDS so the draws leave as 64-byte runs.  A send
// draws iff now < sim_end (worker.rs:334-341); send times are non-decreasing within a host (a
// host's sends happen in simulated-time order; the stamp checks it), so the drawing sends are a
// prefix of the host's range, found from its last send (binary search when it is skipped).
#ifndef SHD_K0_WAVES
#define SHD_K0_WAVES 1
#endif
#ifdef SHD_STAMP_PROF
// K0 (relay_draws, tuning builds): per wave, shader clocks of setup / draws / stores and its
// 100 MHz start / end (tools/k0_prof.py)
__device__ unsigned long long g_k0_prof[4096][5];
#endif
constexpr uint32_t kK0Waves = SHD_K0_WAVES;   // waves (64 hosts each) per K0 workgroup
__global__ __launch_bounds__(64 * kK0Waves) void relay_draws(RelayArgs3 a, uint32_t* __restrict__ draw) {
    __shared__ uint32_t s_all[kK0Waves][kDrawSlice][65];   // the draws' top 32 bits (draw_drops)
    __shared__ uint32_t s_beg_all[kK0Waves][64], s_nd_all[kK0Waves][64];
    const uint32_t wv = threadIdx.x >> 6;
    auto& s = s_all[wv];
    uint32_t* s_beg = s_beg_all[wv];
    uint32_t* s_nd = s_nd_all[wv];
    const uint32_t lane = threadIdx.x & 63, hl = (blockIdx.x * kK0Waves + wv) * 64 + lane, h = a.src_lo + hl;
#ifdef SHD_STAMP_PROF
    const uint64_t k0_t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t k0_c = __builtin_amdgcn_s_memtime(), k0_acc[3] = {0, 0, 0};
#define K0_MARK(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); k0_acc[i] += t_ - k0_c; k0_c = t_; } while (0)
#else
#define K0_MARK(i) do { } while (0)
#endif
    uint32_t nd = 0;
    Xoshiro r{0, 0, 0, 0};
    if (hl < a.n_src) {
        // the stream's state first: its loads need nothing below, so they share the first trip
        r = Xoshiro{a.rng[4 * (size_t)h], a.rng[4 * (size_t)h + 1], a.rng[4 * (size_t)h + 2],
                    a.rng[4 * (size_t)h + 3]};
        const uint32_t b = a.src_off[hl], e = a.src_off[hl + 1];
        nd = e - b;
        if (nd && !(a.send_time[e - 1] < a.sim_end)) {   // first send with now >= sim_end
            uint32_t lo = b, hi = e;
            while (lo < hi) {
                const uint32_t m = (lo + hi) >> 1;
                if (a.send_time[m] < a.sim_end) lo = m + 1; else hi = m;
            }
            nd = lo - b;
        }
        s_beg[lane] = b;
    } else {
        s_beg[lane] = 0;
    }
    s_nd[lane] = nd;
    uint32_t mx = nd;
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the store pattern below: kDrawSlice lanes per host write its kDrawSlice consecutive draws
    // (4 B each), 64 / kDrawSlice hosts per step.  The hosts' (count, start) a lane stores for
    // are the same every slice: read once into registers (read per store, each store waited on
    // two dependent LDS round trips: C5 K0 alone 34.6 -> 30.1 us)
    K0_MARK(0);
    constexpr uint32_t kG = kDrawSlice, kHpg = 64 / kDrawSlice;
    const uint32_t kl = lane % kDrawSlice;
    uint32_t g_nd[kG], g_beg[kG];
#pragma unroll
    for (uint32_t g = 0; g < kG; ++g) {
        const uint32_t hl = g * kHpg + lane / kDrawSlice;
        g_nd[g] = s_nd[hl];
        g_beg[g] = s_beg[hl];
    }
    for (uint32_t j0 = 0; j0 < mx; j0 += kDrawSlice) {
        // the slice's draws in registers first, then to LDS together: a draw written to LDS as it
        // came made the next draw wait for that write (its registers were reused), an LDS round
        // trip per draw on the generator's chain
        uint32_t dv[kDrawSlice];
#pragma unroll
        for (uint32_t k = 0; k < kDrawSlice; ++k) {
            dv[k] = 0u;
            if (j0 + k < nd) dv[k] = (uint32_t)(r.next() >> 32);
        }
        K0_MARK(1);
#pragma unroll
        for (uint32_t k = 0; k < kDrawSlice; ++k) s[k][lane] = dv[k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t v[kG];
#pragma unroll
        for (uint32_t g = 0; g < kG; ++g) v[g] = s[kl][g * kHpg + lane / kDrawSlice];
#pragma unroll
        for (uint32_t g = 0; g < kG; ++g)
            if (j0 + kl < g_nd[g]) draw[g_beg[g] + j0 + kl] = v[g];
        __builtin_amdgcn_wave_barrier();
        K0_MARK(2);
    }
    if (hl < a.n_src) {
        a.rng_out[4 * (size_t)h] = r.s0;
        a.rng_out[4 * (size_t)h + 1] = r.s1;
        a.rng_out[4 * (size_t)h + 2] = r.s2;
        a.rng_out[4 * (size_t)h + 3] = r.s3;
    }
#ifdef SHD_STAMP_PROF
    {
        const uint32_t wid = blockIdx.x * kK0Waves + wv;
        if (lane == 0 && wid < 4096) {
            g_k0_prof[wid][0] = k0_acc[0];
            g_k0_prof[wid][1] = k0_acc[1];
            g_k0_prof[wid][2] = k0_acc[2];
            g_k0_prof[wid][3] = k0_t0;
            g_k0_prof[wid][4] = __builtin_amdgcn_s_memrealtime();
        }
    }
#endif
#undef K0_MARK
}

// A path-table entry from global memory through an explicit global (addrspace 1) pointer.  Next
// to an LDS-staged alternative a plain `cond ? s_rows[i] : path[j]` lets the compiler select the
// pointer and issue a flat load, and a flat load makes every later s_waitcnt wait for the
// wave's outstanding stores as well -- which serialised the stamp's record stores.
__device__ __forceinline__ uint2 path_global(const uint2* p, size_t i) {
    const unsigned long long v = ((const __attribute__((address_space(1))) unsigned long long*)p)[i];
    return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}

// K1 relay_stamp_v5: a workgroup owns kS5Hosts source hosts taken in source-node order
// (R.order), so its path lookups stay in one or two table rows, staged in LDS when they fit.
// The hosts' sends (one contiguous range per host) form one list, processed in chunks of
// kS5Cap positions with consecutive lanes on consecutive positions (coalesced inside every
// host's range).  No sequential work is left: lane per send, the raw loads, the draw (K0), the
// destination node and path, the drop rule and deliver stamp (worker.rs:370-402); a block-wide
// exclusive scan of the sent flags gives every sent packet its event id (host.rs:580-584).
constexpr uint32_t kS5Hosts = 64;
constexpr uint32_t kS5Per = 4;                  // sends per thread per chunk
constexpr uint32_t kS5Cap = 256 * kS5Per;
constexpr uint32_t kS5RowLds = 2048;            // staged path-table entries (16 KB)

// (round 6: the chunk's loads issued together -- the sends' fields, then the destinations' nodes,
// then the path entries, each a batch of independent loads -- instead of one guarded chain per
// send; CH as relay_stamp_v6's)
template <bool CH>
__global__ __launch_bounds__(256) void relay_stamp_v5(RelayArgs3 a, const uint32_t* __restrict__ draw) {
    __shared__ uint2 s_rows[kS5RowLds];
    __shared__ uint16_t s_scan[kS5Cap + 1];
    __shared__ uint32_t s_host[kS5Hosts], s_beg[kS5Hosts], s_pre[kS5Hosts + 1], s_node[kS5Hosts];
    __shared__ uint32_t s_rowof[kS5Hosts], s_rownode[kS5Hosts], s_run[kS5Hosts], s_base[kS5Hosts];
    __shared__ uint32_t s_wsum[4], s_nrows;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t h0 = blockIdx.x * kS5Hosts;
    const uint32_t nh = min(kS5Hosts, a.n_src - h0);
    if (tid < 64) {   // wave 0: this workgroup's hosts, their ranges (prefix) and staged rows
        uint32_t len = 0, nd = 0;
        if (tid < nh) {
            const uint32_t h = a.order[h0 + tid];
            const uint32_t b = a.src_off[h - a.src_lo];
            len = a.src_off[h - a.src_lo + 1] - b;
            nd = a.host_node[h];
            s_host[tid] = h;
            s_beg[tid] = b;
            s_node[tid] = nd;
            s_run[tid] = 0;
            s_base[tid] = a.abs_seq ? (uint32_t)a.next_id[h] : 0u;
        }
        uint32_t incl = len;
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (tid < nh) s_pre[tid + 1] = incl;
        if (tid == 0) s_pre[0] = 0;
        const uint32_t prev = __shfl_up(nd, 1);
        const bool first = tid < nh && (tid == 0 || nd != prev);
        const uint64_t fm = __ballot(first);
        if (tid < nh) {
            const uint32_t ri = (uint32_t)__popcll(fm & ((2ull << tid) - 1ull)) - 1u;
            s_rowof[tid] = ri;
            if (first) s_rownode[ri] = nd;
        }
        if (tid == 0) s_nrows = (uint32_t)__popcll(fm);
    }
    __syncthreads();
    const bool staged = (uint64_t)s_nrows * a.n_nodes <= kS5RowLds;
    if (staged) {
        const uint32_t tot = s_nrows * a.n_nodes;
        for (uint32_t e = tid; e < tot; e += 256) {
            const uint32_t rr = e / a.n_nodes, c = e - rr * a.n_nodes;
            s_rows[e] = a.path[(size_t)s_rownode[rr] * a.n_nodes + c];
        }
    }
    __syncthreads();
    const uint32_t T = s_pre[nh];
    uint64_t min_d = ~0ull, min_l = ~0ull;
    bool wide = false, disorder = false;
    for (uint32_t c0 = 0; c0 < T; c0 += kS5Cap) {
        const uint32_t cn = min(kS5Cap, T - c0);
        uint8_t st[kS5Per];
        uint32_t doff[kS5Per], dst[kS5Per], idx[kS5Per], hl[kS5Per], dn[kS5Per];
        bool k0[kS5Per];
        // (a) owners and packet indices (positions past the chunk clamped onto its last packet,
        // so every load below is in bounds and unconditional)
#pragma unroll
        for (uint32_t i = 0; i < kS5Per; ++i) {
            const uint32_t gp = c0 + min(tid + 256 * i, cn - 1);
            uint32_t lo = 0, hi = nh;       // s_pre[lo] <= gp < s_pre[lo + 1]
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_pre[mid] <= gp) lo = mid; else hi = mid;
            }
            hl[i] = lo;
            const uint32_t k = gp - s_pre[lo];
            k0[i] = k == 0;
            idx[i] = s_beg[lo] + k;
        }
        // (b) the sends' fields, (c) their destinations' nodes, (d) the path entries
        uint64_t now[kS5Per], prv[kS5Per];
        std::conditional_t<CH, double, uint32_t> rv[kS5Per];
        uint32_t pay[kS5Per];
#pragma unroll
        for (uint32_t i = 0; i < kS5Per; ++i) {
            now[i] = a.send_time[idx[i]];
            prv[i] = a.send_time[idx[i] - (k0[i] ? 0u : 1u)];
            dst[i] = a.dst_host[idx[i]];
            pay[i] = a.payload[idx[i]];
            if constexpr (CH) rv[i] = a.chance[idx[i]];
            else rv[i] = draw[idx[i]];
        }
#pragma unroll
        for (uint32_t i = 0; i < kS5Per; ++i) dn[i] = a.host_node[min(dst[i], a.n_hosts - 1)];
        uint2 pp[kS5Per];
#pragma unroll
        for (uint32_t i = 0; i < kS5Per; ++i)
            pp[i] = staged ? s_rows[s_rowof[hl[i]] * a.n_nodes + dn[i]]
                           : path_global(a.path, (size_t)s_node[hl[i]] * a.n_nodes + dn[i]);
#pragma unroll
        for (uint32_t i = 0; i < kS5Per; ++i) {
            const uint32_t pos = tid + 256 * i;
            st[i] = kStSkipped;
            doff[i] = 0;
            if (pos < cn) {
                // a drawing send after a skipped one breaks K0's prefix rule
                disorder |= !k0[i] & (now[i] < a.sim_end) & !(prv[i] < a.sim_end);
                if (dst[i] >= a.n_hosts) {      // "No host ID for dest address" (worker.rs:350-355)
                    atomicMin(&a.red[3], (unsigned long long)idx[i]);
                } else if (now[i] < a.sim_end) {
                    const double reliability = (double)one_minus(__uint_as_float(pp[i].y));
                    bool tie = false;
                    bool ge;
                    if constexpr (CH) ge = rv[i] >= reliability;
                    else ge = draw_drops(rv[i], reliability, tie);
                    wide |= tie;   // a draw whose low bits would decide: redo the round on pipeline 1
                    if (!(now[i] < a.bootstrap_end) && ge && pay[i] > 0) {
                        st[i] = kStDropped;
                    } else {
                        uint64_t tt = now[i] + pp[i].x;
                        if (tt < a.round_end) tt = a.round_end;
                        const uint64_t dd = tt - a.round_end;
                        wide |= (dd >> 32) != 0;
                        min_d = tt < min_d ? tt : min_d;
                        min_l = pp[i].x < min_l ? pp[i].x : min_l;
                        doff[i] = (uint32_t)dd;
                        st[i] = kStSent;
                    }
                }
            }
            s_scan[pos] = st[i] == kStSent ? 1 : 0;
        }
        __syncthreads();
        {   // block-wide exclusive scan of the sent flags (kS5Per consecutive entries per thread)
            uint32_t v[kS5Per], sum = 0;
#pragma unroll
            for (uint32_t i = 0; i < kS5Per; ++i) {
                v[i] = s_scan[tid * kS5Per + i];
                sum += v[i];
            }
            uint32_t incl = sum;
#pragma unroll
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            if (lane == 63) s_wsum[w] = incl;
            __syncthreads();
            uint32_t run = incl - sum;
            for (uint32_t ww = 0; ww < w; ++ww) run += s_wsum[ww];
#pragma unroll
            for (uint32_t i = 0; i < kS5Per; ++i) {
                s_scan[tid * kS5Per + i] = (uint16_t)run;
                run += v[i];
            }
            if (tid == 255) s_scan[kS5Cap] = (uint16_t)run;
        }
        __syncthreads();
        // stores; event id = host's running count + sent sends before this one in its range
#pragma unroll
        for (uint32_t i = 0; i < kS5Per; ++i) {
            const uint32_t pos = tid + 256 * i;
            if (pos < cn) {
                a.status[idx[i]] = st[i];
                a.key[idx[i]] = st[i] == kStSent ? dst[i] : a.n_hosts;
                if (st[i] == kStSent) {
                    const uint32_t first = max(s_pre[hl[i]], c0) - c0;
                    const uint32_t local = s_base[hl[i]] + s_run[hl[i]] + s_scan[pos] - s_scan[first];
                    a.rec[idx[i]] = make_uint4(doff[i], s_host[hl[i]], local, idx[i]);
                    if (a.counts) atomicAdd(&a.counts[(size_t)s_node[hl[i]] * a.n_nodes + dn[i]], 1ull);
                }
            }
        }
        __syncthreads();
        if (tid < nh) {   // running counts for the next chunk
            const uint32_t pb = max(s_pre[tid], c0), pe = min(s_pre[tid + 1], c0 + cn);
            if (pe > pb) s_run[tid] += s_scan[pe - c0] - s_scan[pb - c0];
        }
        __syncthreads();
    }
    uint64_t ns = 0;
    if (tid < nh) {
        const size_t h = s_host[tid];
        if (a.chance || a.keep_rng)
            for (int k = 0; k < 4; ++k) a.rng_out[4 * h + k] = a.rng[4 * h + k];
        ns = s_run[tid];
        a.next_id_out[h] = a.next_id[h] + ns;
    }
    min_d = wave_min_u64(min_d);
    min_l = wave_min_u64(min_l);
    for (int o = 32; o > 0; o >>= 1) ns += __shfl_xor(ns, o);
    const bool any_wide = __ballot(wide) != 0, any_disorder = __ballot(disorder) != 0;
    if (lane == 0) {
        if (min_d != ~0ull) atomicMin(&a.red[0], (unsigned long long)min_d);
        if (min_l != ~0ull) atomicMin(&a.red[1], (unsigned long long)min_l);
        if (ns) atomicAdd(&a.red[2], (unsigned long long)ns);
        if (any_wide) atomicOr(&a.red[4], 1ull);
        if (any_disorder) atomicOr(&a.red[5], 1ull);
    }
}

// K1 (small node count): relay_stamp_v6 is relay_stamp_v5 with the host -> node map resident in
// LDS, bit-packed at ceil(log2 n_nodes) bits per host (C5: 100k hosts x 10 bits = 125 KB), so
// the destination-node lookup -- otherwise one random 64-byte L2 request per send, the stamp's
// dominant cost -- becomes an LDS read.  One persistent 1024-thread workgroup per CU loads the
// packed map once and walks the host groups (kS5Hosts hosts each, in source-node order).
constexpr uint32_t kS6Threads = 1024;
#ifndef SHD_S6PER
#define SHD_S6PER 4   // sends per thread and chunk (5 and 6 spill registers: slower)
#endif
constexpr uint32_t kS6Per = SHD_S6PER;
constexpr uint32_t kS6Cap = kS6Threads * kS6Per;
constexpr uint32_t kS6FixedLds = kS5RowLds * 8 + (kS6Cap + 2) * 2 + kS6Cap + 4096;   // rows + scan + owners + small

__device__ __forceinline__ uint32_t packed_get(const uint32_t* t, uint32_t j, uint32_t bits) {
    const uint32_t o = j * bits, w = o >> 5, sh = o & 31;
    uint64_t v = t[w];
    if (sh + bits > 32) v |= (uint64_t)t[w + 1] << 32;
    return (uint32_t)(v >> sh) & ((1u << bits) - 1u);
}

#ifdef SHD_STAMP_PROF
// tuning builds only (tools/stamp_prof.sh): shader clocks per phase, summed over workgroups
__device__ unsigned long long g_stamp_prof[12];
#define SP_MARK(slot) do { if (threadIdx.x == 0) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    sp_acc[slot] += t_ - sp_t; sp_t = t_; } } while (0)
#else
#define SP_MARK(slot) do { } while (0)
#endif

// BIN (pipeline v7): every packet with a valid destination is also placed, sent or not, into
// its destination bin (kBinDst consecutive destinations): the workgroup's slots of bin b are
// the segment bin_base[b] + seg_pre[g][b] counted by relay_bin_hist; the slot inside the
// segment comes from an LDS counter (one u32 per bin holding the absolute next slot).  The records carry the
// status and the destination's low bits so bin_sort_v7 can filter and split them.
constexpr uint32_t kBinShift = 5;
constexpr uint32_t kBinDst = 1u << kBinShift;

// the bin of a destination and its place dl in the bin (RelayArgs3::sh_per)
__device__ __forceinline__ uint32_t dst_bin(const RelayArgs3& a, uint32_t dst, uint32_t& dl) {
    if (a.sh_per == 0) {
        dl = dst & (kBinDst - 1);
        return dst >> kBinShift;
    }
    // dst / sh_per: exact for dst, sh_per < 2^18 (the error of the rounded-up reciprocal stays
    // below 2^-22, under the smallest distance 1 / sh_per of a fraction from the next integer)
    const uint32_t r = (uint32_t)(((uint64_t)dst * a.sh_mul) >> 40);
    const uint32_t x = dst - r * a.sh_per;
    dl = x & (kBinDst - 1);
    return r * a.sh_bpr + (x >> kBinShift);
}
constexpr uint32_t kHistSplit = 2;   // histogram rows per stamp workgroup (relay_bin_hist)

// CH: the batch carries f64 chances (a.chance) instead of K0's draws.  A template parameter, not
// a run-time select: `a.chance ? chance64[i] : draw[i]` compiled to a branch whose join moved the
// loaded value with an s_waitcnt vmcnt(0), so each of a thread's kS6Per load sets waited for the
// one before it (four memory round trips per chunk instead of one).
// MAP = false (round 6, C5b): the host -> node map does not fit the LDS (50k nodes: 16 bits x
// 100k hosts), so each chunk gathers its destinations' nodes from global memory (a 400 KB array,
// L2-resident) and, the rows being too long to stage, its path entries from the packed table --
// each a batch of unconditional loads -- and the records still go straight to their bins
// (pipeline 7 instead of pipeline 3's radix sort: the bins need only the slot counters in LDS).
template <bool BIN, bool CH, bool MAP = true>
__global__ __launch_bounds__(kS6Threads) void relay_stamp_v6(RelayArgs3 a, const uint32_t* __restrict__ draw,
                                                             const uint32_t* __restrict__ packed,
                                                             uint32_t n_words, uint32_t bits) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_tbl[];   // packed host -> node
    // BIN: per bin, the next record slot of this workgroup's segment (absolute: bin base + segment
    // start + records placed), so placing a record is one LDS atomic -- no per-record loads of
    // the bases (a scattered load costs ~64 TA cycles per wave instruction: ~30 us of the stamp)
    uint32_t* s_slot = s_tbl + n_words;
    if (BIN && a.red[6]) return;   // a bin overflowed bin_sort_v7's LDS stage: the host reruns v3
    constexpr uint32_t kW = kS6Threads / 64;
    static_assert(kS6Per * kW <= 64, "one wave scans the chunk's (i, wave) sent totals");
    __shared__ uint2 s_rows[kS5RowLds];
    __shared__ uint32_t s_host[kS5Hosts], s_beg[kS5Hosts], s_pre[kS5Hosts + 1], s_node[kS5Hosts];
    __shared__ uint32_t s_rowof[kS5Hosts], s_rownode[kS5Hosts], s_run[kS5Hosts], s_base[kS5Hosts];
    __shared__ uint32_t s_off[kS5Hosts];    // a host's event id = s_off + the chunk's sent prefix
    __shared__ uint32_t s_wt[64], s_nrows;  // sent sends per (i, wave) of the chunk
    __shared__ uint8_t s_own[kS6Cap];   // chunk position -> host slot in the group
    // next group's distinct source nodes: up to one per host of the group (a group of kS5Hosts
    // hosts spans at most kS5Hosts nodes; the prefetch stages pn * n_nodes <= kS5RowLds entries)
    __shared__ uint32_t s_pfnode[kS5Hosts], s_pfn;
    static_assert(kS5RowLds % kS6Threads == 0, "row prefetch: whole entries per thread");
    constexpr uint32_t kPf = kS5RowLds / kS6Threads;
    uint2 pf[kPf];             // the next group's staged path rows, prefetched during this group
    bool have_pf = false;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#ifdef SHD_STAMP_PROF
    uint64_t sp_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, sp_t = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (MAP)
        for (uint32_t i = tid; i < n_words; i += kS6Threads) s_tbl[i] = packed[i];
    if (BIN)
        for (uint32_t b = tid; b < a.n_bins; b += kS6Threads)
            s_slot[b] = a.bin_base[b] + a.seg_pre[(size_t)blockIdx.x * a.n_bins + b];
    const uint32_t n_groups = (a.n_src + a.gs - 1) / a.gs;
    uint64_t min_d = ~0ull, min_l = ~0ull, ns_total = 0;
    bool wide = false, disorder = false;
    // wave 0 keeps the next group's host descriptors in registers: order[] is fetched when a
    // group starts and the dependent src_off / host_node / next_id loads are issued once its
    // path rows are staged, so neither latency sits on the critical path of the next group
    uint32_t p_h = 0, p_b = 0, p_len = 0, p_nd = 0, p_base = 0;
    auto fetch_hosts = [&](uint32_t g) {
        const uint32_t hh0 = g * a.gs;
        if (g < n_groups && tid < min(a.gs, a.n_src - hh0)) {
            p_b = a.src_off[p_h - a.src_lo];
            p_len = a.src_off[p_h - a.src_lo + 1] - p_b;
            p_nd = a.host_node[p_h];
            p_base = a.abs_seq ? (uint32_t)a.next_id[p_h] : 0u;
        }
    };
    if (tid < 64 && blockIdx.x < n_groups && tid < min(a.gs, a.n_src - blockIdx.x * a.gs)) {
        p_h = a.order[blockIdx.x * a.gs + tid];
    }
    if (tid < 64) fetch_hosts(blockIdx.x);
    // 16 threads per host slot fill the owner map of the chunk starting at position cb
    static_assert(kS6Threads == kS5Hosts * 16, "owner fill: 16 threads per host slot");
    auto fill_owner = [&](uint32_t cb, uint32_t nh) {
        const uint32_t hh = tid >> 4, sub = tid & 15;
        if (hh < nh) {
            const uint32_t pb = max(s_pre[hh], cb), pe = min(s_pre[hh + 1], cb + kS6Cap);
            for (uint32_t p = pb + sub; p < pe; p += 16) s_own[p - cb] = (uint8_t)hh;
        }
    };
    const uint64_t* __restrict__ chance64 = reinterpret_cast<const uint64_t*>(a.chance);
    for (uint32_t grp = blockIdx.x; grp < n_groups; grp += gridDim.x) {
        const uint32_t h0 = grp * a.gs;
        const uint32_t nh = min(a.gs, a.n_src - h0);
        const uint32_t nxt = grp + gridDim.x;
        __syncthreads();   // the previous group's host arrays / rows are no longer read
        SP_MARK(0);
        if (tid < 64) {
            uint32_t len = 0, nd = 0;
            if (tid < nh) {
                len = p_len;
                nd = p_nd;
                s_host[tid] = p_h;
                s_beg[tid] = p_b;
                s_node[tid] = nd;
                s_run[tid] = 0;
                s_base[tid] = p_base;
            }
            if (nxt < n_groups && tid < min(a.gs, a.n_src - nxt * a.gs))
                p_h = a.order[nxt * a.gs + tid];
            uint32_t incl = len;
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            if (tid < nh) s_pre[tid + 1] = incl;
            if (tid == 0) s_pre[0] = 0;
            const uint32_t prev = __shfl_up(nd, 1);
            const bool first = tid < nh && (tid == 0 || nd != prev);
            const uint64_t fm = __ballot(first);
            if (tid < nh) {
                const uint32_t ri = (uint32_t)__popcll(fm & ((2ull << tid) - 1ull)) - 1u;
                s_rowof[tid] = ri;
                if (first) s_rownode[ri] = nd;
            }
            if (tid == 0) s_nrows = (uint32_t)__popcll(fm);
        }
        __syncthreads();
        SP_MARK(1);
        const bool staged = MAP && (uint64_t)s_nrows * a.n_nodes <= kS5RowLds;
        if (staged) {
            const uint32_t tot = s_nrows * a.n_nodes;
            if (have_pf) {   // rows loaded during the previous group (same node list by construction)
#pragma unroll
                for (uint32_t j = 0; j < kPf; ++j)
                    if (tid + j * kS6Threads < tot) s_rows[tid + j * kS6Threads] = pf[j];
            } else {
                for (uint32_t e = tid; e < tot; e += kS6Threads) {
                    const uint32_t rr = e / a.n_nodes, c = e - rr * a.n_nodes;
                    s_rows[e] = a.path[(size_t)s_rownode[rr] * a.n_nodes + c];
                }
            }
        }
        have_pf = false;
        fill_owner(0, nh);
        if (tid < 64) fetch_hosts(nxt);
        __syncthreads();
        SP_MARK(2);
        const uint32_t T = s_pre[nh];
        for (uint32_t c0 = 0; c0 < T; c0 += kS6Cap) {
            const uint32_t cn = min(kS6Cap, T - c0);
            if (c0 == 0 && tid < 64) {   // the next group's distinct source nodes, as at its start
                const uint32_t nh2 = nxt < n_groups ? min(a.gs, a.n_src - nxt * a.gs) : 0u;
                const uint32_t nd = p_nd, prev = __shfl_up(nd, 1);
                const bool first = tid < nh2 && (tid == 0 || nd != prev);
                const uint64_t fm = __ballot(first);
                if (first) {
                    const uint32_t ri = (uint32_t)__popcll(fm & ((2ull << tid) - 1ull)) - 1u;
                    s_pfnode[ri] = nd;   // ri < nh2 <= kS5Hosts
                }
                if (tid == 0) s_pfn = (uint32_t)__popcll(fm);
            }
            // (a) positions -> packet indices through the owner map (positions past the chunk end
            // are clamped onto its last packet so every load below is in bounds and unconditional)
            // hl: the host slot, plus kFirst / kLast when the position is the host's first / last send
            // (the position inside the host is needed only for those and the load below: one
            // register per position less)
            constexpr uint32_t kFirst = 0x100, kLast = 0x200, kSlot = 0xFF;
            uint32_t idx[kS6Per], hl[kS6Per];
#pragma unroll
            for (uint32_t i = 0; i < kS6Per; ++i) {
                const uint32_t q = min(tid + kS6Threads * i, cn - 1);
                const uint32_t gp = c0 + q;
                const uint32_t lo = s_own[q];       // s_pre[lo] <= gp < s_pre[lo + 1]
                const uint32_t k = gp - s_pre[lo];
                hl[i] = lo | (k == 0 ? kFirst : 0u) | (gp + 1 == s_pre[lo + 1] ? kLast : 0u);
                idx[i] = s_beg[lo] + k;
            }
            SP_MARK(8);
            // (b) all loads of the chunk in flight together
            uint64_t now[kS6Per], prv[kS6Per];
            std::conditional_t<CH, uint64_t, uint32_t> rv[kS6Per];
            uint32_t dst[kS6Per], pay[kS6Per];
#pragma unroll
            for (uint32_t i = 0; i < kS6Per; ++i) {
                now[i] = a.send_time[idx[i]];
                prv[i] = a.send_time[idx[i] - ((hl[i] & kFirst) ? 0u : 1u)];
                dst[i] = a.dst_host[idx[i]];
                pay[i] = a.payload[idx[i]];
                if constexpr (CH) rv[i] = chance64[idx[i]];
                else rv[i] = draw[idx[i]];
            }
            SP_MARK(9);
            uint32_t dn[kS6Per];
            uint2 pg[kS6Per];   // (!MAP: the path entries, gathered together)
            if constexpr (!MAP) {
#pragma unroll
                for (uint32_t i = 0; i < kS6Per; ++i) dn[i] = a.host_node[min(dst[i], a.n_hosts - 1)];
#pragma unroll
                for (uint32_t i = 0; i < kS6Per; ++i)   // (unconditional: a select on `staged` made
                                                         // each a branch, waited at its join)
                    pg[i] = path_global(a.path, (size_t)s_node[hl[i] & kSlot] * a.n_nodes + dn[i]);
            }
            // (c) decisions
            uint8_t st[kS6Per];
            uint32_t doff[kS6Per];
#pragma unroll
            for (uint32_t i = 0; i < kS6Per; ++i) {
                const uint32_t pos = tid + kS6Threads * i;
                st[i] = kStSkipped;
                doff[i] = 0;
                if constexpr (MAP) dn[i] = 0;
                if (pos < cn) {
                    // a drawing send after a skipped one breaks K0's prefix rule
                    // (bitwise, not short-circuit: a `&&` chain let the compiler sink prv's load
                    // under the now[i] test -- a second, dependent memory round trip)
                    disorder |= !(hl[i] & kFirst) & (now[i] < a.sim_end) & !(prv[i] < a.sim_end);
                    if (dst[i] >= a.n_hosts) {      // "No host ID for dest address" (worker.rs:350-355)
                        atomicMin(&a.red[3], (unsigned long long)idx[i]);
                    } else if (now[i] < a.sim_end) {
                        uint2 pp;
                        if constexpr (MAP) {
                            dn[i] = packed_get(s_tbl, dst[i], bits);
                            pp = staged ? s_rows[s_rowof[hl[i] & kSlot] * a.n_nodes + dn[i]]
                                        : path_global(a.path, (size_t)s_node[hl[i] & kSlot] * a.n_nodes + dn[i]);
                        } else {
                            pp = pg[i];   // (no row staging without the LDS map: see `staged`)
                        }
                        const double reliability = (double)one_minus(__uint_as_float(pp.y));
                        bool tie = false;
                        const bool ge = CH ? __longlong_as_double((long long)rv[i]) >= reliability
                                           : draw_drops((uint32_t)rv[i], reliability, tie);
                        wide |= tie;   // a draw whose low bits would decide: redo the round on pipeline 1
                        if (!(now[i] < a.bootstrap_end) && ge && pay[i] > 0) {
                            st[i] = kStDropped;
                        } else {
                            uint64_t tt = now[i] + pp.x;
                            if (tt < a.round_end) tt = a.round_end;
                            const uint64_t dd = tt - a.round_end;
                            wide |= (dd >> 32) != 0;
                            min_d = tt < min_d ? tt : min_d;
                            min_l = pp.x < min_l ? pp.x : min_l;
                            doff[i] = (uint32_t)dd;
                            st[i] = kStSent;
                        }
                    }
                }
            }
            SP_MARK(10);
            // the chunk's event ids without a block scan: sent flags -> one ballot per (i, wave),
            // the 64 wave totals through LDS, and every wave scans those itself (one barrier).
            // Position order is pos = tid + kS6Threads * i: i-major, then wave, then lane.
            uint64_t sm[kS6Per];
#pragma unroll
            for (uint32_t i = 0; i < kS6Per; ++i) sm[i] = __ballot(st[i] == kStSent);
            if (lane == 0) {
#pragma unroll
                for (uint32_t i = 0; i < kS6Per; ++i) s_wt[i * kW + w] = (uint32_t)__popcll(sm[i]);
            }
            __syncthreads();
            SP_MARK(3);
            if (c0 == 0) {   // prefetch the next group's rows; they land while this group runs
                const uint32_t pn = s_pfn;
                if (MAP && pn && (uint64_t)pn * a.n_nodes <= kS5RowLds) {
#pragma unroll
                    for (uint32_t j = 0; j < kPf; ++j) {
                        const uint32_t e = tid + j * kS6Threads;
                        if (e < pn * a.n_nodes) {
                            const uint32_t rr = e / a.n_nodes, c = e - rr * a.n_nodes;
                            pf[j] = path_global(a.path, (size_t)s_pfnode[rr] * a.n_nodes + c);
                        }
                    }
                    have_pf = true;
                }
            }
            uint32_t pre[kS6Per];   // sent sends of the chunk before each own position
            {
                const uint32_t v = lane < kS6Per * kW ? s_wt[lane] : 0u;
                uint32_t incl = v;
#pragma unroll
                for (uint32_t o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(incl, o);
                    if (lane >= o) incl += y;
                }
                const uint32_t ex = incl - v;
#pragma unroll
                for (uint32_t i = 0; i < kS6Per; ++i)
                    pre[i] = (uint32_t)__shfl((int)ex, (int)(i * kW + w)) +
                             __builtin_amdgcn_mbcnt_hi((uint32_t)(sm[i] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm[i], 0u));
            }
            // a host's first position in the chunk (its first send, or the chunk's start) fixes the
            // offset of its ids in this chunk: id = s_off + pre
#pragma unroll
            for (uint32_t i = 0; i < kS6Per; ++i) {
                const uint32_t pos = tid + kS6Threads * i;
                const uint32_t h = hl[i] & kSlot;
                if (pos < cn && ((hl[i] & kFirst) || pos == 0)) s_off[h] = s_base[h] + s_run[h] - pre[i];
            }
            __syncthreads();
            SP_MARK(4);
            // stores: the ids, each record's slot in its bin (one LDS atomic), then every store; a
            // host's last position in the chunk carries its sent count into s_run
            uint32_t local[kS6Per], slot[kS6Per];
#pragma unroll
            for (uint32_t i = 0; i < kS6Per; ++i) {
                const uint32_t pos = tid + kS6Threads * i;
                local[i] = 0;
                slot[i] = 0;
                if (pos < cn) {
                    const uint32_t h = hl[i] & kSlot, so = s_off[h];
                    if (st[i] == kStSent) local[i] = so + pre[i];
                    if (BIN && dst[i] < a.n_hosts) {
                        uint32_t dl;
                        slot[i] = atomicAdd(&s_slot[dst_bin(a, dst[i], dl)], 1u);
                    }
                    if (pos == cn - 1 || (hl[i] & kLast))
                        s_run[h] = so + pre[i] + (st[i] == kStSent ? 1u : 0u) - s_base[h];
                }
            }
#pragma unroll
            for (uint32_t i = 0; i < kS6Per; ++i) {
                const uint32_t pos = tid + kS6Threads * i;
                if (pos < cn) {
#ifndef SHD_PRICE_STATUS   // (tuning builds: price the stamp's stores away; wrong output)
                    a.status[idx[i]] = st[i];
#endif
                    if (!BIN) {
                        a.key[idx[i]] = st[i] == kStSent ? dst[i] : a.n_hosts;
                        if (st[i] == kStSent) a.rec[idx[i]] = make_uint4(doff[i], s_host[hl[i] & kSlot], local[i], idx[i]);
                    } else if (dst[i] < a.n_hosts) {
                        uint32_t dl;
                        dst_bin(a, dst[i], dl);
#if defined(SHD_PRICE_REC) && SHD_PRICE_REC == 2
                        if (slot[i] == 0xFFFFFFFFu)   // never: the record store priced away
#elif defined(SHD_PRICE_REC)
                        slot[i] = idx[i];             // coalesced by packet index instead of the bin slot
#endif
                        a.rec[slot[i]] = make_uint4(doff[i],
                                                    s_host[hl[i] & kSlot] | (dl << 18) |
                                                        ((uint32_t)st[i] << 24),
                                                    local[i], idx[i]);
                    }
                    if (st[i] == kStSent && a.counts)
                        atomicAdd(&a.counts[(size_t)s_node[hl[i] & kSlot] * a.n_nodes + dn[i]], 1ull);
                }
            }
            if (c0 + kS6Cap < T) fill_owner(c0 + kS6Cap, nh);   // s_own of this chunk is consumed
            __syncthreads();
            SP_MARK(5);
        }
        if (tid < nh) {
            const size_t h = s_host[tid];
            if (a.chance || a.keep_rng)
                for (int k = 0; k < 4; ++k) a.rng_out[4 * h + k] = a.rng[4 * h + k];
            ns_total += s_run[tid];
            a.next_id_out[h] = a.next_id[h] + s_run[tid];
        }
    }
#ifdef SHD_STAMP_PROF
    SP_MARK(7);
    if (tid == 0)
        for (int q = 0; q < 12; ++q) atomicAdd(&g_stamp_prof[q], (unsigned long long)sp_acc[q]);
#endif
    min_d = wave_min_u64(min_d);
    min_l = wave_min_u64(min_l);
    for (int o = 32; o > 0; o >>= 1) ns_total += __shfl_xor(ns_total, o);
    const bool any_wide = __ballot(wide) != 0, any_disorder = __ballot(disorder) != 0;
#ifndef SHD_RED_PER_WAVE   // (tuning A/B: one set of global atomics per wave)
    // the workgroup's 16 waves combine in LDS first: one atomic per word per workgroup instead of
    // per wave -- the grid's waves all end together, and 4096 atomics on the same few words
    // serialise at the memory side (~12 ns each)
    __shared__ unsigned long long s_red[3][kS6Threads / 64];
    __shared__ uint32_t s_flag[kS6Threads / 64];
    if (lane == 0) {
        s_red[0][w] = min_d;
        s_red[1][w] = min_l;
        s_red[2][w] = ns_total;
        s_flag[w] = (any_wide ? 1u : 0u) | (any_disorder ? 2u : 0u);
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long md = ~0ull, ml = ~0ull, ns = 0;
        uint32_t fl = 0;
        for (uint32_t k = 0; k < kS6Threads / 64; ++k) {
            md = s_red[0][k] < md ? s_red[0][k] : md;
            ml = s_red[1][k] < ml ? s_red[1][k] : ml;
            ns += s_red[2][k];
            fl |= s_flag[k];
        }
        if (md != ~0ull) atomicMin(&a.red[0], md);
        if (ml != ~0ull) atomicMin(&a.red[1], ml);
        if (ns) atomicAdd(&a.red[2], ns);
        if (fl & 1u) atomicOr(&a.red[4], 1ull);
        if (fl & 2u) atomicOr(&a.red[5], 1ull);
    }
#else
    if (lane == 0) {
        if (min_d != ~0ull) atomicMin(&a.red[0], (unsigned long long)min_d);
        if (min_l != ~0ull) atomicMin(&a.red[1], (unsigned long long)min_l);
        if (ns_total) atomicAdd(&a.red[2], (unsigned long long)ns_total);
        if (any_wide) atomicOr(&a.red[4], 1ull);
        if (any_disorder) atomicOr(&a.red[5], 1ull);
    }
#endif
}

// the bit-packed host -> node map for relay_stamp_v6 (built at setup)
__global__ __launch_bounds__(256) void pack_host_node(const uint32_t* __restrict__ host_node,
                                                      uint32_t n_hosts, uint32_t bits,
                                                      uint32_t n_words, uint32_t* __restrict__ out) {
    const uint32_t wi = blockIdx.x * 256 + threadIdx.x;
    if (wi >= n_words) return;
    // word wi holds bits [32 wi, 32 wi + 32) of the concatenated entries
    const uint64_t b0 = (uint64_t)wi * 32;
    uint32_t word = 0;
    for (uint64_t j = b0 / bits; j < n_hosts && j * bits < b0 + 32; ++j) {
        const int64_t sh = (int64_t)(j * bits) - (int64_t)b0;
        const uint64_t v = host_node[j];
        word |= sh >= 0 ? (uint32_t)(v << sh) : (uint32_t)(v >> -sh);
    }
    out[wi] = word;
}

// pack the routing table for the narrow pipeline: one 8-byte gather per packet
__global__ __launch_bounds__(256) void pack_path(const uint64_t* __restrict__ lat,
                                                 const float* __restrict__ loss, uint64_t nn,
                                                 uint2* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < nn) out[i] = make_uint2((uint32_t)lat[i], __float_as_uint(loss[i]));
}

// ev_off[d] = first position of destination d in the sorted keys (lower bound), d in [0, H]
__global__ __launch_bounds__(256) void bucket_offsets(const uint32_t* __restrict__ key, uint64_t n,
                                                      uint32_t n_hosts, uint32_t* __restrict__ ev_off) {
    const uint32_t d = blockIdx.x * 256 + threadIdx.x;
    if (d > n_hosts) return;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t m = (lo + hi) >> 1;
        if (key[m] < d) lo = m + 1; else hi = m;
    }
    ev_off[d] = (uint32_t)lo;
}

__device__ __forceinline__ bool rec_less(const uint4& a, const uint4& b) {
    if (a.x != b.x) return a.x < b.x;     // deliver offset
    if (a.y != b.y) return a.y < b.y;     // src host
    return a.z < b.z;                     // event id offset
}

constexpr uint32_t kWaveSeg = 256;

// Sort one destination run held in LDS (xs[0..n), n <= kWaveSeg) by one wave; writes the sorted
// order as LDS positions pm[e] = base + position.  32-bit keys ((offset - min) << PB | position)
// when the run's deliver offsets leave room for PB position bits, else 64-bit keys.
template <int NPL, int PB>
__device__ __forceinline__ void wave_sort_perm(uint32_t n, uint32_t lane, const uint4* xs,
                                               uint32_t lo, uint32_t span, uint16_t* pm,
                                               uint32_t base) {
    if (span < (1u << (32 - PB)) - 1u) {
        uint32_t k[NPL];
#pragma unroll
        for (int c = 0; c < NPL; ++c) {
            const uint32_t e = lane + 64u * c;
            k[c] = e < n ? ((xs[e].x - lo) << PB) | e : ~0u;
        }
        wave_bitonic32<NPL>(k, lane);
#pragma unroll
        for (int c = 0; c < NPL; ++c) {
            const uint32_t e = lane + 64u * c;
            if (e < n) pm[e] = (uint16_t)(base + (k[c] & ((1u << PB) - 1u)));
        }
    } else {
        uint64_t k[NPL];
#pragma unroll
        for (int c = 0; c < NPL; ++c) {
            const uint32_t e = lane + 64u * c;
            k[c] = e < n ? (((uint64_t)xs[e].x << 32) | e) : ~0ull;
        }
        wave_bitonic<NPL>(k, lane);
#pragma unroll
        for (int c = 0; c < NPL; ++c) {
            const uint32_t e = lane + 64u * c;
            if (e < n) pm[e] = (uint16_t)(base + (uint32_t)k[c]);
        }
    }
}

__device__ __forceinline__ void wave_sort_run(uint32_t n, uint32_t lane, const uint4* xs,
                                              uint16_t* pm, uint32_t base) {
    uint32_t lo = ~0u, hi = 0;
    for (uint32_t e = lane; e < n; e += 64) {
        lo = min(lo, xs[e].x);
        hi = max(hi, xs[e].x);
    }
    lo = wave_min_u32(lo, lane);
    const uint32_t span = wave_max_u32(hi, lane) - lo;
    if (n <= 64) wave_sort_perm<1, 6>(n, lane, xs, lo, span, pm, base);
    else if (n <= 128) wave_sort_perm<2, 7>(n, lane, xs, lo, span, pm, base);
    else wave_sort_perm<4, 8>(n, lane, xs, lo, span, pm, base);
}

// K4: a workgroup owns kSegDst consecutive destinations; their runs are one contiguous range of
// the sorted records, so it is loaded and stored in bulk (coalesced) while each wave sorts whole
// runs in LDS.  Runs longer than kWaveSeg go to the merge kernel; a range larger than the LDS
// stage (only with such runs) is handled run by run.
constexpr uint32_t kSegDst = 8;
constexpr uint32_t kRunCap = 1536;

__global__ __launch_bounds__(256) void segment_sort_v5(
    uint32_t n_hosts, const uint32_t* __restrict__ ev_off, const uint4* __restrict__ brec,
    uint64_t round_end, const uint64_t* __restrict__ seq_base, uint64_t* __restrict__ ev_deliver,
    uint32_t* __restrict__ ev_src, uint64_t* __restrict__ ev_seq, uint32_t* __restrict__ ev_pkt,
    uint32_t* __restrict__ big) {
    __shared__ uint4 x[kRunCap];
    __shared__ uint16_t pm[kRunCap];
    __shared__ uint32_t off[kSegDst + 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t d0 = blockIdx.x * kSegDst;
    const uint32_t nd = min(kSegDst, n_hosts - d0);
    if (tid <= nd) off[tid] = ev_off[d0 + tid];
    __syncthreads();
    const uint32_t B = off[0], N = off[nd] - B;
    if (N > kRunCap) {   // run by run through a per-wave stage
        uint4* xw = x + w * kWaveSeg;
        uint16_t* pw = pm + w * kWaveSeg;
        for (uint32_t dl = w; dl < nd; dl += 4) {
            const uint32_t b = off[dl], n = off[dl + 1] - b;
            if (n == 0) continue;
            if (n > kWaveSeg) {
                if (lane == 0) big[atomicAdd(&big[0], 1u) + 1] = d0 + dl;
                continue;
            }
            for (uint32_t e = lane; e < n; e += 64) xw[e] = brec[b + e];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            wave_sort_run(n, lane, xw, pw, 0);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (uint32_t e = lane; e < n; e += 64) {
                const uint4 r = xw[pw[e]];
                ev_deliver[b + e] = round_end + r.x;
                ev_src[b + e] = r.y;
                ev_seq[b + e] = seq_base ? seq_base[r.y] + r.z : r.z;
                ev_pkt[b + e] = r.w;
            }
            __builtin_amdgcn_wave_barrier();
        }
        return;
    }
    for (uint32_t i = tid; i < N; i += 256) x[i] = brec[B + i];
    __syncthreads();
    for (uint32_t dl = w; dl < nd; dl += 4) {
        const uint32_t b = off[dl] - B, n = off[dl + 1] - off[dl];
        if (n == 0) continue;
        if (n > kWaveSeg) {   // the merge kernel writes this run; the bulk store skips it
            if (lane == 0) big[atomicAdd(&big[0], 1u) + 1] = d0 + dl;
            for (uint32_t e = lane; e < n; e += 64) pm[b + e] = 0xFFFFu;
            continue;
        }
        wave_sort_run(n, lane, x + b, pm + b, b);
    }
    __syncthreads();
    for (uint32_t i = tid; i < N; i += 256) {
        const uint32_t p = pm[i];
        if (p == 0xFFFFu) continue;
        const uint4 r = x[p];
        ev_deliver[B + i] = round_end + r.x;
        ev_src[B + i] = r.y;
        ev_seq[B + i] = seq_base ? seq_base[r.y] + r.z : r.z;
        ev_pkt[B + i] = r.w;
    }
}

// Runs longer than kWaveSeg: bottom-up merge passes by one workgroup in a
// global scratch copy of the bucket (rank by binary search in the sibling run; keys unique).
__global__ __launch_bounds__(256) void segment_sort_v2_big(
    const uint32_t* __restrict__ big, const uint32_t* __restrict__ ev_off, uint4* __restrict__ brec,
    uint4* __restrict__ tmp, uint64_t round_end, const uint64_t* __restrict__ seq_base,
    uint64_t* __restrict__ ev_deliver, uint32_t* __restrict__ ev_src, uint64_t* __restrict__ ev_seq,
    uint32_t* __restrict__ ev_pkt) {
    for (uint32_t bi = blockIdx.x; bi < big[0]; bi += gridDim.x) {
        const uint32_t d = big[1 + bi];
        const uint32_t b = ev_off[d], n = ev_off[d + 1] - b;
        uint4* A = brec + b;
        uint4* T = tmp + b;
        for (uint32_t w = 1; w < n; w <<= 1) {
            for (uint32_t o = threadIdx.x; o < n; o += 256) {
                const uint32_t lo = (o / (2 * w)) * 2 * w;
                const uint32_t mid = min(lo + w, n), hi = min(lo + 2 * w, n);
                const uint4 xv = A[o];
                uint32_t rank;
                if (o < mid) {
                    uint32_t l = mid, h = hi;
                    while (l < h) {
                        const uint32_t m = (l + h) >> 1;
                        if (rec_less(A[m], xv)) l = m + 1; else h = m;
                    }
                    rank = (o - lo) + (l - mid);
                } else {
                    uint32_t l = lo, h = mid;
                    while (l < h) {
                        const uint32_t m = (l + h) >> 1;
                        if (rec_less(xv, A[m])) h = m; else l = m + 1;
                    }
                    rank = (o - mid) + (l - lo);
                }
                T[lo + rank] = xv;
            }
            __syncthreads();
            for (uint32_t o = threadIdx.x; o < n; o += 256) A[o] = T[o];
            __syncthreads();
        }
        for (uint32_t i = threadIdx.x; i < n; i += 256) {
            const uint4 e = A[i];
            ev_deliver[b + i] = round_end + e.x;
            ev_src[b + i] = e.y;
            ev_seq[b + i] = seq_base ? seq_base[e.y] + e.z : e.z;
            ev_pkt[b + i] = e.w;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// Multi-GPU receive side: k-way merge of per-sender runs.  The input is n_runs chunks laid end
// to end; chunk r holds its events grouped by destination (local offsets off[r][0..n_dst]) and
// each destination's run sorted in EventQueue order.  Senders own disjoint source-host ranges,
// so the merged order is again (deliver, src, seq): every event finds its output rank by a
// binary search in each sibling run (keys are unique) -- no atomics, deterministic.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ bool ev3_less(uint64_t ta, uint32_t sa, uint64_t qa, uint64_t tb,
                                         uint32_t sb, uint64_t qb) {
    if (ta != tb) return ta < tb;
    if (sa != sb) return sa < sb;
    return qa < qb;
}

__global__ __launch_bounds__(256) void merge_offsets(uint32_t n_runs, uint32_t n_dst,
                                                     const uint32_t* __restrict__ off,
                                                     uint32_t* __restrict__ out_off) {
    const uint32_t d = blockIdx.x * 256 + threadIdx.x;
    if (d > n_dst) return;
    uint32_t t = 0;
    for (uint32_t r = 0; r < n_runs; ++r) t += off[(size_t)r * (n_dst + 1) + d] - off[(size_t)r * (n_dst + 1)];
    out_off[d] = t;
}

__global__ void max_u64_kernel(const uint64_t* __restrict__ d, uint64_t n,
                               unsigned long long* __restrict__ out) {
    uint64_t m = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        m = d[i] > m ? d[i] : m;
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(m, o);
        m = w > m ? w : m;
    }
    // one atomic per workgroup: 4 waves per block on one address contend (97 us for 8 MB)
    __shared__ uint64_t part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; w++) m = part[w] > m ? part[w] : m;
        atomicMax(out, (unsigned long long)m);
    }
}

__global__ void min_u64_kernel(const uint64_t* __restrict__ d, uint64_t n,
                               unsigned long long* __restrict__ out) {
    uint64_t m = ~0ull;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        m = d[i] < m ? d[i] : m;
    m = wave_min_u64(m);
    __shared__ uint64_t part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; w++) m = part[w] < m ? part[w] : m;
        atomicMin(out, (unsigned long long)m);
    }
}

shd_status min_u64_device(shd_ctx* ctx, const uint64_t* d, uint64_t n, uint64_t* out) {
    SHD_TRY(ctx->g_aux.ensure(8));
    SHD_HIP(hipMemsetAsync(ctx->g_aux.p, 0xFF, 8, ctx->stream));
    const uint32_t grid = (uint32_t)std::min<uint64_t>(1024, (n + 255) / 256);
    min_u64_kernel<<<grid ? grid : 1, 256, 0, ctx->stream>>>(
        d, n, reinterpret_cast<unsigned long long*>(ctx->g_aux.p));
    SHD_HIP(hipMemcpyAsync(out, ctx->g_aux.p, 8, hipMemcpyDeviceToHost, ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    return SHD_OK;
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
// v1 pipeline: u64 deliver times (used when a path latency or deliver offset needs > 32 bits)
static shd_status relay_device_v1(shd_ctx* ctx, const shd_batch* b, const shd_round* rd,
                                  shd_relay_out* o) {
    RelayState& R = ctx->relay;
    hipStream_t s = ctx->stream;
    const uint64_t n = b->n_packets;
    const uint32_t H = R.n_hosts;
    SHD_TRY(R.ev_key.ensure(std::max<uint64_t>(n, 1) * 8));   // deliver per packet
    SHD_TRY(R.ev_key2.ensure(std::max<uint64_t>(n, 1) * 8));  // seq per packet
    SHD_TRY(R.ev_val.ensure(std::max<uint64_t>(n, 1) * 4));   // slot per packet
    unsigned long long init[8] = {~0ull, ~0ull, 0ull, ~0ull, 0ull, 0ull, 0ull, 0ull};
    SHD_HIP(hipMemcpyAsync(R.red.p, init, sizeof(init), hipMemcpyHostToDevice, s));
    SHD_HIP(hipMemsetAsync(R.dst_cnt.p, 0, (size_t)(H + 1) * 4, s));
    RelayArgs a{};
    a.n_hosts = H;
    a.n_nodes = R.n_nodes;
    a.src_lo = R.src_lo;
    a.n_src = R.n_src;
    a.src_off = b->src_off;
    a.send_time = b->send_time;
    a.dst_host = b->dst_host;
    a.payload = b->payload;
    a.chance = b->chance;
    a.draw_cpu = R.cpu_draws ? R.draws.as<uint32_t>() : nullptr;
    a.host_node = R.host_node.as<uint32_t>();
    a.lat = R.own_table ? R.lat.as<uint64_t>() : ctx->t_lat.as<uint64_t>();
    a.loss = R.own_table ? R.loss.as<float>() : ctx->t_loss.as<float>();
    a.rng = R.rng.as<uint64_t>();
    a.next_id = R.next_id.as<uint64_t>();
    a.rng_out = R.rng2.as<uint64_t>();
    a.next_id_out = R.next_id2.as<uint64_t>();
    a.counts = R.count_on ? R.counts_round.as<unsigned long long>() : nullptr;
    a.round_end = rd->round_end;
    a.sim_end = rd->sim_end;
    a.bootstrap_end = rd->bootstrap_end;
    a.status = o->status;
    a.deliver = R.ev_key.as<uint64_t>();
    a.seq = R.ev_key2.as<uint64_t>();
    a.slot = R.ev_val.as<uint32_t>();
    a.dst_cnt = R.dst_cnt.as<uint32_t>();
    a.red = R.red.as<unsigned long long>();
    relay_stamp<<<div_up(std::max<uint32_t>(R.n_src, 1), 256), 256, 0, s>>>(a);
    SHD_HIP(hipGetLastError());
    // destination offsets: one hand-written look-back scan launch (scan.h); ev_off must be
    // 16-byte aligned (the relay's own buffers are; a caller's device array from hipMalloc too)
    SHD_TRY(scan_excl2(R.scan, R.dst_cnt.as<uint32_t>(), o->ev_off, nullptr, nullptr, (uint64_t)H + 1, s));
    if (n)
        relay_scatter<<<div_up(n, 256), 256, 0, s>>>(n, R.n_src, R.src_lo, b->src_off, o->status, b->dst_host,
                                                     R.ev_val.as<uint32_t>(), R.ev_key.as<uint64_t>(),
                                                     R.ev_key2.as<uint64_t>(), o->ev_off, o->ev_deliver,
                                                     o->ev_src, o->ev_seq, o->ev_pkt);
    SHD_TRY(R.ev_val2.ensure((size_t)(H + 2) * 4));
    SHD_HIP(hipMemsetAsync(R.ev_val2.p, 0, 4, s));
    segment_sort<<<H, 256, 0, s>>>(H, o->ev_off, o->ev_deliver, o->ev_src, o->ev_seq, o->ev_pkt,
                                   R.ev_val2.as<uint32_t>());
    SHD_HIP(hipGetLastError());
    uint32_t n_big = 0;
    SHD_HIP(hipMemcpyAsync(&n_big, R.ev_val2.p, 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipMemcpyAsync(R.red_host, R.red.p, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    if (n_big) {
        SHD_TRY(R.tmp.ensure(std::max<uint64_t>(n, 1) * sizeof(EvKey)));
        segment_sort_big<<<n_big, 256, 0, s>>>(R.ev_val2.as<uint32_t>(), o->ev_off, o->ev_deliver,
                                               o->ev_src, o->ev_seq, o->ev_pkt, R.tmp.as<EvKey>());
        SHD_HIP(hipGetLastError());
        SHD_HIP(hipStreamSynchronize(s));
    }
    return SHD_OK;
}


// ==========================================================================================
// Pipeline v7: destination-bin placement instead of a radix sort.  The stamp writes every
// packet's record straight into its destination bin (kBinDst destinations); the slots of a
// (stamp workgroup, bin) pair are counted beforehand by relay_bin_hist, which walks exactly the
// packets that workgroup will stamp.  bin_sort_v7 then loads one bin into LDS, drops the unsent
// records, splits the rest by destination and sorts each destination's run by
// (deliver, packet index) -- packet-index order is (src host, event id) order, the EventQueue
// tie-break -- so the slot order inside a bin never shows in the output.  Global traffic: the
// stamp's 16-byte record write plus one coalesced read of it, instead of two radix passes.
// ==========================================================================================
constexpr uint32_t kV7MaxHosts = 1u << 18;      // src host bits in the record
constexpr uint32_t kV7MaxPackets = 1u << 24;    // packet-index bits in bin_sort_v7's key
#ifndef SHD_B7_THREADS
#define SHD_B7_THREADS 512
#endif
constexpr uint32_t kB7Threads = SHD_B7_THREADS;
constexpr uint32_t kB7Cap = 3584;               // records per bin staged in LDS (C5: ~3200)
constexpr uint32_t kB7Per = (kB7Cap + kB7Threads - 1) / kB7Threads;
constexpr unsigned long long kLbAgg = 1ull << 62, kLbIncl = 2ull << 62, kLbMask = (1ull << 62) - 1;

// Histogram row r = g * kHistSplit + k counts, per destination bin, the packets of the host
// groups g + (k + j * kHistSplit) * G (j = 0, 1, ...) -- together the rows g * kHistSplit + k
// cover exactly the groups the stamp's workgroup g walks, every packet with a valid
// destination.  The rows' exclusive prefix at row g * kHistSplit is that workgroup's segment
// start.  A group's packet positions are flattened over the workgroup (owner by binary search
// in the 64-entry prefix) with kHistUnroll independent loads in flight per thread.
constexpr uint32_t kHistUnroll = 8;

__global__ __launch_bounds__(256) void relay_bin_hist(RelayArgs3 a, uint32_t G, uint32_t* __restrict__ cnt) {
    extern __shared__ uint32_t s_cnt[];
    __shared__ uint32_t s_beg[kS5Hosts], s_pre[kS5Hosts + 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    if (blockIdx.x == 0 && tid < 8) a.red[tid] = (tid <= 1 || tid == 3) ? ~0ull : 0ull;   // as red_init
    const uint32_t g = blockIdx.x / kHistSplit, k = blockIdx.x % kHistSplit;
    for (uint32_t i = tid; i < a.n_bins; i += 256) s_cnt[i] = 0;
    const uint32_t n_groups = (a.n_src + a.gs - 1) / a.gs;
    for (uint32_t grp = g + k * G; grp < n_groups; grp += kHistSplit * G) {
        const uint32_t h0 = grp * a.gs, nh = min(a.gs, a.n_src - h0);
        __syncthreads();
        if (tid < 64) {
            uint32_t len = 0;
            if (tid < nh) {
                const uint32_t h = a.order[h0 + tid];
                s_beg[tid] = a.src_off[h - a.src_lo];
                len = a.src_off[h - a.src_lo + 1] - s_beg[tid];
            }
            uint32_t incl = len;
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            if (tid < nh) s_pre[tid + 1] = incl;
            if (tid == 0) s_pre[0] = 0;
        }
        __syncthreads();
        const uint32_t T = s_pre[nh];
        for (uint32_t base = 0; base < T; base += 256 * kHistUnroll) {
            uint32_t d[kHistUnroll];
#pragma unroll
            for (uint32_t u = 0; u < kHistUnroll; ++u) {
                const uint32_t p = base + u * 256 + tid;
                d[u] = ~0u;
                if (p < T) {
                    uint32_t lo = 0, hi = nh;   // s_pre[lo] <= p < s_pre[lo + 1]
                    while (hi - lo > 1) {
                        const uint32_t m = (lo + hi) >> 1;
                        if (s_pre[m] <= p) lo = m; else hi = m;
                    }
                    d[u] = a.dst_host[s_beg[lo] + (p - s_pre[lo])];
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < kHistUnroll; ++u)
                if (d[u] < a.n_hosts) {
                    uint32_t dl;
                    atomicAdd(&s_cnt[dst_bin(a, d[u], dl)], 1u);
                }
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < a.n_bins; i += 256) cnt[(size_t)blockIdx.x * a.n_bins + i] = s_cnt[i];
}

// relay_bin_hist, vector form (the batch's dst_host 16-byte aligned): the same rows, but four
// threads per host of a group walk the host's own range in aligned 16-byte chunks (chunk c =
// destinations [4c, 4c + 4), entries outside the host's range skipped), so no position needs a
// search for its owner and each load brings four destinations.  Chunks reaching past the batch
// end are read element by element.
constexpr uint32_t kHist4Threads = 1024;   // four groups at a time: 4 threads x 64 host slots each

__global__ __launch_bounds__(kHist4Threads) void relay_bin_hist4(RelayArgs3 a, uint32_t G, uint32_t n_pkt,
                                                                 uint32_t* __restrict__ cnt) {
    extern __shared__ uint32_t s_cnt[];
    const uint32_t tid = threadIdx.x, hs = (tid >> 2) & 63, qq = tid & 3;
    const uint32_t g = blockIdx.x / kHistSplit, k = blockIdx.x % kHistSplit;
    if (blockIdx.x == 0 && tid < 8) a.red[tid] = (tid <= 1 || tid == 3) ? ~0ull : 0ull;   // as red_init
    for (uint32_t i = tid; i < a.n_bins; i += kHist4Threads) s_cnt[i] = 0;
    __syncthreads();
    const uint32_t n_groups = (a.n_src + a.gs - 1) / a.gs;
    const uint32_t full = n_pkt & ~3u;   // chunks below this lie inside the batch
    for (uint32_t grp = g + (k + (tid >> 8) * kHistSplit) * G; grp < n_groups; grp += 4 * kHistSplit * G) {
        const uint32_t h0 = grp * a.gs, nh = min(a.gs, a.n_src - h0);
        if (hs >= nh) continue;
        const uint32_t h = a.order[h0 + hs];
        const uint32_t b = a.src_off[h - a.src_lo], e = a.src_off[h - a.src_lo + 1];
#ifndef SHD_HIST_UNROLL
#define SHD_HIST_UNROLL 4   // (C5 histogram 49.9 -> 41.1 us; 1 and 2 for A/B builds)
#endif
        // HU chunks per thread per step, their loads in flight together (a C5 host's ~100 sends
        // are ~6 chunks per thread: one dependent load after another at HU = 1)
        constexpr uint32_t HU = SHD_HIST_UNROLL;
        for (uint32_t c0 = (b >> 2) + qq; 4 * c0 < e; c0 += 4 * HU) {
            uint32_t d[HU][4];
#pragma unroll
            for (uint32_t j = 0; j < HU; ++j) {
                const uint32_t c = c0 + 4 * j;
                if (4 * c >= e) {
                    d[j][0] = d[j][1] = d[j][2] = d[j][3] = ~0u;
                } else if (4 * c + 4 <= full) {
                    const uint4 v = reinterpret_cast<const uint4*>(a.dst_host)[c];
                    d[j][0] = v.x; d[j][1] = v.y; d[j][2] = v.z; d[j][3] = v.w;
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) d[j][u] = 4 * c + u < n_pkt ? a.dst_host[4 * c + u] : ~0u;
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < HU; ++j)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t i = 4 * (c0 + 4 * j) + u;
                    if (i >= b && i < e && d[j][u] < a.n_hosts) {
                        uint32_t dl;
                        atomicAdd(&s_cnt[dst_bin(a, d[j][u], dl)], 1u);
                    }
                }
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < a.n_bins; i += kHist4Threads) cnt[(size_t)blockIdx.x * a.n_bins + i] = s_cnt[i];
}

// seg[g][b] = number of bin-b slots of stamp workgroups before g (the sum of kHistSplit
// histogram rows per workgroup, exclusive prefix over g); tot[b] = all of bin b.  Lane = bin,
// wave = a slice of workgroups; every row load of a slice is independent.  A workgroup count
// (the stamp's slot counters are 32-bit since round 6: no workgroup count overflows them).
constexpr uint32_t kColMaxG = 256;   // stamp workgroups (one per CU)

// (base != nullptr: bin_base_scan folded in -- each block's 64 bin totals, a wave scan, and a
// decoupled look-back over the earlier blocks (blockIdx order: at most 128 blocks, all resident)
// give the bins' record bases; the look-back states carry an epoch (scan.h layout), so they are
// never cleared.  One launch and one queue gap less per round.)
__global__ __launch_bounds__(1024) void bin_col_scan(uint32_t G, uint32_t n_bins, const uint32_t* __restrict__ cnt,
                                                     uint32_t* __restrict__ seg, uint32_t* __restrict__ tot,
                                                     unsigned long long* __restrict__ red,
                                                     uint32_t* __restrict__ base = nullptr,
                                                     unsigned long long* __restrict__ lb = nullptr,
                                                     unsigned long long* __restrict__ state = nullptr,
                                                     uint32_t epoch = 0) {
    __shared__ uint32_t s[16][64];
    constexpr uint32_t kPer = kColMaxG / 16;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, b = blockIdx.x * 64 + lane;
    const uint32_t g0 = min(G, w * kPer), g1 = min(G, g0 + kPer);
    uint32_t c[kPer];
    uint32_t sum = 0;
    // every row load unconditional (indices clamped, values masked) so all of them are in flight
    // together instead of one guarded load at a time
    const uint32_t bc = min(b, n_bins - 1);
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
        const uint32_t g = min(g0 + i, G - 1);
        c[i] = 0;
#pragma unroll
        for (uint32_t k = 0; k < kHistSplit; ++k) c[i] += cnt[((size_t)g * kHistSplit + k) * n_bins + bc];
    }
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
        if (!(g0 + i < g1 && b < n_bins)) c[i] = 0;
        sum += c[i];
    }
    s[w][lane] = sum;
    __syncthreads();
    uint32_t run = 0;
    for (uint32_t u = 0; u < w; ++u) run += s[u][lane];
    if (b < n_bins) {
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const uint32_t g = g0 + i;
            if (g < g1) seg[(size_t)g * n_bins + b] = run;
            run += c[i];
        }
        if (w == 15) tot[b] = run;
    }
    if (base && w == 15) {   // wave 15 holds the 64 bin totals of this block
        const uint32_t t = b < n_bins ? run : 0u;
        if (t > kB7Cap) atomicOr(&red[6], 1ull);
        uint32_t incl = t;
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const uint32_t agg = __shfl(incl, 63);
        const unsigned long long tag = (unsigned long long)epoch << 34;
        unsigned long long* st = state + 2 + (size_t)blockIdx.x * 2;
        uint32_t excl = 0;
        if (blockIdx.x != 0) {
            if (lane == 0) __hip_atomic_store(st, tag | (1ull << 32) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int64_t hi = (int64_t)blockIdx.x - 1;;) {   // 64 earlier blocks a step
                const int64_t j = hi - (int64_t)lane;
                const unsigned long long v =
                    j >= 0 ? __hip_atomic_load(&state[2 + (size_t)j * 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : tag | (2ull << 32);   // before block 0: an inclusive 0
                const uint32_t f = (uint32_t)(v >> 32) & 3u;
                const bool ok = (uint32_t)(v >> 34) == epoch && f != 0;
                const uint64_t incl_m = __ballot(ok && f == 2), bad_m = __ballot(!ok);
                const uint32_t fi = incl_m ? (uint32_t)__builtin_ctzll(incl_m) : 64u;
                const uint64_t upto = fi == 64 ? ~0ull : ((2ull << fi) - 1ull);
                if (bad_m & upto) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint32_t add = lane <= fi ? (uint32_t)v : 0u;
                for (int o = 32; o > 0; o >>= 1) add += __shfl_xor(add, o);
                excl += add;
                if (fi < 64) break;
                hi -= 64;
            }
        }
        if (lane == 0) __hip_atomic_store(st, tag | (2ull << 32) | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (b < n_bins) {
            base[b] = excl + incl - t;
            lb[b] = 0;   // bin_sort_v7's look-back states
        }
        if (b == n_bins - 1) {
            base[n_bins] = excl + incl;
            lb[n_bins] = 0;   // its ticket
        }
    }
}

// one workgroup: bin_base = exclusive scan of tot (bin_base[n_bins] = total); clears the
// look-back states and the ticket of bin_sort_v7; a bin larger than its LDS stage flags red[6]
__global__ __launch_bounds__(1024) void bin_base_scan(uint32_t n_bins, const uint32_t* __restrict__ tot,
                                                      uint32_t* __restrict__ base,
                                                      unsigned long long* __restrict__ lb,
                                                      unsigned long long* __restrict__ red) {
    __shared__ uint32_t s_w[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t per = (n_bins + 1023) / 1024, b0 = min(n_bins, tid * per), b1 = min(n_bins, b0 + per);
    uint32_t sum = 0;
    bool over = false;
    for (uint32_t b = b0; b < b1; ++b) {
        sum += tot[b];
        over |= tot[b] > kB7Cap;
    }
    if (over) atomicOr(&red[6], 1ull);
    uint32_t incl = sum;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (uint32_t u = 0; u < w; ++u) run += s_w[u];
    for (uint32_t b = b0; b < b1; ++b) {
        base[b] = run;
        run += tot[b];
    }
    if (tid == 1023) base[n_bins] = run;
    for (uint32_t b = tid; b <= n_bins; b += 1024) lb[b] = 0;   // lb[n_bins]: the ticket
}

// 64-bit wave bitonic (element e = lane + 64 c), lane exchanges through xor_lane on both halves
template <int NPL>
__device__ __forceinline__ void wave_bitonic64(uint64_t (&k)[NPL], uint32_t lane) {
#pragma unroll
    for (uint32_t kk = 2; kk <= 64u * NPL; kk <<= 1) {
#pragma unroll
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
                const uint32_t cj = j / 64;
#pragma unroll
                for (int c = 0; c < NPL; ++c) {
                    if ((c & cj) == 0) {
                        const bool asc = ((lane + 64u * c) & kk) == 0;
                        const uint64_t x = k[c], y = k[c | cj];
                        const bool sw = (y < x) == asc;   // unique keys
                        k[c] = sw ? y : x;
                        k[c | cj] = sw ? x : y;
                    }
                }
            } else {
#pragma unroll
                for (int c = 0; c < NPL; ++c) {
                    const uint32_t lo = xor_lane((uint32_t)k[c], j, lane);
                    const uint32_t hi = xor_lane((uint32_t)(k[c] >> 32), j, lane);
                    const uint64_t o = ((uint64_t)hi << 32) | lo;
                    // keys are unique: take the partner's key iff it is smaller where this lane
                    // keeps the minimum (one 64-bit compare, one select)
                    const bool take_min = ((lane & j) == 0) == (((lane + 64u * c) & kk) == 0);
                    k[c] = (o < k[c]) == take_min ? o : k[c];
                }
            }
        }
    }
}

struct V7Out {
    uint64_t* deliver;
    uint32_t* src;
    uint64_t* seq;
    uint32_t* pkt;
    const uint64_t* seq_base;
    uint64_t round_end;
    // a flush round (shd_relay_flush, one context): the compact event records instead of the
    // arrays -- {deliver - round_end, src, id relative to the source's first of the round (the
    // records hold relative ids then), send index in stage order = perm[packet]}, 16 or 12 bytes
    void* fl_out = nullptr;
    const uint32_t* fl_perm = nullptr;
    uint32_t fl_b12 = 0;
};

__device__ __forceinline__ void v7_emit(const V7Out& o, size_t at, const uint4& r) {
    const uint32_t src = r.y & (kV7MaxHosts - 1);
    if (o.fl_out) {
        const uint32_t send = o.fl_perm[r.w];
        if (o.fl_b12) {
            uint32_t* e = static_cast<uint32_t*>(o.fl_out) + 3 * at;
            e[0] = r.x;
            e[1] = r.z;
            e[2] = send;
        } else {
            static_cast<uint4*>(o.fl_out)[at] = make_uint4(r.x, src, r.z, send);
        }
        return;
    }
    o.deliver[at] = o.round_end + r.x;
    o.src[at] = src;
    o.seq[at] = o.seq_base ? o.seq_base[src] + r.z : r.z;
    o.pkt[at] = r.w;
}

// one destination run (bin slots ls[0..n), n <= 256) sorted by (deliver offset, packet index),
// key = (x - lo) << 32 | (pkt - pmin) << 8 | e  (pkt - pmin < 2^24, e < 256: unique); writes
// the run's order as slots: pm[rank] = slot
template <int NPL>
__device__ __forceinline__ void v7_sort_run(uint32_t n, uint32_t lane, const uint4* x, const uint16_t* ls,
                                            uint16_t* pm) {
    uint2 v[NPL];
    uint32_t lo = ~0u, pmin = ~0u;
#pragma unroll
    for (int c = 0; c < NPL; ++c) {
        const uint32_t e = lane + 64u * c;
        if (e < n) {
            const uint4 r = x[ls[e]];
            v[c] = make_uint2(r.x, r.w);
        } else {
            v[c] = make_uint2(~0u, ~0u);
        }
        lo = min(lo, v[c].x);
        pmin = min(pmin, v[c].y);
    }
    lo = wave_min_u32(lo, lane);
    pmin = wave_min_u32(pmin, lane);
    {   // 32-bit keys (deliver - lo) << 8 | e when the run's deliver times span < 2^24 ns: half the
        // lane exchanges and compares of the 64-bit network.  Equal deliver times would need the
        // packet order: a run with any is redone on the 64-bit keys below.
        uint32_t hi = 0;
#pragma unroll
        for (int c = 0; c < NPL; ++c)
            if (lane + 64u * c < n) hi = max(hi, v[c].x);
        hi = wave_max_u32(hi, lane);
        if (hi - lo < (1u << 24)) {
            uint32_t k32[NPL];
#pragma unroll
            for (int c = 0; c < NPL; ++c) {
                const uint32_t e = lane + 64u * c;
                k32[c] = e < n ? ((v[c].x - lo) << 8) | e : ~0u;
            }
            wave_bitonic32<NPL>(k32, lane);
            // sorted: element r = lane + 64 c; a tie is an equal upper 24 bits in neighbours r, r + 1
            bool tie = false;
#pragma unroll
            for (int c = 0; c < NPL; ++c) {
                // (both shuffles with every lane active: a read of an inactive lane returns 0)
                const uint32_t down = (uint32_t)__shfl_down((int)k32[c], 1);
                const uint32_t first = c + 1 < NPL ? (uint32_t)__shfl((int)k32[c + 1 < NPL ? c + 1 : c], 0) : ~0u;
                const uint32_t nx = lane == 63 ? first : down;
                const uint32_t r = lane + 64u * c;
                if (r + 1 < n && (nx >> 8) == (k32[c] >> 8)) tie = true;
            }
            if (__ballot(tie) == 0) {
#pragma unroll
                for (int c = 0; c < NPL; ++c) {
                    const uint32_t rank = lane + 64u * c;
                    if (rank < n) pm[rank] = ls[k32[c] & 0xFFu];
                }
                return;
            }
        }
    }
    uint64_t k[NPL];
#pragma unroll
    for (int c = 0; c < NPL; ++c) {
        const uint32_t e = lane + 64u * c;
        k[c] = e < n ? ((uint64_t)(v[c].x - lo) << 32) | ((uint64_t)(v[c].y - pmin) << 8) | e : ~0ull;
    }
    wave_bitonic64<NPL>(k, lane);
#pragma unroll
    for (int c = 0; c < NPL; ++c) {
        const uint32_t rank = lane + 64u * c;
        if (rank < n) pm[rank] = ls[(uint32_t)k[c] & 0xFFu];
    }
}

// K4 of a sharded round (relay_round_sharded_v7, X = true): bin j of this rank's own bins takes
// its records from every sender's received slice: sender q's records of the bin start at
// rbase[q] + sc[q * stride + fb + j] - sc[q * stride + fb] (sc: the senders' exclusive bin scans
// from the gathered sizing rows).  Packet indices are per sender; the sort key uses the global
// packet order (the senders' batches back to back, pbase[q] = packets of the senders before q),
// which is (src host, event id) order because the senders own increasing source ranges.
struct XSrc {
    uint32_t world, me, fb, stride, kq;
    const uint32_t* sc;
    const uint32_t* rbase;   // sender q's slice in the received records (q != me)
    const uint32_t* pbase;
    const uint4* own;        // this rank's own records stay where its stamp put them (never exchanged)
    const uint64_t* rst;     // [world] the status each sender carried into the exchange (own: own_st)
    uint32_t own_st;
};

// the round's agreed status from the exchange's status part: the lowest failing rank's
__device__ __forceinline__ uint32_t xs_status(const XSrc& xs) {
    for (uint32_t q = 0; q < xs.world; ++q) {
        const uint32_t v = q == xs.me ? xs.own_st : (uint32_t)xs.rst[q];
        if (v) return v;
    }
    return 0u;
}

// a rank without bins: no bin sort writes its event count and the agreed status
__global__ __launch_bounds__(64) void xs_fin_empty(XSrc xs, uint32_t* __restrict__ ev_off) {
    if (threadIdx.x == 0) {
        ev_off[0] = 0;
        ev_off[1] = xs_status(xs);
    }
}

// K4 (v7): one workgroup per bin, bins taken in ticket order so the event offsets can use a
// decoupled look-back (publish the bin's sent count, add the predecessors' counts).  The bin's
// records are staged in LDS, grouped by destination, each run sorted by one wave into the
// bin's output order, and the bin's events stored in that order (coalesced).
template <bool X>
__global__ __launch_bounds__(kB7Threads) void bin_sort_v7(uint32_t n_hosts, uint32_t n_bins,
                                                          const uint32_t* __restrict__ bin_base,
                                                          const uint4* __restrict__ rec,
                                                          unsigned long long* __restrict__ lb,
                                                          uint32_t* __restrict__ ev_off, V7Out o,
                                                          const unsigned long long* __restrict__ red,
                                                          uint32_t stop,   // tuning: stop after phase
                                                          XSrc xs) {
    __shared__ uint4 x[kB7Cap];
    __shared__ uint16_t ls[kB7Cap], pm[kB7Cap];
    __shared__ uint32_t s_cnt[kBinDst], s_off[kBinDst + 1], s_cur[kBinDst], s_bin, s_excl;
    __shared__ uint32_t s_pb[X ? 64 : 1];
    // (X: the own sender's records are read from xs.own, every other sender's from rec)
    if (!X && red[6]) return;   // overflow: the host reruns the round on v3
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_bin = atomicAdd(reinterpret_cast<unsigned int*>(&lb[n_bins]), 1u);
    if (tid < kBinDst) s_cnt[tid] = s_cur[tid] = 0;
    __syncthreads();
    const uint32_t bin = s_bin;
    uint32_t B = 0, N = 0;
    // X: every wave reads the senders' segments of the bin itself (lane q: sender q) and keeps
    // them in registers, so no wave waits at a barrier for another's loads before its record
    // loads (measured the same as a wave-0 table in LDS behind a barrier: the X form's extra
    // ~25 us over bin_sort_v7<false> at world size 1 is its look-back phase, +13 us, and the
    // loads, +6 us; tools/r06_b7x_phases.sh)
    uint32_t x_at = 0, x_pre = 0, x_pb = 0;
    if constexpr (X) {
        uint32_t c = 0;
        if (lane < xs.world) {
            const uint32_t* sq = xs.sc + (size_t)lane * xs.stride + xs.fb;
            const uint32_t a0 = sq[0], a1 = sq[bin], a2 = sq[bin + 1];
            x_at = lane == xs.me ? a1 : xs.rbase[lane] + (a1 - a0);
            c = a2 - a1;
            x_pb = xs.pbase[lane];
        }
        uint32_t incl = c;
        for (uint32_t q = 1; q < 64; q <<= 1) {
            const uint32_t y = __shfl_up(incl, q);
            if (lane >= q) incl += y;
        }
        x_pre = incl - c;
        if (w == 0) s_pb[lane] = x_pb;   // (read by the emit, behind later barriers)
        N = __shfl(incl, xs.world - 1);   // <= kB7Cap: the host checked every bin's total before the exchange
    } else {
        B = bin_base[bin];
        N = bin_base[bin + 1] - B;
    }
    {   // every load of the bin in flight at once (N <= kB7Cap)
        uint4 r[kB7Per];
        uint32_t qs[kB7Per], pbq[kB7Per];   // X: each record's sender and its packet base
#pragma unroll
        for (uint32_t u = 0; u < kB7Per; ++u) {
            const uint32_t i = tid + u * kB7Threads;
            if constexpr (X) {
                // (the shuffles run on every lane, outside the i < N guard: a bpermute must not
                // read a lane that skipped the computation)
                uint32_t q = 0;   // the sender of staged index i: the last q with pre[q] <= i
                for (uint32_t k = xs.kq; k > 0; k >>= 1) {   // (kq: the largest power of two < world)
                    const uint32_t pk = (uint32_t)__shfl((int)x_pre, (int)min(q + k, xs.world - 1));
                    if (q + k < xs.world && pk <= i) q += k;
                }
                const uint32_t at = (uint32_t)__shfl((int)x_at, (int)q), pre = (uint32_t)__shfl((int)x_pre, (int)q);
                qs[u] = q;
                pbq[u] = (uint32_t)__shfl((int)x_pb, (int)q);
                if (i < N) r[u] = (q == xs.me ? xs.own : rec)[at + (i - pre)];
            } else {
                if (i < N) r[u] = rec[B + i];
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < kB7Per; ++u) {
            const uint32_t i = tid + u * kB7Threads;
            if (i < N) {
                if constexpr (X) {
                    r[u].w += pbq[u];          // global packet order
                    r[u].y |= qs[u] << 26;     // the sender, for the packet index of the output
                }
                x[i] = r[u];
                if (((r[u].y >> 24) & 3u) == kStSent) atomicAdd(&s_cnt[(r[u].y >> 18) & (kBinDst - 1)], 1u);
            }
        }
    }
    __syncthreads();
    if (stop == 1) return;
    if (w == 0) {
        const uint32_t c = lane < kBinDst ? s_cnt[lane] : 0u;
        uint32_t incl = c;
        for (uint32_t q = 1; q < 64; q <<= 1) {
            const uint32_t y = __shfl_up(incl, q);
            if (lane >= q) incl += y;
        }
        if (lane <= kBinDst) s_off[lane] = incl - c;
        const uint32_t agg = __shfl(incl, 63);
        unsigned long long excl = 0;
        if (bin == 0) {
            if (lane == 0) __hip_atomic_store(&lb[0], kLbIncl | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(&lb[bin], kLbAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // look-back 64 predecessors at a time: lane l reads bin hi - l; the nearest inclusive
            // state ends the walk once every state up to it has been published (bin 0 always is)
            for (int32_t hi = (int32_t)bin - 1;;) {
                const int32_t j = hi - (int32_t)lane;
                const unsigned long long v =
                    j >= 0 ? __hip_atomic_load(&lb[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbIncl;
                const uint64_t incl_m = __ballot((v & kLbIncl) != 0), zero_m = __ballot(v == 0);
                const uint32_t fi = incl_m ? (uint32_t)__builtin_ctzll(incl_m) : 64u;
                const uint64_t upto = fi == 64 ? ~0ull : ((2ull << fi) - 1ull);
                if (zero_m & upto) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                unsigned long long add = lane <= fi ? (v & kLbMask) : 0ull;
                for (int q = 32; q > 0; q >>= 1) add += __shfl_xor(add, q);
                excl += add;
                if (fi < 64) break;
                hi -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&lb[bin], kLbIncl | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_excl = (uint32_t)excl;
    }
    __syncthreads();
    const uint32_t excl = s_excl, d0 = bin * kBinDst, S = s_off[kBinDst];
    if (tid < kBinDst && d0 + tid < n_hosts) ev_off[d0 + tid] = excl + s_off[tid];
    if (tid == 0 && bin == n_bins - 1) {
        ev_off[n_hosts] = excl + S;
        if constexpr (X) ev_off[n_hosts + 1] = xs_status(xs);   // (read back with the count)
    }
    if (stop == 2) return;
    for (uint32_t i = tid; i < N; i += kB7Threads) {
        const uint32_t y = x[i].y;
        if (((y >> 24) & 3u) == kStSent) {
            const uint32_t dl = (y >> 18) & (kBinDst - 1);
            ls[s_off[dl] + atomicAdd(&s_cur[dl], 1u)] = (uint16_t)i;
        }
    }
    __syncthreads();
    if (stop == 3) return;
    for (uint32_t dl = w; dl < kBinDst; dl += kB7Threads / 64) {
        const uint32_t b = s_off[dl], n = s_off[dl + 1] - b;
        if (n == 0) continue;
        if (n <= 64) v7_sort_run<1>(n, lane, x, ls + b, pm + b);
        else if (n <= 128) v7_sort_run<2>(n, lane, x, ls + b, pm + b);
        else if (n <= 256) v7_sort_run<4>(n, lane, x, ls + b, pm + b);
        else {   // long run (rare): rank = number of smaller (deliver, packet) keys
            for (uint32_t e = lane; e < n; e += 64) {
                const uint4 q0 = x[ls[b + e]];
                uint32_t rank = 0;
                for (uint32_t f = 0; f < n; ++f) {
                    const uint4 q = x[ls[b + f]];
                    rank += (q.x < q0.x || (q.x == q0.x && q.w < q0.w)) ? 1u : 0u;
                }
                pm[b + rank] = ls[b + e];
            }
        }
    }
    __syncthreads();
    if (stop == 4) return;
    for (uint32_t p = tid; p < S; p += kB7Threads) {
        uint4 r = x[pm[p]];
        if constexpr (X) {
            r.w -= s_pb[r.y >> 26];   // back to the index in the sender's batch
            r.y &= kV7MaxHosts - 1;
        }
        v7_emit(o, (size_t)excl + p, r);
    }
}

// Narrow pipeline: K1 stamp, K2 radix sort by destination, K3 offsets, K4 per-run sort; one
// host sync (for the round reductions).
// the round's reductions: [0] min deliver, [1] min latency, [2] sent, [3] first bad index,
// [4] wide offset, [5] send-order violation; plus the big-run counter of K4
__global__ __launch_bounds__(64) void red_init(unsigned long long* __restrict__ red, uint32_t* __restrict__ n_big) {
    const uint32_t t = threadIdx.x;
    if (t < 8) red[t] = (t <= 1 || t == 3) ? ~0ull : 0ull;
    if (t == 0) *n_big = 0;
}

static RelayArgs3 relay_args3(shd_ctx* ctx, const shd_batch* b, const shd_round* rd, shd_relay_out* o) {
    RelayState& R = ctx->relay;
    const uint64_t n = b->n_packets;
    const uint32_t H = R.n_hosts;
    RelayArgs3 a{};
    a.gs = kS5Hosts;
    a.n_hosts = H;
    a.n_nodes = R.n_nodes;
    a.src_lo = R.src_lo;
    a.n_src = R.n_src;
    a.src_off = b->src_off;
    a.send_time = b->send_time;
    a.dst_host = b->dst_host;
    a.payload = b->payload;
    a.chance = b->chance;
    a.keep_rng = R.cpu_draws ? 1u : 0u;
    a.host_node = R.host_node.as<uint32_t>();
    a.path = R.path.as<uint2>();
    a.order = R.order.as<uint32_t>();
    a.rng = R.rng.as<uint64_t>();
    a.next_id = R.next_id.as<uint64_t>();
    a.rng_out = R.rng2.as<uint64_t>();
    a.next_id_out = R.next_id2.as<uint64_t>();
    a.counts = R.count_on ? R.counts_round.as<unsigned long long>() : nullptr;
    a.round_end = rd->round_end;
    a.sim_end = rd->sim_end;
    a.bootstrap_end = rd->bootstrap_end;
    // event ids below 2^32 for the whole round: records carry absolute ids, no per-event gather
    // (rel_ids: records keep the id relative to the host's first of the round)
    a.abs_seq = !R.rel_ids && R.seq_bound + n < (1ull << 32) ? 1u : 0u;
    a.status = o->status;
    a.rec = R.rec.as<uint4>();
    a.key = R.ev_val.as<uint32_t>();
    a.red = R.red.as<unsigned long long>();
    return a;
}

static shd_status relay_device_v3(shd_ctx* ctx, const shd_batch* b, const shd_round* rd,
                                  shd_relay_out* o) {
    RelayState& R = ctx->relay;
    hipStream_t s = ctx->stream;
    const uint64_t n = b->n_packets;
    const uint32_t H = R.n_hosts;
    const size_t nn = std::max<uint64_t>(n, 1);
    SHD_TRY(R.rec.ensure(nn * 16));
    SHD_TRY(R.brec.ensure(nn * 16));
    SHD_TRY(R.ev_val.ensure(nn * 4));    // keys
    SHD_TRY(R.ev_key.ensure(nn * 4));    // keys (second buffer)
    SHD_TRY(R.ev_val2.ensure((size_t)(H + 2) * 4));
    SHD_TRY(R.draws.ensure(nn * 4));
    red_init<<<1, 64, 0, s>>>(R.red.as<unsigned long long>(), R.ev_val2.as<uint32_t>());
    RelayArgs3 a = relay_args3(ctx, b, rd, o);
    const uint64_t* seq_base = a.abs_seq ? nullptr : R.next_id.as<uint64_t>();
    if (!b->chance && !R.cpu_draws && R.n_src)   // K0: the per-host generator streams
        relay_draws<<<div_up(R.n_src, 64 * kK0Waves), 64 * kK0Waves, 0, s>>>(a, R.draws.as<uint32_t>());
    if (R.n_src == 0) {
    } else if (R.hn_bits) {   // host -> node map fits the LDS: persistent stamp, no node gathers
        const uint32_t groups = div_up(R.n_src, kS5Hosts);
        auto* k = a.chance ? &relay_stamp_v6<false, true> : &relay_stamp_v6<false, false>;
        k<<<std::min<uint32_t>(groups, (uint32_t)ctx->n_cu), kS6Threads, (size_t)R.hn_words * 4, s>>>(
            a, R.draws.as<uint32_t>(), R.hn_packed.as<uint32_t>(), R.hn_words, R.hn_bits);
    } else {
        (a.chance ? relay_stamp_v5<true> : relay_stamp_v5<false>)<<<div_up(R.n_src, kS5Hosts), 256, 0, s>>>(
            a, R.draws.as<uint32_t>());
    }
    SHD_HIP(hipGetLastError());
    // stable LSD radix sort of the records by destination (keys <= H), hand-written (scan.h)
    uint32_t bits = 1;
    while (bits < 32 && (H >> bits) != 0) ++bits;
    bool first = true;
    SHD_TRY(radix_sort_pairs(R.rs_counts, R.rs_scan, R.ev_val.as<uint32_t>(), R.rec.as<uint4>(),
                             R.ev_key.as<uint32_t>(), R.brec.as<uint4>(), n, bits, &first, s));
    uint4* sorted = first ? R.rec.as<uint4>() : R.brec.as<uint4>();
    uint4* spare = first ? R.brec.as<uint4>() : R.rec.as<uint4>();
    const uint32_t* skeys = first ? R.ev_val.as<uint32_t>() : R.ev_key.as<uint32_t>();
    bucket_offsets<<<div_up((uint64_t)H + 1, 256), 256, 0, s>>>(skeys, n, H, o->ev_off);
    segment_sort_v5<<<div_up(H, kSegDst), 256, 0, s>>>(
        H, o->ev_off, sorted, rd->round_end, seq_base, o->ev_deliver, o->ev_src,
        o->ev_seq, o->ev_pkt, R.ev_val2.as<uint32_t>());
    segment_sort_v2_big<<<64, 256, 0, s>>>(R.ev_val2.as<uint32_t>(), o->ev_off, sorted,
                                           spare, rd->round_end, seq_base,
                                           o->ev_deliver, o->ev_src, o->ev_seq, o->ev_pkt);
    SHD_HIP(hipGetLastError());
    SHD_TRY(readback(ctx, s, 8, R.red.p, 8 * sizeof(unsigned long long)));
    std::memcpy(R.red_host, ctx->h_pin + 8, sizeof(R.red_host));
    return SHD_OK;
}


// v7 eligibility: narrow table, LDS host map, src ids and packet indices within the record /
// key fields, and the stamp's LDS (map + slot counters) within the CU's 160 KB
static bool relay_v7_ok(shd_ctx* ctx, uint64_t n, uint32_t n_bins) {
    RelayState& R = ctx->relay;
    if (R.force_v3 || R.n_hosts > kV7MaxHosts || n > kV7MaxPackets) return false;
    if (R.n_src == 0 || std::min<uint32_t>(div_up(R.n_src, kS5Hosts), (uint32_t)ctx->n_cu) > kColMaxG) return false;
    // the stamp's static LDS, asked once (a function-local static: initialised once even when
    // two in-process ranks call the relay from two threads)
    static const size_t stat_lds = [] {
        hipFuncAttributes at{};
        // (both chance forms' static LDS: the larger)
        const void* ks[] = {reinterpret_cast<const void*>(&relay_stamp_v6<true, false>),
                            reinterpret_cast<const void*>(&relay_stamp_v6<true, true>),
                            reinterpret_cast<const void*>(&relay_stamp_v6<true, false, false>),
                            reinterpret_cast<const void*>(&relay_stamp_v6<true, true, false>)};
        size_t m = 0;
        for (const void* k : ks) {
            if (hipFuncGetAttributes(&at, k) != hipSuccess) return (size_t)0;
            m = std::max(m, (size_t)at.sharedSizeBytes);
        }
        return m;
    }();
    if (!stat_lds) return false;
    return stat_lds + (R.hn_bits ? (size_t)R.hn_words * 4 : 0) + (size_t)n_bins * 4 <= 160 * 1024;
}

// Hosts per stamp group: about S sends per group (SHD_RELAY_GROUP_SENDS, 0 = fixed kS5Hosts),
// so a group is one full chunk of the stamp, and a group count that is a multiple of the stamp's
// G workgroups, so no pass of the persistent grid runs with most workgroups idle.
static uint32_t v7_group_size(const shd_ctx* ctx, uint32_t n_src, uint32_t G, uint64_t n) {
    // default: one chunk's worth (C5: 40 hosts, ~4000 sends; stamp 310 -> 283 us; 36 hosts: 290)
    const uint64_t S = ctx->knobs.get64(K_RELAY_GROUP_SENDS, (uint64_t)kS6Cap);
    if (!S || !n || !n_src || !G) return kS5Hosts;
    const double per_host = (double)n / n_src;
    const uint32_t want = (uint32_t)std::min<double>(kS5Hosts, std::max<double>(8.0, (double)S / per_host));
    const uint64_t m = div_up((uint64_t)n_src, (uint64_t)G * want);
    return (uint32_t)std::min<uint64_t>(kS5Hosts, std::max<uint64_t>(1, div_up((uint64_t)n_src, (uint64_t)G * m)));
}

// The bins of a sharded round (relay_round_sharded_v7): rank r's destinations [r * per, ...)
// start bin r * bpr; n_bins over all ranks
struct XShard {
    uint32_t per = 0, bpr = 0, n_bins = 0;
    uint64_t mul = 0;
    uint32_t first_bin(uint32_t r) const { return std::min<uint32_t>(r * bpr, n_bins); }
};

static XShard xshard(uint32_t H, uint32_t world) {
    XShard x;
    x.per = (uint32_t)div_up((uint64_t)H, (uint64_t)world);
    x.bpr = div_up(x.per, kBinDst);
    x.mul = ((1ull << 40) + x.per - 1) / x.per;
    for (uint32_t r = 0; r < world; ++r) {
        uint32_t lo = 0, hi = 0;
        shard_range(H, (int)world, (int)r, &lo, &hi);
        x.n_bins += div_up(hi - lo, kBinDst);
    }
    return x;
}

// v7 up to and including the stamp; with xsh (a sharded round) the records stay in their bins
// for the exchange (no bin sort, no read-back), else the bin sort and the reductions' read-back
static shd_status relay_device_v7(shd_ctx* ctx, const shd_batch* b, const shd_round* rd,
                                  shd_relay_out* o, const XShard* xsh = nullptr) {
    RelayState& R = ctx->relay;
    hipStream_t s = ctx->stream;
    const uint64_t n = b->n_packets;
    const uint32_t H = R.n_hosts;
    const size_t nn = std::max<uint64_t>(n, 1);
    const uint32_t n_bins = xsh ? xsh->n_bins : div_up(H, kBinDst);
    const uint32_t G = std::min<uint32_t>(div_up(R.n_src, kS5Hosts), (uint32_t)ctx->n_cu);
    SHD_TRY(R.rec.ensure(nn * 16));
    SHD_TRY(R.draws.ensure(nn * 4));
    SHD_TRY(R.bin_cnt.ensure((size_t)G * (kHistSplit + 1) * n_bins * 4));
    SHD_TRY(R.bin_base.ensure((size_t)(2 * n_bins + 1) * 4));
    SHD_TRY(R.bin_lb.ensure((size_t)(n_bins + 1) * 8));
    RelayArgs3 a = relay_args3(ctx, b, rd, o);
    a.gs = v7_group_size(ctx, R.n_src, G, n);
    if (xsh) {
        a.sh_per = xsh->per;
        a.sh_bpr = xsh->bpr;
        a.sh_mul = xsh->mul;
    }
    uint32_t* tot = R.bin_base.as<uint32_t>() + n_bins + 1;
    a.bin_base = R.bin_base.as<uint32_t>();
    a.n_bins = n_bins;
    uint32_t* seg = R.bin_cnt.as<uint32_t>() + (size_t)G * kHistSplit * n_bins;
    a.seg_pre = seg;
    // (side-stream form: K0 goes first -- with the draws kept as 4 bytes and the histogram at 30
    // us, K0 plus the stream join (~12 us from its end to the stamp's start) was the longer of the
    // two chains, so its fork is issued before anything else.  The fork event follows the
    // caller's work on the stream, e.g. the kernels that wrote the batch.)
    const bool k0 = !b->chance && !R.cpu_draws;   // (shd_relay_flush filled the draws from the CPU's)
    // K0 in line before the histogram (default, round 5): K0 30 us + histogram 21 us back to back
    // beat K0 beside the histogram (39 ‖ 41 us, each slowed by the other taking wave slots) plus
    // the fork / join events: C5 round 0.467-0.476 -> 0.457 ms.  SHD_RELAY_K0_INLINE=0: the side stream.
    const bool k0_inline = k0 && ctx->knobs.get(K_RELAY_K0_INLINE, 1) != 0;
    if (k0_inline) {
        relay_draws<<<div_up(R.n_src, 64 * kK0Waves), 64 * kK0Waves, 0, s>>>(a, R.draws.as<uint32_t>());
    } else if (k0) {   // K0: the per-host generator streams, on the side stream next to the bins
        SHD_HIP(hipEventRecord(ctx->sev[0], s));
        SHD_HIP(hipStreamWaitEvent(ctx->side, ctx->sev[0], 0));
        relay_draws<<<div_up(R.n_src, 64 * kK0Waves), 64 * kK0Waves, 0, ctx->side>>>(a, R.draws.as<uint32_t>());
    }
    // the histogram's first block also resets the round's reductions (red_init's job: one
    // launch less; only the scans and the stamp read them, all after the histogram)
    // (SHD_HIST_SCALAR=1, tuning A/B: the flattened-position form)
    if (((uintptr_t)b->dst_host & 15) == 0 && n < (1ull << 31) && !ctx->knobs.on(K_HIST_SCALAR))
        relay_bin_hist4<<<G * kHistSplit, kHist4Threads, (size_t)n_bins * 4, s>>>(a, G, (uint32_t)n,
                                                                             R.bin_cnt.as<uint32_t>());
    else
        relay_bin_hist<<<G * kHistSplit, 256, (size_t)n_bins * 4, s>>>(a, G, R.bin_cnt.as<uint32_t>());
    if (k0 && !k0_inline) SHD_HIP(hipEventRecord(ctx->sev[1], ctx->side));   // after the histogram's launch
    if (ctx->knobs.get(K_RELAY_SCAN2, 0) != 0 || div_up(n_bins, 64) > 128) {   // (A/B: two launches)
        bin_col_scan<<<div_up(n_bins, 64), 1024, 0, s>>>(G, n_bins, R.bin_cnt.as<uint32_t>(), seg, tot, a.red);
        bin_base_scan<<<1, 1024, 0, s>>>(n_bins, tot, R.bin_base.as<uint32_t>(), R.bin_lb.as<unsigned long long>(), a.red);
    } else {   // the bases from the column scan's own look-back (bin_col_scan)
        ScanScratch& SS = R.col_scan;
        const uint64_t blocks = div_up(n_bins, 64);
        if (blocks * 16 + 16 > SS.state.bytes) {
            SHD_TRY(SS.state.ensure(blocks * 16 + 16));
            SHD_HIP(hipMemsetAsync(SS.state.p, 0, SS.state.bytes, s));
            SS.epoch = 0;
        }
        if (++SS.epoch >= (1u << 30)) {
            SHD_HIP(hipMemsetAsync(SS.state.p, 0, SS.state.bytes, s));
            SS.epoch = 1;
        }
        bin_col_scan<<<(uint32_t)blocks, 1024, 0, s>>>(G, n_bins, R.bin_cnt.as<uint32_t>(), seg, tot, a.red,
                                                       R.bin_base.as<uint32_t>(), R.bin_lb.as<unsigned long long>(),
                                                       SS.state.as<unsigned long long>(), SS.epoch);
    }
    if (k0 && !k0_inline) SHD_HIP(hipStreamWaitEvent(s, ctx->sev[1], 0));
    // (no LDS host map -- e.g. C5b's 50k nodes -- : the stamp gathers the destinations' nodes)
    auto* stamp = R.hn_bits ? (a.chance ? &relay_stamp_v6<true, true> : &relay_stamp_v6<true, false>)
                            : (a.chance ? &relay_stamp_v6<true, true, false> : &relay_stamp_v6<true, false, false>);
    stamp<<<G, kS6Threads, (R.hn_bits ? (size_t)R.hn_words * 4 : 0) + (size_t)n_bins * 4, s>>>(
        a, R.draws.as<uint32_t>(), R.hn_packed.as<uint32_t>(), R.hn_bits ? R.hn_words : 0u, R.hn_bits);
    if (xsh) {
        SHD_HIP(hipGetLastError());
        return SHD_OK;
    }
    V7Out vo{o->ev_deliver, o->ev_src, o->ev_seq, o->ev_pkt,
             a.abs_seq ? nullptr : R.next_id.as<uint64_t>(), rd->round_end};
    if (R.fl_ev_out && !a.abs_seq) {   // a flush round: compact records straight from the bin sort
        vo.fl_out = R.fl_ev_out;
        vo.fl_perm = R.fl_perm.as<uint32_t>();
        vo.fl_b12 = R.fl_b12;
        R.fl_direct = true;
    }
    const uint32_t stop = ctx->knobs.get(K_B7_STOP, 0);   // tuning only: partial K4 (wrong output)
    bin_sort_v7<false><<<n_bins, kB7Threads, 0, s>>>(H, n_bins, R.bin_base.as<uint32_t>(), R.rec.as<uint4>(),
                                                    R.bin_lb.as<unsigned long long>(), o->ev_off, vo, a.red,
                                                    stop, XSrc{});
    SHD_HIP(hipGetLastError());
    SHD_TRY(readback(ctx, s, 8, R.red.p, 8 * sizeof(unsigned long long)));
    std::memcpy(R.red_host, ctx->h_pin + 8, sizeof(R.red_host));
    return SHD_OK;
}

// One round: the new host state (RNG streams, event ids) is written to the second buffer and
// committed only when the round succeeds, so a failed round leaves the hosts untouched.
__global__ __launch_bounds__(256) void counts_commit(unsigned long long* __restrict__ counts,
                                                     const unsigned long long* __restrict__ delta,
                                                     uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n && delta[i]) {   // RoutingInfo::increment_packet_count saturates (graph/mod.rs:451-458)
        const unsigned long long c = counts[i], d = delta[i];
        counts[i] = c + d < c ? ~0ull : c + d;
    }
}

// The round's pipelines and checks; nothing of the hosts' state is committed yet.
static shd_status relay_run(shd_ctx* ctx, const shd_batch* b, const shd_round* rd, shd_relay_out* o) {
    RelayState& R = ctx->relay;
    const uint32_t H = R.n_hosts;
    const uint64_t nn = (uint64_t)R.n_nodes * R.n_nodes;
    SHD_TRY(R.red.ensure(64));
    SHD_TRY(R.dst_cnt.ensure((size_t)(H + 1) * 4));
    // every pipeline attempt counts into a zeroed per-round buffer; only the committed attempt
    // reaches the counters (a rerun or a failed round must not count)
    auto zero_counts = [&]() -> shd_status {
        if (R.count_on) SHD_HIP(hipMemsetAsync(R.counts_round.p, 0, nn * 8, ctx->stream));
        return SHD_OK;
    };
    if (R.count_on) SHD_TRY(R.counts_round.ensure(nn * 8));
    bool v2 = R.table_narrow && !R.force_v1;
    R.last_pipe = 1;
    if (v2) {
        bool done = false;
        if (relay_v7_ok(ctx, b->n_packets, div_up(H, kBinDst))) {
            SHD_TRY(zero_counts());
            SHD_TRY(relay_device_v7(ctx, b, rd, o));
            done = !R.red_host[6];   // else a bin overflowed: redo with the radix pipeline
            R.last_pipe = 7;
        }
        if (!done) {
            SHD_TRY(zero_counts());
            SHD_TRY(relay_device_v3(ctx, b, rd, o));
            R.last_pipe = 3;
        }
        if (R.red_host[4]) v2 = false;   // a deliver offset needs 64 bits: redo with v1
    }
    if (!v2) R.last_pipe = 1;
    if (!v2) {
        SHD_TRY(zero_counts());
        SHD_TRY(relay_device_v1(ctx, b, rd, o));
    }
    if (R.red_host[3] != ~0ull) return SHD_ERR_NO_HOST;
    if (v2 && R.red_host[5]) return SHD_ERR_INVALID;   // a host's send times went backwards
    R.last_v2 = v2;
    return SHD_OK;
}

// Commit a successful round: the per-path counters, the new RNG streams and event ids.
static shd_status relay_commit(shd_ctx* ctx, shd_relay_out* o) {
    RelayState& R = ctx->relay;
    const uint64_t nn = (uint64_t)R.n_nodes * R.n_nodes;
    if (R.count_on && nn) {
        counts_commit<<<div_up(nn, 256), 256, 0, ctx->stream>>>(
            R.counts.as<unsigned long long>(), R.counts_round.as<unsigned long long>(), nn);
        SHD_HIP(hipGetLastError());
    }
    std::swap(R.rng, R.rng2);
    std::swap(R.next_id, R.next_id2);
    R.seq_bound += R.red_host[2];
    o->min_deliver = R.red_host[0];
    o->min_latency = R.red_host[1];
    o->n_sent = R.red_host[2];
    return SHD_OK;
}

static shd_status relay_device(shd_ctx* ctx, const shd_batch* b, const shd_round* rd,
                               shd_relay_out* o) {
    SHD_TRY(relay_run(ctx, b, rd, o));
    SHD_TRY(relay_commit(ctx, o));
    o->n_dst = ctx->relay.n_hosts;
    o->n_events = (uint32_t)o->n_sent;
    round_note(ctx, o->min_deliver, o->min_latency);
    return SHD_OK;
}

// shd_relay_flush (flush.hip): one round on the batch it grouped on the device
shd_status relay_flush_round(shd_ctx* ctx, const shd_batch* b, const shd_round* rd, shd_relay_out* o) {
    return relay_device(ctx, b, rd, o);
}

// ------------------------------------------------------------------------------------------
// Sharded rounds (hosts split by id over the ranks).  Each rank stamps its own
// source hosts (their RNG streams and event ids live there) into events grouped by destination
// over ALL hosts; the events bound for rank r's hosts are one contiguous slice.  Per round:
//   1. local pipeline (as one GPU) -> events grouped by destination, in EventQueue order;
//   2. pack them as 24-byte records (deliver, seq, src, packet) and write, per peer, the
//      peer's per-destination offsets; one all-gather of every rank's sizing row -- its status,
//      reductions, receive capacity and event count per peer -- so every rank sees the whole
//      count matrix: the round's reductions ride on it, and whether any rank must grow its
//      receive buffers is known to all (then a second, one-word agreement follows the growth);
//   3. one host sync: sizes, and every rank's status (a failed round on any rank fails the
//      round everywhere, no host state is committed);
//   4. one grouped point-to-point exchange (offsets + records to every peer);
//   5. device k-way merge of the per-sender runs into this rank's destinations' events: the
//      senders own disjoint source ranges, so the merge by (deliver, src, seq) is EventQueue
//      order again (event.rs:84-155).
// No rank returns between two collectives on a local failure: allocations that depend on the
// round are folded into the status of the next agreement, the rest is sized at setup.
// ------------------------------------------------------------------------------------------
struct Ev24 {
    uint64_t deliver, seq;
    uint32_t src, pkt;
};
static_assert(sizeof(Ev24) == 24, "24-byte event record");
// sizing row of a rank: [0] status [1] min deliver [2] min latency [3] sent [4] receive
// capacity (events) [5..7] spare, then [kXHead + r] = events for rank r
constexpr uint32_t kXHead = 8;

// rel (a sharded flush, RelayState::rel_ids): ids relative to the source host's first id of the
// round, which only the sender holds
__global__ __launch_bounds__(256) void pack_events24(uint64_t n, const uint64_t* __restrict__ t,
                                                     const uint64_t* __restrict__ q, const uint32_t* __restrict__ sv,
                                                     const uint32_t* __restrict__ p, const uint64_t* __restrict__ rel,
                                                     Ev24* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = Ev24{t[i], rel ? q[i] - rel[sv[i]] : q[i], sv[i], p[i]};
}

__device__ __forceinline__ void shard_of(uint32_t total, uint32_t world, uint32_t r, uint32_t* lo, uint32_t* hi) {
    const uint64_t per = ((uint64_t)total + world - 1) / world;
    const uint64_t a = min((uint64_t)r * per, (uint64_t)total);
    *lo = (uint32_t)a;
    *hi = (uint32_t)min(a + per, (uint64_t)total);
}

__global__ __launch_bounds__(64) void shard_words(uint32_t world, uint32_t H, const uint32_t* __restrict__ ev_off,
                                                  uint64_t st, uint64_t md, uint64_t ml, uint64_t ns, uint64_t cap,
                                                  uint64_t* __restrict__ w) {
    for (uint32_t r = threadIdx.x; r < world; r += 64) {
        uint32_t lo, hi;
        shard_of(H, world, r, &lo, &hi);
        w[kXHead + r] = ev_off ? (uint64_t)(ev_off[hi] - ev_off[lo]) : 0ull;
    }
    if (threadIdx.x < kXHead) {
        const uint64_t v[kXHead] = {st, md, ml, ns, cap, 0, 0, 0};
        w[threadIdx.x] = v[threadIdx.x];
    }
}

// peer r's block: its destinations' offsets relative to the slice start, at stage[lo_r + r ..]
__global__ __launch_bounds__(256) void shard_offsets(uint32_t world, uint32_t H, const uint32_t* __restrict__ ev_off,
                                                     uint32_t* __restrict__ stage) {
    const uint32_t r = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    uint32_t lo, hi;
    shard_of(H, world, r, &lo, &hi);
    if (i <= hi - lo) stage[lo + r + i] = ev_off[lo + i] - ev_off[lo];
}

// thread per received event: its rank among its destination's events of all runs
__global__ __launch_bounds__(256) void merge_runs24(uint32_t n_runs, uint32_t n_dst,
                                                    const uint32_t* __restrict__ base,   // [n_runs + 1]
                                                    const uint32_t* __restrict__ off,    // [n_runs][n_dst + 1]
                                                    const Ev24* __restrict__ in,
                                                    const uint32_t* __restrict__ out_off,
                                                    uint64_t* __restrict__ out_t, uint32_t* __restrict__ out_s,
                                                    uint64_t* __restrict__ out_q, uint32_t* __restrict__ out_p) {
    // The event's destination d: a run's events are in destination order and a block takes 256
    // consecutive events, so threads 0 and 1 search the whole offset row for the block's first
    // and last event (when both lie in one run) and every thread then searches only between the
    // two (~3 destinations on C5) -- instead of 17 dependent loads over 100k offsets per event.
    __shared__ uint32_t s_d[2];
    const uint32_t total = base[n_runs];
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    const uint32_t e0 = blockIdx.x * 256, e1 = min(e0 + 255, total - 1);
    auto run_of = [&](uint32_t x) {
        uint32_t r = 0;
        while (r + 1 < n_runs && base[r + 1] <= x) ++r;
        return r;
    };
    auto dst_of = [&](const uint32_t* o, uint32_t le, uint32_t lo, uint32_t hi) {   // o[d] <= le < o[d+1]
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (o[m] <= le) lo = m; else hi = m;
        }
        return lo;
    };
    const uint32_t rb0 = run_of(e0), rb1 = run_of(e1);
    const uint32_t* ob = off + (size_t)rb0 * (n_dst + 1);
    if (rb0 == rb1 && threadIdx.x < 2) s_d[threadIdx.x] = dst_of(ob, (threadIdx.x ? e1 : e0) - base[rb0], 0, n_dst);
    __syncthreads();
    if (e >= total) return;   // no barrier follows
    const uint32_t r = rb0 == rb1 ? rb0 : run_of(e);
    const uint32_t le = e - base[r];
    const uint32_t* o = off + (size_t)r * (n_dst + 1);
    const uint32_t d = rb0 == rb1 ? dst_of(o, le, s_d[0], s_d[1] + 1) : dst_of(o, le, 0, n_dst);
    const Ev24 x = in[e];
    uint32_t rank = le - o[d];
    for (uint32_t r2 = 0; r2 < n_runs; ++r2) {
        if (r2 == r) continue;
        const uint32_t* o2 = off + (size_t)r2 * (n_dst + 1);
        uint32_t a = base[r2] + o2[d], b = base[r2] + o2[d + 1];
        const uint32_t a0 = a;
        while (a < b) {   // run r2's events of destination d that come before this one
            const uint32_t m = (a + b) >> 1;
            const Ev24 y = in[m];
            if (ev3_less(y.deliver, y.src, y.seq, x.deliver, x.src, x.seq)) a = m + 1; else b = m;
        }
        rank += a - a0;
    }
    const uint32_t pos = out_off[d] + rank;
    out_t[pos] = x.deliver;
    out_s[pos] = x.src;
    out_q[pos] = x.seq;
    out_p[pos] = x.pkt;
}

// merge_runs24 by destination (default): a wave per destination takes the destination's
// events of every sender run (<= 128: C5 has ~100 per destination), sorts the unique keys
// (deliver - tmin) << 8 | index with the wave network (wave.h) and stores them in rank order,
// coalesced -- instead of a thread per event searching every sibling run's segment (a chain of
// dependent 24-byte loads per run).  A destination with more events, a deliver-time span of
// 2^24 ns or more, or two equal deliver times (their order needs (src, seq)) is merged by the
// per-event searches in the same wave.
__global__ __launch_bounds__(256) void merge_dst24(uint32_t n_runs, uint32_t n_dst, const uint32_t* __restrict__ base,
                                                   const uint32_t* __restrict__ off, const Ev24* __restrict__ in,
                                                   const uint32_t* __restrict__ out_off, uint64_t* __restrict__ out_t,
                                                   uint32_t* __restrict__ out_s, uint64_t* __restrict__ out_q,
                                                   uint32_t* __restrict__ out_p) {
    constexpr int NPL = 2;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t d = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (d >= n_dst) return;   // wave-uniform; no barrier in this kernel
    // lane q < n_runs: run q's segment of destination d
    uint32_t seg = 0, cnt = 0;
    if (lane < n_runs) {
        const uint32_t* o = off + (size_t)lane * (n_dst + 1);
        seg = base[lane] + o[d];
        cnt = o[d + 1] - o[d];
    }
    uint32_t incl = cnt;
    for (uint32_t k = 1; k < 64; k <<= 1) {
        const uint32_t y = __shfl_up(incl, k);
        if (lane >= k) incl += y;
    }
    const uint32_t pre = incl - cnt;
    // the destination's event count from the merged offsets (every run, also past lane 63)
    const uint32_t out0 = out_off[d], n = out_off[d + 1] - out0;
    bool done = false;
    if (n <= 64u * NPL && n_runs <= 64) {
        Ev24 x[NPL];
        uint64_t tmn = ~0ull, tmx = 0;
#pragma unroll
        for (int c = 0; c < NPL; ++c) {
            const uint32_t i = lane + 64u * c;
            // the run holding staged index i: the last q whose prefix is <= i (ballot over lanes)
            const uint64_t m = __ballot(lane < n_runs && cnt > 0);
            uint32_t at = 0;
            for (uint64_t mm = m; mm; mm &= mm - 1) {
                const int q = __builtin_ctzll(mm);
                const uint32_t pq = __shfl(pre, q), sq = __shfl(seg, q);
                if (i < n && pq <= i) at = sq + (i - pq);
            }
            x[c] = i < n ? in[at] : Ev24{~0ull, 0, 0, 0};
            if (i < n) {
                tmn = x[c].deliver < tmn ? x[c].deliver : tmn;
                tmx = x[c].deliver > tmx ? x[c].deliver : tmx;
            }
        }
        for (int k = 32; k > 0; k >>= 1) {
            const uint64_t a = __shfl_xor(tmn, k), b = __shfl_xor(tmx, k);
            tmn = a < tmn ? a : tmn;
            tmx = b > tmx ? b : tmx;
        }
        if (n > 0 && tmx - tmn < (1ull << 24)) {
            uint32_t k32[NPL];
#pragma unroll
            for (int c = 0; c < NPL; ++c) {
                const uint32_t i = lane + 64u * c;
                k32[c] = i < n ? ((uint32_t)(x[c].deliver - tmn) << 8) | i : ~0u;
            }
            wave_bitonic32<NPL>(k32, lane);
            bool tie = false;
#pragma unroll
            for (int c = 0; c < NPL; ++c) {
                const uint32_t down = (uint32_t)__shfl_down((int)k32[c], 1);
                const uint32_t first = c + 1 < NPL ? (uint32_t)__shfl((int)k32[c + 1 < NPL ? c + 1 : c], 0) : ~0u;
                const uint32_t nx = lane == 63 ? first : down;
                if (lane + 64u * c + 1 < n && (nx >> 8) == (k32[c] >> 8)) tie = true;
            }
            if (__ballot(tie) == 0) {
#pragma unroll
                for (int c = 0; c < NPL; ++c) {
                    const uint32_t r = lane + 64u * c, i = k32[c] & 0xFFu;
                    const int src_lane = (int)(i & 63u);
                    // element i sits in lane i % 64, register i / 64 (every lane shuffles both)
                    Ev24 y{0, 0, 0, 0};
#pragma unroll
                    for (int c2 = 0; c2 < NPL; ++c2) {
                        const uint64_t t = __shfl(x[c2].deliver, src_lane), q = __shfl(x[c2].seq, src_lane);
                        const uint32_t sv = (uint32_t)__shfl((int)x[c2].src, src_lane);
                        const uint32_t pv = (uint32_t)__shfl((int)x[c2].pkt, src_lane);
                        if ((i >> 6) == (uint32_t)c2) y = Ev24{t, q, sv, pv};
                    }
                    if (r < n) {
                        out_t[out0 + r] = y.deliver;
                        out_s[out0 + r] = y.src;
                        out_q[out0 + r] = y.seq;
                        out_p[out0 + r] = y.pkt;
                    }
                }
                done = true;
            }
        }
    }
    if (done) return;
    // per-event searches (merge_runs24's rank rule) over this destination's events
    for (uint32_t i = lane; i < n; i += 64) {
        uint32_t q0 = 0, at = 0, rank = 0;
        uint32_t acc = 0;   // i's run: the segment counts' running sum
        for (uint32_t q = 0; q < n_runs; ++q) {
            const uint32_t* o = off + (size_t)q * (n_dst + 1);
            const uint32_t c = o[d + 1] - o[d];
            if (i >= acc && i < acc + c) {
                q0 = q;
                at = base[q] + o[d] + (i - acc);
                rank = i - acc;
            }
            acc += c;
        }
        const Ev24 x = in[at];
        for (uint32_t r2 = 0; r2 < n_runs; ++r2) {
            if (r2 == q0) continue;
            const uint32_t* o2 = off + (size_t)r2 * (n_dst + 1);
            uint32_t a = base[r2] + o2[d], b = base[r2] + o2[d + 1];
            const uint32_t a0 = a;
            while (a < b) {
                const uint32_t m = (a + b) >> 1;
                const Ev24 y = in[m];
                if (ev3_less(y.deliver, y.src, y.seq, x.deliver, x.src, x.seq)) a = m + 1; else b = m;
            }
            rank += a - a0;
        }
        out_t[out0 + rank] = x.deliver;
        out_s[out0 + rank] = x.src;
        out_q[out0 + rank] = x.seq;
        out_p[out0 + rank] = x.pkt;
    }
}

// ------------------------------------------------------------------------------------------
// Sharded rounds without the merge (relay_round_sharded_v7, the default when every rank runs
// pipeline 7).  The stamp places every record into its destination bin as on one GPU, but the
// bins restart at every rank's first destination (XShard), so the records bound for rank r are
// one contiguous slice of the stamp's output and each of r's bins is a sub-slice of it.  The
// exchange moves those 16-byte records as they lie -- no packing, no per-peer offsets: every
// rank's per-bin counts ride in the one sizing all-gather -- and the receiver runs the bin sort
// over its own bins with each bin's records gathered from every sender's slice (bin_sort_v7<X>):
// that yields its destinations' events in EventQueue order directly, so no merge pass follows.
// One host sync sizes the exchange (statuses, reductions, counts, fallback flags of every
// rank); a second reads the number of events received.
// The sizing row of a rank (u64 words): [0] status [1] min deliver [2] min latency [3] sent
// [4] receive capacity (events) [5] fallback flags [6] packets [7] spare, then the u32 record
// count of every bin (all ranks' bins) from word kXsHead on.
constexpr uint32_t kXsHead = 8;
constexpr uint32_t kXsOverflow = 1, kXsWide = 2, kXsHost = 4;

static size_t xs_row_words(uint32_t n_bins) { return kXsHead + ((size_t)n_bins + 1) / 2; }

__global__ __launch_bounds__(256) void xs_row(const unsigned long long* __restrict__ red, const uint32_t* __restrict__ tot,
                                              uint32_t n_bins, uint32_t ran, int32_t st_local, uint64_t cap,
                                              uint64_t n_pkt, uint32_t host_flags, int32_t st_nohost,
                                              int32_t st_invalid, uint64_t* __restrict__ row) {
    const uint32_t t = threadIdx.x, b = blockIdx.x * 256 + t;
    uint32_t* rt = reinterpret_cast<uint32_t*>(row + kXsHead);
    if (b < n_bins) rt[b] = ran ? tot[b] : 0u;   // a bin per thread (one block: 13 dependent trips, 7 us)
    if (blockIdx.x == 0 && t == 0) {
        uint64_t st = (uint64_t)(int64_t)st_local, md = ~0ull, ml = ~0ull, ns = 0;
        uint32_t fl = host_flags;
        if (ran) {
            if (red[6]) {
                fl |= kXsOverflow;   // the stamp did not run: the fallback reruns the round
            } else {
                if (red[3] != ~0ull) st = (uint64_t)(int64_t)st_nohost;   // as relay_run: NO_HOST first
                else if (red[5]) st = (uint64_t)(int64_t)st_invalid;
                if (red[4]) fl |= kXsWide;
                md = red[0];
                ml = red[1];
                ns = red[2];
            }
        }
        row[0] = st;
        row[1] = md;
        row[2] = ml;
        row[3] = ns;
        row[4] = cap;
        row[5] = fl;
        row[6] = n_pkt;
        row[7] = 0;
    }
}

// bins per thread of xs_sizing's 1024: n_bins <= 2^18 / 32 hosts + 64 ranks (relay_round_sharded_v7)
constexpr uint32_t kXsPer = 9;
static_assert(kXsPer * 1024 >= (kV7MaxHosts >> kBinShift) + 64, "xs_sizing: bins per thread");

// The sizing summary every rank derives alike from the gathered rows, one workgroup: sender by
// sender, the exclusive scan of its bin counts -> sc[q * (n_bins + 1) + b] (a thread's counts in
// registers); then out[0] = the largest bin over all senders (the receiver's LDS stage bound),
// out[1 ..] the world headers, then the record counts M[q][r] (sender q -> rank r); xb[q] =
// sender q's slice in this rank's received records (own records are not received), xb[world +
// q] = the packets of the senders before q.  (A block per sender with the last one to finish
// writing the summary took 15 us at world size 1: its device-scope fences write the XCD's L2
// back after the stamp's stores.  One workgroup needs no fence beyond its own.)
__global__ __launch_bounds__(1024) void xs_sizing(const uint64_t* __restrict__ rows, size_t row_words, uint32_t n_bins,
                                                  uint32_t world, uint32_t me, uint32_t bpr, uint32_t* sc,
                                                  uint64_t* __restrict__ out, uint32_t* __restrict__ xb) {
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_max;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t per = (n_bins + 1023) / 1024, b0 = min(n_bins, tid * per), b1 = min(n_bins, b0 + per);
    if (tid == 0) s_max = 0;
    uint32_t tot[kXsPer];
#pragma unroll
    for (uint32_t j = 0; j < kXsPer; ++j) tot[j] = 0;
    for (uint32_t q = 0; q < world; ++q) {
        const uint32_t* t = reinterpret_cast<const uint32_t*>(rows + (size_t)q * row_words + kXsHead);
        uint32_t* o = sc + (size_t)q * (n_bins + 1);
        uint32_t v[kXsPer];   // (per <= kXsPer: every load of the thread in flight at once)
#pragma unroll
        for (uint32_t j = 0; j < kXsPer; ++j) v[j] = b0 + j < b1 ? t[b0 + j] : 0u;
        uint32_t sum = 0;
#pragma unroll
        for (uint32_t j = 0; j < kXsPer; ++j) {
            sum += v[j];
            tot[j] += v[j];
        }
        uint32_t incl = sum;
        for (uint32_t k = 1; k < 64; k <<= 1) {
            const uint32_t y = __shfl_up(incl, k);
            if (lane >= k) incl += y;
        }
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        uint32_t run = incl - sum;
        for (uint32_t u = 0; u < w; ++u) run += s_w[u];
#pragma unroll
        for (uint32_t j = 0; j < kXsPer; ++j) {
            if (b0 + j < b1) o[b0 + j] = run;
            run += v[j];
        }
        if (tid == 1023) o[n_bins] = run;
        __syncthreads();   // (s_w is rewritten by the next sender)
    }
    uint32_t mx = 0;
#pragma unroll
    for (uint32_t j = 0; j < kXsPer; ++j) mx = max(mx, tot[j]);
    atomicMax(&s_max, mx);
    for (uint32_t i = tid; i < world * kXsHead; i += 1024) out[1 + i] = rows[(size_t)(i / kXsHead) * row_words + i % kXsHead];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the scans' stores, before the reads below
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    uint64_t* M = out + 1 + (size_t)world * kXsHead;
    for (uint32_t i = tid; i < world * world; i += 1024) {
        const uint32_t p = i / world, r = i % world;
        const uint32_t* sp = sc + (size_t)p * (n_bins + 1);
        M[i] = sp[min(r * bpr + bpr, n_bins)] - sp[min(r * bpr, n_bins)];
    }
    if (tid == 0) {
        uint32_t rb = 0;
        uint64_t pb = 0;
        for (uint32_t p = 0; p < world; ++p) {
            const uint32_t* sp = sc + (size_t)p * (n_bins + 1);
            xb[p] = rb;
            if (p != me) rb += sp[min(me * bpr + bpr, n_bins)] - sp[min(me * bpr, n_bins)];
            xb[world + p] = (uint32_t)pb;
            pb += rows[(size_t)p * row_words + 6];
        }
        out[0] = s_max;
    }
}

// sharded rounds' buffers that depend only on the host count and the ranks (shd_relay_setup)
static shd_status relay_shard_alloc(shd_ctx* ctx) {
    RelayState& R = ctx->relay;
    const uint32_t world = (uint32_t)ctx->comm->size, H = R.n_hosts;
    uint32_t own_lo = 0, own_hi = 0;
    shard_range(H, (int)world, ctx->comm->rank, &own_lo, &own_hi);
    const size_t n_own = own_hi - own_lo;
    const XShard xsh = xshard(H, world);
    const size_t rw = std::max<size_t>(xs_row_words(xsh.n_bins), kXHead + world);
    SHD_TRY(R.x_words.ensure((size_t)world * rw * 8 + (size_t)world * 8 + 64));
    SHD_TRY(R.xs_sc.ensure((size_t)world * (xsh.n_bins + 1) * 4));
    const size_t out_bytes = (1 + (size_t)world * kXsHead + (size_t)world * world) * 8 + 64;
    SHD_TRY(R.xs_out.ensure(out_bytes));
    SHD_TRY(R.xs_pin.ensure(out_bytes));
    SHD_TRY(R.xs_b.ensure((size_t)world * 8 + 64));
    SHD_TRY(R.x_off.ensure(((size_t)H + world) * 4));
    SHD_TRY(R.x_roff.ensure((size_t)world * (n_own + 1) * 4 + (size_t)(world + 1) * 4));
    SHD_TRY(R.m_off.ensure((n_own + 4) * 4));   // + the received statuses' word (bin_sort_v7<true>)
    SHD_TRY(R.xs_st.ensure(((size_t)world + 1) * 8));
    SHD_HIP(hipMemsetAsync(R.xs_st.p, 0, ((size_t)world + 1) * 8, ctx->stream));
    R.xs_st_dirty = false;
    SHD_TRY(R.ev_off.ensure(((size_t)H + 1) * 4));
    R.x_cap = 0;
    return SHD_OK;
}

// receive side of a sharded round for n events (records, merged arrays), with headroom
static shd_status relay_recv_grow(RelayState& R, uint64_t n) {
    const uint64_t m = std::max<uint64_t>(n + n / 2, 1024);
    SHD_TRY(R.x_rrec.ensure(m * 24));
    SHD_TRY(R.m_deliver.ensure(m * 8));
    SHD_TRY(R.m_src.ensure(m * 4));
    SHD_TRY(R.m_seq.ensure(m * 8));
    SHD_TRY(R.m_pkt.ensure(m * 4));
    R.x_cap = m;
    return SHD_OK;
}

static shd_status relay_round_sharded_x24(shd_ctx* ctx, const shd_batch* b, const shd_round* rd,
                                          shd_relay_out* d_out) {
    RelayState& R = ctx->relay;
    Comm& C = *ctx->comm;
    hipStream_t s = ctx->stream;
    const uint32_t H = R.n_hosts, world = (uint32_t)C.size, WR = kXHead + world;
    const uint64_t n = b->n_packets;
    const size_t nn = std::max<uint64_t>(n, 1);
    // 1. the local pipeline into internal buffers (the caller's status array); a failure here is
    //    this rank's status in the sizing row, not a return
    shd_status st = SHD_OK;
    shd_relay_out lo{};
    if (R.ev_deliver.ensure(nn * 8) != SHD_OK || R.ev_src.ensure(nn * 4) != SHD_OK ||
        R.ev_seq.ensure(nn * 8) != SHD_OK || R.ev_pkt.ensure(nn * 4) != SHD_OK || R.x_rec.ensure(nn * 24) != SHD_OK)
        st = SHD_ERR_NOMEM;
    if (st == SHD_OK) {
        lo.status = d_out->status;
        lo.ev_off = R.ev_off.as<uint32_t>();
        lo.ev_deliver = R.ev_deliver.as<uint64_t>();
        lo.ev_src = R.ev_src.as<uint32_t>();
        lo.ev_seq = R.ev_seq.as<uint64_t>();
        lo.ev_pkt = R.ev_pkt.as<uint32_t>();
        st = relay_run(ctx, b, rd, &lo);
    }
    // 2. records, per-peer offset blocks, this rank's sizing row (buffers sized at setup)
    uint64_t* rows = R.x_words.as<uint64_t>();            // [world][WR] after the all-gather
    uint64_t* agree = rows + (size_t)world * WR;           // [world] growth agreement
    const uint64_t ns_local = st == SHD_OK ? R.red_host[2] : 0;
    if (st == SHD_OK && ns_local)
        pack_events24<<<div_up(ns_local, 256), 256, 0, s>>>(ns_local, lo.ev_deliver, lo.ev_seq, lo.ev_src,
                                                            lo.ev_pkt, R.rel_ids ? R.next_id.as<uint64_t>() : nullptr,
                                                            R.x_rec.as<Ev24>());
    shard_words<<<1, 64, 0, s>>>(world, H, st == SHD_OK ? lo.ev_off : nullptr, (uint64_t)st,
                                 st == SHD_OK ? R.red_host[0] : ~0ull, st == SHD_OK ? R.red_host[1] : ~0ull,
                                 ns_local, R.x_cap, rows + (size_t)C.rank * WR);
    if (st == SHD_OK)
        shard_offsets<<<dim3(div_up((uint64_t)(H + world - 1) / world + 1, 256), world), 256, 0, s>>>(
            world, H, lo.ev_off, R.x_off.as<uint32_t>());
    if (hipGetLastError() != hipSuccess && st == SHD_OK) st = SHD_ERR_HIP;
    SHD_TRY(C.all_gather(rows + (size_t)C.rank * WR, rows, (size_t)WR * 8, s));   // agreed (LocalComm) / fatal (RCCL)
    // 3. one host sync: the count matrix, every rank's outcome and capacity
    std::vector<uint64_t> w((size_t)world * WR);
    SHD_HIP(hipMemcpyAsync(w.data(), rows, w.size() * 8, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    auto row = [&](uint32_t q) { return w.data() + (size_t)q * WR; };
    uint64_t md = ~0ull, ml = ~0ull, ns = 0;
    for (uint32_t q = 0; q < world; ++q)
        if ((shd_status)row(q)[0] != SHD_OK) return (shd_status)row(q)[0];   // the lowest failing rank's
    for (uint32_t q = 0; q < world; ++q) {
        md = std::min<uint64_t>(md, row(q)[1]);
        ml = std::min<uint64_t>(ml, row(q)[2]);
        ns += row(q)[3];
    }
    // receive totals of every rank: whether any rank must grow is known to all of them
    bool grow = false;
    for (uint32_t r = 0; r < world; ++r) {
        uint64_t t = 0;
        for (uint32_t q = 0; q < world; ++q) t += row(q)[kXHead + r];
        grow = grow || t > row(r)[4];
    }
    uint32_t own_lo = 0, own_hi = 0;
    shard_range(H, (int)world, C.rank, &own_lo, &own_hi);
    const uint32_t n_own = own_hi - own_lo;
    std::vector<uint32_t> rbase(world + 1, 0);
    for (uint32_t q = 0; q < world; ++q) rbase[q + 1] = rbase[q] + (uint32_t)row(q)[kXHead + C.rank];
    const uint64_t n_recv = rbase[world];
    if (grow) {   // every rank takes this branch: one more agreement, on the growth's outcome
        shd_status gs = n_recv > R.x_cap ? relay_recv_grow(R, n_recv) : SHD_OK;
        ctx->h_pin[44] = (uint64_t)gs;
        if (hipMemcpyAsync(agree + C.rank, ctx->h_pin + 44, 8, hipMemcpyHostToDevice, s) != hipSuccess && gs == SHD_OK)
            gs = SHD_ERR_HIP;   // (the row still goes out: the peers wait for it)
        SHD_TRY(C.all_gather(agree + C.rank, agree, 8, s));
        std::vector<uint64_t> a(world);
        SHD_HIP(hipMemcpyAsync(a.data(), agree, world * 8, hipMemcpyDeviceToHost, s));
        SHD_HIP(hipStreamSynchronize(s));
        for (uint32_t q = 0; q < world; ++q)
            if ((shd_status)a[q] != SHD_OK) return (shd_status)a[q];
        if (gs != SHD_OK) return gs;
    }
    // 4. the exchange: part 0 = offsets block, part 1 = records
    std::vector<const void*> sp(2 * world);
    std::vector<void*> rp(2 * world);
    std::vector<size_t> sb(2 * world), rb(2 * world);
    uint64_t sent_before = 0;
    const uint64_t* mine = row((uint32_t)C.rank);
    for (uint32_t r = 0; r < world; ++r) {
        uint32_t a = 0, z = 0;
        shard_range(H, (int)world, (int)r, &a, &z);
        sp[2 * r] = R.x_off.as<uint32_t>() + a + r;
        sb[2 * r] = (size_t)(z - a + 1) * 4;
        sp[2 * r + 1] = R.x_rec.as<Ev24>() + sent_before;
        sb[2 * r + 1] = (size_t)mine[kXHead + r] * 24;
        sent_before += mine[kXHead + r];
        rp[2 * r] = R.x_roff.as<uint32_t>() + (size_t)r * (n_own + 1);
        rb[2 * r] = (size_t)(n_own + 1) * 4;
        rp[2 * r + 1] = R.x_rrec.as<Ev24>() + rbase[r];
        rb[2 * r + 1] = (size_t)row(r)[kXHead + C.rank] * 24;
    }
    SHD_TRY(C.exchange(2, sp.data(), sb.data(), rp.data(), rb.data(), s));   // agreed (LocalComm) / fatal (RCCL)
    // 5. merge the per-sender runs (no collective follows: a HIP failure from here on is local)
    uint32_t* d_base = R.x_roff.as<uint32_t>() + (size_t)world * (n_own + 1);
    SHD_HIP(hipMemcpyAsync(d_base, rbase.data(), (world + 1) * 4, hipMemcpyHostToDevice, s));
    merge_offsets<<<div_up((uint64_t)n_own + 1, 256), 256, 0, s>>>(world, n_own, R.x_roff.as<uint32_t>(),
                                                                  R.m_off.as<uint32_t>());
    if (n_recv && ctx->knobs.get(K_MERGE_BY_EVENT, 0) != 1)
        merge_dst24<<<div_up(n_own, 4), 256, 0, s>>>(world, n_own, d_base, R.x_roff.as<uint32_t>(),
                                                     R.x_rrec.as<Ev24>(), R.m_off.as<uint32_t>(),
                                                     R.m_deliver.as<uint64_t>(), R.m_src.as<uint32_t>(),
                                                     R.m_seq.as<uint64_t>(), R.m_pkt.as<uint32_t>());
    else if (n_recv)
        merge_runs24<<<div_up(n_recv, 256), 256, 0, s>>>(world, n_own, d_base, R.x_roff.as<uint32_t>(),
                                                        R.x_rrec.as<Ev24>(), R.m_off.as<uint32_t>(),
                                                        R.m_deliver.as<uint64_t>(), R.m_src.as<uint32_t>(),
                                                        R.m_seq.as<uint64_t>(), R.m_pkt.as<uint32_t>());
    SHD_HIP(hipGetLastError());
    SHD_TRY(relay_commit(ctx, &lo));
    SHD_HIP(hipStreamSynchronize(s));   // rbase (host memory) was read by the copy above
    d_out->ev_off = R.m_off.as<uint32_t>();
    d_out->ev_deliver = R.m_deliver.as<uint64_t>();
    d_out->ev_src = R.m_src.as<uint32_t>();
    d_out->ev_seq = R.m_seq.as<uint64_t>();
    d_out->ev_pkt = R.m_pkt.as<uint32_t>();
    d_out->min_deliver = md;
    d_out->min_latency = ml;
    d_out->n_sent = ns;
    d_out->n_dst = n_own;
    d_out->n_events = (uint32_t)n_recv;
    round_note(ctx, md, ml);
    R.last_recv = n_recv;
    return SHD_OK;
}


// One sharded round without the merge (see xs_row above).  *fallback = true (the same on every
// rank: the decision reads only the gathered rows) when any rank cannot take this path -- not
// pipeline 7, a bin over its LDS stage, a deliver offset or event ids
// past 32 bits, more than 2^24 packets over all ranks -- and the caller then runs the packing
// path (relay_round_sharded_x24), which reruns the round from the uncommitted state.
static shd_status relay_round_sharded_v7(shd_ctx* ctx, const shd_batch* b, const shd_round* rd,
                                         shd_relay_out* d_out, bool* fallback) {
    RelayState& R = ctx->relay;
    Comm& C = *ctx->comm;
    hipStream_t s = ctx->stream;
    const uint32_t H = R.n_hosts, world = (uint32_t)C.size, me = (uint32_t)C.rank;
    const uint64_t n = b->n_packets;
    const XShard xsh = xshard(H, world);
    const uint32_t n_bins = xsh.n_bins;
    const size_t rw = xs_row_words(n_bins);
    *fallback = false;
    // 1. the local pipeline up to the stamp (records left in their bins); a failure is this
    //    rank's status in its sizing row, not a return
    const bool ok7 = world <= 64 && R.n_src > 0 && R.table_narrow && !R.force_v1 && relay_v7_ok(ctx, n, n_bins);
    // absolute ids must fit the records' 32 bits; relative ids (a sharded flush) always do
    const bool abs_seq = R.rel_ids || R.seq_bound + n < (1ull << 32);
    shd_status st = SHD_OK;
    shd_relay_out lo{};
    lo.status = d_out->status;
    bool ran = false;
    if (ok7 && abs_seq) {
        const uint64_t nn = (uint64_t)R.n_nodes * R.n_nodes;   // the round's counter increments start at 0
        if (R.red.ensure(64) != SHD_OK || (R.count_on && R.counts_round.ensure(nn * 8) != SHD_OK))
            st = SHD_ERR_NOMEM;
        else if (R.count_on && hipMemsetAsync(R.counts_round.p, 0, nn * 8, s) != hipSuccess)
            st = SHD_ERR_HIP;
        if (st == SHD_OK) st = relay_device_v7(ctx, b, rd, &lo, &xsh);
        ran = st == SHD_OK;
    }
    uint64_t* rows = R.x_words.as<uint64_t>();
    uint64_t* agree = rows + (size_t)world * rw;
    xs_row<<<std::max<uint32_t>(1, div_up(n_bins, 256)), 256, 0, s>>>(ran ? R.red.as<unsigned long long>() : nullptr,
                             ran ? R.bin_base.as<uint32_t>() + n_bins + 1 : nullptr, n_bins, ran ? 1u : 0u,
                             (int32_t)st, R.x_cap, n, (ok7 && abs_seq) ? 0u : kXsHost, (int32_t)SHD_ERR_NO_HOST,
                             (int32_t)SHD_ERR_INVALID, rows + (size_t)me * rw);
    if (hipGetLastError() != hipSuccess) {
        // the row the peers size the exchange from must carry the failure: written from the host
        if (st == SHD_OK) st = SHD_ERR_HIP;
        std::vector<uint64_t> hrow(rw, 0);
        hrow[0] = (uint64_t)(int64_t)st;
        hrow[1] = hrow[2] = ~0ull;
        (void)hipMemcpy(rows + (size_t)me * rw, hrow.data(), rw * 8, hipMemcpyHostToDevice);
    }
    SHD_TRY(C.all_gather(rows + (size_t)me * rw, rows, rw * 8, s));   // agreed (LocalComm) / fatal (RCCL)
    // 2. the sizing summary, one host sync.  From here on a local failure is carried into the
    //    exchange (its status part) instead of returned: the peers are on their way to it.  A
    //    failure of the summary's own read-back leaves this rank without the sizes, which is fatal
    //    to the communicator, as an RCCL failure is.
    shd_status st_post = SHD_OK;
    uint32_t* xb = R.xs_b.as<uint32_t>();
    xs_sizing<<<1, 1024, 0, s>>>(rows, rw, n_bins, world, me, xsh.bpr, R.xs_sc.as<uint32_t>(),
                                 R.xs_out.as<uint64_t>(), xb);
    const size_t out_words = 1 + (size_t)world * kXsHead + (size_t)world * world;
    SHD_TRY(readback_into(ctx, s, R.xs_out.p, out_words * 8, R.xs_pin.as<unsigned long long>()));
    if (hipGetLastError() != hipSuccess) st_post = SHD_ERR_HIP;
    if (ctx->knobs.get(K_TEST_FAIL, 0) == 1) st_post = SHD_ERR_HIP;   // (fault injection, tests)
    const uint64_t* pin = R.xs_pin.as<uint64_t>();
    auto hdr = [&](uint32_t q) { return pin + 1 + (size_t)q * kXsHead; };
    auto M = [&](uint32_t q, uint32_t r) { return pin[1 + (size_t)world * kXsHead + (size_t)q * world + r]; };
    for (uint32_t q = 0; q < world; ++q)
        if ((shd_status)hdr(q)[0] != SHD_OK) return (shd_status)hdr(q)[0];   // the lowest failing rank's
    uint64_t pk = 0;
    bool fb = pin[0] > kB7Cap;
    for (uint32_t q = 0; q < world; ++q) {
        fb = fb || hdr(q)[5] != 0;
        pk += hdr(q)[6];
    }
    if (fb || pk >= kV7MaxPackets) {
        *fallback = true;
        return SHD_OK;
    }
    uint64_t md = ~0ull, ml = ~0ull, ns = 0;
    for (uint32_t q = 0; q < world; ++q) {
        md = std::min<uint64_t>(md, hdr(q)[1]);
        ml = std::min<uint64_t>(ml, hdr(q)[2]);
        ns += hdr(q)[3];
    }
    // receive capacity (records, and the events they hold): whether any rank grows is known to all
    bool grow = false;
    uint64_t n_recv = 0;
    for (uint32_t r = 0; r < world; ++r) {
        uint64_t t = 0;
        for (uint32_t q = 0; q < world; ++q) t += M(q, r);
        grow = grow || t > hdr(r)[4];
        if (r == me) n_recv = t;
    }
    if (grow) {   // every rank takes this branch: one more agreement, on the growth's outcome
        shd_status gs = n_recv > R.x_cap ? relay_recv_grow(R, n_recv) : SHD_OK;
        ctx->h_pin[44] = (uint64_t)gs;
        if (hipMemcpyAsync(agree + me, ctx->h_pin + 44, 8, hipMemcpyHostToDevice, s) != hipSuccess && gs == SHD_OK)
            gs = SHD_ERR_HIP;   // (the row still goes out: the peers wait for it)
        SHD_TRY(C.all_gather(agree + me, agree, 8, s));
        std::vector<uint64_t> a(world);
        SHD_HIP(hipMemcpyAsync(a.data(), agree, world * 8, hipMemcpyDeviceToHost, s));
        SHD_HIP(hipStreamSynchronize(s));   // (a failed read-back of the agreement: fatal, as above)
        for (uint32_t q = 0; q < world; ++q)
            if ((shd_status)a[q] != SHD_OK) return (shd_status)a[q];
    }
    // 3. the exchange: part 0 is the sender's status after the gather (every rank learns every
    //    peer's, under RCCL too), part 1 the records of rank r's bins as the stamp laid them out
    //    (own: none)
    uint64_t* xst = R.xs_st.as<uint64_t>();
    if (st_post != SHD_OK || R.xs_st_dirty) {
        if (hipMemsetD32Async(xst, (uint32_t)st_post, 1, s) != hipSuccess && st_post == SHD_OK) st_post = SHD_ERR_HIP;
        R.xs_st_dirty = st_post != SHD_OK;
    }
    std::vector<const void*> sp(2 * (size_t)world);
    std::vector<void*> rp(2 * (size_t)world);
    std::vector<size_t> sb(2 * (size_t)world), rb(2 * (size_t)world);
    uint64_t sent_before = 0, recv_before = 0;
    for (uint32_t r = 0; r < world; ++r) {
        sp[2 * r] = xst;
        sb[2 * r] = r == me ? 0 : 8;
        rp[2 * r] = xst + 1 + r;
        rb[2 * r] = r == me ? 0 : 8;
        sp[2 * r + 1] = R.rec.as<uint4>() + sent_before;
        sb[2 * r + 1] = r == me ? 0 : (size_t)M(me, r) * 16;
        sent_before += M(me, r);
        rp[2 * r + 1] = R.x_rrec.as<uint4>() + recv_before;
        rb[2 * r + 1] = r == me ? 0 : (size_t)M(r, me) * 16;
        if (r != me) recv_before += M(r, me);
    }
    SHD_TRY(C.exchange(2, sp.data(), sb.data(), rp.data(), rb.data(), s, st_post));   // agreed (LocalComm, HostComm)
    // 4. the bin sort of this rank's bins over every sender's records; it also combines the
    //    statuses of part 0, which come back with the event count (no collective follows)
    uint32_t own_lo = 0, own_hi = 0;
    shard_range(H, (int)world, (int)me, &own_lo, &own_hi);
    const uint32_t n_own = own_hi - own_lo;
    const uint32_t fb_me = xsh.first_bin(me), nb = xsh.first_bin(me + 1) - fb_me;
    uint32_t kq = 0;
    while ((kq ? 2 * kq : 1u) < world) kq = kq ? 2 * kq : 1u;
    XSrc xs{world, me, fb_me, n_bins + 1, kq, R.xs_sc.as<uint32_t>(), xb, xb + world, R.rec.as<uint4>(),
            xst + 1, (uint32_t)st_post};
    if (nb) {
        V7Out vo{R.m_deliver.as<uint64_t>(), R.m_src.as<uint32_t>(), R.m_seq.as<uint64_t>(), R.m_pkt.as<uint32_t>(),
                 nullptr, rd->round_end};
        bin_sort_v7<true><<<nb, kB7Threads, 0, s>>>(n_own, nb, nullptr, R.x_rrec.as<uint4>(),
                                                    R.bin_lb.as<unsigned long long>(), R.m_off.as<uint32_t>(), vo,
                                                    nullptr, ctx->knobs.get(K_B7_STOP, 0), xs);   // (stop: tuning only)
    } else {
        xs_fin_empty<<<1, 64, 0, s>>>(xs, R.m_off.as<uint32_t>());
    }
    SHD_HIP(hipGetLastError());
    // 5. the number of events this rank received (= its destinations' SENT events: the bins also
    //    hold the dropped packets' records, so the record matrix does not give it) and the agreed
    //    status: 16 aligned bytes holding m_off[n_own] and m_off[n_own + 1]
    SHD_TRY(readback_into(ctx, s, R.m_off.as<uint32_t>() + (n_own & ~1u), 16, R.xs_pin.as<unsigned long long>()));
    const uint32_t n_ev = R.xs_pin.as<uint32_t>()[n_own & 1u];
    const shd_status agreed = (shd_status)R.xs_pin.as<uint32_t>()[(n_own & 1u) + 1];
    // every rank: nothing of the hosts' state is committed (B7_STOP, tuning only: the bin sort
    // stopped before writing the count and the status)
    if (agreed != SHD_OK && ctx->knobs.get(K_B7_STOP, 0) == 0) return agreed;
    R.red_host[0] = hdr(me)[1];
    R.red_host[1] = hdr(me)[2];
    R.red_host[2] = hdr(me)[3];
    R.last_pipe = 8;   // pipeline 7's stamp, its bins exchanged and sorted by their destination ranks
    R.last_v2 = true;
    SHD_TRY(relay_commit(ctx, &lo));
    d_out->ev_off = R.m_off.as<uint32_t>();
    d_out->ev_deliver = R.m_deliver.as<uint64_t>();
    d_out->ev_src = R.m_src.as<uint32_t>();
    d_out->ev_seq = R.m_seq.as<uint64_t>();
    d_out->ev_pkt = R.m_pkt.as<uint32_t>();
    d_out->min_deliver = md;
    d_out->min_latency = ml;
    d_out->n_sent = ns;
    d_out->n_dst = n_own;
    d_out->n_events = n_ev;
    round_note(ctx, md, ml);
    R.last_recv = n_ev;
    return SHD_OK;
}

static shd_status relay_round_sharded(shd_ctx* ctx, const shd_batch* b, const shd_round* rd, shd_relay_out* d_out) {
    // (more hosts than the records' source bits: every rank has the same host count, so every
    // rank takes the packing path without asking; xs_sizing's registers also assume it)
    if (ctx->knobs.on(K_RELAY_SHARD_X24) || ctx->relay.n_hosts > kV7MaxHosts)
        return relay_round_sharded_x24(ctx, b, rd, d_out);
    bool fallback = false;
    SHD_TRY(relay_round_sharded_v7(ctx, b, rd, d_out, &fallback));
    return fallback ? relay_round_sharded_x24(ctx, b, rd, d_out) : SHD_OK;
}

// shd_relay_flush under a communicator (flush.hip): this rank's grouped sends, the CPU's draws
shd_status relay_flush_round_sharded(shd_ctx* ctx, const shd_batch* b, const shd_round* rd, shd_relay_out* o) {
    return relay_round_sharded(ctx, b, rd, o);
}

}  // namespace shd

using namespace shd;

extern "C" {

shd_status shd_relay_setup(shd_ctx* ctx, uint32_t n_hosts, const uint32_t* host_node,
                           uint32_t n_nodes, const uint64_t* lat, const float* loss,
                           const uint64_t* rng_state, const uint64_t* next_event_id) {
    if (!ctx || n_hosts == 0 || !host_node || !rng_state || !next_event_id || n_nodes == 0)
        return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    RelayState& R = ctx->relay;
    hipStream_t s = ctx->stream;
    for (uint32_t h = 0; h < n_hosts; h++)
        if (host_node[h] >= n_nodes) return SHD_ERR_INVALID;
    if ((lat == nullptr) != (loss == nullptr)) return SHD_ERR_INVALID;
    if (!lat) {
        if (!ctx->t_full || ctx->t_cols != n_nodes) return SHD_ERR_STATE;
        R.own_table = false;
    } else {
        const size_t nn = (size_t)n_nodes * n_nodes;
        SHD_TRY(R.lat.ensure(nn * 8));
        SHD_TRY(R.loss.ensure(nn * 4));
        SHD_HIP(hipMemcpyAsync(R.lat.p, lat, nn * 8, hipMemcpyHostToDevice, s));
        SHD_HIP(hipMemcpyAsync(R.loss.p, loss, nn * 4, hipMemcpyHostToDevice, s));
        R.own_table = true;
    }
    SHD_TRY(R.host_node.ensure((size_t)n_hosts * 4));
    SHD_TRY(R.rng.ensure((size_t)n_hosts * 32));
    SHD_TRY(R.next_id.ensure((size_t)n_hosts * 8));
    SHD_TRY(R.rng2.ensure((size_t)n_hosts * 32));
    SHD_TRY(R.next_id2.ensure((size_t)n_hosts * 8));
    SHD_TRY(R.counts.ensure((size_t)n_nodes * n_nodes * 8));
    SHD_HIP(hipMemcpyAsync(R.host_node.p, host_node, (size_t)n_hosts * 4, hipMemcpyHostToDevice, s));
    // under a communicator of > 1 ranks this context stamps only its shard of the hosts
    R.sharded = ctx->comm && ctx->comm->size > 1;
    uint32_t src_lo = 0, src_hi = n_hosts;
    if (R.sharded) shard_range(n_hosts, ctx->comm->size, ctx->comm->rank, &src_lo, &src_hi);
    R.src_lo = src_lo;
    R.n_src = src_hi - src_lo;
    {   // stamp workgroups take hosts in source-node order: their path gathers share table rows
        std::vector<uint32_t> ord(R.n_src);
        for (uint32_t h = 0; h < R.n_src; h++) ord[h] = src_lo + h;
        std::stable_sort(ord.begin(), ord.end(),
                         [&](uint32_t x, uint32_t y) { return host_node[x] < host_node[y]; });
        SHD_TRY(R.order.ensure(std::max<size_t>(ord.size(), 1) * 4));
        if (!ord.empty())
            SHD_HIP(hipMemcpyAsync(R.order.p, ord.data(), ord.size() * 4, hipMemcpyHostToDevice, s));
        SHD_HIP(hipStreamSynchronize(s));
    }
    // both state buffers hold every host: a round writes only its source hosts' entries into the
    // second buffer, so the others keep their values across the swap
    SHD_HIP(hipMemcpyAsync(R.rng.p, rng_state, (size_t)n_hosts * 32, hipMemcpyHostToDevice, s));
    SHD_HIP(hipMemcpyAsync(R.next_id.p, next_event_id, (size_t)n_hosts * 8, hipMemcpyHostToDevice, s));
    SHD_HIP(hipMemcpyAsync(R.rng2.p, rng_state, (size_t)n_hosts * 32, hipMemcpyHostToDevice, s));
    SHD_HIP(hipMemcpyAsync(R.next_id2.p, next_event_id, (size_t)n_hosts * 8, hipMemcpyHostToDevice, s));
    R.seq_bound = 0;   // upper bound of every next event id (grows by n_sent per round)
    for (uint32_t h = 0; h < n_hosts; h++) R.seq_bound = std::max<uint64_t>(R.seq_bound, next_event_id[h]);
    SHD_HIP(hipMemsetAsync(R.counts.p, 0, (size_t)n_nodes * n_nodes * 8, s));
    SHD_HIP(hipStreamSynchronize(s));
    R.n_hosts = n_hosts;
    R.n_nodes = n_nodes;
    if (ctx->comm) SHD_TRY(relay_shard_alloc(ctx));   // shd_relay_round_sharded at any rank count
    {   // v2 needs every path latency < 2^32 ns (max over the table)
        const uint64_t* tl = R.own_table ? R.lat.as<uint64_t>() : ctx->t_lat.as<uint64_t>();
        SHD_TRY(ctx->g_aux.ensure(8));
        SHD_HIP(hipMemsetAsync(ctx->g_aux.p, 0, 8, s));
        const uint64_t nn = (uint64_t)n_nodes * n_nodes;
        max_u64_kernel<<<(uint32_t)std::min<uint64_t>(1024, (nn + 255) / 256), 256, 0, s>>>(
            tl, nn, reinterpret_cast<unsigned long long*>(ctx->g_aux.p));
        uint64_t mx = 0;
        SHD_HIP(hipMemcpyAsync(&mx, ctx->g_aux.p, 8, hipMemcpyDeviceToHost, s));
        SHD_HIP(hipStreamSynchronize(s));
        R.table_narrow = (mx >> 32) == 0;
        if (R.table_narrow) {   // packed {lat32, loss} table: one 8-byte gather per packet
            const float* tp = R.own_table ? R.loss.as<float>() : ctx->t_loss.as<float>();
            SHD_TRY(R.path.ensure(nn * 8));
            pack_path<<<div_up(nn, 256), 256, 0, s>>>(tl, tp, nn, R.path.as<uint2>());
            SHD_HIP(hipGetLastError());
            SHD_HIP(hipStreamSynchronize(s));
        }
    }
    R.force_v1 = ctx->knobs.on(K_RELAY_FORCE_V1);
    R.force_v3 = ctx->knobs.on(K_RELAY_FORCE_V3);   // testing: radix pipeline instead of v7
    {   // bit-packed host -> node map for the LDS-resident stamp, when it fits
        uint32_t bits = 1;
        while (bits < 32 && (n_nodes - 1) >> bits) ++bits;
        const uint64_t words = ((uint64_t)n_hosts * bits + 31) / 32 + 1;
        R.hn_bits = 0;   // (SHD_RELAY_NO_LDS_MAP=1, testing: force the gather path)
        if (words * 4 + kS6FixedLds <= ctx->max_lds && !ctx->knobs.on(K_RELAY_NO_LDS_MAP)) {
            SHD_TRY(R.hn_packed.ensure(words * 4));
            pack_host_node<<<div_up(words, 256), 256, 0, s>>>(R.host_node.as<uint32_t>(), n_hosts, bits,
                                                              (uint32_t)words, R.hn_packed.as<uint32_t>());
            SHD_HIP(hipGetLastError());
            SHD_HIP(hipStreamSynchronize(s));
            R.hn_bits = bits;
            R.hn_words = (uint32_t)words;
        }
    }
    R.ready = true;
    return SHD_OK;
}

shd_status shd_relay_round_device(shd_ctx* ctx, const shd_batch* d_batch, const shd_round* round,
                                  shd_relay_out* d_out) {
    if (!ctx || !d_batch || !round || !d_out) return SHD_ERR_INVALID;
    if (!ctx->relay.ready || ctx->relay.sharded) return SHD_ERR_STATE;
    if (!d_batch->src_off || (d_batch->n_packets && (!d_batch->send_time || !d_batch->dst_host ||
                                                     !d_batch->payload)))
        return SHD_ERR_INVALID;
    if (!d_out->status || !d_out->ev_off || !d_out->ev_deliver || !d_out->ev_src ||
        !d_out->ev_seq || !d_out->ev_pkt)
        return SHD_ERR_INVALID;
    // an output slot lent by shd_equeue_batch_buffers holds lend_cap events: a round that could
    // send more would write past it, so it is refused before any kernel runs
    const EqState& Q = ctx->eq;
    if (Q.ready && Q.lend >= 0 && d_out->ev_deliver == Q.run[Q.lend].deliver.p &&
        d_batch->n_packets > Q.lend_cap)
        return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    return relay_device(ctx, d_batch, round, d_out);
}

shd_status shd_relay_round(shd_ctx* ctx, const shd_batch* batch, const shd_round* round,
                           shd_relay_out* out) {
    if (!ctx || !batch || !round || !out || !batch->src_off) return SHD_ERR_INVALID;
    RelayState& R = ctx->relay;
    if (!R.ready || R.sharded) return SHD_ERR_STATE;
    SHD_HIP(hipSetDevice(ctx->device));
    const uint64_t n = batch->n_packets;
    const uint32_t H = R.n_hosts;
    if (batch->src_off[0] != 0 || batch->src_off[H] != n) return SHD_ERR_INVALID;
    for (uint32_t h = 0; h < H; h++)
        if (batch->src_off[h + 1] < batch->src_off[h]) return SHD_ERR_INVALID;
    hipStream_t s = ctx->stream;
    const size_t nn = std::max<uint64_t>(n, 1);
    SHD_TRY(R.pk_off.ensure((size_t)(H + 1) * 4));
    SHD_TRY(R.pk_time.ensure(nn * 8));
    SHD_TRY(R.pk_dst.ensure(nn * 4));
    SHD_TRY(R.pk_pay.ensure(nn * 4));
    SHD_TRY(R.st.ensure(nn));
    SHD_TRY(R.ev_off.ensure((size_t)(H + 1) * 4));
    SHD_TRY(R.ev_deliver.ensure(nn * 8));
    SHD_TRY(R.ev_src.ensure(nn * 4));
    SHD_TRY(R.ev_seq.ensure(nn * 8));
    SHD_TRY(R.ev_pkt.ensure(nn * 4));
    SHD_HIP(hipMemcpyAsync(R.pk_off.p, batch->src_off, (size_t)(H + 1) * 4, hipMemcpyHostToDevice, s));
    if (n) {
        SHD_HIP(hipMemcpyAsync(R.pk_time.p, batch->send_time, n * 8, hipMemcpyHostToDevice, s));
        SHD_HIP(hipMemcpyAsync(R.pk_dst.p, batch->dst_host, n * 4, hipMemcpyHostToDevice, s));
        SHD_HIP(hipMemcpyAsync(R.pk_pay.p, batch->payload, n * 4, hipMemcpyHostToDevice, s));
    }
    const double* d_chance = nullptr;
    if (batch->chance && n) {
        SHD_TRY(R.pk_chance.ensure(n * 8));
        SHD_HIP(hipMemcpyAsync(R.pk_chance.p, batch->chance, n * 8, hipMemcpyHostToDevice, s));
        d_chance = R.pk_chance.as<double>();
    }
    shd_batch db{n, R.pk_off.as<uint32_t>(), R.pk_time.as<uint64_t>(), R.pk_dst.as<uint32_t>(),
                 R.pk_pay.as<uint32_t>(), d_chance};
    shd_relay_out dout{};
    dout.status = R.st.as<uint8_t>();
    dout.ev_off = R.ev_off.as<uint32_t>();
    dout.ev_deliver = R.ev_deliver.as<uint64_t>();
    dout.ev_src = R.ev_src.as<uint32_t>();
    dout.ev_seq = R.ev_seq.as<uint64_t>();
    dout.ev_pkt = R.ev_pkt.as<uint32_t>();
    SHD_TRY(relay_device(ctx, &db, round, &dout));
    const uint64_t ns = dout.n_sent;
    if (out->status && n) SHD_HIP(hipMemcpyAsync(out->status, dout.status, n, hipMemcpyDeviceToHost, s));
    if (out->ev_off) SHD_HIP(hipMemcpyAsync(out->ev_off, dout.ev_off, (size_t)(H + 1) * 4, hipMemcpyDeviceToHost, s));
    if (ns) {
        if (out->ev_deliver) SHD_HIP(hipMemcpyAsync(out->ev_deliver, dout.ev_deliver, ns * 8, hipMemcpyDeviceToHost, s));
        if (out->ev_src) SHD_HIP(hipMemcpyAsync(out->ev_src, dout.ev_src, ns * 4, hipMemcpyDeviceToHost, s));
        if (out->ev_seq) SHD_HIP(hipMemcpyAsync(out->ev_seq, dout.ev_seq, ns * 8, hipMemcpyDeviceToHost, s));
        if (out->ev_pkt) SHD_HIP(hipMemcpyAsync(out->ev_pkt, dout.ev_pkt, ns * 4, hipMemcpyDeviceToHost, s));
    }
    SHD_HIP(hipStreamSynchronize(s));
    out->min_deliver = dout.min_deliver;
    out->min_latency = dout.min_latency;
    out->n_sent = ns;
    out->n_dst = H;
    out->n_events = (uint32_t)ns;
    return SHD_OK;
}

shd_status shd_relay_round_sharded(shd_ctx* ctx, const shd_batch* d_batch, const shd_round* round,
                                   shd_relay_out* d_out) {
    if (!ctx || !d_batch || !round || !d_out) return SHD_ERR_INVALID;
    if (!ctx->comm || !ctx->relay.ready || ctx->relay.sharded != (ctx->comm->size > 1))
        return SHD_ERR_STATE;
    if (!d_batch->src_off || (d_batch->n_packets && (!d_batch->send_time || !d_batch->dst_host ||
                                                     !d_batch->payload)))
        return SHD_ERR_INVALID;
    if (d_batch->n_packets && !d_out->status) return SHD_ERR_INVALID;
    if (!ctx->relay.x_words.p || !ctx->relay.x_roff.p) return SHD_ERR_STATE;   // set up before the communicator
    SHD_HIP(hipSetDevice(ctx->device));
    return relay_round_sharded(ctx, d_batch, round, d_out);
}

shd_status shd_relay_get_host_state(shd_ctx* ctx, uint64_t* rng_state, uint64_t* next_event_id) {
    if (!ctx) return SHD_ERR_INVALID;
    RelayState& R = ctx->relay;
    if (!R.ready) return SHD_ERR_STATE;
    SHD_HIP(hipSetDevice(ctx->device));
    if (rng_state)
        SHD_HIP(hipMemcpyAsync(rng_state, R.rng.p, (size_t)R.n_hosts * 32, hipMemcpyDeviceToHost, ctx->stream));
    if (next_event_id)
        SHD_HIP(hipMemcpyAsync(next_event_id, R.next_id.p, (size_t)R.n_hosts * 8, hipMemcpyDeviceToHost, ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    return SHD_OK;
}

shd_status shd_relay_last_pipeline(const shd_ctx* ctx, int32_t* pipeline) {
    if (!ctx || !pipeline) return SHD_ERR_INVALID;
    *pipeline = ctx->relay.last_pipe;
    return SHD_OK;
}

shd_status shd_relay_set_counters(shd_ctx* ctx, int32_t enabled) {
    if (!ctx) return SHD_ERR_INVALID;
    ctx->relay.count_on = enabled != 0;
    return SHD_OK;
}

shd_status shd_path_packet_counts(shd_ctx* ctx, uint64_t* counts) {
    if (!ctx || !counts) return SHD_ERR_INVALID;
    RelayState& R = ctx->relay;
    if (!R.ready) return SHD_ERR_STATE;
    SHD_HIP(hipSetDevice(ctx->device));
    SHD_HIP(hipMemcpyAsync(counts, R.counts.p, (size_t)R.n_nodes * R.n_nodes * 8, hipMemcpyDeviceToHost, ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    return SHD_OK;
}

}  // extern "C"

#ifdef SHD_STAMP_PROF
extern "C" int shd_debug_k0_prof(unsigned long long* out) {   // 4096 x 5 words
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(shd::g_k0_prof), sizeof(unsigned long long) * 4096 * 5) != hipSuccess;
}
extern "C" int shd_debug_stamp_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(shd::g_stamp_prof), sizeof(unsigned long long) * 12) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[12] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(shd::g_stamp_prof), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif
