// Hand-written scans and the destination radix sort of the fallback relay pipelines (no library
// kernels on any path).
//
// scan_excl2: exclusive scans of one or two u32 arrays in ONE launch: a tile of 8192 entries per
// 1024-thread workgroup (8 per thread, two 16-byte loads), a block scan, then a decoupled
// look-back over the earlier tiles' published sums (a workgroup's tile comes from a ticket
// counter, so a tile waits only on tiles whose workgroups already run).  Each tile's state word is epoch << 34 | flag << 32 | value (flag 1:
// the tile's own sum, 2: the inclusive prefix); the epoch changes every launch, so the states are
// never cleared between launches.
//
// radix_sort_dst: stable LSD radix sort of (u32 key, 16-byte record) pairs, 6 bits per pass --
// a per-tile digit histogram, one scan of the digit-major counts, and a stable scatter (each
// thread ranks its 16 consecutive keys, a block scan orders the tile digit-major).
#pragma once
#include "ctx.h"

namespace shd {

constexpr uint32_t kScanT = 1024, kScanV = 8, kScanTile = kScanT * kScanV;

__device__ __forceinline__ void scan_load8(const uint32_t* in, uint64_t at, uint64_t n, uint32_t* v, bool vec) {
    if (in && vec && at + kScanV <= n) {
        const uint4 x = *reinterpret_cast<const uint4*>(in + at);
        const uint4 y = *reinterpret_cast<const uint4*>(in + at + 4);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    } else {
#pragma unroll
        for (uint32_t i = 0; i < kScanV; ++i) v[i] = in && at + i < n ? in[at + i] : 0u;
    }
}

// A workgroup's tile index: the next ticket of this launch, not blockIdx.x -- a tile then only
// waits on tiles whose workgroups are already running, whatever order the dispatcher uses.  The
// ticket word holds epoch << 32 | tickets taken; the first taker of a new epoch restarts it at 1.
__device__ __forceinline__ uint32_t scan_ticket(unsigned long long* t, uint32_t epoch) {
    unsigned long long v = __hip_atomic_load(t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        const unsigned long long want =
            (uint32_t)(v >> 32) == epoch ? v + 1 : ((unsigned long long)epoch << 32) | 1ull;
        const unsigned long long prev = atomicCAS(t, v, want);
        if (prev == v) return (uint32_t)want - 1u;
        v = prev;
    }
}

// in-place is allowed (a_out == a_in): a thread reads its 8 entries before any write
static __global__ __launch_bounds__(1024) void scan_excl2_kernel(uint64_t n, const uint32_t* a_in, uint32_t* a_out,
                                                                 const uint32_t* b_in, uint32_t* b_out,
                                                                 unsigned long long* __restrict__ state,
                                                                 uint32_t epoch) {
    __shared__ uint32_t s_w[16][2];
    __shared__ uint32_t s_pref[2];
    __shared__ uint32_t s_tile;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // state[0]: the launch's ticket word; tile t's states at state[2 + 2t]
    if (tid == 0) s_tile = scan_ticket(state, epoch);
    __syncthreads();
    const uint32_t tile = s_tile;
    state += 2;
    const uint64_t at = (uint64_t)tile * kScanTile + (uint64_t)tid * kScanV;
    // 16-byte vector accesses when every array allows them (a caller's ev_off may be offset)
    const bool vec = ((reinterpret_cast<uintptr_t>(a_in) | reinterpret_cast<uintptr_t>(a_out) |
                       reinterpret_cast<uintptr_t>(b_in) | reinterpret_cast<uintptr_t>(b_out)) & 15u) == 0;
    uint32_t va[kScanV], vb[kScanV];
    scan_load8(a_in, at, n, va, vec);
    scan_load8(b_in, at, n, vb, vec);
    uint32_t sa = 0, sb = 0;
#pragma unroll
    for (uint32_t i = 0; i < kScanV; ++i) {
        sa += va[i];
        sb += vb[i];
    }
    uint32_t ia = sa, ib = sb;   // inclusive within the wave
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t ya = __shfl_up(ia, o), yb = __shfl_up(ib, o);
        if (lane >= o) {
            ia += ya;
            ib += yb;
        }
    }
    if (lane == 63) {
        s_w[w][0] = ia;
        s_w[w][1] = ib;
    }
    __syncthreads();
    uint32_t wa = 0, wb = 0, ta = 0, tb = 0;   // waves before this one; the tile's total
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t xa = s_w[k][0], xb = s_w[k][1];
        if (k < w) {
            wa += xa;
            wb += xb;
        }
        ta += xa;
        tb += xb;
    }
    if (w == 0) {
        // wave 0: publish the tile's sums, then a wave-wide look-back -- lane l reads tile - 1 - l
        // for both arrays at once, so the predecessors' states come in one round trip per 64
        // tiles instead of one dependent load per tile and array (the 13-tile scan of a
        // 100k-host queue advance: 12.5 -> 10.4 us)
        unsigned long long* st = state + (size_t)tile * 2;
        const unsigned long long tag = (unsigned long long)epoch << 34;
        uint32_t ea = 0, eb = 0;
        if (tile != 0) {
            if (lane == 0) {
                __hip_atomic_store(&st[0], tag | (1ull << 32) | ta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&st[1], tag | (1ull << 32) | tb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            bool da = false, db = false;   // array done (its nearest inclusive state reached)
            for (int64_t hi = (int64_t)tile - 1; !(da && db);) {
                const int64_t j = hi - (int64_t)lane;
                unsigned long long v[2];
#pragma unroll
                for (uint32_t k = 0; k < 2; ++k)   // (before tile 0: an inclusive 0)
                    v[k] = j >= 0 ? __hip_atomic_load(&state[(size_t)j * 2 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : tag | (2ull << 32);
                bool again = false;
                uint32_t add[2] = {0u, 0u};
                bool fin[2] = {false, false};
#pragma unroll
                for (uint32_t k = 0; k < 2; ++k) {
                    if (k == 0 ? da : db) {
                        fin[k] = true;
                        continue;
                    }
                    const uint32_t f = (uint32_t)(v[k] >> 32) & 3u;
                    const bool ok = (uint32_t)(v[k] >> 34) == epoch && f != 0;
                    const uint64_t incl_m = __ballot(ok && f == 2), bad_m = __ballot(!ok);
                    const uint32_t fi = incl_m ? (uint32_t)__builtin_ctzll(incl_m) : 64u;
                    const uint64_t upto = fi == 64 ? ~0ull : ((2ull << fi) - 1ull);
                    if (bad_m & upto) {   // a state this walk needs is not published yet
                        again = true;
                        continue;
                    }
                    add[k] = lane <= fi ? (uint32_t)v[k] : 0u;
                    fin[k] = fi < 64;
                }
                if (again) {   // (whole window again: the other array's part is redone with it)
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
#pragma unroll
                for (uint32_t k = 0; k < 2; ++k)
                    for (int o = 32; o > 0; o >>= 1) add[k] += (uint32_t)__shfl_xor((int)add[k], o);
                if (!da) ea += add[0];
                if (!db) eb += add[1];
                da = da || fin[0];
                db = db || fin[1];
                hi -= 64;
            }
        }
        if (lane == 0) {
            __hip_atomic_store(&st[0], tag | (2ull << 32) | (uint32_t)(ea + ta), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&st[1], tag | (2ull << 32) | (uint32_t)(eb + tb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_pref[0] = ea;
            s_pref[1] = eb;
        }
    }
    __syncthreads();
    uint32_t ra = s_pref[0] + wa + ia - sa, rb = s_pref[1] + wb + ib - sb;   // this thread's exclusive prefix
    uint32_t oa[kScanV], ob[kScanV];
#pragma unroll
    for (uint32_t i = 0; i < kScanV; ++i) {
        oa[i] = ra;
        ob[i] = rb;
        ra += va[i];
        rb += vb[i];
    }
    if (vec && at + kScanV <= n) {
        *reinterpret_cast<uint4*>(a_out + at) = make_uint4(oa[0], oa[1], oa[2], oa[3]);
        *reinterpret_cast<uint4*>(a_out + at + 4) = make_uint4(oa[4], oa[5], oa[6], oa[7]);
        if (b_out) {
            *reinterpret_cast<uint4*>(b_out + at) = make_uint4(ob[0], ob[1], ob[2], ob[3]);
            *reinterpret_cast<uint4*>(b_out + at + 4) = make_uint4(ob[4], ob[5], ob[6], ob[7]);
        }
    } else {
#pragma unroll
        for (uint32_t i = 0; i < kScanV; ++i)
            if (at + i < n) {
                a_out[at + i] = oa[i];
                if (b_out) b_out[at + i] = ob[i];
            }
    }
}

// exclusive scans of n entries of a (and b; b_in / b_out may be null)
static shd_status scan_excl2(ScanScratch& S, const uint32_t* a_in, uint32_t* a_out, const uint32_t* b_in,
                             uint32_t* b_out, uint64_t n, hipStream_t s) {
    if (n == 0) return SHD_OK;
    const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
    if (tiles * 16 + 16 > S.state.bytes) {   // grown: fresh states (epoch 0 is never a live epoch)
        SHD_TRY(S.state.ensure(tiles * 16 + 16));   // + the ticket word
        SHD_HIP(hipMemsetAsync(S.state.p, 0, S.state.bytes, s));
        S.epoch = 0;
    }
    if (++S.epoch >= (1u << 30)) {   // epochs wrap: clear the states once
        SHD_HIP(hipMemsetAsync(S.state.p, 0, S.state.bytes, s));
        S.epoch = 1;
    }
    scan_excl2_kernel<<<(uint32_t)tiles, kScanT, 0, s>>>(n, a_in, a_out, b_in, b_out,
                                                           S.state.as<unsigned long long>(), S.epoch);
    SHD_HIP(hipGetLastError());
    return SHD_OK;
}

// ------------------------------------------------------------------------------ radix sort
constexpr uint32_t kRsT = 256, kRsK = 16, kRsTile = kRsT * kRsK;   // 4096 pairs per tile
constexpr uint32_t kRsBits = 6, kRsDig = 1u << kRsBits;

// counts[d * n_tiles + tile] = keys of the tile with digit d
static __global__ __launch_bounds__(kRsT) void rs_hist(const uint32_t* __restrict__ keys, uint64_t n, uint32_t shift,
                                                        uint32_t n_tiles, uint32_t* __restrict__ counts) {
    __shared__ uint32_t h[kRsDig];
    const uint32_t tid = threadIdx.x, tile = blockIdx.x;
    if (tid < kRsDig) h[tid] = 0;
    __syncthreads();
    const uint64_t b = (uint64_t)tile * kRsTile;
#pragma unroll 4
    for (uint32_t j = 0; j < kRsK; ++j) {
        const uint64_t i = b + (uint64_t)j * kRsT + tid;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & (kRsDig - 1)], 1u);
    }
    __syncthreads();
    if (tid < kRsDig) counts[(size_t)tid * n_tiles + tile] = h[tid];
}

// stable scatter: thread t owns the tile's keys [t*K, t*K+K); its keys' ranks come from a
// digit-major block scan of the per-thread digit counts (LDS, u16)
static __global__ __launch_bounds__(kRsT) void rs_scatter(const uint32_t* __restrict__ kin, const uint4* __restrict__ vin,
                                                           uint32_t* __restrict__ kout, uint4* __restrict__ vout,
                                                           uint64_t n, uint32_t shift, uint32_t n_tiles,
                                                           const uint32_t* __restrict__ offs) {
    constexpr uint32_t S = kRsT + 1;   // padded row (bank spread)
    __shared__ uint16_t cnt[kRsDig * S];
    __shared__ uint32_t s_part[kRsT];
    __shared__ uint32_t s_dstart[kRsDig];
    const uint32_t tid = threadIdx.x, tile = blockIdx.x;
    const uint64_t b = (uint64_t)tile * kRsTile + (uint64_t)tid * kRsK;
    uint32_t key[kRsK], rank[kRsK];
    for (uint32_t d = 0; d < kRsDig; ++d) cnt[d * S + tid] = 0;
#pragma unroll
    for (uint32_t j = 0; j < kRsK; ++j) key[j] = b + j < n ? kin[b + j] : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t j = 0; j < kRsK; ++j) {
        if (b + j < n) {
            const uint32_t d = (key[j] >> shift) & (kRsDig - 1);
            rank[j] = cnt[d * S + tid]++;
        }
    }
    __syncthreads();
    // digit-major exclusive scan over (d, t): thread x takes row d = x / 4, columns (x % 4) * 64 ..
    const uint32_t d0 = tid >> 2, c0 = (tid & 3) * 64;
    uint32_t sum = 0;
    for (uint32_t c = 0; c < 64; ++c) sum += cnt[d0 * S + c0 + c];
    s_part[tid] = sum;
    __syncthreads();
    if (tid < 64) {   // one wave scans the 256 partial sums (4 per lane)
        uint32_t p[4], t = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            p[i] = s_part[tid * 4 + i];
            t += p[i];
        }
        uint32_t incl = t;
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (tid >= o) incl += y;
        }
        uint32_t run = incl - t;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s_part[tid * 4 + i] = run;
            run += p[i];
        }
    }
    __syncthreads();
    {
        uint32_t run = s_part[tid];
        if ((tid & 3) == 0) s_dstart[d0] = run;   // the digit's first position in the tile
        for (uint32_t c = 0; c < 64; ++c) {
            const uint32_t v = cnt[d0 * S + c0 + c];
            cnt[d0 * S + c0 + c] = (uint16_t)run;
            run += v;
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kRsK; ++j) {
        if (b + j < n) {
            const uint32_t d = (key[j] >> shift) & (kRsDig - 1);
            const uint32_t pos = cnt[d * S + tid] + rank[j];   // position in the digit-major tile
            const uint64_t gp = (uint64_t)offs[(size_t)d * n_tiles + tile] + (pos - s_dstart[d]);
            kout[gp] = key[j];
            vout[gp] = vin[b + j];
        }
    }
}

// Stable sort of n (key, record) pairs by the low `bits` bits of the key, ping-ponging between
// (k0, v0) and (k1, v1); *in_first says where the result is (true: k0 / v0).
static shd_status radix_sort_pairs(DevBuf& counts, ScanScratch& scan, uint32_t* k0, uint4* v0, uint32_t* k1, uint4* v1, uint64_t n,
                                   uint32_t bits, bool* in_first, hipStream_t s) {
    *in_first = true;
    if (n == 0) return SHD_OK;
    const uint32_t n_tiles = (uint32_t)((n + kRsTile - 1) / kRsTile);
    const uint64_t nc = (uint64_t)n_tiles * kRsDig;
    SHD_TRY(counts.ensure(nc * 4 + 16));
    uint32_t* kin = k0;
    uint4* vin = v0;
    uint32_t* kout = k1;
    uint4* vout = v1;
    for (uint32_t shift = 0; shift < bits; shift += kRsBits) {
        rs_hist<<<n_tiles, kRsT, 0, s>>>(kin, n, shift, n_tiles, counts.as<uint32_t>());
        SHD_HIP(hipGetLastError());
        SHD_TRY(scan_excl2(scan, counts.as<uint32_t>(), counts.as<uint32_t>(), nullptr, nullptr, nc, s));
        rs_scatter<<<n_tiles, kRsT, 0, s>>>(kin, vin, kout, vout, n, shift, n_tiles, counts.as<uint32_t>());
        SHD_HIP(hipGetLastError());
        std::swap(kin, kout);
        std::swap(vin, vout);
        *in_first = !*in_first;
    }
    return SHD_OK;
}

}  // namespace shd
