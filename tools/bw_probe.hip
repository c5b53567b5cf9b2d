// Memory-pattern probe for the relay stamp (tuning tool, not part of the library):
//   A  lane per packet, packets in batch order: read 24 B (time, dst, payload, draw), write 21 B
//   B  the same bytes, packets visited per host group (64 hosts in node order, per-host ranges)
//   C  B + one random 4-byte gather per packet into a 400 KB host -> node table
//   D  A + the same random gather
// hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o tools/bw_probe && tools/bw_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <string>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Buf {
    const uint64_t* t; const uint32_t* d; const uint32_t* p; const uint64_t* r;
    uint8_t* st; uint32_t* key; uint4* rec; const uint32_t* hn;
};

__global__ __launch_bounds__(256) void kA(Buf b, uint32_t n, int gather) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint64_t t = b.t[i];
        uint32_t d = b.d[i];
        const uint32_t p = b.p[i];
        const uint64_t r = b.r[i];
        if (gather) d = b.hn[d];
        b.st[i] = (uint8_t)(t ^ r);
        b.key[i] = d + p;
        b.rec[i] = make_uint4((uint32_t)t, d, p, (uint32_t)r);
    }
}

__global__ __launch_bounds__(256) void kB(Buf b, const uint32_t* order, const uint32_t* off,
                                          uint32_t H, int gather) {
    __shared__ uint32_t s_beg[64], s_pre[65];
    const uint32_t tid = threadIdx.x, h0 = blockIdx.x * 64, nh = min(64u, H - h0);
    if (tid < 64) {
        uint32_t len = 0;
        if (tid < nh) {
            const uint32_t h = order[h0 + tid];
            s_beg[tid] = off[h];
            len = off[h + 1] - off[h];
        }
        uint32_t incl = len;
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if ((tid & 63) >= o) incl += y;
        }
        if (tid < nh) s_pre[tid + 1] = incl;
        if (tid == 0) s_pre[0] = 0;
    }
    __syncthreads();
    const uint32_t T = s_pre[nh];
    for (uint32_t gp = tid; gp < T; gp += 256) {
        uint32_t lo = 0, hi = nh;
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (s_pre[m] <= gp) lo = m; else hi = m;
        }
        const uint32_t i = s_beg[lo] + gp - s_pre[lo];
        const uint64_t t = b.t[i];
        uint32_t d = b.d[i];
        const uint32_t p = b.p[i];
        const uint64_t r = b.r[i];
        if (gather) d = b.hn[d];
        b.st[i] = (uint8_t)(t ^ r);
        b.key[i] = d + p;
        b.rec[i] = make_uint4((uint32_t)t, d, p, (uint32_t)r);
    }
}


// P: persistent workgroup per CU (1024 threads, 4 positions each per chunk) over host groups
__global__ __launch_bounds__(1024) void kP(Buf b, const uint32_t* order, const uint32_t* off,
                                           uint32_t H, int gather) {
    __shared__ uint32_t s_beg[64], s_pre[65];
    __shared__ uint16_t s_flag[4096];
    const uint32_t tid = threadIdx.x, ng = (H + 63) / 64;
    for (uint32_t g = blockIdx.x; g < ng; g += gridDim.x) {
        const uint32_t h0 = g * 64, nh = min(64u, H - h0);
        __syncthreads();
        if (tid < 64) {
            uint32_t len = 0;
            if (tid < nh) {
                const uint32_t h = order[h0 + tid];
                s_beg[tid] = off[h];
                len = off[h + 1] - off[h];
            }
            uint32_t incl = len;
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (tid >= o) incl += y;
            }
            if (tid < nh) s_pre[tid + 1] = incl;
            if (tid == 0) s_pre[0] = 0;
        }
        __syncthreads();
        const uint32_t T = s_pre[nh];
        for (uint32_t c0 = 0; c0 < T; c0 += 4096) {
            const uint32_t cn = min(4096u, T - c0);
            uint32_t idx[4];
            uint64_t t[4], r[4];
            uint32_t d[4], p[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t gp = c0 + min(tid + 1024u * i, cn - 1);
                uint32_t lo = 0, hi = nh;
                while (hi - lo > 1) {
                    const uint32_t m = (lo + hi) >> 1;
                    if (s_pre[m] <= gp) lo = m; else hi = m;
                }
                idx[i] = s_beg[lo] + gp - s_pre[lo];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                t[i] = b.t[idx[i]]; d[i] = b.d[idx[i]]; p[i] = b.p[idx[i]]; r[i] = b.r[idx[i]];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (gather) d[i] = b.hn[d[i]];
                s_flag[tid + 1024 * i] = (uint16_t)(t[i] ^ r[i]);
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (tid + 1024u * i < cn) {
                    b.st[idx[i]] = (uint8_t)s_flag[tid ^ 1];
                    b.key[idx[i]] = d[i] + p[i];
                    b.rec[idx[i]] = make_uint4((uint32_t)t[i], d[i], p[i], (uint32_t)r[i]);
                }
            }
            __syncthreads();
        }
    }
}


// H: per-destination histogram with device-scope atomics (no return)
__global__ __launch_bounds__(256) void kH(const uint32_t* d, uint32_t n, uint32_t* cnt) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        atomicAdd(&cnt[d[i]], 1u);
}
// S: 16-byte records scattered to pseudo-random unique slots
__global__ __launch_bounds__(256) void kS(const uint32_t* d, uint32_t n, uint4* out) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint32_t j = (uint32_t)(((uint64_t)i * 2654435761ull) % n);
        out[j] = make_uint4(i, d[i], 0, 0);
    }
}
// SA: claim a slot in the destination bucket with a returning atomic, write the record there
__global__ __launch_bounds__(256) void kSA(const uint32_t* d, uint32_t n, uint32_t* cur, uint4* out) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint32_t slot = atomicAdd(&cur[d[i]], 1u);
        out[slot % n] = make_uint4(i, d[i], 0, 0);
    }
}

// Q: kP plus the stamp's extras, switchable: MAP = destination node from a 125 KB bit-packed
// LDS table, ROWS = (lat, loss) from a path row staged in LDS per group
template <bool MAP, bool ROWS>
__global__ __launch_bounds__(1024) void kQ(Buf b, const uint32_t* order, const uint32_t* off,
                                           uint32_t H, const uint32_t* packed, uint32_t n_words,
                                           const uint2* path) {
    extern __shared__ uint32_t s_tbl[];
    __shared__ uint32_t s_beg[64], s_pre[65];
    __shared__ uint16_t s_flag[4096];
    __shared__ uint2 s_rows[1000];
    const uint32_t tid = threadIdx.x, ng = (H + 63) / 64;
    if (MAP) for (uint32_t i = tid; i < n_words; i += 1024) s_tbl[i] = packed[i];
    for (uint32_t g = blockIdx.x; g < ng; g += gridDim.x) {
        const uint32_t h0 = g * 64, nh = min(64u, H - h0);
        __syncthreads();
        if (tid < 64) {
            uint32_t len = 0;
            if (tid < nh) {
                const uint32_t h = order[h0 + tid];
                s_beg[tid] = off[h];
                len = off[h + 1] - off[h];
            }
            uint32_t incl = len;
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (tid >= o) incl += y;
            }
            if (tid < nh) s_pre[tid + 1] = incl;
            if (tid == 0) s_pre[0] = 0;
        }
        if (ROWS) for (uint32_t e = tid; e < 1000; e += 1024) s_rows[e] = path[(size_t)(g % 1000) * 1000 + e];
        __syncthreads();
        const uint32_t T = s_pre[nh];
        for (uint32_t c0 = 0; c0 < T; c0 += 4096) {
            const uint32_t cn = min(4096u, T - c0);
            uint32_t idx[4];
            uint64_t t[4], r[4];
            uint32_t d[4], p[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t gp = c0 + min(tid + 1024u * i, cn - 1);
                uint32_t lo = 0, hi = nh;
                while (hi - lo > 1) {
                    const uint32_t m = (lo + hi) >> 1;
                    if (s_pre[m] <= gp) lo = m; else hi = m;
                }
                idx[i] = s_beg[lo] + gp - s_pre[lo];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                t[i] = b.t[idx[i]]; d[i] = b.d[idx[i]]; p[i] = b.p[idx[i]]; r[i] = b.r[idx[i]];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t dn = d[i] % 1000;
                if (MAP) {
                    const uint32_t o = d[i] * 10, w = o >> 5, sh = o & 31;
                    uint64_t v = s_tbl[w];
                    if (sh + 10 > 32) v |= (uint64_t)s_tbl[w + 1] << 32;
                    dn = (uint32_t)(v >> sh) & 1023u;
                }
                if (ROWS) {
                    const uint2 pp = s_rows[dn];
                    t[i] += pp.x;
                    r[i] ^= pp.y;
                } else {
                    t[i] += dn;
                }
                s_flag[tid + 1024 * i] = (uint16_t)(t[i] ^ r[i]);
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (tid + 1024u * i < cn) {
                    b.st[idx[i]] = (uint8_t)s_flag[tid ^ 1];
                    b.key[idx[i]] = d[i] + p[i];
                    b.rec[idx[i]] = make_uint4((uint32_t)t[i], d[i], p[i], (uint32_t)r[i]);
                }
            }
            __syncthreads();
        }
    }
}

// W: relay_stamp_v7's structure -- persistent 1024-thread workgroup, 64-host groups, each wave
// walks 4 hosts' ranges together 64 sends per step, no barriers inside a group
__global__ __launch_bounds__(1024) void kW(Buf b, const uint32_t* order, const uint32_t* off, uint32_t H) {
    __shared__ uint32_t s_beg[64], s_len[64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6, ng = (H + 63) / 64;
    for (uint32_t g = blockIdx.x; g < ng; g += gridDim.x) {
        const uint32_t h0 = g * 64, nh = min(64u, H - h0);
        __syncthreads();
        if (tid < nh) {
            const uint32_t h = order[h0 + tid];
            s_beg[tid] = off[h];
            s_len[tid] = off[h + 1] - off[h];
        }
        __syncthreads();
        uint32_t beg[4], len[4], maxlen = 0, anyb = 0;
        for (int q = 0; q < 4; ++q) {
            const uint32_t j = w + 16 * q;
            beg[q] = j < nh ? s_beg[j] : 0u;
            len[q] = j < nh ? s_len[j] : 0u;
            if (len[q] > maxlen) { maxlen = len[q]; anyb = beg[q]; }
        }
        for (uint32_t k0 = 0; k0 < maxlen; k0 += 64) {
            const uint32_t kk = k0 + lane;
            uint32_t idx[4], d[4], p[4];
            uint64_t t[4], r[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) idx[q] = len[q] ? beg[q] + min(kk, len[q] - 1) : anyb;
#pragma unroll
            for (int q = 0; q < 4; ++q) { t[q] = b.t[idx[q]]; d[q] = b.d[idx[q]]; p[q] = b.p[idx[q]]; r[q] = b.r[idx[q]]; }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (kk >= len[q]) continue;
                const uint32_t i = beg[q] + kk;
                b.st[i] = (uint8_t)(t[q] ^ r[q]);
                b.key[i] = d[q] + p[q];
                b.rec[i] = make_uint4((uint32_t)t[q], d[q], p[q], (uint32_t)r[q]);
            }
        }
    }
}

int main(int argc, char** argv) {
    const char* only = argc > 1 ? argv[1] : nullptr;   // run only the cases with this prefix
    const uint32_t H = 100000, N = 10000000;
    std::mt19937_64 g(4);
    std::vector<uint32_t> cnt(H, 0);
    for (uint32_t i = 0; i < N; ++i) cnt[g() % H]++;
    std::vector<uint32_t> off(H + 1, 0), order(H), hn(H), dst(N);
    for (uint32_t h = 0; h < H; ++h) off[h + 1] = off[h] + cnt[h];
    for (uint32_t h = 0; h < H; ++h) { order[h] = h; hn[h] = h % 1000; }
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return hn[a] < hn[b]; });
    for (uint32_t i = 0; i < N; ++i) dst[i] = g() % H;
    uint64_t *t, *r; uint32_t *d, *p, *key, *o_off, *o_ord, *o_hn; uint8_t* st; uint4* rec;
    CK(hipMalloc(&t, N * 8)); CK(hipMalloc(&r, N * 8)); CK(hipMalloc(&d, N * 4)); CK(hipMalloc(&p, N * 4));
    CK(hipMalloc(&key, N * 4)); CK(hipMalloc(&st, N)); CK(hipMalloc(&rec, (size_t)N * 16));
    CK(hipMalloc(&o_off, (H + 1) * 4)); CK(hipMalloc(&o_ord, H * 4)); CK(hipMalloc(&o_hn, H * 4));
    CK(hipMemset(t, 1, N * 8)); CK(hipMemset(r, 2, N * 8)); CK(hipMemset(p, 3, N * 4));
    CK(hipMemcpy(d, dst.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(o_off, off.data(), (H + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(o_ord, order.data(), H * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(o_hn, hn.data(), H * 4, hipMemcpyHostToDevice));
    Buf b{t, d, p, r, st, key, rec, o_hn};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        if (only && std::string(name).rfind(only, 0) != 0) return 0;
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int k = 0; k < 10; ++k) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%-40s %8.1f us  %6.2f TB/s (45 B/packet)\n", name, ms * 100.0, 45.0 * N / (ms * 1e-4) / 1e12);
        return 0;
    };
    run("A batch order", [&] { kA<<<2048, 256>>>(b, N, 0); });
    run("A batch order, grid = N/256", [&] { kA<<<(N + 255) / 256, 256>>>(b, N, 0); });
    run("B node-ordered host groups", [&] { kB<<<(H + 63) / 64, 256>>>(b, o_ord, o_off, H, 0); });
    run("C node-ordered + node gather", [&] { kB<<<(H + 63) / 64, 256>>>(b, o_ord, o_off, H, 1); });
    run("D batch order + node gather", [&] { kA<<<2048, 256>>>(b, N, 1); });
    std::vector<uint32_t> ident(H);
    for (uint32_t h = 0; h < H; ++h) ident[h] = h;
    uint32_t* o_id;
    CK(hipMalloc(&o_id, H * 4));
    CK(hipMemcpy(o_id, ident.data(), H * 4, hipMemcpyHostToDevice));
    run("B batch-ordered host groups", [&] { kB<<<(H + 63) / 64, 256>>>(b, o_id, o_off, H, 0); });
    run("P persistent, node-ordered", [&] { kP<<<256, 1024>>>(b, o_ord, o_off, H, 0); });
    run("P persistent, batch-ordered", [&] { kP<<<256, 1024>>>(b, o_id, o_off, H, 0); });
    run("P persistent x2/CU, node-ordered", [&] { kP<<<512, 1024>>>(b, o_ord, o_off, H, 0); });
    run("P non-persistent, node-ordered", [&] { kP<<<(H + 63) / 64, 1024>>>(b, o_ord, o_off, H, 0); });
    uint32_t* pk;
    uint2* pth;
    const uint32_t nw = (H * 10 + 31) / 32;
    CK(hipMalloc(&pk, nw * 4 + 4));
    CK(hipMemset(pk, 0, nw * 4 + 4));
    CK(hipMalloc(&pth, 1000 * 1000 * 8));
    CK(hipMemset(pth, 1, 1000 * 1000 * 8));
    CK(hipFuncSetAttribute((const void*)kQ<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, nw * 4));
    CK(hipFuncSetAttribute((const void*)kQ<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, nw * 4));
    run("Q0 kP-equivalent", [&] { kQ<false, false><<<256, 1024>>>(b, o_ord, o_off, H, pk, nw, pth); });
    run("Q1 + LDS map", [&] { kQ<true, false><<<256, 1024, nw * 4>>>(b, o_ord, o_off, H, pk, nw, pth); });
    run("Q2 + rows", [&] { kQ<false, true><<<256, 1024>>>(b, o_ord, o_off, H, pk, nw, pth); });
    run("Q3 + LDS map + rows", [&] { kQ<true, true><<<256, 1024, nw * 4>>>(b, o_ord, o_off, H, pk, nw, pth); });
    run("W v7 structure, node-ordered", [&] { kW<<<256, 1024>>>(b, o_ord, o_off, H); });
    run("W v7 structure, batch-ordered", [&] { kW<<<256, 1024>>>(b, o_id, o_off, H); });
    run("W v7 structure, 1563 groups", [&] { kW<<<(H + 63) / 64, 1024>>>(b, o_ord, o_off, H); });
    uint32_t* hcnt;
    uint4* sc;
    CK(hipMalloc(&hcnt, H * 4 * 2));
    CK(hipMalloc(&sc, (size_t)N * 16));
    CK(hipMemset(hcnt, 0, H * 8));
    run("H atomic histogram (100k bins)", [&] { kH<<<4096, 256>>>(d, N, hcnt); });
    run("S random 16-B scatter", [&] { kS<<<4096, 256>>>(d, N, sc); });
    run("SA atomic slot claim + 16-B scatter", [&] { kSA<<<4096, 256>>>(d, N, hcnt, sc); });
    return 0;
}
