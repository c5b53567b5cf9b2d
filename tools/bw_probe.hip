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

int main() {
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
    return 0;
}
