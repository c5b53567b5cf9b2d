// Wave-level exchanges and sorts shared by the relay's destination sorts (relay.hip) and the
// event queues' per-host merge (equeue.hip): 64-lane gfx950 waves, keys held NPL per lane
// (element e = lane + 64 c).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace shd {

// xor lane exchange inside a wave for a compile-time distance (the bitonic loops below are fully
// unrolled, so j folds): DPP quad_perm for 1 and 2, DPP row_ror:8 for 8, ds_swizzle (bitmask
// mode) for 4, v_permlane16_swap / v_permlane32_swap (gfx950) for 16 and 32.
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, uint32_t j, uint32_t lane) {
    switch (j) {
        case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
        case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
        case 4: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (4 << 10) | 0x1F);
        case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
        case 16: {
            const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            return (lane & 16) ? r[0] : r[1];
        }
        default: {
            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            return (lane & 32) ? r[0] : r[1];
        }
    }
}

// Bitonic sort of 64 * NPL 32-bit keys held NPL per lane (element e = lane + 64 c), ascending.
template <int NPL>
__device__ __forceinline__ void wave_bitonic32(uint32_t (&k)[NPL], uint32_t lane) {
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
                        const uint32_t x = k[c], y = k[c | cj];
                        k[c] = asc ? min(x, y) : max(x, y);
                        k[c | cj] = asc ? max(x, y) : min(x, y);
                    }
                }
            } else {
#pragma unroll
                for (int c = 0; c < NPL; ++c) {
                    const uint32_t o = xor_lane(k[c], j, lane);
                    const bool take_min = ((lane & j) == 0) == (((lane + 64u * c) & kk) == 0);
                    k[c] = take_min ? min(o, k[c]) : max(o, k[c]);
                }
            }
        }
    }
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v, uint32_t lane) {
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) v = min(v, xor_lane(v, o, lane));
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v, uint32_t lane) {
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) v = max(v, xor_lane(v, o, lane));
    return v;
}


// Bitonic sort of 64 * NPL keys held NPL per lane (element e = lane + 64 c), ascending.
template <int NPL>
__device__ __forceinline__ void wave_bitonic(uint64_t (&k)[NPL], uint32_t lane) {
#pragma unroll
    for (uint32_t kk = 2; kk <= 64u * NPL; kk <<= 1) {
#pragma unroll
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            if (j >= 64) {               // partner in another register of the same lane
                const uint32_t cj = j / 64;
#pragma unroll
                for (int c = 0; c < NPL; ++c) {
                    if ((c & cj) == 0) {
                        const uint32_t e = lane + 64u * c;
                        const bool asc = (e & kk) == 0;
                        const uint64_t x = k[c], y = k[c | cj];
                        const bool sw = (y < x) == asc;   // equal keys: the swap is a no-op
                        k[c] = sw ? y : x;
                        k[c | cj] = sw ? x : y;
                    }
                }
            } else {                     // partner lane ^ j
#pragma unroll
                for (int c = 0; c < NPL; ++c) {
                    const uint32_t e = lane + 64u * c;
                    const uint32_t olo = xor_lane((uint32_t)k[c], j, lane);
                    const uint32_t ohi = xor_lane((uint32_t)(k[c] >> 32), j, lane);
                    const uint64_t o = ((uint64_t)ohi << 32) | olo;
                    const bool lower = (lane & j) == 0;
                    const bool asc = (e & kk) == 0;
                    const bool take_min = lower == asc;
                    k[c] = (o < k[c]) == take_min ? o : k[c];
                }
            }
        }
    }
}

}  // namespace shd
