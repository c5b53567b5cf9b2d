// Shared host/device helpers for the shd_accel engine (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <string>

#include "../../include/shd_accel.h"

#define SHD_HIP(call)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "shd_accel: %s failed: %s (%s:%d)\n", #call,             \
                         hipGetErrorString(e_), __FILE__, __LINE__);                      \
            return SHD_ERR_HIP;                                                           \
        }                                                                                 \
    } while (0)

#define SHD_TRY(expr)                         \
    do {                                      \
        shd_status s_ = (expr);               \
        if (s_ != SHD_OK) return s_;          \
    } while (0)

namespace shd {

constexpr uint32_t kLat32Inf = 0xFFFFFFFFu;          // "unreached" in narrow (u32) labels
constexpr uint64_t kKeyInf = 0xFFFFFFFFFFFFFFFFull;  // packed (lat32 << 32 | loss bits) infinity

// PathProperties::add loss part (graph/mod.rs:324-333) with q = 1f32 - p precomputed:
//   1f32 - (1f32 - p) * (1f32 - e)  ==  1f32 - (q_p * q_e)      (each q rounded exactly as Rust)
// __fmul_rn / __fsub_rn forbid contraction into an FMA whatever the -ffp-contract setting.
__device__ __forceinline__ float fold_q(float q_p, float q_e) {
    return __fsub_rn(1.0f, __fmul_rn(q_p, q_e));
}
__device__ __forceinline__ float one_minus(float p) { return __fsub_rn(1.0f, p); }

// Lexicographic (latency, loss) key: loss is in [0,1] and never -0.0 on a folded path, so its
// IEEE bits order like the value and the u64 compares lexicographically.
__host__ __device__ __forceinline__ uint64_t pack_key(uint32_t lat, float loss) {
    return ((uint64_t)lat << 32) | (uint64_t)__builtin_bit_cast(uint32_t, loss);
}
__host__ __device__ __forceinline__ uint32_t key_lat(uint64_t k) { return (uint32_t)(k >> 32); }
__host__ __device__ __forceinline__ float key_loss(uint64_t k) {
    return __builtin_bit_cast(float, (uint32_t)(k & 0xFFFFFFFFu));
}

inline uint32_t div_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

}  // namespace shd
