// Tuning and testing knobs of one context.  None changes a result: they pick grids, kernel
// variants or an equivalent fallback pipeline -- except TEST_FAIL, fault injection for the
// failure-agreement tests (1: a sharded relay round fails on this rank after its sizing summary
// is read; 3: the host transport's staging cannot be allocated).  Each starts from the environment variable
// SHD_<name>, read ONCE by shd_open, so a caller's environment cannot change grids between two
// builds; shd_set_knob / shd_get_knob (api.cpp) change or inspect them per context afterwards.
#pragma once
#include <stdint.h>

#include <cstdlib>
#include <cstring>

namespace shd {

#define SHD_KNOB_LIST(X)                                                                         \
    X(SSSP_NO_PAD) X(SSSP_LFLAT) X(SSSP_NO_OFFL) X(SSSP_G) X(SSSP_BLOCK) X(SSSP_NO_REORDER)      \
    X(SSSP_DYN) X(SSSP_FLAT) X(SSSP_NO_BKT) X(SSSP_WMIN) X(SSSP_SLOTS) X(SSSP_NO_LDS_LABELS)     \
    X(SSSP_RESERVE) X(FW_TILE) X(PRUNE_K) X(SSSP_REORDER) X(REORDER_MODE) X(SSSP_NO_SPREAD) X(SSSP_GLOBAL)        \
    X(SSSP_NO_DELTA) X(SSSP_DELTA) X(SSSP_STATS) X(SPIN_WAIT)                                   \
    X(PRUNE_DENSE_BUILD) X(SSSP_HUB) X(SYNC_KERNEL)                                               \
    X(EQ_COUNT_BLOCKS) X(EQ_WAVE_MERGE) X(EQ_SEARCH_ONLY) X(EQ_MAX_RUNS) X(RELAY_GROUP_SENDS) X(HIST_SCALAR) X(B7_STOP) X(RELAY_FORCE_V1)         \
    X(RELAY_FORCE_V3) X(RELAY_NO_LDS_MAP) X(MERGE_BY_EVENT) X(SHARD_CHUNK_ROWS) X(SHARD_REPLICATE_MB)             \
    X(SHARD_RESERVE_SLOTS) X(RELAY_SHARD_X24) X(FLUSH_COPY) X(PRUNE_SHAPE) X(PRUNE_SHAPE_SH) X(EQ_FOLD) X(EQ_FOLD_TAKE) X(RELAY_K0_INLINE) X(RELAY_SCAN2)   \
    X(TEST_FAIL)

enum Knob : int {
#define SHD_KNOB_ENUM(n) K_##n,
    SHD_KNOB_LIST(SHD_KNOB_ENUM)
#undef SHD_KNOB_ENUM
    K_COUNT
};

struct Knobs {
    int64_t v[K_COUNT];   // < 0: not set (the call site's built-in default applies)

    static const char* name(int k) {
        static const char* const names[K_COUNT] = {
#define SHD_KNOB_NAME(n) #n,
            SHD_KNOB_LIST(SHD_KNOB_NAME)
#undef SHD_KNOB_NAME
        };
        return k >= 0 && k < K_COUNT ? names[k] : nullptr;
    }
    static int find(const char* n) {
        if (!n) return -1;
        if (std::strncmp(n, "SHD_", 4) == 0) n += 4;   // either spelling
        for (int k = 0; k < K_COUNT; ++k)
            if (std::strcmp(n, name(k)) == 0) return k;
        return -1;
    }
    // the environment snapshot shd_open takes: SHD_<name>=<unsigned integer>
    void from_env() {
        for (int k = 0; k < K_COUNT; ++k) {
            char var[64] = "SHD_";
            std::strncat(var, name(k), sizeof(var) - 5);
            const char* s = std::getenv(var);
            v[k] = s && *s ? (int64_t)std::strtoull(s, nullptr, 10) : -1;
        }
    }
    uint32_t get(Knob k, uint32_t dflt) const { return v[k] < 0 ? dflt : (uint32_t)v[k]; }
    uint64_t get64(Knob k, uint64_t dflt) const { return v[k] < 0 ? dflt : (uint64_t)v[k]; }
    bool on(Knob k) const { return v[k] == 1; }      // "=1" switches
    bool set(Knob k) const { return v[k] >= 0; }
};

}  // namespace shd
