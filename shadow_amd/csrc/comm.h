// Multi-GPU transport of the engine: the three collectives the sharded paths
// need, behind one interface so the sharding logic is the same whatever moves the bytes.
//   RcclComm  -- one process per GPU, RCCL over xGMI (ncclAllToAll, grouped ncclSend/ncclRecv,
//                ncclAllGather); the production path.
//   LocalComm -- every rank in this process (one host thread per rank, e.g. Shadow's manager
//                driving several GPUs, or several contexts on one GPU in the tests): device
//                copies between the ranks' buffers, host barriers between phases.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stddef.h>
#include <stdint.h>

#include "../../include/shd_accel.h"

namespace shd {

// Status contract: a collective either returns the same status on every rank (LocalComm agrees
// on the lowest failing rank's status before it returns) or, for an RCCL enqueue failure, leaves
// the communicator unusable (RCCL's own rule).  Callers therefore never return between two
// collectives on a local error: they carry it into the next status agreement instead.
struct Comm {
    int rank = 0, size = 1;
    virtual ~Comm() = default;
    // send[r * count ..] goes to rank r; recv[q * count ..] comes from rank q (device u64 words)
    virtual shd_status all_to_all_u64(const uint64_t* send, uint64_t* recv, size_t count, hipStream_t s) = 0;
    // point to point with every rank in one group: part k of the message to rank r is
    // send[r * n_parts + k] (send_bytes[..]); part k of the message from rank q lands in
    // recv[q * n_parts + k] (recv_bytes[..]).  Sizes were agreed before (zero parts are skipped
    // on both sides).  local: the caller's own status on entry, a failure it carries into this
    // collective instead of returning before it -- LocalComm and HostComm agree it (every rank
    // returns the lowest failing rank's status); RCCL cannot, so a caller that needs the agreement
    // there sends the status in-band as a part of its own (relay_round_sharded_v7).
    virtual shd_status exchange(int n_parts, const void* const* send, const size_t* send_bytes,
                                void* const* recv, const size_t* recv_bytes, hipStream_t s,
                                shd_status local = SHD_OK) = 0;
    // recv holds size * bytes; rank q's send lands at recv + q * bytes (in place allowed:
    // send == recv + rank * bytes)
    virtual shd_status all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
};

// device words of shd_ctx::comm_scratch: the sharded routing build's status agreement (16 B
// per rank + this rank's 16 B) and the sharded relay's growth agreement (8 B per rank)
inline size_t comm_scratch_bytes(int n_ranks) { return ((size_t)n_ranks + 1) * 16 + (size_t)n_ranks * 8 + 64; }

// Row / host shard of rank r among n ranks: contiguous blocks of ceil(total / n).
inline void shard_range(uint32_t total, int n, int r, uint32_t* lo, uint32_t* hi) {
    const uint64_t per = ((uint64_t)total + n - 1) / n;
    const uint64_t a = std::min<uint64_t>((uint64_t)r * per, total);
    *lo = (uint32_t)a;
    *hi = (uint32_t)std::min<uint64_t>(a + per, total);
}

}  // namespace shd
