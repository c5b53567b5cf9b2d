// Host-side IP assignment for the routing build's caller (host code, no GPU).
//
// Reference: assign_ips (src/main/core/sim_config.rs:399-420) over IpAssignment
// (src/main/network/graph/mod.rs:354-422): hosts with a configured address first (a repeated
// address is the "IP address has already been assigned" error), then every other host, in
// HostId order, takes the next free address after the last one handed out, starting from
// 11.0.0.1 and skipping x.x.x.0 and x.x.x.255.  generate_routing_info (sim_config.rs:424-461)
// then builds the table over the nodes that own at least one address (get_nodes()).
//
// The engine's relay addresses path rows by used-node column, so this also returns, per host,
// the column of its node in the used list (WorkerShared::latency's two IpAssignment lookups,
// worker.rs:529-543, resolved once instead of per packet).
#include <algorithm>
#include <unordered_map>
#include <vector>

#include "../../include/shd_accel.h"

extern "C" {

shd_status shd_assign_ips(uint32_t n_hosts, const uint32_t* node_gml_id, const uint32_t* ip_in,
                          uint32_t* ip_out, uint32_t* used_gml, uint32_t* n_used, uint32_t* host_col,
                          uint32_t* err_host) {
    if (!node_gml_id || !ip_out || !n_used) return SHD_ERR_INVALID;
    std::unordered_map<uint32_t, uint32_t> map;   // address -> node id
    map.reserve((size_t)n_hosts * 2);
    for (uint32_t h = 0; h < n_hosts; h++) {   // configured addresses first
        if (!ip_in || ip_in[h] == 0) continue;
        if (!map.emplace(ip_in[h], node_gml_id[h]).second) {
            if (err_host) *err_host = h;
            return SHD_ERR_INVALID;   // IpPreviouslyAssignedError
        }
        ip_out[h] = ip_in[h];
    }
    uint32_t last = 11u << 24;   // 11.0.0.0: the first address handed out is 11.0.0.1
    for (uint32_t h = 0; h < n_hosts; h++) {
        if (ip_in && ip_in[h] != 0) continue;
        for (;;) {
            do {
                ++last;   // increment_address: skip .0 and .255
            } while ((last & 0xFFu) == 0 || (last & 0xFFu) == 0xFFu);
            if (map.emplace(last, node_gml_id[h]).second) break;
        }
        ip_out[h] = last;
    }
    // get_nodes(): the distinct node ids that own an address (ascending: any order gives the same
    // RoutingInfo, whose keys are GML ids)
    std::vector<uint32_t> nodes;
    nodes.reserve(map.size());
    for (const auto& kv : map) nodes.push_back(kv.second);
    std::sort(nodes.begin(), nodes.end());
    nodes.erase(std::unique(nodes.begin(), nodes.end()), nodes.end());
    *n_used = (uint32_t)nodes.size();
    if (used_gml) std::copy(nodes.begin(), nodes.end(), used_gml);
    if (host_col)
        for (uint32_t h = 0; h < n_hosts; h++)
            host_col[h] = (uint32_t)(std::lower_bound(nodes.begin(), nodes.end(), node_gml_id[h]) - nodes.begin());
    return SHD_OK;
}

}  // extern "C"
