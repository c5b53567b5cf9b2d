// GML network-graph loader: GML text -> the edge arrays the routing build
// takes (shd_graph), natively, in one pass over the text.
//
// Reference semantics (FlyearthR/shadow):
//   src/lib/gml-parser/src/parser.rs:44-262  grammar: key, item, gml, node, edge, value (int |
//     float | string, each followed by `newline` = space0 multispace1 space0), int = digit1 as
//     i32, float = recognize_float + str::parse::<f32> (correctly rounded), string =
//     escaped_transform(is_not("\""), ...), int_as_bool, duplicate-key and 'directed' checks;
//   src/lib/gml-parser/src/lib.rs:52-57      parse() -- trailing text after the graph is ignored;
//   src/main/network/graph/mod.rs:30-113     ShadowNode / ShadowEdge try_from (messages below);
//   src/main/network/graph/mod.rs:136-183    NetworkGraph::parse: nodes in order (a repeated id
//     maps to the later node), then edges in order, source/target looked up by GML id;
//   src/main/network/graph/mod.rs:335-342    edge latency -> ns via convert(Nano).unwrap();
//   src/main/core/support/units.rs:142-178,214-280,405-438  unit strings ("<u64> <prefix><suffix>").
//
// Host code (no GPU): the reference parser is single-threaded nom; this is a hand-written
// recursive-descent scanner over the bytes with no per-token allocation.  Errors carry the
// reference's message text for every validation the reference names; grammar errors report
// the byte offset (nom's VerboseError trace is not reproduced).
#include <dlfcn.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "shd_accel.h"

struct shd_gml {
    int32_t directed = 0;
    std::vector<uint32_t> node_ids;
    std::vector<uint64_t> bw_down, bw_up;          // bits/s, UINT64_MAX = not given
    std::vector<uint32_t> src, dst;
    std::vector<uint64_t> lat_ns;
    std::vector<float> loss;
};

namespace {

enum class VT { Int, Float, Str };
struct Val {
    VT t;
    int32_t i = 0;
    float f = 0.0f;
    std::string_view s;
};
struct KV {
    std::string_view k;
    Val v;
};

struct Fail {
    shd_status st;
    std::string msg;
};

bool is_space(char c) { return c == ' ' || c == '\t'; }
bool is_multispace(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
bool is_alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
bool is_digit(char c) { return c >= '0' && c <= '9'; }

struct Scanner {
    const char* s;
    size_t n, i = 0;

    [[noreturn]] void fail(const char* what) const {
        char buf[160];
        std::snprintf(buf, sizeof(buf), "GML parse error at byte %zu: %s", i, what);
        throw Fail{SHD_ERR_INVALID, buf};
    }
    void space0() {
        while (i < n && is_space(s[i])) ++i;
    }
    void multispace0() {
        while (i < n && is_multispace(s[i])) ++i;
    }
    // recognize(tuple((space0, multispace1, space0))): multispace1 is greedy over [ \t\r\n]
    bool newline() {
        const size_t j = i;
        space0();
        if (i >= n || !is_multispace(s[i])) {
            i = j;
            return false;
        }
        multispace0();
        return true;
    }
    bool tag(std::string_view t) {
        if (n - i >= t.size() && std::memcmp(s + i, t.data(), t.size()) == 0) {
            i += t.size();
            return true;
        }
        return false;
    }
    // [a-zA-Z_][a-zA-Z0-9_]* (parser.rs:45-51; chars are tested as their low byte)
    bool key(std::string_view* out) {
        if (i >= n || !(is_alpha(s[i]) || s[i] == '_')) return false;
        size_t j = i + 1;
        while (j < n && (is_alpha(s[j]) || is_digit(s[j]) || s[j] == '_')) ++j;
        *out = std::string_view(s + i, j - i);
        i = j;
        return true;
    }
    // nom recognize_float: [+-]? (digits (. digits*)? | . digits) ([eE] [+-]? digits)? -- an
    // exponent marker without digits is a hard (cut) failure
    size_t float_len(size_t at) const {
        size_t j = at;
        if (j < n && (s[j] == '+' || s[j] == '-')) ++j;
        const size_t d0 = j;
        while (j < n && is_digit(s[j])) ++j;
        const bool int_digits = j > d0;
        bool frac_digits = false;
        if (j < n && s[j] == '.') {
            size_t k = j + 1;
            while (k < n && is_digit(s[k])) ++k;
            frac_digits = k > j + 1;
            if (int_digits || frac_digits) j = k;
        }
        if (!int_digits && !frac_digits) return 0;
        if (j < n && (s[j] == 'e' || s[j] == 'E')) {
            size_t k = j + 1;
            if (k < n && (s[k] == '+' || s[k] == '-')) ++k;
            const size_t e0 = k;
            while (k < n && is_digit(s[k])) ++k;
            if (k == e0) {
                Scanner* self = const_cast<Scanner*>(this);
                self->i = k;
                fail("float exponent without digits");
            }
            j = k;
        }
        return j - at;
    }
    // value (parser.rs:214-224): space0, then (int newline) | (float newline) | (string newline)
    Val value() {
        space0();
        const size_t start = i;
        {   // int: digit1 parsed as i32; a parse failure (too large) falls through to float
            size_t j = i;
            uint64_t v = 0;
            while (j < n && is_digit(s[j])) {
                if (v <= 0x7FFFFFFFull) v = v * 10 + (uint64_t)(s[j] - '0');   // saturates past i32
                ++j;
            }
            if (j > i) {
                if (v <= 0x7FFFFFFFull) {
                    i = j;
                    if (newline()) return Val{VT::Int, (int32_t)v, 0.0f, {}};
                    i = start;
                }
            }
        }
        if (const size_t fl = float_len(i)) {
            // Rust str::parse::<f32> and glibc strtof are both correctly rounded (ties-to-even)
            char buf[128];
            float f;
            if (fl < sizeof(buf)) {
                std::memcpy(buf, s + i, fl);
                buf[fl] = 0;
                f = std::strtof(buf, nullptr);   // ERANGE still yields the rounded value
            } else {
                const std::string big(s + i, fl);
                f = std::strtof(big.c_str(), nullptr);
            }
            i += fl;
            if (newline()) return Val{VT::Float, 0, f, {}};
            i = start;
        }
        if (tag("\"")) {
            // escaped_transform(is_not("\""), '\\', ..): the `normal` parser is_not("\"")
            // already takes backslashes, so the string is everything up to the next '"'
            const char* q = static_cast<const char*>(std::memchr(s + i, '"', n - i));
            if (!q) fail("unterminated string");
            if (q == s + i) fail("empty string");
            Val v{VT::Str, 0, 0.0f, std::string_view(s + i, (size_t)(q - (s + i)))};
            i = (size_t)(q - s) + 1;
            if (newline()) return v;
        }
        i = start;
        fail("invalid value");
    }
    // space0 '[' newline many_till((key, value), ']') + duplicate-key check, then newline
    // the block's pairs are appended to `all`; returns where they start
    size_t kv_block(std::vector<KV>* all) {
        space0();
        if (!tag("[")) fail("expected '['");
        if (!newline()) fail("expected a newline after '['");
        const size_t b0 = all->size();
        while (!tag("]")) {
            std::string_view k;
            if (!key(&k)) fail("expected a key");
            Val v = value();
            all->push_back(KV{k, v});
        }
        for (size_t a = b0; a < all->size(); ++a)
            for (size_t b = a + 1; b < all->size(); ++b)
                if ((*all)[a].k == (*all)[b].k) throw Fail{SHD_ERR_INVALID, "Duplicate keys are not supported"};
        if (!newline()) fail("expected a newline after ']'");
        return b0;
    }
};

struct Block {   // one node / edge: pairs [b, e) of the flat pair array
    const KV* b;
    const KV* e;
};

const Val* find(const Block& blk, std::string_view k) {
    for (const KV* kv = blk.b; kv != blk.e; ++kv)
        if (kv->k == k) return &kv->v;
    return nullptr;
}

std::string_view trim(std::string_view v) {
    // Rust str::trim (Unicode White_Space); ASCII whitespace and U+00A0/U+3000 etc. are rare
    // in unit strings -- the ASCII set plus \v\f is handled here
    auto ws = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; };
    while (!v.empty() && ws(v.front())) v.remove_prefix(1);
    while (!v.empty() && ws(v.back())) v.remove_suffix(1);
    return v;
}

// `^([+-]?[0-9\.]*)\s*(.*)$` then value.trim().parse::<u64>() (units.rs:405-438).  `.` does not
// match '\n', so a string with a line break after the number has no match.
bool split_unit(std::string_view s, std::string_view* value, std::string_view* unit, std::string* err) {
    size_t j = 0;
    if (j < s.size() && (s[j] == '+' || s[j] == '-')) ++j;
    while (j < s.size() && (is_digit(s[j]) || s[j] == '.')) ++j;
    size_t k = j;
    while (k < s.size() && (s[k] == ' ' || s[k] == '\t' || s[k] == '\n' || s[k] == '\r' || s[k] == '\v' || s[k] == '\f')) ++k;
    if (std::memchr(s.data() + k, '\n', s.size() - k)) {
        *err = "Unable to identify value and unit";
        return false;
    }
    *value = trim(s.substr(0, j));
    *unit = trim(s.substr(k));
    return true;
}

// Rust u64::from_str and its ParseIntError texts: optional '+', then ASCII digits
bool parse_u64(std::string_view v, uint64_t* out, std::string* err) {
    if (v.empty()) {
        *err = "cannot parse integer from empty string";
        return false;
    }
    if (v.front() == '+' && v.size() > 1) v.remove_prefix(1);
    uint64_t x = 0;
    for (char c : v) {
        if (!is_digit(c)) {
            *err = "invalid digit found in string";
            return false;
        }
        const uint64_t d = (uint64_t)(c - '0');
        if (x > (UINT64_MAX - d) / 10) {
            *err = "number too large to fit in target type";
            return false;
        }
        x = x * 10 + d;
    }
    *out = x;
    return true;
}

// Time<TimePrefix> (unit suffix ""): the whole unit is the prefix; "" = seconds
bool parse_time(std::string_view s, uint64_t* value, uint64_t* ns_per, std::string* err) {
    std::string_view v, u;
    if (!split_unit(s, &v, &u, err)) return false;
    static constexpr struct { std::string_view name; uint64_t ns; } kPre[] = {
        {"ns", 1}, {"nanosecond", 1}, {"nanoseconds", 1},
        {"us", 1000}, {"\xCE\xBC" "s", 1000}, {"microsecond", 1000}, {"microseconds", 1000},
        {"ms", 1000000}, {"millisecond", 1000000}, {"milliseconds", 1000000},
        {"s", 1000000000}, {"sec", 1000000000}, {"secs", 1000000000}, {"second", 1000000000},
        {"seconds", 1000000000},
        {"m", 60000000000ull}, {"min", 60000000000ull}, {"mins", 60000000000ull},
        {"minute", 60000000000ull}, {"minutes", 60000000000ull},
        {"h", 3600000000000ull}, {"hr", 3600000000000ull}, {"hrs", 3600000000000ull},
        {"hour", 3600000000000ull}, {"hours", 3600000000000ull}};
    uint64_t mag = 0;
    if (u.empty()) {
        mag = 1000000000;
    } else {
        for (const auto& p : kPre)
            if (u == p.name) mag = p.ns;
        if (!mag) {
            *err = "Unit was not one of (ns|nanosecond|nanoseconds|us|\xCE\xBCs|microsecond|microseconds"
                   "|ms|millisecond|milliseconds|s|sec|secs|second|seconds|m|min|mins|minute|minutes"
                   "|h|hr|hrs|hour|hours)";
            return false;
        }
    }
    if (!parse_u64(v, value, err)) return false;
    *ns_per = mag;
    return true;
}

// BitsPerSec<SiPrefixUpper> (suffixes "bit", "bits"): bits/s, saturated at UINT64_MAX - 1
bool parse_bandwidth(std::string_view s, uint64_t* bps, std::string* err) {
    std::string_view v, u;
    if (!split_unit(s, &v, &u, err)) return false;
    std::string_view pre = u;
    for (std::string_view suf : {std::string_view("bit"), std::string_view("bits")}) {
        if (u.size() >= suf.size() && u.substr(u.size() - suf.size()) == suf) {
            pre = u.substr(0, u.size() - suf.size());
            break;
        }
    }
    static constexpr struct { std::string_view a, b; uint64_t mag; } kPre[] = {
        {"K", "kilo", 1000}, {"Ki", "kibi", 1024}, {"M", "mega", 1000000}, {"Mi", "mebi", 1ull << 20},
        {"G", "giga", 1000000000}, {"Gi", "gibi", 1ull << 30}, {"T", "tera", 1000000000000ull},
        {"Ti", "tebi", 1ull << 40}};
    unsigned __int128 mag = 0;
    if (pre.empty()) {
        mag = 1;
    } else {
        for (const auto& p : kPre)
            if (pre == p.a || pre == p.b) mag = p.mag;
        if (!mag) {
            *err = "Unit prefix was not one of (K|kilo|Ki|kibi|M|mega|Mi|mebi|G|giga|Gi|gibi|T|tera|Ti|tebi)";
            return false;
        }
    }
    uint64_t x = 0;
    if (!parse_u64(v, &x, err)) return false;
    const unsigned __int128 b = (unsigned __int128)x * mag;
    *bps = b >= (unsigned __int128)(UINT64_MAX - 1) ? UINT64_MAX - 1 : (uint64_t)b;
    return true;
}

// a value kept for the validation pass: text offsets instead of pointers (16 bytes)
struct CV {
    uint32_t off = 0, len = 0;
    int32_t i = 0;
    float f = 0.0f;
    uint8_t t = 0;   // 0 = absent, else 1 + VT
};
struct NodeRec {
    CV id, bw[2];
};
struct EdgeRec {
    int32_t src, dst;
    CV lat, jit, loss;
};

void parse_into(const char* text, size_t len, shd_gml* g) {
    Scanner c{text, len};
    c.multispace0();
    if (!c.tag("graph")) c.fail("expected 'graph'");
    c.space0();
    if (!c.tag("[")) c.fail("expected '['");
    if (!c.newline()) c.fail("expected a newline after '['");
    auto cv = [&](const Val* v) {
        CV o;
        if (!v) return o;
        o.t = (uint8_t)(1 + (int)v->t);
        o.i = v->i;
        o.f = v->f;
        if (v->t == VT::Str) {
            o.off = (uint32_t)(v->s.data() - text);
            o.len = (uint32_t)v->s.size();
        }
        return o;
    };
    // grammar pass: every block is checked as the reference's node()/edge() do, and only the
    // fields the validation pass reads are kept (the reference validates after the whole parse)
    std::vector<KV> blkv;
    std::vector<NodeRec> nodes;
    std::vector<EdgeRec> edges;
    std::vector<KV> others;
    int n_directed = 0;
    int32_t directed = 0;
    while (!c.tag("]")) {
        std::string_view k;
        if (!c.key(&k)) c.fail("expected an item key");
        if (k == "node" || k == "edge") {
            blkv.clear();
            c.kv_block(&blkv);
            const Block blk{blkv.data(), blkv.data() + blkv.size()};
            if (k == "node") {
                const Val* id = find(blk, "id");
                if (id && id->t != VT::Int) throw Fail{SHD_ERR_INVALID, "Incorrect 'id' type"};
                nodes.push_back(NodeRec{cv(id), {cv(find(blk, "host_bandwidth_down")),
                                                 cv(find(blk, "host_bandwidth_up"))}});
            } else {
                for (const char* end : {"source", "target"}) {
                    const Val* v = find(blk, end);
                    if (!v) throw Fail{SHD_ERR_INVALID, std::string("'") + end + "' doesn't exist"};
                    if (v->t != VT::Int) throw Fail{SHD_ERR_INVALID, std::string("Incorrect '") + end + "' type"};
                }
                edges.push_back(EdgeRec{find(blk, "source")->i, find(blk, "target")->i,
                                        cv(find(blk, "latency")), cv(find(blk, "jitter")),
                                        cv(find(blk, "packet_loss"))});
            }
        } else if (k == "directed") {
            const Val v = c.value();
            if (v.t != VT::Int) throw Fail{SHD_ERR_INVALID, "Value was not an integer"};
            if (v.i != 0 && v.i != 1) throw Fail{SHD_ERR_INVALID, "Bool must be 0 or 1"};
            directed = v.i;
            ++n_directed;
        } else {
            others.push_back(KV{k, c.value()});
        }
    }
    if (n_directed > 1) throw Fail{SHD_ERR_INVALID, "The 'directed' key must only be specified once"};
    for (size_t a = 0; a < others.size(); ++a)
        for (size_t b = a + 1; b < others.size(); ++b)
            if (others[a].k == others[b].k) throw Fail{SHD_ERR_INVALID, "Duplicate keys are not supported"};
    g->directed = directed;

    // NetworkGraph::parse: nodes (ShadowNode::try_from), then edges in order
    auto sv = [&](const CV& v) { return std::string_view(text + v.off, v.len); };
    constexpr uint8_t kInt = 1 + (int)VT::Int, kFloat = 1 + (int)VT::Float, kStr = 1 + (int)VT::Str;
    std::string err;
    std::unordered_map<uint32_t, uint32_t> id_map;
    id_map.reserve(nodes.size() * 2);
    g->node_ids.reserve(nodes.size());
    for (const NodeRec& nr : nodes) {
        if (!nr.id.t) throw Fail{SHD_ERR_INVALID, "Node 'id' was not provided"};
        uint64_t bw[2] = {UINT64_MAX, UINT64_MAX};
        const char* names[2] = {"host_bandwidth_down", "host_bandwidth_up"};
        for (int b = 0; b < 2; ++b) {
            const CV& v = nr.bw[b];
            if (!v.t) continue;
            if (v.t != kStr) throw Fail{SHD_ERR_INVALID, std::string("Node '") + names[b] + "' is not a string"};
            if (!parse_bandwidth(sv(v), &bw[b], &err))
                throw Fail{SHD_ERR_INVALID, std::string("Node '") + names[b] + "' is not a valid unit: " + err};
        }
        const uint32_t gid = (uint32_t)nr.id.i;
        id_map[gid] = (uint32_t)g->node_ids.size();
        g->node_ids.push_back(gid);
        g->bw_down.push_back(bw[0]);
        g->bw_up.push_back(bw[1]);
    }
    g->src.reserve(edges.size());
    g->dst.reserve(edges.size());
    g->lat_ns.reserve(edges.size());
    g->loss.reserve(edges.size());
    for (const EdgeRec& er : edges) {
        if (!er.lat.t) throw Fail{SHD_ERR_INVALID, "Edge 'latency' was not provided"};
        if (er.lat.t != kStr) throw Fail{SHD_ERR_INVALID, "Edge 'latency' is not a string"};
        uint64_t lv = 0, lmag = 0, jv = 0, jmag = 0;
        if (!parse_time(sv(er.lat), &lv, &lmag, &err))
            throw Fail{SHD_ERR_INVALID, "Edge 'latency' is not a valid unit: " + err};
        if (er.jit.t) {   // parsed and validated, then unused
            if (er.jit.t != kStr) throw Fail{SHD_ERR_INVALID, "Edge 'jitter' is not a string"};
            if (!parse_time(sv(er.jit), &jv, &jmag, &err))
                throw Fail{SHD_ERR_INVALID, "Edge 'jitter' is not a valid unit: " + err};
        }
        float loss = 0.0f;
        if (er.loss.t) {
            if (er.loss.t != kFloat) throw Fail{SHD_ERR_INVALID, "Edge 'packet_loss' is not a float"};
            loss = er.loss.f;
        }
        if (loss < 0.0f || loss > 1.0f)
            throw Fail{SHD_ERR_INVALID, "Edge 'packet_loss' is not in the range [0,1]"};
        if (lv == 0) throw Fail{SHD_ERR_INVALID, "Edge 'latency' must not be 0"};
        const uint32_t s_id = (uint32_t)er.src, t_id = (uint32_t)er.dst;
        const auto si = id_map.find(s_id);
        if (si == id_map.end()) throw Fail{SHD_ERR_INVALID, "Edge source " + std::to_string(s_id) + " doesn't exist"};
        const auto ti = id_map.find(t_id);
        if (ti == id_map.end()) throw Fail{SHD_ERR_INVALID, "Edge target " + std::to_string(t_id) + " doesn't exist"};
        // From<&ShadowEdge> for PathProperties: convert(Nano).unwrap() (the reference panics)
        const unsigned __int128 ns = (unsigned __int128)lv * lmag;
        if (ns > UINT64_MAX) throw Fail{SHD_ERR_LATENCY_OVERFLOW, "Edge 'latency' does not fit u64 nanoseconds"};
        g->src.push_back(si->second);
        g->dst.push_back(ti->second);
        g->lat_ns.push_back((uint64_t)ns);
        g->loss.push_back(loss);
    }
    (void)kInt;
}

}  // namespace

extern "C" {

shd_status shd_gml_parse(const char* text, size_t len, shd_gml** out, char* msg, size_t msg_len) {
    if (msg && msg_len) msg[0] = 0;
    if (!out || (!text && len)) return SHD_ERR_INVALID;
    *out = nullptr;
    shd_gml* g = new (std::nothrow) shd_gml();
    if (!g) return SHD_ERR_NOMEM;
    try {
        parse_into(text, len, g);
    } catch (const Fail& f) {
        if (msg && msg_len) std::snprintf(msg, msg_len, "%s", f.msg.c_str());
        delete g;
        return f.st;
    } catch (const std::bad_alloc&) {
        delete g;
        return SHD_ERR_NOMEM;
    }
    *out = g;
    return SHD_OK;
}

}  // extern "C"

namespace {

// xz through the system liblzma (loaded on first use; the reference decompresses with lzma-rs
// 0.3.0, graph/mod.rs:482-494).  liblzma's stable C ABI (5.x): an lzma_stream starts zeroed
// (LZMA_STREAM_INIT), lzma_stream_decoder(strm, memlimit, flags), lzma_code(strm, action) with
// LZMA_RUN = 0 / LZMA_FINISH = 3 returning LZMA_OK = 0 / LZMA_STREAM_END = 1, lzma_end(strm).
struct XzStream {
    const uint8_t* next_in;
    size_t avail_in;
    uint64_t total_in;
    uint8_t* next_out;
    size_t avail_out;
    uint64_t total_out;
    const void* allocator;
    void* internal;
    void* reserved_ptr[4];
    uint64_t reserved_int1, reserved_int2;
    size_t reserved_int3, reserved_int4;
    int reserved_enum1, reserved_enum2;
    unsigned char slack[64];   // room beyond the 5.x layout, never read by us
};

struct Lzma {
    int (*decoder)(XzStream*, uint64_t, uint32_t) = nullptr;
    int (*code)(XzStream*, int) = nullptr;
    void (*end)(XzStream*) = nullptr;
    bool ok = false;
    Lzma() {
        void* h = dlopen("liblzma.so.5", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        decoder = reinterpret_cast<int (*)(XzStream*, uint64_t, uint32_t)>(dlsym(h, "lzma_stream_decoder"));
        code = reinterpret_cast<int (*)(XzStream*, int)>(dlsym(h, "lzma_code"));
        end = reinterpret_cast<void (*)(XzStream*)>(dlsym(h, "lzma_end"));
        ok = decoder && code && end;
    }
};

bool xz_decompress(const std::string& in, std::string& out, std::string& why) {
    static Lzma lz;
    if (!lz.ok) {
        why = "liblzma.so.5 not available";
        return false;
    }
    XzStream st;
    std::memset(&st, 0, sizeof(st));
    if (lz.decoder(&st, UINT64_MAX, 0) != 0) {
        why = "decoder init failed";
        return false;
    }
    st.next_in = reinterpret_cast<const uint8_t*>(in.data());
    st.avail_in = in.size();
    out.clear();
    std::vector<uint8_t> buf(1 << 20);
    int rc = 0;
    for (;;) {
        st.next_out = buf.data();
        st.avail_out = buf.size();
        rc = lz.code(&st, 3);   // LZMA_FINISH: all input is given
        out.append(reinterpret_cast<const char*>(buf.data()), buf.size() - st.avail_out);
        if (rc != 0) break;
    }
    lz.end(&st);
    if (rc != 1) {
        why = "xz data error " + std::to_string(rc);
        return false;
    }
    return true;
}

// String::from_utf8 (graph/mod.rs:493): strict UTF-8
bool valid_utf8(const std::string& s) {
    const auto* p = reinterpret_cast<const unsigned char*>(s.data());
    const size_t n = s.size();
    for (size_t i = 0; i < n;) {
        const unsigned c = p[i];
        size_t k;
        uint32_t cp;
        if (c < 0x80) { ++i; continue; }
        if ((c & 0xE0) == 0xC0) { k = 1; cp = c & 0x1F; }
        else if ((c & 0xF0) == 0xE0) { k = 2; cp = c & 0x0F; }
        else if ((c & 0xF8) == 0xF0) { k = 3; cp = c & 0x07; }
        else return false;
        for (size_t j = 1; j <= k; ++j) {
            if (i + j >= n || (p[i + j] & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (p[i + j] & 0x3F);
        }
        if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000) || cp > 0x10FFFF ||
            (cp >= 0xD800 && cp <= 0xDFFF))
            return false;
        i += k + 1;
    }
    return true;
}

}  // namespace

extern "C" {

shd_status shd_gml_load(const char* path, int32_t xz, shd_gml** out, char* msg, size_t msg_len) {
    if (msg && msg_len) msg[0] = 0;
    if (!path || !out) return SHD_ERR_INVALID;
    *out = nullptr;
    auto fail = [&](const std::string& m) {
        if (msg && msg_len) std::snprintf(msg, msg_len, "%s", m.c_str());
        return SHD_ERR_INVALID;
    };
    std::string raw;
    {
        FILE* f = std::fopen(path, "rb");
        if (!f) return fail(std::string(xz ? "Failed to open file: \"" : "Failed to read file: ") + path +
                            (xz ? "\"" : ""));
        char buf[1 << 16];
        size_t k;
        while ((k = std::fread(buf, 1, sizeof(buf), f)) > 0) raw.append(buf, k);
        const bool err = std::ferror(f) != 0;
        std::fclose(f);
        if (err) return fail(std::string("Failed to read file: ") + path);
    }
    std::string text;
    if (xz) {
        std::string why;
        if (!xz_decompress(raw, text, why)) return fail("Failed to decompress file: " + why);
    } else {
        text.swap(raw);
    }
    if (!valid_utf8(text)) return fail(xz ? "invalid utf-8 sequence" : std::string("Failed to read file: ") + path);
    return shd_gml_parse(text.data(), text.size(), out, msg, msg_len);
}

shd_status shd_gml_graph(const shd_gml* g, shd_graph* view) {
    if (!g || !view) return SHD_ERR_INVALID;
    if (g->node_ids.size() > UINT32_MAX || g->src.size() > UINT32_MAX) return SHD_ERR_INVALID;
    view->n_nodes = (uint32_t)g->node_ids.size();
    view->n_edges = (uint32_t)g->src.size();
    view->edge_src = g->src.data();
    view->edge_dst = g->dst.data();
    view->edge_latency_ns = g->lat_ns.data();
    view->edge_packet_loss = g->loss.data();
    view->node_ids = g->node_ids.data();
    view->directed = g->directed;
    return SHD_OK;
}

shd_status shd_gml_node_bandwidth(const shd_gml* g, uint64_t* down_bps, uint64_t* up_bps) {
    if (!g) return SHD_ERR_INVALID;
    if (down_bps) std::memcpy(down_bps, g->bw_down.data(), g->bw_down.size() * 8);
    if (up_bps) std::memcpy(up_bps, g->bw_up.data(), g->bw_up.size() * 8);
    return SHD_OK;
}

void shd_gml_free(shd_gml* g) { delete g; }

}  // extern "C"
