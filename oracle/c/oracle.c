/*
 * CPU restatement of Shadow's routing build and per-round packet relay.
 *
 * TEST INFRASTRUCTURE ONLY: this is the bit-exact checker for large sizes and the timed
 * CPU baseline ("kind": "port") of bench.py.  The product library (shadow_amd/) never
 * links or calls it.  Built by oracle/c/Makefile into oracle/build/liboracle.so.
 *
 * Routing restates src/main/network/graph/mod.rs:185-230 (compute_shortest_paths), :232-254
 * (get_direct_paths), :258-295 (get_edge_weight), :298-333 (PathProperties) over petgraph
 * 0.6.3 algo::dijkstra (lazy-deletion binary heap, strict '<' improvement, visited set).
 * Sources run in parallel over OpenMP threads, the analogue of the reference's rayon
 * into_par_iter over used sources (graph/mod.rs:192-210).
 *   variant ORC_FAITHFUL keeps the reference's per-entry `nodes.contains(dst)` linear scan
 *   (mod.rs:205) and materialises the n^2 result in a hash map (mod.rs:192-210) before the
 *   dense copy-out; ORC_TIDY uses a used-node bitmap and writes the dense table directly.
 *
 * Relay restates src/main/core/worker.rs:328-413 (send_packet) with a per-destination mutex
 * + binary heap (worker.rs:619-629, event_queue.rs:28-48) and event order event.rs:84-155.
 *
 * Compile with -ffp-contract=off: Rust never contracts 1-(1-p)*(1-e) into an FMA.
 */
#include <math.h>
#include <omp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_NO_EDGE 1
#define ORC_MULTI_EDGE 2
#define ORC_UNREACHABLE 3
#define ORC_NOMEM 4

#define ORC_TIDY 0
#define ORC_FAITHFUL 1

typedef struct { uint64_t lat; float loss; uint32_t node; } hent;

static inline int key_lt(uint64_t la, float pa, uint64_t lb, float pb) {
    return la < lb || (la == lb && pa < pb);
}
static inline float fold(float p, float e) { return 1.0f - (1.0f - p) * (1.0f - e); }

/* binary min-heap on (lat, loss) */
typedef struct { hent* a; size_t n, cap; } heap_t;
static int heap_push(heap_t* h, hent x) {
    if (h->n == h->cap) {
        size_t nc = h->cap ? h->cap * 2 : 1024;
        hent* na = (hent*)realloc(h->a, nc * sizeof(hent));
        if (!na) return -1;
        h->a = na; h->cap = nc;
    }
    size_t i = h->n++;
    while (i) {
        size_t p = (i - 1) / 2;
        if (!key_lt(x.lat, x.loss, h->a[p].lat, h->a[p].loss)) break;
        h->a[i] = h->a[p]; i = p;
    }
    h->a[i] = x;
    return 0;
}
static hent heap_pop(heap_t* h) {
    hent top = h->a[0], x = h->a[--h->n];
    size_t i = 0;
    for (;;) {
        size_t l = 2 * i + 1, r = l + 1, m = i;
        hent* cand = &x;
        if (l < h->n && key_lt(h->a[l].lat, h->a[l].loss, cand->lat, cand->loss)) { m = l; cand = &h->a[l]; }
        if (r < h->n && key_lt(h->a[r].lat, h->a[r].loss, cand->lat, cand->loss)) { m = r; cand = &h->a[r]; }
        if (m == i) break;
        h->a[i] = h->a[m]; i = m;
    }
    if (h->n) h->a[i] = x;
    return top;
}

/* adjacency in petgraph edges(node) semantics */
typedef struct { uint32_t* off; uint32_t* dst; uint64_t* lat; float* loss; } adj_t;
static int build_adj(uint32_t V, uint32_t E, const uint32_t* es, const uint32_t* ed,
                     const uint64_t* el, const float* ep, int directed, adj_t* a) {
    uint32_t* deg = (uint32_t*)calloc(V + 1, sizeof(uint32_t));
    if (!deg) return -1;
    for (uint32_t i = 0; i < E; i++) {
        deg[es[i] + 1]++;
        if (!directed && es[i] != ed[i]) deg[ed[i] + 1]++;
    }
    for (uint32_t v = 0; v < V; v++) deg[v + 1] += deg[v];
    size_t na = deg[V];
    a->off = deg;
    a->dst = (uint32_t*)malloc(na * sizeof(uint32_t) + 1);
    a->lat = (uint64_t*)malloc(na * sizeof(uint64_t) + 1);
    a->loss = (float*)malloc(na * sizeof(float) + 1);
    uint32_t* fill = (uint32_t*)malloc((V + 1) * sizeof(uint32_t));
    if (!a->dst || !a->lat || !a->loss || !fill) return -1;
    memcpy(fill, deg, (V + 1) * sizeof(uint32_t));
    for (uint32_t i = 0; i < E; i++) {
        uint32_t k = fill[es[i]]++;
        a->dst[k] = ed[i]; a->lat[k] = el[i]; a->loss[k] = ep[i];
        if (!directed && es[i] != ed[i]) {
            k = fill[ed[i]]++;
            a->dst[k] = es[i]; a->lat[k] = el[i]; a->loss[k] = ep[i];
        }
    }
    free(fill);
    return 0;
}
static void free_adj(adj_t* a) { free(a->off); free(a->dst); free(a->lat); free(a->loss); }

/* exactly one edge src->dst ({src,dst} if undirected) -- get_edge_weight (mod.rs:258-295),
 * scanning the adjacency of src like petgraph's edges_connecting */
static int edge_weight(const adj_t* a, uint32_t s, uint32_t d, uint64_t* lat, float* loss) {
    int found = 0;
    for (uint32_t k = a->off[s]; k < a->off[s + 1]; k++) {
        if (a->dst[k] != d) continue;
        if (found) return ORC_MULTI_EDGE;
        found = 1; *lat = a->lat[k]; *loss = a->loss[k];
    }
    return found ? ORC_OK : ORC_NO_EDGE;
}

/* simple open-addressing map (src,dst)->(lat,loss) for the faithful variant */
typedef struct { uint64_t key; uint64_t lat; float loss; } hslot;

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

/*
 * Returns ORC_* ; on error err_a / err_b hold the GML-order node indices involved.
 * lat_out/loss_out: n_used x n_used row-major (used-list order).
 */
/*
 * Rows [rb, re) of the n_used x n_used table (sources used[rb..re)); lat_out/loss_out hold
 * (re - rb) x n_used.  The self-loop rule is checked over every used node in `nodes` order as
 * the reference does; unreachable pairs only over the rows built.  This is what checks a few
 * source rows of a graph whose full table does not fit (C4: 50k x 50k = 30 GB).
 */
int orc_shortest_paths_rows(uint32_t V, uint32_t E, const uint32_t* es, const uint32_t* ed,
                            const uint64_t* el, const float* ep, int directed,
                            const uint32_t* used, uint32_t n_used, uint32_t rb, uint32_t re,
                            int variant, int threads, uint64_t* lat_out, float* loss_out,
                            uint32_t* err_a, uint32_t* err_b) {
    adj_t a;
    if (rb > re || re > n_used) return ORC_NOMEM;
    if (build_adj(V, E, es, ed, el, ep, directed, &a)) return ORC_NOMEM;
    int32_t* col = (int32_t*)malloc(V * sizeof(int32_t));
    for (uint32_t v = 0; v < V; v++) col[v] = -1;
    for (uint32_t i = 0; i < n_used; i++) col[used[i]] = (int32_t)i;
    const uint64_t UNSET = ~0ULL;
    const size_t nn = (size_t)(re - rb) * n_used;
    for (size_t i = 0; i < nn; i++) lat_out[i] = UNSET;

    hslot* map = NULL; size_t mcap = 0;
    if (variant == ORC_FAITHFUL) {
        mcap = 1; while (mcap < nn * 2) mcap <<= 1;
        map = (hslot*)malloc(mcap * sizeof(hslot));
        if (!map) { free_adj(&a); free(col); return ORC_NOMEM; }
        for (size_t i = 0; i < mcap; i++) map[i].key = UNSET;
    }
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
    {
        uint64_t* score_lat = (uint64_t*)malloc(V * sizeof(uint64_t));
        float* score_loss = (float*)malloc(V * sizeof(float));
        uint8_t* visited = (uint8_t*)malloc(V);
        uint32_t* touched = (uint32_t*)malloc(V * sizeof(uint32_t));
        heap_t h = {0, 0, 0};
#pragma omp for schedule(dynamic, 1)
        for (uint32_t si = rb; si < re; si++) {
            uint32_t src = used[si];
            const size_t orow = (size_t)(si - rb) * n_used;
            for (uint32_t v = 0; v < V; v++) { score_lat[v] = UNSET; visited[v] = 0; }
            uint32_t nt = 0;
            score_lat[src] = 0; score_loss[src] = 0.0f; touched[nt++] = src;
            h.n = 0;
            heap_push(&h, (hent){0, 0.0f, src});
            while (h.n) {
                hent cur = heap_pop(&h);
                uint32_t u = cur.node;
                if (visited[u]) continue;
                for (uint32_t k = a.off[u]; k < a.off[u + 1]; k++) {
                    uint32_t v = a.dst[k];
                    if (visited[v]) continue;
                    uint64_t nl = cur.lat + a.lat[k];
                    float np_ = fold(cur.loss, a.loss[k]);
                    if (score_lat[v] == UNSET) {
                        score_lat[v] = nl; score_loss[v] = np_; touched[nt++] = v;
                        heap_push(&h, (hent){nl, np_, v});
                    } else if (key_lt(nl, np_, score_lat[v], score_loss[v])) {
                        score_lat[v] = nl; score_loss[v] = np_;
                        heap_push(&h, (hent){nl, np_, v});
                    }
                }
                visited[u] = 1;
            }
            /* iterate the result map (petgraph returns a HashMap of reached nodes) */
            for (uint32_t t = 0; t < nt; t++) {
                uint32_t v = touched[t];
                int32_t cj;
                if (variant == ORC_FAITHFUL) {
                    cj = -1;
                    for (uint32_t q = 0; q < n_used; q++) if (used[q] == v) { cj = (int32_t)q; break; }
                    if (cj < 0) continue;
                    uint64_t key = ((uint64_t)(si - rb) << 32) | (uint32_t)cj;
                    size_t pos = mix64(key) & (mcap - 1);
                    for (;;) {
                        uint64_t cur = __atomic_load_n(&map[pos].key, __ATOMIC_RELAXED);
                        if (cur == UNSET &&
                            __atomic_compare_exchange_n(&map[pos].key, &cur, key, 0,
                                                        __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
                            map[pos].lat = score_lat[v]; map[pos].loss = score_loss[v];
                            break;
                        }
                        pos = (pos + 1) & (mcap - 1);
                    }
                } else {
                    cj = col[v];
                    if (cj < 0) continue;
                    lat_out[orow + cj] = score_lat[v];
                    loss_out[orow + cj] = score_loss[v];
                }
            }
        }
        free(score_lat); free(score_loss); free(visited); free(touched); free(h.a);
    }
    if (variant == ORC_FAITHFUL) {
        for (size_t i = 0; i < mcap; i++) {
            if (map[i].key == UNSET) continue;
            size_t r = map[i].key >> 32, c = map[i].key & 0xffffffffu;
            lat_out[r * n_used + c] = map[i].lat;
            loss_out[r * n_used + c] = map[i].loss;
        }
        free(map);
    }
    int rc = ORC_OK;
    /* self-loop diagonal, in `nodes` order (mod.rs:213-219) */
    for (uint32_t i = 0; i < n_used && rc == ORC_OK; i++) {
        uint64_t l; float p;
        int r = edge_weight(&a, used[i], used[i], &l, &p);
        if (r != ORC_OK) { rc = r; *err_a = used[i]; *err_b = used[i]; break; }
        if (i < rb || i >= re) continue;
        lat_out[(size_t)(i - rb) * n_used + i] = l;
        loss_out[(size_t)(i - rb) * n_used + i] = p;
    }
    if (rc == ORC_OK) {
        for (size_t i = 0; i < nn; i++) {
            if (lat_out[i] == UNSET) {
                rc = ORC_UNREACHABLE; *err_a = used[rb + i / n_used]; *err_b = used[i % n_used];
                break;
            }
        }
    }
    free_adj(&a); free(col);
    return rc;
}

int orc_shortest_paths(uint32_t V, uint32_t E, const uint32_t* es, const uint32_t* ed,
                       const uint64_t* el, const float* ep, int directed,
                       const uint32_t* used, uint32_t n_used, int variant, int threads,
                       uint64_t* lat_out, float* loss_out, uint32_t* err_a, uint32_t* err_b) {
    return orc_shortest_paths_rows(V, E, es, ed, el, ep, directed, used, n_used, 0, n_used,
                                   variant, threads, lat_out, loss_out, err_a, err_b);
}

/* get_direct_paths (mod.rs:232-254): src-major over nodes, first error wins */
int orc_direct_paths(uint32_t V, uint32_t E, const uint32_t* es, const uint32_t* ed,
                     const uint64_t* el, const float* ep, int directed, const uint32_t* used,
                     uint32_t n_used, uint64_t* lat_out, float* loss_out, uint32_t* err_a,
                     uint32_t* err_b) {
    adj_t a;
    if (build_adj(V, E, es, ed, el, ep, directed, &a)) return ORC_NOMEM;
    int rc = ORC_OK;
    for (uint32_t i = 0; i < n_used && rc == ORC_OK; i++)
        for (uint32_t j = 0; j < n_used; j++) {
            int r = edge_weight(&a, used[i], used[j], &lat_out[(size_t)i * n_used + j],
                                &loss_out[(size_t)i * n_used + j]);
            if (r != ORC_OK) { *err_a = used[i]; *err_b = used[j]; rc = r; break; }
        }
    free_adj(&a);
    return rc;
}

/* ------------------------------------------------------------------ RNG (rand_xoshiro 0.6) */
static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t xoshiro_next(uint64_t* s) {
    uint64_t res = rotl64(s[0] + s[3], 23) + s[0];
    uint64_t t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t;
    s[3] = rotl64(s[3], 45);
    return res;
}
void orc_xoshiro_seed(uint64_t seed, uint64_t* s) {
    uint64_t x = seed;
    for (int i = 0; i < 4; i++) {
        x += 0x9e3779b97f4a7c15ULL;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        s[i] = z ^ (z >> 31);
    }
}

/* ------------------------------------------------------------------ relay */
typedef struct { uint64_t t; uint32_t src; uint32_t pad; uint64_t seq; uint32_t pkt; uint32_t pad2; } ev_t;
static inline int ev_lt(const ev_t* a, const ev_t* b) {
    if (a->t != b->t) return a->t < b->t;
    if (a->src != b->src) return a->src < b->src;
    return a->seq < b->seq;
}
typedef struct { ev_t* a; uint32_t n, cap; pthread_mutex_t mu; } evq_t;
static void evq_push(evq_t* q, ev_t e) {
    if (q->n == q->cap) {
        q->cap = q->cap ? q->cap * 2 : 16;
        q->a = (ev_t*)realloc(q->a, (size_t)q->cap * sizeof(ev_t));
    }
    uint32_t i = q->n++;
    while (i) {
        uint32_t p = (i - 1) / 2;
        if (!ev_lt(&e, &q->a[p])) break;
        q->a[i] = q->a[p]; i = p;
    }
    q->a[i] = e;
}
static ev_t evq_pop(evq_t* q) {
    ev_t top = q->a[0], x = q->a[--q->n];
    uint32_t i = 0;
    for (;;) {
        uint32_t l = 2 * i + 1, r = l + 1, m = i;
        const ev_t* c = &x;
        if (l < q->n && ev_lt(&q->a[l], c)) { m = l; c = &q->a[l]; }
        if (r < q->n && ev_lt(&q->a[r], c)) { m = r; c = &q->a[r]; }
        if (m == i) break;
        q->a[i] = q->a[m]; i = m;
    }
    if (q->n) q->a[i] = x;
    return top;
}

/*
 * Packets grouped by source host: host h's sends are pkt[src_off[h] .. src_off[h+1]) in send
 * order.  The round is processed host-parallel (the reference runs hosts on worker threads);
 * every SENT packet is pushed under the destination's mutex into its binary heap -- the
 * reference's Mutex<EventQueue> (worker.rs:619-629).
 * If out_* are non-NULL the heaps are drained into per-destination sorted segments:
 * out_off[n_hosts+1], out_deliver/out_src/out_seq/out_pkt[n_sent].
 * Returns number of SENT packets; fills status[n], deliver[n], seq[n], min_deliver, min_latency.
 * rng/next_id are updated in place.  chance (nullable) replaces the draws.
 */
int orc_eq_push_one(void* p, uint32_t dst, uint64_t t, uint32_t src, uint64_t seq, uint64_t tag);

/* eq != NULL (orc_relay_round_eq): every SENT packet goes into the persistent destination queues
 * of oracle/c/equeue.c instead (tag = batch_no << 32 | packet index); out_* are then unused. */
static int64_t relay_round_impl(uint32_t n_hosts, const uint32_t* src_off, const uint64_t* send_time,
                                const uint32_t* dst_host, const uint32_t* payload, const double* chance,
                                const uint32_t* host_node, uint32_t n_nodes, const uint64_t* lat,
                                const float* loss, uint64_t* rng, uint64_t* next_id,
                                uint64_t round_end, uint64_t sim_end, uint64_t bootstrap_end,
                                int threads, uint8_t* status, uint64_t* deliver, uint64_t* seq,
                                uint64_t* min_deliver, uint64_t* min_latency,
                                uint32_t* out_off, uint64_t* out_deliver, uint32_t* out_src,
                                uint64_t* out_seq, uint32_t* out_pkt, void* eq, uint64_t batch_no) {
    evq_t* q = eq ? NULL : (evq_t*)calloc(n_hosts, sizeof(evq_t));
    if (q)
        for (uint32_t h = 0; h < n_hosts; h++) pthread_mutex_init(&q[h].mu, NULL);
    uint64_t gmin_d = ~0ULL, gmin_l = ~0ULL;
    int64_t n_sent = 0;
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel reduction(min : gmin_d, gmin_l) reduction(+ : n_sent)
    {
#pragma omp for schedule(dynamic, 64)
        for (uint32_t h = 0; h < n_hosts; h++) {
            uint64_t* s = &rng[(size_t)h * 4];
            uint64_t id = next_id[h];
            uint32_t sn = host_node[h];
            for (uint32_t i = src_off[h]; i < src_off[h + 1]; i++) {
                uint64_t now = send_time[i];
                status[i] = 0; deliver[i] = 0; seq[i] = 0;
                if (now >= sim_end) continue;
                uint32_t d = dst_host[i], dn = host_node[d];
                size_t pi = (size_t)sn * n_nodes + dn;
                double reliability = (double)(1.0f - loss[pi]);
                double c = chance ? chance[i]
                                  : (double)(xoshiro_next(s) >> 11) * (1.0 / 9007199254740992.0);
                int boot = now < bootstrap_end;
                if (!boot && c >= reliability && payload[i] > 0) { status[i] = 1; continue; }
                uint64_t delay = lat[pi];
                if (delay < gmin_l) gmin_l = delay;
                uint64_t t = now + delay;
                if (t < round_end) t = round_end;
                if (t < gmin_d) gmin_d = t;
                status[i] = 2; deliver[i] = t; seq[i] = id;
                ev_t e = {t, h, 0, id, i, 0};
                id++;
                n_sent++;
                if (eq) {
                    orc_eq_push_one(eq, d, t, h, e.seq, (batch_no << 32) | i);
                } else {
                    pthread_mutex_lock(&q[d].mu);
                    evq_push(&q[d], e);
                    pthread_mutex_unlock(&q[d].mu);
                }
            }
            next_id[h] = id;
        }
    }
    *min_deliver = gmin_d; *min_latency = gmin_l;
    if (!q) return n_sent;
    if (out_off) {
        out_off[0] = 0;
        for (uint32_t h = 0; h < n_hosts; h++) out_off[h + 1] = out_off[h] + q[h].n;
#pragma omp parallel for schedule(dynamic, 64)
        for (uint32_t h = 0; h < n_hosts; h++) {
            uint32_t o = out_off[h];
            while (q[h].n) {
                ev_t e = evq_pop(&q[h]);
                out_deliver[o] = e.t; out_src[o] = e.src; out_seq[o] = e.seq; out_pkt[o] = e.pkt;
                o++;
            }
        }
    }
    for (uint32_t h = 0; h < n_hosts; h++) { free(q[h].a); pthread_mutex_destroy(&q[h].mu); }
    free(q);
    return n_sent;
}

int64_t orc_relay_round(uint32_t n_hosts, const uint32_t* src_off, const uint64_t* send_time,
                        const uint32_t* dst_host, const uint32_t* payload, const double* chance,
                        const uint32_t* host_node, uint32_t n_nodes, const uint64_t* lat,
                        const float* loss, uint64_t* rng, uint64_t* next_id,
                        uint64_t round_end, uint64_t sim_end, uint64_t bootstrap_end,
                        int threads, uint8_t* status, uint64_t* deliver, uint64_t* seq,
                        uint64_t* min_deliver, uint64_t* min_latency,
                        uint32_t* out_off, uint64_t* out_deliver, uint32_t* out_src,
                        uint64_t* out_seq, uint32_t* out_pkt) {
    return relay_round_impl(n_hosts, src_off, send_time, dst_host, payload, chance, host_node, n_nodes, lat, loss,
                            rng, next_id, round_end, sim_end, bootstrap_end, threads, status, deliver, seq,
                            min_deliver, min_latency, out_off, out_deliver, out_src, out_seq, out_pkt, NULL, 0);
}

/* send_packet for a round with push_packet_to_host into persistent destination queues (orc_eq_new) */
int64_t orc_relay_round_eq(uint32_t n_hosts, const uint32_t* src_off, const uint64_t* send_time,
                           const uint32_t* dst_host, const uint32_t* payload, const double* chance,
                           const uint32_t* host_node, uint32_t n_nodes, const uint64_t* lat,
                           const float* loss, uint64_t* rng, uint64_t* next_id,
                           uint64_t round_end, uint64_t sim_end, uint64_t bootstrap_end,
                           int threads, uint8_t* status, uint64_t* deliver, uint64_t* seq,
                           uint64_t* min_deliver, uint64_t* min_latency, void* eq, uint64_t batch_no) {
    return relay_round_impl(n_hosts, src_off, send_time, dst_host, payload, chance, host_node, n_nodes, lat, loss,
                            rng, next_id, round_end, sim_end, bootstrap_end, threads, status, deliver, seq,
                            min_deliver, min_latency, NULL, NULL, NULL, NULL, NULL, eq, batch_no);
}

int orc_max_threads(void) { return omp_get_max_threads(); }

/*
 * Next hops from a finished table (test infrastructure: the checker of shd_routing_run_next_hops).
 * The reference keeps none; the definition is the engine's: pred(s, v) = the lowest
 * node index u with an arc u -> v, u != v, whose label extended by the arc equals v's label bit
 * for bit (label(s, s) = PathProperties::default() = (0, 0.0), not the self-loop diagonal);
 * next_hop(s, d) = the node after s on d's pred chain; next_hop(s, s) = s.  `used` must list every
 * node (the table then holds every label).  Rows [rb, re) of the table are given.
 */
int orc_next_hops(uint32_t V, uint32_t E, const uint32_t* es, const uint32_t* ed, const uint64_t* el,
                  const float* ep, int directed, const uint32_t* used, uint32_t n_used, uint32_t rb,
                  uint32_t re, const uint64_t* lat, const float* loss, int threads, uint32_t* out) {
    if (n_used != V) return ORC_NOMEM;
    adj_t a;
    if (build_adj(V, E, es, ed, el, ep, directed, &a)) return ORC_NOMEM;
    int32_t* col = (int32_t*)malloc(V * sizeof(int32_t));
    for (uint32_t i = 0; i < n_used; i++) col[used[i]] = (int32_t)i;
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
    {
        uint32_t* pred = (uint32_t*)malloc(V * sizeof(uint32_t));
#pragma omp for schedule(dynamic, 1)
        for (uint32_t si = rb; si < re; si++) {
            const uint32_t src = used[si];
            const uint64_t* L = lat + (size_t)(si - rb) * n_used;
            const float* P = loss + (size_t)(si - rb) * n_used;
            for (uint32_t v = 0; v < V; v++) pred[v] = 0xFFFFFFFFu;
            for (uint32_t u = 0; u < V; u++) {
                const uint64_t lu = u == src ? 0 : L[col[u]];
                const float pu = u == src ? 0.0f : P[col[u]];
                for (uint32_t k = a.off[u]; k < a.off[u + 1]; k++) {
                    const uint32_t v = a.dst[k];
                    if (v == u || v == src) continue;
                    const uint64_t cl = lu + a.lat[k];
                    const float cp = fold(pu, a.loss[k] + 0.0f);
                    if (cl == L[col[v]] && memcmp(&cp, &P[col[v]], 4) == 0 && u < pred[v]) pred[v] = u;
                }
            }
            for (uint32_t j = 0; j < n_used; j++) {
                const uint32_t v = used[j];
                uint32_t nh = 0xFFFFFFFFu;
                if (v == src) {
                    nh = src;
                } else {
                    uint32_t w = v, pw = pred[w];
                    for (uint32_t hop = 0; hop < V && pw != src && pw != 0xFFFFFFFFu; hop++) { w = pw; pw = pred[w]; }
                    if (pw == src) nh = w;
                }
                out[(size_t)(si - rb) * n_used + j] = nh;
            }
        }
        free(pred);
    }
    free_adj(&a); free(col);
    return ORC_OK;
}
