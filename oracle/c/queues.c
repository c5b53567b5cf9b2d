/*
 * CPU restatements of the two per-host state machines beside the relay (TEST INFRASTRUCTURE /
 * the timed CPU baselines of bench.py's codel and tbucket legs; the product never links this):
 *
 *   CoDel inbound router queue -- src/main/network/router/codel_queue.rs:19-330 (FlyearthR/
 *     shadow): push; pop with the store / drop modes (:125-198); codel_pop = RFC 8289 dodequeue
 *     (:201-223); process_standing_delay (:227-255); should_drop / was_dropping_recently /
 *     apply_control_law (:258-286, time + round(INTERVAL / sqrt(count)) in f64, saturating).
 *     The queue is the reference's VecDeque: unbounded (a growing ring here).
 *   Token-bucket relays -- src/main/network/relay/token_bucket.rs:37-157 (lazy_refill,
 *     conforming_remove, compute_conforming_duration) as Relay::forward_until_blocked drives it
 *     (relay/mod.rs:112-160, 200-287: Pending skips, exempt local / bootstrapping packets).
 *
 * Same batch form as the engine (ops grouped by host / relay, each in time order) and as
 * oracle/codel.py / oracle/token_bucket.py, which pin these against the reference's unit tests;
 * hosts run in parallel over OpenMP threads (the reference runs hosts on worker threads).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CD_TARGET 10000000ULL
#define CD_INTERVAL 100000000ULL
#define CD_MTU 1500ULL
#define CD_POP 0xFFFFFFFFu

static inline uint64_t sat_add(uint64_t a, uint64_t b) { return a + b < a ? ~0ULL : a + b; }
static inline uint64_t sat_sub(uint64_t a, uint64_t b) { return a > b ? a - b : 0; }

static uint64_t control_law(uint64_t t, uint64_t count) {
    const double sq = count == 0 ? 1.0 : sqrt((double)count);
    return sat_add(t, (uint64_t)round((double)CD_INTERVAL / sq));   /* f64::round: half away from 0 */
}

typedef struct { uint32_t pkt, size; uint64_t ts; } cd_ent;
typedef struct {
    cd_ent* a; uint32_t cap, head, n;
    uint64_t total, interval_end, drop_next, cur, prev;
    int has_ie, has_dn, drop_mode;
} cd_q;

static int cd_pop_raw(cd_q* q, uint64_t now, uint32_t* pkt, int* ok_to_drop) {
    if (q->n == 0) { q->has_ie = 0; return 0; }
    cd_ent e = q->a[q->head];
    q->head = q->head + 1 == q->cap ? 0 : q->head + 1;
    q->n--;
    q->total = sat_sub(q->total, e.size);
    const uint64_t standing = sat_sub(now, e.ts);
    *pkt = e.pkt;
    if (standing < CD_TARGET || q->total <= CD_MTU) { q->has_ie = 0; *ok_to_drop = 0; }
    else if (q->has_ie) *ok_to_drop = now >= q->interval_end;
    else { q->interval_end = sat_add(now, CD_INTERVAL); q->has_ie = 1; *ok_to_drop = 0; }
    return 1;
}

static void cd_push(cd_q* q, uint32_t pkt, uint32_t size, uint64_t now) {
    if (q->n == q->cap) {   /* grow the ring, keeping order */
        uint32_t nc = q->cap ? q->cap * 2 : 64;
        cd_ent* na = (cd_ent*)malloc((size_t)nc * sizeof(cd_ent));
        for (uint32_t i = 0; i < q->n; i++) na[i] = q->a[(q->head + i) % q->cap];
        free(q->a);
        q->a = na; q->cap = nc; q->head = 0;
    }
    q->a[(q->head + q->n) % q->cap] = (cd_ent){pkt, size, now};
    q->n++;
    q->total += size;
}

/* returns the packet popped or CD_POP; dropped packets are marked in fate */
static uint32_t cd_pop(cd_q* q, uint64_t now, uint32_t op, uint64_t* fate, uint32_t n_ids) {
    uint32_t pkt = 0; int drop = 0;
#define MARK(p) do { if ((p) < n_ids) fate[p] = ((uint64_t)op << 2) | 2; } while (0)
    if (!cd_pop_raw(q, now, &pkt, &drop)) { q->drop_mode = 0; return CD_POP; }
    if (!drop) { q->drop_mode = 0; return pkt; }
    if (!q->drop_mode) {   /* drop_from_store_mode */
        MARK(pkt);
        uint32_t nxt = 0; int nd = 0;
        const int have = cd_pop_raw(q, now, &nxt, &nd);
        q->drop_mode = 1;
        const uint64_t delta = sat_sub(q->cur, q->prev);
        const int recently = q->has_dn && sat_sub(now, q->drop_next) < CD_INTERVAL * 16;
        q->cur = recently && delta > 1 ? delta : 1;
        q->drop_next = control_law(now, q->cur);
        q->has_dn = 1;
        q->prev = q->cur;
        return have ? nxt : CD_POP;
    }
    int have = 1, item_drop = 1;   /* drop_from_drop_mode */
    while (have && q->drop_mode && q->has_dn && now >= q->drop_next) {
        MARK(pkt);
        q->cur++;
        have = cd_pop_raw(q, now, &pkt, &item_drop);
        if (have && item_drop) q->drop_next = control_law(q->drop_next, q->cur);
        else q->drop_mode = 0;
    }
#undef MARK
    return have ? pkt : CD_POP;
}

/* fresh queues; pop_out[n_ops], fate[n_ids] = (op << 2) | 1 dequeued / 2 dropped */
void orc_codel_run(uint32_t n_hosts, const uint32_t* off, const uint64_t* time, const uint32_t* size,
                   const uint32_t* pkt, uint32_t* pop_out, uint64_t* fate, uint32_t n_ids, int threads) {
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 64)
    for (uint32_t h = 0; h < n_hosts; h++) {
        cd_q q;
        memset(&q, 0, sizeof(q));
        for (uint32_t k = off[h]; k < off[h + 1]; k++) {
            if (size[k] == CD_POP) {
                const uint32_t got = cd_pop(&q, time[k], k, fate, n_ids);
                pop_out[k] = got;
                if (got != CD_POP && got < n_ids) fate[got] = ((uint64_t)k << 2) | 1;
            } else {
                pop_out[k] = CD_POP;
                cd_push(&q, pkt[k], size[k], time[k]);
            }
        }
        free(q.a);
    }
}

/* ------------------------------------------------------------------ token buckets */
#define SIMTIME_MAX 17500059273709551614ULL
#define EMUTIME_MAX (~0ULL - 1)

static int simtime_sat_mul(uint64_t t, uint64_t k, uint64_t* out) {
    const __uint128_t p = (__uint128_t)t * k;
    if (p > (__uint128_t)~0ULL) { *out = SIMTIME_MAX; return 0; }
    if ((uint64_t)p > SIMTIME_MAX) return 1;   /* the reference's unwrap panics */
    *out = (uint64_t)p;
    return 0;
}
static int simtime_sat_add(uint64_t a, uint64_t b, uint64_t* out) {
    const __uint128_t s = (__uint128_t)a + b;
    if (s > (__uint128_t)~0ULL) { *out = SIMTIME_MAX; return 0; }
    if ((uint64_t)s > SIMTIME_MAX) return 1;
    *out = (uint64_t)s;
    return 0;
}
static inline uint64_t emutime_sat_add(uint64_t t, uint64_t d) {
    const __uint128_t s = (__uint128_t)t + d;
    return s > EMUTIME_MAX ? EMUTIME_MAX : (uint64_t)s;
}

/* status: 0 forwarded (value = balance after, UINT64_MAX without a bucket), 1 blocked (value =
 * duration until conforming), 2 skipped (value = pending deadline); returns the number of
 * attempts where the reference panics (the relay's later attempts are then skipped) */
int64_t orc_tb_run(uint32_t n_relays, const uint64_t* capacity, const uint64_t* increment,
                   const uint64_t* interval, const uint64_t* last_refill, const uint32_t* off,
                   const uint64_t* time, const uint32_t* size, const uint8_t* flags, uint8_t* status,
                   uint64_t* value, int threads) {
    int64_t panics = 0;
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : panics)
    for (uint32_t r = 0; r < n_relays; r++) {
        const int unlimited = capacity[r] == 0;
        uint64_t bal = capacity[r], last = last_refill[r], pending = 0;
        const uint64_t cap = capacity[r], inc = increment[r], itv = interval[r];
        for (uint32_t k = off[r]; k < off[r + 1]; k++) {
            const uint64_t now = time[k];
            if (now < pending) { status[k] = 2; value[k] = pending; continue; }
            if (unlimited) { status[k] = 0; value[k] = ~0ULL; continue; }
            if (flags[k] & 1) { status[k] = 0; value[k] = bal; continue; }
            /* lazy_refill */
            if (now < last) { panics++; status[k] = 2; value[k] = 0; pending = ~0ULL; continue; }
            uint64_t span = now - last;
            if (span >= itv) {
                const uint64_t n = span / itv;
                const __uint128_t tk = (__uint128_t)inc * n;
                const uint64_t tokens = tk > (__uint128_t)~0ULL ? ~0ULL : (uint64_t)tk;
                uint64_t b = sat_add(bal, tokens);
                bal = b < cap ? b : cap;
                uint64_t step;
                if (simtime_sat_mul(itv, n, &step)) { panics++; pending = ~0ULL; status[k] = 2; continue; }
                last = emutime_sat_add(last, step);
                if (now < last) { panics++; pending = ~0ULL; status[k] = 2; continue; }
                span = now - last;
            }
            const uint64_t next_span = itv - span;
            const uint64_t dec = size[k];
            if (bal >= dec) { bal -= dec; status[k] = 0; value[k] = bal; continue; }
            /* compute_conforming_duration */
            const uint64_t req = dec - bal;
            const uint64_t n = req / inc + (req % inc ? 1 : 0);
            uint64_t dur;
            if (n == 1) dur = next_span;
            else {
                uint64_t m;
                if (simtime_sat_mul(itv, n - 1, &m) || simtime_sat_add(next_span, m, &dur)) {
                    panics++; pending = ~0ULL; status[k] = 2; continue;
                }
            }
            status[k] = 1;
            value[k] = dur;
            pending = emutime_sat_add(now, dur);
        }
    }
    return panics;
}
