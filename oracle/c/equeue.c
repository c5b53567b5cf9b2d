/*
 * CPU restatement of the destination hosts' packet-event queues.
 *
 * TEST INFRASTRUCTURE ONLY: the checker of shd_equeue_advance at full C5 scale and the CPU
 * baseline of bench.py's relay + merge leg.  The product library (shadow_amd/) never links or
 * calls it.  Built by oracle/c/Makefile into oracle/build/liboracle.so.
 *
 * Restates, per destination host:
 *   EventQueue (src/main/core/work/event_queue.rs:10-49): BinaryHeap<Reverse<PanickingOrd<Event>>>
 *     -- push, pop (asserting that time never moves backwards, :34-41), next_event_time (:44-46);
 *   the packet-event order (event.rs:84-155): time, then src host id, then src host event id
 *     (all events here are packets, so the Packet-before-Local rule never decides);
 *   push_packet_to_host (worker.rs:619-629): the push under the destination's Mutex;
 *   Host::execute's pop loop (host.rs:697-706): pop while next_event_time < window end.
 * Each event carries a tag (batch number << 32 | packet index) so a checker can name the packet.
 */
#include <omp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t t; uint32_t src; uint32_t pad; uint64_t seq; uint64_t tag; } qev_t;

static inline int qev_lt(const qev_t* a, const qev_t* b) {
    if (a->t != b->t) return a->t < b->t;
    if (a->src != b->src) return a->src < b->src;
    return a->seq < b->seq;
}

typedef struct {
    qev_t* a;
    uint32_t n, cap;
    uint64_t last;          /* last_popped_event_time */
    pthread_mutex_t mu;
    qev_t* pop;             /* this advance's popped events (reused) */
    uint32_t npop, popcap;
} hq_t;

typedef struct {
    uint32_t n_hosts;
    hq_t* q;
} orc_eq_t;

static int hq_push(hq_t* q, qev_t e) {
    if (q->n == q->cap) {
        uint32_t c = q->cap ? q->cap * 2 : 16;
        qev_t* na = (qev_t*)realloc(q->a, (size_t)c * sizeof(qev_t));
        if (!na) return 1;
        q->a = na;
        q->cap = c;
    }
    uint32_t i = q->n++;
    while (i) {
        uint32_t p = (i - 1) / 2;
        if (!qev_lt(&e, &q->a[p])) break;
        q->a[i] = q->a[p];
        i = p;
    }
    q->a[i] = e;
    return 0;
}

static qev_t hq_pop(hq_t* q) {
    qev_t top = q->a[0], x = q->a[--q->n];
    uint32_t i = 0;
    for (;;) {
        uint32_t l = 2 * i + 1, r = l + 1, m = i;
        const qev_t* c = &x;
        if (l < q->n && qev_lt(&q->a[l], c)) { m = l; c = &q->a[l]; }
        if (r < q->n && qev_lt(&q->a[r], c)) { m = r; c = &q->a[r]; }
        if (m == i) break;
        q->a[i] = q->a[m];
        i = m;
    }
    if (q->n) q->a[i] = x;
    return top;
}

void* orc_eq_new(uint32_t n_hosts) {
    orc_eq_t* e = (orc_eq_t*)calloc(1, sizeof(orc_eq_t));
    if (!e) return NULL;
    e->n_hosts = n_hosts;
    e->q = (hq_t*)calloc(n_hosts ? n_hosts : 1, sizeof(hq_t));
    if (!e->q) { free(e); return NULL; }
    for (uint32_t h = 0; h < n_hosts; h++) {
        pthread_mutex_init(&e->q[h].mu, NULL);
        e->q[h].last = 0;   /* EmulatedTime::SIMULATION_START and later: any real time passes */
    }
    return e;
}

void orc_eq_free(void* p) {
    orc_eq_t* e = (orc_eq_t*)p;
    if (!e) return;
    for (uint32_t h = 0; h < e->n_hosts; h++) {
        free(e->q[h].a);
        free(e->q[h].pop);
        pthread_mutex_destroy(&e->q[h].mu);
    }
    free(e->q);
    free(e);
}

/* push_packet_to_host for one event, under the destination's mutex (callable from any thread) */
int orc_eq_push_one(void* p, uint32_t dst, uint64_t t, uint32_t src, uint64_t seq, uint64_t tag) {
    orc_eq_t* e = (orc_eq_t*)p;
    hq_t* q = &e->q[dst];
    qev_t x = {t, src, 0, seq, tag};
    pthread_mutex_lock(&q->mu);
    int rc = hq_push(q, x);
    pthread_mutex_unlock(&q->mu);
    return rc;
}

/* A batch grouped by destination (off[n_hosts + 1]), tag = batch_no << 32 | pkt[k]. */
int orc_eq_push_batch(void* p, const uint32_t* off, const uint64_t* t, const uint32_t* src, const uint64_t* seq,
                      const uint32_t* pkt, uint64_t batch_no, int threads) {
    orc_eq_t* e = (orc_eq_t*)p;
    int bad = 0;
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 64) reduction(| : bad)
    for (uint32_t h = 0; h < e->n_hosts; h++)
        for (uint32_t k = off[h]; k < off[h + 1]; k++) {
            qev_t x = {t[k], src[k], 0, seq[k], (batch_no << 32) | pkt[k]};
            bad |= hq_push(&e->q[h], x);
        }
    return bad;
}

/*
 * Every host pops its events with time < window_end, in order (host.rs:697-706).  out_* may be
 * NULL (count only).  Returns the number popped, or -1 when a pop would move a host's time
 * backwards (event_queue.rs:36-40 panics).  *n_pending = events left, *next_time = the minimum
 * next_event_time over the hosts (UINT64_MAX when every queue is empty).
 */
int64_t orc_eq_pop(void* p, uint64_t window_end, uint32_t* out_off, uint64_t* out_t, uint32_t* out_src,
                   uint64_t* out_seq, uint64_t* out_tag, uint64_t* n_pending, uint64_t* next_time, int threads) {
    orc_eq_t* e = (orc_eq_t*)p;
    const uint32_t H = e->n_hosts;
    int bad = 0;
    uint64_t left = 0, head = ~0ULL;
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 64) reduction(| : bad) reduction(+ : left) reduction(min : head)
    for (uint32_t h = 0; h < H; h++) {
        hq_t* q = &e->q[h];
        q->npop = 0;
        while (q->n && q->a[0].t < window_end) {
            qev_t x = hq_pop(q);
            if (x.t < q->last) bad = 1;
            q->last = x.t;
            if (q->npop == q->popcap) {
                uint32_t c = q->popcap ? q->popcap * 2 : 16;
                qev_t* na = (qev_t*)realloc(q->pop, (size_t)c * sizeof(qev_t));
                if (!na) { bad = 1; break; }
                q->pop = na;
                q->popcap = c;
            }
            q->pop[q->npop++] = x;
        }
        left += q->n;
        if (q->n && q->a[0].t < head) head = q->a[0].t;
    }
    if (n_pending) *n_pending = left;
    if (next_time) *next_time = head;
    if (bad) return -1;
    uint64_t tot = 0;
    for (uint32_t h = 0; h < H; h++) {
        if (out_off) out_off[h] = (uint32_t)tot;
        tot += e->q[h].npop;
    }
    if (out_off) out_off[H] = (uint32_t)tot;
    if (out_t) {
#pragma omp parallel for schedule(dynamic, 64)
        for (uint32_t h = 0; h < H; h++) {
            const hq_t* q = &e->q[h];
            for (uint32_t k = 0; k < q->npop; k++) {
                const size_t o = (size_t)out_off[h] + k;
                out_t[o] = q->pop[k].t;
                if (out_src) out_src[o] = q->pop[k].src;
                if (out_seq) out_seq[o] = q->pop[k].seq;
                if (out_tag) out_tag[o] = q->pop[k].tag;
            }
        }
    }
    return (int64_t)tot;
}

/* The pending events of every host in pop order (a sorted copy of each heap). */
uint64_t orc_eq_pending(void* p, uint32_t* out_off, uint64_t* out_t, uint32_t* out_src, uint64_t* out_seq,
                        uint64_t* out_tag) {
    orc_eq_t* e = (orc_eq_t*)p;
    uint64_t tot = 0;
    for (uint32_t h = 0; h < e->n_hosts; h++) {
        if (out_off) out_off[h] = (uint32_t)tot;
        tot += e->q[h].n;
    }
    if (out_off) out_off[e->n_hosts] = (uint32_t)tot;
    if (!out_t) return tot;
#pragma omp parallel for schedule(dynamic, 64)
    for (uint32_t h = 0; h < e->n_hosts; h++) {
        hq_t* q = &e->q[h];
        hq_t tmp = {0};
        tmp.a = (qev_t*)malloc(((size_t)q->n + 1) * sizeof(qev_t));
        memcpy(tmp.a, q->a, (size_t)q->n * sizeof(qev_t));
        tmp.n = tmp.cap = q->n;
        for (uint32_t k = 0; k < q->n; k++) {
            const qev_t x = hq_pop(&tmp);
            const size_t o = (size_t)out_off[h] + k;
            out_t[o] = x.t;
            if (out_src) out_src[o] = x.src;
            if (out_seq) out_seq[o] = x.seq;
            if (out_tag) out_tag[o] = x.tag;
        }
        free(tmp.a);
    }
    return tot;
}
