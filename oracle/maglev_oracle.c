/*
 * TEST INFRASTRUCTURE ONLY — C oracle for the Maglev flow-steering path.
 *
 * Independent CPU restatement of NetBricks' test/maglev hot path.  It is the
 * bit-exact checker for full-size GPU runs and the timed CPU baseline
 * ("kind": "port") in bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load it; the product library never links it.
 *
 * Restated reference items (paths relative to the NetBricks repo root):
 *   offset/skip       test/maglev/src/nf.rs:21-31
 *   permutations      test/maglev/src/nf.rs:33-42   (computed on the fly)
 *   LUT fill          test/maglev/src/nf.rs:44-68
 *   lookup            test/maglev/src/nf.rs:78-81   (lut[hash % M])
 *   flow cache        test/maglev/src/nf.rs:91,104  (FNV-keyed memo, result-identical)
 *   MAC swap          framework/src/headers/mac.rs:140-145
 *   flow extraction   framework/src/utils/flow.rs:53-62 (payload = frame[14..len])
 *   Flow layout       framework/src/utils/flow.rs:10-18 (packed, little-endian)
 *   flow hash         framework/src/utils/flow.rs:96-110 (FNV-1a 64 over 13 B)
 *   group_by          framework/src/operators/group_by.rs:43-55 (per-group FIFO)
 *   mpsc enqueue      framework/src/queues/mpsc_mbuf_queue.rs:91-115 (1024-slot ring)
 *   burst size        framework/src/operators/receive_batch.rs:26 (32 packets)
 *
 * XXH64 comes from the upstream xxHash header vendored in this image
 * (pyarrow/include/arrow/vendored/xxhash/xxhash.h, the published algorithm that
 * twox-hash 1.x `XxHash` implements), NOT from the product's own XXH64, so the
 * two implementations check each other.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define XXH_INLINE_ALL
#include "xxhash.h"

#define ORC_ETH 14
#define ORC_EMPTY 0x8000u
#define ORC_SENTINEL 0xFFFFu

static const uint64_t FNV_OFF = 0xcbf29ce484222325ULL;
static const uint64_t FNV_PRIME = 0x100000001b3ULL;

static uint64_t fnv1a(const uint8_t *p, size_t n) {
    uint64_t h = FNV_OFF;
    for (size_t i = 0; i < n; i++) {
        h ^= p[i];
        h *= FNV_PRIME;
    }
    return h;
}

uint64_t orc_fnv1a64(const uint8_t *p, uint64_t n) { return fnv1a(p, (size_t)n); }
uint64_t orc_xxh64(const uint8_t *p, uint64_t n, uint64_t seed) { return XXH64(p, (size_t)n, seed); }

/* nf.rs:21-31 — Rust `str: Hash` feeds name bytes then 0xFF. */
void orc_offset_skip(const char *name, uint32_t len, uint64_t m, uint64_t *offset, uint64_t *skip) {
    uint8_t *b = (uint8_t *)malloc(len + 1);
    memcpy(b, name, len);
    b[len] = 0xff;
    uint64_t h1 = fnv1a(b, len + 1);
    uint64_t h2 = XXH64(b, len + 1, 0);
    free(b);
    *offset = h2 % m;
    *skip = h1 % (m - 1) + 1;
}

/* nf.rs:44-68 with perm[i][j] = (offset_i + j*skip_i) % M evaluated on demand. */
int orc_lut_build(const char *const *names, const uint32_t *lens, uint32_t n, uint64_t m, uint32_t *entry) {
    if (n == 0 || m < 2) return -22;
    uint64_t *off = (uint64_t *)malloc(n * sizeof(uint64_t));
    uint64_t *skip = (uint64_t *)malloc(n * sizeof(uint64_t));
    uint64_t *next = (uint64_t *)calloc(n, sizeof(uint64_t));
    for (uint32_t i = 0; i < n; i++) orc_offset_skip(names[i], lens[i], m, &off[i], &skip[i]);
    for (uint64_t j = 0; j < m; j++) entry[j] = ORC_EMPTY;
    uint64_t filled = 0;
    while (filled < m) {
        for (uint32_t i = 0; i < n; i++) {
            uint64_t c = (off[i] + (unsigned __int128)next[i] * skip[i] % m) % m;
            while (entry[c] != ORC_EMPTY) {
                next[i]++;
                if (next[i] >= m) { /* permutations[i][m] is out of bounds: the reference panics */
                    free(off);
                    free(skip);
                    free(next);
                    return -34;
                }
                c = (off[i] + (unsigned __int128)next[i] * skip[i] % m) % m;
            }
            if (entry[c] == ORC_EMPTY) {
                entry[c] = i;
                next[i]++;
                filled++;
            }
            if (filled >= m) break;
        }
    }
    free(off);
    free(skip);
    free(next);
    return 0;
}

/* flow.rs:53-62 + flow.rs:105-110.  Returns 0 when the Rust slice would panic. */
static int flow_hash_of(const uint8_t *frame, uint32_t len, uint64_t *out) {
    if (len < ORC_ETH) return 0;
    const uint8_t *p = frame + ORC_ETH;
    uint32_t plen = len - ORC_ETH;
    if (plen < 1) return 0;
    uint32_t ps = (uint32_t)(p[0] & 0xf) * 4;
    if (plen < 20 || plen < ps + 4) return 0;
    uint32_t src = (uint32_t)p[12] << 24 | (uint32_t)p[13] << 16 | (uint32_t)p[14] << 8 | p[15];
    uint32_t dst = (uint32_t)p[16] << 24 | (uint32_t)p[17] << 16 | (uint32_t)p[18] << 8 | p[19];
    uint16_t sport = (uint16_t)(p[ps] << 8 | p[ps + 1]);
    uint16_t dport = (uint16_t)(p[ps + 2] << 8 | p[ps + 3]);
    uint8_t flow[13]; /* #[repr(C, packed)] Flow, little-endian fields */
    memcpy(flow + 0, &src, 4);
    memcpy(flow + 4, &dst, 4);
    memcpy(flow + 8, &sport, 2);
    memcpy(flow + 10, &dport, 2);
    flow[12] = p[9];
    *out = fnv1a(flow, 13);
    return 1;
}

static inline void mac_swap(uint8_t *frame) {
    uint8_t tmp[6];
    memcpy(tmp, frame, 6);
    memcpy(frame, frame + 6, 6);
    memcpy(frame + 6, tmp, 6);
}

static inline uint64_t pkt_off(const uint64_t *offs, uint64_t stride, uint64_t i) {
    return offs ? offs[i] : i * stride;
}

static inline uint32_t pkt_len(const uint16_t *lens, uint32_t fixed_len, uint64_t i) {
    return lens ? lens[i] : fixed_len;
}

/* Per-packet classify (no cache): backend[i] = lut[fnv(flow) % M] or the sentinel.
 * `buf` is mutated by the MAC swap when swap != 0. */
void orc_classify(uint8_t *buf, const uint64_t *offs, uint64_t stride, const uint16_t *lens, uint32_t fixed_len,
                  uint64_t n, const uint32_t *lut, uint64_t m, int swap, uint16_t *backend) {
    for (uint64_t i = 0; i < n; i++) {
        uint8_t *f = buf + pkt_off(offs, stride, i);
        uint32_t len = pkt_len(lens, fixed_len, i);
        if (len < ORC_ETH) {
            backend[i] = ORC_SENTINEL;
            continue;
        }
        if (swap) mac_swap(f);
        uint64_t h;
        backend[i] = flow_hash_of(f, len, &h) ? (uint16_t)lut[h % m] : ORC_SENTINEL;
    }
}

uint64_t orc_flow_hash(const uint8_t *frame, uint32_t len, int *ok) {
    uint64_t h = 0;
    *ok = flow_hash_of(frame, len, &h);
    return h;
}

/* Stable partition by backend: groups 0..nb-1 then the sentinel group (index nb). */
void orc_group(const uint16_t *backend, uint64_t n, uint32_t nb, uint32_t *perm, uint32_t *counts) {
    uint64_t *start = (uint64_t *)calloc(nb + 1, sizeof(uint64_t));
    memset(counts, 0, (nb + 1) * sizeof(uint32_t));
    for (uint64_t i = 0; i < n; i++) counts[backend[i] == ORC_SENTINEL ? nb : backend[i]]++;
    uint64_t acc = 0;
    for (uint32_t b = 0; b <= nb; b++) {
        start[b] = acc;
        acc += counts[b];
    }
    for (uint64_t i = 0; i < n; i++) {
        uint32_t b = backend[i] == ORC_SENTINEL ? nb : backend[i];
        perm[start[b]++] = (uint32_t)i;
    }
    free(start);
}

/* ------------------------------------------------------------------------- */
/* CPU baseline: the reference's per-core producer loop, restated.            */
/* Per 32-packet burst (receive_batch.rs:26): MAC swap over the burst          */
/* (transform_batch.rs:70-81), then per packet group_fn with the FNV-keyed     */
/* memo map (nf.rs:91,104), save_header_and_offset (2 stores, packet.rs:217),  */
/* enqueue_one into the group's 1024-slot ring (mpsc_mbuf_queue.rs:91-115).    */
/* Rings are drained by the same thread after each burst (the consumer side    */
/* runs on the same core in the reference's scheduler).                        */
/* ------------------------------------------------------------------------- */

typedef struct {
    uint64_t *keys; /* hash+1, 0 = empty */
    uint32_t *vals;
    uint64_t mask;
    uint64_t used;
} memo_t;

static void memo_init(memo_t *mm, uint64_t cap_pow2) {
    mm->keys = (uint64_t *)calloc(cap_pow2, sizeof(uint64_t));
    mm->vals = (uint32_t *)calloc(cap_pow2, sizeof(uint32_t));
    mm->mask = cap_pow2 - 1;
    mm->used = 0;
}

static void memo_free(memo_t *mm) {
    free(mm->keys);
    free(mm->vals);
}

static void memo_grow(memo_t *mm) {
    memo_t nm;
    memo_init(&nm, (mm->mask + 1) * 2);
    for (uint64_t i = 0; i <= mm->mask; i++) {
        if (!mm->keys[i]) continue;
        uint64_t k = mm->keys[i] - 1;
        uint64_t s = fnv1a((const uint8_t *)&k, 8) & nm.mask;
        while (nm.keys[s]) s = (s + 1) & nm.mask;
        nm.keys[s] = mm->keys[i];
        nm.vals[s] = mm->vals[i];
        nm.used++;
    }
    memo_free(mm);
    *mm = nm;
}

/* cache.entry(hash).or_insert_with(|| lut.lookup(hash)) — the map's own hasher is FNV. */
static inline uint32_t memo_get(memo_t *mm, uint64_t h, const uint32_t *lut, uint64_t m) {
    uint64_t s = fnv1a((const uint8_t *)&h, 8) & mm->mask;
    for (;;) {
        uint64_t k = mm->keys[s];
        if (k == h + 1) return mm->vals[s];
        if (k == 0) break;
        s = (s + 1) & mm->mask;
    }
    uint32_t v = lut[h % m];
    mm->keys[s] = h + 1;
    mm->vals[s] = v;
    if (++mm->used * 2 > mm->mask) memo_grow(mm);
    return v;
}

typedef struct {
    uint8_t *buf;
    const uint64_t *offs;
    uint64_t stride;
    const uint16_t *lens;
    uint32_t fixed_len;
    uint64_t begin, end;
    const uint32_t *lut;
    uint64_t m;
    uint32_t nb;
    int use_cache;
    int cpu;
    uint32_t reps; /* passes over the shard (the memo map persists, as across the reference's batches) */
    uint16_t *backend; /* optional output */
    uint64_t checksum;
    double seconds;
    double t_start, t_end; /* CLOCK_MONOTONIC seconds around the thread's loop */
    /* chain (config C5): test/lpm's stage before maglev when tbl24 is set */
    const uint16_t *tbl24, *tbl_long;
    uint32_t lpm_groups;
} orc_shard_t;

static inline uint16_t lpm_lookup(const uint16_t *tbl24, const uint16_t *tbl_long, uint32_t ip);

#define RING 1024
#define BURST 32

/* Thread placement of the baseline: thread t on CPU g_cpu_order[t % n] when a caller set an order
 * (orc_set_cpu_order; bench.py passes the drop-in path's own placement), else on the t-th allowed CPU. */
static int g_cpu_order[1024];
static int g_cpu_order_n = 0;

void orc_set_cpu_order(const int *cpus, int n) {
    g_cpu_order_n = 0;
    for (int i = 0; cpus && i < n && i < 1024; i++) g_cpu_order[g_cpu_order_n++] = cpus[i];
}

static void *shard_main(void *arg) {
    orc_shard_t *s = (orc_shard_t *)arg;
    if (s->cpu >= 0 && g_cpu_order_n > 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(g_cpu_order[s->cpu % g_cpu_order_n], &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    } else if (s->cpu >= 0) { /* pin to the cpu-th CPU of the allowed set (cgroup-safe) */
        cpu_set_t allowed, set;
        CPU_ZERO(&allowed);
        if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0) {
            int seen = 0;
            for (int c = 0; c < CPU_SETSIZE; c++) {
                if (!CPU_ISSET(c, &allowed)) continue;
                if (seen++ == s->cpu) {
                    CPU_ZERO(&set);
                    CPU_SET(c, &set);
                    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
                    break;
                }
            }
        }
    }
    uint32_t ng = s->nb + 1;
    uint8_t ***ring = (uint8_t ***)malloc(ng * sizeof(uint8_t **));
    uint64_t *head = (uint64_t *)calloc(ng, sizeof(uint64_t));
    uint64_t *tail = (uint64_t *)calloc(ng, sizeof(uint64_t));
    uint64_t (*meta)[2] = malloc(BURST * sizeof(*meta));
    for (uint32_t g = 0; g < ng; g++) ring[g] = (uint8_t **)malloc(RING * sizeof(uint8_t *));
    memo_t memo;
    memo_init(&memo, 1 << 12);
    uint64_t sum = 0;
    /* chain: test/lpm's group_by(lpm_groups) rings of packet indices */
    uint32_t nl = s->tbl24 ? s->lpm_groups : 0;
    uint64_t **lring = (uint64_t **)calloc(nl ? nl : 1, sizeof(uint64_t *));
    uint64_t *lhead = (uint64_t *)calloc(nl ? nl : 1, sizeof(uint64_t));
    uint64_t *ltail = (uint64_t *)calloc(nl ? nl : 1, sizeof(uint64_t));
    for (uint32_t g = 0; g < nl; g++) lring[g] = (uint64_t *)malloc(RING * sizeof(uint64_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint32_t rep = 0; rep < s->reps; rep++)
    for (uint64_t b = s->begin; b < s->end; b += BURST) {
        uint64_t e = b + BURST < s->end ? b + BURST : s->end;
        if (nl) {
            /* test/lpm (nf.rs:212-221): parse Mac + Ip, lookup_entry on the source address,
             * transform (MAC swap), group_by(lpm_groups); a packet the reference would panic on
             * (runt, gate >= lpm_groups) gets the sentinel and goes no further */
            for (uint64_t i = b; i < e; i++) {
                uint8_t *f = s->buf + pkt_off(s->offs, s->stride, i);
                uint32_t len = pkt_len(s->lens, s->fixed_len, i);
                uint32_t gate = ORC_SENTINEL;
                if (len >= ORC_ETH + 20) {
                    const uint8_t *ip = f + ORC_ETH;
                    gate = lpm_lookup(s->tbl24, s->tbl_long,
                                      (uint32_t)ip[12] << 24 | (uint32_t)ip[13] << 16 | (uint32_t)ip[14] << 8 | ip[15]);
                }
                if (gate >= nl) {
                    if (s->backend) s->backend[i] = ORC_SENTINEL;
                    continue;
                }
                mac_swap(f);
                if (lhead[gate] - ltail[gate] < RING - 1) lring[gate][lhead[gate]++ & (RING - 1)] = i;
            }
            /* test/maglev over the lpm groups in order: MAC swap back, group_fn, enqueue */
            for (uint32_t lg = 0; lg < nl; lg++) {
                while (ltail[lg] != lhead[lg]) {
                    uint64_t i = lring[lg][ltail[lg]++ & (RING - 1)];
                    uint8_t *f = s->buf + pkt_off(s->offs, s->stride, i);
                    uint32_t len = pkt_len(s->lens, s->fixed_len, i);
                    mac_swap(f);
                    uint64_t h;
                    uint32_t g;
                    if (!flow_hash_of(f, len, &h))
                        g = s->nb;
                    else
                        g = s->use_cache ? memo_get(&memo, h, s->lut, s->m) : s->lut[h % s->m];
                    if (s->backend) s->backend[i] = g == s->nb ? ORC_SENTINEL : (uint16_t)g;
                    meta[0][0] = (uint64_t)(uintptr_t)f;
                    meta[0][1] = ORC_ETH;
                    if (head[g] - tail[g] < RING - 1) ring[g][head[g]++ & (RING - 1)] = f;
                }
            }
            for (uint32_t g = 0; g < ng; g++) {
                while (tail[g] != head[g]) {
                    uint8_t *f = ring[g][tail[g]++ & (RING - 1)];
                    sum += (uint64_t)f[0] * (g + 1) + meta[0][1];
                }
            }
            continue;
        }
        /* transform: MAC swap over the burst */
        for (uint64_t i = b; i < e; i++) {
            uint8_t *f = s->buf + pkt_off(s->offs, s->stride, i);
            if (pkt_len(s->lens, s->fixed_len, i) >= ORC_ETH) mac_swap(f);
        }
        /* group_by producer */
        for (uint64_t i = b; i < e; i++) {
            uint8_t *f = s->buf + pkt_off(s->offs, s->stride, i);
            uint32_t len = pkt_len(s->lens, s->fixed_len, i);
            uint64_t h;
            uint32_t g;
            if (!flow_hash_of(f, len, &h))
                g = s->nb;
            else
                g = s->use_cache ? memo_get(&memo, h, s->lut, s->m) : s->lut[h % s->m];
            if (s->backend) s->backend[i] = g == s->nb ? ORC_SENTINEL : (uint16_t)g;
            meta[i - b][0] = (uint64_t)(uintptr_t)f; /* save_header_and_offset */
            meta[i - b][1] = ORC_ETH;
            if (head[g] - tail[g] < RING - 1) ring[g][head[g]++ & (RING - 1)] = f;
        }
        /* consumers: drain each group FIFO (merge + send stand-in) */
        for (uint32_t g = 0; g < ng; g++) {
            while (tail[g] != head[g]) {
                uint8_t *f = ring[g][tail[g]++ & (RING - 1)];
                sum += (uint64_t)f[0] * (g + 1) + meta[0][1];
            }
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    s->seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    s->t_start = (double)t0.tv_sec + 1e-9 * (double)t0.tv_nsec;
    s->t_end = (double)t1.tv_sec + 1e-9 * (double)t1.tv_nsec;
    s->checksum = sum;
    memo_free(&memo);
    for (uint32_t g = 0; g < nl; g++) free(lring[g]);
    free(lring);
    free(lhead);
    free(ltail);
    for (uint32_t g = 0; g < ng; g++) free(ring[g]);
    free(ring);
    free(head);
    free(tail);
    free(meta);
    return NULL;
}

/* Runs `threads` pinned threads, each `reps` times over a contiguous shard of [0, n).
 * Returns wall seconds from the first thread's loop start to the last thread's loop end (thread
 * start-up excluded; threads that do not run concurrently, e.g. under a CPU quota, count in full). */
static double run_shards(uint8_t *buf, const uint64_t *offs, uint64_t stride, const uint16_t *lens,
                         uint32_t fixed_len, uint64_t n, const uint16_t *tbl24, const uint16_t *tbl_long,
                         uint32_t lpm_groups, const uint32_t *lut, uint64_t m, uint32_t nb, int use_cache, int threads,
                         uint32_t reps, uint16_t *backend) {
    if (threads < 1) threads = 1;
    if (reps < 1) reps = 1;
    orc_shard_t *sh = (orc_shard_t *)calloc(threads, sizeof(orc_shard_t));
    pthread_t *tid = (pthread_t *)calloc(threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        sh[t] = (orc_shard_t){buf, offs, stride, lens, fixed_len, n * t / threads, n * (t + 1) / threads,
                              lut, m, nb, use_cache, threads > 1 ? t : -1, reps, backend, 0, 0.0, 0.0, 0.0,
                              tbl24, tbl_long, lpm_groups};
        pthread_create(&tid[t], NULL, shard_main, &sh[t]);
    }
    double first = 0.0, last = 0.0;
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        if (t == 0 || sh[t].t_start < first) first = sh[t].t_start;
        if (t == 0 || sh[t].t_end > last) last = sh[t].t_end;
    }
    free(sh);
    free(tid);
    return last - first;
}

double orc_cpu_baseline_reps(uint8_t *buf, const uint64_t *offs, uint64_t stride, const uint16_t *lens,
                             uint32_t fixed_len, uint64_t n, const uint32_t *lut, uint64_t m, uint32_t nb, int use_cache,
                             int threads, uint32_t reps, uint16_t *backend) {
    return run_shards(buf, offs, stride, lens, fixed_len, n, NULL, NULL, 0, lut, m, nb, use_cache, threads, reps,
                      backend);
}

/* The chained lpm -> maglev loop (config C5): per 32-packet burst test/lpm's stage (lookup,
 * swap, group_by(lpm_groups) rings), then test/maglev's over those groups in order. */
double orc_cpu_baseline_chain_reps(uint8_t *buf, const uint64_t *offs, uint64_t stride, const uint16_t *lens,
                                   uint32_t fixed_len, uint64_t n, const uint16_t *tbl24, const uint16_t *tbl_long,
                                   uint32_t lpm_groups, const uint32_t *lut, uint64_t m, uint32_t nb, int use_cache,
                                   int threads, uint32_t reps, uint16_t *backend) {
    return run_shards(buf, offs, stride, lens, fixed_len, n, tbl24, tbl_long, lpm_groups ? lpm_groups : 1, lut, m, nb,
                      use_cache, threads, reps, backend);
}

/* One pass per thread (the round-1 entry point). */
double orc_cpu_baseline(uint8_t *buf, const uint64_t *offs, uint64_t stride, const uint16_t *lens, uint32_t fixed_len,
                        uint64_t n, const uint32_t *lut, uint64_t m, uint32_t nb, int use_cache, int threads,
                        uint16_t *backend) {
    return orc_cpu_baseline_reps(buf, offs, stride, lens, fixed_len, n, lut, m, nb, use_cache, threads, 1, backend);
}


/* ---- test/lpm (chained before test/maglev, config C5) ------------------------------
 * IPLookup::construct_table (test/lpm/src/nf.rs:49-86) over routes given as arrays;
 * one length's routes are applied in ascending prefix order (see maglev_ref.IPLookup).
 * tbl24 and tbl_long have ORC_TBL24 entries each.  Returns 0, or -34 where the reference
 * panics (a fill past a table's end, prefix length > 32). */
#define ORC_TBL24 ((1u << 24) + 1u)

typedef struct { uint32_t k; uint16_t v; uint64_t seq; } orc_route;

static int route_cmp(const void *a, const void *b) {
    const orc_route *x = (const orc_route *)a, *y = (const orc_route *)b;
    if (x->k != y->k) return x->k < y->k ? -1 : 1;
    return x->seq < y->seq ? -1 : (x->seq > y->seq);
}

int orc_lpm_build(const uint32_t *prefixes, const uint8_t *lens, const uint16_t *gates, uint64_t n,
                  uint16_t *tbl24, uint16_t *tbl_long, uint64_t *long_used) {
    memset(tbl24, 0, ORC_TBL24 * sizeof(uint16_t));
    memset(tbl_long, 0, ORC_TBL24 * sizeof(uint16_t));
    uint64_t cur = 0;
    for (uint32_t len = 0; len <= 32; len++) {
        uint64_t cnt = 0;
        for (uint64_t i = 0; i < n; i++) {
            if (lens[i] > 32) return -34;
            cnt += lens[i] == len;
        }
        if (!cnt) continue;
        orc_route *r = (orc_route *)malloc(cnt * sizeof(orc_route));
        uint64_t c = 0;
        for (uint64_t i = 0; i < n; i++)
            if (lens[i] == len) { r[c].k = prefixes[i]; r[c].v = gates[i]; r[c].seq = i; c++; }
        qsort(r, cnt, sizeof(orc_route), route_cmp);
        for (uint64_t i = 0; i < cnt; i++) {
            if (i + 1 < cnt && r[i + 1].k == r[i].k) continue; /* HashMap::insert: the last one wins */
            const uint32_t k = r[i].k;
            const uint16_t v = r[i].v;
            if (len <= 24) {
                uint64_t start = k >> 8, end = start + (1ull << (24 - len));
                if (end > ORC_TBL24) { free(r); return -34; }
                for (uint64_t p = start; p < end; p++) tbl24[p] = v;
            } else {
                uint16_t t24 = tbl24[k >> 8];
                if (!(t24 & 0x8000)) {
                    if (cur + 256 > ORC_TBL24) { free(r); return -34; }
                    uint64_t start = cur + (k & 0xff), end = start + (1ull << (32 - len));
                    for (uint64_t j = cur; j < cur + 256; j++) tbl_long[j] = (j < start || j >= end) ? t24 : v;
                    tbl24[k >> 8] = (uint16_t)((uint16_t)(cur >> 8) | 0x8000);
                    cur += 256;
                } else {
                    uint64_t start = ((uint64_t)(t24 & 0x7fff) << 8) + (k & 0xff), end = start + (1ull << (32 - len));
                    if (end > ORC_TBL24) { free(r); return -34; }
                    for (uint64_t j = start; j < end; j++) tbl_long[j] = v;
                }
            }
        }
        free(r);
    }
    *long_used = cur;
    return 0;
}

static inline uint16_t lpm_lookup(const uint16_t *tbl24, const uint16_t *tbl_long, uint32_t ip) {
    uint16_t t = tbl24[ip >> 8];
    return (t & 0x8000) ? tbl_long[((uint32_t)(t & 0x7fff) << 8) + (ip & 0xff)] : t;
}

void orc_lpm_lookup(const uint16_t *tbl24, const uint16_t *tbl_long, const uint32_t *ips, uint64_t n, uint16_t *gate) {
    for (uint64_t i = 0; i < n; i++) gate[i] = lpm_lookup(tbl24, tbl_long, ips[i]);
}

/* lpm() -> maglev() per packet (test/lpm/src/nf.rs:212-228, test/maglev/src/nf.rs:92-106);
 * the two MAC swaps cancel, so `buf` is only read. */
void orc_chain_classify(const uint8_t *buf, const uint64_t *offs, uint64_t stride, const uint16_t *lens,
                        uint32_t fixed_len, uint64_t n, const uint16_t *tbl24, const uint16_t *tbl_long,
                        uint32_t lpm_groups, const uint32_t *lut, uint64_t m, uint16_t *gate, uint16_t *backend) {
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *f = buf + pkt_off(offs, stride, i);
        uint32_t len = pkt_len(lens, fixed_len, i);
        gate[i] = ORC_SENTINEL;
        backend[i] = ORC_SENTINEL;
        if (len < ORC_ETH + 20) continue; /* parse::<MacHeader>, parse::<IpHeader> asserts */
        const uint8_t *ip = f + ORC_ETH;
        uint32_t src = (uint32_t)ip[12] << 24 | (uint32_t)ip[13] << 16 | (uint32_t)ip[14] << 8 | ip[15];
        gate[i] = lpm_lookup(tbl24, tbl_long, src);
        if (gate[i] >= lpm_groups) continue; /* group index out of range: the reference panics */
        uint64_t h;
        if (flow_hash_of(f, len, &h)) backend[i] = (uint16_t)lut[h % m];
    }
}
