/*
 * hj_oracle.c — CPU restatement of the reference's hash-join hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker or the reported CPU
 * baseline — never as the product path (the product is the gfx950 HIP library, which
 * has no CPU fallback).
 *
 * Reference: jamesfer/datafusion-parallelism (paths relative to that repository).
 * The reference is nightly Rust whose version 10 needs aarch64 NEON; nothing of it can
 * be built or run here, so this is a restatement, pinned by the
 * reference's own known-answer tests (tests/golden/reference_kats.json).
 *
 * Two entry points:
 *
 *  1. ora_inner_join — the reference semantics, single-threaded, parallelism 1:
 *     build = the chained insert of Version 1 / ConcurrentSelfHashJoinMap
 *       (src/utils/concurrent_self_hash_join_map.rs:83-90: map[hash] = row+1, the
 *        previous head goes to overflow[row+1]; 223-249: iterate head, overflow[...]),
 *     probe = get_matching_indices (src/shared/shared.rs:29-47) in probe order with the
 *       chain order newest -> oldest, then equal_rows_arr (src/shared/
 *       datafusion_private.rs:40-80): keep a candidate only if both keys are non-null
 *       and equal (eq with null_equals_null = false). Null rows are hashed and chained
 *       like any row (their hash is a fixed value) and removed by the equality filter.
 *     The hash is this file's own (ahash 0.8.11 with seed 0 is not available here);
 *     hash_mode 1 uses a deliberately weak 4-bit hash to force collisions so that the
 *     equality filter is exercised. Emitted pairs do not depend on the hash.
 *
 *  2. ora_v10_* — the CPU baseline: a multithreaded restatement of the Version 10
 *     lock-free table (src/operator/version10/new_map_3/fixed_table.rs:560-672
 *     insert_atomically, 209-236 get; group.rs:529-531 tag = max(h>>56, 1);
 *     probe_sequence.rs:56-85 stride (2*tag+1)*8; fixed_table.rs:1008-1029 capacity
 *     next_pow2(n*8/7)), chains in an overflow array
 *     (version10/parallel_join_execution_state.rs:91-133), probe + chain walk
 *     (version10/lookup_implementation_3.rs:22-59) + key re-check. Pre-sized: the
 *     generation growth/migration of new_map_3.rs:325-411 is not restated (it only
 *     adds work), which favours the baseline.
 */
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t ora_fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

uint64_t ora_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline int valid_bit(const uint8_t* v, int64_t i) {
    return v == NULL ? 1 : (v[i >> 3] >> (i & 7)) & 1;
}

/* hash of a (possibly null) key; null rows get the fixed value 0 */
static inline uint64_t key_hash(int64_t key, int is_valid, int hash_mode) {
    if (!is_valid) return 0;
    if (hash_mode == 1) return (uint64_t)key & 0xF; /* weak: many collisions */
    return ora_fmix64((uint64_t)key);
}

/* ---------------------------------------------------------------------------
 * 1. reference semantics
 * ------------------------------------------------------------------------- */

/* hash -> head map (open addressing over the 64-bit hash value, like the reference's
 * DashMap<u64, usize, BypassHasher>) */
typedef struct {
    uint64_t* h;
    uint64_t* head; /* 0 = empty, else row + 1 */
    uint64_t mask;
} OraMap;

static int map_init(OraMap* m, int64_t n) {
    uint64_t cap = 16;
    while (cap < (uint64_t)n * 2 + 16) cap <<= 1;
    m->h = (uint64_t*)calloc(cap, 8);
    m->head = (uint64_t*)calloc(cap, 8);
    m->mask = cap - 1;
    return m->h && m->head;
}

static void map_free(OraMap* m) {
    free(m->h);
    free(m->head);
}

/* insert (hash -> v); returns the previous value or 0 */
static uint64_t map_insert(OraMap* m, uint64_t h, uint64_t v) {
    uint64_t i = ora_fmix64(h ^ 0x5bd1e995ull) & m->mask;
    for (;;) {
        if (m->head[i] == 0) {
            m->h[i] = h;
            m->head[i] = v;
            return 0;
        }
        if (m->h[i] == h) {
            uint64_t prev = m->head[i];
            m->head[i] = v;
            return prev;
        }
        i = (i + 1) & m->mask;
    }
}

static uint64_t map_get(const OraMap* m, uint64_t h) {
    uint64_t i = ora_fmix64(h ^ 0x5bd1e995ull) & m->mask;
    for (;;) {
        if (m->head[i] == 0) return 0;
        if (m->h[i] == h) return m->head[i];
        i = (i + 1) & m->mask;
    }
}

/* Returns the number of matching pairs (or -1 on allocation failure); writes the first
 * min(count, cap) pairs in canonical order. bkeys/pkeys are int64 (int32 inputs are
 * widened by the caller). */
int64_t ora_inner_join(const int64_t* bkeys, const uint8_t* bvalid, int64_t nb, const int64_t* pkeys,
                       const uint8_t* pvalid, int64_t np, int hash_mode, uint64_t* out_b, uint32_t* out_p,
                       int64_t cap) {
    OraMap m;
    if (!map_init(&m, nb)) return -1;
    uint64_t* overflow = (uint64_t*)calloc((size_t)nb + 1, 8);
    if (!overflow) {
        map_free(&m);
        return -1;
    }
    for (int64_t i = 0; i < nb; ++i) {
        const int vb = valid_bit(bvalid, i);
        const uint64_t prev = map_insert(&m, key_hash(bkeys[i], vb, hash_mode), (uint64_t)i + 1);
        overflow[i + 1] = prev; /* Inserter::insert: buffer[index] = existing */
    }
    int64_t count = 0;
    for (int64_t j = 0; j < np; ++j) {
        const int vp = valid_bit(pvalid, j);
        uint64_t idx = map_get(&m, key_hash(pkeys[j], vp, hash_mode));
        while (idx != 0) { /* ReadOnlyJoinMapIterator::next */
            const int64_t b = (int64_t)idx - 1;
            /* equal_rows_arr: eq(take(build), take(probe)); null -> not equal */
            if (vp && valid_bit(bvalid, b) && bkeys[b] == pkeys[j]) {
                if (count < cap) {
                    out_b[count] = (uint64_t)b;
                    out_p[count] = (uint32_t)j;
                }
                ++count;
            }
            idx = overflow[idx];
        }
    }
    free(overflow);
    map_free(&m);
    return count;
}

/* Chain links at parallelism 1: prev[i] = the next older row in i's chain (after the
 * reference's insert returns the previous value), -1 if none. Chains are by hash; with
 * hash_mode 0 (no collisions at test sizes) they equal chains by key. */
int64_t ora_chain_links(const int64_t* bkeys, const uint8_t* bvalid, int64_t nb, int hash_mode, int64_t* prev) {
    OraMap m;
    if (!map_init(&m, nb)) return -1;
    for (int64_t i = 0; i < nb; ++i) {
        const int vb = valid_bit(bvalid, i);
        const uint64_t p = map_insert(&m, key_hash(bkeys[i], vb, hash_mode), (uint64_t)i + 1);
        prev[i] = (int64_t)p - 1;
    }
    map_free(&m);
    return 0;
}

/* ---------------------------------------------------------------------------
 * 2. Version 10 restatement (multithreaded CPU baseline)
 * ------------------------------------------------------------------------- */

#define V10_GROUP 8
#define V10_OCCUPIED (1ull << 63)

typedef struct {
    _Atomic uint64_t h; /* hash | bit63, 0 = empty */
    _Atomic uint64_t v; /* row + 1 */
} V10Slot;

typedef struct {
    _Atomic uint8_t* tags; /* cap + GROUP, the first GROUP mirrored at the end */
    V10Slot* slots;
    uint64_t mask;
    uint64_t max_attempts;
    uint64_t* overflow; /* n + 1 chain links */
    const int64_t* bkeys;
    int64_t nb;
} V10Table;

static inline uint8_t v10_tag(uint64_t h) {
    uint8_t t = (uint8_t)(h >> 56);
    return t > 1 ? t : 1;
}

static inline uint64_t v10_next(uint64_t idx, uint8_t tag, uint64_t mask) {
    return (idx + ((uint64_t)tag * 2 + 1) * V10_GROUP) & mask;
}

static void v10_set_tag(V10Table* t, uint64_t idx, uint8_t tag) {
    const uint64_t idx2 = ((idx - V10_GROUP) & t->mask) + V10_GROUP; /* wrap mirror */
    atomic_store_explicit(&t->tags[idx], tag, memory_order_relaxed);
    atomic_store_explicit(&t->tags[idx2], tag, memory_order_relaxed);
}

/* insert_atomically: returns the previous value (0 = none), or UINT64_MAX if full */
static uint64_t v10_insert(V10Table* t, uint64_t hash, uint64_t value) {
    const uint8_t tag = v10_tag(hash);
    const uint64_t sh = hash | V10_OCCUPIED;
    uint64_t idx = hash & t->mask;
    for (uint64_t attempt = 0; attempt < t->max_attempts; ++attempt) {
        uint8_t g[V10_GROUP];
        for (int p = 0; p < V10_GROUP; ++p) g[p] = atomic_load_explicit(&t->tags[idx + p], memory_order_relaxed);
        for (int p = 0; p < V10_GROUP; ++p) {
            if (g[p] != tag) continue;
            V10Slot* s = &t->slots[(idx + p) & t->mask];
            const uint64_t ih = atomic_load_explicit(&s->h, memory_order_relaxed);
            if (ih == sh) return atomic_exchange_explicit(&s->v, value, memory_order_relaxed);
            if (ih == 0) g[p] = 0; /* tag seen before hash: treat as empty, re-check */
        }
        for (int p = 0; p < V10_GROUP; ++p) {
            if (g[p] != 0) continue;
            const uint64_t i = (idx + p) & t->mask;
            V10Slot* s = &t->slots[i];
            uint64_t expected = 0;
            if (atomic_compare_exchange_strong_explicit(&s->h, &expected, sh, memory_order_relaxed,
                                                        memory_order_relaxed)) {
                const uint64_t prev = atomic_exchange_explicit(&s->v, value, memory_order_relaxed);
                v10_set_tag(t, i, tag);
                return prev;
            }
            if (expected == sh) return atomic_exchange_explicit(&s->v, value, memory_order_relaxed);
        }
        idx = v10_next(idx, tag, t->mask);
    }
    return UINT64_MAX;
}

static uint64_t v10_get(const V10Table* t, uint64_t hash) {
    const uint8_t tag = v10_tag(hash);
    const uint64_t sh = hash | V10_OCCUPIED;
    uint64_t idx = hash & t->mask;
    for (uint64_t attempt = 0; attempt <= t->max_attempts; ++attempt) {
        int has_empty = 0;
        for (int p = 0; p < V10_GROUP; ++p) {
            const uint8_t tg = atomic_load_explicit(&t->tags[idx + p], memory_order_relaxed);
            if (tg == tag) {
                const V10Slot* s = &t->slots[(idx + p) & t->mask];
                if (atomic_load_explicit(&((V10Slot*)s)->h, memory_order_relaxed) == sh)
                    return atomic_load_explicit(&((V10Slot*)s)->v, memory_order_relaxed);
            } else if (tg == 0) {
                has_empty = 1;
            }
        }
        if (has_empty) return 0;
        idx = v10_next(idx, tag, t->mask);
    }
    return 0;
}

typedef struct {
    V10Table* t;
    const int64_t* keys;
    const uint8_t* valid;
    int64_t begin, end;
    int fail;
    /* probe */
    uint64_t* out_b;
    uint32_t* out_p;
    int64_t cap, count;
} V10Work;

static void* v10_build_worker(void* arg) {
    V10Work* w = (V10Work*)arg;
    for (int64_t i = w->begin; i < w->end; ++i) {
        const int vb = valid_bit(w->valid, i);
        const uint64_t prev = v10_insert(w->t, key_hash(w->keys[i], vb, 0), (uint64_t)i + 1);
        if (prev == UINT64_MAX) {
            w->fail = 1;
            return NULL;
        }
        w->t->overflow[i + 1] = prev;
    }
    return NULL;
}

static void* v10_probe_worker(void* arg) {
    V10Work* w = (V10Work*)arg;
    const V10Table* t = w->t;
    int64_t c = 0;
    const int emit = w->cap > 0;
    for (int64_t j = w->begin; j < w->end; ++j) {
        const int vp = valid_bit(w->valid, j);
        uint64_t idx = v10_get(t, key_hash(w->keys[j], vp, 0));
        while (idx != 0) {
            const int64_t b = (int64_t)idx - 1;
            if (vp && t->bkeys[b] == w->keys[j]) {
                if (emit) {  /* ProbeBuildIndices grow as the reference's Vec builders do */
                    if (c == w->cap) {
                        w->cap *= 2;
                        w->out_b = (uint64_t*)realloc(w->out_b, (size_t)w->cap * 8);
                        w->out_p = (uint32_t*)realloc(w->out_p, (size_t)w->cap * 4);
                        if (!w->out_b || !w->out_p) {
                            w->fail = 1;
                            return NULL;
                        }
                    }
                    w->out_b[c] = (uint64_t)b;
                    w->out_p[c] = (uint32_t)j;
                }
                ++c;
            }
            idx = t->overflow[idx];
        }
    }
    w->count = c;
    return NULL;
}

static int run_threads(void* (*fn)(void*), V10Work* w, int nthreads) {
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    if (!th) return -1;
    for (int i = 1; i < nthreads; ++i) pthread_create(&th[i], NULL, fn, &w[i]);
    fn(&w[0]);
    for (int i = 1; i < nthreads; ++i) pthread_join(th[i], NULL);
    free(th);
    return 0;
}

/* Build over n rows with nthreads partitions (contiguous row ranges); returns an opaque
 * table or NULL. Null rows are chained under hash 0 like the reference. */
void* ora_v10_build(const int64_t* bkeys, const uint8_t* bvalid, int64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    V10Table* t = (V10Table*)calloc(1, sizeof(V10Table));
    if (!t) return NULL;
    uint64_t want = (uint64_t)n * 8 / 7;
    uint64_t cap = V10_GROUP;
    while (cap < want) cap <<= 1;
    t->mask = cap - 1;
    t->max_attempts = cap / V10_GROUP;
    t->tags = (_Atomic uint8_t*)calloc(cap + V10_GROUP, 1);
    t->slots = (V10Slot*)calloc(cap, sizeof(V10Slot));
    t->overflow = (uint64_t*)calloc((size_t)n + 1, 8);
    t->bkeys = bkeys;
    t->nb = n;
    if (!t->tags || !t->slots || !t->overflow) return NULL;
    V10Work* w = (V10Work*)calloc((size_t)nthreads, sizeof(V10Work));
    for (int i = 0; i < nthreads; ++i) {
        w[i].t = t;
        w[i].keys = bkeys;
        w[i].valid = bvalid;
        w[i].begin = n * i / nthreads;
        w[i].end = n * (i + 1) / nthreads;
    }
    run_threads(v10_build_worker, w, nthreads);
    int fail = 0;
    for (int i = 0; i < nthreads; ++i) fail |= w[i].fail;
    free(w);
    if (fail) return NULL;
    return t;
}

/* Probe with nthreads contiguous chunks. If out_b/out_p are given (cap > 0) the pairs
 * are written chunk after chunk (probe ascending; chains newest first). Returns the
 * total count. */
int64_t ora_v10_probe(void* table, const int64_t* pkeys, const uint8_t* pvalid, int64_t n, int nthreads,
                      uint64_t* out_b, uint32_t* out_p, int64_t cap) {
    if (nthreads < 1) nthreads = 1;
    V10Table* t = (V10Table*)table;
    V10Work* w = (V10Work*)calloc((size_t)nthreads, sizeof(V10Work));
    /* per-thread scratch, then concatenated in chunk order */
    for (int i = 0; i < nthreads; ++i) {
        w[i].t = t;
        w[i].keys = pkeys;
        w[i].valid = pvalid;
        w[i].begin = n * i / nthreads;
        w[i].end = n * (i + 1) / nthreads;
        const int64_t len = w[i].end - w[i].begin;
        /* per-thread pair buffers start at the chunk's rows and double when full */
        w[i].cap = cap > 0 ? len + 64 : 0;
        w[i].out_b = w[i].cap ? (uint64_t*)malloc((size_t)w[i].cap * 8) : NULL;
        w[i].out_p = w[i].cap ? (uint32_t*)malloc((size_t)w[i].cap * 4) : NULL;
    }
    run_threads(v10_probe_worker, w, nthreads);
    int64_t total = 0;
    for (int i = 0; i < nthreads; ++i) {
        if (w[i].fail) total = INT64_MIN / 2; /* allocation failure: report a negative count */
        if (cap > 0) {
            const int64_t c = w[i].count < w[i].cap ? w[i].count : w[i].cap;
            for (int64_t k = 0; k < c && total + k < cap; ++k) {
                out_b[total + k] = w[i].out_b[k];
                out_p[total + k] = w[i].out_p[k];
            }
        }
        total += w[i].count;
        free(w[i].out_b);
        free(w[i].out_p);
    }
    free(w);
    return total;
}

/* One probe pass that emits: the per-thread pair buffers concatenated in chunk order into
 * malloc'd arrays (*out_b, *out_p; release with ora_free). Returns the pair count, < 0 on
 * allocation failure. */
int64_t ora_v10_probe_emit(void* table, const int64_t* pkeys, const uint8_t* pvalid, int64_t n, int nthreads,
                           uint64_t** out_b, uint32_t** out_p) {
    if (nthreads < 1) nthreads = 1;
    V10Table* t = (V10Table*)table;
    V10Work* w = (V10Work*)calloc((size_t)nthreads, sizeof(V10Work));
    for (int i = 0; i < nthreads; ++i) {
        w[i].t = t;
        w[i].keys = pkeys;
        w[i].valid = pvalid;
        w[i].begin = n * i / nthreads;
        w[i].end = n * (i + 1) / nthreads;
        w[i].cap = (w[i].end - w[i].begin) + 64;
        w[i].out_b = (uint64_t*)malloc((size_t)w[i].cap * 8);
        w[i].out_p = (uint32_t*)malloc((size_t)w[i].cap * 4);
    }
    run_threads(v10_probe_worker, w, nthreads);
    int64_t total = 0;
    int fail = 0;
    for (int i = 0; i < nthreads; ++i) {
        total += w[i].count;
        fail |= w[i].fail;
    }
    uint64_t* ob = fail ? NULL : (uint64_t*)malloc((size_t)(total > 0 ? total : 1) * 8);
    uint32_t* op = fail ? NULL : (uint32_t*)malloc((size_t)(total > 0 ? total : 1) * 4);
    int64_t pos = 0;
    for (int i = 0; i < nthreads; ++i) {
        if (ob && op) {
            memcpy(ob + pos, w[i].out_b, (size_t)w[i].count * 8);
            memcpy(op + pos, w[i].out_p, (size_t)w[i].count * 4);
        }
        pos += w[i].count;
        free(w[i].out_b);
        free(w[i].out_p);
    }
    free(w);
    if (!ob || !op) {
        free(ob);
        free(op);
        return -1;
    }
    *out_b = ob;
    *out_p = op;
    return total;
}

void ora_free(void* p) { free(p); }

/* The lookup_speed bench's timed loop (benches/lookup_speed.rs:240-246): get_iter(&i) for
 * the raw values i in [start, start + count) used as hashes (IndexLookup<u64> is keyed by
 * hash, version10/lookup_implementation_3.rs:46-59), each chain walked to the end as
 * .collect() does. Single thread, as the reference calls the partitions' lookup
 * functions one after another. Returns the number of rows the chains yielded. */
int64_t ora_v10_lookup_hashes(void* table, uint64_t start, int64_t count) {
    const V10Table* t = (const V10Table*)table;
    int64_t rows = 0;
    for (int64_t k = 0; k < count; ++k) {
        uint64_t idx = v10_get(t, start + (uint64_t)k);
        while (idx != 0) {
            ++rows;
            idx = t->overflow[idx];
        }
    }
    return rows;
}

void ora_v10_free(void* table) {
    V10Table* t = (V10Table*)table;
    if (!t) return;
    free((void*)t->tags);
    free(t->slots);
    free(t->overflow);
    free(t);
}

/* splitmix64 generator: out[i] = splitmix64(seed + i) mod range */
void ora_gen_uniform(int64_t* out, int64_t n, uint64_t seed, int64_t range) {
    for (int64_t i = 0; i < n; ++i) out[i] = (int64_t)(ora_splitmix64(seed + (uint64_t)i) % (uint64_t)range);
}

/* src/api_utils.rs:15-23 make_exponential_int_array: x = n as f32 / diff as f32,
 * y = (16f32.pow(x) - 1) / 15, value = min + (y * diff as f32) as i32. f32::powf lowers
 * to libm powf (glibc on the reference's Linux hosts); numpy's float32 power is a
 * different approximation (it differs in 2,097,710 of the 10^7 C3 inputs and moves
 * 619,311 keys), so the restatement calls powf itself, through a volatile pointer so
 * that the compiler neither folds nor vectorizes it. */
void ora_make_exponential(int32_t* out, int32_t lo, int32_t hi) {
    float (*volatile pw)(float, float) = powf;
    const int32_t diff = hi - lo;
    const float base = 16.0f;
    for (int32_t n = 0; n < diff; ++n) {
        const float x = (float)n / (float)diff;
        const float y = (pw(base, x) - 1.0f) / (base - 1.0f);
        out[n] = lo + (int32_t)(y * (float)diff);
    }
}
