/*
 * swim_oracle.c — single-threaded CPU restatement of ringpop-go's swim protocol round.
 *
 * TEST INFRASTRUCTURE ONLY. It is the parity checker, never the product (swim_oracle.h has the
 * header). It follows the reference's data model: a per-node memberlist, a map-based
 * disseminator and a map-based timer table. It runs the canonical schedule of
 * docs/ROUND_SEMANTICS.md. Citations are maniacs-ops/ringpop-go swim/ file:line.
 */
#include "swim_oracle.h"

#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* int32-keyed open-addressing map (the reference uses Go maps keyed by address string)        */
/* ------------------------------------------------------------------------------------------ */
typedef struct slot {
    int32_t key; /* -1 empty, -2 deleted */
    int32_t a;   /* dissem: p          | timer: state */
    int32_t b;   /* dissem: source     | timer: fired */
    int32_t _pad;
    int64_t x;   /* dissem: source inc | timer: deadline ms */
    int64_t y;   /*                    | timer: subject inc */
} slot;

typedef struct omap {
    slot *s;
    uint32_t cap, used, live;
} omap;

static uint32_t hkey(int32_t k) {
    uint32_t h = (uint32_t)k * 0x9E3779B1u;
    return h ^ (h >> 15);
}

static void omap_init(omap *m) { m->s = NULL; m->cap = m->used = m->live = 0; }
static void omap_free(omap *m) { free(m->s); omap_init(m); }

static slot *omap_find(const omap *m, int32_t k) {
    if (!m->cap) return NULL;
    uint32_t i = hkey(k) & (m->cap - 1);
    for (;;) {
        slot *e = &m->s[i];
        if (e->key == k) return e;
        if (e->key == -1) return NULL;
        i = (i + 1) & (m->cap - 1);
    }
}

static void omap_rehash(omap *m, uint32_t ncap) {
    slot *old = m->s;
    uint32_t ocap = m->cap;
    m->s = (slot *)malloc(sizeof(slot) * ncap);
    for (uint32_t i = 0; i < ncap; i++) m->s[i].key = -1;
    m->cap = ncap;
    m->used = m->live = 0;
    for (uint32_t i = 0; i < ocap; i++) {
        if (old[i].key >= 0) {
            uint32_t j = hkey(old[i].key) & (ncap - 1);
            while (m->s[j].key != -1) j = (j + 1) & (ncap - 1);
            m->s[j] = old[i];
            m->used++;
            m->live++;
        }
    }
    free(old);
}

/* returns the slot for k, inserting an empty one (key set, fields zeroed) when absent */
static slot *omap_get(omap *m, int32_t k, int *created) {
    slot *e = omap_find(m, k);
    if (e) { if (created) *created = 0; return e; }
    if ((m->used + 1) * 2 > m->cap) omap_rehash(m, m->cap ? (m->live * 2 + 2 > m->cap / 2 ? m->cap * 2 : m->cap) : 16);
    uint32_t i = hkey(k) & (m->cap - 1);
    while (m->s[i].key >= 0) i = (i + 1) & (m->cap - 1);
    if (m->s[i].key == -1) m->used++;
    m->live++;
    e = &m->s[i];
    memset(e, 0, sizeof(*e));
    e->key = k;
    if (created) *created = 1;
    return e;
}

static void omap_erase(omap *m, int32_t k) {
    slot *e = omap_find(m, k);
    if (!e) return;
    e->key = -2;
    m->live--;
}

static void omap_clear(omap *m) {
    for (uint32_t i = 0; i < m->cap; i++) m->s[i].key = -1;
    m->used = m->live = 0;
}

/* ------------------------------------------------------------------------------------------ */
/* simulator state                                                                             */
/* ------------------------------------------------------------------------------------------ */
typedef struct obs {
    omap dis;             /* disseminator.changes (disseminator.go:44-45) */
    int32_t nmem;         /* len(memberlist.members.list) (memberlist.go:174-179), kept incrementally */
    /* applied-change log of a watched observer (MemberlistChangesAppliedEvent, events.go:56-61):
     * the last applied change of every member since the last drain */
    int32_t watched;
    uint32_t wcs_prev;    /* checksum at the last drain (the event's OldChecksum) */
    uint8_t *wdirty;      /* [n] */
    or_change *wlast;     /* [n] */
    /* watched == 2: every applied change, one event per applying Update, in Update order */
    or_change *wev;
    int64_t *wev_seq;
    size_t wev_n, wev_cap;
    int64_t wseq;         /* applying Updates so far */
    uint32_t wcs_ev_prev;
    omap tim;             /* stateTransitions.timers (state_transitions.go:49) */
    int64_t clock_off;
    uint32_t cs;          /* memberlist.members.checksum (memberlist.go:46) */
    int32_t cs_dirty;
    int32_t maxp;         /* disseminator.maxP (disseminator.go:49) */
    int32_t pfactor;
    int32_t pingable;     /* incrementally maintained NumPingableMembers (memberlist.go:188-198) */
    int64_t it_idx;       /* memberlistIter.currentIndex (memberlist_iter.go:31) */
    uint32_t it_epoch;    /* number of reshuffles */
    int32_t live, part;
    int32_t njobs;
    int32_t *jobs;
} obs;

struct or_sim {
    or_config cfg;
    uint32_t n;
    uint32_t round;
    uint8_t *st;          /* [n][n] */
    int64_t *inc;         /* [n][n] */
    obs *o;
    char *addr;           /* [n][addr_cap] */
    uint32_t *addr_len;
    uint32_t addr_cap;
    uint64_t counters[OR_NCOUNTERS];
    int32_t *last_target;
};

/* Per-thread scratch: the OpenMP build (libswim_oracle_omp.so, CPU baseline only) runs the per-observer
 * loops of a phase in parallel. Observers of one phase touch only their own row, maps and timers, so the
 * results equal the single-threaded oracle's; counters are atomic. */
static __thread char *tl_csbuf;
static __thread size_t tl_csbuf_cap;
static __thread int64_t tl_now_override = -1;  /* >= 0 inside a timer callback: Mock.Add sets now = deadline */
#define CTR_ADD(s, c, v) __atomic_fetch_add(&(s)->counters[(c)], (uint64_t)(v), __ATOMIC_RELAXED)

#define ST(s, o, m) ((s)->st[(size_t)(o) * (s)->n + (m)])
#define INC(s, o, m) ((s)->inc[(size_t)(o) * (s)->n + (m)])

static int64_t now_ms(const or_sim *s, uint32_t o) {
    if (tl_now_override >= 0) return tl_now_override;
    return s->cfg.t0_ms + (int64_t)s->round * s->cfg.period_ms + s->o[o].clock_off;
}

static int is_pingable_status(int32_t st) { return st == OR_ALIVE || st == OR_SUSPECT; }

/* maxP = pFactor * ceil(log(n+1)/log(10)) (disseminator.go:81), exact integer form */
static int32_t digits10(int64_t n) {
    int32_t d = 0;
    while (n > 0) { d++; n /= 10; }
    return d;
}

or_sim *or_create(const or_config *cfg) {
    or_sim *s = (or_sim *)calloc(1, sizeof(or_sim));
    s->cfg = *cfg;
    s->n = cfg->n;
    size_t nn = (size_t)s->n * s->n;
    s->st = (uint8_t *)malloc(nn);
    s->inc = (int64_t *)malloc(nn * sizeof(int64_t));
    memset(s->st, OR_UNKNOWN, nn);
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < nn; i++) s->inc[i] = cfg->t0_ms;  /* never-known entries read e = 0 */
    s->o = (obs *)calloc(s->n, sizeof(obs));
    for (uint32_t i = 0; i < s->n; i++) {
        omap_init(&s->o[i].dis);
        omap_init(&s->o[i].tim);
        s->o[i].live = 1;
        s->o[i].it_idx = -1;
        s->o[i].pfactor = (int32_t)cfg->p_factor;
        s->o[i].maxp = (int32_t)cfg->p_factor;
        s->o[i].jobs = (int32_t *)calloc(cfg->max_rfs_jobs + 1, sizeof(int32_t));
        s->o[i].cs_dirty = 1;
    }
    if (cfg->addresses) {
        s->addr_cap = cfg->addr_stride;
        s->addr = (char *)calloc((size_t)s->n, s->addr_cap + 1);
        s->addr_len = (uint32_t *)calloc(s->n, sizeof(uint32_t));
        for (uint32_t i = 0; i < s->n; i++) {
            const char *a = cfg->addresses + (size_t)i * cfg->addr_stride;
            size_t l = strnlen(a, cfg->addr_stride);
            memcpy(s->addr + (size_t)i * (s->addr_cap + 1), a, l);
            s->addr_len[i] = (uint32_t)l;
        }
    } else {
        s->addr_cap = 19;
        s->addr = (char *)calloc((size_t)s->n, s->addr_cap + 1);
        s->addr_len = (uint32_t *)calloc(s->n, sizeof(uint32_t));
        for (uint32_t i = 0; i < s->n; i++) {
            char *a = s->addr + (size_t)i * (s->addr_cap + 1);
            snprintf(a, s->addr_cap + 1, "10.%03u.%03u.%03u:7000", (i >> 16) & 255, (i >> 8) & 255, i & 255);
            s->addr_len[i] = (uint32_t)strlen(a);
        }
    }
    s->last_target = (int32_t *)malloc(sizeof(int32_t) * s->n);
    for (uint32_t i = 0; i < s->n; i++) s->last_target[i] = -1;
    return s;
}

void or_destroy(or_sim *s) {
    if (!s) return;
    for (uint32_t i = 0; i < s->n; i++) {
        omap_free(&s->o[i].dis);
        omap_free(&s->o[i].tim);
        free(s->o[i].jobs);
        free(s->o[i].wdirty);
        free(s->o[i].wlast);
        free(s->o[i].wev);
        free(s->o[i].wev_seq);
    }
    free(s->o); free(s->st); free(s->inc); free(s->addr); free(s->addr_len);
    free(s->last_target);
    free(s);
}

void or_recompute_pingable(or_sim *s, uint32_t o) {
    int32_t c = 0;
    for (uint32_t m = 0; m < s->n; m++)
        if (m != o && is_pingable_status(ST(s, o, m))) c++;
    s->o[o].pingable = c;
}

void or_init_converged(or_sim *s) {
#pragma omp parallel for schedule(static)
    for (uint32_t o = 0; o < s->n; o++) {
        for (uint32_t m = 0; m < s->n; m++) {
            ST(s, o, m) = OR_ALIVE;
            INC(s, o, m) = s->cfg.t0_ms;
        }
        s->o[o].nmem = (int32_t)s->n;
        or_recompute_pingable(s, o);
        s->o[o].maxp = s->o[o].pfactor * digits10(s->o[o].pingable);
        s->o[o].cs_dirty = 1;
    }
}

void or_init_self_only(or_sim *s) {
    for (uint32_t o = 0; o < s->n; o++) {
        ST(s, o, o) = OR_ALIVE;
        INC(s, o, o) = s->cfg.t0_ms;
        s->o[o].nmem = 1;
        or_recompute_pingable(s, o);
        s->o[o].maxp = s->o[o].pfactor;  /* newDisseminator: maxP = defaultPFactor (disseminator.go:62) */
        s->o[o].cs_dirty = 1;
    }
}

void or_set_member(or_sim *s, uint32_t o, uint32_t m, int32_t status, int64_t inc) {
    ST(s, o, m) = (uint8_t)status;
    INC(s, o, m) = inc;
    or_recompute_pingable(s, o);
    s->o[o].nmem = or_num_members(s, o);
    s->o[o].cs_dirty = 1;
}

void or_set_clock_offset(or_sim *s, uint32_t o, int64_t off) { s->o[o].clock_off = off; }
void or_set_live(or_sim *s, uint32_t o, int32_t live) { s->o[o].live = live; }
void or_set_partition(or_sim *s, uint32_t o, int32_t label) { s->o[o].part = label; }
void or_set_round(or_sim *s, uint32_t r) { s->round = r; }
void or_set_maxp(or_sim *s, uint32_t o, int32_t maxp, int32_t pf) { s->o[o].maxp = maxp; s->o[o].pfactor = pf; }
void or_clear_changes(or_sim *s, uint32_t o) { omap_clear(&s->o[o].dis); } /* disseminator.go:217-221 */
void or_clear_change(or_sim *s, uint32_t o, uint32_t m) { omap_erase(&s->o[o].dis, (int32_t)m); } /* 229-233 */

static int reach(const or_sim *s, uint32_t a, uint32_t b) {
    return s->o[a].live && s->o[b].live && s->o[a].part == s->o[b].part;
}

/* ------------------------------------------------------------------------------------------ */
/* FarmHash-32 "mk" — go-farm Fingerprint32 (= Hash32, farmhashmk), glide.lock:18-19           */
/* ------------------------------------------------------------------------------------------ */
static const uint32_t FH_C1 = 0xcc9e2d51u, FH_C2 = 0x1b873593u;
static uint32_t fetch32(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
static uint32_t rot32(uint32_t v, int sh) { return sh == 0 ? v : ((v >> sh) | (v << (32 - sh))); }
static uint32_t fmix(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}
static uint32_t mur(uint32_t a, uint32_t h) {
    a *= FH_C1; a = rot32(a, 17); a *= FH_C2;
    h ^= a; h = rot32(h, 19);
    return h * 5 + 0xe6546b64u;
}
static uint32_t h32_13to24(const uint8_t *s, size_t len) {
    uint32_t a = fetch32(s - 4 + (len >> 1)), b = fetch32(s + 4), c = fetch32(s + len - 8);
    uint32_t d = fetch32(s + (len >> 1)), e = fetch32(s), f = fetch32(s + len - 4);
    uint32_t h = d * FH_C1 + (uint32_t)len;
    a = rot32(a, 12) + f;
    h = mur(c, h) + a;
    a = rot32(a, 3) + c;
    h = mur(e, h) + a;
    a = rot32(a + f, 12) + d;
    h = mur(b, h) + a;
    return fmix(h);
}
static uint32_t h32_0to4(const uint8_t *s, size_t len) {
    uint32_t b = 0, c = 9;
    for (size_t i = 0; i < len; i++) {
        int8_t v = (int8_t)s[i];
        b = b * FH_C1 + (uint32_t)(int32_t)v;
        c ^= b;
    }
    return fmix(mur(b, mur((uint32_t)len, c)));
}
static uint32_t h32_5to12(const uint8_t *s, size_t len) {
    uint32_t a = (uint32_t)len, b = (uint32_t)len * 5, c = 9, d = b;
    a += fetch32(s);
    b += fetch32(s + len - 4);
    c += fetch32(s + ((len >> 1) & 4));
    return fmix(mur(c, mur(b, mur(a, d))));
}
uint32_t or_fingerprint32(const uint8_t *s, size_t len) {
    if (len <= 24) return len <= 12 ? (len <= 4 ? h32_0to4(s, len) : h32_5to12(s, len)) : h32_13to24(s, len);
    uint32_t h = (uint32_t)len, g = FH_C1 * (uint32_t)len, f = g;
    uint32_t a0 = rot32(fetch32(s + len - 4) * FH_C1, 17) * FH_C2;
    uint32_t a1 = rot32(fetch32(s + len - 8) * FH_C1, 17) * FH_C2;
    uint32_t a2 = rot32(fetch32(s + len - 16) * FH_C1, 17) * FH_C2;
    uint32_t a3 = rot32(fetch32(s + len - 12) * FH_C1, 17) * FH_C2;
    uint32_t a4 = rot32(fetch32(s + len - 20) * FH_C1, 17) * FH_C2;
    h ^= a0; h = rot32(h, 19); h = h * 5 + 0xe6546b64u;
    h ^= a2; h = rot32(h, 19); h = h * 5 + 0xe6546b64u;
    g ^= a1; g = rot32(g, 19); g = g * 5 + 0xe6546b64u;
    g ^= a3; g = rot32(g, 19); g = g * 5 + 0xe6546b64u;
    f += a4; f = rot32(f, 19) + 113;
    size_t iters = (len - 1) / 20;
    do {
        uint32_t a = fetch32(s), b = fetch32(s + 4), c = fetch32(s + 8), d = fetch32(s + 12), e = fetch32(s + 16);
        h += a; g += b; f += c;
        h = mur(d, h) + e;
        g = mur(c, g) + a;
        f = mur(b + e * FH_C1, f) + d;
        f += g; g += f;
        s += 20;
    } while (--iters != 0);
    g = rot32(g, 11) * FH_C1; g = rot32(g, 17) * FH_C1;
    f = rot32(f, 11) * FH_C1; f = rot32(f, 17) * FH_C1;
    h = rot32(h + g, 19); h = h * 5 + 0xe6546b64u; h = rot32(h, 17) * FH_C1;
    h = rot32(h + f, 19); h = h * 5 + 0xe6546b64u; h = rot32(h, 17) * FH_C1;
    return h;
}

/* ------------------------------------------------------------------------------------------ */
/* checksum (memberlist.go:83-128)                                                             */
/* ------------------------------------------------------------------------------------------ */
static const char *STATUS_STR[5] = {"alive", "suspect", "faulty", "leave", "tombstone"};

static int cmp_cstr(const void *a, const void *b) { return strcmp(*(const char *const *)a, *(const char *const *)b); }

/* %lld of v (Go's %v of an int64, memberlist.go:120) without snprintf's per-call overhead */
static size_t fmt_i64(char *out, int64_t v) {
    char tmp[24];
    size_t k = 0, len = 0;
    uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    do { tmp[k++] = (char)('0' + u % 10); u /= 10; } while (u);
    if (v < 0) out[len++] = '-';
    while (k) out[len++] = tmp[--k];
    return len;
}

static void csbuf_reserve(size_t need) {
    if (tl_csbuf_cap >= need) return;
    tl_csbuf_cap = need * 2;
    tl_csbuf = (char *)realloc(tl_csbuf, tl_csbuf_cap);
}

/* GenChecksumString: fmt.Sprintf("%s%s%v", addr, status, inc) per non-tombstone member, sorted,
 * each followed by ";" (memberlist.go:106-128). Returns length; writes into tl_csbuf. */
static size_t gen_checksum_string(or_sim *s, uint32_t o) {
    size_t per = s->addr_cap + 32;
    csbuf_reserve((size_t)s->n * per + 1);
    size_t len = 0;
    if (s->cfg.faithful_checksum) {
        char *pool = (char *)malloc((size_t)s->n * per);
        char **v = (char **)malloc(sizeof(char *) * s->n);
        uint32_t k = 0;
        for (uint32_t m = 0; m < s->n; m++) {
            int32_t st = ST(s, o, m);
            if (st == OR_UNKNOWN || st == OR_TOMBSTONE) continue;
            char *p = pool + (size_t)k * per;
            snprintf(p, per, "%s%s%lld", s->addr + (size_t)m * (s->addr_cap + 1), STATUS_STR[st], (long long)INC(s, o, m));
            v[k++] = p;
        }
        qsort(v, k, sizeof(char *), cmp_cstr);
        for (uint32_t i = 0; i < k; i++) {
            size_t l = strlen(v[i]);
            memcpy(tl_csbuf + len, v[i], l);
            len += l;
            tl_csbuf[len++] = ';';
        }
        free(pool);
        free(v);
    } else {
        /* fixed-width ascending addresses: sorted order == member index order */
        for (uint32_t m = 0; m < s->n; m++) {
            int32_t st = ST(s, o, m);
            if (st == OR_UNKNOWN || st == OR_TOMBSTONE) continue;
            memcpy(tl_csbuf + len, s->addr + (size_t)m * (s->addr_cap + 1), s->addr_len[m]);
            len += s->addr_len[m];
            size_t sl = strlen(STATUS_STR[st]);
            memcpy(tl_csbuf + len, STATUS_STR[st], sl);
            len += sl;
            len += fmt_i64(tl_csbuf + len, INC(s, o, m));
            tl_csbuf[len++] = ';';
        }
    }
    return len;
}

size_t or_checksum_string(or_sim *s, uint32_t o, char *out, size_t cap) {
    size_t len = gen_checksum_string(s, o);
    if (out && cap) {
        size_t c = len < cap ? len : cap;
        memcpy(out, tl_csbuf, c);
    }
    return len;
}

uint32_t or_checksum(or_sim *s, uint32_t o) {
    obs *ob = &s->o[o];
    if (ob->cs_dirty) {
        size_t len = gen_checksum_string(s, o);
        ob->cs = or_fingerprint32((const uint8_t *)tl_csbuf, len);
        ob->cs_dirty = 0;
    }
    return ob->cs;
}

/* ------------------------------------------------------------------------------------------ */
/* Philox4x32-10 and the Feistel permutation (docs/ROUND_SEMANTICS.md §6)                      */
/* ------------------------------------------------------------------------------------------ */
void or_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; r++) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static uint32_t philox_u32(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t purpose, uint32_t i) {
    uint32_t ctr[4] = {c0, c1, purpose, i >> 2};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t out[4];
    or_philox4x32_10(ctr, key, out);
    return out[i & 3];
}

static uint32_t mulhi_n(uint32_t x, uint32_t n) { return (uint32_t)(((uint64_t)x * n) >> 32); }

static uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

typedef struct feistel { uint32_t k[4]; uint32_t half, mask; } feistel;

static feistel feistel_make(uint64_t seed, uint32_t o, uint32_t epoch, uint32_t n) {
    feistel f;
    uint32_t ctr[4] = {epoch, o, 1u, 0u};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    or_philox4x32_10(ctr, key, f.k);
    uint32_t b = 2;
    while (b < 32 && ((uint64_t)1 << b) < n) b += 2;
    f.half = b / 2;
    f.mask = (1u << f.half) - 1u;
    return f;
}
static uint32_t feistel_enc(const feistel *f, uint32_t x) {
    uint32_t L = x >> f->half, R = x & f->mask;
    for (int i = 0; i < 4; i++) {
        uint32_t nl = R, nr = L ^ (fmix32(R ^ f->k[i]) & f->mask);
        L = nl; R = nr;
    }
    return (L << f->half) | R;
}
static uint32_t feistel_dec(const feistel *f, uint32_t x) {
    uint32_t L = x >> f->half, R = x & f->mask;
    for (int i = 3; i >= 0; i--) {
        uint32_t pr = L, pl = R ^ (fmix32(L ^ f->k[i]) & f->mask);
        L = pl; R = pr;
    }
    return (L << f->half) | R;
}
uint32_t or_perm(uint64_t seed, uint32_t o, uint32_t epoch, uint32_t n, uint32_t idx) {
    feistel f = feistel_make(seed, o, epoch, n);
    uint32_t x = idx;
    do { x = feistel_enc(&f, x); } while (x >= n);
    return x;
}
uint32_t or_perm_inv(uint64_t seed, uint32_t o, uint32_t epoch, uint32_t n, uint32_t m) {
    feistel f = feistel_make(seed, o, epoch, n);
    uint32_t x = m;
    do { x = feistel_dec(&f, x); } while (x >= n);
    return x;
}

/* ------------------------------------------------------------------------------------------ */
/* member precedence (member.go:79-128)                                                        */
/* ------------------------------------------------------------------------------------------ */
int32_t or_non_local_override(int64_t cur_inc, int32_t cur_st, int64_t ch_inc, int32_t ch_st) {
    if (ch_inc > cur_inc) return 1;      /* member.go:81-83 */
    if (ch_inc < cur_inc) return 0;      /* member.go:86-88 */
    return ch_st > cur_st;               /* member.go:92, statePrecedence */
}
int32_t or_local_override(int32_t is_local, int64_t cur_inc, int64_t ch_inc, int32_t ch_st) {
    if (!is_local) return 0;             /* member.go:99-101 */
    if (ch_inc < cur_inc) return 0;      /* member.go:105-107 */
    return ch_st == OR_FAULTY || ch_st == OR_SUSPECT || ch_st == OR_TOMBSTONE; /* member.go:109 */
}

/* ------------------------------------------------------------------------------------------ */
/* timers (state_transitions.go:90-176)                                                        */
/* ------------------------------------------------------------------------------------------ */
static int64_t timeout_for(const or_sim *s, int32_t state) {
    return state == OR_SUSPECT ? s->cfg.suspect_ms : state == OR_FAULTY ? s->cfg.faulty_ms : s->cfg.tombstone_ms;
}

void or_schedule(or_sim *s, uint32_t o, uint32_t m, int32_t state, int64_t subj) {
    if (o == m) return;                                  /* state_transitions.go:125-128 */
    obs *ob = &s->o[o];
    slot *e = omap_find(&ob->tim, (int32_t)m);
    if (e && e->a == state) return;                      /* same state: no-op (130-136) */
    e = omap_get(&ob->tim, (int32_t)m, NULL);            /* replace / create (142-152) */
    e->a = state;
    e->b = 0;
    e->x = now_ms(s, o) + timeout_for(s, state);
    e->y = subj;
}

void or_cancel(or_sim *s, uint32_t o, uint32_t m) { omap_erase(&s->o[o].tim, (int32_t)m); } /* 163-176 */

/* ------------------------------------------------------------------------------------------ */
/* memberlist.Update + node.handleChanges (memberlist.go:310-390, 418-449; node.go:424-447)    */
/* ------------------------------------------------------------------------------------------ */
static void apply_row(or_sim *s, uint32_t j, const or_change *c) {
    int32_t old = ST(s, j, c->member);
    if ((uint32_t)c->member != j) {
        s->o[j].pingable += (is_pingable_status(c->status) ? 1 : 0) - (is_pingable_status(old) ? 1 : 0);
    }
    if (old == OR_UNKNOWN) s->o[j].nmem++;
    ST(s, j, c->member) = (uint8_t)c->status;
    INC(s, j, c->member) = c->inc;
}

static void handle_changes(or_sim *s, uint32_t j, const or_change *applied, int32_t na) {
    obs *ob = &s->o[j];
    ob->maxp = ob->pfactor * digits10(ob->pingable);   /* AdjustMaxPropagations (disseminator.go:75-97) */
    for (int32_t i = 0; i < na; i++) {
        const or_change *c = &applied[i];
        slot *e = omap_get(&ob->dis, c->member, NULL);   /* RecordChange (disseminator.go:223-227) */
        e->a = 0;
        e->b = c->source;
        e->x = c->source_inc;
        switch (c->status) {
        case OR_ALIVE: or_cancel(s, j, (uint32_t)c->member); break;
        case OR_SUSPECT: or_schedule(s, j, (uint32_t)c->member, OR_SUSPECT, c->inc); break;
        case OR_FAULTY: or_schedule(s, j, (uint32_t)c->member, OR_FAULTY, c->inc); break;
        case OR_LEAVE: or_cancel(s, j, (uint32_t)c->member); break;
        case OR_TOMBSTONE: or_schedule(s, j, (uint32_t)c->member, OR_TOMBSTONE, c->inc); break;
        }
    }
}

int32_t or_update(or_sim *s, uint32_t j, const or_change *ch, int32_t n, or_change *applied_out, int32_t cap) {
    if (n <= 0) return 0;                                 /* memberlist.go:311-313 */
    or_change *applied = (or_change *)malloc(sizeof(or_change) * (size_t)n);
    int32_t na = 0;
    for (int32_t i = 0; i < n; i++) {
        or_change c = ch[i];                              /* validateIncoming is the identity here */
        int32_t cur = ST(s, j, c.member);
        if (cur == OR_UNKNOWN) {                          /* memberlist.go:328-334, Apply 418-449 */
            if (c.status == OR_TOMBSTONE) continue;       /* memberlist.go:424-426 */
            apply_row(s, j, &c);
            applied[na++] = c;
            continue;
        }
        if (or_local_override((uint32_t)c.member == j, INC(s, j, c.member), c.inc, c.status)) {
            int64_t t = now_ms(s, j);                     /* memberlist.go:337-354 */
            or_change ov = {c.member, OR_ALIVE, (int32_t)j, 0, t, t};
            apply_row(s, j, &ov);
            applied[na++] = ov;
            CTR_ADD(s, OR_C_REFUTES, 1);
            continue;
        }
        if (or_non_local_override(INC(s, j, c.member), cur, c.inc, c.status)) { /* 357-361 */
            apply_row(s, j, &c);
            applied[na++] = c;
        }
    }
    if (na > 0) {
        obs *ob = &s->o[j];
        ob->cs_dirty = 1;                                 /* ComputeChecksum (memberlist.go:367-368) */
        if (s->cfg.reference_cost) {
            /* the reference's cost model: checksum string rebuilt (and sorted when faithful_checksum) and
             * hashed at every Update that applied something; NumPingableMembers rescans the list in
             * AdjustMaxPropagations (disseminator.go:78, memberlist.go:188-198). Same results. */
            or_checksum(s, j);
            or_recompute_pingable(s, j);
        }
        if (ob->watched)                                  /* MemberlistChangesAppliedEvent (memberlist.go:378-383) */
            for (int32_t i = 0; i < na; i++) {
                ob->wdirty[applied[i].member] = 1;
                ob->wlast[applied[i].member] = applied[i];
            }
        if (ob->watched == 2) {                           /* one event per applying Update */
            if (ob->wev_n + (size_t)na > ob->wev_cap) {
                ob->wev_cap = (ob->wev_n + (size_t)na) * 2;
                ob->wev = (or_change *)realloc(ob->wev, sizeof(or_change) * ob->wev_cap);
                ob->wev_seq = (int64_t *)realloc(ob->wev_seq, sizeof(int64_t) * ob->wev_cap);
            }
            for (int32_t i = 0; i < na; i++) {
                ob->wev[ob->wev_n] = applied[i];
                ob->wev_seq[ob->wev_n++] = ob->wseq;
            }
            ob->wseq++;
        }
        handle_changes(s, j, applied, na);                /* memberlist.go:384 */
        CTR_ADD(s, OR_C_APPLIED, (uint64_t)na);
    }
    if (applied_out) memcpy(applied_out, applied, sizeof(or_change) * (size_t)(na < cap ? na : cap));
    free(applied);
    return na;
}

int or_make_change(or_sim *s, uint32_t o, uint32_t m, int64_t inc, int32_t status) {
    or_change c = {(int32_t)m, status, (int32_t)o, 0, inc, INC(s, o, o)};  /* memberlist.go:292-299 */
    return or_update(s, o, &c, 1, NULL, 0);
}

/* Evict → RemoveMember (memberlist.go:141-162,271-279): no handleChanges, checksum recomputed */
static void evict(or_sim *s, uint32_t o, uint32_t m) {
    if (o == m) return;
    if (ST(s, o, m) == OR_UNKNOWN) return;
    if (is_pingable_status(ST(s, o, m))) s->o[o].pingable--;
    ST(s, o, m) = OR_UNKNOWN;   /* incarnation kept: the buffered change still reads (tombstone, inc) */
    s->o[o].nmem--;
    s->o[o].cs_dirty = 1;
    if (s->cfg.reference_cost) or_checksum(s, o);         /* RemoveMember → ComputeChecksum (memberlist.go:156-159) */
}

/* ------------------------------------------------------------------------------------------ */
/* disseminator (disseminator.go:107-215)                                                      */
/* ------------------------------------------------------------------------------------------ */
static int cmp_change_member(const void *a, const void *b) {
    const or_change *x = (const or_change *)a, *y = (const or_change *)b;
    return (x->member > y->member) - (x->member < y->member);
}

/* issueChanges: every buffered change, validateOutgoing; listed in member order */
static or_change *issue_changes(or_sim *s, uint32_t j, int32_t *n_out) {
    omap *d = &s->o[j].dis;
    or_change *v = (or_change *)malloc(sizeof(or_change) * (d->live + 1));
    int32_t k = 0;
    for (uint32_t i = 0; i < d->cap; i++) {
        const slot *e = &d->s[i];
        if (e->key < 0) continue;
        int32_t st = ST(s, j, e->key);
        or_change c = {e->key, st == OR_UNKNOWN ? OR_TOMBSTONE : st, e->b, 0, INC(s, j, e->key), e->x};
        v[k++] = c;
    }
    qsort(v, (size_t)k, sizeof(or_change), cmp_change_member);
    *n_out = k;
    return v;
}

/* memberlist.AddJoinList (memberlist.go:398-406): Update, then ClearChange of every applied change whose
 * address is not the node's own. Returns the number of applied changes. */
int32_t or_add_join_list(or_sim *s, uint32_t j, const or_change *ch, int32_t n) {
    if (n <= 0) return 0;
    or_change *applied = (or_change *)malloc(sizeof(or_change) * (size_t)n);
    const int32_t na = or_update(s, j, ch, n, applied, n);
    for (int32_t i = 0; i < na; i++)
        if ((uint32_t)applied[i].member != j) or_clear_change(s, j, (uint32_t)applied[i].member);
    free(applied);
    return na;
}

int32_t or_issue_as_sender(or_sim *s, uint32_t j, or_change *out, int32_t cap) {
    int32_t k;
    or_change *v = issue_changes(s, j, &k);
    if (out) memcpy(out, v, sizeof(or_change) * (size_t)(k < cap ? k : cap));
    free(v);
    return k;
}

void or_bump(or_sim *s, uint32_t j, const or_change *ch, int32_t n) {   /* disseminator.go:135-149 */
    obs *ob = &s->o[j];
    for (int32_t i = 0; i < n; i++) {
        slot *e = omap_find(&ob->dis, ch[i].member);
        if (!e) continue;
        e->a++;
        if (e->a >= ob->maxp) omap_erase(&ob->dis, ch[i].member);
    }
}

static or_change *membership_as_changes(or_sim *s, uint32_t j, int32_t *n_out) {
    or_change *v = (or_change *)malloc(sizeof(or_change) * (s->n + 1));
    int32_t k = 0;
    int64_t self_inc = INC(s, j, j);
    for (uint32_t m = 0; m < s->n; m++) {
        int32_t st = ST(s, j, m);
        if (st == OR_UNKNOWN) continue;
        or_change c = {(int32_t)m, st, (int32_t)j, 0, INC(s, j, m), self_inc};
        v[k++] = c;
    }
    *n_out = k;
    return v;
}

int32_t or_membership_as_changes(or_sim *s, uint32_t j, or_change *out, int32_t cap) {
    int32_t k;
    or_change *v = membership_as_changes(s, j, &k);
    if (out) memcpy(out, v, sizeof(or_change) * (size_t)(k < cap ? k : cap));
    free(v);
    return k;
}

/* IssueAsReceiver (disseminator.go:156-181) + filterChangesFromSender (185-199) */
static or_change *issue_as_receiver(or_sim *s, uint32_t j, int32_t sender, int64_t sinc, uint32_t scs,
                                    int32_t *n_out, int32_t *fs) {
    int32_t k;
    or_change *v = issue_changes(s, j, &k);
    int32_t w = 0;
    for (int32_t i = 0; i < k; i++) {
        if (v[i].source_inc == sinc && v[i].source == sender && sender != OR_SOURCE_NONE) continue;
        v[w++] = v[i];
    }
    or_bump(s, j, v, w);
    *fs = 0;
    if (w > 0 || or_checksum(s, j) == scs) {
        *n_out = w;
        return v;
    }
    free(v);
    *fs = 1;
    return membership_as_changes(s, j, n_out);
}

int32_t or_issue_as_receiver(or_sim *s, uint32_t j, int32_t sender, int64_t sender_inc, uint32_t sender_cs,
                             or_change *out, int32_t cap, int32_t *full_sync) {
    int32_t k;
    or_change *v = issue_as_receiver(s, j, sender, sender_inc, sender_cs, &k, full_sync);
    if (out) memcpy(out, v, sizeof(or_change) * (size_t)(k < cap ? k : cap));
    free(v);
    return k;
}

/* ------------------------------------------------------------------------------------------ */
/* target selection: memberlistIter.Next (memberlist_iter.go:50-72)                            */
/* ------------------------------------------------------------------------------------------ */
int32_t or_next(or_sim *s, uint32_t o) {
    obs *ob = &s->o[o];
    uint32_t n = s->n;
    int32_t max_to_visit = ob->nmem;                      /* NumMembers: len(list) (memberlist_iter.go:51) */
    /* visited set: a short list while the walk is short (the common case), a bitmap beyond */
    uint32_t few[64];
    uint8_t *visited = NULL;
    int32_t nvisited = 0, result = -1;
    while (nvisited < max_to_visit) {
        ob->it_idx++;
        if (ob->it_idx >= (int64_t)n) {                   /* wrap → reshuffle (57-61) */
            ob->it_idx = 0;
            ob->it_epoch++;
        }
        uint32_t m = or_perm(s->cfg.seed, o, ob->it_epoch, n, (uint32_t)ob->it_idx);
        if (ST(s, o, m) == OR_UNKNOWN) continue;          /* not a list entry */
        int seen = 0;
        if (visited) {
            seen = visited[m];
        } else {
            for (int32_t i = 0; i < nvisited && !seen; i++) seen = few[i] == m;
        }
        if (!seen) {
            if (!visited && nvisited == 64) {
                visited = (uint8_t *)calloc(n, 1);
                for (int32_t i = 0; i < 64; i++) visited[few[i]] = 1;
            }
            if (visited) visited[m] = 1;
            else few[nvisited] = m;
            nvisited++;
        }
        if (m != o && is_pingable_status(ST(s, o, m))) { result = (int32_t)m; break; } /* Pingable 181-185 */
    }
    free(visited);
    return result;
}

/* RandomPingableMembers (memberlist.go:201-219), Philox draw rule of ROUND_SEMANTICS §3 */
int32_t or_random_pingable(or_sim *s, uint32_t o, int32_t k, int32_t exclude, int32_t *out) {
    uint32_t n = s->n;
    int32_t eligible = 0;
    for (uint32_t m = 0; m < n; m++)
        if (m != o && (int32_t)m != exclude && is_pingable_status(ST(s, o, m))) eligible++;
    int32_t need = k < eligible ? k : eligible, got = 0;
    for (uint32_t i = 0; i < 64 && got < need; i++) {
        uint32_t c = mulhi_n(philox_u32(s->cfg.seed, s->round, o, 2u, i), n);
        if (c == o || (int32_t)c == exclude || !is_pingable_status(ST(s, o, c))) continue;
        int dup = 0;
        for (int32_t q = 0; q < got; q++) dup |= out[q] == (int32_t)c;
        if (!dup) out[got++] = (int32_t)c;
    }
    if (got < need) {
        uint32_t start = mulhi_n(philox_u32(s->cfg.seed, s->round, o, 2u, 64u), n);
        for (uint32_t q = 0; q < n && got < need; q++) {
            uint32_t c = (start + q) % n;
            if (c == o || (int32_t)c == exclude || !is_pingable_status(ST(s, o, c))) continue;
            int dup = 0;
            for (int32_t z = 0; z < got; z++) dup |= out[z] == (int32_t)c;
            if (!dup) out[got++] = (int32_t)c;
        }
    }
    return got;
}

/* ------------------------------------------------------------------------------------------ */
/* timer firing on the round clock (benbjohnson/clock Mock.Add semantics)                      */
/* ------------------------------------------------------------------------------------------ */
typedef struct due { int64_t deadline; int32_t member, state; int64_t subj; } due;
static int cmp_due(const void *a, const void *b) {
    const due *x = (const due *)a, *y = (const due *)b;
    if (x->deadline != y->deadline) return (x->deadline > y->deadline) - (x->deadline < y->deadline);
    return (x->member > y->member) - (x->member < y->member);
}

void or_fire_timers(or_sim *s, uint32_t o) {
    obs *ob = &s->o[o];
    int64_t t = now_ms(s, o);
    due *v = (due *)malloc(sizeof(due) * (ob->tim.live + 1));
    int32_t k = 0;
    for (uint32_t i = 0; i < ob->tim.cap; i++) {
        const slot *e = &ob->tim.s[i];
        if (e->key < 0 || e->b || e->x > t) continue;
        due d = {e->x, e->key, e->a, e->y};
        v[k++] = d;
    }
    qsort(v, (size_t)k, sizeof(due), cmp_due);
    for (int32_t i = 0; i < k; i++) {
        slot *e = omap_find(&ob->tim, v[i].member);
        if (!e) continue;
        e->b = 1;                                         /* fired; the entry stays in s.timers */
        CTR_ADD(s, OR_C_TIMERS_FIRED, 1);
        tl_now_override = v[i].deadline;                  /* clock.Mock.runNextTimer: now = t.next */
        if (v[i].state == OR_SUSPECT) or_make_change(s, o, (uint32_t)v[i].member, v[i].subj, OR_FAULTY);  /* 90-97 */
        else if (v[i].state == OR_FAULTY) or_make_change(s, o, (uint32_t)v[i].member, v[i].subj, OR_TOMBSTONE); /* 100-107 */
        else evict(s, o, (uint32_t)v[i].member);          /* 110-117 */
        tl_now_override = -1;
    }
    free(v);
}

/* ------------------------------------------------------------------------------------------ */
/* heal (heal_via_discover_provider.go:120-177, heal_partition.go:33-145)                      */
/* ------------------------------------------------------------------------------------------ */
static void queue_rfs(or_sim *s, uint32_t j, int32_t src) {   /* tryStartReverseFullSync 257-278 */
    obs *ob = &s->o[j];
    if ((uint32_t)ob->njobs < s->cfg.max_rfs_jobs) ob->jobs[ob->njobs++] = src;
    else CTR_ADD(s, OR_C_RFS_OMITTED, 1);
}

/* sendPingWithChanges o → t, response discarded (heal_partition.go:97-124) */
static void ping_with_changes(or_sim *s, uint32_t o, uint32_t t, const or_change *ch, int32_t n) {
    uint32_t cs = or_checksum(s, o);
    int64_t inc = INC(s, o, o);
    or_update(s, t, ch, n, NULL, 0);                       /* handlePing: ping_handler.go:40 */
    int32_t k, fs;
    or_change *r = issue_as_receiver(s, t, (int32_t)o, inc, cs, &k, &fs);
    if (fs) { CTR_ADD(s, OR_C_FULL_SYNCS, 1); queue_rfs(s, t, (int32_t)o); }
    free(r);
}

static int32_t outgoing_status(int32_t st) { return st == OR_TOMBSTONE ? OR_FAULTY : st; } /* member.go:161-167 */
static int change_overrides(int64_t ai, int32_t as, int64_t bi, int32_t bs) { /* member.go:178-187 */
    if (ai > bi) return 1;
    if (ai < bi) return 0;
    return outgoing_status(as) > outgoing_status(bs);
}

static int32_t del_target(int32_t *t, int32_t n, int32_t v) {  /* del (heal_via_discover_provider.go:181-191) */
    for (int32_t i = 0; i < n; i++) {
        if (t[i] != v) continue;
        t[i] = t[n - 1];
        n--;
        i--;
    }
    return n;
}

int32_t or_heal(or_sim *s, uint32_t o, int32_t *ret_out, int32_t cap) {
    uint32_t n = s->n;
    int32_t *targets = (int32_t *)malloc(sizeof(int32_t) * n);
    int32_t nt = 0;
    for (uint32_t m = 0; m < n; m++) {                     /* 136-142 */
        int32_t st = ST(s, o, m);
        if (st == OR_UNKNOWN || st >= OR_FAULTY) targets[nt++] = (int32_t)m;
    }
    for (int32_t i = 0; i < nt; i++) {                     /* ShuffleStringsInPlace (util.go:189-194) */
        uint32_t jj = mulhi_n(philox_u32(s->cfg.seed, s->round, o, 3u, (uint32_t)i), (uint32_t)i + 1);
        int32_t tmp = targets[i]; targets[i] = targets[jj]; targets[jj] = tmp;
    }
    int32_t failures = 0, nret = 0;
    while (nt != 0 && failures < 10) {
        int32_t target = targets[0];
        nt = del_target(targets, nt, target);
        CTR_ADD(s, OR_C_HEAL_ATTEMPTS, 1);
        if (!reach(s, o, (uint32_t)target)) {              /* sendJoinRequest fails */
            failures++;
            CTR_ADD(s, OR_C_HEAL_FAILURES, 1);
            continue;
        }
        int32_t na, nb;
        or_change *MA = membership_as_changes(s, o, &na);
        or_change *MB = membership_as_changes(s, (uint32_t)target, &nb);
        /* index MA by member */
        int32_t *ma_idx = (int32_t *)malloc(sizeof(int32_t) * n);
        for (uint32_t m = 0; m < n; m++) ma_idx[m] = -1;
        for (int32_t i = 0; i < na; i++) ma_idx[MA[i].member] = i;
        or_change *A = (or_change *)malloc(sizeof(or_change) * (size_t)(nb + 1));
        or_change *B = (or_change *)malloc(sizeof(or_change) * (size_t)(nb + 1));
        int32_t nA = 0, nB = 0;
        for (int32_t i = 0; i < nb; i++) {                 /* nodesThatNeedToReincarnate (64-92) */
            const or_change *b = &MB[i];
            if (ma_idx[b->member] < 0) continue;
            const or_change *a = &MA[ma_idx[b->member]];
            int32_t as = outgoing_status(a->status), bs = outgoing_status(b->status);
            if (is_pingable_status(bs) && change_overrides(a->inc, as, b->inc, bs) && !is_pingable_status(as)) {
                or_change c = {a->member, OR_SUSPECT, OR_SOURCE_NONE, 0, a->inc, 0};
                B[nB++] = c;
            }
            if (is_pingable_status(as) && change_overrides(b->inc, bs, a->inc, as) && !is_pingable_status(bs)) {
                or_change c = {b->member, OR_SUSPECT, OR_SOURCE_NONE, 0, b->inc, 0};
                A[nA++] = c;
            }
        }
        if (nA || nB) {                                    /* reincarnateNodes (97-108) */
            or_update(s, o, A, nA, NULL, 0);
            if (nB) ping_with_changes(s, o, (uint32_t)target, B, nB);
        } else {                                           /* mergePartitions (112-124) */
            or_update(s, o, MB, nb, NULL, 0);
            int32_t na2;
            or_change *MA2 = membership_as_changes(s, o, &na2);
            ping_with_changes(s, o, (uint32_t)target, MA2, na2);
            free(MA2);
        }
        for (int32_t i = 0; i < nb; i++)                   /* pingableHosts (127-134), 163-165 */
            if (is_pingable_status(outgoing_status(MB[i].status))) nt = del_target(targets, nt, MB[i].member);
        if (ret_out && nret < cap) ret_out[nret] = target;
        nret++;
        free(MA); free(MB); free(ma_idx); free(A); free(B);
    }
    free(targets);
    return nret;
}

/* ------------------------------------------------------------------------------------------ */
/* the round (docs/ROUND_SEMANTICS.md §4)                                                       */
/* ------------------------------------------------------------------------------------------ */
typedef struct msg { or_change *v; int32_t n; } msg;

static void reincarnate(or_sim *s, uint32_t a) {           /* memberlist.go:234-236 */
    or_make_change(s, a, a, now_ms(s, a), OR_ALIVE);
}

static void apply_event(or_sim *s, const or_event *e) {
    uint32_t a = (uint32_t)e->a;
    switch (e->kind) {
    case OR_EV_KILL: s->o[a].live = 0; break;
    case OR_EV_REVIVE: s->o[a].live = 1; reincarnate(s, a); break;      /* handlers.go:140-143 */
    case OR_EV_REINCARNATE: if (s->o[a].live) reincarnate(s, a); break;
    case OR_EV_LEAVE: if (s->o[a].live) or_make_change(s, a, a, INC(s, a, a), OR_LEAVE); break; /* 145-148 */
    case OR_EV_PARTITION: s->o[a].part = e->b; break;
    case OR_EV_HEAL: if (s->o[a].live) or_heal(s, a, NULL, 0); break;
    case OR_EV_REAP:                                                     /* handlers.go:154-163 */
        if (s->o[a].live)
            for (uint32_t m = 0; m < s->n; m++)
                if (ST(s, a, m) == OR_FAULTY) or_make_change(s, a, m, INC(s, a, m), OR_TOMBSTONE);
        break;
    }
}

void or_step(or_sim *s, const or_event *ev, size_t nev) {
    uint32_t n = s->n;
    uint32_t k = s->cfg.ping_request_size;
    /* E */
    for (size_t i = 0; i < nev; i++)
        if (ev[i].round == s->round) apply_event(s, &ev[i]);
    /* T */
#pragma omp parallel for schedule(dynamic, 64)
    for (uint32_t o = 0; o < n; o++)
        if (s->o[o].live) or_fire_timers(s, o);
    /* S */
    int32_t *t = s->last_target;
#pragma omp parallel for schedule(dynamic, 64)
    for (uint32_t o = 0; o < n; o++) t[o] = s->o[o].live ? or_next(s, o) : -1;
    /* I */
    msg *S = (msg *)calloc(n, sizeof(msg));
    uint32_t *C = (uint32_t *)calloc(n, sizeof(uint32_t));
    int64_t *I = (int64_t *)calloc(n, sizeof(int64_t));
#pragma omp parallel for schedule(dynamic, 64)
    for (uint32_t o = 0; o < n; o++) {
        if (t[o] < 0) continue;
        S[o].v = issue_changes(s, o, &S[o].n);
        C[o] = or_checksum(s, o);
        I[o] = INC(s, o, o);
        CTR_ADD(s, OR_C_PINGS, 1);
        CTR_ADD(s, OR_C_MSG_CHANGES, (uint64_t)S[o].n);
    }
    /* D: receiver j processes its inbox in ascending sender order (receivers are independent) */
    int32_t *cnt = (int32_t *)calloc(n + 1, sizeof(int32_t));
    for (uint32_t o = 0; o < n; o++)
        if (t[o] >= 0 && reach(s, o, (uint32_t)t[o])) cnt[t[o] + 1]++;
    for (uint32_t j = 0; j < n; j++) cnt[j + 1] += cnt[j];
    int32_t *inbox = (int32_t *)malloc(sizeof(int32_t) * (cnt[n] + 1));
    int32_t *fill = (int32_t *)calloc(n, sizeof(int32_t));
    for (uint32_t o = 0; o < n; o++)
        if (t[o] >= 0 && reach(s, o, (uint32_t)t[o])) inbox[cnt[t[o]] + fill[t[o]]++] = (int32_t)o;
    msg *R = (msg *)calloc(n, sizeof(msg));
#pragma omp parallel for schedule(dynamic, 16)
    for (uint32_t j = 0; j < n; j++) {
        for (int32_t q = cnt[j]; q < cnt[j + 1]; q++) {
            uint32_t o = (uint32_t)inbox[q];
            or_update(s, j, S[o].v, S[o].n, NULL, 0);                   /* ping_handler.go:40 */
            int32_t fs;
            R[o].v = issue_as_receiver(s, j, (int32_t)o, I[o], C[o], &R[o].n, &fs);
            CTR_ADD(s, OR_C_MSG_CHANGES, (uint64_t)R[o].n);
            if (fs) { CTR_ADD(s, OR_C_FULL_SYNCS, 1); queue_rfs(s, j, (int32_t)o); }
        }
    }
    /* R */
#pragma omp parallel for schedule(dynamic, 16)
    for (uint32_t o = 0; o < n; o++) {
        if (t[o] < 0 || !reach(s, o, (uint32_t)t[o])) continue;
        CTR_ADD(s, OR_C_PINGS_OK, 1);
        or_bump(s, o, S[o].v, S[o].n);                                 /* ping_sender.go:52 */
        or_update(s, o, R[o].v, R[o].n, NULL, 0);                      /* node.go:488 */
    }
    /* Q1 */
    int32_t *H = (int32_t *)malloc(sizeof(int32_t) * (size_t)n * (k ? k : 1));
    int32_t *nh = (int32_t *)calloc(n, sizeof(int32_t));
    msg *S2 = (msg *)calloc(n, sizeof(msg));
    uint32_t *C2 = (uint32_t *)calloc(n, sizeof(uint32_t));
    int64_t *I2 = (int64_t *)calloc(n, sizeof(int64_t));
    uint8_t *failed = (uint8_t *)calloc(n, 1);
#pragma omp parallel for schedule(dynamic, 16)
    for (uint32_t o = 0; o < n; o++) {
        if (t[o] < 0 || reach(s, o, (uint32_t)t[o])) continue;
        failed[o] = 1;
        CTR_ADD(s, OR_C_PINGREQS, 1);
        nh[o] = or_random_pingable(s, o, (int32_t)k, t[o], H + (size_t)o * k);
        S2[o].v = issue_changes(s, o, &S2[o].n);
        C2[o] = or_checksum(s, o);
        I2[o] = INC(s, o, o);
    }
    /* Q2: helper h processes (o, slot) in ascending (o, slot) order; helpers are independent */
    msg *R2 = (msg *)calloc((size_t)n * (k ? k : 1), sizeof(msg));
    int32_t *hcnt = (int32_t *)calloc(n + 1, sizeof(int32_t));
    for (uint32_t o = 0; o < n; o++)
        for (int32_t q = 0; failed[o] && q < nh[o]; q++) {
            int32_t h = H[(size_t)o * k + q];
            if (reach(s, o, (uint32_t)h)) hcnt[h + 1]++;
        }
    for (uint32_t j = 0; j < n; j++) hcnt[j + 1] += hcnt[j];
    int32_t *hin = (int32_t *)malloc(sizeof(int32_t) * (hcnt[n] + 1));
    memset(fill, 0, sizeof(int32_t) * n);
    for (uint32_t o = 0; o < n; o++)
        for (int32_t q = 0; failed[o] && q < nh[o]; q++) {
            int32_t h = H[(size_t)o * k + q];
            if (reach(s, o, (uint32_t)h)) hin[hcnt[h] + fill[h]++] = (int32_t)(o * k + (uint32_t)q);
        }
#pragma omp parallel for schedule(dynamic, 16)
    for (uint32_t h = 0; h < n; h++) {
        for (int32_t q = hcnt[h]; q < hcnt[h + 1]; q++) {
            uint32_t o = (uint32_t)hin[q] / k;
            CTR_ADD(s, OR_C_HELPER_CALLS, 1);
            CTR_ADD(s, OR_C_MSG_CHANGES, (uint64_t)S2[o].n);
            or_update(s, h, S2[o].v, S2[o].n, NULL, 0);                /* ping_request_handler.go:48 */
            /* helper's ping to t_o fails (reachability is an equivalence; ROUND_SEMANTICS §2) */
            int32_t fs;
            msg *r = &R2[hin[q]];
            r->v = issue_as_receiver(s, h, (int32_t)o, I2[o], C2[o], &r->n, &fs); /* 66-69 */
            CTR_ADD(s, OR_C_MSG_CHANGES, (uint64_t)r->n);
            if (fs) CTR_ADD(s, OR_C_FULL_SYNCS_PINGREQ, 1);
        }
    }
    /* Q3 */
#pragma omp parallel for schedule(dynamic, 16)
    for (uint32_t o = 0; o < n; o++) {
        if (!failed[o]) continue;
        uint32_t errs = 0;
        for (int32_t q = 0; q < nh[o]; q++) {
            int32_t h = H[(size_t)o * k + q];
            if (!reach(s, o, (uint32_t)h)) {
                errs++;
                CTR_ADD(s, OR_C_HELPER_ERRORS, 1);
                or_bump(s, o, S2[o].v, S2[o].n);                       /* ping_request_sender.go:105-106 */
            } else {
                msg *r = &R2[(size_t)o * k + q];
                or_update(s, o, r->v, r->n, NULL, 0);                  /* ping_request_sender.go:77-79 */
            }
        }
        if (errs == k) { CTR_ADD(s, OR_C_INCONCLUSIVE, 1); continue; } /* node.go:497-504 */
        CTR_ADD(s, OR_C_SUSPECT_DECL, 1);
        or_make_change(s, o, (uint32_t)t[o], INC(s, o, t[o]), OR_SUSPECT);  /* node.go:506-509 */
    }
    /* F: reverse full syncs; sources snapshotted at phase start */
    msg *snap = (msg *)calloc(n, sizeof(msg));
    uint8_t *need = (uint8_t *)calloc(n, 1);
    for (uint32_t j = 0; j < n; j++)
        for (int32_t q = 0; q < s->o[j].njobs; q++) need[s->o[j].jobs[q]] = 1;
#pragma omp parallel for schedule(dynamic, 16)
    for (uint32_t src = 0; src < n; src++)
        if (need[src]) snap[src].v = membership_as_changes(s, src, &snap[src].n);
    free(need);
#pragma omp parallel for schedule(dynamic, 16)
    for (uint32_t j = 0; j < n; j++) {
        for (int32_t q = 0; q < s->o[j].njobs; q++) {
            int32_t src = s->o[j].jobs[q];
            CTR_ADD(s, OR_C_RFS_DONE, 1);
            or_update(s, j, snap[src].v, snap[src].n, NULL, 0);        /* disseminator.go:300 */
        }
        s->o[j].njobs = 0;
    }
    /* C */
#pragma omp parallel for schedule(dynamic, 16)
    for (uint32_t o = 0; o < n; o++) or_checksum(s, o);
    CTR_ADD(s, OR_C_ROUNDS, 1);
    s->round++;

    for (uint32_t o = 0; o < n; o++) {
        free(S[o].v); free(R[o].v); free(S2[o].v); free(snap[o].v);
    }
    for (size_t i = 0; i < (size_t)n * (k ? k : 1); i++) free(R2[i].v);
    free(S); free(C); free(I); free(cnt); free(inbox); free(fill); free(R);
    free(H); free(nh); free(S2); free(C2); free(I2); free(failed); free(R2); free(hcnt); free(hin); free(snap);
}

/* ------------------------------------------------------------------------------------------ */
/* applied-change stream of watched observers (MemberlistChangesAppliedEvent, events.go:56-61)  */
/* ------------------------------------------------------------------------------------------ */
void or_watch(or_sim *s, uint32_t o, int32_t on) {
    obs *ob = &s->o[o];
    if (on && !ob->watched) {
        ob->wdirty = (uint8_t *)calloc(s->n, 1);
        ob->wlast = (or_change *)calloc(s->n, sizeof(or_change));
        ob->wcs_prev = or_checksum(s, o);
    } else if (!on && ob->watched) {
        free(ob->wdirty); free(ob->wlast);
        ob->wdirty = NULL; ob->wlast = NULL;
    }
    if (on == 2 && ob->watched != 2) {                   /* the per-Update stream starts empty */
        ob->wev_n = 0;
        ob->wcs_ev_prev = or_checksum(s, o);
    }
    ob->watched = on == 2 ? 2 : on ? 1 : 0;
}

/* the per-Update stream (watched == 2): every applied change since the last drain, event_seq[i] = the index of its
 * Update among this drain's applying Updates (0, 1, ...), changes of one Update in the order Update applied them;
 * the checksum at the previous drain, the current one and NumMembers. Returns the number of changes. */
int32_t or_drain_events(or_sim *s, uint32_t o, or_change *out, int32_t *event_seq, int32_t cap, uint32_t *old_cs,
                        uint32_t *new_cs, int32_t *num_members) {
    obs *ob = &s->o[o];
    if (ob->watched != 2) return -1;
    int32_t ev = -1;
    for (size_t i = 0; i < ob->wev_n; i++) {
        if (i == 0 || ob->wev_seq[i] != ob->wev_seq[i - 1]) ev++;
        if ((int32_t)i < cap) {
            out[i] = ob->wev[i];
            event_seq[i] = ev;
        }
    }
    const int32_t k = (int32_t)ob->wev_n;
    ob->wev_n = 0;
    const uint32_t cs = or_checksum(s, o);
    if (old_cs) *old_cs = ob->wcs_ev_prev;
    if (new_cs) *new_cs = cs;
    if (num_members) *num_members = ob->nmem;
    ob->wcs_ev_prev = cs;
    return k;
}

/* every member with an applied change since the last drain (its last applied change), in member order,
 * the checksum at the last drain (OldChecksum), the current one (NewChecksum) and NumMembers */
int32_t or_drain_applied(or_sim *s, uint32_t o, or_change *out, int32_t cap, uint32_t *old_cs, uint32_t *new_cs,
                         int32_t *num_members) {
    obs *ob = &s->o[o];
    if (!ob->watched) return -1;
    int32_t k = 0;
    for (uint32_t m = 0; m < s->n; m++) {
        if (!ob->wdirty[m]) continue;
        ob->wdirty[m] = 0;
        if (k < cap) out[k] = ob->wlast[m];
        k++;
    }
    const uint32_t cs = or_checksum(s, o);
    if (old_cs) *old_cs = ob->wcs_prev;
    if (new_cs) *new_cs = cs;
    if (num_members) *num_members = ob->nmem;
    ob->wcs_prev = cs;
    return k;
}

/* ------------------------------------------------------------------------------------------ */
/* readback                                                                                    */
/* ------------------------------------------------------------------------------------------ */
uint32_t or_round(const or_sim *s) { return s->round; }
void or_row(const or_sim *s, uint32_t o, uint8_t *status, int64_t *inc) {
    memcpy(status, s->st + (size_t)o * s->n, s->n);
    memcpy(inc, s->inc + (size_t)o * s->n, sizeof(int64_t) * s->n);
}
int32_t or_maxp(const or_sim *s, uint32_t o) { return s->o[o].maxp; }
int32_t or_num_pingable(const or_sim *s, uint32_t o) {
    int32_t c = 0;                                                     /* memberlist.go:188-198 */
    for (uint32_t m = 0; m < s->n; m++) if (m != o && is_pingable_status(ST(s, o, m))) c++;
    return c;
}
int32_t or_count_reachable(const or_sim *s, uint32_t o) {              /* memberlist.go:485-497 */
    int32_t c = 0;
    for (uint32_t m = 0; m < s->n; m++) if (is_pingable_status(ST(s, o, m))) c++;
    return c;
}
int32_t or_num_members(const or_sim *s, uint32_t o) {
    int32_t c = 0;
    for (uint32_t m = 0; m < s->n; m++) if (ST(s, o, m) != OR_UNKNOWN) c++;
    return c;
}
int32_t or_changes_count(const or_sim *s, uint32_t o) { return (int32_t)s->o[o].dis.live; }
int32_t or_live(const or_sim *s, uint32_t o) { return s->o[o].live; }

int32_t or_dis_entries(const or_sim *s, uint32_t o, int32_t *member, int32_t *p, int32_t *src, int64_t *sinc,
                       int32_t cap) {
    const omap *d = &s->o[o].dis;
    int32_t k = 0;
    for (uint32_t m = 0; m < s->n; m++) {
        const slot *e = omap_find(d, (int32_t)m);
        if (!e) continue;
        if (k < cap) { member[k] = (int32_t)m; p[k] = e->a; src[k] = e->b; sinc[k] = e->x; }
        k++;
    }
    return k;
}

int32_t or_timer_entries(const or_sim *s, uint32_t o, int32_t *member, int32_t *state, int32_t *fired,
                         int64_t *deadline, int64_t *subj, int32_t cap) {
    const omap *d = &s->o[o].tim;
    int32_t k = 0;
    for (uint32_t m = 0; m < s->n; m++) {
        const slot *e = omap_find(d, (int32_t)m);
        if (!e) continue;
        if (k < cap) { member[k] = (int32_t)m; state[k] = e->a; fired[k] = e->b; deadline[k] = e->x; subj[k] = e->y; }
        k++;
    }
    return k;
}

void or_iter_state(const or_sim *s, uint32_t o, int64_t *idx, uint32_t *epoch) {
    *idx = s->o[o].it_idx;
    *epoch = s->o[o].it_epoch;
}
void or_counters(const or_sim *s, uint64_t *out) { memcpy(out, s->counters, sizeof(s->counters)); }
int32_t or_last_targets(const or_sim *s, int32_t *out) {
    memcpy(out, s->last_target, sizeof(int32_t) * s->n);
    return (int32_t)s->n;
}

/* canonical digests shared with the engine (swimsim_digest): sums of a 64-bit mix */
static uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return k;
}
static uint64_t mix4(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
    return fmix64(a * 0x9E3779B97F4A7C15ULL ^ fmix64(b * 0xC2B2AE3D27D4EB4FULL ^ fmix64(c * 0x165667B19E3779F9ULL ^ fmix64(d + 0xD6E8FEB86659FD93ULL))));
}
static uint64_t to_e(const or_sim *s, int64_t inc) {
    return s->cfg.period_ms ? (uint64_t)((inc - s->cfg.t0_ms) / s->cfg.period_ms) : (uint64_t)inc;
}
static uint64_t round_of_deadline(const or_sim *s, int64_t dl) {
    if (!s->cfg.period_ms) return (uint64_t)dl;
    int64_t d = dl - s->cfg.t0_ms;
    return (uint64_t)((d + s->cfg.period_ms - 1) / s->cfg.period_ms);
}
void or_digest(or_sim *s, uint64_t *rows, uint64_t *dis, uint64_t *tim) {
    uint64_t r = 0, d = 0, t = 0;
    /* sums mod 2^64 are order-independent, so the OpenMP build's reduction equals the serial digest */
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : r, d, t)
    for (uint32_t o = 0; o < s->n; o++) {
        for (uint32_t m = 0; m < s->n; m++) r += mix4(o, m, ST(s, o, m), to_e(s, INC(s, o, m)));
        const omap *dm = &s->o[o].dis;
        for (uint32_t i = 0; i < dm->cap; i++) {
            const slot *e = &dm->s[i];
            if (e->key < 0) continue;
            uint64_t se = e->b == OR_SOURCE_NONE ? 0 : to_e(s, e->x);
            d += mix4((uint64_t)o | (1ULL << 40), (uint64_t)e->key, (uint64_t)e->a | ((uint64_t)(uint32_t)(e->b + 1) << 8), se);
        }
        const omap *tm = &s->o[o].tim;
        for (uint32_t i = 0; i < tm->cap; i++) {
            const slot *e = &tm->s[i];
            if (e->key < 0) continue;
            t += mix4((uint64_t)o | (2ULL << 40), (uint64_t)e->key,
                      (uint64_t)e->a | ((uint64_t)e->b << 4) | (round_of_deadline(s, e->x) << 8), to_e(s, e->y));
        }
    }
    *rows = r; *dis = d; *tim = t;
}
