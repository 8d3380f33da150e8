/* ring_oracle.c — TEST INFRASTRUCTURE ONLY (tests/, never the product): a sequential CPU
 * restatement of hashring.HashRing (hashring/hashring.go) for the parity tests of the MI355X ring.
 *
 * It follows the reference call by call: AddRemoveServers (hashring.go:199-229) adds each server
 * that is not in the server set, inserting its replica points Fingerprint32(server ‖ decimal(i)),
 * i = 0..R-1 (hashring.go:148-155), one at a time into a map keyed by the point value where an
 * existing value is kept (redBlackTree.Insert stops at an equal value, rbtree.go:122-126); then it
 * removes each server in the set, deleting the values of its replica points whoever holds them
 * (hashring.go:182-188). The ordered walk of the tree (Lookup / LookupN, hashring.go:258-301,
 * rbtree.go:262-286) is a sorted copy of the map. Checksum = Fingerprint32(join(sort(servers), ";"))
 * (hashring.go:100-118), 0 before the first change. Fingerprint32 is or_fingerprint32 (parity of its
 * absolute values: see swim_oracle.h).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

uint32_t or_fingerprint32(const uint8_t *s, size_t len);

typedef struct {
    uint32_t R;
    /* server names and set */
    char **names;
    uint8_t *in_set;
    size_t nnames, names_cap;
    /* point map: open addressing, key = value, val = name index; state 0 empty, 1 full, 2 deleted */
    uint32_t *key;
    int32_t *val;
    uint8_t *st;
    size_t cap, used, live;
    /* sorted view */
    uint64_t *sorted;
    size_t nsorted;
    int dirty;
    uint32_t checksum;
} or_ring;

static size_t slot_of(uint32_t k, size_t cap) { return (size_t)((k * 0x9E3779B1u) & (uint32_t)(cap - 1)); }

static void map_rehash(or_ring *r, size_t ncap) {
    uint32_t *ok = r->key;
    int32_t *ov = r->val;
    uint8_t *os = r->st;
    size_t oc = r->cap;
    r->key = (uint32_t *)calloc(ncap, 4);
    r->val = (int32_t *)calloc(ncap, 4);
    r->st = (uint8_t *)calloc(ncap, 1);
    r->cap = ncap;
    r->used = r->live = 0;
    for (size_t i = 0; i < oc; i++)
        if (os[i] == 1) {
            size_t p = slot_of(ok[i], ncap);
            while (r->st[p]) p = (p + 1) & (ncap - 1);
            r->st[p] = 1; r->key[p] = ok[i]; r->val[p] = ov[i];
            r->used++; r->live++;
        }
    free(ok); free(ov); free(os);
}

/* redBlackTree.Insert: false if the value exists */
static int map_insert(or_ring *r, uint32_t k, int32_t v) {
    if ((r->used + 1) * 2 > r->cap) map_rehash(r, r->live * 4 > r->cap ? r->cap * 2 : r->cap);
    size_t p = slot_of(k, r->cap), tomb = (size_t)-1;
    while (r->st[p]) {
        if (r->st[p] == 1 && r->key[p] == k) return 0;
        if (r->st[p] == 2 && tomb == (size_t)-1) tomb = p;
        p = (p + 1) & (r->cap - 1);
    }
    if (tomb != (size_t)-1) p = tomb; else r->used++;
    r->st[p] = 1; r->key[p] = k; r->val[p] = v;
    r->live++;
    r->dirty = 1;
    return 1;
}

/* redBlackTree.Delete by value */
static void map_delete(or_ring *r, uint32_t k) {
    size_t p = slot_of(k, r->cap);
    while (r->st[p]) {
        if (r->st[p] == 1 && r->key[p] == k) {
            r->st[p] = 2;
            r->live--;
            r->dirty = 1;
            return;
        }
        p = (p + 1) & (r->cap - 1);
    }
}

static int32_t intern(or_ring *r, const char *s) {
    for (size_t i = 0; i < r->nnames; i++)
        if (strcmp(r->names[i], s) == 0) return (int32_t)i;
    if (r->nnames == r->names_cap) {
        r->names_cap = r->names_cap ? 2 * r->names_cap : 64;
        r->names = (char **)realloc(r->names, r->names_cap * sizeof(char *));
        r->in_set = (uint8_t *)realloc(r->in_set, r->names_cap);
    }
    r->names[r->nnames] = strdup(s);
    r->in_set[r->nnames] = 0;
    return (int32_t)r->nnames++;
}

static int32_t find(const or_ring *r, const char *s) {
    for (size_t i = 0; i < r->nnames; i++)
        if (strcmp(r->names[i], s) == 0) return (int32_t)i;
    return -1;
}

static uint32_t replica_hash(const char *name, uint32_t i) {
    char buf[512];
    size_t n = strlen(name);
    memcpy(buf, name, n);
    char dig[12];
    int nd = 0;
    do { dig[nd++] = (char)('0' + i % 10u); i /= 10u; } while (i);
    for (int k = 0; k < nd; k++) buf[n + k] = dig[nd - 1 - k];
    return or_fingerprint32((const uint8_t *)buf, n + (size_t)nd);
}

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}
static int cmp_str(const void *a, const void *b) { return strcmp(*(char *const *)a, *(char *const *)b); }

static void refresh_sorted(or_ring *r) {
    if (!r->dirty) return;
    free(r->sorted);
    r->sorted = (uint64_t *)malloc((r->live + 1) * 8);
    r->nsorted = 0;
    for (size_t i = 0; i < r->cap; i++)
        if (r->st[i] == 1) r->sorted[r->nsorted++] = ((uint64_t)r->key[i] << 32) | (uint32_t)r->val[i];
    qsort(r->sorted, r->nsorted, 8, cmp_u64);
    r->dirty = 0;
}

static void compute_checksum(or_ring *r) {
    size_t n = 0, bytes = 0;
    char **v = (char **)malloc((r->nnames + 1) * sizeof(char *));
    for (size_t i = 0; i < r->nnames; i++)
        if (r->in_set[i]) { v[n++] = r->names[i]; bytes += strlen(r->names[i]) + 1; }
    qsort(v, n, sizeof(char *), cmp_str);
    char *j = (char *)malloc(bytes + 1);
    size_t len = 0;
    for (size_t i = 0; i < n; i++) {
        if (i) j[len++] = ';';
        size_t l = strlen(v[i]);
        memcpy(j + len, v[i], l);
        len += l;
    }
    r->checksum = or_fingerprint32((const uint8_t *)j, len);
    free(j);
    free(v);
}

or_ring *or_ring_new(uint32_t replica_points) {
    or_ring *r = (or_ring *)calloc(1, sizeof(or_ring));
    r->R = replica_points;
    r->cap = 1024;
    r->key = (uint32_t *)calloc(r->cap, 4);
    r->val = (int32_t *)calloc(r->cap, 4);
    r->st = (uint8_t *)calloc(r->cap, 1);
    return r;
}

void or_ring_free(or_ring *r) {
    if (!r) return;
    for (size_t i = 0; i < r->nnames; i++) free(r->names[i]);
    free(r->names); free(r->in_set); free(r->key); free(r->val); free(r->st); free(r->sorted);
    free(r);
}

int or_ring_add_remove(or_ring *r, const char *const *add, size_t nadd, const char *const *rem, size_t nrem) {
    int changed = 0;
    for (size_t a = 0; a < nadd; a++) {
        int32_t id = intern(r, add[a]);
        if (r->in_set[id]) continue;
        r->in_set[id] = 1;
        for (uint32_t i = 0; i < r->R; i++) map_insert(r, replica_hash(add[a], i), id);
        changed = 1;
    }
    for (size_t k = 0; k < nrem; k++) {
        int32_t id = find(r, rem[k]);
        if (id < 0 || !r->in_set[id]) continue;
        r->in_set[id] = 0;
        for (uint32_t i = 0; i < r->R; i++) map_delete(r, replica_hash(rem[k], i));
        changed = 1;
    }
    if (changed) compute_checksum(r);
    return changed;
}

uint32_t or_ring_checksum(or_ring *r) { return r->checksum; }

uint32_t or_ring_server_count(or_ring *r) {
    uint32_t n = 0;
    for (size_t i = 0; i < r->nnames; i++) n += r->in_set[i];
    return n;
}

/* Lookup: owner name, or NULL for an empty ring */
const char *or_ring_lookup(or_ring *r, const uint8_t *key, size_t len) {
    refresh_sorted(r);
    if (!r->nsorted) return NULL;
    const uint32_t h = or_fingerprint32(key, len);
    size_t lo = 0, hi = r->nsorted;
    while (lo < hi) {
        size_t mid = (lo + hi) / 2;
        if ((uint32_t)(r->sorted[mid] >> 32) < h) lo = mid + 1; else hi = mid;
    }
    if (lo == r->nsorted) lo = 0;
    return r->names[(uint32_t)r->sorted[lo]];
}

/* LookupN: up to n distinct owner names into out (order not significant) */
size_t or_ring_lookup_n(or_ring *r, const uint8_t *key, size_t len, uint32_t n, const char **out) {
    size_t got = 0;
    const uint32_t cnt = or_ring_server_count(r);
    if (n >= cnt) {
        for (size_t i = 0; i < r->nnames; i++)
            if (r->in_set[i]) out[got++] = r->names[i];
        return got;
    }
    refresh_sorted(r);
    const uint32_t h = or_fingerprint32(key, len);
    size_t start = 0;
    while (start < r->nsorted && (uint32_t)(r->sorted[start] >> 32) < h) start++;
    for (int pass = 0; pass < 2 && got < n; pass++)
        for (size_t p = pass ? 0 : start; p < r->nsorted && got < n; p++) {
            const char *o = r->names[(uint32_t)r->sorted[p]];
            int seen = 0;
            for (size_t q = 0; q < got && !seen; q++) seen = out[q] == o;
            if (!seen) out[got++] = o;
        }
    return got;
}

/* the ordered tree: value and owner name of every point, ascending */
size_t or_ring_points(or_ring *r, uint32_t *hash, const char **owner, size_t cap) {
    refresh_sorted(r);
    for (size_t i = 0; i < r->nsorted && i < cap; i++) {
        if (hash) hash[i] = (uint32_t)(r->sorted[i] >> 32);
        if (owner) owner[i] = r->names[(uint32_t)r->sorted[i]];
    }
    return r->nsorted;
}
