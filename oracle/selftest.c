/*
 * selftest.c — TEST INFRASTRUCTURE ONLY: a driver that runs the CPU oracle through every workload kind
 * under AddressSanitizer / UndefinedBehaviorSanitizer (`make -C oracle sanitize`, run by
 * tests/test_oracle_sanitize.py). It exercises the protocol round (kills, revives, reincarnations, leaves,
 * partitions, heals, reaps; SURVEY.md §5 "ASan/UBSan build of the oracle"), every read-back, the
 * applied-change stream, AddJoinList, the checksum in both cost models, and the hash-ring oracle, and checks
 * two consistency properties on the way:
 *   - the checksum in the reference's cost model (string rebuilt, sorted and hashed at every applying
 *     Update, memberlist.go:106-128) equals the static-order one every round;
 *   - the reference cost model leaves every state digest unchanged.
 * Exit status 0 when every check holds; the sanitizers abort on the first memory or UB error.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "swim_oracle.h"

typedef struct or_ring or_ring;
or_ring *or_ring_new(uint32_t replica_points);
void or_ring_free(or_ring *r);
int or_ring_add_remove(or_ring *r, const char *const *add, size_t nadd, const char *const *rem, size_t nrem);
uint32_t or_ring_checksum(or_ring *r);
uint32_t or_ring_server_count(or_ring *r);
const char *or_ring_lookup(or_ring *r, const uint8_t *key, size_t len);
size_t or_ring_lookup_n(or_ring *r, const uint8_t *key, size_t len, uint32_t n, const char **out);
size_t or_ring_points(or_ring *r, uint32_t *hash, const char **owner, size_t cap);

static int failures = 0;
#define CHECK(cond, ...)                                                                                         \
    do {                                                                                                         \
        if (!(cond)) {                                                                                           \
            fprintf(stderr, "selftest: " __VA_ARGS__);                                                           \
            fputc('\n', stderr);                                                                                 \
            failures++;                                                                                          \
        }                                                                                                        \
    } while (0)

static or_config config(uint32_t n, uint32_t faithful, uint32_t refcost, uint64_t seed) {
    or_config c;
    memset(&c, 0, sizeof c);
    c.n = n;
    c.t0_ms = 1500000000000LL;
    c.period_ms = 200;
    c.suspect_ms = 5000;
    c.faulty_ms = 24LL * 3600 * 1000;
    c.tombstone_ms = 60000;
    c.ping_request_size = 3;
    c.max_rfs_jobs = 5;
    c.p_factor = 15;
    c.faithful_checksum = faithful;
    c.seed = seed;
    c.reference_cost = refcost;
    return c;
}

/* one workload: events over `rounds` rounds, run three ways (static checksum, faithful checksum, reference
   cost model); the three must agree on every checksum and digest */
static void run_workload(const char *name, uint32_t n, int self_only, const or_event *ev, size_t nev,
                         uint32_t rounds, uint32_t faulty_ms_short) {
    or_config c0 = config(n, 0, 0, 7), c1 = config(n, 1, 0, 7), c2 = config(n, 0, 1, 7);
    if (faulty_ms_short) c0.faulty_ms = c1.faulty_ms = c2.faulty_ms = faulty_ms_short;
    or_sim *s[3] = {or_create(&c0), or_create(&c1), or_create(&c2)};
    for (int k = 0; k < 3; k++) {
        CHECK(s[k] != NULL, "%s: or_create failed", name);
        if (!s[k]) return;
        if (self_only) or_init_self_only(s[k]);
        else or_init_converged(s[k]);
        or_watch(s[k], 0, 1);
    }
    or_change *buf = malloc(sizeof(or_change) * (size_t)(4 * n + 8));
    int32_t *ia = malloc(sizeof(int32_t) * (size_t)(4 * n + 8)), *ib = malloc(sizeof(int32_t) * (size_t)(4 * n + 8));
    int32_t *ic = malloc(sizeof(int32_t) * (size_t)(4 * n + 8));
    int64_t *la = malloc(sizeof(int64_t) * (size_t)(4 * n + 8)), *lb = malloc(sizeof(int64_t) * (size_t)(4 * n + 8));
    uint8_t *st = malloc(n);
    char *str = malloc((size_t)n * 64 + 64);
    for (uint32_t r = 0; r < rounds; r++) {
        size_t a = 0, b = 0;
        while (a < nev && ev[a].round < r) a++;
        b = a;
        while (b < nev && ev[b].round == r) b++;
        for (int k = 0; k < 3; k++) or_step(s[k], ev + a, b - a);
        uint64_t d[3][3];
        for (int k = 0; k < 3; k++) or_digest(s[k], &d[k][0], &d[k][1], &d[k][2]);
        for (int k = 1; k < 3; k++)
            CHECK(!memcmp(d[0], d[k], sizeof d[0]), "%s: round %u: digests of run %d differ", name, r, k);
        for (uint32_t o = 0; o < n; o += 1 + n / 16) {
            const uint32_t cs0 = or_checksum(s[0], o), cs1 = or_checksum(s[1], o), cs2 = or_checksum(s[2], o);
            CHECK(cs0 == cs1 && cs0 == cs2, "%s: round %u observer %u: checksums %08x %08x %08x", name, r, o, cs0,
                  cs1, cs2);
            /* every read-back */
            int64_t idx;
            uint32_t ep;
            or_row(s[0], o, st, la);
            (void)or_maxp(s[0], o);
            (void)or_num_pingable(s[0], o);
            (void)or_count_reachable(s[0], o);
            (void)or_num_members(s[0], o);
            (void)or_changes_count(s[0], o);
            (void)or_dis_entries(s[0], o, ia, ib, ic, lb, (int32_t)(4 * n));
            (void)or_timer_entries(s[0], o, ia, ib, ic, la, lb, (int32_t)(4 * n));
            or_iter_state(s[0], o, &idx, &ep);
            (void)or_live(s[0], o);
            const size_t len = or_checksum_string(s[0], o, str, (size_t)n * 64 + 64);
            CHECK(len == 0 || or_fingerprint32((const uint8_t *)str, len) == cs0,
                  "%s: round %u observer %u: checksum string does not hash to the checksum", name, r, o);
        }
        uint32_t ocs, ncs;
        int32_t nm;
        (void)or_drain_applied(s[0], 0, buf, (int32_t)(4 * n), &ocs, &ncs, &nm);
        (void)or_last_targets(s[0], ia);
        uint64_t ctr[OR_NCOUNTERS];
        or_counters(s[0], ctr);
    }
    /* unit-level primitives on the final state */
    const int32_t m = or_membership_as_changes(s[0], 1 % n, buf, (int32_t)(4 * n));
    CHECK(m >= 0, "%s: MembershipAsChanges failed", name);
    if (m > 0) {
        (void)or_update(s[0], 2 % n, buf, m, buf + m, (int32_t)(3 * n));
        (void)or_add_join_list(s[0], 3 % n, buf, m < (int32_t)n ? m : (int32_t)n);
    }
    int32_t fs = 0;
    (void)or_issue_as_sender(s[0], 0, buf, (int32_t)(4 * n));
    (void)or_issue_as_receiver(s[0], 0, 1 % n, c0.t0_ms, 0x12345678u, buf, (int32_t)(4 * n), &fs);
    (void)or_random_pingable(s[0], 0, 3, 1 % n, ia);
    (void)or_heal(s[0], 0, ia, (int32_t)(4 * n));
    for (int k = 0; k < 3; k++) or_destroy(s[k]);
    free(buf); free(ia); free(ib); free(ic); free(la); free(lb); free(st); free(str);
}

static void ring_workload(void) {
    or_ring *r = or_ring_new(100);
    enum { NS = 300 };
    static char names[NS][32];
    const char *p[NS];
    for (int i = 0; i < NS; i++) {
        snprintf(names[i], sizeof names[i], "10.0.%d.%d:%d", i / 250, i % 250, 3000 + i % 7);
        p[i] = names[i];
    }
    CHECK(or_ring_checksum(r) == 0, "ring: checksum before the first change");
    or_ring_add_remove(r, p, NS, NULL, 0);
    CHECK(or_ring_server_count(r) == NS, "ring: %u servers after adding %d", or_ring_server_count(r), NS);
    or_ring_add_remove(r, p, 10, p + 10, 20);                  /* re-adds are no-ops, then 20 removals */
    CHECK(or_ring_server_count(r) == NS - 20, "ring: %u servers after removing 20", or_ring_server_count(r));
    const char *out[64];
    for (int k = 0; k < 1000; k++) {
        char key[24];
        const int len = snprintf(key, sizeof key, "key%d", k);
        const char *o = or_ring_lookup(r, (const uint8_t *)key, (size_t)len);
        CHECK(o != NULL, "ring: lookup of %s failed", key);
        const size_t nn = or_ring_lookup_n(r, (const uint8_t *)key, (size_t)len, 5, out);
        CHECK(nn == 5, "ring: LookupN(5) returned %zu", nn);
    }
    const size_t np = or_ring_points(r, NULL, NULL, 0);
    uint32_t *h = malloc(sizeof(uint32_t) * (np + 1));
    const char **ow = malloc(sizeof(char *) * (np + 1));
    CHECK(or_ring_points(r, h, ow, np) == np, "ring: points read-back");
    for (size_t i = 1; i < np; i++) CHECK(h[i - 1] < h[i], "ring: points not strictly ascending at %zu", i);
    free(h);
    free(ow);
    or_ring_free(r);
}

int main(void) {
    /* Fingerprint32 on every length path (0..4, 5..12, 13..24, > 24) */
    uint8_t bytes[200];
    for (int i = 0; i < 200; i++) bytes[i] = (uint8_t)(i * 37 + 11);
    for (size_t len = 0; len <= 200; len++) (void)or_fingerprint32(bytes, len);

    /* config 1/3 style: converged, kills and the suspect -> faulty -> tombstone cascade (short faulty
       timeout so eviction and reap run inside the window) */
    const or_event cascade[] = {{5, OR_EV_KILL, 3, 0}, {5, OR_EV_KILL, 17, 0}, {30, OR_EV_REVIVE, 3, 0},
                                {40, OR_EV_LEAVE, 9, 0}, {60, OR_EV_REAP, 17, 0}};
    run_workload("cascade", 48, 0, cascade, sizeof cascade / sizeof cascade[0], 130, 6000);
    /* config 2 style: churn with reincarnations */
    or_event churn[64];
    size_t nc = 0;
    for (uint32_t r = 2; r < 60 && nc < 64; r += 2) churn[nc++] = (or_event){r, (r / 2) % 2 ? OR_EV_KILL : OR_EV_REVIVE, (int32_t)(r % 40), 0};
    for (uint32_t r = 3; r < 60 && nc < 64; r += 7) churn[nc++] = (or_event){r, OR_EV_REINCARNATE, (int32_t)(r % 40), 0};
    /* events must be in round order */
    for (size_t i = 1; i < nc; i++)
        for (size_t j = i; j > 0 && churn[j - 1].round > churn[j].round; j--) {
            const or_event t = churn[j];
            churn[j] = churn[j - 1];
            churn[j - 1] = t;
        }
    run_workload("churn", 40, 0, churn, nc, 80, 0);
    /* config 4 style: partition and heal */
    or_event part[40];
    size_t np = 0;
    for (int32_t o = 0; o < 32; o++) part[np++] = (or_event){1, OR_EV_PARTITION, o, o < 16 ? 0 : 1};
    part[np++] = (or_event){40, OR_EV_HEAL, 0, 0};
    run_workload("partition", 32, 0, part, np, 70, 0);
    /* self-only start: full syncs and reverse full syncs */
    run_workload("self_only", 24, 1, NULL, 0, 40, 0);
    ring_workload();
    if (failures) {
        fprintf(stderr, "selftest: %d check(s) failed\n", failures);
        return 1;
    }
    printf("selftest ok\n");
    return 0;
}
