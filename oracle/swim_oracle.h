/*
 * swim_oracle.h — CPU restatement of ringpop-go's swim hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X engine. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product (libswimsim.so) never links or calls it.
 *
 * Semantics: docs/ROUND_SEMANTICS.md. Each function cites the reference file:line it restates
 * (maniacs-ops/ringpop-go, package swim/).
 *
 * Parity pinning. The merge/dissemination/timer/iterator/heal rules are pinned by the reference's
 * own test assertions (tests/golden/reference_kats.json, tests/test_oracle_kats.py). The Philox
 * generator is pinned by the published Random123 known-answer vectors.
 * Fingerprint32 (go-farm @ fc41e106, FarmHash-32 "mk") absolute values are PARITY UNPINNED:
 * neither the reference tree nor this image holds a FarmHash implementation or vectors.
 * SURVEY.md §8(c) has the details.
 */
#ifndef SWIM_ORACLE_H
#define SWIM_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* statuses == statePrecedence (swim/member.go:112-128); UNKNOWN = not in the memberlist */
enum { OR_ALIVE = 0, OR_SUSPECT = 1, OR_FAULTY = 2, OR_LEAVE = 3, OR_TOMBSTONE = 4, OR_UNKNOWN = 7 };
#define OR_SOURCE_NONE (-1)

/* a wire change (swim/member.go:135-145); tombstone travels as status 4 (validateIncoming/Outgoing) */
typedef struct or_change {
    int32_t member;
    int32_t status;
    int32_t source;      /* member index or OR_SOURCE_NONE */
    int32_t _pad;
    int64_t inc;         /* incarnation, ms */
    int64_t source_inc;  /* ms */
} or_change;

typedef struct or_config {
    uint32_t n;                       /* members */
    int64_t t0_ms;                    /* clock at round 0 (= initial incarnation) */
    int64_t period_ms;                /* MinProtocolPeriod (swim/node.go:80) */
    int64_t suspect_ms, faulty_ms, tombstone_ms;  /* StateTimeouts (swim/node.go:74-78) */
    uint32_t ping_request_size;       /* swim/node.go:86 */
    uint32_t max_rfs_jobs;            /* MaxReverseFullSyncJobs, swim/node.go:96 */
    uint32_t p_factor;                /* swim/disseminator.go:35 */
    uint32_t faithful_checksum;       /* 1: sprintf + sort (memberlist.go:106-128); 0: static order */
    uint64_t seed;                    /* Philox key */
    const char *addresses;            /* NULL: synthetic 10.%03u.%03u.%03u:7000; else n strings */
    uint32_t addr_stride;             /* bytes per address slot when addresses != NULL */
    uint32_t reference_cost;          /* 1: checksum + pingable rescan at every applying Update (the
                                         reference's cost model, CPU baseline); results unchanged */
} or_config;

enum {
    OR_EV_KILL = 1, OR_EV_REVIVE = 2, OR_EV_REINCARNATE = 3, OR_EV_LEAVE = 4,
    OR_EV_PARTITION = 5, OR_EV_HEAL = 6, OR_EV_REAP = 7
};
typedef struct or_event { uint32_t round; uint32_t kind; int32_t a; int32_t b; } or_event;

enum {
    OR_C_ROUNDS, OR_C_PINGS, OR_C_PINGS_OK, OR_C_PINGREQS, OR_C_HELPER_CALLS, OR_C_HELPER_ERRORS,
    OR_C_INCONCLUSIVE, OR_C_SUSPECT_DECL, OR_C_APPLIED, OR_C_REFUTES, OR_C_FULL_SYNCS,
    OR_C_FULL_SYNCS_PINGREQ, OR_C_RFS_DONE, OR_C_RFS_OMITTED, OR_C_TIMERS_FIRED, OR_C_MSG_CHANGES,
    OR_C_HEAL_ATTEMPTS, OR_C_HEAL_FAILURES, OR_NCOUNTERS
};

typedef struct or_sim or_sim;

or_sim *or_create(const or_config *cfg);
void or_destroy(or_sim *s);

/* --- setup --- */
void or_init_converged(or_sim *s);          /* every row: all alive @ t0, maxP = f(N-1) */
void or_init_self_only(or_sim *s);          /* every row: only self alive @ t0, maxP = pFactor */
void or_set_member(or_sim *s, uint32_t o, uint32_t m, int32_t status, int64_t inc);
void or_set_clock_offset(or_sim *s, uint32_t o, int64_t off_ms);
void or_set_live(or_sim *s, uint32_t o, int32_t live);
void or_set_partition(or_sim *s, uint32_t o, int32_t label);
void or_set_round(or_sim *s, uint32_t r);
void or_set_maxp(or_sim *s, uint32_t o, int32_t maxp, int32_t p_factor);
int or_make_change(or_sim *s, uint32_t o, uint32_t m, int64_t inc, int32_t status); /* #applied */
void or_clear_changes(or_sim *s, uint32_t o);
void or_clear_change(or_sim *s, uint32_t o, uint32_t m);   /* disseminator.ClearChange */
int32_t or_add_join_list(or_sim *s, uint32_t j, const or_change *ch, int32_t n);  /* memberlist.AddJoinList */
void or_recompute_pingable(or_sim *s, uint32_t o);

/* --- round driver (docs/ROUND_SEMANTICS.md §4) --- */
void or_step(or_sim *s, const or_event *ev, size_t nev);

/* --- readback --- */
uint32_t or_round(const or_sim *s);
uint32_t or_checksum(or_sim *s, uint32_t o);
void or_row(const or_sim *s, uint32_t o, uint8_t *status, int64_t *inc);
int32_t or_maxp(const or_sim *s, uint32_t o);
int32_t or_num_pingable(const or_sim *s, uint32_t o);
int32_t or_count_reachable(const or_sim *s, uint32_t o);
int32_t or_num_members(const or_sim *s, uint32_t o);
int32_t or_changes_count(const or_sim *s, uint32_t o);
int32_t or_dis_entries(const or_sim *s, uint32_t o, int32_t *member, int32_t *p, int32_t *src,
                       int64_t *sinc, int32_t cap);
int32_t or_timer_entries(const or_sim *s, uint32_t o, int32_t *member, int32_t *state, int32_t *fired,
                         int64_t *deadline, int64_t *subj, int32_t cap);
void or_iter_state(const or_sim *s, uint32_t o, int64_t *idx, uint32_t *epoch);
void or_counters(const or_sim *s, uint64_t *out);
int32_t or_last_targets(const or_sim *s, int32_t *out);  /* phase-S targets of the last round */
int32_t or_live(const or_sim *s, uint32_t o);
/* canonical digests (docs/ROUND_SEMANTICS.md; inc mapped to e = (inc - t0)/period) */
void or_digest(or_sim *s, uint64_t *rows, uint64_t *dis, uint64_t *tim);

/* --- applied-change stream (MemberlistChangesAppliedEvent, swim/events.go:56-61) --- */
void or_watch(or_sim *s, uint32_t o, int32_t on);
int32_t or_drain_applied(or_sim *s, uint32_t o, or_change *out, int32_t cap, uint32_t *old_cs, uint32_t *new_cs,
                         int32_t *num_members);
/* per-Update stream of an observer watched with on = 2: every applied change since the last drain, event_seq[i] =
 * index of its applying Update within the drain; old/new checksum and NumMembers as or_drain_applied */
int32_t or_drain_events(or_sim *s, uint32_t o, or_change *out, int32_t *event_seq, int32_t cap, uint32_t *old_cs,
                        uint32_t *new_cs, int32_t *num_members);

/* --- unit-level primitives (for the reference KATs) --- */
int32_t or_non_local_override(int64_t cur_inc, int32_t cur_st, int64_t ch_inc, int32_t ch_st);
int32_t or_local_override(int32_t is_local, int64_t cur_inc, int64_t ch_inc, int32_t ch_st);
int32_t or_update(or_sim *s, uint32_t j, const or_change *ch, int32_t n, or_change *applied, int32_t cap);
int32_t or_issue_as_sender(or_sim *s, uint32_t j, or_change *out, int32_t cap);
int32_t or_issue_as_receiver(or_sim *s, uint32_t j, int32_t sender, int64_t sender_inc,
                             uint32_t sender_cs, or_change *out, int32_t cap, int32_t *full_sync);
void or_bump(or_sim *s, uint32_t j, const or_change *ch, int32_t n);
int32_t or_membership_as_changes(or_sim *s, uint32_t j, or_change *out, int32_t cap);
int32_t or_next(or_sim *s, uint32_t o);
int32_t or_random_pingable(or_sim *s, uint32_t o, int32_t k, int32_t exclude, int32_t *out);
void or_fire_timers(or_sim *s, uint32_t o);
int32_t or_heal(or_sim *s, uint32_t o, int32_t *targets_out, int32_t cap);
void or_schedule(or_sim *s, uint32_t o, uint32_t m, int32_t state, int64_t subj_inc);
void or_cancel(or_sim *s, uint32_t o, uint32_t m);

/* --- arithmetic building blocks --- */
uint32_t or_fingerprint32(const uint8_t *s, size_t len);
void or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint32_t or_perm(uint64_t seed, uint32_t o, uint32_t epoch, uint32_t n, uint32_t idx);
uint32_t or_perm_inv(uint64_t seed, uint32_t o, uint32_t epoch, uint32_t n, uint32_t m);
size_t or_checksum_string(or_sim *s, uint32_t o, char *out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
