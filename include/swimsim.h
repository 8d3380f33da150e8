/*
 * swimsim.h — C ABI of libswimsim.so, the MI355X-native SWIM protocol-round engine.
 *
 * This is the drop-in boundary for ringpop-go's swim hot path. The reference has no FFI: its
 * path sits behind the Go interface swim.NodeInterface (swim/node.go:137-147) and the internal
 * Memberlist / Disseminator / stateTransitions types. Each entry point below says which
 * reference call it replaces. INTEGRATION.md shows the cgo binding a maintainer would add.
 *
 * Conventions
 *  - One handle = one simulated cluster of N members. Observer o is member o's swim.Node.
 *  - Incarnations cross the ABI as int64 milliseconds, like swim.Member.Incarnation
 *    (member.go:52). Inside they are kept as e = (inc - t0_ms) / protocol_period_ms.
 *  - Status codes equal statePrecedence (member.go:112-128): alive 0, suspect 1, faulty 2,
 *    leave 3, tombstone 4. SWIMSIM_UNKNOWN (7) means "not in this node's memberlist".
 *  - Return values: 0 = OK, negative = SWIMSIM_E*. swimsim_last_error() gives the message.
 *    HIP errors are mapped, never aborted on.
 *  - Calls on one handle must be serialized. swimsim_step() blocks and is deterministic.
 *  - The caller owns every output buffer (caller allocates, library fills). No device pointer
 *    escapes.
 */
#ifndef SWIMSIM_H
#define SWIMSIM_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWIMSIM_ABI_VERSION 5

enum {
    SWIMSIM_OK = 0,
    SWIMSIM_EINVAL = -1,     /* bad argument */
    SWIMSIM_ENOMEM = -2,     /* device allocation failed */
    SWIMSIM_EHIP = -3,       /* HIP runtime error */
    SWIMSIM_ECAPACITY = -4,  /* a device pool overflowed (message / dense-snapshot pool) */
    SWIMSIM_ERANGE = -5      /* incarnation not representable as t0 + e*period */
};

enum { SWIMSIM_ALIVE = 0, SWIMSIM_SUSPECT = 1, SWIMSIM_FAULTY = 2, SWIMSIM_LEAVE = 3, SWIMSIM_TOMBSTONE = 4,
       SWIMSIM_UNKNOWN = 7 };
#define SWIMSIM_SOURCE_NONE (-1)

/* Mirrors swim.Options (swim/node.go:45-100) plus the simulation inputs. A zero field means
 * the reference default (util.SelectInt / SelectDuration semantics, util/util.go:220-245). */
typedef struct swimsim_config {
    uint32_t num_members;              /* N */
    uint32_t device;                   /* HIP device ordinal */
    int64_t t0_ms;                     /* clock at round 0 = initial incarnation (default 1.5e12) */
    uint32_t protocol_period_ms;       /* MinProtocolPeriod, default 200 (node.go:80) */
    uint32_t suspect_timeout_ms;       /* StateTimeouts.Suspect, default 5 s (node.go:75) */
    uint32_t faulty_timeout_ms;        /* StateTimeouts.Faulty, default 24 h (node.go:76) */
    uint32_t tombstone_timeout_ms;     /* StateTimeouts.Tombstone, default 1 min (node.go:77) */
    uint32_t ping_request_size;        /* PingRequestSize, default 3 (node.go:86) */
    uint32_t max_reverse_full_sync_jobs; /* MaxReverseFullSyncJobs, default 5 (node.go:96) */
    uint32_t p_factor;                 /* disseminator pFactor, default 15 (disseminator.go:35) */
    uint64_t seed;                     /* Philox key (docs/ROUND_SEMANTICS.md §6) */
    const char *addresses;             /* NULL: synthetic "10.%03u.%03u.%03u:7000"; else N fixed-width,
                                          strictly ascending addresses, each addr_stride bytes */
    uint32_t addr_stride;
    uint32_t max_rounds;               /* incarnation table capacity (default 65536 rounds) */
    uint64_t message_pool_bytes;       /* change-record pool; 0 = automatic */
    uint32_t observer_begin, observer_end; /* shard of observer rows held by this handle; 0,0 = all */
    const struct swimsim_tuning *tuning;   /* NULL: the production engine; else variants for tests (below). Callers
                                              zero-initialise the struct (memset), so a field added later reads 0 */
} swimsim_config;

/* Engine variants the tests and diagnostics select per handle (results are identical in every variant; only where
 * and how the work runs changes). Every field: -1 = the production default. */
typedef struct swimsim_tuning {
    int32_t hot_slots;        /* hot-column slots per row; 0 = no hot columns; default 2,048 */
    int32_t dense_slots;      /* dense snapshot slots (at least 64); default: 2 per row + 64, bounded by a third of
                                 the free HBM; small pools exercise the lazy-snapshot fallbacks */
    int32_t cs_async;         /* 0: every phase-C checksum on the main stream; default 1 (side stream) */
    int32_t cs_async_rows;    /* phase-C launches of at most this many rows go to the side stream; default 12,288 */
    int32_t cs_narrow_rows;   /* launches of at most this many rows use the narrow checksum kernel; 0 = the wide
                                 kernel only; default 8,192 */
    int32_t cs_ref;           /* the reference-row checksum path: 0 off, 1 wide launches (default), 2
                                 every launch of at least 1,024 rows */
    int32_t fault_inject;     /* tests only, bits: 1 = the reference-row path's buffers fail to allocate (the production
                                 kernels stay in charge, create and step succeed); 2 = the next reference-row launch fails
                                 with SWIMSIM_EHIP (the step returns it); 4 = exception rings of 8 entries (ring waits,
                                 wrap-arounds and the fallback rows run); 8 = dedup keys narrowed to 3 bits (fingerprint
                                 groups of unequal rows); 16 = the reference-row kernel's stager waves at raised issue
                                 priority (a schedule in which the chain waves drift apart); 32 = the reference-row
                                 path's exception entries capped at 24 per row (rows ending within the stager's
                                 prefetch of the cap); 64 = seeded sleeps before the reference-row kernel's hand-over
                                 waits and signals, bits 8-11 selecting the delayed roles (g/f chains, h chains,
                                 record stagers, window stagers), bits 12-30 the seed; 128 = no side-stream buffer
                                 set for the reference-row path (side launches keep the narrow kernel); 256 = side
                                 launches of 1,024 rows and more take that path (4,097 by default); 1024 = one
                                 generation of side-stream snapshot slots (phase C waits for the previous round's side
                                 launch); default 0. Results are identical with 4, 8, 16, 32, 64, 128, 256 and 1024. */
} swimsim_tuning;
/* Environment, read at swimsim_create (A/B experiments; results are identical either way): SWIMSIM_SYNC_SPIN=0 waits for
 * the main stream's host round trips in the runtime's stream wait instead of polling an event; SWIMSIM_SIDE2=0 runs both
 * generations of side-stream checksum launches on one stream. */

/* Events applied in phase E of a round (docs/ROUND_SEMANTICS.md §4). */
enum {
    SWIMSIM_EV_KILL = 1,        /* process stops (unreachable, frozen) */
    SWIMSIM_EV_REVIVE = 2,      /* process back + Reincarnate (handlers.go:140-143) */
    SWIMSIM_EV_REINCARNATE = 3, /* memberlist.Reincarnate (memberlist.go:234-236) */
    SWIMSIM_EV_LEAVE = 4,       /* adminLeaveHandler (handlers.go:145-148) */
    SWIMSIM_EV_PARTITION = 5,   /* set partition label of member a to b */
    SWIMSIM_EV_HEAL = 6,        /* discoverProviderHealer.Heal on observer a (heal_via_discover_provider.go:120) */
    SWIMSIM_EV_REAP = 7         /* reapFaultyMembersHandler on observer a (handlers.go:154-163) */
};
typedef struct swimsim_event { uint32_t round; uint32_t kind; int32_t a; int32_t b; } swimsim_event;

enum {
    SWIMSIM_C_ROUNDS, SWIMSIM_C_PINGS, SWIMSIM_C_PINGS_OK, SWIMSIM_C_PINGREQS, SWIMSIM_C_HELPER_CALLS,
    SWIMSIM_C_HELPER_ERRORS, SWIMSIM_C_INCONCLUSIVE, SWIMSIM_C_SUSPECT_DECL, SWIMSIM_C_APPLIED,
    SWIMSIM_C_REFUTES, SWIMSIM_C_FULL_SYNCS, SWIMSIM_C_FULL_SYNCS_PINGREQ, SWIMSIM_C_RFS_DONE,
    SWIMSIM_C_RFS_OMITTED, SWIMSIM_C_TIMERS_FIRED, SWIMSIM_C_MSG_CHANGES, SWIMSIM_C_HEAL_ATTEMPTS,
    SWIMSIM_C_HEAL_FAILURES, SWIMSIM_NCOUNTERS
};

typedef struct swimsim swimsim_t;

/* ---- lifecycle: swim.NewNode (node.go:194-238) for every member, Destroy (node.go:306-318) ---- */
int swimsim_create(const swimsim_config *cfg, swimsim_t **out);
int swimsim_destroy(swimsim_t *h);
const char *swimsim_last_error(swimsim_t *h);
int swimsim_abi_version(void);

/* ---- initial state ---- */
/* converged bootstrap: bootstrapNodes + waitForConvergence + ClearChanges (heal_partition_test.go:416-422) */
int swimsim_init_converged(swimsim_t *h);
/* every node knows only itself (NewNode + MakeAlive(self)), maxP = pFactor (disseminator.go:62) */
int swimsim_init_self_only(swimsim_t *h);
/* raw row write, no side effects (scenario setup) */
int swimsim_set_member(swimsim_t *h, uint32_t observer, uint32_t member, int32_t status, int64_t inc_ms);
/* raw write of a whole row (status[N], inc_ms[N]; SWIMSIM_UNKNOWN = not a member), no side effects:
 * seeds an observer from a received membership, e.g. a joinResponse's (join_handler.go:27-32,
 * memberlist.go:325-334 takes unseen members wholesale). Incarnations must be t0 + e*period. */
int swimsim_set_row(swimsim_t *h, uint32_t observer, const uint8_t *status, const int64_t *inc_ms);
/* memberlist.MakeChange (memberlist.go:282-307): returns #applied (0/1) or an error */
int swimsim_make_change(swimsim_t *h, uint32_t observer, uint32_t member, int64_t inc_ms, int32_t status);
/* disseminator.ClearChanges (disseminator.go:217-221) */
int swimsim_clear_changes(swimsim_t *h, uint32_t observer);
/* memberlist.AddJoinList (memberlist.go:398-406), called by the joiner for each joinResponse
 * (join_sender.go:411): Update of the n changes (distinct members, as MembershipAsChanges lists them;
 * source -1 = not a member, source/source_inc_ms may be NULL), then ClearChange of every applied change
 * except the observer's own. One device launch. *applied = number of applied changes. */
int swimsim_add_join_list(swimsim_t *h, uint32_t observer, const int32_t *member, const int32_t *status,
                          const int64_t *inc_ms, const int32_t *source, const int64_t *source_inc_ms, size_t n,
                          uint32_t *applied);
int swimsim_set_live(swimsim_t *h, uint32_t member, int32_t live);
int swimsim_set_partition(swimsim_t *h, uint32_t member, int32_t label);
int swimsim_set_round(swimsim_t *h, uint32_t round);

/* ---- the hot path: nrounds protocol periods of every live node (gossip.ProtocolPeriod,
 *      gossip.go:178-188, for all N nodes under docs/ROUND_SEMANTICS.md). events are applied
 *      in phase E of the round equal to their .round field. ---- */
int swimsim_step(swimsim_t *h, uint32_t nrounds, const swimsim_event *events, size_t nevents);
/* Heal() on one observer right now (heal_via_discover_provider.go:120-177); targets may be NULL */
int swimsim_heal(swimsim_t *h, uint32_t observer, int32_t *targets, size_t cap, size_t *ntargets);

/* ---- read-back: NodeInterface / memberlist / disseminator views ---- */
uint32_t swimsim_round(swimsim_t *h);
/* GetChecksum (node.go:137-147 → memberlist.Checksum, memberlist.go:73-80), all observers */
int swimsim_checksums(swimsim_t *h, uint32_t *out);
/* memberlist.GetMembers (memberlist.go:459-468) as a dense row: status[N], inc_ms[N] */
int swimsim_row(swimsim_t *h, uint32_t observer, uint8_t *status, int64_t *inc_ms);
/* CountReachableMembers (memberlist.go:485-497) */
int swimsim_count_reachable(swimsim_t *h, uint32_t observer, uint32_t *out);
/* GetReachableMembers (memberlist.go:471-483): member indices, ascending */
int swimsim_reachable(swimsim_t *h, uint32_t observer, uint32_t *idx, size_t cap, size_t *n);
/* NumPingableMembers (memberlist.go:188-198), disseminator.maxP (disseminator.go:49),
 * ChangesCount (disseminator.go:239-244), NumMembers (memberlist.go:174-179) */
int swimsim_node_stats(swimsim_t *h, uint32_t observer, int32_t *pingable, int32_t *maxp,
                       int32_t *changes, int32_t *members);
/* disseminator.changes: members, p, source (or -1), source incarnation (ms) */
int swimsim_changes(swimsim_t *h, uint32_t observer, int32_t *member, int32_t *p, int32_t *source,
                    int64_t *source_inc_ms, size_t cap, size_t *n);
/* stateTransitions.timers: members, state, fired, deadline (ms), subject incarnation (ms) */
int swimsim_timers(swimsim_t *h, uint32_t observer, int32_t *member, int32_t *state, int32_t *fired,
                   int64_t *deadline_ms, int64_t *subject_inc_ms, size_t cap, size_t *n);
/* memberlistIter state: currentIndex, number of reshuffles */
int swimsim_iter_state(swimsim_t *h, uint32_t observer, int64_t *idx, uint32_t *epoch);
/* phase-S ping targets of the last round (-1 = none) */
int swimsim_last_targets(swimsim_t *h, int32_t *out);
int swimsim_counters(swimsim_t *h, uint64_t *out);
/* canonical state digests (same definition as the oracle): rows, dissemination, timers */
int swimsim_digest(swimsim_t *h, uint64_t *rows, uint64_t *dissemination, uint64_t *timers);
/* converged (test_utils.go:188-198): no live node has changes and all live checksums equal */
int swimsim_converged(swimsim_t *h, int32_t *out);

/* ---- upward coupling: NodeInterface.RegisterListener (node.go:146) ----
 * MemberlistChangesAppliedEvent{Changes, OldChecksum, NewChecksum, NumMembers} (swim/events.go:56-61) is
 * emitted by memberlist.Update whenever it applied something (memberlist.go:366-384); Ringpop feeds its
 * hash ring from it (ringpop.go:398-400,550-563). Watch an observer to record its applied changes (off by
 * default: unwatched rows pay one predicated branch per applied change); a drain returns, in member order,
 * the last applied change of every member since the previous drain (the per-Update events of the rounds in
 * between, coalesced per member: the ring's final membership depends only on each member's last change),
 * the checksum at the previous drain (OldChecksum), the current one (NewChecksum) and NumMembers. n = 0:
 * nothing applied, no event. Evictions are not events (RemoveMember emits none, memberlist.go:141-162).
 * At most 64 watched observers per handle.
 * on = 1: the coalesced drain below. on = 2: also the per-Update stream (swimsim_applied_events). on = 0: off. */
int swimsim_watch(swimsim_t *h, uint32_t observer, int32_t on);
int swimsim_applied_changes(swimsim_t *h, uint32_t observer, int32_t *member, int32_t *status, int64_t *inc_ms,
                            int32_t *source, int64_t *source_inc_ms, size_t cap, size_t *n, uint32_t *old_checksum,
                            uint32_t *new_checksum, int32_t *num_members);
/* The per-Update stream of an observer watched with on = 2, without coalescing: one event per Update that applied
 * something (memberlist.go:366-384), in the order the node ran its Updates (docs/ROUND_SEMANTICS.md §4: events, each
 * fired timer in (deadline, member) order, the inbox in sender order, the response, the ping-req relays, the
 * reverse full syncs). Change i belongs to event event[i] (0 .. *nevents-1, ascending); the changes of one event
 * are listed in member order (the reference lists a message's changes in Go map order, which is random). Ringpop's
 * per-change statistics (ringpop.go:398-406) and its ring's insertion order are those of this stream.
 * OldChecksum / NewChecksum / NumMembers are per DRAIN, not per event: the checksum at the previous drain of this
 * stream, the current checksum and the current member count (the reference computes one checksum per Update,
 * memberlist.go:367; this engine keeps the per-round ones). *n = total changes (also when > cap: only cap are
 * written). SWIMSIM_ECAPACITY: more than 4*N changes since the last drain (the stream restarts empty). */
int swimsim_applied_events(swimsim_t *h, uint32_t observer, int32_t *member, int32_t *status, int64_t *inc_ms,
                           int32_t *source, int64_t *source_inc_ms, uint32_t *event, size_t cap, size_t *n,
                           size_t *nevents, uint32_t *old_checksum, uint32_t *new_checksum, int32_t *num_members);

/* NodeInterface.ProtocolStats (node.go:137-147, stats.go:81-104). Each round is one ProtocolPeriod of every
 * live node (gossip.go:178-188), so the Timing histogram is over rounds: the device wall time of each round
 * (HIP events on the engine's stream), in ns. ProtocolRate = max(2 x median, MinProtocolPeriod)
 * (AdjustProtocolRate, gossip.go:110-115). ServerRate = pings and ping-reqs handled per node per simulated
 * second (ping_handler.go:37, ping_request_handler.go:45); ClientRate is never marked by the reference (0).
 * Deviation (documented, not pinnable): the reference's Timing is metrics.NewHistogram(NewUniformSample(10))
 * (gossip.go:65), so its Min/Max/Sum/Mean/Variance/percentiles come from a 10-element random reservoir (Count is
 * the total), and AdjustProtocolRate takes that reservoir's median; its rates are go-metrics Meter.Rate1() (a
 * one-minute EWMA). Here every statistic is over every round (up to 2^20) and rates are means over the run. The
 * reservoir is filled from Go's global math/rand, so no restatement could match it sample for sample. */
typedef struct swimsim_protocol_stats {
    int64_t count;
    double min_ns, max_ns, sum_ns, mean_ns, variance, stddev_ns, median_ns, p75_ns, p95_ns, p99_ns, p999_ns;
    int64_t protocol_rate_ns;
    double client_rate, server_rate, total_rate;
} swimsim_protocol_stats_t;
int swimsim_protocol_stats(swimsim_t *h, swimsim_protocol_stats_t *out);

/* device memory of the handle (DESIGN.md §2 budget): bytes of the row words, dissemination entries (+ presence
 * bits), timers (+ block bounds), message pool and dense snapshots, total bytes held; the dense-snapshot slots
 * (main, side stream) and how many phases hashed their dirty senders before issue because the lazy C_o
 * snapshots would not have fit in the slots (exact either way) */
typedef struct swimsim_memory_t {
    uint64_t row_words, dissemination, timers, message_pool, dense_snapshots, total;
    uint32_t dense_cap, side_cap;
    uint64_t lazy_fallbacks;
} swimsim_memory_t;
int swimsim_memory(swimsim_t *h, swimsim_memory_t *out);

/* ---- measurement ---- */
/* average device time (ms) of each kernel family since the last reset, for roofline reporting */
int swimsim_kernel_times(swimsim_t *h, const char **names, double *avg_ms, uint64_t *launches,
                         double *alg_bytes, size_t cap, size_t *n);
/* enable: 0 off, 1 every kernel family, 2 only the families the bench line's roofline reports (checksum chains, merges,
 * issue; each timed family costs an event pair per launch in the timed stream) */
int swimsim_enable_timing(swimsim_t *h, int32_t enable);
/* the unit counts behind those byte figures since swimsim_enable_timing (rows hashed by each checksum kernel,
 * changes processed / applied by each merge kernel, records issued, ...): names[i], values[i]; "hot_slots" is
 * the number of hot-column slots in use now (not a count since the reset) */
int swimsim_kernel_units(swimsim_t *h, const char **names, double *values, size_t cap, size_t *n);
/* profiler window marker: one tiny kernel (k_profile_mark) on the engine's stream, after the side stream drained */
int swimsim_profile_mark(swimsim_t *h, uint32_t id);
/* time the checksum kernel alone on the first nrows rows — average ms per launch. mode 0: the production choice for
 * nrows rows, 1: the wide kernel (k_checksum3), 2: the narrow kernel (k_checksum_q16), 4: k_checksum3 with four row
 * groups per workgroup, 5: the reference-row path forced (reference row, k_csd_scan, k_csr_rec, k_csr3 and the
 * fallback launches for the rows it leaves), 6: the same on the side stream with its own buffer set (csr2; at most
 * 12,288 rows; SWIMSIM_EINVAL when the set was not allocated); other modes (diagnostic variants) only in the diagnostics library
 * tools/libswimsim_diag.so */
int swimsim_bench_checksum(swimsim_t *h, uint32_t nrows, int32_t mode, int32_t reps, double *ms);
/* the reference-row checksum path so far (swimsim_checksum_ref.hip + swimsim_checksum_csr.hip; swimsim_tuning.cs_ref =
 * 0 off, 1 wide launches, 2 every launch of >= 1024 rows): its launches, the rows it left to the production kernels
 * and, per reason (8 entries: short string, exception-entry capacity, workgroup window plan, record capacity,
 * exception slots of a wave, 5..7 reserved = 0), how many of those rows had it. The counts are kept on the device and
 * read here (no host synchronisation inside a round). */
int swimsim_checksum_path_stats(swimsim_t *h, uint64_t *delta_launches, uint64_t *fallback_rows, uint64_t *reasons);
/* diagnostics library only: the 32-bit words of every 20-byte block the checksum kernel hashes for row o (W = 19) */
int swimsim_debug_cs_stream(swimsim_t *h, uint32_t o, uint32_t *out, size_t cap_words);

/* ---- shards: one cluster's observer rows split over G shards ----
 * The reference runs one swim.Node per process; here a shard owns observer rows
 * [N*r/G, N*(r+1)/G) of one simulated cluster and exchanges every cross-shard message (ping
 * requests and responses, ping-req relays, reverse-full-sync and heal memberships) with the other
 * shards at fixed points of the round. With G > 1 swimsim_step() is collective: every shard calls
 * it with the same events. Results stay bit-identical to G = 1. */
/* G shards in this process (one thread each in swimsim_group_step), all on cfg->device or on
 * devices[i]; copies between shards are device-to-device (peer copies across GPUs) */
int swimsim_group_create(const swimsim_config *cfg, uint32_t nshards, const int32_t *devices, swimsim_t **out);
int swimsim_group_step(swimsim_t *const *handles, uint32_t nshards, uint32_t nrounds, const swimsim_event *events,
                       size_t nevents);
/* one process per GPU: rank 0 makes an id, the launcher broadcasts it, every rank attaches its
 * handle (created with observer_begin/end = its canonical shard); exchanges use RCCL send/recv */
int swimsim_comm_unique_id(uint8_t *out, size_t cap);   /* returns the id length (128) */
int swimsim_comm_attach(swimsim_t *h, uint32_t nranks, uint32_t rank, const uint8_t *id, size_t len);
int swimsim_shard_info(swimsim_t *h, uint32_t *nshards, uint32_t *rank, uint32_t *lo, uint32_t *hi,
                       uint64_t *exchanged_bytes, uint64_t *exchanges);
/* Host synchronisations the cross-shard exchanges of this handle took so far (measurement): one per exchange on the
 * RCCL transport (segment sizes travel on the device behind the pack-size kernel), three on the local and host
 * transports. */
int swimsim_exchange_syncs(swimsim_t *h, uint64_t *syncs);
/* one process per shard with a caller-supplied host transport (any process group: a test harness
 * over gloo, an MPI job, ...). The library stages the packed parcels through host memory and calls:
 *   alltoall_u64: k values to every shard; recv[s*k + i] = shard s's send[rank*k + i]
 *   alltoallv:    segment p of sbuf ([soff[p], soff[p] + sbytes[p])) goes to shard p; the segment
 *                 from shard s lands at rbuf + roff[s] (rbytes[s] bytes, known from a prior alltoall_u64)
 *   bcast:        bytes of shard root to every shard
 * Each returns 0 on success. Same collective call order as the RCCL transport. */
typedef struct swimsim_host_transport {
    void *ctx;
    int (*alltoall_u64)(void *ctx, const uint64_t *send, uint64_t *recv, int32_t k);
    int (*alltoallv)(void *ctx, const uint8_t *sbuf, const uint64_t *soff, const uint64_t *sbytes, uint8_t *rbuf,
                     const uint64_t *roff, const uint64_t *rbytes);
    int (*bcast)(void *ctx, void *buf, size_t bytes, uint32_t root);
} swimsim_host_transport;
int swimsim_comm_attach_host(swimsim_t *h, uint32_t nranks, uint32_t rank, const swimsim_host_transport *t);
/* diagnostics (transport conformance): one collective exchange of caller bytes through the handle's shard
 * transport, exactly as the round's parcel exchange moves them (size exchange, then the segments). send holds
 * the segments for shards 0..G-1 back to back (sbytes[G]); recv receives the segments from shards 0..G-1 back
 * to back (rbytes[G] = their sizes). Every shard calls it. */
int swimsim_debug_exchange(swimsim_t *h, const uint8_t *send, const uint64_t *sbytes, uint8_t *recv, size_t rcap,
                           uint64_t *rbytes);

#ifdef __cplusplus
}
#endif
#endif
