// swimsim_device.h — device-side data layout and inline building blocks of the MI355X engine.
//
// Layout in HBM (one handle, NL observer rows of a padded stride NP = roundup(N, 64)):
//   mw  u32 [NL][NP]   member word = (e << 3) | status. e = (inc - t0)/period. Status codes =
//                      statePrecedence (swim/member.go:112-128), 7 = not in the memberlist.
//                      (e,status) as one integer makes nonLocalOverride (member.go:79-93) a single
//                      unsigned compare.
//   dent u32x2[NL][NP] dissemination entry (disseminator.go:39-42): {source | p << 24, source e};
//                      p = 0xFF: no entry. The entry's (status, incarnation) is the row's member
//                      word (every Apply is followed by RecordChange, node.go:424-428).
//   tst u8  [NL][NP]   timer state (suspect 1 / faulty 2 / tombstone 4) | 0x80 fired
//   tmr u32x2 [NL][NP] timer {deadline round, subject e}
//   dbit u32 [NL][NBIT] bit m: member m has a dissemination entry (exactly: p != 0xFF)
//   tblk u32 [NL][NB]  lower bound of the unfired timer deadlines in block b
// Messages are pools of 16-byte change records {member | status<<24, e, source, source e} (plus the member's hot slot
// in spare bits, rec_make below), or dense row snapshots for MembershipAsChanges (disseminator.go:107-123).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swimdev {

constexpr uint32_t ST_ALIVE = 0, ST_SUSPECT = 1, ST_FAULTY = 2, ST_LEAVE = 3, ST_TOMB = 4, ST_UNKNOWN = 7;
constexpr uint32_t SRC_NONE = 0xFFFFFFFFu;
constexpr uint32_t NO_DEADLINE = 0xFFFFFFFFu;
constexpr uint8_t DP_NONE = 0xFF;
// dissemination entry word 0: source (24 bits, 0xFFFFFF = none) | p << 24
constexpr uint32_t DE_NONE = 0xFFFFFFFFu;                      // no entry, no source
__host__ __device__ inline uint32_t de_p(uint32_t x) { return x >> 24; }
__host__ __device__ inline uint32_t de_src(uint32_t x) { return (x & 0xFFFFFFu) == 0xFFFFFFu ? SRC_NONE : (x & 0xFFFFFFu); }
__host__ __device__ inline uint32_t de_x(uint32_t src, uint32_t p) { return (src & 0xFFFFFFu) | (p << 24); }

enum Counter {
    C_ROUNDS, C_PINGS, C_PINGS_OK, C_PINGREQS, C_HELPER_CALLS, C_HELPER_ERRORS, C_INCONCLUSIVE,
    C_SUSPECT_DECL, C_APPLIED, C_REFUTES, C_FULL_SYNCS, C_FULL_SYNCS_PINGREQ, C_RFS_DONE, C_RFS_OMITTED,
    C_TIMERS_FIRED, C_MSG_CHANGES, C_HEAL_ATTEMPTS, C_HEAL_FAILURES, C_NCOUNTERS,
    // measurement-only counters (not part of the parity record)
    // (merges and applies of k_recv and k_resp are counted apart: C_X_MERGED + 5 / C_X_APPLIED + 5)
    // (C_X_CS_ROWS / C_X_CS_ROWS_N: rows hashed by k_checksum3 or k_cs_delta / k_checksum_q16 launches, snapshots
    // included; C_X_CSD_SCANNED: rows k_csd_scan read)
    C_X_MERGED = C_NCOUNTERS, C_X_APPLIED, C_X_ISSUED, C_X_CS_ROWS, C_X_CS_DUP,
    C_X_MERGED_R, C_X_APPLIED_R, C_X_RISSUED, C_X_RCALLS, C_X_BUMPED, C_X_CS_ROWS_N, C_X_CSD_SCANNED,
    // dense messages merged (MembershipAsChanges: full-sync responses in k_resp / k_resolve, reverse full syncs in
    // k_jobs_merge, heal lists), and the changes the reverse full syncs applied
    C_X_DENSE_RESP, C_X_DENSE_JOBS, C_X_JOBS_APPLIED, C_X_DENSE_HEAL,
    // deferred full-sync decisions (k_defer_eq): all, settled by row equality, with no issue-time row to compare with
    // (C_X_DEFER_REP: settled against a clean row of the sender's issue-time checksum, k_cs_reps)
    // (C_X_DEFER_UNDO: settled against the sender's row with this phase's logged merges undone, d.ulog)
    C_X_DEFER, C_X_DEFER_EQ, C_X_DEFER_NOROW, C_X_DEFER_REP, C_X_DEFER_UNDO, C_NALL
};

constexpr int CTR_SHARDS = 64, CTR_STRIDE = 48;   // d.ctr is [CTR_SHARDS][CTR_STRIDE] u64
static_assert(C_NALL + 8 <= CTR_STRIDE, "counter block too small (8 diagnostic slots follow C_NALL)");
constexpr uint32_t POOL_SHARDS = 64, POOL_CUR_STRIDE = 16;   // d.pool_cur is [POOL_SHARDS][POOL_CUR_STRIDE] u64

enum ErrBits : uint32_t {
    E_POOL = 1, E_DENSE = 2, E_ECAP = 4, E_SHORT = 8, E_ITER = 16, E_COUNT = 32, E_XCAP = 64
};

struct MsgDesc {        // a change list in flight
    uint32_t off_lo, off_hi;  // sparse: record offset in the pool; dense: slot index in off_lo
    uint32_t len;             // records (dense: number of known members)
    uint32_t kind;            // 0 sparse, 1 dense, 2 none
};

struct DS {
    uint32_t N, NP, NL, lo, NB, NBW;
    uint32_t W;
    uint32_t pfactor, K, maxjobs;
    uint32_t to_susp, to_faulty, to_tomb;  // timeouts in rounds
    uint32_t ecap;
    uint64_t seed;
    uint32_t *mw;
    uint2 *dent;            // {source | p << 24, source e}
    uint8_t *tst;
    uint2 *tmr;             // {timer deadline round, timer subject e}
    uint32_t *dbit;         // [NL][NBIT] dissemination presence bits
    uint32_t NBIT;          // words per row of dbit (multiple of 4)
    int32_t *ping, *maxp, *dcnt;
    uint32_t *dirty, *cs;
    int32_t *it_idx;
    uint32_t *it_ep, *tmin, *njobs, *jobs;
    uint32_t *tblk;
    uint8_t *live;
    int32_t *part;
    const uint32_t *addrw;  // [N][6]
    const uint32_t *tailw;  // [ecap*4][8]: tail bytes status‖digits‖';' as words, word 6 = tail length
    const uint32_t *rtail;  // [ecap*4][8]: record bytes [4*(W/4), 4*(W/4) + 28) of addr‖tail with the
                            // address bytes zeroed (tail pre-shifted by W%4 bytes); byte 27 (word 6's
                            // high byte, never a record byte) = record length; word 7 = the record's
                            // last 4 bytes
    const uint32_t *rtail8; // [ecap*8][8]: rtail indexed by the member word itself (e << 3 | status), the
                            // entries of statuses 4..7 all zero (record length 0: not in the string)
    unsigned long long *ctr;
    uint32_t *err;
    uint4 *pool;
    unsigned long long *pool_cur;    // sub-pool cursors (pool_alloc)
    unsigned long long pool_cap;
    uint32_t *dense;        // [dense_cap][NP]
    uint4 *dense_meta;      // {source, source e, known count, unused}
    uint32_t *dense_cur;
    uint32_t dense_cap;
    uint32_t *dense_len;    // checksum-string length of each snapshot
    int32_t *dense_last;    // last included member of each snapshot (-2: rescan)
    uint32_t *dense_cs;     // checksum of each snapshot (deferred full-sync decisions)
    // slots [dense_cap, dense_cap + snap_cap) of the dense arrays hold the round-end snapshots whose
    // checksums are hashed on the side stream while the next round runs
    uint32_t *cpslot;       // [NL] dense slot whose dense_cs will hold the row's checksum, or SRC_NONE
    uint32_t *clen;         // [NL] checksum-string length of each row
    int32_t *clast;         // [NL] last included member (-2: rescan)
    unsigned long long *fp; // [NL] row fingerprint: sum over members of fpmix(m, member word), kept by the merges
    uint32_t dig_d0;          // decimal digits of t0
    uint32_t max_tail;        // longest record tail (status ‖ digits ‖ ';') in the incarnation table
    uint32_t min_tail;        // shortest one
    uint32_t G, rank;         // observer-row shards of the cluster and this handle's shard
    const uint32_t *shard_lo; // [G+1] first observer of each shard (ascending, shard_lo[G] = N)
    uint32_t dig_thr[8];      // e at which t0 + e*period gains a digit (0xFFFFFFFF = never)
    // applied-change stream of watched rows (MemberlistChangesAppliedEvent, swim/events.go:56-61)
    uint32_t *wslot;          // [NL] watched row -> slot of wlog, SRC_NONE if unwatched; nullptr: no row watched
    uint4 *wlog;              // [slots][NP] per member, the last change applied since the last drain:
                              // {member word, source, source e, 1}; .w = 0: none
    // per-Update stream of the watched rows whose slot bit is set in wev_mask (swimsim_watch on = 2): every applied
    // change in apply order, {member, member word, source, source e}, tagged with its Update's sequence number
    // (useq of the row when the Update began; all changes of one Update share it, memberlist.go:366-384)
    uint64_t wev_mask;
    uint4 **wevs;             // [slots] -> [wev_cap] records (allocated when the slot first turns on = 2)
    unsigned long long **wevts; // [slots] -> [wev_cap] Update tags
    uint32_t *wev_cnt;        // [slots] records appended since the last drain (may exceed wev_cap: overflow)
    uint32_t wev_cap;
    unsigned long long *useq; // [NL] Update sequence of each row (nullptr: no event stream on); +1 per applying
                              // Update; phase T's timers take tags above it in (deadline, member) order
    // hot columns: compact copies of the row words and dissemination cells of the members that
    // sit in dissemination buffers, so that issue, merge and bump gather from a few KB per row instead of one
    // 64-B sector per member. hmw[ol][k] == mw[ol][hlist[k]] for every slot k < hot_cnt[0] (every write of a hot
    // member's word goes to both copies: snapshots and checksums stream the dense words). hde[ol][k] IS the
    // dissemination cell of member hlist[k]: merges, bumps and evictions of a hot member write only the slot, and
    // dent[ol][hlist[k]] is stale until k_hot_flush writes the slots back (before hot_reset drops them and
    // before a host read-back of dent). hidx = nullptr: off.
    uint32_t *hidx;           // [N] member -> hot slot, SRC_NONE if not hot
    uint32_t *hlist;          // [HP] slot -> member
    uint32_t *hmw;            // [NL][HP]
    uint2 *hde;               // [NL][HP]
    uint32_t *colx;           // [NBIT] columns in which rows may differ: every row-word write since the rows were last
                              // known equal marks its member (the reference-row scan reads only these columns)
    uint32_t *hotnew;         // [NBIT] members that got a new dissemination entry while not hot
    uint32_t *hot_cnt;        // {slots in use, slots filled}
    uint32_t HP;              // hot slots per row
    int32_t *nhe;             // [NL] dissemination entries of members WITHOUT a hot slot; 0: every buffered member of
                              // the row is hot, so issue walks the hot slots instead of the presence bitmap
    // the divergent columns (colx) as lists, rebuilt by k_ucols before every kernel that compares or scans rows by
    // them: ucl = every colx column in member order (ucnt[0] of them) with its hot slot uhk (SRC_NONE: none), ucold =
    // the colx columns without a hot slot (ucnt[1], any order). Rows are equal iff equal at the hot slots and ucold.
    uint32_t *ucl, *uhk, *ucold, *ucnt;
    // the words a receive phase's merges overwrote (k_recv, phases D and Q2): per row up to ULOG_CAP {member, old word}
    // in apply order and their count (ULOG_CAP + 1: more, not usable). A row that was clean when it issued its message
    // and changed only in the phase since is its issue-time row with the first old word of each logged member restored
    // (k_defer_eq); nullptr: off
    uint2 *ulog;
    uint32_t *ulog_cnt;
};
constexpr uint32_t ULOG_CAP = 64;

// hot slot of member m, SRC_NONE when m has none (or hot columns are off)
__device__ __forceinline__ uint32_t hot_slot(const DS &d, uint32_t m) { return d.hidx ? d.hidx[m] : SRC_NONE; }

__host__ __device__ inline bool is_pingable(uint32_t st) { return st <= ST_SUSPECT; }

// A change record in the message pool is 16 B: {member | status << 24 | tag_lo << 27, e | tag_hi << 24, source,
// source e} (e < 2^24: ensure_ecap). The 13-bit tag carries the member's hot slot in the receiving handle,
// written by the issuer, which has just read the member's cell from that slot, so the merge, the bump and the
// receiver's RecordChange test reach the hot word without the dependent hidx lookup: 0 = not known (the consumer looks
// it up: heal diffs), k + 1 = slot k, RT_COLD = no slot. Slots are assigned only at the start of phase I, and records
// never outlive their round (the pool restarts every round), so a tag stays right until its record is consumed;
// k_x_unpack re-tags imported records with the receiving shard's own slots.
constexpr uint32_t RT_LOOKUP = 0, RT_COLD = 8191, RT_MAXSLOTS = 8128;   // (hot slots per row at most RT_MAXSLOTS)
__host__ __device__ inline uint32_t rec_m(const uint4 &r) { return r.x & 0xFFFFFFu; }
__host__ __device__ inline uint32_t rec_st(const uint4 &r) { return (r.x >> 24) & 7u; }
__host__ __device__ inline uint32_t rec_e(const uint4 &r) { return r.y & 0xFFFFFFu; }
__host__ __device__ inline uint32_t rec_tag(const uint4 &r) { return (r.x >> 27) | ((r.y >> 24) << 5); }
__host__ __device__ inline uint32_t tag_of_slot(uint32_t hk) { return hk == SRC_NONE ? RT_COLD : hk + 1u; }
__host__ __device__ inline uint4 rec_make(uint32_t m, uint32_t st, uint32_t e, uint32_t src, uint32_t sinc, uint32_t tag) {
    return make_uint4(m | (st << 24) | (tag << 27), e | ((tag >> 5) << 24), src, sinc);
}
__host__ __device__ inline uint4 rec_retag(const uint4 &r, uint32_t tag) {
    return make_uint4((r.x & 0x07FFFFFFu) | (tag << 27), (r.y & 0xFFFFFFu) | ((tag >> 5) << 24), r.z, r.w);
}
// the hot slot of a record's member in this handle (SRC_NONE: none)
__device__ __forceinline__ uint32_t rec_slot(const DS &d, const uint4 &r) {
    const uint32_t t = rec_tag(r);
    return t == RT_LOOKUP ? hot_slot(d, rec_m(r)) : t == RT_COLD ? SRC_NONE : t - 1u;
}

// shard that owns observer row o (G is small: a linear scan over the shard boundaries)
__device__ __forceinline__ uint32_t owner_of(const DS &d, uint32_t o) {
    uint32_t r = 0;
    while (r + 1 < d.G && o >= d.shard_lo[r + 1]) r++;
    return r;
}

__host__ __device__ inline int32_t digits10(int32_t n) {
    int32_t d = 0;
    while (n > 0) { d++; n /= 10; }
    return d;
}

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. 2011, Random123 constants) and the Feistel permutation
// ---------------------------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };

__host__ __device__ inline U4 philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; r++) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
    }
    return U4{c0, c1, c2, c3};
}

__host__ __device__ inline uint32_t pick(const U4 &v, uint32_t i) {
    return (i & 3) == 0 ? v.x : (i & 3) == 1 ? v.y : (i & 3) == 2 ? v.z : v.w;
}

__host__ __device__ inline uint32_t mulhi_n(uint32_t x, uint32_t n) { return (uint32_t)(((uint64_t)x * n) >> 32); }

__host__ __device__ inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

struct Feistel {
    uint32_t k0, k1, k2, k3, half, mask;
    __host__ __device__ void init(uint64_t seed, uint32_t o, uint32_t epoch, uint32_t n) {
        U4 k = philox10(epoch, o, 1u, 0u, seed);
        k0 = k.x; k1 = k.y; k2 = k.z; k3 = k.w;
        uint32_t b = 2;
        while (b < 32 && ((uint64_t)1 << b) < n) b += 2;
        half = b / 2;
        mask = (1u << half) - 1u;
    }
    __host__ __device__ uint32_t enc(uint32_t x) const {
        uint32_t L = x >> half, R = x & mask, t;
        t = L ^ (fmix32(R ^ k0) & mask); L = R; R = t;
        t = L ^ (fmix32(R ^ k1) & mask); L = R; R = t;
        t = L ^ (fmix32(R ^ k2) & mask); L = R; R = t;
        t = L ^ (fmix32(R ^ k3) & mask); L = R; R = t;
        return (L << half) | R;
    }
    __host__ __device__ uint32_t dec(uint32_t x) const {
        uint32_t L = x >> half, R = x & mask, t;
        t = R ^ (fmix32(L ^ k3) & mask); R = L; L = t;
        t = R ^ (fmix32(L ^ k2) & mask); R = L; L = t;
        t = R ^ (fmix32(L ^ k1) & mask); R = L; L = t;
        t = R ^ (fmix32(L ^ k0) & mask); R = L; L = t;
        return (L << half) | R;
    }
    __host__ __device__ uint32_t perm(uint32_t idx, uint32_t n) const {
        uint32_t x = idx;
        do { x = enc(x); } while (x >= n);
        return x;
    }
    __host__ __device__ uint32_t inv(uint32_t m, uint32_t n) const {
        uint32_t x = m;
        do { x = dec(x); } while (x >= n);
        return x;
    }
};

// ---------------------------------------------------------------------------------------------
// FarmHash-32 "mk" pieces (go-farm Fingerprint32; glide.lock:18-19, call site memberlist.go:86)
// ---------------------------------------------------------------------------------------------
constexpr uint32_t FH_C1 = 0xcc9e2d51u, FH_C2 = 0x1b873593u;

__host__ __device__ inline uint32_t ror32(uint32_t v, int s) { return (v >> s) | (v << (32 - s)); }

__host__ __device__ inline uint32_t fh_mur(uint32_t a, uint32_t h) {
    a *= FH_C1; a = ror32(a, 17); a *= FH_C2;
    h ^= a; h = ror32(h, 19);
    return h * 5 + 0xe6546b64u;
}

struct FH {
    uint32_t h, g, f;
    __host__ __device__ void block(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e) {
        h += a; g += b; f += c;
        h = fh_mur(d, h) + e;
        g = fh_mur(c, g) + a;
        f = fh_mur(b + e * FH_C1, f) + d;
        f += g; g += f;
    }
    // len > 24 prologue from the last 20 bytes t0..t4 (= Fetch32 at len-20, -16, -12, -8, -4)
    __host__ __device__ void init(uint32_t len, uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3, uint32_t t4) {
        h = len; g = FH_C1 * len; f = g;
        uint32_t a0 = ror32(t4 * FH_C1, 17) * FH_C2;
        uint32_t a1 = ror32(t3 * FH_C1, 17) * FH_C2;
        uint32_t a2 = ror32(t1 * FH_C1, 17) * FH_C2;
        uint32_t a3 = ror32(t2 * FH_C1, 17) * FH_C2;
        uint32_t a4 = ror32(t0 * FH_C1, 17) * FH_C2;
        h ^= a0; h = ror32(h, 19); h = h * 5 + 0xe6546b64u;
        h ^= a2; h = ror32(h, 19); h = h * 5 + 0xe6546b64u;
        g ^= a1; g = ror32(g, 19); g = g * 5 + 0xe6546b64u;
        g ^= a3; g = ror32(g, 19); g = g * 5 + 0xe6546b64u;
        f += a4; f = ror32(f, 19) + 113;
    }
    __host__ __device__ uint32_t fin() {
        g = ror32(g, 11) * FH_C1; g = ror32(g, 17) * FH_C1;
        f = ror32(f, 11) * FH_C1; f = ror32(f, 17) * FH_C1;
        h = ror32(h + g, 19); h = h * 5 + 0xe6546b64u; h = ror32(h, 17) * FH_C1;
        h = ror32(h + f, 19); h = h * 5 + 0xe6546b64u; h = ror32(h, 17) * FH_C1;
        return h;
    }
};

// per-member term of the row fingerprint (order-free sum; equal rows have equal sums, so the
// checksum kernel hashes one row per distinct content after an exact comparison)
__host__ __device__ inline uint64_t fpmix(uint32_t m, uint32_t w) {
    uint64_t k = ((uint64_t)m << 32) | w;
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return k;
}

// canonical state digest mix (identical definition in oracle/swim_oracle.c or_digest)
__host__ __device__ inline uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return k;
}
__host__ __device__ inline uint64_t mix4(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
    return fmix64(a * 0x9E3779B97F4A7C15ULL ^
                  fmix64(b * 0xC2B2AE3D27D4EB4FULL ^ fmix64(c * 0x165667B19E3779F9ULL ^ fmix64(d + 0xD6E8FEB86659FD93ULL))));
}

}  // namespace swimdev
