// swimsim_kernels.hip — gfx950 kernels of the SWIM protocol-round engine.
//
// Every kernel restates one phase of docs/ROUND_SEMANTICS.md. The reference functions they
// replace are cited at each kernel (maniacs-ops/ringpop-go, package swim/). There is no MFMA:
// nothing on this path is a dense contraction. The design is one 64-lane wave per observer
// row for merges and buffer scans (the changes in one message are distinct members, so lanes
// never conflict), and one lane per row for the FarmHash chain (it is sequential within a row).
#include "swimsim_kernels.h"

namespace swimdev {

// ---- wave scans and reductions on DPP (GFX9 data-parallel moves: shifts within a row of 16 lanes, then the rows'
// last lanes broadcast to the rows after them) instead of ds_bpermute, whose every step is an LDS crossbar round trip:
// six VALU steps for a 64-lane inclusive scan. Callers run them with every lane of the wave active. ----
#define SWIM_DPP(old, src, ctrl, rm) ((uint32_t)__builtin_amdgcn_update_dpp((int)(old), (int)(src), (ctrl), (rm), 0xf, false))
template <typename Op>
__device__ __forceinline__ uint32_t dpp_scan(uint32_t x, uint32_t id, Op op) {
    x = op(x, SWIM_DPP(id, x, 0x111, 0xf));                     // row_shr:1
    x = op(x, SWIM_DPP(id, x, 0x112, 0xf));                     // row_shr:2
    x = op(x, SWIM_DPP(id, x, 0x114, 0xf));                     // row_shr:4
    x = op(x, SWIM_DPP(id, x, 0x118, 0xf));                     // row_shr:8
    x = op(x, SWIM_DPP(id, x, 0x142, 0xa));                     // row_bcast:15 into rows 1 and 3
    x = op(x, SWIM_DPP(id, x, 0x143, 0xc));                     // row_bcast:31 into rows 2 and 3
    return x;
}
__device__ __forceinline__ uint32_t dpp_scan_add(uint32_t x) { return dpp_scan(x, 0u, [](uint32_t a, uint32_t b) { return a + b; }); }
__device__ __forceinline__ uint32_t dpp_scan_umin(uint32_t x) {
    return dpp_scan(x, 0xFFFFFFFFu, [](uint32_t a, uint32_t b) { return min(a, b); });
}
__device__ __forceinline__ int32_t dpp_scan_imax(int32_t x) {
    return (int32_t)dpp_scan((uint32_t)x, 0x80000000u, [](uint32_t a, uint32_t b) { return (uint32_t)max((int32_t)a, (int32_t)b); });
}
__device__ __forceinline__ int32_t dpp_scan_imin(int32_t x) {
    return (int32_t)dpp_scan((uint32_t)x, 0x7FFFFFFFu, [](uint32_t a, uint32_t b) { return (uint32_t)min((int32_t)a, (int32_t)b); });
}
__device__ __forceinline__ uint32_t dpp_scan_or(uint32_t x) { return dpp_scan(x, 0u, [](uint32_t a, uint32_t b) { return a | b; }); }
__device__ __forceinline__ uint32_t lane63(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); }
// lane i gets lane i - 1's value (lane 0: id)
__device__ __forceinline__ uint32_t dpp_shr1(uint32_t x, uint32_t id) { return SWIM_DPP(id, x, 0x138, 0xf); }   // wave_shr:1

__device__ __forceinline__ int wsum(int v) { return (int)lane63(dpp_scan_add((uint32_t)v)); }
__device__ __forceinline__ uint32_t wmin(uint32_t v) { return lane63(dpp_scan_umin(v)); }
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ uint32_t wave_gid() { return (blockIdx.x * blockDim.x + threadIdx.x) >> 6; }
__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

__device__ __forceinline__ unsigned long long bcast64(unsigned long long v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 0);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 0);
    return ((unsigned long long)hi << 32) | lo;
}
// the wave's sum of a 64-bit value, as three 32-bit DPP sums (the low word in 16-bit halves: no carry is lost)
__device__ __forceinline__ unsigned long long wsum64(unsigned long long v) {
    const uint32_t a = lane63(dpp_scan_add((uint32_t)v & 0xFFFFu)), b = lane63(dpp_scan_add((uint32_t)v >> 16));
    const uint32_t c = lane63(dpp_scan_add((uint32_t)(v >> 32)));
    return ((unsigned long long)c << 32) + ((unsigned long long)b << 16) + (unsigned long long)a;
}

// protocol counters: CTR_SHARDS copies on separate lines, picked by workgroup, summed at read-back
// (one shared word saturates at ~88 atomics/us, MI355X_MICROARCH.md row "dequeue")
__device__ __forceinline__ void ctr_add(const DS &d, int c, unsigned long long v) {
    atomicAdd(&d.ctr[(size_t)(blockIdx.x & (CTR_SHARDS - 1)) * CTR_STRIDE + c], v);
}

__device__ __forceinline__ uint32_t timeout_rounds(const DS &d, uint32_t st) {
    return st == ST_SUSPECT ? d.to_susp : st == ST_FAULTY ? d.to_faulty : d.to_tomb;
}

__device__ __forceinline__ bool reach(const DS &d, uint32_t a, uint32_t b) {
    return d.live[a] && d.live[b] && d.part[a] == d.part[b];
}

// ---------------------------------------------------------------------------------------------
// memberlist.Update for one change (memberlist.go:310-390, Apply 418-449) + handleChanges per
// applied change (node.go:424-447: RecordChange, timer schedule/cancel). Row totals are folded
// by wave_finalize (AdjustMaxPropagations, disseminator.go:75-97).
// ---------------------------------------------------------------------------------------------
struct MAcc {
    int dping, ddc, napp, nref, nproc, evict, dlen, maxlast, inval;
    int dnh;                  // entries created for members without a hot slot (d.nhe)
    unsigned long long dfp;   // row fingerprint delta
    unsigned long long tag;   // Update tag of the per-Update event stream (d.useq of the row at the Update's start)
    __device__ MAcc() : dping(0), ddc(0), napp(0), nref(0), nproc(0), evict(0), dlen(0), maxlast(-1), inval(0), dnh(0),
                        dfp(0), tag(0) {}
};

// start of one Update on row ol: its changes carry the row's current sequence number (event stream only)
__device__ __forceinline__ void acc_begin(const DS &d, uint32_t ol, MAcc &acc) {
    if (d.useq) acc.tag = d.useq[ol];
}

// bytes of one member's checksum record addr ‖ status ‖ decimal(inc) ‖ ';' (memberlist.go:115-121);
// tombstones and unknown members contribute nothing (memberlist.go:112-114)
__device__ __forceinline__ int reclen(const DS &d, uint32_t st, uint32_t e) {
    if (st >= 4u) return 0;
    uint32_t dl = d.dig_d0;
#pragma unroll
    for (int k = 0; k < 8; k++) dl += e >= d.dig_thr[k] ? 1u : 0u;
    return (int)(d.W + 5u + (st == ST_SUSPECT ? 2u : 0u) + (st == ST_FAULTY ? 1u : 0u) + dl + 1u);
}

// keep the per-row checksum-string length and last included member current (the FarmHash
// prologue needs both before the chain starts)
__device__ __forceinline__ void track_len(const DS &d, uint32_t ol, uint32_t m, uint32_t old_w, uint32_t new_w, MAcc &acc) {
    const uint32_t os = old_w & 7u, ns = new_w & 7u;
    acc.dlen += reclen(d, ns, new_w >> 3) - reclen(d, os, old_w >> 3);
    if (ns < 4u) acc.maxlast = max(acc.maxlast, (int)m);
    else if (os < 4u && (int)m == d.clast[ol]) acc.inval = 1;
}

// a row word of member m changes: its column may now differ between rows (DS::colx; a relaxed test first, the bit is
// set once per column and epoch)
__device__ __forceinline__ void colmark(const DS &d, uint32_t m) {
    uint32_t *w = d.colx + (m >> 5);
    const uint32_t bit = 1u << (m & 31);
    if (!(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(w, bit);
}

// cur = the row word d.mw[ol][m] (callers batch these loads), hk_in = m's hot slot (SRC_NONE: none; HK_LAZY: looked up
// here, only when the change applies)
constexpr uint32_t HK_LAZY = 0xFFFFFFFEu;
__device__ __forceinline__ void merge_change_w(const DS &d, uint32_t ol, uint32_t o, uint32_t m, uint32_t cur, uint32_t cst,
                                               uint32_t ce, uint32_t csrc, uint32_t csinc, uint32_t now_e, uint32_t sched_r,
                                               MAcc &acc, uint32_t hk_in = HK_LAZY) {
    const size_t idx = (size_t)ol * d.NP + m;
    const uint32_t cur_st = cur & 7u;
    uint32_t nst, ne, nsrc, nsinc;
    acc.nproc++;
    if (cur_st == ST_UNKNOWN) {                                    // memberlist.go:329-334
        if (cst == ST_TOMB) return;                                // memberlist.go:424-426
        nst = cst; ne = ce; nsrc = csrc; nsinc = csinc;
    } else if (m == o && ce >= (cur >> 3) && (cst == ST_SUSPECT || cst == ST_FAULTY || cst == ST_TOMB)) {
        nst = ST_ALIVE; ne = now_e; nsrc = o; nsinc = now_e;       // refute: memberlist.go:337-354
        acc.nref++;
    } else if (((ce << 3) | cst) > cur) {                          // nonLocalOverride: member.go:79-93
        nst = cst; ne = ce; nsrc = csrc; nsinc = csinc;
    } else {
        return;
    }
    const uint32_t nw_ = (ne << 3) | nst;
    const uint32_t hk = hk_in == HK_LAZY ? hot_slot(d, m) : hk_in;
    const size_t hx = (size_t)ol * d.HP + hk;
    d.mw[idx] = nw_;
    if (hk != SRC_NONE) d.hmw[hx] = nw_;
    colmark(d, m);
    track_len(d, ol, m, cur, nw_, acc);
    acc.dfp += fpmix(m, (ne << 3) | nst) - fpmix(m, cur);
    if (m != o) acc.dping += (int)is_pingable(nst) - (int)is_pingable(cur_st);
    // RecordChange (disseminator.go:223-227): entry = {p 0, source, source incarnation}
    if (de_p(hk != SRC_NONE ? d.hde[hx].x : d.dent[idx].x) == DP_NONE) {   // hot: the slot's cell is the entry
        acc.ddc++;
        atomicOr(&d.dbit[(size_t)ol * d.NBIT + (m >> 5)], 1u << (m & 31));
        if (hk == SRC_NONE) acc.dnh++;
        if (hk == SRC_NONE && d.hidx) {                           // a candidate for the next round's hot columns
            uint32_t *hw = d.hotnew + (m >> 5);
            if (!(__hip_atomic_load(hw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & (1u << (m & 31))))
                atomicOr(hw, 1u << (m & 31));
        }
    }
    const uint2 cell = make_uint2(de_x(nsrc, 0), nsinc);
    if (hk != SRC_NONE) d.hde[hx] = cell;
    else d.dent[idx] = cell;
    if (d.wslot) {                                                 // watched row: MemberlistChangesAppliedEvent
        const uint32_t ws = d.wslot[ol];                           // (memberlist.go:378-383)
        if (ws != SRC_NONE) {
            d.wlog[(size_t)ws * d.NP + m] = make_uint4(nw_, nsrc, nsinc, 1u);
            if ((d.wev_mask >> ws) & 1ull) {                       // per-Update stream: append in apply order
                const uint32_t at = atomicAdd(d.wev_cnt + ws, 1u);
                if (at < d.wev_cap) {
                    d.wevs[ws][at] = make_uint4(m, nw_, nsrc, nsinc);
                    d.wevts[ws][at] = acc.tag;
                }
            }
        }
    }
    if (m != o) {                                                  // no timers for the local member
        const uint8_t ts = d.tst[idx];
        const uint32_t tstate = ts & 7u;
        if (nst == ST_ALIVE || nst == ST_LEAVE) {
            if (ts) d.tst[idx] = 0;                                // Cancel (state_transitions.go:163-176)
        } else if (tstate != nst) {                                // same state: no-op (130-136)
            const uint32_t dl = sched_r + timeout_rounds(d, nst);
            d.tst[idx] = (uint8_t)nst;
            d.tmr[idx] = make_uint2(dl, ne);                       // subject = the applied change
            atomicMin(&d.tblk[(size_t)ol * d.NB + (m >> 6)], dl);
            atomicMin(&d.tmin[ol], dl);
        }
    }
    acc.napp++;
}

__device__ __forceinline__ void merge_change(const DS &d, uint32_t ol, uint32_t o, uint32_t m, uint32_t cst, uint32_t ce,
                                             uint32_t csrc, uint32_t csinc, uint32_t now_e, uint32_t sched_r, MAcc &acc) {
    merge_change_w(d, ol, o, m, d.mw[(size_t)ol * d.NP + m], cst, ce, csrc, csinc, now_e, sched_r, acc);
}

__device__ __forceinline__ void fold_row(const DS &d, uint32_t ol, int dping, int ddc, int napp, int nref, int evict,
                                         int dlen, int maxlast, int inval, unsigned long long dfp, bool next_update = true,
                                         int dnh = 0) {
    if (!(dnh | dping | ddc | napp | evict | dlen | inval) && !dfp && maxlast <= -1 && !nref) return;
    // every read first, then the writes: one memory round trip per Update instead of one per field (each
    // read-modify-write of a row field below would otherwise wait for its own load)
    const int nhe0 = d.nhe[ol], ping0 = d.ping[ol], dcnt0 = d.dcnt[ol], clast0 = d.clast[ol];
    const unsigned long long fp0 = d.fp[ol];
    const uint32_t clen0 = d.clen[ol];
    const unsigned long long useq0 = d.useq ? d.useq[ol] : 0ull;
    if (napp && next_update && d.useq) d.useq[ol] = useq0 + 1ull;  // the next Update of this row takes the next tag
    if (dnh) d.nhe[ol] = nhe0 + dnh;
    if (dfp) d.fp[ol] = fp0 + dfp;
    const int ping1 = ping0 + dping;
    if (dping) d.ping[ol] = ping1;
    if (ddc) d.dcnt[ol] = dcnt0 + ddc;
    if (napp) {
        d.maxp[ol] = (int32_t)d.pfactor * digits10(ping1);          // AdjustMaxPropagations
        ctr_add(d, C_APPLIED, (unsigned long long)napp);
    }
    if (napp || evict) d.dirty[ol] = 1;                            // ComputeChecksum pending
    if (dlen) d.clen[ol] = clen0 + (uint32_t)dlen;
    if (maxlast > clast0) d.clast[ol] = maxlast;
    else if (inval) d.clast[ol] = -2;                              // rescanned by the checksum kernel
    if (nref) ctr_add(d, C_REFUTES, (unsigned long long)nref);
}

__device__ __forceinline__ int wmax(int v) { return (int)lane63((uint32_t)dpp_scan_imax(v)); }

__device__ __forceinline__ void wave_finalize(const DS &d, uint32_t ol, const MAcc &acc, int cset = 0, bool next_update = true) {
    const int dping = wsum(acc.dping), ddc = wsum(acc.ddc), napp = wsum(acc.napp), nref = wsum(acc.nref);
    const int ev = wsum(acc.evict), np = wsum(acc.nproc), dl = wsum(acc.dlen), ml = wmax(acc.maxlast);
    const int inv = wmax(acc.inval), dnh = wsum(acc.dnh);
    const unsigned long long dfp = wsum64(acc.dfp);
    if (lane_id() == 0) {
        fold_row(d, ol, dping, ddc, napp, nref, ev, dl, ml, inv, dfp, next_update, dnh);
        if (np && cset < 2) ctr_add(d, cset ? C_X_MERGED_R : C_X_MERGED, (unsigned long long)np);
        if (napp && cset < 2) ctr_add(d, cset ? C_X_APPLIED_R : C_X_APPLIED, (unsigned long long)napp);
        if (napp && cset == 3) ctr_add(d, C_X_JOBS_APPLIED, (unsigned long long)napp);
    }
    __threadfence_block();
}

// The row scalars of observer row ol while one wave runs the row's Updates (a receiver's wave in k_recv, a sender's in
// k_resp: no other wave writes them during the launch). They are loaded once, together with the first message's
// records, kept current in registers and written back as they change, so an Update's epilogue (fold_row's reads),
// IssueAsReceiver's count, maxP and cold-entry test and the full-sync branch's dirty / checksum reads cost no round
// trip of their own (round 6: each was a dependent load on every message's path).
struct RowPre {
    int32_t nhe, ping, dcnt, clast, maxp;
    uint32_t clen, dirty, cs, cpslot;
    unsigned long long fp, useq;
    uint32_t ulog;                    // entries logged in d.ulog this phase (k_recv)
};
// (wave-uniform by construction: readfirstlane tells the compiler so, and the copy lives in scalar registers instead of
// 13 vector registers that k_recv's merge and issue loops would otherwise spill)
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ unsigned long long uni64(unsigned long long x) {
    return ((unsigned long long)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}
__device__ __forceinline__ RowPre row_pre(const DS &d, uint32_t ol) {
    RowPre p;
    p.nhe = (int32_t)uni((uint32_t)d.nhe[ol]); p.ping = (int32_t)uni((uint32_t)d.ping[ol]);
    p.dcnt = (int32_t)uni((uint32_t)d.dcnt[ol]); p.clast = (int32_t)uni((uint32_t)d.clast[ol]);
    p.maxp = (int32_t)uni((uint32_t)d.maxp[ol]);
    p.clen = uni(d.clen[ol]); p.dirty = uni(d.dirty[ol]); p.cs = uni(d.cs[ol]); p.cpslot = uni(d.cpslot[ol]);
    p.fp = uni64(d.fp[ol]);
    p.useq = d.useq ? uni64(d.useq[ol]) : 0ull;
    p.ulog = 0;
    return p;
}

// fold_row on the registers (every lane computes the same values; lane 0 writes what changed)
__device__ __forceinline__ void fold_row_pre(const DS &d, uint32_t ol, RowPre &p, int dping, int ddc, int napp, int nref,
                                             int evict, int dlen, int maxlast, int inval, unsigned long long dfp, int dnh) {
    if (!(dnh | dping | ddc | napp | evict | dlen | inval) && !dfp && maxlast <= -1 && !nref) return;
    const bool l0 = lane_id() == 0;
    if (napp && d.useq) { p.useq += 1ull; if (l0) d.useq[ol] = p.useq; }
    if (dnh) { p.nhe += dnh; if (l0) d.nhe[ol] = p.nhe; }
    if (dfp) { p.fp += dfp; if (l0) d.fp[ol] = p.fp; }
    if (dping) { p.ping += dping; if (l0) d.ping[ol] = p.ping; }
    if (ddc) { p.dcnt += ddc; if (l0) d.dcnt[ol] = p.dcnt; }
    if (napp) {
        p.maxp = (int32_t)d.pfactor * digits10(p.ping);            // AdjustMaxPropagations
        if (l0) { d.maxp[ol] = p.maxp; ctr_add(d, C_APPLIED, (unsigned long long)napp); }
    }
    if (napp || evict) { p.dirty = 1; if (l0) d.dirty[ol] = 1; }  // ComputeChecksum pending
    if (dlen) { p.clen += (uint32_t)dlen; if (l0) d.clen[ol] = p.clen; }
    if (maxlast > p.clast) { p.clast = maxlast; if (l0) d.clast[ol] = maxlast; }
    else if (inval) { p.clast = -2; if (l0) d.clast[ol] = -2; }   // rescanned by the checksum kernel
    if (nref && l0) ctr_add(d, C_REFUTES, (unsigned long long)nref);
}

__device__ __forceinline__ void wave_finalize_pre(const DS &d, uint32_t ol, const MAcc &acc, int cset, RowPre &p) {
    const int dping = wsum(acc.dping), ddc = wsum(acc.ddc), napp = wsum(acc.napp), nref = wsum(acc.nref);
    const int ev = wsum(acc.evict), np = wsum(acc.nproc), dl = wsum(acc.dlen), ml = wmax(acc.maxlast);
    const int inv = wmax(acc.inval), dnh = wsum(acc.dnh);
    const unsigned long long dfp = wsum64(acc.dfp);
    fold_row_pre(d, ol, p, dping, ddc, napp, nref, ev, dl, ml, inv, dfp, dnh);
    if (lane_id() == 0) {
        if (np && cset < 2) ctr_add(d, cset ? C_X_MERGED_R : C_X_MERGED, (unsigned long long)np);
        if (napp && cset < 2) ctr_add(d, cset ? C_X_APPLIED_R : C_X_APPLIED, (unsigned long long)napp);
        if (napp && cset == 3) ctr_add(d, C_X_JOBS_APPLIED, (unsigned long long)napp);
    }
    __threadfence_block();
}

// Batched gathers: the loops below issue MB independent loads per lane before using any of them (a
// message's changes are distinct members, so no load of a batch depends on a store of the same batch).
constexpr int MB = 4;
constexpr int SNAP_MB = 8;             // row copies (snapshots): 16-B loads in flight per lane

// one wave copies n 16-B items, SNAP_MB loads in flight per lane (a loop of load-then-store waits for each load: one
// HBM round trip per 1 KB)
__device__ __forceinline__ void wave_copy16(uint4 *dst, const uint4 *src, uint32_t n) {
    for (uint32_t i = lane_id(); i < n; i += 64 * SNAP_MB) {
        uint4 v[SNAP_MB];
#pragma unroll
        for (int u = 0; u < SNAP_MB; u++)
            if (i + 64u * u < n) v[u] = src[i + 64u * u];
#pragma unroll
        for (int u = 0; u < SNAP_MB; u++)
            if (i + 64u * u < n) dst[i + 64u * u] = v[u];
    }
}

// a dense message (MembershipAsChanges: full sync, reverse full sync, heal) streams the whole row. (Kept
// inline: an out-of-line call makes every launch copy the DS argument block to scratch, 480 B per lane.)
__device__ __forceinline__ void wave_merge_dense(const DS &d, uint32_t ol, uint32_t o, const MsgDesc &md,
                                                           uint32_t now_e, uint32_t sched_r, MAcc &acc) {
    const uint32_t *rowp = d.mw + (size_t)ol * d.NP;
    const uint32_t slot = md.off_lo;
    const uint4 meta = d.dense_meta[slot];
    const uint32_t *snap = d.dense + (size_t)slot * d.NP;
    for (uint32_t base = 0; base < d.N; base += 64 * MB) {
        uint32_t w[MB], cur[MB];
#pragma unroll
        for (int u = 0; u < MB; u++) {
            const uint32_t m = base + u * 64 + lane_id();
            w[u] = m < d.N ? snap[m] : ST_UNKNOWN;
            cur[u] = m < d.N ? rowp[m] : 0u;
        }
#pragma unroll
        for (int u = 0; u < MB; u++) {
            const uint32_t m = base + u * 64 + lane_id();
            if ((w[u] & 7u) != ST_UNKNOWN)
                merge_change_w(d, ol, o, m, cur[u], w[u] & 7u, w[u] >> 3, meta.x, meta.y, now_e, sched_r, acc);
        }
    }
}

// merge a whole message into row ol (wave-wide; the changes of one message are distinct members)
// the first MB records per lane of a sparse message, loaded ahead (k_resp issues them with the bump's loads)
__device__ __forceinline__ void merge_first(const DS &d, const MsgDesc &md, uint4 (&rec)[MB]) {
    const unsigned long long off = ((unsigned long long)md.off_hi << 32) | md.off_lo;
#pragma unroll
    for (int u = 0; u < MB; u++) {
        const uint32_t i = u * 64 + lane_id();
        rec[u] = md.kind == 0 && i < md.len ? d.pool[off + i] : make_uint4(0xFFFFFFFFu, 0, 0, 0);
    }
}
// (dctr >= 0: the measurement counter a dense message adds one to; pre0: the first batch from merge_first, or null;
// ulog: the receive phase's undo log position of this row (k_recv), or null)
__device__ __forceinline__ void wave_merge_body(const DS &d, uint32_t ol, uint32_t o, const MsgDesc &md, uint32_t now_e,
                                                uint32_t sched_r, MAcc &acc, int dctr, const uint4 *pre0 = nullptr,
                                                uint32_t *ulog = nullptr) {
    const uint32_t *rowp = d.mw + (size_t)ol * d.NP;
    const uint32_t *hrow = d.hmw + (size_t)ol * d.HP;
    if (md.kind == 0) {
        const unsigned long long off = ((unsigned long long)md.off_hi << 32) | md.off_lo;
        for (uint32_t base = 0; base < md.len; base += 64 * MB) {
            uint4 rec[MB];
            uint32_t cur[MB], hk[MB];
#pragma unroll
            for (int u = 0; u < MB; u++) {
                const uint32_t i = base + u * 64 + lane_id();
                rec[u] = pre0 && base == 0 ? pre0[u] : i < md.len ? d.pool[off + i] : make_uint4(0xFFFFFFFFu, 0, 0, 0);
            }
            // (the record's tag names the member's hot slot: the row word is the second load of the chain, not the
            // third after an hidx lookup)
#pragma unroll
            for (int u = 0; u < MB; u++) hk[u] = rec[u].x != 0xFFFFFFFFu ? rec_slot(d, rec[u]) : SRC_NONE;
#pragma unroll
            for (int u = 0; u < MB; u++)
                cur[u] = rec[u].x == 0xFFFFFFFFu ? 0u : hk[u] != SRC_NONE ? hrow[hk[u]] : rowp[rec_m(rec[u])];
#pragma unroll
            for (int u = 0; u < MB; u++) {
                const int before = acc.napp;
                if (rec[u].x != 0xFFFFFFFFu)
                    merge_change_w(d, ol, o, rec_m(rec[u]), cur[u], rec_st(rec[u]), rec_e(rec[u]), rec[u].z, rec[u].w, now_e,
                                   sched_r, acc, hk[u]);
                if (ulog) {                                        // the overwritten word, in apply order
                    const bool ap = acc.napp != before;
                    const unsigned long long b = __ballot(ap);
                    const uint32_t at = *ulog + (uint32_t)__popcll(b & lanemask_lt());
                    if (ap && at < ULOG_CAP) d.ulog[(size_t)ol * ULOG_CAP + at] = make_uint2(rec_m(rec[u]), cur[u]);
                    *ulog += (uint32_t)__popcll(b);
                }
            }
        }
    } else if (md.kind == 1) {
        wave_merge_dense(d, ol, o, md, now_e, sched_r, acc);
        if (dctr >= 0 && lane_id() == 0) ctr_add(d, dctr, 1ull);
        if (ulog) *ulog = ULOG_CAP + 1u;                           // (not logged: the row's issue-time words are lost)
    }
    __threadfence_block();
}
// cset selects the measurement counters (0: k_recv's C_X_MERGED/C_X_APPLIED, 1: k_resp's pair, 2: none, 3: the reverse
// full syncs' C_X_JOBS_APPLIED)
__device__ void wave_merge_msg(const DS &d, uint32_t ol, uint32_t o, const MsgDesc &md, uint32_t now_e, uint32_t sched_r,
                               int cset = 0, int dctr = -1) {
    MAcc acc;
    acc_begin(d, ol, acc);
    wave_merge_body(d, ol, o, md, now_e, sched_r, acc, dctr);
    wave_finalize(d, ol, acc, cset);
}
// the same on a wave's register copy of the row scalars (RowPre)
__device__ __forceinline__ void wave_merge_msg_pre(const DS &d, uint32_t ol, uint32_t o, const MsgDesc &md, uint32_t now_e,
                                                   uint32_t sched_r, int cset, RowPre &p, int dctr = -1,
                                                   const uint4 *pre0 = nullptr, bool logit = false) {
    MAcc acc;
    acc.tag = p.useq;
    wave_merge_body(d, ol, o, md, now_e, sched_r, acc, dctr, pre0, logit && d.ulog ? &p.ulog : nullptr);
    wave_finalize_pre(d, ol, acc, cset, p);
}

// bumpPiggybackCounters over a sparse list (disseminator.go:135-149); returns the wave's deleted entries (all, and those
// of members without a hot slot) for the caller to fold into the row's counts
__device__ __forceinline__ int2 wave_bump_body(const DS &d, uint32_t ol, const MsgDesc &md, int maxp) {
    if (md.kind != 0) return make_int2(0, 0);
    const unsigned long long off = ((unsigned long long)md.off_hi << 32) | md.off_lo;
    uint32_t *dx = (uint32_t *)(d.dent + (size_t)ol * d.NP);       // word 0 of each entry, stride 2
    uint32_t *hx = (uint32_t *)(d.hde + (size_t)ol * d.HP);        // the same in the hot columns
    int del = 0, delnh = 0;
    for (uint32_t base = 0; base < md.len; base += 64 * MB) {
        uint32_t m[MB], x[MB], hk[MB];
#pragma unroll
        for (int u = 0; u < MB; u++) {
            const uint32_t i = base + u * 64 + lane_id();
            const uint2 xy = i < md.len ? *(const uint2 *)(d.pool + off + i) : make_uint2(0xFFFFFFFFu, 0u);
            const uint4 r = make_uint4(xy.x, xy.y, 0u, 0u);
            m[u] = xy.x != 0xFFFFFFFFu ? rec_m(r) : 0xFFFFFFFFu;
            hk[u] = xy.x != 0xFFFFFFFFu ? rec_slot(d, r) : SRC_NONE;    // (the record's tag: no hidx lookup)
        }
#pragma unroll
        for (int u = 0; u < MB; u++)
            x[u] = m[u] == 0xFFFFFFFFu ? DE_NONE : hk[u] != SRC_NONE ? hx[(size_t)hk[u] * 2] : dx[(size_t)m[u] * 2];
#pragma unroll
        for (int u = 0; u < MB; u++) {
            const uint32_t p = de_p(x[u]);
            if (p == DP_NONE) continue;
            uint32_t nx;
            if ((int)(p + 1) >= maxp) {
                nx = x[u] | 0xFF000000u;
                atomicAnd(&d.dbit[(size_t)ol * d.NBIT + (m[u] >> 5)], ~(1u << (m[u] & 31)));
                del++;
                delnh += hk[u] == SRC_NONE;
            } else {
                nx = x[u] + (1u << 24);
            }
            if (hk[u] != SRC_NONE) hx[(size_t)hk[u] * 2] = nx;
            else dx[(size_t)m[u] * 2] = nx;
        }
    }
    return make_int2(wsum(del), wsum(delnh));
}
__device__ void wave_bump(const DS &d, uint32_t ol, const MsgDesc &md) {
    if (md.kind != 0) return;
    const int2 dd = wave_bump_body(d, ol, md, d.maxp[ol]);
    if (lane_id() == 0 && dd.x) d.dcnt[ol] -= dd.x;
    if (lane_id() == 0 && dd.y) d.nhe[ol] -= dd.y;
    __threadfence_block();
}
__device__ __forceinline__ void wave_bump_pre(const DS &d, uint32_t ol, const MsgDesc &md, RowPre &p) {
    if (md.kind != 0) return;
    const int2 dd = wave_bump_body(d, ol, md, p.maxp);
    if (dd.x) { p.dcnt -= dd.x; if (lane_id() == 0) d.dcnt[ol] = p.dcnt; }
    if (dd.y) { p.nhe -= dd.y; if (lane_id() == 0) d.nhe[ol] = p.nhe; }
    __threadfence_block();
}

// The message pool is split into POOL_SHARDS sub-pools with a cursor each (own 128-B line): one returning
// atomic per issuing wave on a single word saturates at ~88 per us (MI355X_MICROARCH.md row "dequeue"), which
// serialised the 65,536 issues of a cascade round. A wave starts at the sub-pool of its wave id and moves on
// to the next one only when its records do not fit, so the pool fails only when every sub-pool is full. A
// sub-pool's cursor only moves when the records fit (compare-and-swap), so a failed attempt strands no space;
// swimsim_create requires every sub-pool to hold N records, the longest message. (A fetch-add instead, one round trip
// fewer, stranded each overflowing attempt's sub-pool tail: config 4's heal messages then overflowed a sharded pool.
// k_recv hides the allocation's round trips behind its merge instead, recv_one_pre.)
// Messages of at most sub / 256 records take one fetch-add instead (one round trip instead of two): an attempt that
// overflows leaves the cursor past its sub-pool's end, which strands less than sub / 256 records of that sub-pool, once.
__device__ __forceinline__ unsigned long long pool_alloc_lane0(const DS &d, uint32_t n) {
    const unsigned long long sub = d.pool_cap / POOL_SHARDS;
    const bool small = n <= sub / 256;
    for (uint32_t t = 0, s = wave_gid() % POOL_SHARDS; t < POOL_SHARDS; t++, s = (s + 1) % POOL_SHARDS) {
        unsigned long long *cur = d.pool_cur + (size_t)s * POOL_CUR_STRIDE;
        if (small) {
            const unsigned long long old = atomicAdd(cur, (unsigned long long)n);
            if (old + n <= sub) return s * sub + old;
            continue;
        }
        unsigned long long old = __hip_atomic_load(cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (old + n <= sub) {
            const unsigned long long seen = atomicCAS(cur, old, old + n);
            if (seen == old) return s * sub + old;
            old = seen;
        }
    }
    atomicOr(d.err, E_POOL);
    return ~0ull;
}
__device__ __forceinline__ unsigned long long pool_alloc(const DS &d, uint32_t n) {
    unsigned long long off = 0;
    if (lane_id() == 0 && n) off = pool_alloc_lane0(d, n);
    return bcast64(off);
}

__device__ __forceinline__ uint32_t wscan_excl(uint32_t v, uint32_t &total) {
    const uint32_t x = dpp_scan_add(v);
    total = lane63(x);
    return x - v;
}

// The dissemination buffer of row ol from its presence bitmap: each lane owns 4 bitmap words (128
// members) per pass and walks its set bits MB at a time, so every gather of a pass is independent
// of the others; a wave prefix sum places the records. Bitmap words are read through L2 (sc1):
// merges set bits with atomics. RECV = IssueAsReceiver (disseminator.go:156-199): drop entries from
// (sender, sinc), bump the rest (p++, delete at maxP). Otherwise IssueAsSender
// (disseminator.go:128-133,201-215). Records are in member order within a lane's range; the order of
// a message does not matter (its changes are distinct members).
// (the body: cnt entries, maxP, the walk, the slots in use and the pool offset of cnt records are the caller's;
// returns the records written, and for RECV the deleted entries in del / delnh, wave sums)
template <bool RECV>
__device__ __forceinline__ uint32_t wave_issue_body(const DS &d, uint32_t ol, uint32_t sender, uint32_t sinc, MsgDesc &out,
                                                    uint32_t cnt, int maxp, bool hotwalk, uint32_t nslots,
                                                    unsigned long long off, int &del_out, int &delnh_out) {
    const size_t rb = (size_t)ol * d.NP, hb = (size_t)ol * d.HP;
    uint32_t *bits = d.dbit + (size_t)ol * d.NBIT;
    uint32_t pos = 0;
    int del = 0, delnh = 0;
    if (hotwalk) {
        // every buffered member of this row has a hot slot: walk the row's slots in use (a few KB,
        // contiguous) instead of the presence bitmap (N/8 bytes) and the gathers it leads to. Records come out in
        // slot order; the order of a message does not matter (its changes are distinct members).
        for (uint32_t base = 0; base < nslots; base += 64 * MB) {
            uint2 ce[MB];
            uint32_t wv[MB], m[MB];
#pragma unroll
            for (int u = 0; u < MB; u++) {
                const uint32_t k = base + u * 64 + lane_id();
                ce[u] = k < nslots ? d.hde[hb + k] : make_uint2(DE_NONE, 0);
                wv[u] = k < nslots ? d.hmw[hb + k] : 0u;
                m[u] = k < nslots ? d.hlist[k] : 0u;
            }
            bool keep[MB];
            uint32_t nk = 0;
#pragma unroll
            for (int u = 0; u < MB; u++) {
                const uint32_t src = de_src(ce[u].x);
                keep[u] = de_p(ce[u].x) != DP_NONE && !(RECV && src == sender && ce[u].y == sinc);   // filterChangesFromSender
                nk += keep[u] ? 1u : 0u;
            }
            uint32_t tot;
            uint32_t at = pos + wscan_excl(nk, tot);
#pragma unroll
            for (int u = 0; u < MB; u++) {
                if (!keep[u]) continue;
                const uint32_t st = (wv[u] & 7u) == ST_UNKNOWN ? ST_TOMB : (wv[u] & 7u);   // evicted: (tombstone, inc)
                if (at < cnt) d.pool[off + at] = rec_make(m[u], st, wv[u] >> 3, de_src(ce[u].x), ce[u].y, base + u * 64 + lane_id() + 1u);
                at++;
                if (RECV) {                                                   // bump
                    const uint32_t k = base + u * 64 + lane_id();
                    uint32_t nx;
                    if ((int)(de_p(ce[u].x) + 1) >= maxp) {
                        nx = ce[u].x | 0xFF000000u;
                        atomicAnd(bits + (m[u] >> 5), ~(1u << (m[u] & 31)));
                        del++;
                    } else {
                        nx = ce[u].x + (1u << 24);
                    }
                    d.hde[hb + k].x = nx;
                }
            }
            pos += tot;
        }
    } else if ((uint64_t)cnt * 4u > d.NP) {
        // a long buffer (more than a quarter of the members: a partition's rows, config 4; churned rows, config 2): the
        // walk streams the row's cells and words (most sectors are touched anyway at that density) instead of
        // driving one gather per set presence bit; a member with a hot slot takes its cell and word from the slot
        // (the dense cell is stale while it holds one). Deletions clear their presence bits one ballot per word.
        const uint2 *dcell = d.dent + rb;
        const uint32_t *drow = d.mw + rb;
        for (uint32_t base = 0; base < d.NP; base += 64 * MB) {
            uint2 ce[MB];
            uint32_t wv[MB], hk[MB];
#pragma unroll
            for (int u = 0; u < MB; u++) {
                const uint32_t m = base + u * 64 + lane_id();
                const bool in = m < d.N;
                hk[u] = in && d.hidx ? d.hidx[m] : SRC_NONE;
                ce[u] = in ? dcell[m] : make_uint2(DE_NONE, 0);
                wv[u] = in ? drow[m] : 0u;
            }
#pragma unroll
            for (int u = 0; u < MB; u++)
                if (hk[u] != SRC_NONE) {
                    ce[u] = d.hde[hb + hk[u]];
                    wv[u] = d.hmw[hb + hk[u]];
                }
            bool keep[MB];
            uint32_t nk = 0;
#pragma unroll
            for (int u = 0; u < MB; u++) {
                keep[u] = de_p(ce[u].x) != DP_NONE &&
                          !(RECV && de_src(ce[u].x) == sender && ce[u].y == sinc);   // filterChangesFromSender
                nk += keep[u] ? 1u : 0u;
            }
            uint32_t tot;
            uint32_t at = pos + wscan_excl(nk, tot);
#pragma unroll
            for (int u = 0; u < MB; u++) {
                const uint32_t m = base + u * 64 + lane_id();
                bool gone = false;
                if (keep[u]) {
                    const uint32_t st = (wv[u] & 7u) == ST_UNKNOWN ? ST_TOMB : (wv[u] & 7u);   // evicted: (tombstone, inc)
                    if (at < cnt) d.pool[off + at] = rec_make(m, st, wv[u] >> 3, de_src(ce[u].x), ce[u].y, tag_of_slot(hk[u]));
                    at++;
                    if (RECV) {                                               // bump
                        uint32_t nx;
                        if ((int)(de_p(ce[u].x) + 1) >= maxp) {
                            nx = ce[u].x | 0xFF000000u;
                            gone = true;
                            del++;
                            delnh += hk[u] == SRC_NONE;
                        } else {
                            nx = ce[u].x + (1u << 24);
                        }
                        if (hk[u] != SRC_NONE) d.hde[hb + hk[u]].x = nx;
                        else d.dent[rb + m].x = nx;
                    }
                }
                if (RECV) {                                                   // (bits of members base + 64 u ..)
                    const unsigned long long g = __ballot(gone);
                    if (lane_id() == 0 && g) {
                        const uint32_t w0 = (base + u * 64) >> 5;
                        if ((uint32_t)g) atomicAnd(bits + w0, ~(uint32_t)g);
                        if (g >> 32) atomicAnd(bits + w0 + 1, ~(uint32_t)(g >> 32));
                    }
                }
            }
            pos += tot;
        }
    } else
    for (uint32_t q0 = 0; q0 < d.NBIT; q0 += 256) {
        const uint32_t q = q0 + lane_id() * 4;
        unsigned long long lo = 0, hi = 0;                       // the lane's 128 presence bits
        if (q < d.NBIT) {
            const uint32_t *bp = bits + q;
            const uint32_t w0 = __hip_atomic_load(bp + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t w1 = __hip_atomic_load(bp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t w2 = __hip_atomic_load(bp + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t w3 = __hip_atomic_load(bp + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lo = ((unsigned long long)w1 << 32) | w0;
            hi = ((unsigned long long)w3 << 32) | w2;
        }
        const uint32_t mbase = q * 32;
        unsigned long long dlo = 0, dhi = 0;                     // deleted entries (RECV)
        while (__any(lo != 0 || hi != 0)) {
            uint32_t m[MB];
#pragma unroll
            for (int k = 0; k < MB; k++) {
                if (lo) { m[k] = mbase + (uint32_t)(__ffsll((long long)lo) - 1); lo &= lo - 1; }
                else if (hi) { m[k] = mbase + 64 + (uint32_t)(__ffsll((long long)hi) - 1); hi &= hi - 1; }
                else m[k] = 0xFFFFFFFFu;
            }
            uint2 ce[MB];                                        // the 8-byte entry and the member word
            uint32_t wv[MB], hk[MB];
#pragma unroll
            for (int k = 0; k < MB; k++) hk[k] = m[k] != 0xFFFFFFFFu ? hot_slot(d, m[k]) : SRC_NONE;
#pragma unroll
            for (int k = 0; k < MB; k++) {
                if (m[k] == 0xFFFFFFFFu) {
                    ce[k] = make_uint2(DE_NONE, 0);
                    wv[k] = 0u;
                } else if (hk[k] != SRC_NONE) {
                    ce[k] = d.hde[hb + hk[k]];
                    wv[k] = d.hmw[hb + hk[k]];
                } else {
                    ce[k] = d.dent[rb + m[k]];
                    wv[k] = d.mw[rb + m[k]];
                }
            }
            uint32_t p[MB];
            uint2 sr[MB];
#pragma unroll
            for (int k = 0; k < MB; k++) {
                p[k] = de_p(ce[k].x);
                sr[k] = make_uint2(de_src(ce[k].x), ce[k].y);
            }
            bool keep[MB];
            uint32_t nk = 0;
#pragma unroll
            for (int k = 0; k < MB; k++) {
                keep[k] = m[k] != 0xFFFFFFFFu && !(RECV && sr[k].x == sender && sr[k].y == sinc);   // filterChangesFromSender
                nk += keep[k] ? 1u : 0u;
            }
            uint32_t tot;
            uint32_t at = pos + wscan_excl(nk, tot);
#pragma unroll
            for (int k = 0; k < MB; k++) {
                if (!keep[k]) continue;
                const uint32_t st = (wv[k] & 7u) == ST_UNKNOWN ? ST_TOMB : (wv[k] & 7u);   // evicted: (tombstone, inc)
                if (at < cnt) d.pool[off + at] = rec_make(m[k], st, wv[k] >> 3, sr[k].x, sr[k].y, tag_of_slot(hk[k]));
                at++;
                if (RECV) {                                                   // bump
                    uint32_t nx;
                    if ((int)(p[k] + 1) >= maxp) {
                        nx = ce[k].x | 0xFF000000u;
                        const uint32_t l = m[k] - mbase;
                        if (l < 64) dlo |= 1ull << l; else dhi |= 1ull << (l - 64);
                        del++;
                        delnh += hk[k] == SRC_NONE;
                    } else {
                        nx = ce[k].x + (1u << 24);
                    }
                    if (hk[k] != SRC_NONE) d.hde[hb + hk[k]].x = nx;
                    else d.dent[rb + m[k]].x = nx;
                }
            }
            pos += tot;
        }
        if (RECV && (dlo | dhi)) {                               // the lane's own words
            if (dlo & 0xFFFFFFFFull) atomicAnd(bits + q + 0, ~(uint32_t)dlo);
            if (dlo >> 32) atomicAnd(bits + q + 1, ~(uint32_t)(dlo >> 32));
            if (dhi & 0xFFFFFFFFull) atomicAnd(bits + q + 2, ~(uint32_t)dhi);
            if (dhi >> 32) atomicAnd(bits + q + 3, ~(uint32_t)(dhi >> 32));
        }
    }
    if (RECV) {
        del_out = wsum(del);
        delnh_out = wsum(delnh);
    } else if (pos != cnt && lane_id() == 0) {
        atomicOr(d.err, E_COUNT);
    }
    out.off_lo = (uint32_t)off;
    out.off_hi = (uint32_t)(off >> 32);
    out.len = min(pos, cnt);
    return out.len;
}

template <bool RECV>
__device__ uint32_t wave_issue_t(const DS &d, uint32_t ol, uint32_t sender, uint32_t sinc, MsgDesc &out) {
    // (the row's reads in one round trip, before the pool allocation's returning atomic)
    const uint32_t cnt = (uint32_t)d.dcnt[ol];
    const int maxp = RECV ? d.maxp[ol] : 0;
    const bool hotwalk = d.hidx && d.nhe[ol] == 0;
    const uint32_t nslots = d.hidx ? d.hot_cnt[0] : 0u;
    out.kind = 0; out.len = 0; out.off_lo = out.off_hi = 0;
    if (cnt == 0) return 0;
    const unsigned long long off = pool_alloc(d, cnt);
    if (off == ~0ull) return 0;
    int del = 0, delnh = 0;
    const uint32_t n = wave_issue_body<RECV>(d, ol, sender, sinc, out, cnt, maxp, hotwalk, nslots, off, del, delnh);
    if (RECV) {
        if (lane_id() == 0 && del) d.dcnt[ol] -= del;
        if (lane_id() == 0 && delnh) d.nhe[ol] -= delnh;
    }
    __threadfence_block();
    return n;
}

// issueChanges / IssueAsSender (disseminator.go:128-133,201-215): snapshot of every entry
__device__ void wave_issue(const DS &d, uint32_t ol, MsgDesc &out) { wave_issue_t<false>(d, ol, 0, 0, out); }

// IssueAsReceiver up to the full-sync decision (disseminator.go:156-199). Returns kept count.
__device__ uint32_t wave_issue_recv(const DS &d, uint32_t ol, uint32_t sender, uint32_t sinc, MsgDesc &out) {
    return wave_issue_t<true>(d, ol, sender, sinc, out);
}

// MembershipAsChanges (disseminator.go:107-123) as a dense snapshot of row ol
__device__ bool wave_snapshot(const DS &d, uint32_t ol, uint32_t o, MsgDesc &out) {
    uint32_t slot = 0;
    if (lane_id() == 0) slot = atomicAdd(d.dense_cur, 1u);
    slot = (uint32_t)__builtin_amdgcn_readlane((int)slot, 0);
    out.kind = 2; out.len = 0; out.off_lo = out.off_hi = 0;
    if (slot >= d.dense_cap) {
        if (lane_id() == 0) atomicOr(d.err, E_DENSE);
        return false;
    }
    const uint4 *src = (const uint4 *)(d.mw + (size_t)ol * d.NP);
    uint4 *dst = (uint4 *)(d.dense + (size_t)slot * d.NP);
    int known = 0;
    // (SNAP_MB loads in flight per lane: one at a time, each copy iteration waited for its load, 256 HBM round trips for
    // a 256-KB row, and the snapshotting senders' waves set k_issue's time: 0.4 ms a launch)
    const uint32_t n4 = d.NP / 4;
    for (uint32_t i = lane_id(); i < n4; i += 64 * SNAP_MB) {
        uint4 v[SNAP_MB];
#pragma unroll
        for (int u = 0; u < SNAP_MB; u++) v[u] = i + u * 64 < n4 ? src[i + u * 64] : make_uint4(ST_UNKNOWN, ST_UNKNOWN, ST_UNKNOWN, ST_UNKNOWN);
#pragma unroll
        for (int u = 0; u < SNAP_MB; u++) {
            if (i + u * 64 < n4) dst[i + u * 64] = v[u];
            known += ((v[u].x & 7u) != ST_UNKNOWN) + ((v[u].y & 7u) != ST_UNKNOWN) + ((v[u].z & 7u) != ST_UNKNOWN) +
                     ((v[u].w & 7u) != ST_UNKNOWN);
        }
    }
    known = wsum(known);
    if (lane_id() == 0) {
        d.dense_meta[slot] = make_uint4(o, d.mw[(size_t)ol * d.NP + o] >> 3, (uint32_t)known, 0);
        d.dense_len[slot] = d.clen[ol];
        d.dense_last[slot] = d.clast[ol];
    }
    out.kind = 1; out.off_lo = slot; out.len = (uint32_t)known;
    return true;
}

// ---------------------------------------------------------------------------------------------
// initialisation
// ---------------------------------------------------------------------------------------------
__global__ void k_init_rows(DS d, int mode, uint32_t e0) {
    const uint32_t ol = wave_gid();
    if (ol >= d.NL) return;
    const uint32_t o = d.lo + ol;
    unsigned long long fp = 0;
    for (uint32_t m = lane_id(); m < d.NP; m += 64) {
        const size_t idx = (size_t)ol * d.NP + m;
        uint32_t w = ST_UNKNOWN;
        if (m < d.N && (mode == 0 || m == o)) w = (e0 << 3) | ST_ALIVE;
        if (m < d.N) fp += fpmix(m, w);
        d.mw[idx] = w;
        d.dent[idx] = make_uint2(DE_NONE, 0);
        d.tst[idx] = 0;
        d.tmr[idx] = make_uint2(NO_DEADLINE, 0);
    }
    for (uint32_t b = lane_id(); b < d.NB; b += 64) d.tblk[(size_t)ol * d.NB + b] = NO_DEADLINE;
    for (uint32_t b = lane_id(); b < d.NBIT; b += 64) d.dbit[(size_t)ol * d.NBIT + b] = 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) fp += __shfl_xor(fp, off, 64);
    if (lane_id() == 0) {
        d.fp[ol] = fp;
        const int32_t p = mode == 0 ? (int32_t)d.N - 1 : 0;
        const uint32_t rl = (uint32_t)reclen(d, ST_ALIVE, e0);
        d.clen[ol] = mode == 0 ? rl * d.N : rl;
        d.clast[ol] = mode == 0 ? (int32_t)d.N - 1 : (int32_t)o;
        d.ping[ol] = p;
        d.maxp[ol] = mode == 0 ? (int32_t)d.pfactor * digits10(p) : (int32_t)d.pfactor;
        d.dcnt[ol] = 0;
        d.nhe[ol] = 0;
        d.dirty[ol] = 1;
        d.cs[ol] = 0;
        d.it_idx[ol] = -1;
        d.it_ep[ol] = 0;
        d.tmin[ol] = NO_DEADLINE;
        d.njobs[ol] = 0;
    }
}

// recount pingable/changes of one row after raw writes (NumPingableMembers, memberlist.go:188-198)
__global__ void k_recount(DS d, uint32_t ol) {
    const uint32_t o = d.lo + ol;
    int p = 0, c = 0, len = 0, last = -1;
    unsigned long long fp = 0;
    for (uint32_t m = lane_id(); m < d.N; m += 64) {
        const size_t idx = (size_t)ol * d.NP + m;
        const uint32_t w = d.mw[idx];
        fp += fpmix(m, w);
        if (m != o && is_pingable(w & 7u)) p++;
        if (de_p(d.dent[idx].x) != DP_NONE) c++;
        len += reclen(d, w & 7u, w >> 3);
        if ((w & 7u) < 4u) last = (int)m;
    }
    p = wsum(p);
    c = wsum(c);
    len = wsum(len);
    last = wmax(last);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) fp += __shfl_xor(fp, off, 64);
    if (lane_id() == 0) {
        d.ping[ol] = p; d.dcnt[ol] = c; d.dirty[ol] = 1; d.clen[ol] = (uint32_t)len; d.clast[ol] = last; d.fp[ol] = fp;
        d.nhe[ol] = c;                                             // raw writes drop every hot slot (hot_reset)
    }
}

__global__ void k_clear_changes(DS d, uint32_t ol) {
    for (uint32_t m = threadIdx.x; m < d.NP; m += blockDim.x) d.dent[(size_t)ol * d.NP + m].x = DE_NONE;
    if (d.hidx)
        for (uint32_t k = threadIdx.x; k < d.HP; k += blockDim.x) d.hde[(size_t)ol * d.HP + k].x = DE_NONE;
    for (uint32_t b = threadIdx.x; b < d.NBIT; b += blockDim.x) d.dbit[(size_t)ol * d.NBIT + b] = 0;
    if (threadIdx.x == 0) {
        d.dcnt[ol] = 0;
        d.nhe[ol] = 0;
    }
}

// hot columns were dropped (hot_reset): every entry of every row belongs to a member without a slot
__global__ void k_nhe_reset(DS d) {
    const uint32_t ol = blockIdx.x * blockDim.x + threadIdx.x;
    if (ol < d.NL) d.nhe[ol] = d.dcnt[ol];
}

// hot columns, start of phase I: members that got a first dissemination entry while not hot take free slots
// (one workgroup; hot_cnt[1] = the first new slot). Members beyond the HP slots stay on the dense path, so the
// hot set only grows; which members are hot changes no result (the columns are copies).
__global__ void __launch_bounds__(1024) k_hot_extend(DS d) {
    __shared__ uint32_t n;
    if (threadIdx.x == 0) {
        n = d.hot_cnt[0];
        d.hot_cnt[1] = n;
    }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < d.NBIT; w += blockDim.x) {
        uint32_t bits = d.hotnew[w];
        if (!bits) continue;
        d.hotnew[w] = 0;
        while (bits) {
            const uint32_t m = w * 32 + (uint32_t)(__ffs(bits) - 1);
            bits &= bits - 1;
            if (m >= d.N || d.hidx[m] != SRC_NONE) continue;
            const uint32_t k = atomicAdd(&n, 1u);
            if (k < d.HP) {
                d.hidx[m] = k;
                d.hlist[k] = m;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) d.hot_cnt[0] = min(n, d.HP);
}

// the columns of the slots k_hot_extend added, one wave per observer row
__global__ void k_hot_fill(DS d) {
    const uint32_t ol = wave_gid();
    if (ol >= d.NL) return;
    const uint32_t k0 = d.hot_cnt[1], k1 = d.hot_cnt[0];
    const size_t rb = (size_t)ol * d.NP, hb = (size_t)ol * d.HP;
    int nowhot = 0;                                                // the row's entries whose member just got a slot
    for (uint32_t k = k0 + lane_id(); k < k1; k += 64 * MB) {      // (MB slots per lane in flight: batched gathers)
        uint32_t m[MB], w[MB];
        uint2 cell[MB];
#pragma unroll
        for (int u = 0; u < MB; u++) m[u] = k + 64u * u < k1 ? d.hlist[k + 64u * u] : 0u;
#pragma unroll
        for (int u = 0; u < MB; u++) {
            cell[u] = d.dent[rb + m[u]];
            w[u] = d.mw[rb + m[u]];
        }
#pragma unroll
        for (int u = 0; u < MB; u++) {
            if (k + 64u * u >= k1) continue;
            d.hmw[hb + k + 64u * u] = w[u];
            d.hde[hb + k + 64u * u] = cell[u];
            nowhot += de_p(cell[u].x) != DP_NONE;
        }
    }
    if (k1 > k0) {
        nowhot = wsum(nowhot);
        if (lane_id() == 0 && nowhot) d.nhe[ol] -= nowhot;
    }
}

// write the hot columns' cells back to the dense cells of rows [ol0, ol0 + nrows), one wave per row: for a hot
// member the slot's cell is the entry (the dense cell is not written while the member holds a slot), so the
// dense array is current only after this (before the slots are dropped, and before a host read-back of a row)
__global__ void k_hot_flush(DS d, uint32_t ol0, uint32_t nrows) {
    const uint32_t i = wave_gid();
    if (i >= nrows) return;
    const uint32_t ol = ol0 + i, k1 = d.hot_cnt[0];
    const size_t rb = (size_t)ol * d.NP, hb = (size_t)ol * d.HP;
    for (uint32_t k = lane_id(); k < k1; k += 64) d.dent[rb + d.hlist[k]] = d.hde[hb + k];
}

// memberlist.AddJoinList (memberlist.go:398-406) on observer row ol, one wave: Update of the join list
// (records {member | status << 24, e, source, source e}, distinct members, as MembershipAsChanges makes them,
// disseminator.go:107-123), then ClearChange (disseminator.go:229-233) of every applied change except the
// observer's own, so the join list is not gossiped. A change applies exactly as in any other Update
// (override rules, refute, timers, maxP, applied-change log); the entry it records is removed again right
// away, which equals clearing after the whole Update because the members are distinct. applied_out = the
// number of applied changes.
__global__ void k_add_join_list(DS d, uint32_t ol, const uint4 *__restrict__ rec, uint32_t n, uint32_t r,
                                uint32_t *applied_out) {
    const uint32_t o = d.lo + ol;
    const uint32_t *rowp = d.mw + (size_t)ol * d.NP;
    MAcc acc;
    acc_begin(d, ol, acc);
    for (uint32_t base = 0; base < n; base += 64 * MB) {
        uint4 c[MB];
        uint32_t cur[MB];
#pragma unroll
        for (int u = 0; u < MB; u++) {
            const uint32_t i = base + u * 64 + lane_id();
            c[u] = i < n ? rec[i] : make_uint4(0xFFFFFFFFu, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < MB; u++) cur[u] = c[u].x != 0xFFFFFFFFu ? rowp[c[u].x & 0xFFFFFFu] : 0u;
#pragma unroll
        for (int u = 0; u < MB; u++) {
            if (c[u].x == 0xFFFFFFFFu) continue;
            const uint32_t m = c[u].x & 0xFFFFFFu;
            const int before = acc.napp;
            merge_change_w(d, ol, o, m, cur[u], c[u].x >> 24, c[u].y, c[u].z, c[u].w, r, r, acc);
            if (acc.napp != before && m != o) {                    // ClearChange(member)
                const size_t idx = (size_t)ol * d.NP + m;
                d.dent[idx].x = DE_NONE;
                const uint32_t hk = hot_slot(d, m);
                if (hk != SRC_NONE) d.hde[(size_t)ol * d.HP + hk].x = DE_NONE;
                else acc.dnh--;
                atomicAnd(&d.dbit[(size_t)ol * d.NBIT + (m >> 5)], ~(1u << (m & 31)));
                acc.ddc--;
            }
        }
    }
    const int napp = wsum(acc.napp);
    __threadfence_block();
    wave_finalize(d, ol, acc, 2);
    if (lane_id() == 0) *applied_out = (uint32_t)napp;
}

// ---------------------------------------------------------------------------------------------
// phase E: host events, applied in order by one thread (few per round)
// ---------------------------------------------------------------------------------------------
// returns the number of applied changes (0/1)
__device__ int thread_make_change(const DS &d, uint32_t ol, uint32_t o, uint32_t m, uint32_t e, uint32_t st, uint32_t r) {
    MAcc acc;
    acc_begin(d, ol, acc);
    const uint32_t self_e = d.mw[(size_t)ol * d.NP + o] >> 3;   // MakeChange: SourceIncarnation = local inc
    merge_change(d, ol, o, m, st, e, o, self_e, r, r, acc);
    fold_row(d, ol, acc.dping, acc.ddc, acc.napp, acc.nref, 0, acc.dlen, acc.maxlast, acc.inval, acc.dfp, true, acc.dnh);
    return acc.napp;
}

__global__ void k_events(DS d, const uint4 *ev, uint32_t nev, uint32_t r, uint32_t *applied_out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (uint32_t i = 0; i < nev; i++) {
        const uint4 e = ev[i];   // {kind, observer, member, e | status << 29 | label}
        const uint32_t kind = e.x, o = e.y;
        if (o < d.lo || o >= d.lo + d.NL) continue;
        const uint32_t ol = o - d.lo;
        int applied = 0;
        switch (kind) {
        case 1:  // MakeChange(o, member, e, status)
            applied = thread_make_change(d, ol, o, e.z, e.w & 0x1FFFFFFFu, e.w >> 29, r);
            break;
        case 2:  // Reincarnate: MakeAlive(self, now) (memberlist.go:234-236)
            applied = thread_make_change(d, ol, o, o, r, ST_ALIVE, r);
            break;
        case 3:  // admin leave: MakeLeave(self, local inc) (handlers.go:145-148)
            applied = thread_make_change(d, ol, o, o, d.mw[(size_t)ol * d.NP + o] >> 3, ST_LEAVE, r);
            break;
        case 4:  // reap: faulty → tombstone (handlers.go:154-163)
            for (uint32_t m = 0; m < d.N; m++) {
                const uint32_t w = d.mw[(size_t)ol * d.NP + m];
                if ((w & 7u) == ST_FAULTY) applied += thread_make_change(d, ol, o, m, w >> 3, ST_TOMB, r);
            }
            break;
        }
        if (applied_out) applied_out[i] = (uint32_t)applied;
    }
}

// ---------------------------------------------------------------------------------------------
// phase T: timers (state_transitions.go:90-160 on the round clock; Mock.Add fires in deadline
// order with now = deadline, so a follow-up schedule is based at the fired deadline)
// ---------------------------------------------------------------------------------------------
__global__ void k_timers(DS d, uint32_t r) {
    const uint32_t ol = wave_gid();
    if (ol >= d.NL) return;
    const uint32_t o = d.lo + ol;
    if (!d.live[o] || d.tmin[ol] > r) return;
    const uint32_t self_e = d.mw[(size_t)ol * d.NP + o] >> 3;
    MAcc acc;
    // every fired timer is its own one-change Update (MakeFaulty / MakeTombstone), in (deadline, member) order
    // (clock.Mock fires in deadline order; equal deadlines by member, docs/ROUND_SEMANTICS.md): event tags above
    // the row's sequence number, ordered by (deadline, member); the row's next Update then tags above them all
    const unsigned long long tbase = d.useq ? d.useq[ol] : 0ull;
    uint32_t newmin = NO_DEADLINE;   // per-lane partial minimum, reduced at the end
    int fired = 0;
    for (uint32_t b0 = 0; b0 < d.NB; b0 += 64) {
        // 64 block lower bounds per wave-instruction; only blocks with a due deadline are scanned
        const uint32_t bl = b0 + lane_id();
        const uint32_t bm = bl < d.NB ? d.tblk[(size_t)ol * d.NB + bl] : NO_DEADLINE;
        unsigned long long due = __ballot(bm <= r);
        if (bm > r) newmin = min(newmin, bm);
        while (due) {
            const uint32_t bb = __ffsll((long long)due) - 1;
            due &= due - 1;
            const uint32_t b = b0 + bb;
            const uint32_t m = (b << 6) + lane_id();
            const size_t idx = (size_t)ol * d.NP + m;
            const uint8_t ts = d.tst[idx];
            const uint32_t state = ts & 7u;
            uint2 a = d.tmr[idx];
            if (state && !(ts & 0x80) && a.x <= r) {
                d.tst[idx] = ts | 0x80;                             // fired; the entry stays
                fired++;
                acc.tag = tbase + ((0xFFFFull - min(r - a.x, 0xFFFFu)) << 24) + m;
                if (state == ST_SUSPECT) merge_change(d, ol, o, m, ST_FAULTY, a.y, o, self_e, r, a.x, acc);   // MakeFaulty
                else if (state == ST_FAULTY) merge_change(d, ol, o, m, ST_TOMB, a.y, o, self_e, r, a.x, acc); // MakeTombstone
                else {                                              // Evict (memberlist.go:271-279)
                    const uint32_t w = d.mw[idx];
                    if ((w & 7u) != ST_UNKNOWN && m != o) {
                        if (is_pingable(w & 7u)) acc.dping--;
                        d.mw[idx] = (w & ~7u) | ST_UNKNOWN;
                        colmark(d, m);
                        const uint32_t hk = hot_slot(d, m);
                        if (hk != SRC_NONE) d.hmw[(size_t)ol * d.HP + hk] = (w & ~7u) | ST_UNKNOWN;
                        track_len(d, ol, m, w, (w & ~7u) | ST_UNKNOWN, acc);
                        acc.dfp += fpmix(m, (w & ~7u) | ST_UNKNOWN) - fpmix(m, w);
                        acc.evict++;
                    }
                }
                a = d.tmr[idx];
            }
            const uint8_t ts2 = d.tst[idx];
            const uint32_t v = ((ts2 & 7u) && !(ts2 & 0x80)) ? a.x : NO_DEADLINE;
            const uint32_t bmin = wmin(v);
            if (lane_id() == 0) d.tblk[(size_t)ol * d.NB + b] = bmin;
            newmin = min(newmin, bmin);
        }
    }
    newmin = wmin(newmin);
    if (lane_id() == 0) d.tmin[ol] = newmin;
    fired = wsum(fired);
    if (lane_id() == 0 && fired) ctr_add(d, C_TIMERS_FIRED, (unsigned long long)fired);
    const int napp_t = wsum(acc.napp);
    if (lane_id() == 0 && napp_t && d.useq) d.useq[ol] = tbase + (1ull << 40);
    __threadfence_block();
    wave_finalize(d, ol, acc, 0, false);
}

// ---------------------------------------------------------------------------------------------
// phase S: memberlistIter.Next (memberlist_iter.go:50-72) on Philox permutations
// ---------------------------------------------------------------------------------------------
__global__ void k_select(DS d, int32_t *tgt, uint32_t *exh_list, uint32_t *exh_cnt) {
    const uint32_t ol = blockIdx.x * blockDim.x + threadIdx.x;
    if (ol >= d.NL) return;
    const uint32_t o = d.lo + ol;
    int32_t target = -1;
    if (d.live[o]) {
        if (d.ping[ol] <= 0) {
            exh_list[atomicAdd(exh_cnt, 1u)] = ol;                // walks every member: rare path
        } else {
            int32_t idx = d.it_idx[ol];
            uint32_t ep = d.it_ep[ol];
            Feistel f;
            f.init(d.seed, o, ep, d.N);
            const uint32_t *row = d.mw + (size_t)ol * d.NP;
            for (uint32_t guard = 0; guard < 4 * d.N + 8; guard++) {
                idx++;
                if (idx >= (int32_t)d.N) { idx = 0; ep++; f.init(d.seed, o, ep, d.N); }
                const uint32_t m = f.perm((uint32_t)idx, d.N);
                const uint32_t st = row[m] & 7u;
                if (st == ST_UNKNOWN) continue;
                if (m != o && is_pingable(st)) { target = (int32_t)m; break; }
            }
            if (target < 0) atomicOr(d.err, E_ITER);
            d.it_idx[ol] = idx;
            d.it_ep[ol] = ep;
        }
    }
    tgt[ol] = target;
}

// no pingable member: the reference loop visits until every known member was seen, then
// returns none; replay it literally with a visited bitmap (one thread per exhausted observer)
__global__ void k_select_exhaust(DS d, const uint32_t *exh_list, const uint32_t *exh_cnt, uint32_t *scratch) {
    const uint32_t cnt = *exh_cnt;
    uint32_t *vis = scratch + (size_t)blockIdx.x * (d.NP / 32);
    for (uint32_t q = blockIdx.x; q < cnt; q += gridDim.x) {
        const uint32_t ol = exh_list[q], o = d.lo + ol;
        for (uint32_t i = threadIdx.x; i < d.NP / 32; i += blockDim.x) vis[i] = 0;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t *row = d.mw + (size_t)ol * d.NP;
            uint32_t known = 0;
            for (uint32_t m = 0; m < d.N; m++) known += (row[m] & 7u) != ST_UNKNOWN;
            int32_t idx = d.it_idx[ol];
            uint32_t ep = d.it_ep[ol], nvis = 0;
            Feistel f;
            f.init(d.seed, o, ep, d.N);
            uint64_t guard = 0;
            while (nvis < known && guard++ < 8ull * d.N + 8) {
                idx++;
                if (idx >= (int32_t)d.N) { idx = 0; ep++; f.init(d.seed, o, ep, d.N); }
                const uint32_t m = f.perm((uint32_t)idx, d.N);
                if ((row[m] & 7u) == ST_UNKNOWN) continue;
                if (!(vis[m >> 5] & (1u << (m & 31)))) { vis[m >> 5] |= 1u << (m & 31); nvis++; }
            }
            d.it_idx[ol] = idx;
            d.it_ep[ol] = ep;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// lists and snapshots
// ---------------------------------------------------------------------------------------------
// mode 0: dirty rows; 1: dirty rows of live senders with a target; 2: dirty rows of failed senders
__global__ void k_list(DS d, int mode, const int32_t *tgt, const uint8_t *failed, uint32_t *list, uint32_t *cnt) {
    const uint32_t ol = blockIdx.x * blockDim.x + threadIdx.x;
    if (ol >= d.NL) return;
    bool take = d.dirty[ol] != 0;
    if (mode == 1) take = take && tgt[ol] >= 0;
    if (mode == 2) take = take && failed[ol];
    if (take) list[atomicAdd(cnt, 1u)] = ol;
    // (phase C: a listed row gets a new checksum, on the main stream or in a new side slot; a pending one of an older
    // side half must not overwrite it when that half retires)
    if (take && mode == 0) d.cpslot[ol] = SRC_NONE;
}

__global__ void k_list_one(uint32_t *list, uint32_t *cnt, uint32_t ol, const DS d) {
    if (threadIdx.x == 0) { *cnt = d.dirty[ol] ? 1u : 0u; list[0] = ol; }
}

// phase I (ping_sender.go:43-66) / Q1: snapshot S_o, C_o, I_o for the senders of this phase
// Lazy C_o (sS != nullptr): a dirty sender's checksum is not computed here. Its row is snapshotted
// (sS[o] = dense slot) and hashed only if a receiver compares it (IssueAsReceiver with nothing left to
// send, disseminator.go:170-180), in the batched deferred resolution after the receive waves.
__global__ void k_issue(DS d, int mode, const int32_t *tgt, const uint8_t *failed, MsgDesc *sdesc, uint32_t *sI,
                        uint32_t *sC, uint32_t *sS) {
    const uint32_t ol = wave_gid();
    if (ol >= d.NL) return;
    if (mode == 0 && tgt[ol] < 0) return;
    if (mode == 1 && !failed[ol]) return;
    const uint32_t o = d.lo + ol;
    // (the row's other reads go with the issue's own first loads: nothing below waits for a round trip of its own)
    const uint32_t dirty = d.dirty[ol], cpslot = d.cpslot[ol], cs = d.cs[ol], selfw = d.mw[(size_t)ol * d.NP + o];
    MsgDesc md;
    wave_issue(d, ol, md);
    uint32_t slot = SRC_NONE;
    if (sS && dirty) {
        MsgDesc sn;
        if (wave_snapshot(d, ol, o, sn)) slot = sn.off_lo;
    } else if (sS) {
        slot = cpslot;                                           // clean, checksum still on the side stream
    }
    if (lane_id() == 0) {
        sdesc[o] = md;                                               // message descriptors are indexed by
        sI[o] = selfw >> 3;                                          // global sender id (remote senders'
        sC[o] = slot == SRC_NONE ? cs : 0u;                          // messages are imported there)
        if (sS) sS[o] = slot;
        if (mode == 0) {
            ctr_add(d, C_PINGS, 1ull);
            ctr_add(d, C_MSG_CHANGES, (unsigned long long)md.len);   // counted per helper call in Q2
        }
        ctr_add(d, C_X_ISSUED, (unsigned long long)md.len);
    }
}

// ---------------------------------------------------------------------------------------------
// phase D / Q2 inbox construction (sorted by receiver; ascending sender inside a receiver)
// ---------------------------------------------------------------------------------------------
// inbox keys are (receiver << 32 | sender value): sorting them orders every receiver's inbox by sender,
// wherever the pair came from (local or imported from another shard)
__device__ __forceinline__ void x_push(uint4 *items, uint32_t *cnt, uint32_t cap, uint32_t *err, uint4 it) {
    const uint32_t i = atomicAdd(cnt, 1u);
    if (i < cap) items[i] = it;
    else atomicOr(err, E_XCAP);
}

__global__ void k_pairs_direct(DS d, const int32_t *tgt, unsigned long long *keys, uint8_t *failed, uint32_t *info,
                               uint4 *xitems, uint32_t *xcnt, uint32_t xcap) {
    const uint32_t ol = blockIdx.x * blockDim.x + threadIdx.x;
    if (ol >= d.NL) return;
    const uint32_t o = d.lo + ol;
    const int32_t t = tgt[ol];
    unsigned long long key = (unsigned long long)d.N << 32;
    uint8_t f = 0;
    if (t >= 0) {
        if (!reach(d, o, (uint32_t)t)) {
            f = 1;
            atomicAdd(&info[2], 1u);
        } else if (d.G > 1 && owner_of(d, (uint32_t)t) != d.rank) {
            x_push(xitems, xcnt, xcap, d.err, make_uint4(owner_of(d, (uint32_t)t), 1u /*P_REQ*/, o, (uint32_t)t));
        } else {
            key = ((unsigned long long)(uint32_t)t << 32) | o;
        }
    }
    keys[ol] = key;
    failed[ol] = f;
}

// RandomPingableMembers(k, {target}) (memberlist.go:201-219) with the Philox draw rule
__global__ void k_helpers(DS d, const int32_t *tgt, const uint8_t *failed, uint32_t *H, uint32_t *nh, uint32_t r) {
    const uint32_t ol = blockIdx.x * blockDim.x + threadIdx.x;
    if (ol >= d.NL) return;
    nh[ol] = 0;
    if (!failed[ol]) return;
    const uint32_t o = d.lo + ol, t = (uint32_t)tgt[ol], K = d.K;
    const uint32_t *row = d.mw + (size_t)ol * d.NP;
    ctr_add(d, C_PINGREQS, 1ull);
    const int32_t eligible = d.ping[ol] - (is_pingable(row[t] & 7u) ? 1 : 0);
    const uint32_t need = (uint32_t)max(0, min((int32_t)K, eligible));
    uint32_t got = 0, h[8];
    U4 blk = U4{0, 0, 0, 0};
    for (uint32_t i = 0; i < 64 && got < need; i++) {
        if ((i & 3) == 0) blk = philox10(r, o, 2u, i >> 2, d.seed);
        const uint32_t c = mulhi_n(pick(blk, i), d.N);
        if (c == o || c == t || !is_pingable(row[c] & 7u)) continue;
        bool dup = false;
        for (uint32_t q = 0; q < got; q++) dup |= h[q] == c;
        if (!dup) h[got++] = c;
    }
    if (got < need) {
        const uint32_t start = mulhi_n(philox10(r, o, 2u, 16u, d.seed).x, d.N);
        for (uint32_t q = 0; q < d.N && got < need; q++) {
            uint32_t c = start + q;
            if (c >= d.N) c -= d.N;
            if (c == o || c == t || !is_pingable(row[c] & 7u)) continue;
            bool dup = false;
            for (uint32_t z = 0; z < got; z++) dup |= h[z] == c;
            if (!dup) h[got++] = c;
        }
    }
    for (uint32_t q = 0; q < got; q++) H[(size_t)ol * K + q] = h[q];
    nh[ol] = got;
}

__global__ void k_pairs_helpers(DS d, const uint8_t *failed, const uint32_t *H, const uint32_t *nh,
                                unsigned long long *keys, uint4 *xitems, uint32_t *xcnt, uint32_t xcap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t K = d.K;
    if (i >= d.NL * K) return;
    const uint32_t ol = i / K, q = i % K, o = d.lo + ol;
    unsigned long long key = (unsigned long long)d.N << 32;
    if (failed[ol] && q < nh[ol]) {
        const uint32_t h = H[i];
        if (reach(d, o, h)) {
            if (d.G > 1 && owner_of(d, h) != d.rank)
                x_push(xitems, xcnt, xcap, d.err, make_uint4(owner_of(d, h), 2u /*P_REQ2*/, o * K + q, h));
            else
                key = ((unsigned long long)h << 32) | (o * K + q);
        }
    }
    keys[i] = key;
}

// sorted 64-bit inbox keys → receiver column (run-length encoded next) and sender-value column
__global__ void k_split_keys(const unsigned long long *keys, uint32_t n, uint32_t *recv, uint32_t *vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long k = keys[i];
    recv[i] = (uint32_t)(k >> 32);
    vals[i] = (uint32_t)k;
}

// runs: number of receivers (excluding the sentinel) and the longest inbox
__global__ void k_runs_info(const uint32_t *ukeys, const uint32_t *counts, const uint32_t *nruns, uint32_t N,
                            uint32_t *info) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *nruns) return;
    if (ukeys[i] == N) return;
    atomicMax(&info[1], counts[i]);
    atomicAdd(&info[0], 1u);
}

// ---------------------------------------------------------------------------------------------
// phase D waves / Q2 waves: receiver merges the w-th message of its inbox, then IssueAsReceiver
// (ping_handler.go:25-58 / ping_request_handler.go:32-76)
// ---------------------------------------------------------------------------------------------
struct RecvArgs {
    const uint32_t *ukeys, *counts, *offs, *vals;   // run-length encoded sorted inbox
    const uint4 *pinfo;                             // per inbox pair (k_pair_info): {sender's message descriptor},
                                                    // {I_o, C_o, lazy slot, sender value}
    uint32_t nruns_max;
    int phase;                                      // 0: direct ping (phase D), 1: ping-req (Q2)
    const MsgDesc *sdesc;                           // sender snapshots (by global sender id)
    const uint32_t *sI, *sC;
    const uint32_t *sS;                             // lazy sender checksum: dense slot of the sender's row, or none
    MsgDesc *rdesc;                                 // responses (by sender id / sender id * K + slot)
    uint4 *defer;                                   // {resp index | rdirty<<31, receiver slot, sender checksum or
                                                    //  slot, pair index | spending<<31}
    uint32_t *defer_cnt;
    uint8_t *fsflag;                                // per inbox pair: the receiver answered with a full sync
    uint32_t r;
};

// the inbox pairs' sender snapshots in pair order (one thread per pair, after the inbox sort): a receiver's wave then
// reads its message's descriptor and the sender's I_o, C_o and lazy slot with one load that depends only on its run's
// offset, instead of the pair's sender value and then four arrays indexed by it (two dependent round trips)
__global__ void k_pair_info(const DS d, const uint32_t *vals, uint32_t n, int phase, const MsgDesc *sdesc, const uint32_t *sI,
                            const uint32_t *sC, const uint32_t *sS, uint4 *pinfo) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = vals[i], sender = phase == 0 ? v : v / d.K;
    if (sender >= d.N) return;                                     // (sentinel keys: no receiver reads them)
    const MsgDesc md = sdesc[sender];
    pinfo[2 * (size_t)i] = make_uint4(md.off_lo, md.off_hi, md.len, md.kind);
    pinfo[2 * (size_t)i + 1] = make_uint4(sI[sender], sC[sender], sS ? sS[sender] : SRC_NONE, v);
}

// the full-sync branch of IssueAsReceiver (disseminator.go:161-180): taken iff the filtered list is
// empty and checksums differ. A dirty receiver snapshots its row (the full-sync payload) and the
// decision waits for one batched checksum of all snapshots after the last wave. Reverse full syncs
// are queued afterwards in inbox order (k_build_jobs).
// On the receiver's register copy of its row scalars (RowPre). The response's records are reserved before the
// merge with a bound (the entries before it + the message's changes), so the pool cursor's round trips run beside the
// merge's gathers. The bound may be twice the need, so a round of long buffers would fill the pool with it (config 4's
// heal rounds did, sharded): a dense message, or a bound above 4,096 records or a sixteenth of a sub-pool, allocates
// the exact count after the merge (at most 4,096 spare records per receiver).
__device__ __forceinline__ void recv_one_pre(const DS &d, const RecvArgs &a, uint32_t j, const uint4 pi0, const uint4 pi1,
                                             uint32_t pair, uint32_t nslots, RowPre &p) {
    const uint32_t ol = j - d.lo;
    const uint32_t v = pi1.w, sender = a.phase == 0 ? v : v / d.K, resp_idx = v;
    MsgDesc md;
    md.off_lo = pi0.x; md.off_hi = pi0.y; md.len = pi0.z; md.kind = pi0.w;
    const uint64_t bound = (uint64_t)(uint32_t)p.dcnt + md.len;
    const bool early = md.kind == 0 && bound > 0 && bound <= min(4096ull, d.pool_cap / POOL_SHARDS / 16);
    unsigned long long roff = 0;
    if (early && lane_id() == 0) roff = pool_alloc_lane0(d, (uint32_t)bound);   // (read after the merge)
    wave_merge_msg_pre(d, ol, j, md, a.r, a.r, 0, p, -1, nullptr, true);
    MsgDesc resp;
    resp.kind = 0; resp.len = 0; resp.off_lo = resp.off_hi = 0;
    uint32_t kept = 0;
    const uint32_t cnt = (uint32_t)p.dcnt;
    if (cnt) {
        const unsigned long long off = early ? bcast64(roff) : pool_alloc(d, cnt);
        if (off != ~0ull) {
            int del = 0, delnh = 0;
            kept = wave_issue_body<true>(d, ol, sender, pi1.x, resp, cnt, p.maxp, d.hidx && p.nhe == 0, nslots, off, del,
                                         delnh);
            if (del) { p.dcnt -= del; if (lane_id() == 0) d.dcnt[ol] = p.dcnt; }
            if (delnh) { p.nhe -= delnh; if (lane_id() == 0) d.nhe[ol] = p.nhe; }
            __threadfence_block();
        }
    }
    if (lane_id() == 0) {
        ctr_add(d, C_X_RISSUED, (unsigned long long)kept);
        ctr_add(d, C_X_RCALLS, 1ull);
    }
    if (kept == 0) {
        const uint32_t scs = pi1.y;
        const uint32_t sslot = a.sS ? pi1.z : SRC_NONE;
        const bool rdirty = p.dirty != 0;
        const uint32_t rpend = rdirty ? SRC_NONE : p.cpslot;          // clean; its checksum is on the side stream
        if (rdirty || rpend != SRC_NONE || sslot != SRC_NONE) {
            // a checksum is not known yet: snapshot the receiver (the full-sync payload if the decision goes that
            // way) and decide after the batched checksum of every deferred snapshot
            if (wave_snapshot(d, ol, j, resp) && lane_id() == 0) {
                if (rpend != SRC_NONE) d.dense_meta[resp.off_lo].w = rpend + 1u;   // read after the side stream
                else if (!rdirty) d.dense_cs[resp.off_lo] = p.cs;
                a.defer[atomicAdd(a.defer_cnt, 1u)] =
                    make_uint4(resp_idx | (rdirty ? 0x80000000u : 0u), resp.off_lo, sslot != SRC_NONE ? sslot : scs,
                               pair | (sslot != SRC_NONE ? 0x80000000u : 0u));
            }
            resp.kind = 2;
        } else if (p.cs != scs) {
            wave_snapshot(d, ol, j, resp);
            if (lane_id() == 0) {
                if (a.phase == 0) a.fsflag[pair] = 1;
                ctr_add(d, a.phase == 0 ? C_FULL_SYNCS : C_FULL_SYNCS_PINGREQ, 1ull);
            }
        }
    }
    if (lane_id() == 0) {
        a.rdesc[resp_idx] = resp;
        if (resp.kind != 2) ctr_add(d, C_MSG_CHANGES, (unsigned long long)resp.len);
        if (a.phase == 1) {
            ctr_add(d, C_HELPER_CALLS, 1ull);
            ctr_add(d, C_MSG_CHANGES, (unsigned long long)md.len);
        }
    }
}

// One wave per receiver runs its whole inbox in sender order. Receivers are independent within the
// phase: a receiver writes only its own row, dissemination buffer and timers, and reads only the
// senders' issue-time snapshots (S_o, I_o, C_o). So this equals the wave-by-wave schedule of
// docs/ROUND_SEMANTICS.md §4 D, without a launch per inbox position. The receiver's row scalars are loaded once
// (RowPre) beside its first pair's snapshot, and the next pair's snapshot is loaded while a message is merged.
// launch bounds: 256 threads (SWIM_WAVE_BLOCK) and at least RECV_MIN_WAVES waves per SIMD. The receive waves are
// gather-latency bound (each message is a chain of dependent loads: pair snapshot, record, row word, then the stores),
// so resident waves, not registers, set the pace
#ifndef RECV_MIN_WAVES
#define RECV_MIN_WAVES 4
#endif
__global__ void __launch_bounds__(256, RECV_MIN_WAVES) k_recv(DS d, RecvArgs a) {
    const uint32_t u = wave_gid();
    if (u >= a.nruns_max) return;
    const uint32_t key = a.ukeys[u];
    if (key >= d.N) return;
    const uint32_t n = a.counts[u], off = a.offs[u];
    RowPre p = row_pre(d, key - d.lo);
    const uint32_t nslots = d.hidx ? d.hot_cnt[0] : 0u;
    for (uint32_t w = 0; w < n; w++) {
        const uint32_t pair = off + w;
        recv_one_pre(d, a, key, a.pinfo[2 * (size_t)pair], a.pinfo[2 * (size_t)pair + 1], pair, nslots, p);
    }
    if (d.ulog_cnt && lane_id() == 0) d.ulog_cnt[key - d.lo] = min(p.ulog, ULOG_CAP + 1u);
}

// DS::colx from the rows themselves (one lane per column, a wave's 64 columns in two bitmap words): after raw row
// writes every column was marked, and the divergent-column scans fell back to whole rows for the rest of the handle's
// life. Run at the next step's start, when no snapshot is alive (every step call ends with the side stream drained).
__global__ void k_colx_rebuild(DS d) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    bool diff = false;
    if (m < d.N) {
        const uint32_t w0 = d.mw[m];
        for (uint32_t ol = 1; ol < d.NL && !diff; ol++) diff = d.mw[(size_t)ol * d.NP + m] != w0;
    }
    const unsigned long long bits = __ballot(diff);
    const uint32_t w = (m & ~63u) >> 5;
    if (lane_id() == 0) {
        if (w < d.NBIT) d.colx[w] = (uint32_t)bits;
        if (w + 1 < d.NBIT) d.colx[w + 1] = (uint32_t)(bits >> 32);
    }
}

// the divergent-column lists (DS::ucl / uhk / ucold / ucnt) from the bitmap (one workgroup of 1024 threads: each thread
// a run of bitmap words, a block prefix sum of their bit counts)
__global__ void __launch_bounds__(1024) k_ucols(DS d) {
    __shared__ uint32_t part[1024];
    __shared__ uint32_t ncold;
    const uint32_t t = threadIdx.x, per = (d.NBIT + 1023) / 1024, w0 = t * per;
    if (t == 0) ncold = 0;
    auto bitsof = [&](uint32_t w) -> uint32_t {                    // (bits of members >= N masked off)
        const uint32_t x = d.colx[w], lo = w * 32;
        return lo + 32 <= d.N ? x : lo >= d.N ? 0u : x & ((1u << (d.N - lo)) - 1u);
    };
    uint32_t c = 0;
    for (uint32_t w = w0; w < min(w0 + per, d.NBIT); w++) c += (uint32_t)__popc(bitsof(w));
    part[t] = c;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {              // inclusive Hillis-Steele scan
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t at = part[t] - c;
    for (uint32_t w = w0; w < min(w0 + per, d.NBIT); w++) {
        uint32_t bits = bitsof(w);
        while (bits) {
            const uint32_t m = w * 32 + (uint32_t)__builtin_ctz(bits);
            bits &= bits - 1;
            const uint32_t k = hot_slot(d, m);
            d.ucl[at] = m;
            d.uhk[at] = k;
            if (k == SRC_NONE) d.ucold[atomicAdd(&ncold, 1u)] = m;
            at++;
        }
    }
    __syncthreads();
    if (t == 0) {
        d.ucnt[0] = part[1023];
        d.ucnt[1] = ncold;
    }
}

// one wave: do two rows differ? Outside the divergent columns every row and every snapshot holds the same word
// (DS::colx), so only those are compared while they are few (at most N/4), the rest being the hot slots' compact
// copies (ha, hb: both rows' hmw, or null for a snapshot) and gathers for the others; every word otherwise.
__device__ bool wave_rows_differ(const DS &d, const uint32_t *a, const uint32_t *b, const uint32_t *ha, const uint32_t *hb) {
    const uint32_t lane = lane_id();
    bool diff = false;
    const uint32_t nu = d.ucnt[0];
    if (nu <= d.N / 4) {
        if (ha && hb) {                                            // live rows: hot slots, then the cold columns
            const uint32_t nh = d.hot_cnt[0], nc = d.ucnt[1];
            for (uint32_t k0 = 0; k0 < nh && !__any(diff); k0 += 64 * MB) {
                uint32_t x[MB], y[MB];
#pragma unroll
                for (int u = 0; u < MB; u++) {
                    const uint32_t k = k0 + u * 64 + lane;
                    x[u] = k < nh ? ha[k] : 0u;
                    y[u] = k < nh ? hb[k] : 0u;
                }
#pragma unroll
                for (int u = 0; u < MB; u++) diff |= x[u] != y[u];
            }
            for (uint32_t c0 = 0; c0 < nc && !__any(diff); c0 += 64 * MB) {
                uint32_t x[MB], y[MB];
#pragma unroll
                for (int u = 0; u < MB; u++) {
                    const uint32_t c = c0 + u * 64 + lane;
                    const uint32_t m = c < nc ? d.ucold[c] : 0u;
                    x[u] = c < nc ? a[m] : 0u;
                    y[u] = c < nc ? b[m] : 0u;
                }
#pragma unroll
                for (int u = 0; u < MB; u++) diff |= x[u] != y[u];
            }
        } else {                                                   // a snapshot: every divergent column
            for (uint32_t c0 = 0; c0 < nu && !__any(diff); c0 += 64 * MB) {
                uint32_t x[MB], y[MB];
#pragma unroll
                for (int u = 0; u < MB; u++) {
                    const uint32_t c = c0 + u * 64 + lane;
                    const uint32_t m = c < nu ? d.ucl[c] : 0u;
                    x[u] = c < nu ? a[m] : 0u;
                    y[u] = c < nu ? b[m] : 0u;
                }
#pragma unroll
                for (int u = 0; u < MB; u++) diff |= x[u] != y[u];
            }
        }
    } else {
        const uint4 *a4 = (const uint4 *)a, *b4 = (const uint4 *)b;
        for (uint32_t base = 0; base < d.NP / 4 && !__any(diff); base += 64 * MB) {
            uint4 x[MB], y[MB];
#pragma unroll
            for (int u = 0; u < MB; u++) {
                const uint32_t k = base + u * 64 + lane;
                x[u] = k < d.NP / 4 ? a4[k] : make_uint4(0, 0, 0, 0);
                y[u] = k < d.NP / 4 ? b4[k] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < MB; u++) diff |= x[u].x != y[u].x || x[u].y != y[u].y || x[u].z != y[u].z || x[u].w != y[u].w;
        }
    }
    return __any(diff);
}

// one wave: does snapshot a differ from live row b as it was before its logged merges (the first logged old word of each
// member restored; nlog <= ULOG_CAP entries of log, members inside the divergent columns: every row-word write marks its
// column)? Only over the divergent columns; false when they are more than N/4 (the caller hashes instead)
__device__ bool wave_rows_differ_undo(const DS &d, const uint32_t *a, const uint32_t *b, const uint2 *log, uint32_t nlog,
                                      bool &done) {
    const uint32_t lane = lane_id();
    const uint32_t nu = d.ucnt[0];
    done = nu <= d.N / 4;
    if (!done) return true;
    const uint2 L = lane < nlog ? log[lane] : make_uint2(0xFFFFFFFFu, 0u);
    bool diff = false;
    for (uint32_t c0 = 0; c0 < nu && !__any(diff); c0 += 64 * MB) {
        uint32_t m[MB], x[MB], y[MB];
#pragma unroll
        for (int u = 0; u < MB; u++) {
            const uint32_t c = c0 + u * 64 + lane;
            m[u] = c < nu ? d.ucl[c] : 0xFFFFFFFEu;
            x[u] = c < nu ? a[m[u]] : 0u;
            y[u] = c < nu ? b[m[u]] : 0u;
        }
        for (int k = (int)nlog - 1; k >= 0; k--) {               // (descending: the first logged word of a member wins)
            const uint32_t lm = (uint32_t)__builtin_amdgcn_readlane((int)L.x, k);
            const uint32_t lw = (uint32_t)__builtin_amdgcn_readlane((int)L.y, k);
#pragma unroll
            for (int u = 0; u < MB; u++) y[u] = m[u] == lm ? lw : y[u];
        }
#pragma unroll
        for (int u = 0; u < MB; u++) diff |= x[u] != y[u];
    }
    return __any(diff);
}

// resolve deferred full-sync decisions once the snapshot checksums exist (phase 2 = heal ping:
// the job is queued at once; heal runs in phase E, before any phase-D job of the round)
// Equal rows have equal checksums: a deferred decision whose receiver snapshot equals the sender's
// issue-time row (word for word) is "no full sync" without hashing either side. The sender's
// issue-time row is its issue snapshot (pending C_o, local or side slot) or, for a sender that was
// clean at issue and is still clean, its current row. Remote senders and heal pings are not checked.
// Checksum representatives (round 6). A sender that was clean at issue gave its checksum C_o, but its row may have
// changed since (it received pings of its own in phase D): then no issue-time row was left to compare with, and the
// decision hashed the receiver's snapshot (a one-row chain, 3.3 ms, on the round's critical path in the cascade's
// suspect wave). Any row whose content is unchanged since it was hashed to C_o has the sender's issue-time content, up
// to a checksum collision that the word comparison itself rules out: the receiver's snapshot equal to such a row has
// checksum C_o exactly. k_cs_reps indexes the clean rows of known checksum by that checksum: a direct-mapped table of
// plain 64-bit stores {8-bit build generation, row, checksum} (any row of a checksum will do, so the last store wins and
// no atomic is needed: a first version with compare-and-swap probing spent 0.15-0.6 ms per build on the many rows that
// share a checksum; two checksums on one slot lose one of them, whose decision then tries the undo log or the hash).
// The table is never cleared (an entry of another build reads as empty) and every hit is verified against the row. It
// runs only when the phase deferred a decision.
__device__ __forceinline__ uint32_t rep_hash(uint32_t cs, uint32_t mask) { return fmix32(cs ^ 0x9E3779B9u) & mask; }
__global__ void k_cs_reps(DS d, const uint32_t *defer_cnt, unsigned long long *tab, uint32_t mask, uint32_t gen) {
    const uint32_t ol = blockIdx.x * blockDim.x + threadIdx.x;
    if (*defer_cnt == 0 || ol >= d.NL) return;
    if (d.dirty[ol] || d.cpslot[ol] != SRC_NONE) return;
    const uint32_t cs = d.cs[ol];
    tab[rep_hash(cs, mask)] = ((unsigned long long)gen << 56) | ((unsigned long long)ol << 32) | cs;
}
// a clean local row whose current checksum is cs, or SRC_NONE
__device__ __forceinline__ uint32_t rep_find(const DS &d, const unsigned long long *tab, uint32_t mask, uint32_t gen,
                                             uint32_t cs) {
    const unsigned long long cur = tab[rep_hash(cs, mask)];
    if ((uint32_t)(cur >> 56) != gen || (uint32_t)cur != cs) return SRC_NONE;
    const uint32_t r = (uint32_t)(cur >> 32) & 0xFFFFFFu;
    return r < d.NL && !d.dirty[r] && d.cpslot[r] == SRC_NONE && d.cs[r] == cs ? r : SRC_NONE;
}

__global__ void k_defer_eq(DS d, const uint4 *defer, const uint32_t *defer_cnt, int phase, uint8_t *eq,
                           const unsigned long long *tab, uint32_t mask, uint32_t gen) {
    const uint32_t i = wave_gid();
    if (i >= *defer_cnt) return;
    const uint4 e = defer[i];
    const uint32_t ri = e.x & 0x7FFFFFFFu, sender = phase == 1 ? ri / d.K : ri;
    const uint32_t *srow = nullptr;
    bool viarep = false;
    if (phase != 2) {
        if (e.w & 0x80000000u) {
            if (!(e.z & 0x80000000u)) srow = d.dense + (size_t)e.z * d.NP;
        } else if (sender >= d.lo && sender < d.lo + d.NL && !d.dirty[sender - d.lo]) {
            srow = d.mw + (size_t)(sender - d.lo) * d.NP;
        } else if (tab) {                                          // C_o = e.z known: a representative of it
            const uint32_t r = rep_find(d, tab, mask, gen, e.z);
            if (r != SRC_NONE) {
                srow = d.mw + (size_t)r * d.NP;
                viarep = true;
            }
        }
    }
    bool same = false, viaundo = false;
    if (srow) {
        same = !wave_rows_differ(d, d.dense + (size_t)e.y * d.NP, srow, nullptr, nullptr);
    } else if (phase != 2 && !(e.w & 0x80000000u) && d.ulog && sender >= d.lo && sender < d.lo + d.NL) {
        // the sender was clean at issue (C_o = e.z) and has changed since only by this phase's merges: its issue-time
        // row is its row with the logged words restored
        const uint32_t sl = sender - d.lo, nlog = d.ulog_cnt[sl];
        if (nlog <= ULOG_CAP) {
            bool done = false;
            const bool differ = wave_rows_differ_undo(d, d.dense + (size_t)e.y * d.NP, d.mw + (size_t)sl * d.NP,
                                                      d.ulog + (size_t)sl * ULOG_CAP, nlog, done);
            viaundo = done;
            same = done && !differ;
        }
    }
    if (lane_id() == 0) {
        eq[i] = same ? 1 : 0;
        ctr_add(d, C_X_DEFER, 1ull);
        if (same) ctr_add(d, viarep ? C_X_DEFER_REP : viaundo ? C_X_DEFER_UNDO : C_X_DEFER_EQ, 1ull);
        if (!srow && !viaundo) ctr_add(d, C_X_DEFER_NOROW, 1ull);
    }
}

__global__ void k_recv_finish(DS d, const uint4 *defer, const uint32_t *defer_cnt, MsgDesc *rdesc, int phase,
                              uint8_t *fsflag, const uint32_t *rcs, const uint8_t *eq) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *defer_cnt) return;
    const uint4 e = defer[i];
    const uint32_t slot = e.y, pair = e.w & 0x7FFFFFFFu;
    const uint32_t ri = e.x & 0x7FFFFFFFu, sender = phase == 1 ? ri / d.K : ri;
    // pending C_o: local snapshot (hashed in this resolution) or remote (answered by its owner shard)
    MsgDesc resp;
    resp.kind = 0; resp.len = 0; resp.off_lo = resp.off_hi = 0;
    bool differ = false;
    if (!eq[i]) {
        const uint32_t scs = !(e.w & 0x80000000u) ? e.z : (e.z & 0x80000000u) ? rcs[sender] : d.dense_cs[e.z];
        const uint32_t alias = d.dense_meta[slot].w;               // receiver clean, hashed on the side stream
        if (alias) d.dense_cs[slot] = d.dense_cs[alias - 1u];
        differ = d.dense_cs[slot] != scs;
    }
    if (differ) {
        resp.kind = 1; resp.off_lo = slot; resp.len = d.dense_meta[slot].z;
        ctr_add(d, phase == 1 ? C_FULL_SYNCS_PINGREQ : C_FULL_SYNCS, 1ull);
        if (phase == 2) {
            const uint32_t ol = d.dense_meta[slot].x - d.lo;
            if (d.njobs[ol] < d.maxjobs) d.jobs[(size_t)ol * d.maxjobs + d.njobs[ol]++] = pair;
            else ctr_add(d, C_RFS_OMITTED, 1ull);
        } else if (phase == 0) {
            fsflag[pair] = 1;
        }
    }
    rdesc[ri] = resp;
    if (phase != 2) ctr_add(d, C_MSG_CHANGES, (unsigned long long)resp.len);
}

// defer list → checksum list of the dense snapshots that need a hash (NL + slot): dirty receivers and
// pending senders (a sender referenced by several deferred decisions is hashed once per reference)
__global__ void k_defer_ids(DS d, const uint4 *defer, const uint32_t *defer_cnt, const uint8_t *eq, uint32_t *list,
                            uint32_t *cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *defer_cnt || eq[i]) return;
    atomicAdd(cnt + 1, 1u);                                        // decisions left to the checksums
    const uint4 e = defer[i];
    if (e.x & 0x80000000u) list[atomicAdd(cnt, 1u)] = d.NL + e.y;
    if ((e.w & 0x80000000u) && !(e.z & 0x80000000u) && e.z < d.dense_cap)                  // local pending
        list[atomicAdd(cnt, 1u)] = d.NL + e.z;                     // (slots >= dense_cap: side stream)
}

// tryStartReverseFullSync (disseminator.go:257-278) in inbox order: at most maxjobs per receiver
__global__ void k_build_jobs(DS d, const uint32_t *ukeys, const uint32_t *counts, const uint32_t *offs,
                             const uint32_t *vals, uint32_t nruns, uint8_t *fsflag) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nruns || ukeys[u] >= d.N) return;
    const uint32_t ol = ukeys[u] - d.lo;
    for (uint32_t w = 0; w < counts[u]; w++) {
        const uint32_t p = offs[u] + w;
        if (!fsflag[p]) continue;
        fsflag[p] = 0;
        if (d.njobs[ol] < d.maxjobs) d.jobs[(size_t)ol * d.maxjobs + d.njobs[ol]++] = vals[p];
        else ctr_add(d, C_RFS_OMITTED, 1ull);
    }
}

// phase R: sender bumps its piggyback counters and merges the response (ping_sender.go:52, node.go:488)
__global__ void k_resp(DS d, const int32_t *tgt, const uint8_t *failed, const MsgDesc *sdesc, const MsgDesc *rdesc,
                       uint32_t r) {
    const uint32_t ol = wave_gid();
    if (ol >= d.NL) return;
    if (tgt[ol] < 0 || failed[ol]) return;
    const uint32_t o = d.lo + ol;
    // (the row scalars, both descriptors: one round trip; RowPre carries them through the bump and the merge)
    RowPre p = row_pre(d, ol);
    const MsgDesc sd = sdesc[o], rd = rdesc[o];
    uint4 rec0[MB];                                                 // (the response's first records ride with the bump's
    merge_first(d, rd, rec0);                                       // loads: the pool is read-only here)
    wave_bump_pre(d, ol, sd, p);
    wave_merge_msg_pre(d, ol, o, rd, r, r, 1, p, C_X_DENSE_RESP, rec0);
    if (lane_id() == 0) {
        ctr_add(d, C_PINGS_OK, 1ull);
        if (sd.kind == 0) ctr_add(d, C_X_BUMPED, (unsigned long long)sd.len);
    }
}

// Q3: resolve indirect pings (ping_request_sender.go:65-138, node.go:494-509)
__global__ void k_resolve(DS d, const int32_t *tgt, const uint8_t *failed, const uint32_t *H, const uint32_t *nh,
                          const MsgDesc *sdesc2, const MsgDesc *rdesc2, uint32_t r) {
    const uint32_t ol = wave_gid();
    if (ol >= d.NL || !failed[ol]) return;
    const uint32_t o = d.lo + ol, K = d.K;
    uint32_t errs = 0;
    for (uint32_t q = 0; q < nh[ol]; q++) {
        const uint32_t h = H[(size_t)ol * K + q];
        if (!reach(d, o, h)) {
            errs++;
            wave_bump(d, ol, sdesc2[o]);                            // bump only on error (105-106)
        } else {
            wave_merge_msg(d, ol, o, rdesc2[(size_t)o * K + q], r, r, 2, C_X_DENSE_RESP);
        }
    }
    if (lane_id() == 0) {
        if (errs) ctr_add(d, C_HELPER_ERRORS, (unsigned long long)errs);
        if (errs == K) {
            ctr_add(d, C_INCONCLUSIVE, 1ull);
        } else {
            ctr_add(d, C_SUSPECT_DECL, 1ull);
            const uint32_t t = (uint32_t)tgt[ol];
            const uint32_t te = d.mw[(size_t)ol * d.NP + t] >> 3;      // member.Incarnation read now (node.go:508)
            thread_make_change(d, ol, o, t, te, ST_SUSPECT, r);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// phase F: reverse full syncs (disseminator.go:257-304); sources are snapshotted first
// ---------------------------------------------------------------------------------------------
__global__ void k_jobs_mark(DS d, uint8_t *need) {
    const uint32_t ol = blockIdx.x * blockDim.x + threadIdx.x;
    if (ol >= d.NL) return;
    for (uint32_t q = 0; q < d.njobs[ol]; q++) need[d.jobs[(size_t)ol * d.maxjobs + q]] = 1;   // [N], global
}

__global__ void k_jobs_snap(DS d, const uint8_t *need, MsgDesc *snapdesc) {
    const uint32_t ol = wave_gid();
    if (ol >= d.NL || !need[d.lo + ol]) return;
    MsgDesc md;
    wave_snapshot(d, ol, d.lo + ol, md);
    if (lane_id() == 0) snapdesc[d.lo + ol] = md;
}

// one wave per row merges its queued sources' snapshots in queue order (the sources are snapshots taken before this
// launch and a row writes only itself, so one launch runs every queue position: round 5 launched one per position)
__global__ void k_jobs_merge(DS d, const MsgDesc *snapdesc, uint32_t r) {
    const uint32_t ol = wave_gid();
    if (ol >= d.NL) return;
    const uint32_t nj = d.njobs[ol];
    for (uint32_t q = 0; q < nj; q++) {
        const uint32_t src = d.jobs[(size_t)ol * d.maxjobs + q];
        wave_merge_msg(d, ol, d.lo + ol, snapdesc[src], r, r, 3, C_X_DENSE_JOBS);
    }
    if (lane_id() == 0 && nj) ctr_add(d, C_RFS_DONE, (unsigned long long)nj);
}

__global__ void k_jobs_reset(DS d, uint8_t *need) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < d.NL) d.njobs[i] = 0;
    if (i < d.N) need[i] = 0;
}

// ---------------------------------------------------------------------------------------------
// phase C dedup: dirty rows with equal content have equal checksums. Rows are grouped by their
// fingerprint (sorted), every row is compared word for word with the first row of its group, and
// only group heads and rows that differ from their head are hashed; the others copy the head's
// checksum. Exact: the fingerprint only proposes the pairs that the comparison checks.
// ---------------------------------------------------------------------------------------------
__global__ void k_fp_keys(DS d, const uint32_t *list, uint32_t n, unsigned long long *keys, uint32_t *vals,
                          unsigned long long keymask) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = d.fp[list[i]] & keymask;                             // (tests narrow the keys: collision groups)
    vals[i] = list[i];
}

__global__ void k_fp_heads(const unsigned long long *keys, uint32_t n, uint32_t *headpos) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    headpos[i] = (i == 0 || keys[i] != keys[i - 1]) ? i : 0u;   // inclusive max-scan gives each row its group head
}

// one wave per sorted row: heads and rows unequal to their head are flagged for hashing (the hash
// list is then rebuilt in row order: rows of one workgroup stay close in memory, few TLB pages)
__global__ void k_fp_verify(DS d, const uint32_t *vals, const uint32_t *headpos, uint32_t n, uint8_t *hflag,
                            uint32_t *dup_of) {
    const uint32_t i = wave_gid();
    if (i >= n) return;
    const uint32_t row = vals[i], hp = headpos[i];
    bool same = false;
    if (hp != i) {
        const uint32_t head = vals[hp];
        const uint32_t *ha = d.hidx ? d.hmw + (size_t)head * d.HP : nullptr, *hb = d.hidx ? d.hmw + (size_t)row * d.HP : nullptr;
        same = !wave_rows_differ(d, d.mw + (size_t)head * d.NP, d.mw + (size_t)row * d.NP, ha, hb);
    }
    if (lane_id() == 0) {
        dup_of[row] = same ? vals[hp] : SRC_NONE;
        hflag[row] = same ? 0 : 1;
    }
}

__global__ void k_list_flagged(uint32_t nl, uint8_t *flag, uint32_t *list, uint32_t *cnt) {
    const uint32_t ol = blockIdx.x * blockDim.x + threadIdx.x;
    if (ol >= nl || !flag[ol]) return;
    flag[ol] = 0;
    list[atomicAdd(cnt, 1u)] = ol;
}

// Round 6: the groups without a sort. Every listed row offers {tag, row} to slot (fp & mask) of a direct-mapped table
// (tag = the fingerprint's high word); the smallest offer wins (atomicMin), so the winner does not depend on the list's
// order or on timing. A row whose slot was won by another tag offers itself again to a second table at slot
// (tag & mask) (the rows that do is again the same set in every run), so that few duplicate groups lose their dedup to
// a slot conflict. A row compares itself with the winner of the first of its slots that holds its own tag (its group
// head); rows that find none are hashed themselves. Exact either way: equality is decided by the comparison.
__device__ __forceinline__ void fp_slot_tag(unsigned long long fp, uint32_t mask, uint32_t &slot, uint32_t &slot2,
                                            uint32_t &tag) {
    slot = (uint32_t)fp & mask;
    tag = (uint32_t)(fp >> 32);
    slot2 = (tag ^ (uint32_t)(fp >> 13)) & mask;
}
// pass 0: every listed row into table 0; pass 1: the rows whose table-0 slot holds another tag into table 1
__global__ void k_fp_table(DS d, const uint32_t *list, uint32_t n, unsigned long long *tab, uint32_t mask,
                           unsigned long long keymask, int pass) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t row = list[i];
    uint32_t slot, slot2, tag;
    fp_slot_tag(d.fp[row] & keymask, mask, slot, slot2, tag);     // (tests narrow the keys: collision groups)
    const unsigned long long key = ((unsigned long long)tag << 32) | row;
    if (pass == 0) atomicMin(tab + slot, key);
    else if ((uint32_t)(tab[slot] >> 32) != tag) atomicMin(tab + (mask + 1) + slot2, key);
}
// one wave per listed row: heads and rows unequal to their head are flagged for hashing, the others get dup_of = head
__global__ void k_fp_verify_tab(DS d, const uint32_t *list, uint32_t n, const unsigned long long *tab, uint32_t mask,
                                unsigned long long keymask, uint8_t *hflag, uint32_t *dup_of) {
    const uint32_t i = wave_gid();
    if (i >= n) return;
    const uint32_t row = list[i];
    uint32_t slot, slot2, tag;
    fp_slot_tag(d.fp[row] & keymask, mask, slot, slot2, tag);
    unsigned long long key = tab[slot];
    if ((uint32_t)(key >> 32) != tag) key = tab[(mask + 1) + slot2];
    const uint32_t head = (uint32_t)key;
    bool same = false;
    if ((uint32_t)(key >> 32) == tag && head != row) {
        const uint32_t *ha = d.hidx ? d.hmw + (size_t)head * d.HP : nullptr, *hb = d.hidx ? d.hmw + (size_t)row * d.HP : nullptr;
        same = !wave_rows_differ(d, d.mw + (size_t)head * d.NP, d.mw + (size_t)row * d.NP, ha, hb);
    }
    if (lane_id() == 0) {
        dup_of[row] = same ? head : SRC_NONE;
        hflag[row] = same ? 0 : 1;
    }
}
// the flagged rows in row order (one workgroup: a thread per run of consecutive rows, read 16 flags at a time; a block
// prefix sum places them); clears the flags and writes the count
__device__ __forceinline__ uint4 flags16(const uint8_t *flag, uint32_t base, uint32_t nl) {
    if (base + 16u <= nl) return *(const uint4 *)(flag + base);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; base + k < nl && k < 16u; k++) w[k >> 2] |= (uint32_t)flag[base + k] << (8u * (k & 3u));
    return make_uint4(w[0], w[1], w[2], w[3]);
}
__global__ void __launch_bounds__(1024) k_list_flagged_ordered(uint32_t nl, uint8_t *flag, uint32_t *list, uint32_t *cnt) {
    __shared__ uint32_t wtot[16];
    const uint32_t t = threadIdx.x, per = ((nl + 1023u) / 1024u + 15u) & ~15u;   // (flags are 0 or 1: a popcount each)
    const uint32_t lo = t * per;
    uint32_t c = 0;
    for (uint32_t q = 0; q < per && lo + q < nl; q += 16) {
        const uint4 v = flags16(flag, lo + q, nl);
        c += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
    }
    uint32_t wt;
    const uint32_t ex = wscan_excl(c, wt);
    if (lane_id() == 63) wtot[t >> 6] = wt;
    __syncthreads();
    uint32_t base = 0, all = 0;
    for (uint32_t w = 0; w < 16; w++) {
        const uint32_t v = wtot[w];
        base += w < (t >> 6) ? v : 0u;
        all += v;
    }
    uint32_t p = base + ex;
    for (uint32_t q = 0; q < per && lo + q < nl && c; q += 16) {
        const uint4 v = flags16(flag, lo + q, nl);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        if ((v.x | v.y | v.z | v.w) == 0) continue;
        for (uint32_t k = 0; k < 16u; k++)
            if ((w4[k >> 2] >> (8u * (k & 3u))) & 0xFFu) {
                list[p++] = lo + q + k;
                flag[lo + q + k] = 0;
            }
    }
    if (t == 0) *cnt = all;
}

__global__ void k_fp_copy(DS d, const uint32_t *vals, uint32_t n, const uint32_t *dup_of) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t row = vals[i], h = dup_of[row];
    if (h == SRC_NONE) return;
    d.cs[row] = d.cs[h];
    d.dirty[row] = 0;
    ctr_add(d, C_X_CS_DUP, 1ull);
}

// ---------------------------------------------------------------------------------------------
// phase C on the side stream: the rows left after dedup are copied into dense slots of one side half
// [slot0, slot0 + n) (one wave per row) and hashed there while the next rounds run on the main stream; every
// listed row (dedup heads and duplicates) is marked clean with cpslot = the slot whose dense_cs carries its
// checksum. k_side_retire writes cs[] on the main stream when the half is reused or synchronised.
// ---------------------------------------------------------------------------------------------
__global__ void k_snap_rows(DS d, const uint32_t *rows, uint32_t n, uint32_t *ids, uint32_t *idcnt, uint32_t slot0) {
    const uint32_t k = wave_gid();
    if (k == 0 && lane_id() == 0) *idcnt = n;
    if (k >= n) return;
    const uint32_t ol = rows[k], slot = slot0 + k;
    const uint4 *src = (const uint4 *)(d.mw + (size_t)ol * d.NP);
    uint4 *dst = (uint4 *)(d.dense + (size_t)slot * d.NP);
    for (uint32_t i = lane_id(); i < d.NP / 4; i += 64 * SNAP_MB) {
        uint4 v[SNAP_MB];
#pragma unroll
        for (int u = 0; u < SNAP_MB; u++) v[u] = i + u * 64 < d.NP / 4 ? src[i + u * 64] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < SNAP_MB; u++)
            if (i + u * 64 < d.NP / 4) dst[i + u * 64] = v[u];
    }
    if (lane_id() == 0) {
        d.dense_meta[slot] = make_uint4(d.lo + ol, 0, 0, 0);
        d.dense_len[slot] = d.clen[ol];
        d.dense_last[slot] = d.clast[ol];
        d.cpslot[ol] = slot;
        d.dirty[ol] = 0;
        ids[k] = d.NL + slot;
    }
}

// dedup duplicates (vals = the dirty rows sorted by fingerprint, dup_of from k_fp_verify) take their
// head's slot (k_side_retire copies the slot's checksum to every row that refers to it)
__global__ void k_snap_dups(DS d, const uint32_t *vals, uint32_t n, const uint32_t *dup_of) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t row = vals[i], h = dup_of ? dup_of[row] : SRC_NONE;
    if (h != SRC_NONE) {
        d.cpslot[row] = d.cpslot[h];
        d.dirty[row] = 0;
    }
}

// a side half's checksums into cs[] of the rows still referring to its slots [lo, hi), on the main stream after the
// half's launch (a row listed by a later phase C had its cpslot cleared or replaced there: its newer checksum stands)
__global__ void k_side_retire(DS d, uint32_t lo, uint32_t hi) {
    const uint32_t ol = blockIdx.x * blockDim.x + threadIdx.x;
    if (ol >= d.NL) return;
    const uint32_t s = d.cpslot[ol];
    if (s < lo || s >= hi) return;
    d.cs[ol] = d.dense_cs[s];
    d.cpslot[ol] = SRC_NONE;
}

#include "swimsim_checksum.hip"

// ---------------------------------------------------------------------------------------------
// heal helpers (heal_partition.go:33-145)
// ---------------------------------------------------------------------------------------------
__global__ void k_snapshot_row(DS d, uint32_t ol, MsgDesc *out) {
    MsgDesc md;
    wave_snapshot(d, ol, d.lo + ol, md);
    if (lane_id() == 0) *out = md;
}

__device__ __forceinline__ uint32_t outgoing(uint32_t st) { return st == ST_TOMB ? ST_FAULTY : st; }

// nodesThatNeedToReincarnate (heal_partition.go:64-92) over dense snapshots MA (slot a), MB (slot b)
__global__ void k_heal_diff(DS d, const MsgDesc *ma, const MsgDesc *mb, MsgDesc *outA, MsgDesc *outB) {
    const uint32_t *A = d.dense + (size_t)ma->off_lo * d.NP;
    const uint32_t *B = d.dense + (size_t)mb->off_lo * d.NP;
    // count
    int na = 0, nb = 0;
    for (uint32_t m = lane_id(); m < d.N; m += 64) {
        const uint32_t a = A[m], b = B[m];
        if ((a & 7u) == ST_UNKNOWN || (b & 7u) == ST_UNKNOWN) continue;
        const uint32_t as = outgoing(a & 7u), bs = outgoing(b & 7u);
        const uint32_t ak = ((a >> 3) << 3) | as, bk = ((b >> 3) << 3) | bs;
        if (is_pingable(bs) && ak > bk && !is_pingable(as)) nb++;
        if (is_pingable(as) && bk > ak && !is_pingable(bs)) na++;
    }
    na = wsum(na);
    nb = wsum(nb);
    const unsigned long long oa = pool_alloc(d, (uint32_t)na);
    const unsigned long long ob = pool_alloc(d, (uint32_t)nb);
    uint32_t pa = 0, pb = 0;
    for (uint32_t base = 0; base < d.NP; base += 64) {
        const uint32_t m = base + lane_id();
        bool wa = false, wb = false;
        uint32_t a = 0, b = 0;
        if (m < d.N) {
            a = A[m]; b = B[m];
            if ((a & 7u) != ST_UNKNOWN && (b & 7u) != ST_UNKNOWN) {
                const uint32_t as = outgoing(a & 7u), bs = outgoing(b & 7u);
                const uint32_t ak = ((a >> 3) << 3) | as, bk = ((b >> 3) << 3) | bs;
                wb = is_pingable(bs) && ak > bk && !is_pingable(as);
                wa = is_pingable(as) && bk > ak && !is_pingable(bs);
            }
        }
        const unsigned long long ma_ = __ballot(wa), mb_ = __ballot(wb);
        if (wa && oa != ~0ull) d.pool[oa + pa + __popcll(ma_ & lanemask_lt())] = rec_make(m, ST_SUSPECT, b >> 3, SRC_NONE, 0, RT_LOOKUP);
        if (wb && ob != ~0ull) d.pool[ob + pb + __popcll(mb_ & lanemask_lt())] = rec_make(m, ST_SUSPECT, a >> 3, SRC_NONE, 0, RT_LOOKUP);
        pa += __popcll(ma_);
        pb += __popcll(mb_);
    }
    if (lane_id() == 0) {
        outA->kind = 0; outA->len = (uint32_t)na; outA->off_lo = (uint32_t)oa; outA->off_hi = (uint32_t)(oa >> 32);
        outB->kind = 0; outB->len = (uint32_t)nb; outB->off_lo = (uint32_t)ob; outB->off_hi = (uint32_t)(ob >> 32);
    }
}

// I_o and C_o of observer row ol (the heal ping's sender fields)
__global__ void k_sender_info(DS d, uint32_t ol, uint32_t *out) {
    if (threadIdx.x) return;
    out[0] = d.mw[(size_t)ol * d.NP + d.lo + ol] >> 3;
    out[1] = d.cs[ol];
}

__global__ void k_apply_msg(DS d, uint32_t ol, const MsgDesc *md, uint32_t r) {
    wave_merge_msg(d, ol, d.lo + ol, *md, r, r, 2, C_X_DENSE_HEAL);
}

// sendPingWithChanges o → t whose response is discarded (heal_partition.go:97-124): target runs
// handlePing: Update, IssueAsReceiver(o, I_o, C_o); a full sync queues a reverse full sync
__global__ void k_ping_with(DS d, uint32_t tol, uint32_t sender, const MsgDesc *md, const uint32_t *sics,
                            MsgDesc *resp_out, uint4 *defer, uint32_t *defer_cnt, uint32_t r) {
    const uint32_t sinc = sics[0], scs = sics[1];
    wave_merge_msg(d, tol, d.lo + tol, *md, r, r, 2);
    MsgDesc resp;
    const uint32_t kept = wave_issue_recv(d, tol, sender, sinc, resp);
    if (kept == 0) {
        if (d.dirty[tol]) {
            if (wave_snapshot(d, tol, d.lo + tol, resp) && lane_id() == 0)
                defer[atomicAdd(defer_cnt, 1u)] = make_uint4(0x80000000u, resp.off_lo, scs, sender);
            resp.kind = 2;
        } else if (d.cs[tol] != scs) {
            wave_snapshot(d, tol, d.lo + tol, resp);
            if (lane_id() == 0) {
                ctr_add(d, C_FULL_SYNCS, 1ull);
                if (d.njobs[tol] < d.maxjobs) d.jobs[(size_t)tol * d.maxjobs + d.njobs[tol]++] = sender;
                else ctr_add(d, C_RFS_OMITTED, 1ull);
            }
        }
    }
    if (lane_id() == 0) *resp_out = resp;
}

// ---------------------------------------------------------------------------------------------
// readback helpers
// ---------------------------------------------------------------------------------------------
// NumMembers of row ol (memberlist.go:174-179): out[0] = members known
__global__ void k_row_known(DS d, uint32_t ol, uint32_t *out) {
    int known = 0;
    for (uint32_t m = lane_id(); m < d.N; m += 64) known += (d.mw[(size_t)ol * d.NP + m] & 7u) != ST_UNKNOWN;
    known = wsum(known);
    if (lane_id() == 0) out[0] = (uint32_t)known;
}

// drain the applied-change log of watched row ol (slot): out[i] = {member, member word, source, source e}
// in member order, the flags cleared; info = {count, NumMembers}. One 1024-thread workgroup: each thread
// takes a contiguous run of members, a block scan of the run counts places the records.
__global__ void __launch_bounds__(1024) k_drain_applied(DS d, uint32_t ol, uint32_t slot, uint4 *out, uint32_t *info) {
    __shared__ uint32_t part[1024];
    __shared__ uint32_t memb[1024];
    const uint32_t t = threadIdx.x, C = (d.NP + 1023) / 1024;
    const uint32_t b = min(t * C, d.N), e = min(b + C, d.N);
    uint4 *lg = d.wlog + (size_t)slot * d.NP;
    const uint32_t *row = d.mw + (size_t)ol * d.NP;
    uint32_t cnt = 0, mem = 0;
    for (uint32_t m = b; m < e; m++) {
        cnt += lg[m].w != 0u;
        mem += (row[m] & 7u) != ST_UNKNOWN;
    }
    part[t] = cnt;
    memb[t] = mem;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {               // inclusive scans (Hillis-Steele)
        const uint32_t v = t >= off ? part[t - off] : 0u, w = t >= off ? memb[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        memb[t] += w;
        __syncthreads();
    }
    uint32_t pos = part[t] - cnt;
    for (uint32_t m = b; m < e; m++) {
        const uint4 v = lg[m];
        if (!v.w) continue;
        out[pos++] = make_uint4(m, v.x, v.y, v.z);
        lg[m] = make_uint4(0, 0, 0, 0);
    }
    if (t == 1023) {
        info[0] = part[1023];
        info[1] = memb[1023];
    }
}

__global__ void k_digest(DS d, unsigned long long *out, uint32_t period_div) {
    const uint32_t ol = wave_gid();
    if (ol >= d.NL) return;
    const uint32_t o = d.lo + ol;
    unsigned long long r = 0, dd = 0, t = 0;
    for (uint32_t m = lane_id(); m < d.N; m += 64) {
        const size_t idx = (size_t)ol * d.NP + m;
        const uint32_t w = d.mw[idx];
        r += mix4(o, m, w & 7u, w >> 3);
        const uint32_t hk = hot_slot(d, m);
        const uint2 ce = hk != SRC_NONE ? d.hde[(size_t)ol * d.HP + hk] : d.dent[idx];
        const uint32_t p = de_p(ce.x);
        if (p != DP_NONE) {
            const uint2 a = make_uint2(de_src(ce.x), ce.y);
            const uint64_t se = a.x == SRC_NONE ? 0ull : (uint64_t)a.y;
            dd += mix4((uint64_t)o | (1ull << 40), m, (uint64_t)p | ((uint64_t)(uint32_t)(a.x + 1u) << 8), se);
        }
        const uint8_t ts = d.tst[idx];
        if (ts & 7u) {
            const uint2 a = d.tmr[idx];
            const uint64_t state = ts & 7u, fired = (ts >> 7) & 1u;
            t += mix4((uint64_t)o | (2ull << 40), m, state | (fired << 4) | ((uint64_t)a.x << 8), a.y);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        r += __shfl_xor(r, off, 64);
        dd += __shfl_xor(dd, off, 64);
        t += __shfl_xor(t, off, 64);
    }
    if (lane_id() == 0) {
        atomicAdd(&out[0], r);
        atomicAdd(&out[1], dd);
        atomicAdd(&out[2], t);
    }
}

}  // namespace swimdev
