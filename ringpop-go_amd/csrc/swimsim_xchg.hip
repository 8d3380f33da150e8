// swimsim_xchg.hip — device side of the observer-row shard exchange.
//
// A cluster's observer rows may be split over G shards (one per GPU, or several in one process for
// testing). Every message whose two ends live on different shards becomes a parcel: a 64-byte
// header plus its payload (16-byte change records, or a dense NP-word row snapshot). Parcels are
// produced from an item list {dest shard, type, index, key}, packed into one contiguous segment per
// destination, moved by the transport (RCCL send/recv over xGMI, or peer copies inside one process)
// and unpacked into the receiving shard's own message pool, dense pool and descriptor arrays, which
// are indexed by global observer id. After an exchange the round's kernels run unchanged.
//
// Segment layout: [u32 parcel offsets, padded to 16 B][parcels]; each parcel 16-byte aligned.
#pragma once

namespace swimdev {

enum ParcelType : uint32_t {
    P_REQ = 1,      // direct ping request: sender o → target t (idx o, key t)
    P_REQ2 = 2,     // ping-req: sender o → helper h (idx o*K+q, key h)
    P_RESP = 3,     // response of a remote receiver to sender o (idx o)
    P_RESP2 = 4,    // helper response (idx o*K+q)
    P_NEED = 5,     // reverse-full-sync source request (idx = source row, key = requesting shard)
    P_SNAP = 6,     // reverse-full-sync source snapshot (idx = source row)
    P_HEALROW = 7,  // heal: target's membership for the healing observer
    P_PING = 8,     // heal: ping-with-changes to a remote target (idx target, key sender)
    P_CSREQ = 9,    // lazy C_o: checksum of sender idx's issue-time snapshot (key = its dense slot on the owner)
    P_CSRESP = 10   // lazy C_o: the answer (idx = sender, key = checksum)
};

struct Parcel {                 // 64 bytes
    uint32_t type, idx, key, kind;
    uint32_t len, sI, sC, pbytes;
    uint4 meta;
    uint32_t dlen;
    int32_t dlast;
    uint32_t dcs, pad;
};

// descriptor arrays and scratch the exchange reads and fills
struct XArgs {
    MsgDesc *sdesc, *sdesc2, *rdesc, *rdesc2, *snapdesc, *hdesc;
    uint32_t *sI, *sC, *sI2, *sC2;
    uint32_t *hsics;              // [4]: heal ping sender fields (out: 0-1, in: 2-3)
    uint8_t *need;                // [N]
    unsigned long long *keys;     // inbox keys (imported pairs are appended)
    uint32_t *npairs;             // append cursor of keys
    uint32_t keycap;
    uint2 *needlist;              // (source row, requesting shard) of imported P_NEED
    uint32_t *needcnt;
    uint32_t needcap;
    uint32_t *sS, *sS2;           // lazy sender checksums: local slot, 0x80000000|remote slot, or none
    uint32_t *rcs;                // [N] checksums of remote senders' snapshots (P_CSRESP)
    uint4 *csreq;                 // imported P_CSREQ: {sender, slot, requesting shard, 0}
    uint32_t *csreqcnt;
    uint32_t csreqcap;
};

__device__ __forceinline__ const MsgDesc *item_desc(const DS &d, const XArgs &x, uint4 it) {
    switch (it.y) {
    case P_REQ: return &x.sdesc[it.z];
    case P_REQ2: return &x.sdesc2[it.z / d.K];
    case P_RESP: return &x.rdesc[it.z];
    case P_RESP2: return &x.rdesc2[it.z];
    case P_SNAP: return &x.snapdesc[it.z];
    case P_HEALROW: return &x.hdesc[6];
    case P_PING: return &x.hdesc[7];
    default: return nullptr;
    }
}

__device__ __forceinline__ uint32_t payload_bytes(const DS &d, const MsgDesc *md) {
    if (!md) return 0;
    if (md->kind == 0) return md->len * 16u;
    if (md->kind == 1) return d.NP * 4u;
    return 0;
}

// per-destination parcel count and byte total
__global__ void k_x_size(DS d, XArgs x, const uint4 *items, const uint32_t *cnt, uint32_t cap, unsigned long long *sz) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= min(*cnt, cap)) return;
    const uint4 it = items[i];
    const uint32_t b = (uint32_t)sizeof(Parcel) + payload_bytes(d, item_desc(d, x, it));
    atomicAdd(&sz[2 * it.x], (unsigned long long)b);
    atomicAdd(&sz[2 * it.x + 1], 1ull);
}

// the segment each destination receives from this shard, {bytes, parcels}, from k_x_size's totals: the layout xchg()
// computes on the host (a 4-B offset per parcel, the table 16-byte aligned, then the parcels). A stream-ordered
// transport sends these to the peers on the device, so the host waits once per exchange
__global__ void k_x_sendsz(const unsigned long long *sz, uint32_t G, unsigned long long *out) {
    for (uint32_t p = threadIdx.x; p < G; p += blockDim.x) {
        const unsigned long long n = sz[2 * p + 1];
        const unsigned long long tbl = (n * 4ull + 15ull) & ~15ull;
        out[2 * p] = n ? tbl + sz[2 * p] : 0ull;
        out[2 * p + 1] = n;
    }
}

// one wave per item: claim a table slot and a parcel offset in the destination's segment, write both
__global__ void k_x_pack(DS d, XArgs x, const uint4 *items, const uint32_t *cnt, uint32_t cap, uint8_t *buf,
                         const unsigned long long *segoff, unsigned long long *tcur, unsigned long long *dcur) {
    const uint32_t i = wave_gid();
    if (i >= min(*cnt, cap)) return;
    const uint4 it = items[i];
    const MsgDesc *md = item_desc(d, x, it);
    const uint32_t pb = payload_bytes(d, md);
    unsigned long long off = 0, ti = 0;
    if (lane_id() == 0) {
        off = atomicAdd(&dcur[it.x], (unsigned long long)(sizeof(Parcel) + pb));
        ti = atomicAdd(&tcur[it.x], 1ull);
    }
    off = bcast64(off);
    ti = bcast64(ti);
    uint8_t *seg = buf + segoff[it.x];
    Parcel *pc = (Parcel *)(seg + off);
    if (lane_id() == 0) {
        ((uint32_t *)seg)[ti] = (uint32_t)off;
        Parcel h{};
        h.type = it.y; h.idx = it.z; h.key = it.w;
        h.kind = md ? md->kind : 2u;
        h.len = md ? md->len : 0u;
        h.pbytes = pb;
        // a dirty sender's C_o travels as "pending" (sI bit 31) with its snapshot slot on this shard
        if (it.y == P_REQ || it.y == P_REQ2) {
            const uint32_t o = it.y == P_REQ ? it.z : it.z / d.K;
            const uint32_t slot = (it.y == P_REQ ? x.sS : x.sS2)[o];
            h.sI = (it.y == P_REQ ? x.sI : x.sI2)[o] | (slot != SRC_NONE ? 0x80000000u : 0u);
            h.sC = slot != SRC_NONE ? slot : (it.y == P_REQ ? x.sC : x.sC2)[o];
        }
        if (it.y == P_PING) { h.sI = x.hsics[0]; h.sC = x.hsics[1]; }
        if (it.y == P_CSREQ) h.sI = d.rank;                        // requesting shard
        if (md && md->kind == 1) {
            const uint32_t slot = md->off_lo;
            h.meta = d.dense_meta[slot];
            h.dlen = d.dense_len[slot];
            h.dlast = d.dense_last[slot];
            h.dcs = d.dense_cs[slot];
        }
        *pc = h;
    }
    if (!md || pb == 0) return;
    uint4 *dst = (uint4 *)(pc + 1);
    const uint4 *src = md->kind == 0
                           ? d.pool + (((unsigned long long)md->off_hi << 32) | md->off_lo)
                           : (const uint4 *)(d.dense + (size_t)md->off_lo * d.NP);
    wave_copy16(dst, src, pb / 16u);
}

// one wave per received parcel; srcs[s] = {segment offset, parcel count, first global parcel index}
__global__ void k_x_unpack(DS d, XArgs x, const uint8_t *buf, const ulonglong2 *srcs, uint32_t nsrc,
                           uint32_t total) {
    const uint32_t i = wave_gid();
    if (i >= total) return;
    uint32_t s = 0;
    while (s + 1 < nsrc && i >= (uint32_t)srcs[s + 1].y) s++;
    const uint8_t *seg = buf + srcs[s].x;
    const uint32_t k = i - (uint32_t)srcs[s].y;
    const Parcel *pc = (const Parcel *)(seg + ((const uint32_t *)seg)[k]);
    const Parcel h = *pc;
    const uint4 *payload = (const uint4 *)(pc + 1);
    MsgDesc md;
    md.kind = h.kind; md.len = h.len; md.off_lo = md.off_hi = 0;
    if (h.kind == 0 && h.len) {                                    // change records → local pool
        const unsigned long long off = pool_alloc(d, h.len);
        if (off == ~0ull) return;
        // (re-tagged with this shard's hot slots: the sender's tags name the sender shard's slots, DS record format)
        for (uint32_t i = lane_id(); i < h.len; i += 64 * SNAP_MB) {
            uint4 v[SNAP_MB];
            uint32_t hk[SNAP_MB];
#pragma unroll
            for (int u = 0; u < SNAP_MB; u++) v[u] = i + 64u * u < h.len ? payload[i + 64u * u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int u = 0; u < SNAP_MB; u++) hk[u] = i + 64u * u < h.len ? hot_slot(d, rec_m(v[u])) : SRC_NONE;
#pragma unroll
            for (int u = 0; u < SNAP_MB; u++)
                if (i + 64u * u < h.len) d.pool[off + i + 64u * u] = rec_retag(v[u], tag_of_slot(hk[u]));
        }
        md.off_lo = (uint32_t)off;
        md.off_hi = (uint32_t)(off >> 32);
    } else if (h.kind == 1) {                                      // dense snapshot → local dense pool
        uint32_t slot = 0;
        if (lane_id() == 0) slot = atomicAdd(d.dense_cur, 1u);
        slot = (uint32_t)__shfl((int)slot, 0, 64);
        if (slot >= d.dense_cap) {
            if (lane_id() == 0) atomicOr(d.err, E_DENSE);
            return;
        }
        uint4 *dst = (uint4 *)(d.dense + (size_t)slot * d.NP);
        wave_copy16(dst, payload, d.NP / 4);
        if (lane_id() == 0) {
            d.dense_meta[slot] = make_uint4(h.meta.x, h.meta.y, h.meta.z, 0u);   // w: a local alias only
            d.dense_len[slot] = h.dlen;
            d.dense_last[slot] = h.dlast;
            d.dense_cs[slot] = h.dcs;
        }
        md.off_lo = slot;
    }
    __threadfence_block();
    if (lane_id() != 0) return;
    switch (h.type) {
    case P_REQ:
    case P_REQ2: {
        const uint32_t o = h.type == P_REQ ? h.idx : h.idx / d.K;
        const uint32_t pend = (h.sI >> 31) ? (0x80000000u | h.sC) : SRC_NONE;
        if (h.type == P_REQ) { x.sdesc[o] = md; x.sI[o] = h.sI & 0x7FFFFFFFu; x.sC[o] = h.sC; x.sS[o] = pend; }
        else { x.sdesc2[o] = md; x.sI2[o] = h.sI & 0x7FFFFFFFu; x.sC2[o] = h.sC; x.sS2[o] = pend; }
        const uint32_t p = atomicAdd(x.npairs, 1u);
        if (p < x.keycap) x.keys[p] = ((unsigned long long)h.key << 32) | h.idx;
        else atomicOr(d.err, E_XCAP);
        break;
    }
    case P_RESP: x.rdesc[h.idx] = md; break;
    case P_RESP2: x.rdesc2[h.idx] = md; break;
    case P_NEED: {
        x.need[h.idx] = 1;
        const uint32_t p = atomicAdd(x.needcnt, 1u);
        if (p < x.needcap) x.needlist[p] = make_uint2(h.idx, h.key);
        else atomicOr(d.err, E_XCAP);
        break;
    }
    case P_SNAP: x.snapdesc[h.idx] = md; break;
    case P_HEALROW: x.hdesc[1] = md; break;
    case P_PING: x.hdesc[5] = md; x.hsics[2] = h.sI; x.hsics[3] = h.sC; break;
    case P_CSREQ: {
        const uint32_t p = atomicAdd(x.csreqcnt, 1u);
        if (p < x.csreqcap) x.csreq[p] = make_uint4(h.idx, h.key, h.sI, 0);
        else atomicOr(d.err, E_XCAP);
        break;
    }
    case P_CSRESP: x.rcs[h.idx] = h.key; break;
    default: break;
    }
}

// deferred full-sync decisions waiting on a remote sender's lazy C_o: ask the owner shard
__global__ void k_x_csreq(DS d, const uint4 *defer, const uint32_t *defer_cnt, int phase, uint4 *items, uint32_t *cnt,
                          uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *defer_cnt) return;
    const uint4 e = defer[i];
    if (!(e.w & 0x80000000u) || !(e.z & 0x80000000u)) return;
    const uint32_t ri = e.x & 0x7FFFFFFFu, o = phase == 0 ? ri : ri / d.K;
    x_push(items, cnt, cap, d.err, make_uint4(owner_of(d, o), P_CSREQ, o, e.z & 0x7FFFFFFFu));
}

// requested snapshots → checksum list (after the local deferred ids)
__global__ void k_csreq_ids(DS d, const uint4 *csreq, const uint32_t *csreqcnt, uint32_t *list, uint32_t *cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *csreqcnt) return;
    if (csreq[i].y < d.dense_cap) list[atomicAdd(cnt, 1u)] = d.NL + csreq[i].y;   // else hashed on the side stream
}

// answers to the requesting shards
__global__ void k_x_csresp(DS d, const uint4 *csreq, const uint32_t *csreqcnt, uint4 *items, uint32_t *cnt,
                           uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *csreqcnt) return;
    const uint4 r = csreq[i];
    x_push(items, cnt, cap, d.err, make_uint4(r.z, P_CSRESP, r.x, d.dense_cs[r.y]));
}

// responses of local receivers to remote senders (after the receive waves resolved them)
__global__ void k_x_resp(DS d, const unsigned long long *keys, uint32_t n, int phase, uint4 *items, uint32_t *cnt,
                         uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long k = keys[i];
    if ((uint32_t)(k >> 32) >= d.N) return;
    const uint32_t v = (uint32_t)k;
    const uint32_t o = phase == 0 ? v : v / d.K;
    const uint32_t r = owner_of(d, o);
    if (r != d.rank) x_push(items, cnt, cap, d.err, make_uint4(r, phase == 0 ? P_RESP : P_RESP2, v, 0));
}

// reverse-full-sync sources held by other shards: one request per distinct source
__global__ void k_x_need(DS d, const uint8_t *need, uint4 *items, uint32_t *cnt, uint32_t cap) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= d.N || !need[o]) return;
    const uint32_t r = owner_of(d, o);
    if (r != d.rank) x_push(items, cnt, cap, d.err, make_uint4(r, P_NEED, o, d.rank));
}

// snapshots for the shards that requested them (sources are local rows, snapshotted by k_jobs_snap)
__global__ void k_x_snap(DS d, const uint2 *needlist, const uint32_t *needcnt, uint4 *items, uint32_t *cnt,
                         uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *needcnt) return;
    const uint2 e = needlist[i];
    x_push(items, cnt, cap, d.err, make_uint4(e.y, P_SNAP, e.x, 0));
}

__global__ void k_x_item(DS d, uint4 it, uint4 *items, uint32_t *cnt, uint32_t cap) {
    if (threadIdx.x == 0) x_push(items, cnt, cap, d.err, it);
}

}  // namespace swimdev
