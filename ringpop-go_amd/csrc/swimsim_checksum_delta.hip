// swimsim_checksum_delta.hip — phase C FarmHash-32 (memberlist.go:83-128, go-farm Fingerprint32) for launches of many
// rows that are nearly equal: the reference-row ("delta") path. Included by swimsim_checksum.hip.
//
// The rows hashed in one round are views of the same membership: in a cascade round a row differs from the
// column-wise majority of the rows in 0.1-100 of 65,536 members (tools/delta_probe.py, profiles/r03_delta_probe.json).
// The FarmHash chain is still one sequential chain per row, but everything the chain consumes besides its own state
// is a function of 32 string bytes (the block's 20 and the next block's first 12). Outside the few blocks whose 32
// bytes touch a differing record, a row's string IS the reference string S_B shifted by the row's accumulated
// record-length difference s, so the block's premixed values are those of S_B at byte offset 20k - s:
//
//   k_csd_ref     reference words B: per member, the Boyer-Moore majority of up to 31 rows sampled from the launch
//   (hipcub)      O_B: B's record offsets (exclusive sum of B's record lengths; O_B[N] = |S_B|)
//   k_csd_string  S_B, B's checksum string, materialised once per launch (2.5 MB at 65,536 members)
//   k_csd_scan    one wave per row: the members whose record differs from B's (one coalesced pass over the row),
//                 merged into runs of "exception" blocks (blocks whose 32 bytes meet a differing record, plus block 0
//                 and the row's last block, whose look-ahead is zero), and the premixed values of every exception
//                 block, generated from the row's own words
//   k_cs_delta    256 rows per workgroup, one workgroup per CU. Four hasher waves (lane = row, one wave per SIMD) run
//                 the chain in carried-sum form: 12 VALU instructions a block, its premixed values read from LDS at
//                 an address that advances by 24 bytes a block and jumps only where an exception run begins or ends.
//                 Four helper waves prepare, one super step (32 blocks) ahead: the window of S_B's premixed blocks at
//                 every phase (-s mod 20) the workgroup's rows use (shared by all 256 rows), the rows' exception
//                 blocks beside it, and each row's jump list.
// Rows the delta path cannot take (entry or LDS-slot overflow, a workgroup whose shifts spread too far) are flagged
// and re-hashed by the production kernels (k_checksum3 / k_checksum_q16); results are bit-exact either way.
//
// Carried-sum block (swimsim_checksum4.hip): with X = state + the block's first word of that lane,
//   F = 5 ror(X ^ M, 19);  Xf' = F_f + F_g + PF;  Xg' = F_g + Xf' + D;  Xh' = F_h + KH
//   M_g = M(c), M_f = M(b + e c1), M_h = M(d), PF = 2C + a + d + c', D = PG - PF = C + a + b' - c', KH = C + e + a'
// (a', b', c' = the next block's first words, zero after the last block, so that X ends as the state itself).

constexpr int CSD_SB = 32;            // blocks per super step
constexpr int CSD_ROWS = 256;         // rows per workgroup
constexpr int CSD_HW = 4;             // hasher waves (waves 0..3); helper waves 4..7 serve the same rows
constexpr int CSD_THREADS = 512;
constexpr int CSD_PWENT = 1280;       // premixed S_B blocks per window buffer (phases x positions)
// exception slots per helper wave per buffer: differing members are column-correlated (the members whose state is
// in flux differ in many rows at once), so a super step can hold a run of 3-4 exception blocks in every row
constexpr int CSD_EXW = 384;
constexpr int CSD_NJ = 6;             // jumps per row per super step (block 0, then a start and an end per run)
constexpr int CSD_E = 8;              // exception entries a helper lane holds in registers
constexpr uint32_t CSD_NOJ = 0xFFFFu; // unused jump slot
constexpr uint32_t CSD_JB = 128;      // jump word: block i << 16 | (target - 3 i + CSD_JB), target in uint2 units
constexpr uint32_t CSD_C = 0xe6546b64u;
constexpr uint32_t CSD_MIN_ROWS = 1024; // launches of fewer rows keep the production kernels
// LDS of k_cs_delta in uint2 units: two window buffers, then 2 x 4 exception regions
constexpr int CSD_EXB = 2 * CSD_PWENT * 3;
constexpr int CSD_LDS2 = CSD_EXB + 2 * CSD_HW * CSD_EXW * 3;

// per listed row: what k_csd_scan found (32 B)
struct CsdRow {
    uint32_t ecnt;       // exception entries
    int32_t smin, smax;  // shift range of the clean blocks
    uint32_t phmask;     // phases (-s mod 20) of the clean blocks
    uint32_t flags;      // nonzero: the delta path does not hash this row
    uint32_t a0, b0, c0; // the string's first three words
};
// flags
constexpr uint32_t CSD_F_SHORT = 1, CSD_F_ECAP = 2, CSD_F_PLAN = 4, CSD_F_BATCH = 8, CSD_F_SLOTS = 16, CSD_F_JUMPS = 32,
                   CSD_F_WIN = 64, CSD_NFLAGS = 7;

struct CsdArgs {
    const uint32_t *B;        // [NP] reference words
    const uint32_t *OB;       // [N+1] reference record offsets, OB[N] = |S_B|
    const uint32_t *SBw;      // S_B as little-endian words, zero padded (sbw_words of them)
    uint32_t sbw_words;
    uint4 *ent;               // [rows][ecap] exception entries, 2 uint4 each: {k, s_after, Mg, D}, {Mf, PF, Mh, KH}
    CsdRow *rinfo;            // [rows]
    uint32_t ecap;
    uint32_t *fb_list, *fb_cnt; // rows left to the production kernels; fb_cnt[1 + b]: rows with flag bit b
};

__device__ __forceinline__ const uint32_t *csd_row(const DS &d, uint32_t id) {
    return id < d.NL ? d.mw + (size_t)id * d.NP : d.dense + (size_t)(id - d.NL) * d.NP;
}
__device__ __forceinline__ uint32_t csd_len(const DS &d, uint32_t id) {
    return id < d.NL ? d.clen[id] : d.dense_len[id - d.NL];
}
__device__ __forceinline__ uint32_t csd_reclen(const DS &d, uint32_t w) { return (uint32_t)reclen(d, w & 7u, w >> 3); }
// rows equal at member m in the checksum string: the same word, or a record in neither
__device__ __forceinline__ bool csd_same(uint32_t a, uint32_t b) { return a == b || ((a & 7u) >= 4u && (b & 7u) >= 4u); }
__device__ __forceinline__ uint32_t csd_phase(int32_t s) { return (uint32_t)(((-s) % 20 + 20) % 20); }
__device__ __forceinline__ int32_t csd_floordiv20(int32_t x) { return x >= 0 ? x / 20 : -((-x + 19) / 20); }

__device__ __forceinline__ void csd_premix(uint32_t a, uint32_t b, uint32_t c, uint32_t dd, uint32_t e, uint32_t an,
                                           uint32_t bn, uint32_t cn, uint32_t (&v)[6]) {
    v[0] = fh_m(c);
    v[1] = CSD_C + a + bn - cn;
    v[2] = fh_m(b + e * FH_C1);
    v[3] = 2u * CSD_C + a + dd + cn;
    v[4] = fh_m(dd);
    v[5] = CSD_C + e + an;
}

__global__ void k_ctr_add(DS d, int c, unsigned long long v) { ctr_add(d, c, v); }

// ---------------------------------------------------------------------------------------------------------------
// reference row and reference string
// ---------------------------------------------------------------------------------------------------------------
__global__ void k_csd_ref(DS d, const uint32_t *list, uint32_t n, uint32_t *B, uint32_t *Lb) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m > d.N) return;
    if (m == d.N) { Lb[m] = 0; return; }
    const uint32_t S = min(n, 31u);
    uint32_t cand = 0, c = 0;
    for (uint32_t s = 0; s < S; s++) {
        const uint32_t id = list[(uint32_t)(((uint64_t)s * n) / S)];
        const uint32_t w = csd_row(d, id)[m];
        if (c == 0) { cand = w; c = 1; }
        else c += w == cand ? 1u : 0xFFFFFFFFu;
    }
    B[m] = cand;
    Lb[m] = csd_reclen(d, cand);
}

template <int W>
__global__ void k_csd_string(DS d, const uint32_t *B, const uint32_t *OB, uint8_t *SB) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= d.N) return;
    uint32_t R[CS_RW];
    const uint32_t L = record<W>(d, m, B[m], R);
    uint8_t *o = SB + OB[m];
    for (uint32_t b = 0; b < L; b++) {
        uint32_t w = 0;
#pragma unroll
        for (int i = 0; i < CS_RW; i++) w = (b >> 2) == (uint32_t)i ? R[i] : w;
        o[b] = (uint8_t)(w >> (8u * (b & 3u)));
    }
}

// ---------------------------------------------------------------------------------------------------------------
// k_csd_scan: one wave per row
// ---------------------------------------------------------------------------------------------------------------
// premixed entries of blocks klo..khi of one row (one lane): the row's string from byte 20 klo, which is byte o0 of
// member m0's record, as a word stream through a window of 8 words. Block j of the run is words [5j, 5j + 8) of the
// stream (words [5j, 5j + 5) and a zero look-ahead for the row's last block kl).
template <int W>
__device__ void csd_run_entries(const DS &d, const uint32_t *row, uint32_t m0, uint32_t o0, uint32_t klo, uint32_t khi,
                                uint32_t kl, int32_t s_after, uint4 *out, CsdRow *ri) {
    const uint32_t N = d.N;
    const uint32_t nbk = khi - klo + 1;
    const bool tail0 = khi == kl;
    uint32_t win[8] = {0, 0, 0, 0, 0, 0, 0, 0}, nw = 0, done = 0;
    uint32_t ready = (nbk == 1 && tail0) ? 5u : 8u;                 // stream words block `done` needs
    uint64_t acc = 0;
    uint32_t nacc = 0;
    auto push = [&](uint32_t w) {
#pragma unroll
        for (int q = 0; q < 7; q++) win[q] = win[q + 1];
        win[7] = w;
        nw++;
        if (done < nbk && nw == ready) {
            const bool z = tail0 && done == nbk - 1;               // words a..e at win[0..4], or win[3..7]
            const uint32_t wa = z ? win[3] : win[0], wb = z ? win[4] : win[1], wc = z ? win[5] : win[2],
                           wd = z ? win[6] : win[3], we = z ? win[7] : win[4];
            uint32_t v[6];
            csd_premix(wa, wb, wc, wd, we, z ? 0u : win[5], z ? 0u : win[6], z ? 0u : win[7], v);
            out[2 * done] = make_uint4(klo + done, (uint32_t)s_after, v[0], v[1]);
            out[2 * done + 1] = make_uint4(v[2], v[3], v[4], v[5]);
            if (klo + done == 0) { ri->a0 = wa; ri->b0 = wb; ri->c0 = wc; }
            done++;
            ready = (tail0 && done == nbk - 1) ? 5u * done + 5u : 5u * done + 8u;
        }
    };
    uint32_t m = m0, o = o0;
    while (done < nbk) {
        if (m < N) {
            uint32_t R[CS_RW];
            const uint32_t L = record<W>(d, m, row[m], R);
#pragma unroll
            for (int i = 0; i < CS_RW; i++) {
                const uint32_t lo = max(o, 4u * i), hi = min(L, 4u * i + 4u);
                if (hi > lo) {
                    const uint32_t nb = hi - lo;
                    const uint32_t v = R[i] >> (8u * (lo - 4u * i));
                    const uint32_t vm = nb == 4 ? v : (v & ((1u << (8u * nb)) - 1u));
                    acc |= (uint64_t)vm << (8u * nacc);
                    nacc += nb;
                    if (nacc >= 4) {
                        push((uint32_t)acc);
                        acc >>= 32;
                        nacc -= 4;
                    }
                }
            }
        } else {                                                    // past the last member: zero bytes
            push((uint32_t)acc);
            acc = 0;
            nacc = 0;
        }
        m++;
        o = 0;
    }
}

template <int W>
__global__ void __launch_bounds__(256) k_csd_scan(DS d, const uint32_t *list, uint32_t n, CsdArgs a) {
    // CSD_SU chunks of 64 members per pass, their loads in flight together (a row is one 256-KB stream). Chunks with
    // differing members are staged in LDS, and the pass's diffs are walked by a loop that is not unrolled; runs wait
    // in LDS for their entries, generated (one lane per run) between passes.
    constexpr uint32_t CSD_SU = 16, RUNCAP = 256, RUNFLUSH = 128;
    __shared__ uint32_t runs[4][RUNCAP][6];                         // {klo, khi, m0, o0, s_after, first entry}
    __shared__ uint32_t stw[4][CSD_SU][64], stb[4][CSD_SU][64];     // staged row / reference words of a pass
    __shared__ uint64_t stm[4][CSD_SU];                             // their diff masks
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t i = blockIdx.x * 4 + wv;
    if (i >= n) return;
    const uint32_t id = list[i];
    const uint32_t *row = csd_row(d, id);
    CsdRow *ri = a.rinfo + i;
    uint4 *ent = a.ent + (size_t)i * a.ecap * 2;
    const uint32_t len = csd_len(d, id);
    const uint32_t N = d.N;
    if (len <= 24) {                                                // FarmHash's short-string paths: not ours
        if (lane == 0) { ri->ecnt = 0; ri->flags = CSD_F_SHORT; ri->smin = 0; ri->smax = 0; ri->phmask = 1; }
        return;
    }
    const uint32_t kl = (len - 1) / 20 - 1;                         // the row's last chain block
    int32_t s = 0;                                                  // row offset - B offset of the clean bytes here
    uint32_t rlo = 0, rhi = 0, rm0 = 0, ro0 = 0;                    // the open run (block 0 always begins one)
    uint32_t nruns = 0, e = 0, flags = 0, phm = 0;
    int32_t smin = 0x7FFFFFFF, smax = -0x7FFFFFFF - 1;
    auto wsync = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto flush = [&]() {
        wsync();
        for (uint32_t q0 = 0; q0 < nruns; q0 += 64) {
            if (q0 + lane < nruns) {
                const uint32_t *q = runs[wv][q0 + lane];
                csd_run_entries<W>(d, row, q[2], q[3], q[0], q[1], kl, (int32_t)q[4], ent + 2 * q[5], ri);
            }
        }
        wsync();
        nruns = 0;
    };
    auto close_run = [&](int32_t s_after) {
        const uint32_t nb = rhi - rlo + 1;
        if (e + nb > a.ecap || nruns == RUNCAP) { flags |= CSD_F_ECAP; return; }
        if (lane == 0) {
            uint32_t *q = runs[wv][nruns];
            q[0] = rlo; q[1] = rhi; q[2] = rm0; q[3] = ro0; q[4] = (uint32_t)s_after; q[5] = e;
        }
        if (rhi < kl) {                                             // clean blocks follow at this shift
            smin = min(smin, s_after);
            smax = max(smax, s_after);
            phm |= 1u << csd_phase(s_after);
        }
        e += nb;
        nruns++;
    };
    auto diff = [&](uint32_t mm, uint32_t wm, uint32_t bm) {
        const int32_t Lr = (int32_t)csd_reclen(d, wm), Lbm = (int32_t)csd_reclen(d, bm);
        const int32_t x = (int32_t)a.OB[mm] + s, y = x + Lr;        // the record's bytes in the row: [x, y)
        // blocks whose 32 bytes [20k, 20k + 32) meet [x, y) (or straddle x when the record is empty)
        const int32_t klo = x >= 32 ? (x - 32) / 20 + 1 : 0;
        int32_t khi = y >= 1 ? (y - 1) / 20 : -1;
        if (khi > (int32_t)kl) khi = (int32_t)kl;
        if (klo <= (int32_t)kl && khi >= klo) {
            if ((uint32_t)klo <= rhi + 1) {
                rhi = max(rhi, (uint32_t)khi);
            } else {
                close_run(s);
                // the new run starts at row byte p = 20 klo, in the clean bytes before mm (shift s): the record
                // holding B offset t = p - s is the last member below mm with O_B <= t
                const uint32_t t = (uint32_t)(20 * klo - s);
                uint32_t m0 = mm - 1;
                while (m0 > 0 && a.OB[m0] > t) m0--;
                rlo = (uint32_t)klo; rhi = (uint32_t)khi; rm0 = m0; ro0 = t - a.OB[m0];
            }
        }
        s += Lr - Lbm;
    };
    for (uint32_t c00 = 0; c00 < N && !flags; c00 += 64 * CSD_SU) {
        uint32_t wv_[CSD_SU], bv_[CSD_SU];
#pragma unroll
        for (uint32_t k = 0; k < CSD_SU; k++) {
            const uint32_t m = c00 + 64 * k + lane;
            wv_[k] = m < N ? row[m] : 0u;
            bv_[k] = m < N ? a.B[m] : 0u;
        }
        uint32_t any = 0;
#pragma unroll
        for (uint32_t k = 0; k < CSD_SU; k++) {
            const uint64_t mk = __ballot(c00 + 64 * k + lane < N && !csd_same(wv_[k], bv_[k]));
            if (mk) {
                stw[wv][k][lane] = wv_[k];
                stb[wv][k][lane] = bv_[k];
            }
            if (lane == 0) stm[wv][k] = mk;
            any |= mk ? 1u : 0u;
        }
        if (!any) continue;
        wsync();
        for (uint32_t k = 0; k < CSD_SU && !flags; k++) {
            uint64_t mask = stm[wv][k];
            while (mask && !flags) {                                // the chunk's differing members, in order
                const uint32_t l = (uint32_t)__builtin_ctzll(mask);
                mask &= mask - 1;
                diff(c00 + 64 * k + l, stw[wv][k][l], stb[wv][k][l]);
            }
        }
        wsync();
        if (nruns >= RUNFLUSH) flush();
    }
    if (!flags) {
        if (rhi + 1 >= kl) {
            rhi = kl;
        } else {                                                    // the last block: a run of its own
            close_run(s);
            const uint32_t t = (uint32_t)(20 * (int32_t)kl - s);
            uint32_t m0 = N - 1;
            while (m0 > 0 && a.OB[m0] > t) m0--;
            rlo = kl; rhi = kl; rm0 = m0; ro0 = t - a.OB[m0];
        }
        close_run(s);
    }
    if (!flags && nruns) flush();
    if (lane == 0) {
        ri->ecnt = e;
        ri->flags = flags;
        ri->smin = phm ? smin : 0;
        ri->smax = phm ? smax : 0;
        ri->phmask = phm ? phm : 1u;
    }
}

// ---------------------------------------------------------------------------------------------------------------
// k_cs_delta: the chains
// ---------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t csd_alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) {
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

template <int W>
__global__ void __launch_bounds__(CSD_THREADS) k_cs_delta(DS d, const uint32_t *list, const uint32_t *count, CsdArgs a) {
    __shared__ uint2 L2[CSD_LDS2];                       // window buffers, then exception regions (24-B entries)
    __shared__ uint32_t jl[2][CSD_ROWS][CSD_NJ];         // per row: jump words (CSD_JB); block CSD_NOJ: unused
    __shared__ uint32_t uni[2][CSD_HW];                  // per hasher wave: blocks where some lane jumps
    __shared__ uint32_t rflag[CSD_ROWS];
    __shared__ int32_t plan[4];
    __shared__ uint32_t phs[20];
    const uint32_t cnt = *count;
    const uint32_t g0 = blockIdx.x * CSD_ROWS;
    if (g0 >= cnt) return;                                          // uniform per workgroup
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const bool hasher = wave < (uint32_t)CSD_HW;
    const uint32_t hw = wave & 3u;
    const uint32_t r = hw * 64 + lane;                              // this lane's row
    const uint32_t gi = g0 + r;
    const bool valid = gi < cnt;
    const uint32_t id = list[valid ? gi : g0];
    const bool is_row = id < d.NL;
    const uint32_t *row = csd_row(d, id);
    const CsdRow ri = a.rinfo[valid ? gi : g0];
    const uint32_t len = csd_len(d, id);
    const uint32_t iters = len > 24 ? (len - 1) / 20 : 0u;
    const bool live = valid && ri.flags == 0 && iters > 0;

    // ---- plan: the workgroup's shift range and phases
    if (threadIdx.x == 0) { plan[0] = 0x7FFFFFFF; plan[1] = -0x7FFFFFFF - 1; plan[2] = 0; plan[3] = 0; }
    __syncthreads();
    if (hasher) {
        rflag[r] = live ? 0u : (ri.flags ? ri.flags : CSD_F_SHORT);
        if (live) {
            atomicMin(&plan[0], ri.smin);
            atomicMax(&plan[1], ri.smax);
            atomicOr((uint32_t *)&plan[2], ri.phmask);
            atomicMax((uint32_t *)&plan[3], iters);
        }
    }
    __syncthreads();
    int32_t smin = plan[0], smax = plan[1];
    uint32_t phm = (uint32_t)plan[2];
    const uint32_t maxit = (uint32_t)plan[3];
    if (phm == 0) { phm = 1; smin = 0; smax = 0; }
    const int32_t cmax = -csd_floordiv20(-smax), fmin = csd_floordiv20(smin);
    const int32_t joff = -cmax - 1;                                 // window of super step t: S_B blocks from t SB + joff
    const uint32_t JW = (uint32_t)(CSD_SB + cmax - fmin + 2);
    const uint32_t nph = (uint32_t)__popc(phm);
    const bool feasible = nph * JW <= (uint32_t)CSD_PWENT;
    const uint32_t T = feasible ? (maxit + CSD_SB - 1) / CSD_SB : 0u;
    if (threadIdx.x < 20 && ((phm >> threadIdx.x) & 1u)) phs[__popc(phm & ((1u << threadIdx.x) - 1u))] = threadIdx.x;
    if (!feasible && hasher) rflag[r] |= CSD_F_PLAN;
    __syncthreads();

    if (!hasher) {
        // ================================= helpers =================================
        const uint32_t th = r;                                      // 0..255
        const uint32_t lenB = a.OB[d.N];
        const uint4 *ent = a.ent + (size_t)(valid ? gi : g0) * a.ecap * 2;
        const uint32_t ecnt = live ? ri.ecnt : 0u;
        int32_t s = 0;
        uint32_t cur = 0;
        // the next CSD_E entries [cur, cur + CSD_E): block, shift after, values
        uint32_t bk[CSD_E];
        int32_t bs[CSD_E];
        uint2 bv[CSD_E][3];
        auto load_batch = [&]() {
#pragma unroll
            for (int q = 0; q < CSD_E; q++) {
                if (cur + q < ecnt) {
                    const uint4 x = ent[2 * (cur + q)], y = ent[2 * (cur + q) + 1];
                    bk[q] = x.x; bs[q] = (int32_t)x.y;
                    bv[q][0] = make_uint2(x.z, x.w); bv[q][1] = make_uint2(y.x, y.y); bv[q][2] = make_uint2(y.z, y.w);
                } else {
                    bk[q] = 0xFFFFFFFFu; bs[q] = 0;
                    bv[q][0] = bv[q][1] = bv[q][2] = make_uint2(0u, 0u);
                }
            }
        };
        load_batch();
        // window entries q = th + 256 u of every super step; their S_B words are loaded one super step ahead (a
        // global load takes longer than a super step's 32 blocks of chain)
        constexpr int QL = (CSD_PWENT + 255) / 256;
        const uint32_t nent = nph * JW;
        uint32_t xs[QL][9];
        auto entry_off = [&](uint32_t tp, uint32_t q) -> int32_t {
            const uint32_t slot = q / JW, jr = q - slot * JW;
            return 20 * ((int32_t)(tp * CSD_SB) + joff + (int32_t)jr) + (int32_t)phs[slot];
        };
        auto load_win = [&](uint32_t tp) {
#pragma unroll
            for (int u = 0; u < QL; u++) {
                const uint32_t q = th + 256u * u;
                const int32_t off = q < nent ? entry_off(tp, q) : -1;
                const bool in = off >= 0 && (uint32_t)off + 32u <= lenB;
                const uint32_t wi = in ? (uint32_t)off >> 2 : 0u;
#pragma unroll
                for (int k = 0; k < 9; k++) xs[u][k] = in ? a.SBw[wi + k] : 0u;
            }
        };
        load_win(0);
        auto prepare = [&](uint32_t tp) {
            const uint32_t bp = tp & 1u;
            const int32_t jlo = (int32_t)(tp * CSD_SB) + joff;
            uint2 *pw = L2 + bp * CSD_PWENT * 3;
            // (a) S_B's premixed blocks at every phase in use, positions jlo .. jlo + JW - 1
#pragma unroll
            for (int u = 0; u < QL; u++) {
                const uint32_t q = th + 256u * u;
                if (q < nent) {
                    const uint32_t sh = (uint32_t)entry_off(tp, q) & 3u;
                    uint32_t w8[8], v[6];
#pragma unroll
                    for (int k = 0; k < 8; k++) w8[k] = csd_alignbyte(xs[u][k + 1], xs[u][k], sh);
                    csd_premix(w8[0], w8[1], w8[2], w8[3], w8[4], w8[5], w8[6], w8[7], v);
                    pw[3 * q] = make_uint2(v[0], v[1]);
                    pw[3 * q + 1] = make_uint2(v[2], v[3]);
                    pw[3 * q + 2] = make_uint2(v[4], v[5]);
                }
            }
            load_win(tp + 1);
            // (b) this row's exception blocks and jumps in blocks K0 .. K0 + SB - 1
            const uint32_t K0 = tp * CSD_SB;
            const bool act = rflag[r] == 0u && K0 < iters;
            uint32_t ne = 0;
#pragma unroll
            for (int q = 0; q < CSD_E; q++) ne += (act && bk[q] < K0 + CSD_SB) ? 1u : 0u;
            uint32_t fl = 0;
            if (ne == (uint32_t)CSD_E && cur + CSD_E < ecnt) fl |= CSD_F_BATCH;   // more than the batch holds
            // exception slots of the helper wave: exclusive prefix of ne over its 64 lanes
            uint32_t pre = ne;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)pre, off, 64);
                if (lane >= (uint32_t)off) pre += y;
            }
            const uint32_t sb = pre - ne;
            if (sb + ne > (uint32_t)CSD_EXW) fl |= CSD_F_SLOTS;
            const uint32_t exb = CSD_EXB + (bp * CSD_HW + hw) * CSD_EXW * 3;   // uint2 index of slot 0
            uint32_t jw[CSD_NJ], nj = 0;
#pragma unroll
            for (int q = 0; q < CSD_NJ; q++) jw[q] = CSD_NOJ << 16;
            auto add_jump = [&](uint32_t i, uint32_t t) {
#pragma unroll
                for (int q = 0; q < CSD_NJ; q++)
                    if ((uint32_t)q == nj) jw[q] = (i << 16) | (t - 3u * i + CSD_JB);
                nj++;
            };
            // clean target of block k at shift sh: uint2 index of S_B's premixed block at offset 20 k - sh
            auto clean = [&](uint32_t k, int32_t sh) -> uint32_t {
                const int32_t tB = 20 * (int32_t)k - sh;
                const int32_t j = csd_floordiv20(tB);
                const uint32_t ph = (uint32_t)(tB - 20 * j);
                const int32_t jr = j - jlo;
                if (!((phm >> ph) & 1u) || jr < 0 || jr >= (int32_t)JW) { fl |= CSD_F_WIN; return bp * CSD_PWENT * 3; }
                const uint32_t slot = (uint32_t)__popc(phm & ((1u << ph) - 1u));
                return bp * CSD_PWENT * 3 + 3u * (slot * JW + (uint32_t)jr);
            };
            if (act && !fl) {
                add_jump(0, (ne && bk[0] == K0) ? exb + 3u * sb : clean(K0, s));
#pragma unroll
                for (int q = 0; q < CSD_E; q++) {
                    if ((uint32_t)q < ne) {
                        const uint32_t k = bk[q], i = k - K0, slot = exb + 3u * (sb + q);
                        L2[slot] = bv[q][0];
                        L2[slot + 1] = bv[q][1];
                        L2[slot + 2] = bv[q][2];
                        const bool starts = q == 0 ? i > 0 : bk[q - 1] + 1 != k;
                        if (starts) add_jump(i, slot);
                        s = bs[q];
                        const bool ends = (uint32_t)(q + 1) < ne ? bk[q + 1] != k + 1 : true;
                        if (ends && i + 1 < (uint32_t)CSD_SB) add_jump(i + 1, clean(k + 1, s));
                    }
                }
                if (nj > (uint32_t)CSD_NJ) fl |= CSD_F_JUMPS;
            }
            if (!act || fl) {                                       // a valid window address, nothing else
#pragma unroll
                for (int q = 0; q < CSD_NJ; q++) jw[q] = q == 0 ? bp * CSD_PWENT * 3 + CSD_JB : CSD_NOJ << 16;
            }
            if (fl) rflag[r] |= fl;
            uint32_t um = 0;
#pragma unroll
            for (int q = 0; q < CSD_NJ; q++) {
                jl[bp][r][q] = jw[q];
                const uint32_t ji = jw[q] >> 16;
                um |= ji < (uint32_t)CSD_SB ? 1u << ji : 0u;
            }
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) um |= (uint32_t)__shfl_xor((int)um, off, 64);
            if (lane == 0) uni[bp][hw] = um;
            if (ne) {                                               // the next batch, needed one super step on
                cur += ne;
                load_batch();
            }
        };
        if (T > 0) prepare(0);
        lds_barrier();
        for (uint32_t t = 0; t < T; t++) {
            if (t + 1 < T) prepare(t + 1);
            lds_barrier();
        }
        return;
    }

    // ================================= hashers =================================
    __builtin_amdgcn_s_setprio(2);
    FH fh{0, 0, 0};
    uint32_t it2 = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, it2);
    uint32_t Xg = fh.g + ri.b0, Xf = fh.f + ri.c0, Xh = fh.h + ri.a0;
    const uint32_t myit = live ? iters : 0u;
    lds_barrier();                                                  // super step 0 prepared
    for (uint32_t t = 0; t < T; t++) {
        const uint32_t bp = t & 1u, K0 = t * CSD_SB;
        uint32_t ji[CSD_NJ], jt[CSD_NJ];
#pragma unroll
        for (int q = 0; q < CSD_NJ; q++) { const uint32_t x = jl[bp][r][q]; ji[q] = x >> 16; jt[q] = (x & 0xFFFFu) - CSD_JB; }
        const uint32_t u = __builtin_amdgcn_readfirstlane(uni[bp][hw]);
        uint32_t base = jt[0];                                      // every row jumps at block 0
        auto apply = [&](uint32_t i) {
#pragma unroll
            for (int q = 1; q < CSD_NJ; q++) base = ji[q] == i ? jt[q] : base;
        };
        const bool full = __all(myit == 0u || K0 + CSD_SB <= myit);
        uint2 v[3][3];
        auto fetch = [&](int i) {
            const uint2 *p = L2 + base + 3 * i;
            v[i % 3][0] = p[0];
            v[i % 3][1] = p[1];
            v[i % 3][2] = p[2];
        };
        auto body = [&](auto FULLC) {
            constexpr bool FULL = decltype(FULLC)::value;
            fetch(0);
            if ((u >> 1) & 1u) apply(1);
            fetch(1);
#pragma unroll
            for (int i = 0; i < CSD_SB; i++) {
                if (i + 2 < CSD_SB) {
                    if ((u >> (i + 2)) & 1u) apply((uint32_t)(i + 2));
                    fetch(i + 2);
                }
                const uint2 g = v[i % 3][0], f = v[i % 3][1], hh = v[i % 3][2];
                const uint32_t Fg = x5(ror32(Xg ^ g.x, 19)), Ff = x5(ror32(Xf ^ f.x, 19)), Fh = x5(ror32(Xh ^ hh.x, 19));
                const uint32_t nf = Ff + Fg + f.y;
                const uint32_t ng = Fg + nf + g.y;
                const uint32_t nh = Fh + hh.y;
                if (FULL || K0 + (uint32_t)i < myit) { Xf = nf; Xg = ng; Xh = nh; }
            }
        };
        if (full) body(std::integral_constant<bool, true>{});
        else body(std::integral_constant<bool, false>{});
        lds_barrier();
    }
    const bool mine = valid && rflag[r] == 0u;
    const uint32_t nmine = (uint32_t)__popcll(__ballot(mine));
    if (lane == 0 && nmine) ctr_add(d, C_X_CS_ROWS, (unsigned long long)nmine);   // rows this launch hashed
    if (!valid) return;
    if (!mine) {                                                    // left to the production kernels
        const uint32_t at = atomicAdd(a.fb_cnt, 1u);
        a.fb_list[at] = id;
        const uint32_t fl = rflag[r];
        for (uint32_t b = 0; b < CSD_NFLAGS; b++)
            if ((fl >> b) & 1u) atomicAdd(a.fb_cnt + 1 + b, 1u);
        return;
    }
    fh.h = Xh; fh.g = Xg; fh.f = Xf;
    const uint32_t hv = ok ? fh.fin() : 0u;
    if (is_row) {
        d.cs[id] = hv;
        d.dirty[id] = 0;
    } else {
        d.dense_cs[id - d.NL] = hv;
    }
}

template <int W>
void launch_csd_w(const DS &d, const uint32_t *list, uint32_t n, const uint32_t *count, const CsdArgs &a, hipStream_t s,
                  int part) {
    if (part == 0) {
        hipLaunchKernelGGL((k_csd_string<W>), dim3((d.N + 255) / 256), dim3(256), 0, s, d, a.B, a.OB, (uint8_t *)a.SBw);
    } else if (part == 1) {
        hipLaunchKernelGGL((k_csd_scan<W>), dim3((n + 3) / 4), dim3(256), 0, s, d, list, n, a);
    } else {
        hipLaunchKernelGGL((k_cs_delta<W>), dim3((n + CSD_ROWS - 1) / CSD_ROWS), dim3(CSD_THREADS), 0, s, d, list, count, a);
    }
}

void launch_csd(const DS &d, const uint32_t *list, uint32_t n, const uint32_t *count, const CsdArgs &a, hipStream_t s,
                int part) {
    switch (d.W) {
#define CS_CASE(Wv) case Wv: launch_csd_w<Wv>(d, list, n, count, a, s, part); break;
        CS_W_CASES(CS_CASE)
#undef CS_CASE
    default: break;
    }
}
