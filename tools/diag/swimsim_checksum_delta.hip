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
constexpr int CSD_PF = 4;             // blocks the chain waves' LDS reads run ahead
// k_cs_delta's workgroup: G row groups of 64 rows, each served by an h-chain wave, a g/f-chain wave and a helper wave.
// G = 4 (256 rows, one workgroup per CU). (A 64-row workgroup, G = 1, measured 5.8 / 6.0 ms against 9.4 / 14.9 ms for
// k_checksum_q16 at 12,288 / 16,384 light rows, but failed parity on the partition workload and is not launched.)
template <int G> struct CsdGeo {
    static constexpr int ROWS = 64 * G, THREADS = 192 * G;
    static constexpr int RING = G == 4 ? 2240 : 1600;   // premixed S_B blocks in the window ring (phases x (ring + mirror))
};
// exception slots per helper wave per buffer: differing members are column-correlated (the members whose state is
// in flux differ in many rows at once), so a super step can hold a run of 3-4 exception blocks in every row
constexpr int CSD_EXW = 320;
#ifndef CSD_NJ_DEF                    // (a build-time define for experiments with other slot counts; even)
#define CSD_NJ_DEF 6
#endif
constexpr int CSD_NJ = CSD_NJ_DEF;    // jumps per row per super step (block 0, then a start and an end per run)
static_assert(CSD_NJ % 2 == 0, "jump words are stored in pairs");
constexpr int CSD_E = 8;              // exception entries a helper lane holds in registers
constexpr uint32_t CSD_NOJ = 0xFFFFu; // unused jump slot
constexpr uint32_t CSD_JB = 128;      // jump word: block i << 16 | (target - 3 i + CSD_JB), target in uint2 units
constexpr int CSD_JWMAX = 160;        // window positions at most (the workgroup's shifts spread < 2,500 bytes)
constexpr int CSD_SBST = 5 * CSD_SB + 16;      // staged S_B words per super step (its SB new positions)
constexpr uint32_t CSD_C = 0xe6546b64u;
constexpr uint32_t CSD_MIN_ROWS = 1024; // launches of fewer rows keep the production kernels


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
    uint32_t dmode;           // diagnostics library only (swimsim_bench_checksum modes 31..46 = dmode + 30, garbage
                              // checksums): 1 helpers alone, 2 chains alone, 3 helpers without the exception work; bit 8:
                              // no barrier between super steps. Ignored by the product library (CSD_DMODE)
};

// the diagnostic split modes exist only in the diagnostics library (tools/libswimsim_diag.so); in the product
// library the mode is the constant 0 and its branches compile away
#ifdef SWIMSIM_DIAG
#define CSD_DMODE(a) ((a).dmode)
#else
#define CSD_DMODE(a) 0u
#endif

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

// the launch's mean distance from B, on CSD_NSAMPLE rows sampled evenly from the list: differing members counted
// into *out (one workgroup per sampled row). Decides whether the reference-row path pays for this launch.
constexpr uint32_t CSD_NSAMPLE = 64;
__global__ void __launch_bounds__(256) k_csd_sample(DS d, const uint32_t *list, uint32_t n, const uint32_t *B, uint32_t *out) {
    const uint32_t id = list[(uint32_t)(((uint64_t)blockIdx.x * n) / CSD_NSAMPLE)];
    const uint32_t *row = csd_row(d, id);
    uint32_t c = 0;
    for (uint32_t m = threadIdx.x; m < d.N; m += 256u) c += csd_same(row[m], B[m]) ? 0u : 1u;
    for (int off = 32; off > 0; off >>= 1) c += (uint32_t)__shfl_xor((int)c, off, 64);
    if ((threadIdx.x & 63u) == 0 && c) atomicAdd(out, c);
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
    constexpr uint32_t CSD_SU = 8, RUNCAP = 128, RUNFLUSH = 64;
    __shared__ uint32_t runs[4][RUNCAP][6];                         // {klo, khi, m0, o0, s_after, first entry}
    __shared__ uint32_t stw[4][CSD_SU][64];                         // staged row words of a pass
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
            if (mk) stw[wv][k][lane] = wv_[k];
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
                const uint32_t mm = c00 + 64 * k + l;
                diff(mm, stw[wv][k][l], a.B[mm]);
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

// one block of the coupled g and f lanes in carried-sum form, the two lanes' instructions interleaved (a wave issues in
// order: each of a pair's dependent successors then waits one instruction less)
__device__ __forceinline__ void csd_gf_step(uint32_t &Xg, uint32_t &Xf, uint32_t mg, uint32_t dd, uint32_t mf, uint32_t pf) {
    uint32_t tg, tf;
    asm volatile("v_xor_b32 %2, %0, %4\n\t"
                 "v_xor_b32 %3, %1, %6\n\t"
                 "v_alignbit_b32 %2, %2, %2, 19\n\t"
                 "v_alignbit_b32 %3, %3, %3, 19\n\t"
                 "v_lshl_add_u32 %2, %2, 2, %2\n\t"
                 "v_lshl_add_u32 %3, %3, 2, %3\n\t"
                 "v_add3_u32 %1, %3, %2, %7\n\t"
                 "v_add3_u32 %0, %2, %1, %5"
                 : "+v"(Xg), "+v"(Xf), "=&v"(tg), "=&v"(tf)
                 : "v"(mg), "v"(dd), "v"(mf), "v"(pf));
}
// one block of the h lane: Xh' = 5 ror(Xh ^ Mh, 19) + KH
__device__ __forceinline__ void csd_h_step(uint32_t &Xh, uint32_t mh, uint32_t kh) {
    asm volatile("v_xor_b32 %0, %0, %1\n\t"
                 "v_alignbit_b32 %0, %0, %0, 19\n\t"
                 "v_lshl_add_u32 %0, %0, 2, %0\n\t"
                 "v_add_u32 %0, %0, %2"
                 : "+v"(Xh)
                 : "v"(mh), "v"(kh));
}

template <int W, int G>
__global__ void __launch_bounds__(CsdGeo<G>::THREADS) k_cs_delta(DS d, const uint32_t *list, const uint32_t *count, CsdArgs a) {
    constexpr int CSD_ROWS = CsdGeo<G>::ROWS, CSD_HW = G, CSD_RING = CsdGeo<G>::RING;
    constexpr uint32_t HT = 64u * G;                     // helper threads
    // LDS in uint2 units: the window ring, then 2 x G exception regions
    constexpr int CSD_EXB = CSD_RING * 3;
    constexpr int CSD_LDS2 = CSD_EXB + 2 * CSD_HW * CSD_EXW * 3;
    __shared__ uint2 L2[CSD_LDS2];                       // window ring, then exception regions (24-B entries)
    __shared__ __attribute__((aligned(8))) uint32_t jl[2][CSD_ROWS][CSD_NJ];   // per row: jump words (CSD_JB);
                                                                                // block CSD_NOJ: unused
    __shared__ uint32_t uni[2][CSD_HW];                  // per row group of 64: blocks where some lane jumps
    __shared__ uint32_t xcnt[2][CSD_HW];                 // exception slots taken, per helper wave and buffer
    __shared__ uint32_t rflag[CSD_ROWS];
    __shared__ uint32_t xh[CSD_ROWS];                    // the h lanes' results, for the g/f waves' finalisation
    __shared__ int32_t plan[4];
    __shared__ uint32_t phs[20];
    __shared__ uint32_t sbst[2][CSD_SBST];               // S_B words of the window's new positions, staged ahead
    __shared__ uint32_t simd_n[4];
    const uint32_t cnt = *count;
    const uint32_t g0 = blockIdx.x * CSD_ROWS;
    if (g0 >= cnt) return;                                          // uniform per workgroup
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    // roles by SIMD: every SIMD should run one h-chain wave, one g/f-chain wave and one helper wave of the same 64
    // rows (two chain waves of one role on a SIMD would share its integer VALU issue, ~2.6 cycles an instruction,
    // and take twice as long). The hardware's placement of a workgroup's waves is read from HW_ID; if it is not
    // three waves per SIMD, the roles follow the wave index.
    uint32_t hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    const uint32_t simd = (hwid >> 4) & 3u;
    if (threadIdx.x < 4) simd_n[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t slot = 0;
    if (lane == 0) slot = atomicAdd(&simd_n[simd], 1u);
    slot = __builtin_amdgcn_readfirstlane(slot);
    __syncthreads();
    const bool even = G == 4 && simd_n[0] == 3u && simd_n[1] == 3u && simd_n[2] == 3u && simd_n[3] == 3u;
    const uint32_t role = even ? slot : wave / G;                   // 0: h chains, 1: g/f chains, 2: helpers
    const uint32_t hw = even ? simd : wave % G;
    if (G == 4 && !even && threadIdx.x == 0) ctr_add(d, C_NALL, 1ull);   // diagnostics: uneven placements
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
    if (role == 0) {
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
    // window of super step t: S_B blocks (20-byte positions) jlo0 + t SB + [0, JW), kept in a ring of R positions per
    // phase (+ a mirror of the first CSD_SB so that a row's 32 consecutive positions never wrap)
    const int32_t jlo0 = -cmax - 1;
    const uint32_t JW = (uint32_t)(CSD_SB + cmax - fmin + 2);
    const uint32_t R = JW + CSD_SB, RS = R + CSD_SB;
    const uint32_t nph = (uint32_t)__popc(phm);
    const bool feasible = nph * RS <= (uint32_t)CSD_RING && JW <= (uint32_t)CSD_JWMAX;
    const uint32_t T = feasible ? (maxit + CSD_SB - 1) / CSD_SB : 0u;
    if (threadIdx.x < 20 && ((phm >> threadIdx.x) & 1u)) phs[__popc(phm & ((1u << threadIdx.x) - 1u))] = threadIdx.x;
    if (!feasible && role == 0) rflag[r] |= CSD_F_PLAN;
    __syncthreads();
    // uint2 index of the ring slot holding position p (relative to jlo0) of phase slot ps
    // uint2 index of ring slot `slot` (< R) of phase slot ps
    auto ring_at = [&](uint32_t ps, uint32_t slot) -> uint32_t { return 3u * (ps * RS + slot); };

    if (role == 2) {
        // ================================= helpers =================================
        const uint32_t th = r;                                      // 0..255
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
        // premixed S_B block of phase slot ps into ring slot `slot` from words x[0..8] (shifted by sh bytes)
        auto put = [&](uint32_t ps, uint32_t slot, const uint32_t (&x)[9], uint32_t sh) {
            uint32_t w8[8], v[6];
#pragma unroll
            for (int k = 0; k < 8; k++) w8[k] = csd_alignbyte(x[k + 1], x[k], sh);
            csd_premix(w8[0], w8[1], w8[2], w8[3], w8[4], w8[5], w8[6], w8[7], v);
            const uint32_t at = ring_at(ps, slot);
            L2[at] = make_uint2(v[0], v[1]);
            L2[at + 1] = make_uint2(v[2], v[3]);
            L2[at + 2] = make_uint2(v[4], v[5]);
            if (slot < (uint32_t)CSD_SB) {                          // the mirror behind the ring's end
                const uint32_t mi = at + 3u * R;
                L2[mi] = make_uint2(v[0], v[1]);
                L2[mi + 1] = make_uint2(v[2], v[3]);
                L2[mi + 2] = make_uint2(v[4], v[5]);
            }
        };
        // window 0 (positions 0 .. JW - 1), from global memory once
        for (uint32_t q = th; q < nph * JW; q += HT) {
            const uint32_t ps = q / JW, p = q - ps * JW;
            const int32_t off = 20 * (jlo0 + (int32_t)p) + (int32_t)phs[ps];
            uint32_t x[9];
            const int32_t wi = off >= 0 ? off >> 2 : -1;
#pragma unroll
            for (int k = 0; k < 9; k++) x[k] = (wi >= 0 && (uint32_t)(wi + k) < a.sbw_words) ? a.SBw[wi + k] : 0u;
            put(ps, p, x, off >= 0 ? (uint32_t)off & 3u : 0u);
        }
        // the SB new positions of super step tp >= 1 are JW + (tp - 1) SB .. JW + tp SB - 1; their S_B words (from byte
        // 20 (jlo0 + JW + (tp - 1) SB) on) are loaded into registers two super steps ahead and staged in LDS one ahead
        constexpr int SL = (CSD_SBST + HT - 1) / HT;
        uint32_t sw[SL];
        auto load_sb = [&](uint32_t tp) {
            const int32_t wb = 5 * (jlo0 + (int32_t)JW + (int32_t)((tp - 1) * CSD_SB));
#pragma unroll
            for (int u = 0; u < SL; u++) {
                const int32_t w = wb + (int32_t)(th + HT * u);
                sw[u] = (th + HT * u < (uint32_t)CSD_SBST && w >= 0 && (uint32_t)w < a.sbw_words) ? a.SBw[w] : 0u;
            }
        };
        auto store_sb = [&](uint32_t tp) {
#pragma unroll
            for (int u = 0; u < SL; u++)
                if (th + HT * u < (uint32_t)CSD_SBST) sbst[tp & 1u][th + HT * u] = sw[u];
        };
        load_sb(1);
        store_sb(1);
        load_sb(2);
        lds_barrier();
        // ring slots of positions tp SB (the super step's first block at shift 0's window start) and JW + (tp - 1) SB
        // (its first new position), advanced by SB per super step instead of taken modulo R
        uint32_t ws = 0, nbs = JW;
        auto prepare = [&](uint32_t tp) {
            const uint32_t bp = tp & 1u;
            // (a) the window's SB new positions at every phase in use
            if (tp >= 1) {
                store_sb(tp + 1);
                load_sb(tp + 2);
                const uint32_t *st = sbst[bp];
                for (uint32_t q = th; q < nph * CSD_SB; q += HT) {
                    const uint32_t ps = q / CSD_SB, u = q - ps * CSD_SB;
                    const uint32_t lo = 20u * u + phs[ps], li = lo >> 2;
                    uint32_t x[9];
#pragma unroll
                    for (int k = 0; k < 9; k++) x[k] = st[li + k];
                    const uint32_t sl = nbs + u;
                    put(ps, sl >= R ? sl - R : sl, x, lo & 3u);
                }
            }
            // (b) this row's exception blocks and jumps in blocks K0 .. K0 + SB - 1
            const uint32_t K0 = tp * CSD_SB;
            const bool act = rflag[r] == 0u && K0 < iters && (CSD_DMODE(a) & 3u) != 3u;
            uint32_t ne = 0;
#pragma unroll
            for (int q = 0; q < CSD_E; q++) ne += (act && bk[q] < K0 + CSD_SB) ? 1u : 0u;
            uint32_t fl = 0;
            // more exception blocks in this super step than the batch holds (a run of adjacent differing records):
            // the rest are counted and read with synchronous loads (rare)
            const bool ovf = ne == (uint32_t)CSD_E && cur + CSD_E < ecnt;
            auto kat = [&](uint32_t e) -> uint32_t { return ((const uint32_t *)(ent + 2 * e))[0]; };
            if (__builtin_expect(__ballot(ovf) != 0, 0)) {
                if (ovf)
                    while (cur + ne < ecnt && kat(cur + ne) < K0 + CSD_SB) ne++;
            }
            // exception slots of the helper wave (only when some lane has exceptions): an LDS counter per wave and buffer
            const bool anyx = __ballot(ne > 0) != 0;
            uint32_t sb = 0;
            if (__builtin_expect(anyx, 0)) {
                if (lane == 0) xcnt[bp][hw] = 0u;                   // the wave's LDS operations complete in order
                if (ne) sb = atomicAdd(&xcnt[bp][hw], ne);
                if (sb + ne > (uint32_t)CSD_EXW) fl |= CSD_F_SLOTS;
            }
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
                const int32_t jr = j - (jlo0 + (int32_t)K0);
                if (!((phm >> ph) & 1u) || jr < 0 || jr >= (int32_t)JW) { fl |= CSD_F_WIN; return 0u; }
                const uint32_t sl = ws + (uint32_t)jr;
                return ring_at((uint32_t)__popc(phm & ((1u << ph) - 1u)), sl >= R ? sl - R : sl);
            };
            if (act && !fl) {
                add_jump(0, (ne && bk[0] == K0) ? exb + 3u * sb : clean(K0, s));
                if (__builtin_expect(anyx, 0)) {
                    // entry q of the super step (block k, shift after, values), its predecessor's and successor's blocks
                    auto place = [&](uint32_t q, uint32_t k, int32_t sa, uint2 v0, uint2 v1, uint2 v2, uint32_t kprev,
                                     uint32_t knext) {
                        const uint32_t i = k - K0, slot = exb + 3u * (sb + q);
                        L2[slot] = v0;
                        L2[slot + 1] = v1;
                        L2[slot + 2] = v2;
                        const bool starts = q == 0 ? i > 0 : kprev + 1 != k;
                        if (starts) add_jump(i, slot);
                        s = sa;
                        const bool ends = q + 1 < ne ? knext != k + 1 : true;
                        if (ends && i + 1 < (uint32_t)CSD_SB) add_jump(i + 1, clean(k + 1, s));
                    };
#pragma unroll
                    for (int q = 0; q < CSD_E; q++) {
                        if ((uint32_t)q < ne) {
                            const uint32_t kn = q + 1 < CSD_E ? bk[q + 1] : (ne > (uint32_t)CSD_E ? kat(cur + CSD_E) : 0u);
                            place((uint32_t)q, bk[q], bs[q], bv[q][0], bv[q][1], bv[q][2], q ? bk[q - 1] : 0u, kn);
                        }
                    }
                    for (uint32_t q = CSD_E; q < ne; q++) {                // the overflow, from global memory
                        const uint4 x = ent[2 * (cur + q)], y = ent[2 * (cur + q) + 1];
                        place(q, x.x, (int32_t)x.y, make_uint2(x.z, x.w), make_uint2(y.x, y.y), make_uint2(y.z, y.w),
                              kat(cur + q - 1), q + 1 < ne ? kat(cur + q + 1) : 0u);
                    }
                    if (nj > (uint32_t)CSD_NJ) fl |= CSD_F_JUMPS;
                }
            }
            if (!act || fl) {                                       // a valid window address, nothing else
#pragma unroll
                for (int q = 0; q < CSD_NJ; q++) jw[q] = q == 0 ? CSD_JB : CSD_NOJ << 16;
            }
            if (fl) rflag[r] |= fl;
            uint2 *jp = (uint2 *)&jl[bp][r][0];
#pragma unroll
            for (int q = 0; q < CSD_NJ; q += 2) jp[q / 2] = make_uint2(jw[q], jw[q + 1]);
            // blocks where some row of the wave jumps: block 0 always, the rest from the (few) rows with exceptions
            if (lane == 0) uni[bp][hw] = 1u;
            if (__builtin_expect(anyx, 0)) {
                uint32_t um = 0;
#pragma unroll
                for (int q = 1; q < CSD_NJ; q++) {
                    const uint32_t ji = jw[q] >> 16;
                    um |= ji < (uint32_t)CSD_SB ? 1u << ji : 0u;
                }
                if (um) atomicOr(&uni[bp][hw], um);
            }
            if (ne) {                                               // the next batch, needed one super step on
                cur += ne;
                load_batch();
            }
            ws = ws + CSD_SB >= R ? ws + CSD_SB - R : ws + CSD_SB;
            if (tp >= 1) nbs = nbs + CSD_SB >= R ? nbs + CSD_SB - R : nbs + CSD_SB;
        };
        const bool hidle = (CSD_DMODE(a) & 3u) == 2u;
        if (hidle) {                                                // diagnostics: every row at window slot 0, no jumps
#pragma unroll
            for (int q = 0; q < CSD_NJ; q++) { jl[0][r][q] = q == 0 ? CSD_JB : CSD_NOJ << 16; jl[1][r][q] = jl[0][r][q]; }
            if (lane == 0) { uni[0][hw] = 1u; uni[1][hw] = 1u; }
        }
        if (T > 0 && !hidle) prepare(0);
        lds_barrier();
        for (uint32_t t = 0; t < T; t++) {
            if (t + 1 < T && !hidle) prepare(t + 1);
            if (!(CSD_DMODE(a) & 8u)) lds_barrier();
        }
        lds_barrier();                                              // the h lanes' results published
        return;
    }

    // ================================= chains =================================
    // role 0 runs the h lane of its 64 rows, role 1 the coupled g and f lanes: two chain waves per SIMD, so that the
    // SIMD issues from one while the other waits on its dependencies (a lone wave issues at most every 4 cycles)
    __builtin_amdgcn_s_setprio(2);
    FH fh{0, 0, 0};
    uint32_t it2 = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, it2);
    uint32_t Xg = fh.g + ri.b0, Xf = fh.f + ri.c0, Xh = fh.h + ri.a0;
    const uint32_t myit = live ? iters : 0u;
    lds_barrier();                                                  // window 0 staged
    lds_barrier();                                                  // super step 0 prepared
    for (uint32_t t = 0; t < T; t++) {
        const uint32_t bp = t & 1u, K0 = t * CSD_SB;
        uint32_t ji[CSD_NJ], jt[CSD_NJ];
#pragma unroll
        for (int q = 0; q < CSD_NJ; q++) { const uint32_t x = jl[bp][r][q]; ji[q] = x >> 16; jt[q] = 8u * ((x & 0xFFFFu) - CSD_JB); }
        const uint32_t u = __builtin_amdgcn_readfirstlane(uni[bp][hw]);
        uint32_t base = jt[0];                                      // byte offset in L2; every row jumps at block 0
        auto apply = [&](uint32_t i) {
#pragma unroll
            for (int q = 1; q < CSD_NJ; q++) base = ji[q] == i ? jt[q] : base;
        };
        const bool full = __all(myit == 0u || K0 + CSD_SB <= myit);
        // CHK: some row of the wave jumps after block 0 in this super step (u > 1). The common case runs a body without
        // per-block tests: a test whose skip branch is taken on the common path costs an instruction-fetch restart
        auto run = [&](auto FULLC, auto ROLEC, auto CHKC) {
            constexpr bool FULL = decltype(FULLC)::value;
            constexpr int RL = decltype(ROLEC)::value;
            constexpr bool CHK = decltype(CHKC)::value;
            // reads run CSD_PF blocks ahead of the chain (LDS latency under twelve waves exceeds two blocks of chain)
            constexpr int PF = CSD_PF;
            uint2 v[PF + 1][2];
            auto fetch = [&](int i) {
                const uint2 *p = (const uint2 *)((const char *)L2 + base + 24 * i);
                if (RL == 0) {
                    v[i % (PF + 1)][0] = p[2];                      // {Mh, KH}
                } else {
                    v[i % (PF + 1)][0] = p[0];                      // {Mg, D}
                    v[i % (PF + 1)][1] = p[1];                      // {Mf, PF}
                }
            };
            fetch(0);
#pragma unroll
            for (int i = 1; i < PF; i++) {
                if (CHK && __builtin_expect((u >> i) & 1u, 0)) apply((uint32_t)i);
                fetch(i);
            }
#pragma unroll
            for (int i = 0; i < CSD_SB; i++) {
                if (i + PF < CSD_SB) {
                    if (CHK && __builtin_expect((u >> (i + PF)) & 1u, 0)) apply((uint32_t)(i + PF));
                    fetch(i + PF);
                }
                if (RL == 0) {
                    const uint2 hh = v[i % (PF + 1)][0];
                    if (FULL) csd_h_step(Xh, hh.x, hh.y);
                    else {
                        uint32_t n = Xh;
                        csd_h_step(n, hh.x, hh.y);
                        Xh = K0 + (uint32_t)i < myit ? n : Xh;
                    }
                } else {
                    const uint2 g = v[i % (PF + 1)][0], f = v[i % (PF + 1)][1];
                    if (FULL) csd_gf_step(Xg, Xf, g.x, g.y, f.x, f.y);
                    else {
                        uint32_t ng = Xg, nf = Xf;
                        csd_gf_step(ng, nf, g.x, g.y, f.x, f.y);
                        const bool act = K0 + (uint32_t)i < myit;
                        Xg = act ? ng : Xg;
                        Xf = act ? nf : Xf;
                    }
                }
            }
        };
        if ((CSD_DMODE(a) & 3u) != 1u) {
            using TT = std::integral_constant<bool, true>;
            using FF = std::integral_constant<bool, false>;
            const bool chk = u > 1u;
            if (role == 0) {
                if (full && !chk) run(TT{}, std::integral_constant<int, 0>{}, FF{});
                else if (full) run(TT{}, std::integral_constant<int, 0>{}, TT{});
                else run(FF{}, std::integral_constant<int, 0>{}, TT{});
            } else {
                if (full && !chk) run(TT{}, std::integral_constant<int, 1>{}, FF{});
                else if (full) run(TT{}, std::integral_constant<int, 1>{}, TT{});
                else run(FF{}, std::integral_constant<int, 1>{}, TT{});
            }
        }
        if (!(CSD_DMODE(a) & 8u)) lds_barrier();
    }
    if (role == 0) xh[r] = Xh;
    lds_barrier();                                                  // the h lanes' results published
    if (role == 0) return;
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
    fh.h = xh[r]; fh.g = Xg; fh.f = Xf;
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
        hipLaunchKernelGGL((k_cs_delta<W, 4>), dim3((n + 255) / 256), dim3(CsdGeo<4>::THREADS), 0, s, d, list, count, a);
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
