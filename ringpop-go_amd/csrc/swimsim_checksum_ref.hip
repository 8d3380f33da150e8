// swimsim_checksum_ref.hip — the reference-row pieces of phase C (memberlist.go:83-128, go-farm Fingerprint32) shared by
// the product's reference-row kernel (k_csr, swimsim_checksum_csr.hip) and the diagnostics library's k_cs_delta
// (tools/diag/swimsim_checksum_delta.hip). Included by swimsim_checksum.hip.
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
//
// Carried-sum block (swimsim_checksum4.hip): with X = state + the block's first word of that lane,
//   F = 5 ror(X ^ M, 19);  Xf' = F_f + F_g + PF;  Xg' = F_g + Xf' + D;  Xh' = F_h + KH
//   M_g = M(c), M_f = M(b + e c1), M_h = M(d), PF = 2C + a + d + c', D = PG - PF = C + a + b' - c', KH = C + e + a'
// (a', b', c' = the next block's first words, zero after the last block, so that X ends as the state itself).

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
    uint4 *ent;               // [rows][ecap] exception entries, 2 uint4 each: {Mg, D, Mf, PF}, {Mh, KH, k, s_after}
    CsdRow *rinfo;            // [rows]
    uint32_t ecap;
    uint32_t *fb_list, *fb_cnt; // rows left to the production kernels; fb_cnt[1 + b]: rows with flag bit b
    const uint32_t *ulist;    // divergent columns in member order (DS::colx), or null: k_csd_scan reads every column
    const uint32_t *ucnt;     // their number
    const uint4 *ucol;        // per divergent column c: {m, B[m], O_B[m], O_B[m - 1]} (k_csr_ucol)
    const uint32_t *uhk;      // per divergent column c: the hot slot of its member, or SRC_NONE (DS::uhk)
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

#ifdef SWIMSIM_DIAG
// (diagnostics library only: round 3's path declines launches on a sample; the product's path never declines)
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
#endif

// the divergent columns' scan table: what k_csd_scan needs of B at each, in one 16-B load
__global__ void k_csr_ucol(const uint32_t *ulist, const uint32_t *ucnt, const uint32_t *B, const uint32_t *OB, uint4 *ucol) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= *ucnt) return;
    const uint32_t m = ulist[c];
    ucol[c] = make_uint4(m, B[m], OB[m], OB[m ? m - 1u : 0u]);
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
            out[2 * done] = make_uint4(v[0], v[1], v[2], v[3]);
            out[2 * done + 1] = make_uint4(v[4], v[5], klo + done, (uint32_t)s_after);
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
// (five workgroups per CU: 96 VGPRs, five waves per SIMD for a latency-bound gather; with 8 chunks in flight and four
// waves per SIMD the path took 0.05-0.15 ms longer on real cascade rounds 14-20, with six it spilled)
#ifndef CSD_SCAN_MINB
#define CSD_SCAN_MINB 5
#endif
__global__ void __launch_bounds__(256, CSD_SCAN_MINB) k_csd_scan(DS d, const uint32_t *list, uint32_t n, CsdArgs a) {
    // CSD_SU chunks of 64 members per pass, their loads in flight together (a row is one 256-KB stream). A chunk's
    // differing members are taken together, one per lane: the shift before each is a wave prefix sum of the record
    // length differences, a member starts a new run of exception blocks when its first block lies past the previous
    // differing member's last block + 1 (their last blocks grow with the member), and each run start closes the run
    // before it (prefix sums place the closed runs and their entries). Round 4's first version walked the members one
    // at a time (the whole wave, scalar): 5.9 ms per launch on a heavy cascade round. Runs wait in LDS for their
    // entries, generated (one lane per run) between passes.
#ifndef CSD_SU_DEF
#define CSD_SU_DEF 4
#endif
    constexpr uint32_t CSD_SU = CSD_SU_DEF, RUNCAP = 256, RUNFLUSH = 128;
    __shared__ uint32_t runs[4][RUNCAP][6];                         // {klo, khi, m0, o0, s_after, first entry}
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
    // (forced inline: called from more than one place, the compiler made it a call that copies the DS block to scratch)
    auto flush = [&]() __attribute__((always_inline)) {
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
        if (nruns == RUNCAP) flush();                               // (wave-uniform here: the walk is the whole wave's)
        if (e + nb > a.ecap) { flags |= CSD_F_ECAP; return; }
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
    auto wred = [&](int32_t v, int op) -> int32_t {                 // wave min (0), max (1) or or (2)
        return (int32_t)lane63(op == 0 ? (uint32_t)dpp_scan_imin(v) : op == 1 ? (uint32_t)dpp_scan_imax(v) : dpp_scan_or((uint32_t)v));
    };
    // one chunk: m = its differing lanes; this lane's member mm, row word wm, B word bm, O_B[mm], O_B[mm - 1]
    auto chunk = [&](uint64_t m, uint32_t mm, uint32_t wm, uint32_t bm, uint32_t obm, uint32_t ob1) {
        const bool dl = (m >> lane) & 1ull;
        const int32_t Lr = dl ? (int32_t)csd_reclen(d, wm) : 0, Lbm = dl ? (int32_t)csd_reclen(d, bm) : 0;
        uint32_t tot;
        const int32_t sb = s + (int32_t)wscan_excl((uint32_t)(Lr - Lbm), tot);   // the shift before this member
        const int32_t x = (int32_t)obm + sb, y = x + Lr;            // the record's bytes in the row: [x, y)
        // blocks whose 32 bytes [20k, 20k + 32) meet [x, y) (or straddle x when the record is empty)
        const int32_t klo = x >= 32 ? (x - 32) / 20 + 1 : 0;
        int32_t khi = y >= 1 ? (y - 1) / 20 : -1;
        if (khi > (int32_t)kl) khi = (int32_t)kl;
        const bool vd = dl && klo <= (int32_t)kl && khi >= klo;
        // the last block of every run before this member: the open run's, or the previous valid member's (a prefix max)
        const int32_t px = dpp_scan_imax(vd ? khi : (-0x7FFFFFFF - 1));
        const int32_t pxe = (int32_t)dpp_shr1((uint32_t)px, 0x80000000u);   // (exclusive: the lanes below this one)
        const int32_t pk = lane ? max(pxe, (int32_t)rhi) : (int32_t)rhi;
        const bool st = vd && klo > pk + 1;                         // this member begins a new run
        const uint64_t sm = __ballot(st);
        if (sm == 0) {                                              // every valid member extends the open run
            rhi = (uint32_t)max((int32_t)rhi, wred(vd ? khi : (-0x7FFFFFFF - 1), 1));
            s += (int32_t)tot;
            return;
        }
        // a new run starts at row byte p = 20 klo, in the clean bytes before mm (shift sb): the record holding B offset
        // t = p - sb is the last member below mm with O_B <= t (mm >= 1: member 0's record meets block 0, which always
        // begins a run)
        uint32_t m0 = 0, o0 = 0;
        if (st) {
            const uint32_t t = (uint32_t)(20 * klo - sb);
            uint32_t q = mm - 1, om = ob1;
            while (q > 0 && om > t) om = a.OB[--q];
            m0 = q;
            o0 = t - om;
        }
        // each start closes the run before it: the previous start's, or the open run
        const uint64_t below = sm & ((1ull << lane) - 1ull);
        const uint32_t src = below ? 63u - (uint32_t)__builtin_clzll(below) : 0u;
        const uint32_t plo = (uint32_t)__shfl(klo, (int)src, 64), pm0 = (uint32_t)__shfl((int)m0, (int)src, 64),
                       po0 = (uint32_t)__shfl((int)o0, (int)src, 64);
        const uint32_t clo = below ? plo : rlo, cm0 = below ? pm0 : rm0, co0 = below ? po0 : ro0, chi = (uint32_t)pk;
        uint32_t ntot;
        const uint32_t eo = wscan_excl(st ? chi - clo + 1 : 0u, ntot);
        const uint32_t K = (uint32_t)__popcll(sm);
        if (e + ntot > a.ecap) { flags |= CSD_F_ECAP; return; }
        if (st) {
            uint32_t *q = runs[wv][nruns + (uint32_t)__popcll(below)];
            q[0] = clo; q[1] = chi; q[2] = cm0; q[3] = co0; q[4] = (uint32_t)sb; q[5] = e + eo;
        }
        const bool cs = st && chi < kl;                             // clean blocks follow the closed run at shift sb
        smin = min(smin, wred(cs ? sb : 0x7FFFFFFF, 0));
        smax = max(smax, wred(cs ? sb : (-0x7FFFFFFF - 1), 1));
        phm |= (uint32_t)wred(cs ? (int32_t)(1u << csd_phase(sb)) : 0, 2);
        e += ntot;
        nruns += K;
        // the last start's run stays open
        const uint32_t ll = 63u - (uint32_t)__builtin_clzll(sm);
        rlo = (uint32_t)__builtin_amdgcn_readlane(klo, (int)ll);   // (ll is wave-uniform)
        rm0 = (uint32_t)__builtin_amdgcn_readlane((int)m0, (int)ll);
        ro0 = (uint32_t)__builtin_amdgcn_readlane((int)o0, (int)ll);
        rhi = (uint32_t)wred(vd && lane >= ll ? khi : (-0x7FFFFFFF - 1), 1);
        s += (int32_t)tot;
    };
    // the columns to compare: every member, or only the divergent columns (DS::colx: outside them every row, and
    // every snapshot of a row, holds the same word, so it equals the majority B there) when they are few
    const uint32_t ucnt = a.ulist ? *a.ucnt : N;
    const bool UL = a.ulist && ucnt <= N / 4;
    const uint32_t ncol = UL ? ucnt : N;
    // (divergent columns come with their B word and offsets from the column table: one dependent load less)
    const bool ULc = UL && a.ucol;
    // (a listed observer row reads its hot members' words from the row's compact hot copy, a few KB, instead of one
    // 64-B sector per word of the 256-KB row; snapshots and cold members from the row)
    const uint32_t *hrow = (ULc && a.uhk && d.hidx && id < d.NL) ? d.hmw + (size_t)id * d.HP : nullptr;
    for (uint32_t c00 = 0; c00 < ncol && !flags; c00 += 64 * CSD_SU) {
        uint32_t wv_[CSD_SU], bv_[CSD_SU], mv_[CSD_SU], ov_[CSD_SU], o1_[CSD_SU];
        if (ULc) {
#pragma unroll
            for (uint32_t k = 0; k < CSD_SU; k++) {
                const uint32_t c = c00 + 64 * k + lane;
                const uint4 u = a.ucol[c < ncol ? c : 0u];
                const uint32_t hk = hrow ? a.uhk[c < ncol ? c : 0u] : SRC_NONE;
                mv_[k] = u.x; bv_[k] = u.y; ov_[k] = u.z; o1_[k] = u.w;
                wv_[k] = *(hk != SRC_NONE ? hrow + hk : row + u.x);
                if (c >= ncol) bv_[k] = wv_[k];                    // (past the list: equal, no diff)
            }
        } else {
#pragma unroll
            for (uint32_t k = 0; k < CSD_SU; k++) {
                const uint32_t c = c00 + 64 * k + lane;
                const uint32_t m = c < ncol ? (UL ? a.ulist[c] : c) : 0u;
                mv_[k] = m;
                wv_[k] = c < ncol ? row[m] : 0u;
                bv_[k] = c < ncol ? a.B[m] : 0u;
            }
        }
        uint64_t mk[CSD_SU];
        uint64_t any = 0;
#pragma unroll
        for (uint32_t k = 0; k < CSD_SU; k++) {
            mk[k] = __ballot(c00 + 64 * k + lane < ncol && !csd_same(wv_[k], bv_[k]));
            any |= mk[k];
        }
        if (!any) continue;
        if (!ULc) {
#pragma unroll
            for (uint32_t k = 0; k < CSD_SU; k++) {
                ov_[k] = a.OB[mv_[k]];
                o1_[k] = a.OB[mv_[k] ? mv_[k] - 1u : 0u];
            }
        }
        // (unrolled: the pass's values stay in registers; picked by a run-time chunk index, they went to memory)
#pragma unroll
        for (uint32_t k = 0; k < CSD_SU; k++) {
            if (mk[k] && !flags) {
                if (nruns + 64 > RUNCAP) flush();                   // (a chunk closes at most 64 runs)
                chunk(mk[k], mv_[k], wv_[k], bv_[k], ov_[k], o1_[k]);
            }
        }
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
// one block of all three lanes as one sequence, the g, f and h instructions interleaved so that every instruction's
// operands were produced at least two instructions earlier (also across consecutive blocks): a dependent integer VALU
// instruction issues about 10 cycles after its producer, an independent one every 5, so the block runs at the issue
// rate, 12 instructions. (csd_gf_step followed by csd_h_step leaves the four h instructions back to back: the compiler
// does not interleave separate asm statements.)
__device__ __forceinline__ void csd_block3(uint32_t &Xg, uint32_t &Xf, uint32_t &Xh, uint32_t mg, uint32_t dd, uint32_t mf,
                                           uint32_t pf, uint32_t mh, uint32_t kh) {
    uint32_t tg, tf;
    asm volatile("v_xor_b32 %4, %1, %7\n\t"
                 "v_xor_b32 %3, %0, %5\n\t"
                 "v_xor_b32 %2, %2, %9\n\t"
                 "v_alignbit_b32 %4, %4, %4, 19\n\t"
                 "v_alignbit_b32 %3, %3, %3, 19\n\t"
                 "v_alignbit_b32 %2, %2, %2, 19\n\t"
                 "v_lshl_add_u32 %3, %3, 2, %3\n\t"
                 "v_lshl_add_u32 %4, %4, 2, %4\n\t"
                 "v_lshl_add_u32 %2, %2, 2, %2\n\t"
                 "v_add3_u32 %1, %4, %3, %8\n\t"
                 "v_add_u32 %2, %2, %10\n\t"
                 "v_add3_u32 %0, %3, %1, %6"
                 : "+v"(Xg), "+v"(Xf), "+v"(Xh), "=&v"(tg), "=&v"(tf)
                 : "v"(mg), "v"(dd), "v"(mf), "v"(pf), "v"(mh), "v"(kh));
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
