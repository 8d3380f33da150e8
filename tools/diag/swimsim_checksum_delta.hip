// tools/diag/swimsim_checksum_delta.hip — DIAGNOSTICS LIBRARY ONLY: round 3's reference-row chain kernel k_cs_delta
// (helper waves premix S_B's window at every phase, copy exception blocks and write jump lists; h-chain and g/f-chain
// waves), kept for comparison with the product's k_csr (csrc/swimsim_checksum_csr.hip). The reference row, string and
// scan it consumes are csrc/swimsim_checksum_ref.hip's.
//
//   k_cs_delta    256 rows per workgroup, one workgroup per CU. Four hasher waves (lane = row, one wave per SIMD) run
//                 the chain in carried-sum form: 12 VALU instructions a block, its premixed values read from LDS at
//                 an address that advances by 24 bytes a block and jumps only where an exception run begins or ends.
//                 Four helper waves prepare, one super step (32 blocks) ahead: the window of S_B's premixed blocks at
//                 every phase (-s mod 20) the workgroup's rows use (shared by all 256 rows), the rows' exception
//                 blocks beside it, and each row's jump list.
// Rows the delta path cannot take (entry or LDS-slot overflow, a workgroup whose shifts spread too far) are flagged
// and re-hashed by the production kernels (k_checksum3 / k_checksum_q16); results are bit-exact either way.

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
                    bk[q] = y.z; bs[q] = (int32_t)y.w;
                    bv[q][0] = make_uint2(x.x, x.y); bv[q][1] = make_uint2(x.z, x.w); bv[q][2] = make_uint2(y.x, y.y);
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
            auto kat = [&](uint32_t e) -> uint32_t { return ((const uint32_t *)(ent + 2 * e + 1))[2]; };
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
                        place(q, y.z, (int32_t)y.w, make_uint2(x.x, x.y), make_uint2(x.z, x.w), make_uint2(y.x, y.y),
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
