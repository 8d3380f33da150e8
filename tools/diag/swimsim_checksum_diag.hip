// swimsim_checksum_diag.hip — DIAGNOSTICS ONLY: superseded checksum kernels and the measurement variants of the
// production ones. Compiled only into tools/libswimsim_diag.so (make -C ringpop-go_amd diag, -DSWIMSIM_DIAG), which
// tools/cs_bench.py, tools/cs_bench_real.py and tools/dbg_cs.py load through SWIMSIM_LIBRARY; libswimsim.so never
// contains them, so production checksums cannot route through untested paths. Included by swimsim_checksum.hip
// after the production kernels.
//   k_checksum      4-wave kernel of round 1 (formatters / h / g+f), MODE variants
//   k_checksum_n16  round-2 narrow kernel (lane = (row, record) formatters, premix wave, h and g/f waves)
//   k_checksum2     round-2 wide kernel (formatter + h on one wave, g/f on the other)

constexpr int CS_IT = 4;                        // members formatted per pipeline step
constexpr int CS_SUP = 16;                      // members per register prefetch of the row (4 steps)
constexpr int CS_RING = 110;                    // ring words per row: whole 20-byte blocks
constexpr int CS_POST = 12;
constexpr int CS_PHYS = CS_PRE + CS_RING + CS_POST;
constexpr int CS_SINK = CS_PHYS;
constexpr int CS_LDSW = CS_PHYS + 12;

// NO = ring words one record can touch (record of at most W + max tail bytes, shifted by <= 3).
// Waves: 0 h chain, 1 g/f chain, 2 and 3 formatters.
// MODE 0: normal; 1: hashers only (formatter skips its stores); 2: formatter only; 3: the g/f wave
// also dumps every block it hashes to dbg (lane 0's row; diagnostics); 4: barrier skeleton (no
// loads, no hashing); 5: formatter loads and positions only. Modes 1, 2, 4, 5 time parts of the kernel
// (swimsim_bench_checksum mode 6 runs k_checksum_n16).
// JMIN = words every record fills completely (shortest record >> 2): their writes need no mask.
template <int W, int NO, int JMIN, int MODE>
__global__ void __launch_bounds__(256) k_checksum(DS d, const uint32_t *list, const uint32_t *count,
                                                  const uint32_t *__restrict__ addrw, const uint4 *__restrict__ rtail,
                                                  uint32_t *dbg = nullptr, uint32_t dbg_cap = 0) {
    __shared__ uint32_t ring[CS_LDSW * CS_ROWS];
    __shared__ uint32_t wp[2][CS_ROWS];
    __shared__ uint32_t xgf[2][CS_ROWS];
    constexpr int Q = W / 4;                      // record words that are pure address words
    static_assert(NO <= CS_PRE + 1 && NO <= CS_POST + 1, "spill areas too small");
    static_assert(NO <= Q + 8, "record tail table holds 7 words after the address words");
    static_assert(CS_RING % 5 == 0, "blocks must tile the ring");
    static_assert(NO <= CS_LDSW - CS_SINK, "sink area too small");
    const uint32_t cnt = *count;
    if (blockIdx.x * CS_ROWS >= cnt) return;                       // uniform per workgroup
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t gi = blockIdx.x * CS_ROWS + lane;
    const bool valid = gi < cnt;
    const uint32_t id = list[valid ? gi : blockIdx.x * CS_ROWS];
    const bool is_row = id < d.NL;
    const uint32_t *row = is_row ? d.mw + (size_t)id * d.NP : d.dense + (size_t)(id - d.NL) * d.NP;
    const uint32_t N = d.N, ecap1 = d.ecap - 1;
    const uint32_t nsup = (N + CS_SUP - 1) / CS_SUP;
    const uint32_t nit = nsup * (CS_SUP / CS_IT);

    if (wave >= 2) {
        // ------------------------------- formatters -------------------------------
        // Interval i covers members 4i..4i+3: formatter f formats members 4i+2f, 4i+2f+1 and only
        // tracks the length and last bytes of the other two. A record writes only its complete
        // words; the word it shares with the next record is written by the next record (from the
        // carried bytes hc), so the two formatters never write the same word.
        // pos = bytes formatted; phys = ring word holding byte pos; hc = the last 4 bytes formatted
        const uint32_t f = wave - 2;
        uint32_t pos = 0, phys = 0, hc = 0;
        uint4 pre[4], cur[4];
        // double-buffered one interval ahead, indexed by compile-time interval parity (no register copies,
        // so a prefetch is only waited for where it is used)
        uint4 ta[2][2], tb[2][CS_IT];                             // tails: own members (ta, tb), others (tb)
        uint32_t A[2][2][Q + 1];                                  // address words of the own members
        auto tails = [&](const uint4 &q4, uint4 (&xa)[2], uint4 (&xb)[CS_IT]) {
            const uint32_t ws[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
            for (int k = 0; k < CS_IT; k++) {
                const uint32_t e = min(ws[k] >> 3, ecap1);
                const uint4 *tp = rtail + ((size_t)e * 4 + (ws[k] & 3u)) * 2;
                if ((k >> 1) == (int)f) xa[k & 1] = tp[0];
                xb[k] = tp[1];
            }
        };
        auto addrs = [&](uint32_t mb, uint32_t (&xA)[2][Q + 1]) {
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const uint32_t *ap = addrw + (size_t)min(mb + 2 * f + k, N - 1) * 6;
#pragma unroll
                for (int i = 0; i <= Q; i++) xA[k][i] = ap[i];
            }
        };
#pragma unroll
        for (int k = 0; k < 4; k++) pre[k] = *(const uint4 *)(row + 4 * k);
        tails(pre[0], ta[0], tb[0]);
        addrs(0, A[0]);
        for (uint32_t sc = 0; sc < nsup; sc++) {
#pragma unroll
            for (int k = 0; k < 4; k++) cur[k] = pre[k];
            if (sc + 1 < nsup) {
#pragma unroll
                for (int k = 0; k < 4; k++) pre[k] = *(const uint4 *)(row + (sc + 1) * CS_SUP + 4 * k);
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int b = u & 1, nb_ = b ^ 1;
                const uint32_t mb = sc * CS_SUP + u * CS_IT;
                if (MODE != 4) {
                    tails(u < 3 ? cur[u + 1] : pre[0], ta[nb_], tb[nb_]);   // next interval's tails and addresses
                    addrs(mb + CS_IT, A[nb_]);
                }
                const uint4 q4 = cur[u];
                const uint32_t ws[4] = {q4.x, q4.y, q4.z, q4.w};
                // positions of the interval's 4 records (a short prefix chain), then the own records'
                // words, branch-free: skipped records and words past a record's last complete word go
                // to a sink area, so the writes of the two records are independent
                uint32_t Lk[CS_IT], sk[CS_IT], pk[CS_IT], hk[CS_IT];
#pragma unroll
                for (int k = 0; k < CS_IT; k++) {
                    const uint32_t c6 = tb[b][k].z, c7 = tb[b][k].w;
                    const uint32_t L = MODE == 4 ? 38u : ((ws[k] & 7u) < 4u && mb + k < N) ? (c6 >> 24) : 0u;
                    const uint32_t sh = pos & 3u;
                    Lk[k] = L; sk[k] = sh; pk[k] = phys; hk[k] = hc;
                    uint32_t np = phys + ((sh + L) >> 2);
                    np = np >= CS_RING ? np - CS_RING : np;
                    phys = np;
                    hc = L ? c7 : hc;
                    pos += L;
                }
                auto emit = [&](auto F) {                            // F = this formatter, a compile-time
                    constexpr int f0 = decltype(F)::value;            // constant on each of the two paths
#pragma unroll
                    for (int kk = 0; kk < 2; kk++) {
                        const int k = 2 * f0 + kk;
                        const uint32_t L = Lk[k], sh = sk[k], ph = pk[k];
                        const uint4 &t0 = ta[b][kk];
                        const uint32_t C[7] = {t0.x, t0.y, t0.z, t0.w, tb[b][k].x, tb[b][k].y, tb[b][k].z};
                        const uint32_t sel = 0x07060504u - sh * 0x01010101u;
                        const uint32_t nw = (sh + L) >> 2;            // complete words of this record
                        uint32_t R[NO], O[NO];
#pragma unroll
                        for (int i = 0; i < NO; i++)
                            R[i] = i < Q ? A[b][kk][i] : (i == Q ? (A[b][kk][Q] | C[0]) : (i - Q < 7 ? C[i - Q] : 0u));
#pragma unroll
                        for (int j = 0; j < NO; j++) O[j] = __builtin_amdgcn_perm(R[j], j ? R[j - 1] : hk[k], sel);
                        const uint32_t sink = CS_SINK * CS_ROWS + lane;
                        const uint32_t i0 = L ? (CS_PRE + ph) * CS_ROWS + lane : sink;
#pragma unroll
                        for (int j = 0; j < NO; j++)
                            ring[(j < JMIN || (uint32_t)j < nw ? i0 : sink) + j * CS_ROWS] = O[j];
                        if (L && ph + nw > CS_RING) {                  // words past the ring end: also at the front
                            const uint32_t i1 = (CS_PRE + ph - CS_RING) * CS_ROWS + lane;
#pragma unroll
                            for (int j = 0; j < NO; j++)
                                ring[(j < JMIN || (uint32_t)j < nw ? i1 : sink) + j * CS_ROWS] = O[j];
                        }
                    }
                };
                if (MODE != 1 && MODE != 4 && MODE != 5) {
                    if (f == 0) emit(std::integral_constant<int, 0>{});
                    else emit(std::integral_constant<int, 1>{});
                }
                if (f == 0) wp[(sc * 4 + u) & 1][lane] = pos;
                lds_barrier();
            }
        }
        lds_barrier();
        return;
    }

    // ------------------------------- hashers -------------------------------
    FH fh{0, 0, 0};
    uint32_t iters = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, iters);
    if (!ok && valid && wave == 0) atomicOr(d.err, E_SHORT);
    uint32_t h = fh.h, g = fh.g, f = fh.f;
    const uint32_t *rb = ring + CS_PRE * CS_ROWS + lane;
    uint32_t done = 0, rq = 0;
    // hash blocks [done, lim) in groups of 4: all loads of a group first, then the arithmetic. While
    // every lane has a whole group left the groups run unpredicated; the last groups of a step use
    // branch-free predication (lanes have different limits)
    auto advance = [&](uint32_t lim) {
        const uint32_t n = done < lim ? min(lim - done, 4u) : 0u;
        done += n;
        rq += 5u * n;
        rq = rq >= CS_RING ? rq - CS_RING : rq;
    };
    auto run_h = [&](uint32_t lim) {
        while (__all(done + 4 <= lim)) {                           // every lane has a whole group left
            uint32_t a[4], dd[4], e[4];
            uint32_t q = rq;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t *p = rb + q * CS_ROWS;
                a[k] = p[0]; dd[k] = p[3 * CS_ROWS]; e[k] = p[4 * CS_ROWS];
                q += 5;
                q = q >= CS_RING ? q - CS_RING : q;
            }
#pragma unroll
            for (int k = 0; k < 4; k++) h = fh_fold(h + a[k], fh_m(dd[k]), e[k]);
            done += 4;
            rq = q;
        }
        while (__any(done < lim)) {
            uint32_t a[4], dd[4], e[4];
            uint32_t q = rq;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t *p = rb + q * CS_ROWS;
                a[k] = p[0]; dd[k] = p[3 * CS_ROWS]; e[k] = p[4 * CS_ROWS];
                q += 5;
                q = q >= CS_RING ? q - CS_RING : q;
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t hn = fh_fold(h + a[k], fh_m(dd[k]), e[k]);
                h = done + k < lim ? hn : h;
            }
            advance(lim);
        }
    };
    auto run_gf = [&](uint32_t lim) {
        if (MODE != 3)
            while (__all(done + 4 <= lim)) {                       // every lane has a whole group left
                uint32_t v[4][5];
                uint32_t q = rq;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t *p = rb + q * CS_ROWS;
#pragma unroll
                    for (int i = 0; i < 5; i++) v[k][i] = p[i * CS_ROWS];
                    q += 5;
                    q = q >= CS_RING ? q - CS_RING : q;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t a = v[k][0], b = v[k][1], c = v[k][2], dd = v[k][3], e = v[k][4];
                    g = fh_fold(g + b, fh_m(c), a);
                    f = fh_fold(f + c, fh_m(b + e * FH_C1), dd);
                    f += g; g += f;
                }
                done += 4;
                rq = q;
            }
        while (__any(done < lim)) {
            uint32_t v[4][5];
            uint32_t q = rq;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t *p = rb + q * CS_ROWS;
#pragma unroll
                for (int i = 0; i < 5; i++) v[k][i] = p[i * CS_ROWS];
                q += 5;
                q = q >= CS_RING ? q - CS_RING : q;
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t a = v[k][0], b = v[k][1], c = v[k][2], dd = v[k][3], e = v[k][4];
                if (MODE == 3 && lane == 0 && done + k < lim && (done + k + 1) * 5 <= dbg_cap)
                    for (int i = 0; i < 5; i++) dbg[(done + k) * 5 + i] = v[k][i];
                uint32_t gn = fh_fold(g + b, fh_m(c), a);
                uint32_t fn = fh_fold(f + c, fh_m(b + e * FH_C1), dd);
                fn += gn; gn += fn;
                const bool act = done + k < lim;
                g = act ? gn : g;
                f = act ? fn : f;
            }
            advance(lim);
        }
    };
    uint32_t avail = 0;
    if (wave == 0) {
        for (uint32_t t = 0; t < nit; t++) {
            if (MODE < 2 || MODE == 3) run_h(MODE == 1 ? min(iters, t * 8u) : min(iters, avail));
            lds_barrier();
            avail = wp[t & 1][lane] / 20;
        }
        if (MODE < 2 || MODE == 3) run_h(iters);
    } else {
        for (uint32_t t = 0; t < nit; t++) {
            if (MODE < 2 || MODE == 3) run_gf(MODE == 1 ? min(iters, t * 8u) : min(iters, avail));
            lds_barrier();
            avail = wp[t & 1][lane] / 20;
        }
        if (MODE < 2 || MODE == 3) run_gf(iters);
    }
    if (wave == 1) { xgf[0][lane] = g; xgf[1][lane] = f; }
    lds_barrier();
    if (wave == 0 && valid) {
        fh.h = h; fh.g = xgf[0][lane]; fh.f = xgf[1][lane];
        const uint32_t hv = ok ? fh.fin() : 0u;
        if (is_row) {
            d.cs[id] = hv;
            d.dirty[id] = 0;
            ctr_add(d, C_X_CS_ROWS, 1ull);
        } else {
            d.dense_cs[id - d.NL] = hv;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Narrow variant for launches of few rows (latency-bound: the launch time is one row's chain).
// 16 rows per workgroup. The per-block work that does not depend on the chain runs across lanes
// instead of rows:
//   waves 2, 3 (formatters): lane = (row r, record k) for the 8 records of each step of 8 rows; a
//                            segmented prefix sum of the record lengths places a row's 8 records;
//   wave 1 (premix)        : lane = (row r, block slot s): M(c), M(d), M(b + e c1) of every block,
//                            5 of the block's 7 multiplies, into a per-row ring of premixed words;
//   wave 4 (h)             : lane r < 16: h = mur(d, h + a) + e with M(d) read;
//   wave 0 (g/f)           : lane r < 16: g, f with M(c), M(b + e c1) read.
// (wave w runs on the SIMD of wave w % 4: the light h chain shares the g/f wave's SIMD.)
// At step t the formatters write step t, premix takes the blocks completed by step t-1 and the
// hashers the blocks premixed at step t-1. Rows are stored row-major in LDS with an odd stride, so
// the hashers' 16 lanes hit 16 banks; ring words [0, 20) and premixed blocks [0, 4) are mirrored
// behind the ring end, so a hasher group of 4 blocks reads at constant offsets.
// ---------------------------------------------------------------------------------------------
constexpr int CN_IT = 8;                        // records per row per step
constexpr int CN_RING = 250;                    // ring words per row (50 blocks): 3 steps of 8 records
constexpr int CN_NBLK = CN_RING / 5;
constexpr int CN_MBLK = 4;
constexpr int CN_SINK = CS_PRE + CN_RING + CN_MIR;
constexpr int CN_STRIDE = CN_SINK + 13;         // landing area + ring + mirror + sink; odd
static_assert(CN_STRIDE % 2 == 1, "row stride must be odd");
constexpr int CN_MSTRIDE = (CN_NBLK + CN_MBLK) * 3;

// NMODE (diagnostics): 0 normal; 1 formatters without stores; 2 formatters only (premix and hashers
// idle); 3 no formatter work at all (fixed 38-byte records; premix and hashers on garbage); 4 as 3
// with premix idle; 5 as 3 with the hashers idle; 6 as 4 with the h wave idle; 7 as 4 with the g/f
// wave idle
template <int W, int NO, int JMIN, int NMODE = 0>
__global__ void __launch_bounds__(320) k_checksum_n16(DS d, const uint32_t *list, const uint32_t *count,
                                                      const uint32_t *__restrict__ addrw, const uint4 *__restrict__ rtail) {
    __shared__ uint32_t ring[CN_ROWS * CN_STRIDE];
    __shared__ uint32_t mring[CN_ROWS * CN_MSTRIDE];                // [row][block][M(c), M(d), M(b + e c1)]
    __shared__ uint32_t wp[4][CN_ROWS];
    __shared__ uint32_t xgf[2][CN_ROWS];
    constexpr int Q = W / 4;
    static_assert(NO <= CS_PRE + 1 && NO <= 13, "spill areas too small");
    static_assert(CS_PRE + CN_MIR - 1 + CN_RING + NO - 1 < CN_STRIDE, "mirror pass overruns the row");
    static_assert(NO <= Q + 8, "record tail table holds 7 words after the address words");
    static_assert(CN_RING * 4 >= 3 * CN_IT * 40 + 24, "ring too small for three steps");
    const uint32_t cnt = *count;
    const uint32_t b0 = blockIdx.x * CN_ROWS;
    if (b0 >= cnt) return;                                         // uniform per workgroup
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t N = d.N, ecap1 = d.ecap - 1;
    const uint32_t nit = (N + CN_IT - 1) / CN_IT;
    const uint32_t nsteps = nit + 2;
    auto row_of = [&](uint32_t r, uint32_t &id, bool &is_row) -> const uint32_t * {
        const uint32_t gi = b0 + r;
        id = list[gi < cnt ? gi : b0];
        is_row = id < d.NL;
        return is_row ? d.mw + (size_t)id * d.NP : d.dense + (size_t)(id - d.NL) * d.NP;
    };

    if (wave == 2 || wave == 3) {
        // ------------------------------- formatters -------------------------------
        const uint32_t r = (wave - 2) * 8 + (lane >> 3), k = lane & 7u;
        uint32_t id; bool is_row;
        const uint32_t *row = row_of(r, id, is_row);
        uint32_t *rrow = ring + r * CN_STRIDE;
        uint32_t pos = 0, phys = 0, hc = 0;                        // per row, kept in all 8 lanes of a segment
        // prefetch: row words two steps ahead, tails and addresses one step ahead
        auto ldw = [&](uint32_t t) { const uint32_t m = CN_IT * t + k; return m < N ? row[m] : (uint32_t)ST_UNKNOWN; };
        uint32_t w0 = ldw(0), w1 = ldw(1);
        auto ldt = [&](uint32_t w, uint4 &xa, uint4 &xb) {
            const size_t ti = ((size_t)min(w >> 3, ecap1) * 4 + (w & 3u)) * 2;
            xa = rtail[ti];
            xb = rtail[ti + 1];
        };
        auto lda = [&](uint32_t t, uint32_t (&xA)[Q + 1]) {
            const uint32_t *ap = addrw + (size_t)min(CN_IT * t + k, N - 1) * 6;
#pragma unroll
            for (int i = 0; i <= Q; i++) xA[i] = ap[i];
        };
        uint4 ta[2], tb[2];
        uint32_t A[2][Q + 1];
        ldt(w0, ta[0], tb[0]);
        lda(0, A[0]);
        auto step = [&](uint32_t t, auto B) {
            constexpr int b = decltype(B)::value, nb_ = b ^ 1;
            if (NMODE >= 3) {
                pos += CN_IT * 38;
                if (k == 0) wp[t & 3][r] = pos;
                lds_barrier();
                return;
            }
            const uint32_t w = w0;
            w0 = w1;
            w1 = ldw(t + 2);
            ldt(w0, ta[nb_], tb[nb_]);                              // next step's tail and address
            lda(t + 1, A[nb_]);
            const uint32_t m = CN_IT * t + k;
            const uint32_t L = ((w & 7u) < 4u && m < N) ? (tb[b].z >> 24) : 0u;
            // segmented prefix sums over the row's 8 records: bytes before this record within the step,
            // and the last bytes of the nearest non-empty record before it (the carry its first word
            // is aligned against)
            uint32_t inc = L, hv = L ? tb[b].w : 0u, hh = L ? 1u : 0u;
#pragma unroll
            for (int off = 1; off < CN_IT; off <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)inc, off, CN_IT);
                const uint32_t v2 = (uint32_t)__shfl_up((int)hv, off, CN_IT), h2 = (uint32_t)__shfl_up((int)hh, off, CN_IT);
                if (k >= (uint32_t)off) {
                    inc += y;
                    if (!hh) { hv = v2; hh = h2; }
                }
            }
            const uint32_t ex = inc - L, total = (uint32_t)__shfl((int)inc, CN_IT - 1, CN_IT);
            const uint32_t cv = (uint32_t)__shfl_up((int)hv, 1, CN_IT), ch = (uint32_t)__shfl_up((int)hh, 1, CN_IT);
            const uint32_t carry = (k >= 1 && ch) ? cv : hc;
            const uint32_t lastv = (uint32_t)__shfl((int)hv, CN_IT - 1, CN_IT), lasth = (uint32_t)__shfl((int)hh, CN_IT - 1, CN_IT);
            const uint32_t sh0 = pos & 3u;
            const uint32_t sh = (sh0 + ex) & 3u;
            uint32_t ph = phys + ((sh0 + ex) >> 2);
            ph = ph >= CN_RING ? ph - CN_RING : ph;
            if (NMODE != 1) {
                const uint32_t C[7] = {ta[b].x, ta[b].y, ta[b].z, ta[b].w, tb[b].x, tb[b].y, tb[b].z};
                const uint32_t sel = 0x07060504u - sh * 0x01010101u;
                const uint32_t nw = (sh + L) >> 2;
                uint32_t R[NO], O[NO];
#pragma unroll
                for (int i = 0; i < NO; i++)
                    R[i] = i < Q ? A[b][i] : (i == Q ? (A[b][Q] | C[0]) : (i - Q < 7 ? C[i - Q] : 0u));
#pragma unroll
                for (int j = 0; j < NO; j++) O[j] = __builtin_amdgcn_perm(R[j], j ? R[j - 1] : carry, sel);
                const uint32_t i0 = L ? CS_PRE + ph : (uint32_t)CN_SINK;
#pragma unroll
                for (int j = 0; j < NO; j++) rrow[(j < JMIN || (uint32_t)j < nw ? i0 : (uint32_t)CN_SINK) + j] = O[j];
                // second pass: a record crossing the ring end is also written one ring length earlier
                // (its words past the end land at the front), one starting in [0, CN_MIR) one ring
                // length later (the mirror; words past the mirror land in the sink)
                if (L && (ph < CN_MIR || ph + nw > CN_RING)) {
                    const uint32_t i1 = CS_PRE + (ph < CN_MIR ? ph + CN_RING : ph - CN_RING);
#pragma unroll
                    for (int j = 0; j < NO; j++) rrow[(j < JMIN || (uint32_t)j < nw ? i1 : (uint32_t)CN_SINK) + j] = O[j];
                }
            }
            uint32_t np = phys + ((sh0 + total) >> 2);
            phys = np >= CN_RING ? np - CN_RING : np;
            pos += total;
            hc = lasth ? lastv : hc;
            if (k == 0) wp[t & 3][r] = pos;
            lds_barrier();
        };
        uint32_t t = 0;
        for (; t + 1 < nit; t += 2) {
            step(t, std::integral_constant<int, 0>{});
            step(t + 1, std::integral_constant<int, 1>{});
        }
        if (t < nit) step(t, std::integral_constant<int, 0>{});
        lds_barrier();                                             // the two drain steps
        lds_barrier();
        lds_barrier();                                             // final g/f hand-over
        return;
    }

    if (wave == 1) {
        // ------------------------------- premix -------------------------------
        const uint32_t r = lane >> 2, s = lane & 3u;
        uint32_t id; bool is_row;
        (void)row_of(r, id, is_row);
        const uint32_t len = is_row ? d.clen[id] : d.dense_len[id - d.NL];
        const uint32_t iters = len > 24 ? (len - 1) / 20 : 0u;
        const uint32_t *rrow = ring + r * CN_STRIDE + CS_PRE;
        uint32_t *mrow = mring + r * CN_MSTRIDE;
        uint32_t blk = s, q = s;                                    // next block of this lane, its ring block
        for (uint32_t t = 0; t < nsteps; t++) {
            const uint32_t lim = (t == 0 || NMODE == 2 || NMODE == 4 || NMODE >= 6) ? 0u : t >= nit ? iters : min(iters, wp[(t - 1) & 3][r] / 20u);
            for (; __any(blk < lim);) {
                if (blk < lim) {
                    const uint32_t *bp = rrow + 5 * q;
                    const uint32_t b = bp[1], c = bp[2], dd = bp[3], e = bp[4];
                    uint32_t ec;
                    asm("v_mul_lo_u32 %0, %1, %2" : "=v"(ec) : "v"(e), "s"(FH_C1));
                    const uint32_t m0 = fh_m(c), m1 = fh_m(dd), m2 = fh_m(b + ec);
                    uint32_t *mp = mrow + 3 * q;
                    mp[0] = m0; mp[1] = m1; mp[2] = m2;
                    if (q < CN_MBLK) { mp[3 * CN_NBLK] = m0; mp[3 * CN_NBLK + 1] = m1; mp[3 * CN_NBLK + 2] = m2; }
                    blk += 4;
                    q += 4;
                    q = q >= CN_NBLK ? q - CN_NBLK : q;
                }
            }
            lds_barrier();
        }
        lds_barrier();
        return;
    }

    // ------------------------------- hashers -------------------------------
    const uint32_t r = lane & (CN_ROWS - 1);                       // lanes >= 16 shadow lane & 15
    uint32_t id; bool is_row;
    const uint32_t *row = row_of(r, id, is_row);
    const bool valid = lane < CN_ROWS && b0 + r < cnt;
    FH fh{0, 0, 0};
    uint32_t iters = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, iters);
    if (!ok && valid && wave == 0) atomicOr(d.err, E_SHORT);
    const uint32_t *rrow = ring + r * CN_STRIDE + CS_PRE;
    const uint32_t *mrow = mring + r * CN_MSTRIDE;
    auto lim_h = [&](uint32_t t) -> uint32_t {                     // blocks premixed by the end of step t-1
        if (t < 2 || NMODE == 2 || NMODE == 5 || (NMODE == 6 && wave == 4) || (NMODE == 7 && wave == 0)) return 0u;
        if (t - 1 >= nit) return iters;
        return min(iters, wp[(t - 2) & 3][r] / 20u);
    };
    uint32_t done = 0, bq = 0;                                     // bq = done mod CN_NBLK
    auto take = [&](uint32_t lim, bool pred) {
        const uint32_t n = pred ? (done < lim ? min(lim - done, 4u) : 0u) : 4u;
        done += n;
        bq += n;
        bq = bq >= CN_NBLK ? bq - CN_NBLK : bq;
    };
    uint32_t h = fh.h, g = fh.g, fv = fh.f;
    // per step: whole groups of 4 blocks while every lane has them, then predicated groups
    if (wave == 4) {
        auto group = [&](uint32_t lim, bool pred) {
            const uint32_t *sp = rrow + 5 * bq, *mp = mrow + 3 * bq;
            uint32_t a[4], e[4], md[4];
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                a[kk] = sp[5 * kk];
                e[kk] = sp[5 * kk + 4];
                md[kk] = mp[3 * kk + 1];
            }
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                const uint32_t hn = fh_fold(h + a[kk], md[kk], e[kk]);
                h = (!pred || done + kk < lim) ? hn : h;
            }
            take(lim, pred);
        };
        for (uint32_t t = 0; t < nsteps; t++) {
            const uint32_t lim = lim_h(t);
            while (__all(done + 4 <= lim)) group(lim, false);
            while (__any(done < lim)) group(lim, true);
            lds_barrier();
        }
    } else {
        auto group = [&](uint32_t lim, bool pred) {
            const uint32_t *sp = rrow + 5 * bq, *mp = mrow + 3 * bq;
            uint32_t v[4][4], mc[4], mbe[4];
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
#pragma unroll
                for (int i = 0; i < 4; i++) v[kk][i] = sp[5 * kk + i];              // a, b, c, d
                mc[kk] = mp[3 * kk];
                mbe[kk] = mp[3 * kk + 2];
            }
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                const uint32_t gn = fh_fold(g + v[kk][1], mc[kk], v[kk][0]);
                uint32_t fn = fh_fold(fv + v[kk][2], mbe[kk], v[kk][3]);
                fn += gn;
                const bool act = !pred || done + kk < lim;
                g = act ? gn + fn : g;
                fv = act ? fn : fv;
            }
            take(lim, pred);
        };
        for (uint32_t t = 0; t < nsteps; t++) {
            const uint32_t lim = lim_h(t);
            while (__all(done + 4 <= lim)) group(lim, false);
            while (__any(done < lim)) group(lim, true);
            lds_barrier();
        }
        if (lane < CN_ROWS) { xgf[0][lane] = g; xgf[1][lane] = fv; }
    }
    lds_barrier();
    if (wave == 4 && valid) {
        fh.h = h; fh.g = xgf[0][lane]; fh.f = xgf[1][lane];
        const uint32_t hv = ok ? fh.fin() : 0u;
        if (is_row) {
            d.cs[id] = hv;
            d.dirty[id] = 0;
            ctr_add(d, C_X_CS_ROWS, 1ull);
        } else {
            d.dense_cs[id - d.NL] = hv;
        }
    }
}

template <int W, int MODE>
void launch_cs_w(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t grid, hipStream_t s,
                 uint32_t *dbg = nullptr, uint32_t cap = 0, uint32_t narrow_grid = 0) {
    if (narrow_grid && (MODE == 0 || MODE >= 7)) {              // few rows: 16 rows per workgroup
        constexpr int NM = MODE >= 7 ? MODE - 6 : 0;           // diagnostics modes 7..13
        if (W == 19 && d.max_tail <= 21 && d.min_tail >= 19)
            hipLaunchKernelGGL((k_checksum_n16<W, cs_no(W, 21), (W + 19) / 4, NM>), dim3(narrow_grid), dim3(320), 0, s, d,
                               list, count, d.addrw, (const uint4 *)d.rtail);
        else
            hipLaunchKernelGGL((k_checksum_n16<W, cs_no(W, 24), (W + 7) / 4>), dim3(narrow_grid), dim3(320), 0, s, d,
                               list, count, d.addrw, (const uint4 *)d.rtail);
        return;
    }
    // the common case: 13-digit incarnations (t0 = 1.5e12 ms): tails of 19..21 bytes
    if (W == 19 && d.max_tail <= 21 && d.min_tail >= 19)
        hipLaunchKernelGGL((k_checksum<W, cs_no(W, 21), (W + 19) / 4, MODE>), dim3(grid), dim3(256), 0, s, d, list, count,
                           d.addrw, (const uint4 *)d.rtail, dbg, cap);
    else  // any tail of 7 ("alive" + 1 digit + ';') to 24 bytes
        hipLaunchKernelGGL((k_checksum<W, cs_no(W, 24), (W + 7) / 4, MODE>), dim3(grid), dim3(256), 0, s, d, list, count,
                           d.addrw, (const uint4 *)d.rtail, dbg, cap);
}

// k_checksum2 (was swimsim_checksum2.hip) — phase C FarmHash-32 over the membership string (memberlist.go:83-128, go-farm
// Fingerprint32), the throughput kernel: 64 rows per workgroup (lane = row), two waves.
//
//   wave 0 (F): formats 4 members per step into a linear LDS buffer that starts at the first 20-byte block
//               the step does not complete yet (double-buffered by step parity), then runs the h lane over the
//               blocks the previous step completed;
//   wave 1 (G): runs the coupled g and f lanes over the same blocks.
// Included by swimsim_kernels.hip after swimsim_checksum.hip (shares its record tables and FarmHash pieces).
//
// Measured (tools/cs_bench.py, one MI355X, 65,536-member rows): 19.2 ms for 65,536 rows, against 22.3 ms for
// its 4-wave predecessor k_checksum, with 34 % fewer VALU instructions (7.1e9 vs 1.08e10 per launch). It is
// still stall-bound: at 2 waves per SIMD every wave waits 41 % of its cycles (SQ_WAIT_ANY), and one wave issues
// a VALU op at most every 4 cycles. A 3-wave pipeline (formatter / h lane + f premix / g,f lanes, three
// buffers, 125 VGPRs, 3 waves per SIMD) measured 12.2 ms on one row group but 25.6 ms at 65,536 rows, so the
// few-row launches keep k_checksum_n16 and the wide ones use this kernel.
//  * one formatter per row group: every record writes all its NO words unconditionally at its position. The
//    word it shares with the previous record is rebuilt from the carried bytes, and the words past its end are
//    rewritten by the next record, so there is no sink, no mask and no second writer;
//  * no ring wrap: each step's buffer begins at a block boundary. The <= 5 words of the block the previous
//    step left incomplete are copied to its front (5 LDS reads + 5 writes per step), so a block never
//    straddles buffers and every read uses one base address with immediate offsets;
//  * the tail-table loads (global, L1/L2-resident) are issued two steps ahead and the row words 16 members
//    ahead, so the formatter never waits on memory. The address words are the same for every lane: one
//    coalesced load per super step (96 words, issued a super step ahead) is staged in LDS and read back as
//    broadcasts. No scalar loads in the loop: their lgkmcnt(0) waits would also drain the LDS traffic;
//  * the hashers take at most NB blocks per step (4 records), all loads first, predicated.
// One LDS barrier per step (LDS-only fences: the prefetches stay in flight).

template <int W, int NO, int NB, int BW>
__global__ void __launch_bounds__(128) k_checksum2(DS d, const uint32_t *list, const uint32_t *count,
                                                   const uint32_t *__restrict__ addrw, const uint4 *__restrict__ rtail) {
    __shared__ uint32_t buf[2 * BW * C2_ROWS];
    __shared__ uint32_t bend[2][C2_ROWS];        // blocks complete after step t (t & 1)
    __shared__ uint32_t xgf[2][C2_ROWS];
    __shared__ uint32_t ast[2][16 * 6];          // address words of a super step's 16 members (F only)
    constexpr int Q = W / 4;                     // record words that are pure address words
    static_assert(NO <= Q + 8, "record tail table holds 7 words after the address words");
    static_assert(5 * NB + 4 < BW, "hasher reads past the buffer");
    const uint32_t cnt = *count;
    if (blockIdx.x * C2_ROWS >= cnt) return;                       // uniform per workgroup
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t gi = blockIdx.x * C2_ROWS + lane;
    const bool valid = gi < cnt;
    const uint32_t id = list[valid ? gi : blockIdx.x * C2_ROWS];
    const bool is_row = id < d.NL;
    const uint32_t *row = is_row ? d.mw + (size_t)id * d.NP : d.dense + (size_t)(id - d.NL) * d.NP;
    const uint32_t N = d.N;
    const uint32_t nsup = (N + 15) / 16;                           // super steps of 16 members (4 steps)
    const uint32_t nsteps = nsup * 4;

    FH fh{0, 0, 0};
    uint32_t iters = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, iters);
    uint32_t *const lb = buf + lane;                               // this lane's column

    if (wave == 0) {
        if (!ok && valid) atomicOr(d.err, E_SHORT);
        // ------------------------------- formatter + h lane -------------------------------
        const uint32_t ecap1 = d.ecap - 1;
        uint32_t pos = 0, hc = 0;                                  // bytes formatted; the stream's last 4 bytes
        uint32_t h = fh.h, ob0 = 0;                                // ob0: base block of the previous step's buffer
        uint4 cur[4], pre[4];                                      // row words: this super step, the next
        uint4 TA[4][C2_IT], TB[4][C2_IT];                          // record tails of steps u .. u+2 (slot u & 3)
        auto tails = [&](uint4 q4, uint4 (&ta)[C2_IT], uint4 (&tb)[C2_IT]) {
            const uint32_t ws[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
            for (int k = 0; k < C2_IT; k++) {
                const uint4 *tp = rtail + ((size_t)min(ws[k] >> 3, ecap1) * 4 + (ws[k] & 3u)) * 2;
                ta[k] = tp[0];
                tb[k] = tp[1];
            }
        };
        // address words: super step s holds addrw[96 s .. 96 s + 95]; lanes 0..63 and 0..31 (+64) load them
        const uint32_t alast = N * 6 - 1;
        auto aload = [&](uint32_t s2, uint32_t &x0, uint32_t &x1) {
            x0 = addrw[min(s2 * 96 + lane, alast)];
            x1 = lane < 32 ? addrw[min(s2 * 96 + 64 + lane, alast)] : 0u;
        };
        uint32_t ap0, ap1;
        aload(0, ap0, ap1);
        ast[0][lane] = ap0;
        if (lane < 32) ast[0][64 + lane] = ap1;
        aload(1, ap0, ap1);                                        // super step 1, staged at super step 0
#pragma unroll
        for (int k = 0; k < 4; k++) cur[k] = *(const uint4 *)(row + 4 * k);
#pragma unroll
        for (int k = 0; k < 4; k++) pre[k] = nsup > 1 ? *(const uint4 *)(row + 16 + 4 * k) : make_uint4(0, 0, 0, 0);
        tails(cur[0], TA[0], TB[0]);
        tails(cur[1], TA[1], TB[1]);
        for (uint32_t sc = 0; sc < nsup; sc++) {
            const uint32_t *as = ast[sc & 1u];
            ast[(sc + 1) & 1u][lane] = ap0;                         // stage super step sc + 1, load sc + 2
            if (lane < 32) ast[(sc + 1) & 1u][64 + lane] = ap1;
            aload(sc + 2, ap0, ap1);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t t = sc * 4 + u;
                const uint32_t mb = t * C2_IT;
                // prefetch: tails two steps ahead, row words one super step ahead
                tails(u < 2 ? cur[u + 2] : pre[u - 2], TA[(u + 2) & 3], TB[(u + 2) & 3]);
                const uint32_t pb = t & 1u;
                uint32_t *B = lb + pb * BW * C2_ROWS;                    // this step's buffer
                const uint32_t *OB = lb + (pb ^ 1u) * BW * C2_ROWS;      // the previous step's
                // h lane: read the blocks the previous step completed (issued before the formatting); they are
                // the blocks [ob0, b0) of the previous buffer
                const uint32_t b0 = pos / 20u;                              // this buffer's base block
                const uint32_t hlim = min(b0, iters);
                uint32_t ha[NB], hd[NB], he[NB];
#pragma unroll
                for (int j = 0; j < NB; j++) {
                    ha[j] = OB[(5 * j + 0) * C2_ROWS];
                    hd[j] = OB[(5 * j + 3) * C2_ROWS];
                    he[j] = OB[(5 * j + 4) * C2_ROWS];
                }
                // carry: the words of the block the previous step left incomplete go to this buffer's front
                uint32_t cw[5];
#pragma unroll
                for (int i = 0; i < 5; i++) cw[i] = OB[(5 * (b0 - ob0) + i) * C2_ROWS];
#pragma unroll
                for (int i = 0; i < 5; i++) B[i * C2_ROWS] = cw[i];
                // format this step's 4 records: every record writes NO words at its position
                const uint4 *ta = TA[u], *tb = TB[u];
                const uint32_t ws[4] = {cur[u].x, cur[u].y, cur[u].z, cur[u].w};
#pragma unroll
                for (int k = 0; k < C2_IT; k++) {
                    const uint32_t m = mb + k;
                    uint32_t A[Q + 1];
#pragma unroll
                    for (int i = 0; i <= Q; i++) A[i] = as[(4 * u + k) * 6 + i];
                    const uint32_t L = ((ws[k] & 7u) < 4u && m < N) ? (tb[k].z >> 24) : 0u;
                    const uint32_t sh = pos & 3u;
                    // sh * 0x01010101 as a byte broadcast (one full-rate v_perm, not a multiply)
                    const uint32_t sel = 0x07060504u - __builtin_amdgcn_perm(0u, sh, 0u);
                    const uint32_t C[7] = {ta[k].x, ta[k].y, ta[k].z, ta[k].w, tb[k].x, tb[k].y, tb[k].z};
                    uint32_t R[NO];
#pragma unroll
                    for (int i = 0; i < NO; i++)
                        R[i] = i < Q ? A[i] : (i == Q ? (A[Q] | C[0]) : (i - Q < 7 ? C[i - Q] : 0u));
                    uint32_t *wb = B + ((pos >> 2) - 5u * b0) * C2_ROWS;
#pragma unroll
                    for (int j = 0; j < NO; j++) wb[j * C2_ROWS] = __builtin_amdgcn_perm(R[j], j ? R[j - 1] : hc, sel);
                    hc = L ? tb[k].w : hc;
                    pos += L;
                }
                bend[pb][lane] = pos / 20u;
                // h lane over the previous step's blocks
#pragma unroll
                for (int j = 0; j < NB; j++) {
                    const uint32_t hn = fh_fold(h + ha[j], fh_m(hd[j]), he[j]);
                    h = ob0 + j < hlim ? hn : h;
                }
                ob0 = b0;
                if (u == 3) {                                               // next super step's row words
#pragma unroll
                    for (int k = 0; k < 4; k++) cur[k] = pre[k];
                    if (sc + 2 < nsup) {
#pragma unroll
                        for (int k = 0; k < 4; k++) pre[k] = *(const uint4 *)(row + (sc + 2) * 16 + 4 * k);
                    }
                }
                lds_barrier();
            }
        }
        // drain: the last step's blocks
        {
            const uint32_t pb = (nsteps - 1) & 1u;
            const uint32_t *OB = lb + pb * BW * C2_ROWS;
            const uint32_t hlim = min(pos / 20u, iters);
#pragma unroll
            for (int j = 0; j < NB; j++) {
                const uint32_t hn = fh_fold(h + OB[(5 * j) * C2_ROWS], fh_m(OB[(5 * j + 3) * C2_ROWS]), OB[(5 * j + 4) * C2_ROWS]);
                h = ob0 + j < hlim ? hn : h;
            }
        }
        lds_barrier();                                             // G's final g, f
        if (valid) {
            fh.h = h; fh.g = xgf[0][lane]; fh.f = xgf[1][lane];
            const uint32_t hv = ok ? fh.fin() : 0u;
            if (is_row) {
                d.cs[id] = hv;
                d.dirty[id] = 0;
                ctr_add(d, C_X_CS_ROWS, 1ull);
            } else {
                d.dense_cs[id - d.NL] = hv;
            }
        }
        return;
    }

    // ------------------------------- g / f lanes -------------------------------
    uint32_t g = fh.g, f = fh.f, done = 0;
    for (uint32_t t = 0; t <= nsteps; t++) {
        if (t) {
            const uint32_t pb = (t - 1) & 1u;
            const uint32_t *OB = lb + pb * BW * C2_ROWS;
            const uint32_t lim = min(bend[pb][lane], iters);
            uint32_t v[NB][5];
#pragma unroll
            for (int j = 0; j < NB; j++)
#pragma unroll
                for (int i = 0; i < 5; i++) v[j][i] = OB[(5 * j + i) * C2_ROWS];
#pragma unroll
            for (int j = 0; j < NB; j++) {
                const uint32_t a = v[j][0], b = v[j][1], c = v[j][2], dd = v[j][3], e = v[j][4];
                uint32_t gn = fh_fold(g + b, fh_m(c), a);
                uint32_t fn = fh_fold(f + c, fh_m(b + e * FH_C1), dd);
                fn += gn;
                gn += fn;
                const bool act = done + j < lim;
                g = act ? gn : g;
                f = act ? fn : f;
            }
            done = bend[pb][lane];
        }
        if (t < nsteps) lds_barrier();
    }
    xgf[0][lane] = g;
    xgf[1][lane] = f;
    lds_barrier();
}

template <int W>
void launch_cs2_w(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t grid, hipStream_t s) {
    if (W == 19 && d.max_tail <= 21 && d.min_tail >= 19) {     // 13-digit incarnations: records of 38..40 bytes
        constexpr int NO = cs_no(W, 21);
        hipLaunchKernelGGL((k_checksum2<W, NO, c2_nb(W + 21), c2_bw(W + 21, NO)>), dim3(grid), dim3(128), 0, s, d, list,
                           count, d.addrw, (const uint4 *)d.rtail);
    } else {                                                   // any tail of up to 24 bytes
        constexpr int NO = cs_no(W, 24);
        hipLaunchKernelGGL((k_checksum2<W, NO, c2_nb(W + 24), c2_bw(W + 24, NO)>), dim3(grid), dim3(128), 0, s, d, list,
                           count, d.addrw, (const uint4 *)d.rtail);
    }
}

// stream dump of one row (diagnostics): every 20-byte block the g/f wave hashes, W = 19 only
void launch_checksum_dump(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t *dbg, uint32_t cap,
                          hipStream_t s) {
    if (d.W == 19) launch_cs_w<19, 3>(d, list, count, 1, s, dbg, cap);
}

// measurement variants (swimsim_bench_checksum): W = 19 only
void launch_checksum_mode(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t maxn, int mode, hipStream_t s) {
    const uint32_t grid = (maxn + CS_ROWS - 1) / CS_ROWS;
    if (grid == 0 || d.W != 19) return;
    const uint32_t ngrid = (maxn + CN_ROWS - 1) / CN_ROWS;
    if (mode == 62) launch_cs6_w<19, 1, 1>(d, list, count, grid, s);
    else if (mode == 63) launch_cs6_w<19, 2, 1>(d, list, count, grid, s);
    else if (mode == 60) launch_cs6_w<19, 1>(d, list, count, grid, s);
    else if (mode == 61) launch_cs6_w<19, 2>(d, list, count, grid, s);
    else if (mode == 50) launch_cs5_w<19, 1>(d, list, count, grid, s);
    else if (mode == 51) launch_cs5_w<19, 2>(d, list, count, grid, s);
    else if (mode == 30) launch_csq_w<19, 8>(d, list, count, ngrid, s);
    else if (mode == 31) launch_csq_w<19, 8, 1>(d, list, count, ngrid, s);
    else if (mode == 32) launch_csq_w<19, 8, 2>(d, list, count, ngrid, s);
    else if (mode == 33) launch_csq_w<19, 16>(d, list, count, ngrid, s);
    else if (mode == 34) launch_csq_w<19, 16, 1>(d, list, count, ngrid, s);
    else if (mode == 35) launch_csq_w<19, 16, 2>(d, list, count, ngrid, s);
    else if (mode == 36) launch_csq_w<19, 16, 3>(d, list, count, ngrid, s);
    else if (mode == 37) launch_csq_w<19, 16, 4>(d, list, count, ngrid, s);
    else if (mode == 38) launch_csq_w<19, 16, 5>(d, list, count, ngrid, s);
    else if (mode == 39) launch_csq_w<19, 16, 7>(d, list, count, ngrid, s);
    else if (mode == 44) launch_csq_w<19, 16, 8>(d, list, count, ngrid, s);
    else if (mode == 46) launch_cs3_w<19, 7>(d, list, count, grid, s);
    else if (mode == 45) launch_csq_w<19, 8, 8>(d, list, count, ngrid, s);
    else if (mode == 20) launch_cs2_w<19>(d, list, count, grid, s);
    else if (mode == 21) launch_cs3_w<19>(d, list, count, grid, s);
    else if (mode == 22) launch_cs3_w<19, 1>(d, list, count, grid, s);
    else if (mode == 23) launch_cs3_w<19, 2>(d, list, count, grid, s);
    else if (mode == 24) launch_cs3_w<19, 3>(d, list, count, grid, s);
    else if (mode == 25) launch_cs3_w<19, 4>(d, list, count, grid, s);
    else if (mode == 26) launch_cs3_w<19, 5>(d, list, count, grid, s);
    else if (mode == 6) launch_cs_w<19, 0>(d, list, count, grid, s, nullptr, 0, ngrid);
    else if (mode == 7) launch_cs_w<19, 7>(d, list, count, grid, s, nullptr, 0, ngrid);
    else if (mode == 8) launch_cs_w<19, 8>(d, list, count, grid, s, nullptr, 0, ngrid);
    else if (mode == 9) launch_cs_w<19, 9>(d, list, count, grid, s, nullptr, 0, ngrid);
    else if (mode == 10) launch_cs_w<19, 10>(d, list, count, grid, s, nullptr, 0, ngrid);
    else if (mode == 11) launch_cs_w<19, 11>(d, list, count, grid, s, nullptr, 0, ngrid);
    else if (mode == 12) launch_cs_w<19, 12>(d, list, count, grid, s, nullptr, 0, ngrid);
    else if (mode == 13) launch_cs_w<19, 13>(d, list, count, grid, s, nullptr, 0, ngrid);
    else if (mode == 1) launch_cs_w<19, 1>(d, list, count, grid, s);
    else if (mode == 2) launch_cs_w<19, 2>(d, list, count, grid, s);
    else if (mode == 4) launch_cs_w<19, 4>(d, list, count, grid, s);
    else if (mode == 5) launch_cs_w<19, 5>(d, list, count, grid, s);
    else launch_cs_w<19, 0>(d, list, count, grid, s);
}
