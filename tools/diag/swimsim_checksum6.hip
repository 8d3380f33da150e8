// swimsim_checksum6.hip — phase C FarmHash-32 over the membership string (memberlist.go:83-128, go-farm
// Fingerprint32) for launches of many rows: 64 rows per workgroup (lane = row), a formatter wave and NH = 1 or 2
// hasher waves. Included by swimsim_checksum.hip after swimsim_checksum5.hip.
//
// Against k_checksum3 / k_checksum5 (profiles/r03_pmc_summary.json: every wave of k_checksum3 is issuing 59 % of
// its cycles; a lone wave issues at most one instruction per 4 cycles, MI355X_MICROARCH.md, so the longest
// per-wave instruction stream of a step sets the step time):
//  * the formatter's common case costs no record-tail loads. A step whose 4 records are (alive, t0) in all 64 rows
//    (in a cascade: every step without a killed member, ~96 %) takes its record tail, length and last bytes from
//    registers loaded once; other steps load their tails when they come (no prefetch arrays: 64-128 fewer VGPRs,
//    which is what lets three waves share a SIMD without spilling);
//  * a hasher step runs its blocks unpredicated when every lane has them all (or all but the last): the per-block
//    v_cndmask triple of the predicated form is paid only where lanes really differ;
//  * NH = 2 splits the chain over two waves (g/f with M(c), M(b + e c1); h with M(d)), as k_checksum5.
// STAMP (diagnostics build only): every wave sums its busy shader cycles per step (s_memtime from the barrier's
// release to its arrival at the next one) into measurement counter slots C_NALL + role (role 0 formatter, 1 g/f or
// h/g/f hasher, 2 h hasher), and its whole loop's cycles into C_NALL + 3 (formatter) (swimsim_kernel_units).
template <int W, int NO, int NB, int BW, int NH, int STAMP = 0>
__global__ void __launch_bounds__(64 * (1 + NH), NH == 2 ? 3 : 2)
k_checksum6(DS d, const uint32_t *list, const uint32_t *count, const uint32_t *__restrict__ addrw,
            const uint4 *__restrict__ rtail) {
    __shared__ uint32_t buf[2 * BW * C2_ROWS];
    __shared__ uint32_t bend[2][C2_ROWS];        // blocks complete after step t (t & 1)
    __shared__ uint32_t ast[2][16 * 6];          // address words of a super step's 16 members (F only)
    __shared__ uint32_t xgf[2][C2_ROWS];         // g, f at the end (NH = 2: GF -> H)
    constexpr int Q = W / 4;                     // record words that are pure address words
    static_assert(NH == 1 || NH == 2, "one or two hasher waves");
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

    uint32_t *const lb = buf + lane;                               // this lane's column

    if (wave == 0) {
        // ------------------------------- formatter -------------------------------
        __builtin_amdgcn_s_setprio(2);
        const uint32_t ecap1 = d.ecap - 1;
        uint32_t pos = 0, hc = 0;                                  // bytes formatted; the stream's last 4 bytes
        uint4 cur[4], pre[4];                                      // row words: this super step, the next
        const char *rtb = (const char *)rtail;
        unsigned long long busy = 0;                               // STAMP
        // the common record's tail: member word 0 = (alive, e = 0), table entry 0
        uint32_t TC[7], HC, LC;
        {
            const uint4 ta = rtail[0], tb = rtail[1];
            TC[0] = ta.x; TC[1] = ta.y; TC[2] = ta.z; TC[3] = ta.w; TC[4] = tb.x; TC[5] = tb.y; TC[6] = tb.z;
            HC = tb.w;
            LC = tb.z >> 24;
        }
        const uint32_t alast = N * 6 - 1;
        auto aload = [&](uint32_t s2, uint32_t &x0, uint32_t &x1) {
            x0 = addrw[min(s2 * 96 + lane, alast)];
            x1 = lane < 32 ? addrw[min(s2 * 96 + 64 + lane, alast)] : 0u;
        };
        uint32_t ap0, ap1;
        aload(0, ap0, ap1);
        ast[0][lane] = ap0;
        if (lane < 32) ast[0][64 + lane] = ap1;
        aload(1, ap0, ap1);
#pragma unroll
        for (int k = 0; k < 4; k++) cur[k] = *(const uint4 *)(row + 4 * k);
#pragma unroll
        for (int k = 0; k < 4; k++) pre[k] = nsup > 1 ? *(const uint4 *)(row + 16 + 4 * k) : make_uint4(0, 0, 0, 0);
        uint32_t AN[C2_IT][Q + 1], cw[5] = {0, 0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < C2_IT; k++)
#pragma unroll
            for (int i = 0; i <= Q; i++) AN[k][i] = ast[0][k * 6 + i];
        // one record: its NO words at its position, aligned against the carried bytes (C = tail words 0..6)
        auto put = [&](uint32_t *B, uint32_t b0, const uint32_t (&A)[Q + 1], const uint32_t (&C)[7], uint32_t sel) {
            uint32_t R[NO];
#pragma unroll
            for (int i = 0; i < NO; i++) R[i] = i < Q ? A[i] : (i == Q ? (A[Q] | C[0]) : (i - Q < 7 ? C[i - Q] : 0u));
            uint32_t *wb = B + ((pos >> 2) - 5u * b0) * C2_ROWS;
#pragma unroll
            for (int j = 0; j < NO; j++) wb[j * C2_ROWS] = __builtin_amdgcn_perm(R[j], j ? R[j - 1] : hc, sel);
        };
        auto selof = [](uint32_t p) { return 0x07060504u - __builtin_amdgcn_perm(0u, p & 3u, 0u); };
        auto sstep = [&](uint32_t sc, uint4 (&cur)[4], uint4 (&pre)[4], auto FULLC) {
            constexpr bool FULL = decltype(FULLC)::value;
            ast[(sc + 1) & 1u][lane] = ap0;
            if (lane < 32) ast[(sc + 1) & 1u][64 + lane] = ap1;
            aload(sc + 2, ap0, ap1);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t t = sc * 4 + u;
                const uint32_t mb = t * C2_IT;
                const unsigned long long ts0 = STAMP ? __builtin_amdgcn_s_memtime() : 0ull;
                uint32_t A[C2_IT][Q + 1];
#pragma unroll
                for (int k = 0; k < C2_IT; k++)
#pragma unroll
                    for (int i = 0; i <= Q; i++) A[k][i] = AN[k][i];
                {
                    const uint32_t *asn = ast[(u < 3 ? sc : sc + 1) & 1u] + (u < 3 ? 4 * (u + 1) : 0) * 6;
#pragma unroll
                    for (int k = 0; k < C2_IT; k++)
#pragma unroll
                        for (int i = 0; i <= Q; i++) AN[k][i] = asn[k * 6 + i];
                }
                const uint32_t pb = t & 1u;
                uint32_t *B = lb + pb * BW * C2_ROWS;
                const uint32_t b0 = pos / 20u;
#pragma unroll
                for (int i = 0; i < 5; i++) B[i * C2_ROWS] = cw[i];
                const uint4 w4 = cur[u];
                if (FULL && __all((w4.x | w4.y | w4.z | w4.w) == 0u)) {
                    // common step: 4 records of LC bytes with the registered tail
#pragma unroll
                    for (int k = 0; k < C2_IT; k++) {
                        put(B, b0, A[k], TC, selof(pos));
                        hc = HC;
                        pos += LC;
                    }
                } else {
                    const uint32_t ws[4] = {w4.x, w4.y, w4.z, w4.w};
                    uint4 ta[C2_IT], tb[C2_IT];
#pragma unroll
                    for (int k = 0; k < C2_IT; k++) {                // 32-byte entries, 32-bit byte offsets
                        const uint32_t off = ((min(ws[k] >> 3, ecap1) << 2) + (ws[k] & 3u)) << 5;
                        ta[k] = *(const uint4 *)(rtb + off);
                        tb[k] = *(const uint4 *)(rtb + off + 16u);
                    }
#pragma unroll
                    for (int k = 0; k < C2_IT; k++) {
                        const uint32_t L = ((ws[k] & 7u) < 4u && (FULL || mb + k < N)) ? (tb[k].z >> 24) : 0u;
                        const uint32_t C[7] = {ta[k].x, ta[k].y, ta[k].z, ta[k].w, tb[k].x, tb[k].y, tb[k].z};
                        put(B, b0, A[k], C, selof(pos));
                        hc = L ? tb[k].w : hc;
                        pos += L;
                    }
                }
                const uint32_t b1 = pos / 20u;
                bend[pb][lane] = b1;
#pragma unroll
                for (int i = 0; i < 5; i++) cw[i] = B[(5 * (b1 - b0) + i) * C2_ROWS];
                if (u == 3 && sc + 2 < nsup) {
#pragma unroll
                    for (int k = 0; k < 4; k++) cur[k] = *(const uint4 *)(row + (sc + 2) * 16 + 4 * k);
                }
                if (STAMP) {
                    __builtin_amdgcn_s_waitcnt(0xc07f);                // the step's LDS work done (lgkmcnt(0))
                    busy += __builtin_amdgcn_s_memtime() - ts0;
                }
                lds_barrier();
            }
        };
        const std::integral_constant<bool, true> full{};
        const std::integral_constant<bool, false> part{};
        const uint32_t nfull = N / 16;
        const unsigned long long tall0 = STAMP ? __builtin_amdgcn_s_memtime() : 0ull;
        uint32_t sc = 0;
        for (; sc + 1 < nfull; sc += 2) {
            sstep(sc, cur, pre, full);
            sstep(sc + 1, pre, cur, full);
        }
        if (sc < nsup) {
            sstep(sc, cur, pre, part);
            if (sc + 1 < nsup) sstep(sc + 1, pre, cur, part);
        }
        if (STAMP && lane == 0) {
            ctr_add(d, C_NALL + 0, busy);
            ctr_add(d, C_NALL + 3, __builtin_amdgcn_s_memtime() - tall0);
        }
        return;
    }

    // ------------------------------- hashers -------------------------------
    // role 0: h, g and f (NH = 1); role 1: g and f; role 2: h
    const uint32_t role = NH == 1 ? 0u : wave;
    FH fh{0, 0, 0};
    uint32_t iters = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, iters);
    const bool last_wave = NH == 1 || wave == 2;
    if (!ok && valid && last_wave) atomicOr(d.err, E_SHORT);
    uint32_t h = fh.h, g = fh.g, f = fh.f;
    auto run = [&](auto ROLEC) {
        constexpr uint32_t RO = decltype(ROLEC)::value;
        constexpr bool DO_H = RO != 1, DO_GF = RO != 2;
        uint32_t done = 0;
        // blocks [0, U) unpredicated, [U, U + P) predicated on j < nb
        auto blocks = [&](const uint32_t *OB, uint32_t nb, auto UC, auto PC) {
            constexpr int U = decltype(UC)::value, P = decltype(PC)::value;
            uint32_t v[U + P][5];
#pragma unroll
            for (int j = 0; j < U + P; j++)
#pragma unroll
                for (int i = 0; i < 5; i++)
                    if (DO_GF || i == 0 || i >= 3) v[j][i] = OB[(5 * j + i) * C2_ROWS];
#pragma unroll
            for (int j = 0; j < U + P; j++) {
                const uint32_t a = v[j][0], dd = v[j][3], e = v[j][4];
                uint32_t hn = h, gn = g, fn = f;
                if (DO_H) hn = fh_fold(h + a, fh_m(dd), e);
                if (DO_GF) {
                    const uint32_t b = v[j][1], c = v[j][2];
                    gn = fh_fold(g + b, fh_m(c), a);
                    fn = fh_fold(f + c, fh_m(b + e * FH_C1), dd);
                    fn += gn;
                    gn += fn;
                }
                if (j < U) {
                    h = hn; g = gn; f = fn;
                } else {
                    const bool act = (uint32_t)j < nb;
                    if (DO_H) h = act ? hn : h;
                    if (DO_GF) {
                        g = act ? gn : g;
                        f = act ? fn : f;
                    }
                }
            }
        };
        unsigned long long hbusy = 0;
        for (uint32_t t = 0; t <= nsteps; t++) {
            const unsigned long long ts0 = STAMP ? __builtin_amdgcn_s_memtime() : 0ull;
            if (t) {
                const uint32_t pb = (t - 1) & 1u;
                const uint32_t *OB = lb + pb * BW * C2_ROWS;
                const uint32_t be = bend[pb][lane];
                const uint32_t lim = min(be, iters);
                const uint32_t nb = lim > done ? lim - done : 0u;
                if (__all(nb >= NB)) blocks(OB, nb, std::integral_constant<int, NB>{}, std::integral_constant<int, 0>{});
                else if (__all(nb >= NB - 1))
                    blocks(OB, nb, std::integral_constant<int, NB - 1>{}, std::integral_constant<int, 1>{});
                else blocks(OB, nb, std::integral_constant<int, 0>{}, std::integral_constant<int, NB>{});
                done = be;
            }
            if (STAMP) {
                if (__any(h == 0x9E3779B9u && g == f)) __builtin_amdgcn_s_sleep(0);   // results consumed first
                hbusy += __builtin_amdgcn_s_memtime() - ts0;
            }
            if (t < nsteps) lds_barrier();
        }
        if (STAMP && lane == 0) ctr_add(d, C_NALL + (NH == 1 ? 1 : RO), hbusy);
    };
    if (NH == 1) run(std::integral_constant<uint32_t, 0>{});
    else if (wave == 1) run(std::integral_constant<uint32_t, 1>{});
    else run(std::integral_constant<uint32_t, 2>{});
    if (NH == 2) {
        if (wave == 1) {
            xgf[0][lane] = g;
            xgf[1][lane] = f;
        }
        lds_barrier();
        if (wave != 2) return;
        g = xgf[0][lane];
        f = xgf[1][lane];
    }
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
    if (lane == 0) ctr_add(d, C_X_CS_ROWS, (unsigned long long)nvalid);   // rows this launch hashed (measurement)
    if (valid) {
        fh.h = h; fh.g = g; fh.f = f;
        const uint32_t hv = ok ? fh.fin() : 0u;
        if (is_row) {
            d.cs[id] = hv;
            d.dirty[id] = 0;
        } else {
            d.dense_cs[id - d.NL] = hv;
        }
    }
}

template <int W, int NH, int STAMP = 0>
void launch_cs6_w(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t grid, hipStream_t s) {
    if (W == 19 && d.max_tail <= 21 && d.min_tail >= 19) {     // 13-digit incarnations: records of 38..40 bytes
        constexpr int NO = cs_no(W, 21);
        hipLaunchKernelGGL((k_checksum6<W, NO, c2_nb(W + 21), c2_bw(W + 21, NO), NH, STAMP>), dim3(grid), dim3(64 * (1 + NH)), 0, s,
                           d, list, count, d.addrw, (const uint4 *)d.rtail);
    } else {                                                   // any tail of up to 24 bytes
        constexpr int NO = cs_no(W, 24);
        hipLaunchKernelGGL((k_checksum6<W, NO, c2_nb(W + 24), c2_bw(W + 24, NO), NH, STAMP>), dim3(grid), dim3(64 * (1 + NH)), 0, s,
                           d, list, count, d.addrw, (const uint4 *)d.rtail);
    }
}
