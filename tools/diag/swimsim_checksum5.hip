// swimsim_checksum5.hip — phase C FarmHash-32 over the membership string (memberlist.go:83-128, go-farm
// Fingerprint32) for launches of many rows: 64 rows per workgroup (lane = row), THREE waves split by role:
//
//   wave 0 (F) : formats 4 members per step into a linear LDS buffer that starts at the first 20-byte block the step
//                does not complete yet (double-buffered by step parity) and publishes each row's count of complete
//                blocks (k_checksum3's formatter, with its record-tail prefetch PF steps ahead);
//   wave 1 (GF): the coupled g and f lanes (g = mur(c, g + b) + a, f = mur(b + e c1, f + c) + d, f += g, g += f),
//                M(c) and M(b + e c1) included, over the blocks F completed one step earlier;
//   wave 2 (H) : the h lane (h = mur(d, h + a) + e), M(d) included, over the same blocks.
// Included by swimsim_checksum.hip after swimsim_checksum3.hip.
//
// Why a third wave: one wave issues at most one VALU instruction per 4 cycles (MI355X_MICROARCH.md, "vector-
// instruction ISSUE cost"), and k_checksum3's hasher wave carried all three lanes: ~310 VALU instructions per step
// of 4 records (8 blocks), i.e. a floor of ~1,240 cycles per step for that wave alone, the same as the whole
// launch's measured step time. Split, the g/f wave issues ~2/3 of them and the h wave ~1/3, and the SIMD (one VALU
// instruction per 2 cycles from any of its waves) is shared by three waves of three workgroups. That needs at most
// 168 VGPRs per wave (three waves per SIMD): the formatter's record-tail prefetch is the large item (PF = 1: 64
// VGPRs, PF = 2: 128).
template <int W, int NO, int NB, int BW, int PF, int MODE = 0>
__global__ void __launch_bounds__(192, 3) k_checksum5(DS d, const uint32_t *list, const uint32_t *count,
                                                   const uint32_t *__restrict__ addrw, const uint4 *__restrict__ rtail) {
    __shared__ uint32_t buf[2 * BW * C2_ROWS];
    __shared__ uint32_t bend[2][C2_ROWS];        // blocks complete after step t (t & 1)
    __shared__ uint32_t ast[2][16 * 6];          // address words of a super step's 16 members (F only)
    __shared__ uint32_t xgf[2][C2_ROWS];         // g, f at the end (GF -> H)
    constexpr int Q = W / 4;                     // record words that are pure address words
    constexpr int NT = 2 * PF;                   // record-tail slots (PF steps ahead, double-buffered)
    static_assert(PF == 1 || PF == 2, "tail prefetch distance");
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
        if (MODE != 7) __builtin_amdgcn_s_setprio(2);
        const uint32_t ecap1 = d.ecap - 1;
        uint32_t pos = 0, hc = 0;                                  // bytes formatted; the stream's last 4 bytes
        uint4 cur[4], pre[4];                                      // row words: this super step, the next
        uint4 TA[NT][C2_IT], TB[NT][C2_IT];                        // record tails of steps u .. u+PF (slot u % NT)
        const char *rtb = (const char *)rtail;
        auto tails = [&](uint4 q4, uint4 (&ta)[C2_IT], uint4 (&tb)[C2_IT]) {
            const uint32_t ws[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
            for (int k = 0; k < C2_IT; k++) {                    // 32-byte entries, 32-bit byte offsets
                const uint32_t off = ((min(ws[k] >> 3, ecap1) << 2) + (ws[k] & 3u)) << 5;
                ta[k] = *(const uint4 *)(rtb + off);
                tb[k] = *(const uint4 *)(rtb + off + 16u);
            }
        };
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
#pragma unroll
        for (int k = 0; k < PF; k++) tails(cur[k], TA[k], TB[k]);
        uint32_t AN[C2_IT][Q + 1], cw[5] = {0, 0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < C2_IT; k++)
#pragma unroll
            for (int i = 0; i <= Q; i++) AN[k][i] = ast[0][k * 6 + i];
        auto sstep = [&](uint32_t sc, uint4 (&cur)[4], uint4 (&pre)[4], auto FULLC) {
            constexpr bool FULL = decltype(FULLC)::value;
            ast[(sc + 1) & 1u][lane] = ap0;
            if (lane < 32) ast[(sc + 1) & 1u][64 + lane] = ap1;
            aload(sc + 2, ap0, ap1);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t t = sc * 4 + u;
                const uint32_t mb = t * C2_IT;
                // prefetch: tails PF steps ahead, row words one super step ahead, next step's address words
                tails(u + PF < 4 ? cur[u + PF] : pre[u + PF - 4], TA[(u + PF) % NT], TB[(u + PF) % NT]);
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
                const uint4 *ta = TA[u % NT], *tb = TB[u % NT];
                const uint32_t ws[4] = {cur[u].x, cur[u].y, cur[u].z, cur[u].w};
#pragma unroll
                for (int k = 0; k < C2_IT; k++) {
                    const uint32_t m = mb + k;
                    const uint32_t L = ((ws[k] & 7u) < 4u && (FULL || m < N)) ? (tb[k].z >> 24) : 0u;
                    const uint32_t sh = pos & 3u;
                    const uint32_t sel = 0x07060504u - __builtin_amdgcn_perm(0u, sh, 0u);
                    const uint32_t C[7] = {ta[k].x, ta[k].y, ta[k].z, ta[k].w, tb[k].x, tb[k].y, tb[k].z};
                    uint32_t R[NO];
#pragma unroll
                    for (int i = 0; i < NO; i++)
                        R[i] = i < Q ? A[k][i] : (i == Q ? (A[k][Q] | C[0]) : (i - Q < 7 ? C[i - Q] : 0u));
                    uint32_t *wb = B + ((pos >> 2) - 5u * b0) * C2_ROWS;
#pragma unroll
                    for (int j = 0; j < NO; j++) wb[j * C2_ROWS] = __builtin_amdgcn_perm(R[j], j ? R[j - 1] : hc, sel);
                    hc = L ? tb[k].w : hc;
                    pos += L;
                }
                const uint32_t b1 = pos / 20u;
                bend[pb][lane] = b1;
#pragma unroll
                for (int i = 0; i < 5; i++) cw[i] = B[(5 * (b1 - b0) + i) * C2_ROWS];
                if (u == 3 && sc + 2 < nsup) {
#pragma unroll
                    for (int k = 0; k < 4; k++) cur[k] = *(const uint4 *)(row + (sc + 2) * 16 + 4 * k);
                }
                lds_barrier();
            }
        };
        const std::integral_constant<bool, true> full{};
        const std::integral_constant<bool, false> part{};
        const uint32_t nfull = N / 16;
        uint32_t sc = 0;
        for (; sc + 1 < nfull; sc += 2) {
            sstep(sc, cur, pre, full);
            sstep(sc + 1, pre, cur, full);
        }
        if (sc < nsup) {
            sstep(sc, cur, pre, part);
            if (sc + 1 < nsup) sstep(sc + 1, pre, cur, part);
        }
        return;
    }

    // ------------------------------- hashers: g/f (wave 1), h (wave 2) -------------------------------
    FH fh{0, 0, 0};
    uint32_t iters = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, iters);
    if (!ok && valid && wave == 2) atomicOr(d.err, E_SHORT);
    uint32_t h = fh.h, g = fh.g, f = fh.f;
    // one loop per role (each wave's own register allocation and schedule); blocks every lane has (a uniform count,
    // no predication) first, then the predicated rest
    auto run = [&](auto GFC) {
        constexpr bool GF = decltype(GFC)::value;
        uint32_t done = 0;
        for (uint32_t t = 0; t <= nsteps; t++) {
            if (t) {
                const uint32_t pb = (t - 1) & 1u;
                const uint32_t *OB = lb + pb * BW * C2_ROWS;
                const uint32_t be = bend[pb][lane];
                const uint32_t lim = min(be, iters);
                const uint32_t nb = lim > done ? lim - done : 0u;
                const uint32_t jall = __all(nb >= NB) ? NB : __all(nb >= NB - 1) ? NB - 1 : 0u;
                if (GF) {
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
                        if ((uint32_t)j < jall) {
                            g = gn; f = fn;
                        } else {
                            const bool act = (uint32_t)j < nb;
                            g = act ? gn : g;
                            f = act ? fn : f;
                        }
                    }
                } else {
                    uint32_t v[NB][3];
#pragma unroll
                    for (int j = 0; j < NB; j++) {
                        v[j][0] = OB[(5 * j) * C2_ROWS];
                        v[j][1] = OB[(5 * j + 3) * C2_ROWS];
                        v[j][2] = OB[(5 * j + 4) * C2_ROWS];
                    }
#pragma unroll
                    for (int j = 0; j < NB; j++) {
                        const uint32_t hn = fh_fold(h + v[j][0], fh_m(v[j][1]), v[j][2]);
                        if ((uint32_t)j < jall) h = hn;
                        else h = (uint32_t)j < nb ? hn : h;
                    }
                }
                done = be;
            }
            if (t < nsteps) lds_barrier();
        }
    };
    if (wave == 1) run(std::integral_constant<bool, true>{});
    else run(std::integral_constant<bool, false>{});
    if (wave == 1) {
        xgf[0][lane] = g;
        xgf[1][lane] = f;
    }
    lds_barrier();
    if (wave != 2) return;
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
    if (lane == 0) ctr_add(d, C_X_CS_ROWS, (unsigned long long)nvalid);   // rows this launch hashed (measurement)
    if (valid) {
        fh.h = h; fh.g = xgf[0][lane]; fh.f = xgf[1][lane];
        const uint32_t hv = ok ? fh.fin() : 0u;
        if (is_row) {
            d.cs[id] = hv;
            d.dirty[id] = 0;
        } else {
            d.dense_cs[id - d.NL] = hv;
        }
    }
}

template <int W, int PF>
void launch_cs5_w(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t grid, hipStream_t s) {
    if (W == 19 && d.max_tail <= 21 && d.min_tail >= 19) {     // 13-digit incarnations: records of 38..40 bytes
        constexpr int NO = cs_no(W, 21);
        hipLaunchKernelGGL((k_checksum5<W, NO, c2_nb(W + 21), c2_bw(W + 21, NO), PF>), dim3(grid), dim3(192), 0, s, d, list,
                           count, d.addrw, (const uint4 *)d.rtail);
    } else {                                                   // any tail of up to 24 bytes
        constexpr int NO = cs_no(W, 24);
        hipLaunchKernelGGL((k_checksum5<W, NO, c2_nb(W + 24), c2_bw(W + 24, NO), PF>), dim3(grid), dim3(192), 0, s, d, list,
                           count, d.addrw, (const uint4 *)d.rtail);
    }
}
