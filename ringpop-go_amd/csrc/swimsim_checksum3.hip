// swimsim_checksum3.hip — phase C FarmHash-32 over the membership string (memberlist.go:83-128, go-farm
// Fingerprint32), 64 rows per workgroup (lane = row), two waves split by role:
//
//   wave 0 (F): formats 4 members per step into a linear LDS buffer that starts at the first 20-byte block the
//               step does not complete yet (double-buffered by step parity) and publishes each row's count of
//               complete blocks. It hashes nothing;
//   wave 1 (H): runs all three FarmHash-mk lanes of every row (h, and the coupled g and f) over the blocks F
//               completed one step earlier, the M() premixes included.
// Included by swimsim_checksum.hip (record tables, buffer geometry C2_* and lds_barrier are defined there). The
// superseded k_checksum2, whose formatter wave also ran the h lane, lives in tools/diag.
//
// Why the split moved: the chain arithmetic needs no LDS round trip of its own, while the formatter's work is
// LDS-latency bound (carry copy, record writes, address-word broadcasts). With the h lane on the formatter,
// the formatter was the slower wave of every step (about 290 VALU instructions per step against the g/f
// wave's 136, profiles/r02_pmc_summary.json and the k_checksum2 ISA), and both waited for it at the barrier.

// MODE (diagnostics): 0 normal; 1 formatter only (the hasher wave only meets the barriers); 2 hasher only (the
// formatter publishes 8 blocks per step and writes nothing; checksums are garbage); 3 as 2 without the
// per-block predication; 4 as 3 without the hasher's LDS reads (block words from registers); 5 formatter only,
// without its record stores (the words are folded into a register)
template <int W, int NO, int NB, int BW, int MODE = 0, int G = 1>
__global__ void __launch_bounds__(128 * G) k_checksum3(DS d, const uint32_t *list, const uint32_t *count,
                                                       const uint32_t *__restrict__ addrw, const uint4 *__restrict__ rtail) {
    __shared__ uint32_t bufs[G][2 * BW * C2_ROWS];
    __shared__ uint32_t bends[G][2][C2_ROWS];    // blocks complete after step t (t & 1)
    __shared__ uint32_t asts[G][2][16 * 6];      // address words of a super step's 16 members (F only)
    constexpr int Q = W / 4;                     // record words that are pure address words
    static_assert(NO <= Q + 8, "record tail table holds 7 words after the address words");
    static_assert(5 * NB + 4 < BW, "hasher reads past the buffer");
    const uint32_t cnt = *count;
    if (blockIdx.x * C2_ROWS * G >= cnt) return;                   // uniform per workgroup
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), grp = 0;
    if (G > 1) {
        // G row groups of 64 rows, each a formatter and a hasher wave. A workgroup of 2 G waves lands on the CU's four
        // SIMDs two per SIMD; each SIMD should hold one formatter and one hasher (two hashers on one SIMD share its
        // VALU and take twice as long), so the roles follow the placement read from HW_ID: on SIMD x the first wave
        // formats and the second hashes row group x. An uneven placement keeps the wave-index roles.
        __shared__ uint32_t simd_n[4];
        uint32_t hwid;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        const uint32_t simd = (hwid >> 4) & 3u;
        if (threadIdx.x < 4) simd_n[threadIdx.x] = 0u;
        __syncthreads();
        uint32_t slot = 0;
        if (lane == 0) slot = atomicAdd(&simd_n[simd], 1u);
        slot = __builtin_amdgcn_readfirstlane(slot);
        __syncthreads();
        const bool even = G == 4 && simd_n[0] == 2u && simd_n[1] == 2u && simd_n[2] == 2u && simd_n[3] == 2u;
        grp = even ? simd : wave % G;
        wave = even ? slot : wave / G;
    }
    uint32_t *const buf = bufs[grp];
    uint32_t (*const bend)[C2_ROWS] = bends[grp];
    uint32_t (*const ast)[16 * 6] = asts[grp];
    const uint32_t gi = (blockIdx.x * G + grp) * C2_ROWS + lane;
    const bool valid = gi < cnt;
    const uint32_t id = list[valid ? gi : blockIdx.x * C2_ROWS * G];
    const bool is_row = id < d.NL;
    const uint32_t *row = is_row ? d.mw + (size_t)id * d.NP : d.dense + (size_t)(id - d.NL) * d.NP;
    const uint32_t N = d.N;
    const uint32_t nsup = (N + 15) / 16;                           // super steps of 16 members (4 steps)
    const uint32_t nsteps = nsup * 4;

    uint32_t *const lb = buf + lane;                               // this lane's column

    if (wave == 0) {
        // ------------------------------- formatter -------------------------------
        // The formatter sets the pace of a step (10.5 ms alone for one row group against the hasher's 9.6), and the
        // SIMD arbitrates VALU issue between its two waves by priority, then age: raised, it takes its issue slots
        // ahead of the co-resident hasher wave (17.8 -> 14.6 ms at 65,536 rows, 17.1 -> 13.6 ms at 32,768)
        if (MODE != 7) __builtin_amdgcn_s_setprio(2);             // (MODE 7: diagnostics without it)
        const uint32_t wmax = d.ecap * 8u - 1u;                     // last member word of the record table
        uint32_t pos = 0, hc = 0;                                  // bytes formatted; the stream's last 4 bytes
        uint4 cur[4], pre[4];                                      // row words: this super step, the next
        uint4 TA[4][C2_IT], TB[4][C2_IT];                          // record tails of steps u .. u+2 (slot u & 3)
        // rtail is d.rtail8, indexed by the member word: 32-byte entries, 32-bit byte offsets
        const char *rtb = (const char *)rtail;
        auto tails = [&](uint4 q4, uint4 (&ta)[C2_IT], uint4 (&tb)[C2_IT]) {
            const uint32_t ws[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
            for (int k = 0; k < C2_IT; k++) {
                const uint32_t off = min(ws[k], wmax) << 5;
                ta[k] = *(const uint4 *)(rtb + off);
                tb[k] = *(const uint4 *)(rtb + off + 16u);
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
        // address words of the next step's 4 records and the carry of the next buffer are read one step ahead
        // (LDS reads complete in issue order: a read issued before a step's record writes is waited for
        // without waiting for those writes)
        uint32_t AN[C2_IT][Q + 1], cw[5] = {0, 0, 0, 0, 0}, sink = 0;
#pragma unroll
        for (int k = 0; k < C2_IT; k++)
#pragma unroll
            for (int i = 0; i <= Q; i++) AN[k][i] = ast[0][k * 6 + i];
        // one super step with row words C (this one) and P (the next). The two alternate between super steps instead of
        // being copied: a copy of just-loaded registers at the loop's back edge made every super step wait for the
        // next one's row loads (s_waitcnt vmcnt(0) at the top of the loop)
        auto sstep = [&](uint32_t sc, uint4 (&cur)[4], uint4 (&pre)[4], auto FULLC) {
            constexpr bool FULL = decltype(FULLC)::value;               // every member of the super step is < N
            ast[(sc + 1) & 1u][lane] = ap0;                         // stage super step sc + 1, load sc + 2
            if (lane < 32) ast[(sc + 1) & 1u][64 + lane] = ap1;
            aload(sc + 2, ap0, ap1);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t t = sc * 4 + u;
                const uint32_t mb = t * C2_IT;
                // prefetch: tails two steps ahead, row words one super step ahead, next step's address words
                tails(u < 2 ? cur[u + 2] : pre[u - 2], TA[(u + 2) & 3], TB[(u + 2) & 3]);
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
                uint32_t *B = lb + pb * BW * C2_ROWS;                    // this step's buffer
                const uint32_t b0 = pos / 20u;                              // this buffer's base block
                // carry: the words of the block the previous step left incomplete (read at its end) go to
                // this buffer's front
                if (MODE >= 2 && MODE <= 4) {
                    bend[pb][lane] = (t + 1) * 8;
                    lds_barrier();
                    continue;
                }
#pragma unroll
                for (int i = 0; i < 5; i++) B[i * C2_ROWS] = cw[i];
                // format this step's 4 records: every record writes NO words at its position
                const uint4 *ta = TA[u], *tb = TB[u];
#pragma unroll
                for (int k = 0; k < C2_IT; k++) {
                    const uint32_t m = mb + k;
                    const uint32_t L = (FULL || m < N) ? (tb[k].z >> 24) : 0u;   // 0: tombstone / unknown
                    const uint32_t sh = pos & 3u;
                    // sh * 0x01010101 as a byte broadcast (one full-rate v_perm, not a multiply)
                    const uint32_t sel = 0x07060504u - __builtin_amdgcn_perm(0u, sh, 0u);
                    const uint32_t C[7] = {ta[k].x, ta[k].y, ta[k].z, ta[k].w, tb[k].x, tb[k].y, tb[k].z};
                    uint32_t R[NO];
#pragma unroll
                    for (int i = 0; i < NO; i++)
                        R[i] = i < Q ? A[k][i] : (i == Q ? (A[k][Q] | C[0]) : (i - Q < 7 ? C[i - Q] : 0u));
                    uint32_t *wb = B + ((pos >> 2) - 5u * b0) * C2_ROWS;
#pragma unroll
                    for (int j = 0; j < NO; j++) {
                        const uint32_t wj = __builtin_amdgcn_perm(R[j], j ? R[j - 1] : hc, sel);
                        if (MODE == 5) sink ^= wj + j; else wb[j * C2_ROWS] = wj;
                    }
                    hc = L ? tb[k].w : hc;
                    pos += L;
                }
                const uint32_t b1 = pos / 20u;
                bend[pb][lane] = b1;
#pragma unroll
                for (int i = 0; i < 5; i++) cw[i] = B[(5 * (b1 - b0) + i) * C2_ROWS];     // the next carry
                if (u == 3 && sc + 2 < nsup) {                             // row words of super step sc + 2
#pragma unroll
                    for (int k = 0; k < 4; k++) cur[k] = *(const uint4 *)(row + (sc + 2) * 16 + 4 * k);
                }
                lds_barrier();
            }
        };
        // super steps whose 16 members all exist skip the per-record bounds test (scalar compares that a lone wave
        // pays issue slots for); at most the last super step is partial
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
        if (MODE == 5 && sink == 0x12345678u) d.ctr[0] = sink;  // keeps the folded words alive (never true)
        return;
    }

    // ------------------------------- h, g and f lanes -------------------------------
    FH fh{0, 0, 0};
    uint32_t iters = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, iters);
    if (!ok && valid) atomicOr(d.err, E_SHORT);
    uint32_t h = fh.h, g = fh.g, f = fh.f, done = 0;
    for (uint32_t t = 0; t <= nsteps; t++) {
        if (t && MODE != 1 && MODE != 5) {
            const uint32_t pb = (t - 1) & 1u;
            const uint32_t *OB = lb + pb * BW * C2_ROWS;
            const uint32_t be = bend[pb][lane];
            const uint32_t lim = min(be, iters);
            uint32_t v[NB][5];
#pragma unroll
            for (int j = 0; j < NB; j++)
#pragma unroll
                for (int i = 0; i < 5; i++) v[j][i] = MODE == 4 ? (t * 977u + j * 31u + i) ^ lane : OB[(5 * j + i) * C2_ROWS];
            // blocks every lane has (a uniform count: no predication) first, then the predicated rest. The three
            // cases are separate code paths: with one loop and a run-time jall the compiler if-converts every block's
            // update into v_cndmask selects (21 per step of 8 blocks, about 5 % of the hasher's VALU cycles)
            const uint32_t nb = lim > done ? lim - done : 0u;
            const uint32_t jall = (MODE == 3 || MODE == 4) ? NB : __all(nb >= NB) ? NB : __all(nb >= NB - 1) ? NB - 1 : 0u;
            auto blocks = [&](auto JALL) {
                constexpr uint32_t JA = decltype(JALL)::value;
#pragma unroll
                for (int j = 0; j < NB; j++) {
                    const uint32_t a = v[j][0], b = v[j][1], c = v[j][2], dd = v[j][3], e = v[j][4];
                    const uint32_t hn = fh_fold(h + a, fh_m(dd), e);
                    uint32_t gn = fh_fold(g + b, fh_m(c), a);
                    uint32_t fn = fh_fold(f + c, fh_m(b + e * FH_C1), dd);
                    fn += gn;
                    gn += fn;
                    if ((uint32_t)j < JA) {
                        h = hn; g = gn; f = fn;
                    } else {
                        const bool act = (uint32_t)j < nb;
                        h = act ? hn : h;
                        g = act ? gn : g;
                        f = act ? fn : f;
                    }
                }
            };
            if (jall == NB) blocks(std::integral_constant<uint32_t, NB>{});
            else if (jall == NB - 1) blocks(std::integral_constant<uint32_t, NB - 1>{});
            else blocks(std::integral_constant<uint32_t, 0>{});
            done = be;
        }
        if (t < nsteps) lds_barrier();
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

template <int W, int MODE = 0, int G = 1>
void launch_cs3_w(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t grid, hipStream_t s) {
    if (W == 19 && d.max_tail <= 21 && d.min_tail >= 19) {     // 13-digit incarnations: records of 38..40 bytes
        constexpr int NO = cs_no(W, 21);
        hipLaunchKernelGGL((k_checksum3<W, NO, c2_nb(W + 21), c2_bw(W + 21, NO), MODE, G>), dim3(grid), dim3(128 * G), 0, s, d,
                           list, count, d.addrw, (const uint4 *)d.rtail8);
    } else {                                                   // any tail of up to 24 bytes
        constexpr int NO = cs_no(W, 24);
        hipLaunchKernelGGL((k_checksum3<W, NO, c2_nb(W + 24), c2_bw(W + 24, NO), 0, G>), dim3(grid), dim3(128 * G), 0, s, d,
                           list, count, d.addrw, (const uint4 *)d.rtail8);
    }
}
