// swimsim_checksum2.hip — phase C FarmHash-32 over the membership string (memberlist.go:83-128, go-farm
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

constexpr int C2_ROWS = 64;
constexpr int C2_IT = 4;                         // members per step
// for records of at most RMAX bytes: blocks one step can complete, words per buffer per lane (the last record
// of a step starts at most 19 + 3 * RMAX bytes past the buffer's base and writes NO words)
constexpr int c2_nb(int rmax) { return (19 + C2_IT * rmax) / 20; }
constexpr int c2_bw(int rmax, int no) {     // and every hasher / carry read of NB blocks stays inside
    return (19 + (C2_IT - 1) * rmax) / 4 + no + 1 > 5 * c2_nb(rmax) + 5 ? (19 + (C2_IT - 1) * rmax) / 4 + no + 1
                                                                       : 5 * c2_nb(rmax) + 5;
}

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
