// swimsim_checksum4.hip — phase C FarmHash-32 for launches of few rows (memberlist.go:83-128, go-farm
// Fingerprint32): the chain in carried-sum form, one row per lane quad. Included by swimsim_kernels.hip after
// swimsim_checksum3.hip (k_checksum_n16's byte ring, record tables and formatter).
//
// A launch of few rows is bounded by one row's chain. The FarmHash-mk block
//     h += a; g += b; f += c; h = mur(d, h) + e; g = mur(c, g) + a; f = mur(b + e c1, f) + d; f += g; g += f
// is rewritten over the values that enter the xor, Xh = h + a, Xg = g + b, Xf = f + c, so that every term
// that does not depend on the chain is folded into per-block constants:
//     F   = 5 ror(X ^ M, 19)                       (M = M(d), M(c), M(b + e c1) for the h, g, f lanes)
//     Xg' = 2 F_g + F_f + PG,   PG = 3C + 2a + d + b'
//     Xf' =   F_f + F_g + PF,   PF = 2C + a + d + c'
//     Xh' =   F_h       + KH,   KH =  C + e + a'
// (C = 0xe6546b64; a', b', c' = the next block's first words, 0 after the last block, so that the carried
// values are h, g and f themselves at the end). Lanes 4r .. 4r+3 carry (Xg, Xf, Xh, 0) of row r; the partner
// term is one DPP quad permutation [1, 0, 3, 3], so a block is five dependent VALU instructions for all three
// lanes (tools/chainq.hip: 43.5 cycles per block fed from LDS, against 97-150 for the per-lane forms).
//
// 16 rows per workgroup, five waves:
//   wave 0     (chain)    : lane = (row, lane of the quad); one ds_read_b64 {M, K} per block;
//   waves 1, 2 (premix)   : lane = (row, block slot s of 8): the three M() premixes and the constants of every
//                           block, into a ring of CQ_MB premixed blocks;
//   waves 3, 4 (formatter): k_checksum_n16's formatters (lane = (row, record of the step)) into the byte ring.
// At step t the formatters write step t, premix takes the blocks whose bytes and the next block's first 12
// bytes were complete at step t-1, and the chain the blocks premixed at step t-1.
constexpr int CQ_MB = 64;                       // premixed blocks per ring (power of two)

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}

__device__ __forceinline__ void fh_quad_step(uint32_t &X, uint32_t m, uint32_t k, uint32_t sh) {
    // s_nop 1: a DPP read of a VGPR needs two wait states after the VALU write of that VGPR
    uint32_t t;
    asm volatile("v_xor_b32 %0, %0, %2\n\t"
        "v_alignbit_b32 %0, %0, %0, 19\n\t"
        "v_lshl_add_u32 %0, %0, 2, %0\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %1, %0, %3 quad_perm:[1,0,3,3] row_mask:0xf bank_mask:0xf\n\t"
        "v_lshl_add_u32 %0, %0, %4, %1"
        : "+v"(X), "=&v"(t)
        : "v"(m), "v"(k), "v"(sh));
}

// IT = records per row per step (8 or 16): IT / 4 formatter waves and IT / 4 premix waves
template <int IT> struct QGeo {
    static constexpr int FW = IT / 4, PW = IT / 4;
    // IT = 16 runs one workgroup per CU (LDS): 12 waves, of which the three that share the chain wave's SIMD
    // (waves 4, 8, 11 of wave w on SIMD (base + w) % 4) exit at once, so the chain has its SIMD to itself
    static constexpr int WAVES = IT == 8 ? 1 + FW + PW : 12, THREADS = 64 * WAVES;
    // role of wave w: 0 chain, 1 + i formatter i, 1 + FW + i premix i, -1 none
    __device__ static int role(int w) {
        if (IT == 8) return w;
        // nibble w of 0xf87f465f3210 (0xf = none)
        const int v = (int)((0xf87f465f3210ull >> (4 * w)) & 0xf);
        return v == 0xf ? -1 : v;
    }
    static constexpr int RING = IT == 8 ? 250 : 530;                 // ring words per row (whole blocks)
    static constexpr int NBLK = RING / 5;
    static constexpr int SINK = CS_PRE + RING + CN_MIR;
    static constexpr int STRIDE = SINK + 13;                         // odd: the rows' words fall in distinct banks
    static constexpr int MB = IT == 8 ? 64 : 128;                    // premixed blocks per ring (power of two)
};

// QMODE (diagnostics): 0 normal; 1 chain idle (premix and formatters only); 2 premix and chain idle; 3 chain only
// (formatters publish 38-byte records without work, premix idle; garbage checksums); 4 formatters and chain (premix
// idle); 5 premix and chain (formatters as in 3); 7 the chain alone over every block, no pipeline (garbage)
template <int W, int NO, int JMIN, int IT, int QMODE = 0>
__global__ void __launch_bounds__(QGeo<IT>::THREADS) k_checksum_q16(DS d, const uint32_t *list, const uint32_t *count,
                                                      const uint32_t *__restrict__ addrw, const uint4 *__restrict__ rtail) {
    using G = QGeo<IT>;
    constexpr int CQ_MB = G::MB;
    __shared__ uint32_t ring[CN_ROWS * G::STRIDE];
    __shared__ uint2 mring[CQ_MB * 64];                             // [block % CQ_MB][row][g, f, h, 0] {M, K}
    __shared__ uint32_t wp[4][CN_ROWS];
    __shared__ uint32_t xinit[CN_ROWS][4];                          // the string's words 1, 2, 0 (g, f, h lanes)
    constexpr int Q = W / 4;
    static_assert(NO <= CS_PRE + 1 && NO <= 13, "spill areas too small");
    static_assert(CS_PRE + CN_MIR - 1 + G::RING + NO - 1 < G::STRIDE, "mirror pass overruns the row");
    static_assert(G::STRIDE % 2 == 1 && G::RING % 5 == 0, "ring geometry");
    static_assert(CQ_MB * 20 >= 2 * IT * 44 + 4 * 20 + 40, "premixed ring too small for two steps");
    static_assert(NO <= Q + 8, "record tail table holds 7 words after the address words");
    static_assert(G::RING * 4 >= 2 * IT * 44 + 32 + 20, "premix reads two steps behind the formatter");
    const uint32_t cnt = *count;
    const uint32_t b0 = blockIdx.x * CN_ROWS;
    if (b0 >= cnt) return;                                         // uniform per workgroup
    const int wrole = G::role(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
    if (wrole < 0) return;                                         // waves that ended do not hold barriers
    if (QMODE == 7 && wrole != 0) return;
    const uint32_t wave = (uint32_t)wrole, lane = threadIdx.x & 63u;
    const uint32_t N = d.N, ecap1 = d.ecap - 1;
    const uint32_t nit = (N + IT - 1) / IT;
    const uint32_t nsteps = nit + 2;
    auto row_of = [&](uint32_t r, uint32_t &id, bool &is_row) -> const uint32_t * {
        const uint32_t gi = b0 + r;
        id = list[gi < cnt ? gi : b0];
        is_row = id < d.NL;
        return is_row ? d.mw + (size_t)id * d.NP : d.dense + (size_t)(id - d.NL) * d.NP;
    };
    // blocks whose bytes and the next block's first 12 bytes are formatted once pos bytes are
    auto premixable = [&](uint32_t pos, uint32_t iters) { return min(iters, pos >= 12u ? (pos - 12u) / 20u : 0u); };

    if (wave >= 1 && wave <= (uint32_t)G::FW) {
        // ------------------------------- formatters (as k_checksum_n16) -------------------------------
        if (QMODE == 8) __builtin_amdgcn_s_setprio(2);
        const uint32_t r = (wave - 1) * (64 / IT) + lane / IT, k = lane % IT;
        uint32_t id; bool is_row;
        const uint32_t *row = row_of(r, id, is_row);
        uint32_t *rrow = ring + r * G::STRIDE;
        uint32_t pos = 0, phys = 0, hc = 0;
        auto ldw = [&](uint32_t t) { const uint32_t m = IT * t + k; return m < N ? row[m] : (uint32_t)ST_UNKNOWN; };
        auto ldt = [&](uint32_t w, uint4 &xa, uint4 &xb) {
            const size_t ti = ((size_t)min(w >> 3, ecap1) * 4 + (w & 3u)) * 2;
            xa = rtail[ti];
            xb = rtail[ti + 1];
        };
        auto lda = [&](uint32_t t, uint32_t (&xA)[Q + 1]) {
            const uint32_t *ap = addrw + (size_t)min(IT * t + k, N - 1) * 6;
#pragma unroll
            for (int i = 0; i <= Q; i++) xA[i] = ap[i];
        };
        // prefetch rings (slot = step & 3): row words four steps ahead, record tails (which need the row
        // word) and address words two steps ahead; a launch of few rows waits on memory latency otherwise
        uint32_t wr[4];
        uint4 ta[4], tb[4];
        uint32_t A[4][Q + 1];
#pragma unroll
        for (int i = 0; i < 4; i++) wr[i] = ldw(i);
        ldt(wr[0], ta[0], tb[0]);
        lda(0, A[0]);
        ldt(wr[1], ta[1], tb[1]);
        lda(1, A[1]);
        auto step = [&](uint32_t t, auto B) {
            constexpr int b = decltype(B)::value, b2 = (b + 2) & 3;
            if (QMODE == 3 || QMODE == 5) {
                pos += IT * 38;
                if (k == 0) wp[t & 3][r] = pos;
                lds_barrier();
                return;
            }
            const uint32_t w = wr[b];
            wr[b] = ldw(t + 4);
            ldt(wr[b2], ta[b2], tb[b2]);
            lda(t + 2, A[b2]);
            const uint32_t m = IT * t + k;
            const uint32_t L = ((w & 7u) < 4u && m < N) ? (tb[b].z >> 24) : 0u;
            // segmented scans over the row's IT records by DPP (lane k of an IT-lane segment; row_shr stays inside
            // a 16-lane row, and the lanes it would take from the neighbouring segment keep their value):
            // inclusive sum of the record lengths, and the last word of the last non-empty record so far
            uint32_t inc = L, hv = L ? tb[b].w : 0u;
            auto scan = [&](auto OFF) {
                constexpr int off = decltype(OFF)::value;
                const uint32_t y = dpp_u32<0x110 + off>(inc), yv = dpp_u32<0x110 + off>(hv);
                hv = k >= (uint32_t)off && !inc ? yv : hv;
                inc = k >= (uint32_t)off ? inc + y : inc;
            };
            scan(std::integral_constant<int, 1>{});
            scan(std::integral_constant<int, 2>{});
            scan(std::integral_constant<int, 4>{});
            if (IT == 16) scan(std::integral_constant<int, 8>{});
            const uint32_t ex = inc - L;
            const uint32_t pinc = dpp_u32<0x111>(inc), pv = dpp_u32<0x111>(hv);
            const uint32_t carry = (k >= 1 && pinc) ? pv : hc;         // last bytes before this record
            // the last lane's totals to the whole segment: (half-)row mirror (lane 0 <- lane IT-1), then copies to
            // lanes 1, 2-3, 4-7 (, 8-15)
            uint32_t total = dpp_u32<IT == 8 ? 0x141 : 0x140>(inc), lastv = dpp_u32<IT == 8 ? 0x141 : 0x140>(hv);
            auto bcast = [&](auto OFF) {
                constexpr int off = decltype(OFF)::value;
                const uint32_t y = dpp_u32<0x110 + off>(total), yv = dpp_u32<0x110 + off>(lastv);
                const bool take = k >= (uint32_t)off && k < 2u * off;
                total = take ? y : total;
                lastv = take ? yv : lastv;
            };
            bcast(std::integral_constant<int, 1>{});
            bcast(std::integral_constant<int, 2>{});
            bcast(std::integral_constant<int, 4>{});
            if (IT == 16) bcast(std::integral_constant<int, 8>{});
            const uint32_t sh0 = pos & 3u;
            const uint32_t sh = (sh0 + ex) & 3u;
            uint32_t ph = phys + ((sh0 + ex) >> 2);
            ph = ph >= G::RING ? ph - G::RING : ph;
            {
                const uint32_t C[7] = {ta[b].x, ta[b].y, ta[b].z, ta[b].w, tb[b].x, tb[b].y, tb[b].z};
                const uint32_t sel = 0x07060504u - sh * 0x01010101u;
                const uint32_t nw = (sh + L) >> 2;
                uint32_t R[NO], O[NO];
#pragma unroll
                for (int i = 0; i < NO; i++)
                    R[i] = i < Q ? A[b][i] : (i == Q ? (A[b][Q] | C[0]) : (i - Q < 7 ? C[i - Q] : 0u));
#pragma unroll
                for (int j = 0; j < NO; j++) O[j] = __builtin_amdgcn_perm(R[j], j ? R[j - 1] : carry, sel);
                const uint32_t i0 = L ? CS_PRE + ph : (uint32_t)G::SINK;
#pragma unroll
                for (int j = 0; j < NO; j++) rrow[(j < JMIN || (uint32_t)j < nw ? i0 : (uint32_t)G::SINK) + j] = O[j];
                if (L && (ph < CN_MIR || ph + nw > G::RING)) {
                    const uint32_t i1 = CS_PRE + (ph < CN_MIR ? ph + G::RING : ph - G::RING);
#pragma unroll
                    for (int j = 0; j < NO; j++) rrow[(j < JMIN || (uint32_t)j < nw ? i1 : (uint32_t)G::SINK) + j] = O[j];
                }
            }
            uint32_t np = phys + ((sh0 + total) >> 2);
            phys = np >= G::RING ? np - G::RING : np;
            pos += total;
            hc = total ? lastv : hc;
            if (k == 0) wp[t & 3][r] = pos;
            lds_barrier();
        };
        uint32_t t = 0;
        for (; t + 3 < nit; t += 4) {
            step(t, std::integral_constant<int, 0>{});
            step(t + 1, std::integral_constant<int, 1>{});
            step(t + 2, std::integral_constant<int, 2>{});
            step(t + 3, std::integral_constant<int, 3>{});
        }
        if (t < nit) step(t, std::integral_constant<int, 0>{});
        if (t + 1 < nit) step(t + 1, std::integral_constant<int, 1>{});
        if (t + 2 < nit) step(t + 2, std::integral_constant<int, 2>{});
        lds_barrier();                                             // the two drain steps
        lds_barrier();
        return;
    }

    if (wave >= 1) {
        // ------------------------------- premix -------------------------------
        const uint32_t pw = wave - 1 - G::FW;
        // lane = (row r, block slot s): the 16 rows of a slot are adjacent lanes, so one write instruction covers
        // a block's 16 rows (512 contiguous bytes) and four blocks, not one row of sixteen blocks (which would
        // all fall in the same banks)
        const uint32_t r = lane & 15u, s = pw * 4 + (lane >> 4);
        for (uint32_t i = pw * 64 + lane; i < CQ_MB * 16; i += 64 * G::PW) mring[i * 4 + 3] = make_uint2(0u, 0u);   // the quads' 4th lanes
        uint32_t id; bool is_row;
        (void)row_of(r, id, is_row);
        const uint32_t len = is_row ? d.clen[id] : d.dense_len[id - d.NL];
        const uint32_t iters = len > 24 ? (len - 1) / 20 : 0u;
        const uint32_t *rrow = ring + r * G::STRIDE + CS_PRE;
        uint2 *mrow = mring + 4 * r;
        uint32_t blk = s, q = s;                                    // next block of this lane, its ring block
        for (uint32_t t = 0; t < nsteps; t++) {
            const uint32_t lim = (t == 0 || (QMODE >= 2 && QMODE <= 4)) ? 0u : t >= nit ? iters : premixable(wp[(t - 1) & 3][r], iters);
            // two blocks per pass (blk and blk + IT), their ring reads issued together
            while (__any(blk < lim)) {
                uint32_t w[2][8];
                const uint32_t q1 = q + IT >= G::NBLK ? q + IT - G::NBLK : q + IT;
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    w[0][i] = rrow[5 * q + i];
                    w[1][i] = rrow[5 * q1 + i];
                }
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const uint32_t bk = blk + IT * u;
                    const uint32_t a = w[u][0], b = w[u][1], c = w[u][2], dd = w[u][3], e = w[u][4];
                    const bool last = bk + 1 >= iters;
                    const uint32_t an = last ? 0u : w[u][5], bn = last ? 0u : w[u][6], cn = last ? 0u : w[u][7];
                    uint32_t ec;
                    asm("v_mul_lo_u32 %0, %1, %2" : "=v"(ec) : "v"(e), "s"(FH_C1));
                    const uint32_t mc = fh_m(c), md = fh_m(dd), mbe = fh_m(b + ec);
                    constexpr uint32_t C = 0xe6546b64u;
                    const uint32_t ad = a + dd;
                    if (bk < lim) {
                        uint2 *mp = mrow + (bk & (CQ_MB - 1)) * 64;
                        *(uint4 *)mp = make_uint4(mc, 3u * C + a + ad + bn, mbe, 2u * C + ad + cn);
                        mp[2] = make_uint2(md, C + e + an);
                        if (bk == 0) {
                            xinit[r][0] = b;
                            xinit[r][1] = c;
                            xinit[r][2] = a;
                        }
                    }
                }
                const uint32_t adv = blk < lim ? (blk + IT < lim ? 2u * IT : (uint32_t)IT) : 0u;
                blk += adv;
                q += adv;
                q = q >= G::NBLK ? q - G::NBLK : q;
            }
            lds_barrier();
        }
        return;
    }

    // ------------------------------- chain: lanes (g, f, h, 0) of 16 rows -------------------------------
    __builtin_amdgcn_s_setprio(3);
    const uint32_t r = lane >> 2, role = lane & 3u;
    uint32_t id; bool is_row;
    const uint32_t *row = row_of(r, id, is_row);
    const bool valid = b0 + r < cnt;
    FH fh{0, 0, 0};
    uint32_t iters = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, iters);
    if (!ok && valid && role == 2) atomicOr(d.err, E_SHORT);
    const uint32_t sh = role == 0 ? 1u : 0u;
    uint32_t X = 0, done = 0;
    bool xset = false;
    const uint2 *mp = mring + lane;
    for (uint32_t t = 0; t < nsteps; t++) {
        const uint32_t lim = QMODE == 7 ? (t == 2 ? iters : 0u) : (t < 2 || QMODE == 1 || QMODE == 2) ? 0u : t - 1 >= nit ? iters : premixable(wp[(t - 2) & 3][r], iters);
        // the string's first words enter with block 0 (premixed, so xinit is written, one step earlier)
        if (!xset && lim > 0 && role < 3) {
            X = (role == 0 ? fh.g : role == 1 ? fh.f : fh.h) + (QMODE == 7 ? 0u : xinit[r][role]);
            xset = true;
        }
        // Groups of GB blocks at GB-aligned block numbers (a group never wraps the ring, so its reads are one base
        // address and immediate offsets, paired into ds_read2st64_b64). Before the last step only whole groups run;
        // the blocks past the last whole group wait for the next step. Groups every row has run unpredicated, two
        // buffers alternating (the next group's reads in flight during this group's arithmetic; the asm steps are
        // volatile, so the reads stay ahead of them); the rest is predicated per row. A lone wave issues one
        // instruction per four cycles at best, so the loop keeps its bookkeeping to a few scalar instructions.
        constexpr uint32_t GB = 16;
        const uint32_t limg = t - 1 >= nit ? lim : lim & ~(GB - 1);
        uint32_t nf = limg > done ? (limg - done) / GB : 0u;             // whole groups left for this row
        auto grp = [&](uint32_t base, uint2 (&v)[GB]) {
            const uint2 *gp = mp + (base & (CQ_MB - 1)) * 64;
#pragma unroll
            for (uint32_t j = 0; j < GB; j++) v[j] = gp[j * 64];
        };
        // uniform whole groups (every row has them)
        uint2 A[GB], B[GB];
        grp(done, A);
        while (__all(nf >= 1)) {
            const bool more = __all(nf >= 2);
            if (more) grp(done + GB, B);
#pragma unroll
            for (uint32_t j = 0; j < GB; j++) fh_quad_step(X, A[j].x, A[j].y, sh);
            done += GB;
            nf--;
            if (!more) break;
            const bool more2 = __all(nf >= 2);
            if (more2) grp(done + GB, A);
#pragma unroll
            for (uint32_t j = 0; j < GB; j++) fh_quad_step(X, B[j].x, B[j].y, sh);
            done += GB;
            nf--;
            if (!more2) break;
        }
        uint32_t ng = limg > done ? (limg - done + GB - 1) / GB : 0u;    // groups left, the last one partial
        while (__any(ng >= 1)) {                                   // predicated: rows ahead of the others, the tail
            grp(done, A);
#pragma unroll
            for (uint32_t j = 0; j < GB; j++) {
                uint32_t Xn = X;
                fh_quad_step(Xn, A[j].x, A[j].y, sh);
                X = ng >= 1 && done + j < limg ? Xn : X;
            }
            done = ng >= 1 ? min(done + GB, limg) : done;
            ng = ng >= 1 ? ng - 1 : 0u;
        }
        if (QMODE != 7) lds_barrier();
    }
    const uint32_t g = (uint32_t)__shfl((int)X, (int)(lane & ~3u)), f = (uint32_t)__shfl((int)X, (int)(lane & ~3u) + 1);
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(role == 2 && valid));
    if (lane == 0) ctr_add(d, C_X_CS_ROWS_N, (unsigned long long)nvalid);  // rows this launch hashed (measurement)
    if (role == 2 && valid) {
        fh.h = X; fh.g = g; fh.f = f;
        const uint32_t hv = ok ? fh.fin() : 0u;
        if (is_row) {
            d.cs[id] = hv;
            d.dirty[id] = 0;
        } else {
            d.dense_cs[id - d.NL] = hv;
        }
    }
}

template <int W, int IT, int QMODE = 0>
void launch_csq_w(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t ngrid, hipStream_t s) {
    constexpr int T = QGeo<IT>::THREADS;
    if (W == 19 && d.max_tail <= 21 && d.min_tail >= 19)
        hipLaunchKernelGGL((k_checksum_q16<W, cs_no(W, 21), (W + 19) / 4, IT, QMODE>), dim3(ngrid), dim3(T), 0, s, d, list,
                           count, d.addrw, (const uint4 *)d.rtail);
    else
        hipLaunchKernelGGL((k_checksum_q16<W, cs_no(W, 24), (W + 7) / 4, IT, QMODE>), dim3(ngrid), dim3(T), 0, s, d, list,
                           count, d.addrw, (const uint4 *)d.rtail);
}
