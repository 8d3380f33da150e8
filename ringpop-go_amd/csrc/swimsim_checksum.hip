// swimsim_checksum.hip — phase C: the membership checksum (memberlist.go:83-128), i.e. go-farm
// Fingerprint32 = FarmHash-32 "mk" over addr ‖ status ‖ decimal(inc) ‖ ';' of every non-tombstone
// member in index order. Fixed-width ascending addresses make the sorted order the index order, so
// the string is generated on the fly and never sorted. Included by swimsim_kernels.hip.
//
// The FarmHash chain is sequential within a row: one lane carries one row's chain, and the length
// of that chain (≈1.9 blocks of 20 bytes per member) sets the latency of a launch. One workgroup
// takes 64 rows (lane l = row l in every wave) and runs three roles:
//   wave 2 (formatter): writes each row's byte stream as 32-bit words into a per-row LDS ring, CS_IT
//                       members per step. A record is assembled from the member's address words
//                       (wave-uniform loads) and a pre-shifted record tail fetched from the tail table
//                       one step ahead (global, L2-resident: few incarnations are live at a time), and
//                       written with v_perm byte alignment against the carried partial word;
//   wave 0 (h chain)  : the h lane of every complete 20-byte block of the previous steps;
//   wave 1 (g/f chain): the coupled g and f lanes of the same blocks.
// One workgroup barrier per step; the hashers trail the formatter by one step. The ring holds the
// hashers' unread step, the step being written and the record spill, so every workgroup fits four
// to a CU (36 KB of LDS) and a 65,536-row launch is resident at once.
// The string length and the last included member (the FarmHash-mk prologue hashes the last 20
// bytes before the chain) come from per-row values kept current by the merges.

#include <type_traits>

constexpr int CS_ROWS = 64;                     // rows per workgroup: one lane per row in each wave
constexpr int CS_IT = 4;                        // members formatted per pipeline step
constexpr int CS_SUP = 16;                      // members per register prefetch of the row (4 steps)
constexpr int CS_RING = 110;                    // ring words per row: whole 20-byte blocks, so a block
                                                // never straddles the ring end (the hashers wrap per block)
constexpr int CS_PRE = 12, CS_POST = 12;        // write spill areas in front of / behind the ring
constexpr int CS_PHYS = CS_PRE + CS_RING + CS_POST;
constexpr int CS_SINK = CS_PHYS;                // write sink (skipped records, words past a record's end)
constexpr int CS_LDSW = CS_PHYS + 12;           // ring + spill areas + sink, in words per row
constexpr int CS_RW = 11;                       // record words of the prologue record (<= 44 bytes)

template <int W, int RW>
__device__ __forceinline__ void build_rec(uint32_t (&R)[RW], const uint32_t *A, const uint32_t (&T)[6]) {
    constexpr int wW = W / 4, bW = W % 4;
#pragma unroll
    for (int i = 0; i < RW; i++) {
        uint32_t v;
        if (i < wW) {
            v = A[i];
        } else if (bW == 0) {
            const int k = i - wW;
            v = k < 6 ? T[k] : 0u;
        } else if (i == wW) {
            v = (A[wW] & ((1u << (8 * bW)) - 1u)) | (T[0] << (8 * bW));
        } else {
            const int k = i - wW - 1;
            const uint32_t lo = k < 6 ? (T[k] >> (32 - 8 * bW)) : 0u;
            const uint32_t hi = (k + 1) < 6 ? (T[k + 1] << (8 * bW)) : 0u;
            v = lo | hi;
        }
        R[i] = v;
    }
}

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh_bits) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh_bits);
}

// record words of member m (member word w), from the unshifted tail table; returns the record length
template <int W>
__device__ __forceinline__ uint32_t record(const DS &d, uint32_t m, uint32_t w, uint32_t (&R)[CS_RW]) {
    const uint32_t st = w & 7u, e = min(w >> 3, d.ecap - 1);
    const uint32_t *tp = d.tailw + ((size_t)e * 4 + (st & 3u)) * 8;
    const uint4 ta = *(const uint4 *)tp;
    const uint4 tb = *(const uint4 *)(tp + 4);
    const uint32_t T[6] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y};
    build_rec<W, CS_RW>(R, d.addrw + (size_t)m * 6, T);
    return (st < 4u && m < d.N) ? W + tb.z : 0u;
}

// Workgroup barrier that orders LDS only. __syncthreads() also fences global memory, which makes
// every wave drain its outstanding global loads (the formatters' one-step-ahead prefetch) first.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// M(x) = mur's data-only half: ror(x * c1, 17) * c2. mur(x, h) = ror(h ^ M(x), 19) * 5 + 0xe6546b64.
__device__ __forceinline__ uint32_t fh_m(uint32_t x) { return ror32(x * FH_C1, 17) * FH_C2; }
__device__ __forceinline__ uint32_t x5(uint32_t h) {          // h * 5 as one full-rate v_lshl_add_u32
    uint32_t r;                                              // (LLVM would re-fold a C shift-add into a
    asm("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(r) : "v"(h)); //  quarter-rate multiply)
    return r;
}
// mur(x, h) + add with M(x) precomputed: ror(h ^ M(x), 19) * 5 + 0xe6546b64 + add
__device__ __forceinline__ uint32_t fh_fold(uint32_t h, uint32_t mx, uint32_t add) {
    return x5(ror32(h ^ mx, 19)) + 0xe6546b64u + add;
}

// FarmHash-mk state after the len > 24 prologue (the last 20 bytes of the string, i.e. of the last
// included member's record) and the number of 20-byte chain blocks. false: string too short / empty.
template <int W>
__device__ __forceinline__ bool cs_prologue(const DS &d, uint32_t id, bool is_row, const uint32_t *row, FH &fh,
                                            uint32_t &iters) {
    const uint32_t N = d.N;
    const uint32_t len = is_row ? d.clen[id] : d.dense_len[id - d.NL];
    int32_t last = is_row ? d.clast[id] : d.dense_last[id - d.NL];
    if (last < 0) {                                                // invalidated: rescan from the end
        last = -1;
        for (int32_t m = (int32_t)N - 1; m >= 0; m--)
            if ((row[m] & 7u) < 4u) { last = m; break; }
    }
    const bool ok = len > 24 && last >= 0;
    uint32_t R[CS_RW];
    const uint32_t L = record<W>(d, (uint32_t)max(last, 0), row[max(last, 0)], R);
    const uint32_t q = L >= 20 ? L - 20 : 0, qw = q >> 2, qb = (q & 3u) * 8u;
    uint32_t t[5];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int s = 0; s < CS_RW; s++) {
            lo = ((uint32_t)s == qw + k) ? R[s] : lo;
            hi = ((uint32_t)s == qw + k + 1) ? R[s] : hi;
        }
        t[k] = funnel(hi, lo, qb);
    }
    fh.init(len, t[0], t[1], t[2], t[3], t[4]);
    iters = ok ? (len - 1) / 20 : 0;
    return ok;
}

// NO = ring words one record can touch (record of at most W + max tail bytes, shifted by <= 3).
// Waves: 0 h chain, 1 g/f chain, 2 and 3 formatters.
// MODE 0: normal; 1: hashers only (formatter skips its stores); 2: formatter only; 3: the g/f wave
// also dumps every block it hashes to dbg (lane 0's row; diagnostics); 4: barrier skeleton (no
// loads, no hashing); 5: formatter loads and positions only. Modes 1, 2, 4, 5 time parts of the kernel.
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

// NO for the address width W and the longest record tail of the handle's incarnation table
constexpr int cs_no(int W, int maxtail) { return (3 + W + maxtail + 3) / 4; }

template <int W, int MODE>
void launch_cs_w(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t grid, hipStream_t s,
                 uint32_t *dbg = nullptr, uint32_t cap = 0) {
    // the common case: 13-digit incarnations (t0 = 1.5e12 ms): tails of 19..21 bytes
    if (W == 19 && d.max_tail <= 21 && d.min_tail >= 19)
        hipLaunchKernelGGL((k_checksum<W, cs_no(W, 21), (W + 19) / 4, MODE>), dim3(grid), dim3(256), 0, s, d, list, count,
                           d.addrw, (const uint4 *)d.rtail, dbg, cap);
    else  // any tail of 7 ("alive" + 1 digit + ';') to 24 bytes
        hipLaunchKernelGGL((k_checksum<W, cs_no(W, 24), (W + 7) / 4, MODE>), dim3(grid), dim3(256), 0, s, d, list, count,
                           d.addrw, (const uint4 *)d.rtail, dbg, cap);
}

void launch_checksum(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t maxn, hipStream_t s) {
    const uint32_t grid = (maxn + CS_ROWS - 1) / CS_ROWS;
    if (grid == 0) return;
    switch (d.W) {
#define CS_CASE(Wv) case Wv: launch_cs_w<Wv, 0>(d, list, count, grid, s); break;
        CS_CASE(13) CS_CASE(14) CS_CASE(15) CS_CASE(16) CS_CASE(17) CS_CASE(18) CS_CASE(19) CS_CASE(20)
#undef CS_CASE
    default: break;
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
    if (mode == 1) launch_cs_w<19, 1>(d, list, count, grid, s);
    else if (mode == 2) launch_cs_w<19, 2>(d, list, count, grid, s);
    else if (mode == 4) launch_cs_w<19, 4>(d, list, count, grid, s);
    else if (mode == 5) launch_cs_w<19, 5>(d, list, count, grid, s);
    else launch_cs_w<19, 0>(d, list, count, grid, s);
}
