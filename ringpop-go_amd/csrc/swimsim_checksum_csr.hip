// swimsim_checksum_csr.hip — phase C FarmHash-32 (memberlist.go:83-128, go-farm Fingerprint32) by reference row, the
// product's kernel for launches of many nearly equal rows: "csr" (checksum by shared reference). Included by
// swimsim_checksum.hip after swimsim_checksum_ref.hip (reference row B, reference string S_B, the per-row scan).
//
// Why: a wide launch spends about half of its VALU cycles formatting each row's byte stream and premixing every
// 20-byte block (three M() = ror(x c1, 17) c2 per block, seven multiplies), and the other half on the chain itself
// (12 VALU instructions per block in carried-sum form). Outside a few "exception" blocks a row's string IS S_B
// shifted by the row's accumulated record-length difference s (swimsim_checksum_ref.hip), so the premixed values of
// every clean block are a function of (phase = -s mod 20, S_B block index) alone. Here they are computed once per
// launch for all 20 phases (k_csr_ptable: the table P, 32 B per S_B block and phase), and the chain kernel only
// streams them from LDS: per block 12 VALU instructions and two LDS reads per row.
//
//   k_csr_ptable  P[phi][k] = premix of S_B bytes [20 k + phi, 20 k + phi + 32)   {0, 0, Mg, D}, {Mf, PF, Mh, KH}
//   k_csr_plan    per workgroup of CSR_ROWS listed rows: the shift range and phases of its clean blocks -> the LDS
//                 window geometry (Wn positions per phase), or "infeasible" (the workgroup's rows fall back)
//   k_csr_rec     per row: one record per super step (CSR_SB blocks) that holds exception blocks: the super step's
//                 32 window codes (u16; an exception block's code = CSR_EXC | its ordinal in the super step), the
//                 shift after it and its first entry (k_csd_scan's entries, sorted by block)
//   k_csr         the chains. 256 rows per workgroup (4 waves, lane = row, one wave per SIMD at one workgroup per CU).
//                 Per super step the waves stage the next super step's window (every phase in use, Wn positions)
//                 from P and the rows' exception entries into the other LDS buffer while the chain of this one
//                 runs: a super step without records in a wave reads entry base(s) + i at block i (no table, no
//                 address arithmetic); otherwise each row's 32 codes come from its record or from its shift.
// Rows the path cannot take (scan flags, an infeasible window, a super step with more exception entries than a
// wave's slots) are listed and hashed by the production kernels (k_checksum3 / k_checksum_q16): bit-exact either way.

constexpr int CSR_ROWS = 256;          // rows per workgroup (4 waves)
constexpr int CSR_SB = 32;             // blocks per super step
constexpr int CSR_WINMAX = 1024;       // window entries (32 B) per buffer: phases in use x Wn
constexpr int CSR_EXW = 128;           // exception entries per wave per buffer
constexpr int CSR_ENT = CSR_WINMAX + 4 * CSR_EXW;   // entries per buffer
constexpr int CSR_TBLW = 18;           // u32 words per row of the code table (32 u16 codes + pad: b64 reads conflict-free)
constexpr int CSR_EREG = 4;            // exception entries of a record prefetched with it
constexpr uint32_t CSR_EXC = 0x8000u;  // code flag: exception entry (low bits: ordinal in the super step)
constexpr uint32_t CSR_F_PLAN = 128, CSR_F_SLOTS = 256, CSR_F_RCAP = 512;   // flags beyond k_csd_scan's

struct CsrPlan {
    int32_t cmax;          // ceil(smax / 20): window position 0 of super step t is S_B block 32 t - cmax
    uint32_t Wn;           // window positions per phase
    uint32_t phm;          // phases in use (bit phi)
    uint32_t nph;          // popcount(phm)
    uint32_t maxit;        // the workgroup's longest chain (blocks)
    uint32_t feasible;
    uint32_t pad0, pad1;
};

// one record per (row, super step with exception blocks), 80 B
struct __attribute__((aligned(16))) CsrRec {
    uint32_t t;            // super step
    int32_t s_end;         // the row's shift after the super step
    uint32_t e0, ne;       // its exception entries: ent[e0 .. e0 + ne)
    uint32_t code[16];     // 32 u16 codes, block i in the low half of code[i / 2] for even i
};

struct CsrArgs {
    const uint4 *P;        // [20][KP] x 2
    uint32_t KP;
    const uint4 *ent;      // k_csd_scan's entries [rows][ecap] x 2: {k, s_after, Mg, D}, {Mf, PF, Mh, KH}
    const CsdRow *rinfo;   // [rows]
    uint32_t ecap;
    CsrPlan *plan;         // [workgroups]
    CsrRec *rec;           // [rows][rcap]
    uint32_t *nrec;        // [rows]
    uint32_t rcap;
    uint32_t *fb_list, *fb_cnt;   // rows left to the production kernels
};

__device__ __forceinline__ int32_t csr_ceil20(int32_t x) { return x >= 0 ? (x + 19) / 20 : -((-x) / 20); }

// window code of a clean block at position i of a super step for a row at shift s (plan of its workgroup)
// (clamped into the window: a shift with no clean block after it, i.e. past the row's last exception run, is only
// ever read by predicated blocks beyond the row's chain)
__device__ __forceinline__ uint32_t csr_base(const CsrPlan &p, int32_t s) {
    const uint32_t phi = csd_phase(s);
    const uint32_t ps = (uint32_t)__popc(p.phm & ((1u << phi) - 1u));
    const int32_t c = ps * (int32_t)p.Wn + (p.cmax - csr_ceil20(s));
    return (uint32_t)min(max(c, 0), CSR_WINMAX - CSR_SB);
}

__global__ void k_csr_ptable(const uint32_t *__restrict__ SBw, uint32_t sbw_words, uint32_t KP, uint4 *__restrict__ P) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= 20u * KP) return;
    const uint32_t phi = q / KP, k = q - phi * KP;
    const uint32_t off = 20u * k + phi, wi = off >> 2, sh = off & 3u;
    uint32_t x[9];
#pragma unroll
    for (int i = 0; i < 9; i++) x[i] = wi + i < sbw_words ? SBw[wi + i] : 0u;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = __builtin_amdgcn_alignbyte(x[i + 1], x[i], sh);
    uint32_t v[6];
    csd_premix(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], v);
    P[2 * q] = make_uint4(0u, 0u, v[0], v[1]);
    P[2 * q + 1] = make_uint4(v[2], v[3], v[4], v[5]);
}

__global__ void __launch_bounds__(CSR_ROWS) k_csr_plan(DS d, const uint32_t *list, uint32_t n, CsrArgs a) {
    __shared__ int32_t sm[2];
    __shared__ uint32_t ph, mi;
    const uint32_t gi = blockIdx.x * CSR_ROWS + threadIdx.x;
    if (threadIdx.x == 0) { sm[0] = 0x7FFFFFFF; sm[1] = -0x7FFFFFFF - 1; ph = 0; mi = 0; }
    __syncthreads();
    if (gi < n) {
        const CsdRow ri = a.rinfo[gi];
        const uint32_t len = csd_len(d, list[gi]);
        if (ri.flags == 0 && len > 24) {
            atomicMin(&sm[0], ri.smin);
            atomicMax(&sm[1], ri.smax);
            atomicOr(&ph, ri.phmask);
            atomicMax(&mi, (len - 1) / 20);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        CsrPlan p{};
        int32_t smin = sm[0], smax = sm[1];
        uint32_t phm = ph;
        if (phm == 0) { phm = 1; smin = 0; smax = 0; }
        p.cmax = csr_ceil20(smax);
        p.Wn = (uint32_t)(CSR_SB + (p.cmax - csr_ceil20(smin)) + 1);
        p.phm = phm;
        p.nph = (uint32_t)__popc(phm);
        p.maxit = mi;
        p.feasible = p.nph * p.Wn <= (uint32_t)CSR_WINMAX && p.Wn < 0x7000u ? 1u : 0u;
        a.plan[blockIdx.x] = p;
    }
}

// records of one row (one thread per listed row): its exception entries grouped by super step
__global__ void k_csr_rec(DS d, const uint32_t *list, uint32_t n, CsrArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const CsdRow ri = a.rinfo[i];
    const CsrPlan p = a.plan[i / CSR_ROWS];
    uint32_t nr = 0;
    if (ri.flags == 0 && p.feasible) {
        const uint32_t len = csd_len(d, list[i]);
        const uint32_t iters = len > 24 ? (len - 1) / 20 : 0u;
        const uint4 *ent = a.ent + (size_t)i * a.ecap * 2;
        CsrRec *rec = a.rec + (size_t)i * a.rcap;
        int32_t s = 0;
        uint32_t e = 0;
        while (e < ri.ecnt) {
            const uint32_t k0 = ent[2 * e].x;
            const uint32_t t = k0 / CSR_SB, K0 = t * CSR_SB;
            if (nr == a.rcap) { nr = 0xFFFFFFFFu; break; }
            CsrRec r;
            r.t = t;
            r.e0 = e;
            uint32_t ne = 0;
            uint32_t kn = k0;                                       // block of entry e + ne
            for (uint32_t q = 0; q < (uint32_t)CSR_SB; q++) {
                const uint32_t j = K0 + q;
                uint32_t c;
                if (e + ne < ri.ecnt && kn == j) {
                    c = CSR_EXC | ne;
                    s = (int32_t)ent[2 * (e + ne)].y;
                    ne++;
                    kn = e + ne < ri.ecnt ? ent[2 * (e + ne)].x : 0xFFFFFFFFu;
                } else {
                    c = j < iters ? csr_base(p, s) + q : 0u;
                }
                if (q & 1u) r.code[q >> 1] |= c << 16;
                else r.code[q >> 1] = c;
            }
            r.s_end = s;
            r.ne = ne;
            rec[nr++] = r;
            e += ne;
        }
    }
    a.nrec[i] = nr;
}

// one block of the coupled g and f lanes and of the h lane in carried-sum form (swimsim_checksum_ref.hip)
__device__ __forceinline__ void csr_block(uint32_t &Xg, uint32_t &Xf, uint32_t &Xh, uint2 gd, uint4 fh) {
    csd_gf_step(Xg, Xf, gd.x, gd.y, fh.x, fh.y);
    csd_h_step(Xh, fh.z, fh.w);
}

template <int W>
__global__ void __launch_bounds__(CSR_ROWS) k_csr(DS d, const uint32_t *list, const uint32_t *count, CsrArgs a) {
    __shared__ uint4 E[2][CSR_ENT * 2];                 // per buffer: window entries, then each wave's exception entries
    __shared__ uint2 T[2][CSR_ROWS * CSR_TBLW / 2];     // per buffer: each row's 32 codes (tables of record super steps)
    __shared__ uint32_t phs[20];
    const uint32_t cnt = *count;
    const uint32_t g0 = blockIdx.x * CSR_ROWS;
    if (g0 >= cnt) return;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const uint32_t gi = g0 + tid;
    const bool valid = gi < cnt;
    const uint32_t id = list[valid ? gi : g0];
    const bool is_row = id < d.NL;
    const uint32_t *row = csd_row(d, id);
    const CsdRow ri = a.rinfo[valid ? gi : g0];
    const CsrPlan p = a.plan[blockIdx.x];
    const uint32_t nrec = valid ? a.nrec[gi] : 0u;
    const uint32_t len = csd_len(d, id);
    const uint32_t iters = len > 24 ? (len - 1) / 20 : 0u;
    uint32_t fl = !valid ? 0u : ri.flags ? ri.flags : !p.feasible ? CSR_F_PLAN : nrec == 0xFFFFFFFFu ? CSR_F_RCAP : 0u;
    if (valid && !fl && iters == 0) fl = CSD_F_SHORT;
    if (tid < 20 && ((p.phm >> tid) & 1u)) phs[__popc(p.phm & ((1u << tid) - 1u))] = tid;   // phase slot -> phase
    const bool live = valid && fl == 0;
    const uint32_t myit = live ? iters : 0u;
    const uint32_t T_ = p.feasible ? (p.maxit + CSR_SB - 1) / CSR_SB : 0u;
    const CsrRec *rec = a.rec + (size_t)(valid ? gi : g0) * a.rcap;
    const uint4 *ent = a.ent + (size_t)(valid ? gi : g0) * a.ecap * 2;
    const uint32_t nr = live ? nrec : 0u;

    // chain state (FarmHash-mk prologue, then X = state + the string's first words)
    FH fh{0, 0, 0};
    uint32_t it2 = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, it2);
    uint32_t Xg = fh.g + ri.b0, Xf = fh.f + ri.c0, Xh = fh.h + ri.a0;
    int32_t s = 0;
    uint32_t base = csr_base(p, 0);

    // the next record and its first exception entries, loaded one record ahead
    uint32_t rcur = 0;
    CsrRec R{};
    uint4 RE0a, RE0b, RE1a, RE1b, RE2a, RE2b, RE3a, RE3b;   // (named registers: an indexed array went to scratch)
    // (unconditional loads from clamped indices: conditionally assigned arrays would live in scratch)
    auto load_rec = [&](uint32_t q) {
        R = rec[min(q, a.rcap - 1u)];
        const uint4 *ep = ent + 2 * min(R.e0, a.ecap - (uint32_t)CSR_EREG);
        RE0a = ep[0]; RE0b = ep[1]; RE1a = ep[2]; RE1b = ep[3]; RE2a = ep[4]; RE2b = ep[5]; RE3a = ep[6]; RE3b = ep[7];
        if (q >= nr) {
            R.t = 0xFFFFFFFFu;
            R.ne = 0;
        }
    };
    load_rec(0);

    // window staging: entries u = tid + 256 v of the next super step's window, through registers
    constexpr int WV = CSR_WINMAX / CSR_ROWS;
    uint4 wst[WV][2];
    const uint32_t nwin = p.nph * p.Wn;
    auto wload = [&](uint32_t t) {
#pragma unroll
        for (int v = 0; v < WV; v++) {
            const uint32_t u = tid + (uint32_t)CSR_ROWS * v;
            wst[v][0] = make_uint4(0, 0, 0, 0);
            wst[v][1] = make_uint4(0, 0, 0, 0);
            if (u < nwin) {
                const uint32_t ps = u / p.Wn, w = u - ps * p.Wn;
                const int32_t k = (int32_t)(t * CSR_SB) - p.cmax + (int32_t)w;
                if (k >= 0 && (uint32_t)k < a.KP) {
                    const uint4 *src = a.P + 2 * ((size_t)phs[ps] * a.KP + (uint32_t)k);
                    wst[v][0] = src[0];
                    wst[v][1] = src[1];
                }
            }
        }
    };
    auto wstore = [&](uint32_t b) {
#pragma unroll
        for (int v = 0; v < WV; v++) {
            const uint32_t u = tid + (uint32_t)CSR_ROWS * v;
            if (u < nwin) {
                E[b][2 * u] = wst[v][0];
                E[b][2 * u + 1] = wst[v][1];
            }
        }
    };
    // a super step's row preparation in buffer b: a row with a record for t writes its codes (exception codes
    // rebased to the wave's slots) and its entries; the others write base + i when the wave needs tables.
    // Returns whether this wave reads tables in super step t (wave-uniform).
    auto prep = [&](uint32_t t, uint32_t b) -> bool {
        const bool has = live && R.t == t;
        const bool any = __ballot(has) != 0;
        if (!any) return false;
        uint32_t ne = has ? R.ne : 0u, tot = 0;
        const uint32_t sb = wscan_excl(ne, tot);                  // this row's first slot in the wave's area
        const uint32_t xb = (uint32_t)CSR_WINMAX + wave * CSR_EXW + sb;
        uint2 *tr = T[b] + (size_t)tid * (CSR_TBLW / 2);
        if (has && sb + ne > (uint32_t)CSR_EXW) fl |= CSR_F_SLOTS;
        if (has) {
            // codes: exception ordinals + the row's slot base, clean codes as the record has them
#pragma unroll
            for (int q = 0; q < 8; q++) {
                uint32_t c0 = R.code[2 * q], c1 = R.code[2 * q + 1];
                uint32_t lo0 = c0 & 0xFFFFu, hi0 = c0 >> 16, lo1 = c1 & 0xFFFFu, hi1 = c1 >> 16;
                lo0 = (lo0 & CSR_EXC) ? xb + (lo0 & 0x7FFFu) : lo0;
                hi0 = (hi0 & CSR_EXC) ? xb + (hi0 & 0x7FFFu) : hi0;
                lo1 = (lo1 & CSR_EXC) ? xb + (lo1 & 0x7FFFu) : lo1;
                hi1 = (hi1 & CSR_EXC) ? xb + (hi1 & 0x7FFFu) : hi1;
                tr[q] = make_uint2(lo0 | (hi0 << 16), lo1 | (hi1 << 16));
            }
            if (!(fl & CSR_F_SLOTS)) {
                uint4 *xe = E[b] + 2 * xb;
                if (ne > 0) { xe[0] = RE0a; xe[1] = RE0b; }
                if (ne > 1) { xe[2] = RE1a; xe[3] = RE1b; }
                if (ne > 2) { xe[4] = RE2a; xe[5] = RE2b; }
                if (ne > 3) { xe[6] = RE3a; xe[7] = RE3b; }
                for (uint32_t k = CSR_EREG; k < ne; k++) {          // more than CSR_EREG: synchronous loads (rare)
                    E[b][2 * (xb + k)] = ent[2 * (R.e0 + k)];
                    E[b][2 * (xb + k) + 1] = ent[2 * (R.e0 + k) + 1];
                }
            }
            s = R.s_end;
        } else {
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint32_t c = base + 4u * q;
                tr[q] = make_uint2(c | ((c + 1u) << 16), (c + 2u) | ((c + 3u) << 16));
            }
        }
        return true;
    };

    // super step 0
    wload(0);
    wstore(0);
    bool tab = prep(0, 0);
    if (live && R.t == 0) { base = csr_base(p, s); rcur++; load_rec(rcur); }
    __syncthreads();
    for (uint32_t t = 0; t < T_; t++) {
        const uint32_t b = t & 1u, K0 = t * CSR_SB;
        if (t + 1 < T_) wload(t + 1);
        // ---- the chain over blocks K0 .. K0 + 31 ----
        const bool full = __all(myit == 0u || K0 + CSR_SB <= myit);
        const uint4 *EB = E[b];
        auto step = [&](uint32_t i, uint32_t c) {
            const uint4 *q = EB + 2 * c;
            const uint4 x = q[0], y = q[1];
            if (full) {
                csr_block(Xg, Xf, Xh, make_uint2(x.z, x.w), y);
            } else {
                uint32_t ng = Xg, nf = Xf, nh = Xh;
                csr_block(ng, nf, nh, make_uint2(x.z, x.w), y);
                const bool act = K0 + i < myit;
                Xg = act ? ng : Xg;
                Xf = act ? nf : Xf;
                Xh = act ? nh : Xh;
            }
        };
        if (!tab) {
#pragma unroll
            for (uint32_t i = 0; i < (uint32_t)CSR_SB; i++) step(i, base + i);
        } else {
            const uint2 *tr = T[b] + (size_t)tid * (CSR_TBLW / 2);
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint2 cc = tr[q];
                step(4 * q + 0, cc.x & 0xFFFFu);
                step(4 * q + 1, cc.x >> 16);
                step(4 * q + 2, cc.y & 0xFFFFu);
                step(4 * q + 3, cc.y >> 16);
            }
        }
        // ---- the next super step's window, rows and entries into the other buffer ----
        if (t + 1 < T_) {
            wstore(b ^ 1u);
            tab = prep(t + 1, b ^ 1u);
            if (live && R.t == t + 1) { base = csr_base(p, s); rcur++; load_rec(rcur); }
        }
        __syncthreads();
    }
    const bool mine = valid && fl == 0;
    const uint32_t nmine = (uint32_t)__popcll(__ballot(mine));
    if (lane == 0 && nmine) ctr_add(d, C_X_CS_ROWS, (unsigned long long)nmine);   // rows this launch hashed
    if (!valid) return;
    if (!mine) {                                                    // left to the production kernels
        const uint32_t at = atomicAdd(a.fb_cnt, 1u);
        a.fb_list[at] = id;
        return;
    }
    fh.h = Xh; fh.g = Xg; fh.f = Xf;
    const uint32_t hv = ok ? fh.fin() : 0u;
    if (is_row) {
        d.cs[id] = hv;
        d.dirty[id] = 0;
    } else {
        d.dense_cs[id - d.NL] = hv;
    }
}

// launches of the path (part): 0 S_B string, 1 P table, 2 scan, 3 plan + records, 4 the chains
template <int W>
void launch_csr_w(const DS &d, const uint32_t *list, uint32_t n, const uint32_t *count, const CsdArgs &ca, const CsrArgs &a,
                  hipStream_t s, int part) {
    if (part == 0) {
        hipLaunchKernelGGL((k_csd_string<W>), dim3((d.N + 255) / 256), dim3(256), 0, s, d, ca.B, ca.OB, (uint8_t *)ca.SBw);
    } else if (part == 1) {
        hipLaunchKernelGGL(k_csr_ptable, dim3((20u * a.KP + 255) / 256), dim3(256), 0, s, ca.SBw, ca.sbw_words, a.KP,
                           (uint4 *)a.P);
    } else if (part == 2) {
        hipLaunchKernelGGL((k_csd_scan<W>), dim3((n + 3) / 4), dim3(256), 0, s, d, list, n, ca);
    } else if (part == 3) {
        hipLaunchKernelGGL(k_csr_plan, dim3((n + CSR_ROWS - 1) / CSR_ROWS), dim3(CSR_ROWS), 0, s, d, list, n, a);
        hipLaunchKernelGGL(k_csr_rec, dim3((n + 255) / 256), dim3(256), 0, s, d, list, n, a);
    } else {
        hipLaunchKernelGGL((k_csr<W>), dim3((n + CSR_ROWS - 1) / CSR_ROWS), dim3(CSR_ROWS), 0, s, d, list, count, a);
    }
}

void launch_csr(const DS &d, const uint32_t *list, uint32_t n, const uint32_t *count, const CsdArgs &ca, const CsrArgs &a,
                hipStream_t s, int part) {
    switch (d.W) {
#define CS_CASE(Wv) case Wv: launch_csr_w<Wv>(d, list, n, count, ca, a, s, part); break;
        CS_W_CASES(CS_CASE)
#undef CS_CASE
    default: break;
    }
}
