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
// streams them from LDS: per block 12 VALU instructions and three LDS reads per row, no address arithmetic.
//
//   k_csr_ptable  P[phi][k] = premix of S_B bytes [20 k + phi, 20 k + phi + 32)   {Mg, D, Mf, PF}, {Mh, KH, 0, 0}
//   k_csr_plan    per workgroup of CSR_ROWS listed rows: the shift range and phases of its clean blocks -> the LDS
//                 window geometry (Wn positions per phase), or "infeasible" (the workgroup's rows fall back)
//   k_csr_rec     per row: one record per super step (CSR_SB blocks) that holds exception blocks: the super step's
//                 32 codes (u16: a clean block's window entry as an LDS byte address, CSR_EXC | ordinal for an
//                 exception block), the shift after it and where its first exceptions are
//   k_csr         the chains. 256 rows per workgroup (4 waves, lane = row, one wave per SIMD at one workgroup per CU).
//                 Per super step the waves stage the next super step's window (every phase in use, Wn positions)
//                 from P and the rows' exception entries into the other LDS buffer while the chain of this one
//                 runs. Each row reads its 32 blocks' entries at the byte addresses in its own LDS table, which its
//                 lane rewrites only when the codes change: from a record (exception codes patched to the wave's
//                 slots), and back to base(s) + i in the super step after one.
// Rows the path cannot take (scan flags, an infeasible window, a super step with more exception entries than a
// wave's slots) are listed and hashed by the production kernels (k_checksum3 / k_checksum_q16): bit-exact either way.

constexpr int CSR_ROWS = 256;          // rows per workgroup (4 waves)
constexpr int CSR_SB = 32;             // blocks per super step
constexpr int CSR_WINMAX = 1024;       // window entries per buffer: phases in use x Wn
constexpr int CSR_EXW = 384;           // exception entries per wave per buffer (128: a third of the rows of heavy cascade
                                       // rounds fell back, a differing column giving every row of a wave exceptions;
                                       // 192: still an eighth in the heaviest)
constexpr int CSR_ENT = CSR_WINMAX + 4 * CSR_EXW;   // entries per buffer
constexpr int CSR_TW = 36;             // u32 words per row of the code table (32 codes + pad: ds_read_b128 conflict-free)
constexpr uint32_t CSR_ESZ = 16;       // a code's unit: an entry's byte offset in each of the two entry arrays
constexpr int CSR_EREG = 4;            // exception entries of a record prefetched with it
#ifndef CSR_PF_DEF
#define CSR_PF_DEF 6
#endif
constexpr int CSR_PF = CSR_PF_DEF;     // blocks the chain's LDS reads run ahead of its arithmetic (6: 7.37 / 11.52 ms
                                       // on rounds 14 / 18 against 7.48 / 11.69 with 4 and 8.00 / 12.00 with 2)
constexpr uint32_t CSR_EXC = 0x8000u;  // code flag: exception entry (low bits: ordinal in the super step)
constexpr uint32_t CSR_F_PLAN = 128, CSR_F_SLOTS = 256, CSR_F_RCAP = 512;   // flags beyond k_csd_scan's

struct CsrPlan {
    int32_t cmax;          // ceil(smax / 20): window position 0 of super step t is S_B block 32 t - cmax
    uint32_t Wn;           // window positions per phase
    uint32_t phm;          // phases in use (bit phi)
    uint32_t nph;          // popcount(phm)
    uint32_t maxit;        // the workgroup's longest chain (blocks)
    uint32_t feasible;
    uint32_t ecmax;        // rows with more exception entries than this are not in the plan (production kernels)
    uint32_t pad1;
};

// one record per (row, super step with exception blocks), 80 B
struct __attribute__((aligned(16))) CsrRec {
    uint32_t t;            // super step
    int32_t s_end;         // the row's shift after the super step
    uint32_t pos4, ne;     // the blocks (bytes 0-3) of its first exception entries (ne <= 4), their number
    uint32_t code[16];     // 32 u16 codes, block i in the low half of code[i / 2] for even i: the byte address of a
                           // clean block's window entry, CSR_EXC | ordinal for an exception block
};

struct CsrArgs {
    const uint4 *P;        // [20][KP] x 2
    uint32_t KP;
    const uint4 *ent;      // k_csd_scan's entries [rows][ecap] x 2: {Mg, D, Mf, PF}, {Mh, KH, k, s_after}
    const CsdRow *rinfo;   // [rows]
    uint32_t ecap;
    CsrPlan *plan;         // [workgroups]
    CsrRec *rec;           // [rows][rcap]
    uint32_t *nrec;        // [rows]
    uint32_t rcap;
    uint32_t *fb_list, *fb_cnt;   // rows left to the production kernels
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

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
    P[2 * q] = make_uint4(v[0], v[1], v[2], v[3]);
    P[2 * q + 1] = make_uint4(v[4], v[5], 0u, 0u);
}

// (a workgroup whose window would not fit plans again without its far rows, those with more than CSR_NEAR exception
// entries: many differences from the reference bring many shifts and phases, and one such row used to send all 256 rows
// of its workgroup to the production kernels; the far rows alone go there now)
constexpr uint32_t CSR_NEAR = 1024;
__global__ void __launch_bounds__(CSR_ROWS) k_csr_plan(DS d, const uint32_t *list, uint32_t n, CsrArgs a) {
    __shared__ int32_t sm[2][2];
    __shared__ uint32_t ph[2], mi[2];
    const uint32_t gi = blockIdx.x * CSR_ROWS + threadIdx.x;
    if (threadIdx.x < 2) { sm[threadIdx.x][0] = 0x7FFFFFFF; sm[threadIdx.x][1] = -0x7FFFFFFF - 1; ph[threadIdx.x] = 0; mi[threadIdx.x] = 0; }
    __syncthreads();
    if (gi < n) {
        const CsdRow ri = a.rinfo[gi];
        const uint32_t len = csd_len(d, list[gi]);
        if (ri.flags == 0 && len > 24) {
            for (int k = 0; k < 2; k++) {                          // 0: every row, 1: the near rows
                if (k == 1 && ri.ecnt > CSR_NEAR) break;
                atomicMin(&sm[k][0], ri.smin);
                atomicMax(&sm[k][1], ri.smax);
                atomicOr(&ph[k], ri.phmask);
                atomicMax(&mi[k], (len - 1) / 20);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        CsrPlan p{};
        for (int k = 0; k < 2; k++) {
            int32_t smin = sm[k][0], smax = sm[k][1];
            uint32_t phm = ph[k];
            if (phm == 0) { phm = 1; smin = 0; smax = 0; }
            p.cmax = csr_ceil20(smax);
            p.Wn = ((uint32_t)(CSR_SB + (p.cmax - csr_ceil20(smin)) + 1) + 30u) / 32u * 32u + 1u;   // = 1 mod 32 (k_csr)
            p.phm = phm;
            p.nph = (uint32_t)__popc(phm);
            p.maxit = mi[k];
            p.feasible = p.nph * p.Wn <= (uint32_t)CSR_WINMAX && p.Wn < 0x7000u ? 1u : 0u;
            p.ecmax = k == 0 ? 0xFFFFFFFFu : CSR_NEAR;
            if (p.feasible) break;
        }
        a.plan[blockIdx.x] = p;
    }
}

// records of one row per wave (4 rows per workgroup): the row's entries in chunks of 64 (lane q holds entry c0 + q's
// block and shift, staged in LDS), and every lane that begins a super step's group of entries builds that group's
// record. A group that runs past the chunk's end is left to the next chunk, which starts at its first entry (a group
// holds at most CSR_SB entries, so every chunk completes at least one group).
__global__ void __launch_bounds__(256) k_csr_rec(DS d, const uint32_t *list, uint32_t n, CsrArgs a) {
    __shared__ uint2 hd[4][64];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t i = blockIdx.x * 4 + wv;
    if (i >= n) return;
    const CsdRow ri = a.rinfo[i];
    const CsrPlan p = a.plan[i / CSR_ROWS];
    uint32_t nr = 0;
    if (ri.flags == 0 && p.feasible && ri.ecnt <= p.ecmax) {
        const uint32_t len = csd_len(d, list[i]);
        const uint32_t iters = len > 24 ? (len - 1) / 20 : 0u;
        const uint4 *ent = a.ent + (size_t)i * a.ecap * 2;
        CsrRec *rec = a.rec + (size_t)i * a.rcap;
        int32_t s_prev = 0;                                          // the shift before entry c0
        uint32_t c0 = 0;
        while (c0 < ri.ecnt) {
            const uint32_t nin = min(64u, ri.ecnt - c0);
            const bool in = lane < nin;
            const uint2 h = in ? ((const uint2 *)(ent + 2 * (c0 + lane) + 1))[1] : make_uint2(0xFFFFFFFFu, 0u);   // {k, s after}
            hd[wv][lane] = h;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t t = h.x / CSR_SB;
            const bool head = in && (lane == 0 || hd[wv][lane - 1].x / CSR_SB != t);
            const uint64_t heads = __ballot(head);
            const uint64_t after = lane < 63 ? heads & ~((2ull << lane) - 1ull) : 0ull;
            const uint32_t gend = after ? (uint32_t)__builtin_ctzll(after) : nin;   // one past the group's last entry
            const bool complete = after != 0 || c0 + nin == ri.ecnt;
            const bool build = head && complete;
            const uint64_t built = __ballot(build);
            if (build) {
                const uint32_t slot = nr + (uint32_t)__popcll(built & ((1ull << lane) - 1ull));
                if (slot < a.rcap) {
                    CsrRec r;
                    int32_t s = lane ? (int32_t)hd[wv][lane - 1].y : s_prev;
                    const uint32_t K0 = t * CSR_SB;
                    uint32_t q = lane, kn = h.x, pos = 0;
                    for (uint32_t b = 0; b < (uint32_t)CSR_SB; b++) {
                        const uint32_t j = K0 + b;
                        uint32_t c;
                        if (q < gend && kn == j) {
                            const uint32_t o = q - lane;
                            c = CSR_EXC | o;
                            if (o < 4) pos |= b << (8 * o);
                            s = (int32_t)hd[wv][q].y;
                            q++;
                            kn = q < gend ? hd[wv][q].x : 0xFFFFFFFFu;
                        } else {
                            c = j < iters ? (csr_base(p, s) + b) * CSR_ESZ : 0u;
                        }
                        if (b & 1u) r.code[b >> 1] |= c << 16;
                        else r.code[b >> 1] = c;
                    }
                    r.t = t;
                    r.s_end = s;
                    r.pos4 = pos;
                    r.ne = gend - lane;
                    rec[slot] = r;
                }
            }
            nr += (uint32_t)__popcll(built);
            // the next chunk begins at the first group left incomplete
            const uint64_t open = heads & ~built;
            const uint32_t adv = open ? (uint32_t)__builtin_ctzll(open) : nin;
            s_prev = adv ? (int32_t)hd[wv][adv - 1].y : s_prev;
            c0 += adv;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (nr > a.rcap) nr = 0xFFFFFFFFu;
    }
    if (lane == 0) a.nrec[i] = nr;
}

template <int W>
__global__ void __launch_bounds__(CSR_ROWS) k_csr(DS d, const uint32_t *list, const uint32_t *count, CsrArgs a) {
    // per buffer: window entries, then each wave's exception entries, in two arrays of 16-B entries, EA {Mg, D, Mf, PF}
    // and EB {Mh, KH, -, -}: a block is two ds_read_b128 at one byte address (the row's code, 16 e) plus each array's
    // base as the immediate offset. ds_read_b128 runs at the LDS array's full rate with one wave per SIMD; 8-byte
    // reads do not (three ds_read_b64 per block of 24-B entries: 10.3 ms per launch against 8.5 for one b64 + one b128).
    // Two rows of a 16-lane group conflict when their entries are 16 apart; with Wn = 1 mod 32 the phases' windows
    // start at different residues.
    // (EB holds both buffers in each 16-B entry, buffer b in bytes 8b..8b+7: a ds_read_b128 of the whole entry and
    // the compile-time buffer's half, with 16 KB more for exception slots)
    __shared__ uint4 EA[2][CSR_ENT];
    __shared__ uint4 EB[CSR_ENT];
    // per row: the byte addresses of its 32 blocks' entries in the super step (one table, not one per buffer: a row's
    // table is read and written only by its own lane, and rewritten only when its codes change)
    __shared__ uint32_t T[CSR_ROWS * CSR_TW];
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
    uint32_t fl = !valid ? 0u : ri.flags ? ri.flags : !p.feasible || ri.ecnt > p.ecmax ? CSR_F_PLAN
                : nrec == 0xFFFFFFFFu ? CSR_F_RCAP : 0u;
    if (valid && !fl && iters == 0) fl = CSD_F_SHORT;
    if (tid < 20 && ((p.phm >> tid) & 1u)) phs[__popc(p.phm & ((1u << tid) - 1u))] = tid;   // phase slot -> phase
    __syncthreads();
    const bool live = valid && fl == 0;
    const uint32_t myit = live ? iters : 0u;
    const uint32_t T_ = p.feasible ? (p.maxit + CSR_SB - 1) / CSR_SB : 0u;
    const CsrRec *rec = a.rec + (size_t)(valid ? gi : g0) * a.rcap;
    const uint4 *ent = a.ent + (size_t)(valid ? gi : g0) * a.ecap * 2;
    const uint32_t nr = live ? nrec : 0u;
    uint32_t *trow = T + (size_t)tid * CSR_TW;

    // chain state (FarmHash-mk prologue, then X = state + the string's first words)
    FH fh{0, 0, 0};
    uint32_t it2 = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, it2);
    uint32_t Xg = fh.g + ri.b0, Xf = fh.f + ri.c0, Xh = fh.h + ri.a0;
    int32_t s = 0;
    uint32_t base = csr_base(p, 0);

    // the next record and its first exception entries, loaded one record ahead
    // (records partition the row's entries in order: record q + 1 begins where record q ends, so the entry loads never
    // wait for the record itself; nothing here selects on a loaded value, which would wait for the load at once)
    // (record and entries are held as whole vector registers, each loaded by one instruction into exactly the
    // registers it lives in: loaded structs split into scalars came out as copies after the loads, each waiting for them)
    uint32_t rcur = 0, ecur = 0;
    bool rv = false;
    u32x4 R0, R1, R2, R3, R4;                                    // CsrRec: {t, s_end, pos4, ne}, code[0..15]
    u32x4 RE0a, RE1a, RE2a, RE3a;                                // entry values {Mg, D, Mf, PF}
    u32x2 RE0b, RE1b, RE2b, RE3b;                                // {Mh, KH}
    // (unconditional loads from clamped indices: conditionally assigned arrays would live in scratch)
    auto load_rec = [&](uint32_t q, uint32_t e0) {
        const u32x4 *rp = (const u32x4 *)(rec + min(q, a.rcap - 1u));
        R0 = rp[0]; R1 = rp[1]; R2 = rp[2]; R3 = rp[3]; R4 = rp[4];
        const u32x4 *ep = (const u32x4 *)(ent + 2 * min(e0, a.ecap - (uint32_t)CSR_EREG));
        RE0a = ep[0]; RE0b = *(const u32x2 *)(ep + 1);
        RE1a = ep[2]; RE1b = *(const u32x2 *)(ep + 3);
        RE2a = ep[4]; RE2b = *(const u32x2 *)(ep + 5);
        RE3a = ep[6]; RE3b = *(const u32x2 *)(ep + 7);
        rv = q < nr;
    };
    load_rec(0, 0);
#ifdef CSR_DIAG_STAMP
    // (diagnostic build only: shader-clock stamps around the loop's sections, summed per wave into the diagnostic
    // counters: 0 chain, 1 staging + preparation, 2 barrier, 3 whole loop; shares only, the stamps drain LDS waits)
    uint64_t st_[4] = {0, 0, 0, 0};
    auto stamp = [&]() -> uint64_t {
        uint64_t tt;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tt) :: "memory");
        __builtin_amdgcn_sched_barrier(0);
        return tt;
    };
#define CSR_STAMP(v) const uint64_t v = stamp()
#define CSR_ACC(k, x) st_[k] += (x)
#else
#define CSR_STAMP(v)
#define CSR_ACC(k, x)
#endif

    // window staging: entries u = tid + 256 v of the next super step's window, through registers
    constexpr int WV = CSR_WINMAX / CSR_ROWS;
    // two staging sets: super step u's window goes through set u & 1, loaded two super steps ahead (the window rows of
    // P miss in L2 at their first touch: one HBM round trip, longer than a super step's chain)
    // (vector types: a struct copy of a uint4 is a memcpy, and the compiler promoted the staging arrays to LDS)
    u32x4 wA0[WV], wB0[WV];
    u32x2 wA1[WV], wB1[WV];
    const uint32_t nwin = p.nph * p.Wn;
    // (each thread's window entries keep their phase and position from super step to super step: their source rows
    // in P are fixed, the S_B block advances by CSR_SB)
    const uint4 *wsrc[WV];
    int32_t wk0[WV];
#pragma unroll
    for (int v = 0; v < WV; v++) {
        const uint32_t u = tid + (uint32_t)CSR_ROWS * v;
        const uint32_t ps = u < nwin ? u / p.Wn : 0u, w = u < nwin ? u - ps * p.Wn : 0u;
        wsrc[v] = a.P + 2 * (size_t)phs[min(ps, 19u)] * a.KP;
        wk0[v] = u < nwin ? (int32_t)w - p.cmax : 0x40000000;
    }
    auto wload = [&](u32x4 (&wst0)[WV], u32x2 (&wst1)[WV], uint32_t t) {
#pragma unroll
        for (int v = 0; v < WV; v++) {
            // (positions outside S_B are read only by predicated blocks past a row's chain: any value does; a select on
            // the loaded value would wait for this load here, one HBM round trip per super step)
            const int32_t k = min(max(wk0[v] + (int32_t)(t * CSR_SB), 0), (int32_t)a.KP - 1);
            const uint4 *src = wsrc[v] + 2 * (uint32_t)k;
            wst0[v] = *(const u32x4 *)src;
            wst1[v] = *(const u32x2 *)(src + 1);
        }
    };
    auto put_entry = [&](uint32_t b, uint32_t e, uint2 x, uint2 y, uint2 z) {
        EA[b][e] = make_uint4(x.x, x.y, y.x, y.y);
        ((uint2 *)&EB[e])[b] = z;
    };
    auto wstore = [&](const u32x4 (&wst0)[WV], const u32x2 (&wst1)[WV], uint32_t b) {
#pragma unroll
        for (int v = 0; v < WV; v++) {
            // (every thread stores all its entries, those past the window into unused window slots: a store on some
            // paths only left its loads pending on the others, and the loop head waited for them)
            const uint32_t u = tid + (uint32_t)CSR_ROWS * v;
            put_entry(b, u, make_uint2(wst0[v].x, wst0[v].y), make_uint2(wst0[v].z, wst0[v].w),
                      make_uint2(wst1[v].x, wst1[v].y));
        }
    };
    // the chain's codes for the super step, per lane in registers: base(s) + i for a row without exception blocks
    // (set in registers when the row's shift changes), a record's codes (through the row's LDS table row, where the
    // exception codes are patched to the wave's slots) otherwise
    uint32_t code[CSR_SB];
    auto set_base = [&]() {
        const uint32_t ba = base * CSR_ESZ;
#pragma unroll
        for (int i = 0; i < CSR_SB; i++) code[i] = ba + (uint32_t)i * CSR_ESZ;
    };
    // (a row that is not hashed reads entry 0)
    if (live) set_base();
    else {
#pragma unroll
        for (int i = 0; i < CSR_SB; i++) code[i] = 0u;
    }
    bool was = false;                                              // the row's codes are a record's
    // a super step's row preparation in buffer b: a row with a record for t writes its codes and its exception
    // entries (exception codes patched to the wave's slots); a row whose last super step had a record writes base + i
    auto prep = [&](uint32_t t, uint32_t b) {
        const bool has = live && rv && R0.x == t;
        if (__ballot(has)) {
            uint32_t ne = has ? R0.w : 0u, tot = 0;
            const uint32_t sb = wscan_excl(ne, tot);              // this row's first slot in the wave's area
            const uint32_t xb = (uint32_t)CSR_WINMAX + wave * CSR_EXW + sb;
            if (has && sb + ne > (uint32_t)CSR_EXW) fl |= CSR_F_SLOTS;
            if (has) {
#pragma unroll
                for (int q = 0; q < 4; q++) {                      // the record's 32 u16 codes
                    const u32x4 Rq = q == 0 ? R1 : q == 1 ? R2 : q == 2 ? R3 : R4;
                    *(u32x4 *)(trow + 8 * q) = u32x4{Rq.x & 0xFFFFu, Rq.x >> 16, Rq.y & 0xFFFFu, Rq.y >> 16};
                    *(u32x4 *)(trow + 8 * q + 4) = u32x4{Rq.z & 0xFFFFu, Rq.z >> 16, Rq.w & 0xFFFFu, Rq.w >> 16};
                }
                const uint32_t xa = xb * CSR_ESZ;
                if (ne <= (uint32_t)CSR_EREG) {                    // exception codes: positions from the record
                    const uint32_t pos = R0.z;
                    if (ne > 0) trow[pos & 31u] = xa;
                    if (ne > 1) trow[(pos >> 8) & 31u] = xa + CSR_ESZ;
                    if (ne > 2) trow[(pos >> 16) & 31u] = xa + 2u * CSR_ESZ;
                    if (ne > 3) trow[(pos >> 24) & 31u] = xa + 3u * CSR_ESZ;
                } else {                                           // (rare) from the codes' flags
                    for (int q = 0; q < CSR_SB; q++) {
                        const uint32_t c = trow[q];
                        if (c & CSR_EXC) trow[q] = xa + (c & 0x7FFFu) * CSR_ESZ;
                    }
                }
                if (!(fl & CSR_F_SLOTS)) {
                    if (ne > 0) put_entry(b, xb + 0, make_uint2(RE0a.x, RE0a.y), make_uint2(RE0a.z, RE0a.w), make_uint2(RE0b.x, RE0b.y));
                    if (ne > 1) put_entry(b, xb + 1, make_uint2(RE1a.x, RE1a.y), make_uint2(RE1a.z, RE1a.w), make_uint2(RE1b.x, RE1b.y));
                    if (ne > 2) put_entry(b, xb + 2, make_uint2(RE2a.x, RE2a.y), make_uint2(RE2a.z, RE2a.w), make_uint2(RE2b.x, RE2b.y));
                    if (ne > 3) put_entry(b, xb + 3, make_uint2(RE3a.x, RE3a.y), make_uint2(RE3a.z, RE3a.w), make_uint2(RE3b.x, RE3b.y));
                    for (uint32_t k = CSR_EREG; k < ne; k++) {      // more than CSR_EREG: synchronous loads (rare)
                        const uint4 x0 = ent[2 * (ecur + k)], x1 = ent[2 * (ecur + k) + 1];
                        put_entry(b, xb + k, make_uint2(x0.x, x0.y), make_uint2(x0.z, x0.w), make_uint2(x1.x, x1.y));
                    }
                }
                s = (int32_t)R0.y;
#pragma unroll
                for (int q = 0; q < 8; q++) {                      // the codes back (this lane's own writes)
                    const u32x4 v = *(const u32x4 *)(trow + 4 * q);
                    code[4 * q] = v.x; code[4 * q + 1] = v.y; code[4 * q + 2] = v.z; code[4 * q + 3] = v.w;
                }
            }
        }
        if (was && !has) set_base();
        was = has;
    };

    // super step 0
    wload(wA0, wA1, 0);
    wstore(wA0, wA1, 0);
    wload(wB0, wB1, 1);
    prep(0, 0);
    if (live && rv && R0.x == 0) { base = csr_base(p, s); rcur++; ecur += R0.w; load_rec(rcur, ecur); }
    __syncthreads();
    CSR_STAMP(tl0);
    // (the loop runs two super steps per trip, one per buffer, so that every staging set and LDS buffer is named at
    // compile time: a buffer chosen at run time made the compiler select between the two sets' addresses and keep
    // both in scratch)
    auto iter = [&](uint32_t t, auto BC) {
        constexpr uint32_t b = decltype(BC)::value;
        const uint32_t K0 = t * CSR_SB;
        // set b is free: super step t is in LDS. (Issued even past the last super step, from clamped positions: with
        // the loads on one path only, the wait before the stores of the other set had to cover the path without them,
        // i.e. these very loads.)
        if constexpr (b) wload(wB0, wB1, t + 2);
        else wload(wA0, wA1, t + 2);
        // ---- the chain over blocks K0 .. K0 + 31 ----
        // The block loop is straight-line code per variant (FULL: every row's chain covers the whole super step, no
        // predication), and each block's three LDS reads are issued CSR_PF blocks ahead of its arithmetic: a read
        // followed at once by its use waits the whole LDS latency (about 120 cycles with four waves reading), twice
        // the chain's own cost of a block.
        CSR_STAMP(ts0);
        const bool full = __all(myit == 0u || K0 + CSR_SB <= myit);
        const char *EAb = (const char *)EA[b], *EBb = (const char *)EB;
        auto run = [&](auto FULLC) {
            constexpr bool FULL = decltype(FULLC)::value;
            u32x4 va[CSR_PF + 1], vb[CSR_PF + 1];
            auto fetch = [&](int i) {
#ifdef CSR_DIAG_BCAST
                // (diagnostic build only: every lane reads lane 0's entries: wrong checksums, no bank conflicts)
                const uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane((int)code[i]);
#else
                const uint32_t c = code[i];
#endif
                va[i % (CSR_PF + 1)] = *(const u32x4 *)(EAb + c);
                vb[i % (CSR_PF + 1)] = *(const u32x4 *)(EBb + c);
            };
#pragma unroll
            for (int i = 0; i < CSR_PF; i++) fetch(i);
#pragma unroll
            for (int i = 0; i < CSR_SB; i++) {
                if (i + CSR_PF < CSR_SB) fetch(i + CSR_PF);
                const u32x4 A = va[i % (CSR_PF + 1)], B = vb[i % (CSR_PF + 1)];
                if (FULL) {
                    csd_block3(Xg, Xf, Xh, A.x, A.y, A.z, A.w, b ? B.z : B.x, b ? B.w : B.y);
                } else {
                    uint32_t ng = Xg, nf = Xf, nh = Xh;
                    csd_block3(ng, nf, nh, A.x, A.y, A.z, A.w, b ? B.z : B.x, b ? B.w : B.y);
                    const bool act = K0 + (uint32_t)i < myit;
                    Xg = act ? ng : Xg;
                    Xf = act ? nf : Xf;
                    Xh = act ? nh : Xh;
                }
            }
        };
        if (full) run(std::integral_constant<bool, true>{});
        else run(std::integral_constant<bool, false>{});
        // ---- the next super step's window, rows and entries into the other buffer ----
        // (kept after the chain: hoisted above it, the stores of a staging set would wait for its loads there)
        asm volatile("" ::: "memory");
        CSR_STAMP(ts1);
        CSR_ACC(0, ts1 - ts0);
        // (run after the last super step too, into a buffer nobody reads: skipped on one path, the staging set's loads
        // stay pending on it, and the compiler waits for every load at the loop head before reusing their registers)
        if constexpr (b) wstore(wA0, wA1, 0u);                      // super step t + 1 (even) -> buffer 0
        else wstore(wB0, wB1, 1u);
        prep(t + 1, b ^ 1u);
        // (the record loads run for the whole wave whenever one of its rows moves on, the others reloading their
        // current record: a load into only some lanes keeps the old values live in the rest, and the compiler
        // copies the loaded registers over them, waiting for the loads right here)
        const bool adv = live && rv && R0.x == t + 1;
        if (adv) { base = csr_base(p, s); rcur++; ecur += R0.w; }
        if (__ballot(adv)) load_rec(rcur, ecur);
        CSR_STAMP(ts2);
        __syncthreads();
        CSR_STAMP(ts3);
        CSR_ACC(1, ts2 - ts1);
        CSR_ACC(2, ts3 - ts2);
    };
    // (both super steps of a trip always run, the odd last one after the loop: the loop head is then reached from
    // one kind of trip only, and the loads in flight there are always the same)
    uint32_t t = 0;
    for (; t + 1 < T_; t += 2) {
        iter(t, std::integral_constant<uint32_t, 0>{});
        iter(t + 1, std::integral_constant<uint32_t, 1>{});
    }
    if (t < T_) iter(t, std::integral_constant<uint32_t, 0>{});
    CSR_STAMP(tl1);
    CSR_ACC(3, tl1 - tl0);
#ifdef CSR_DIAG_STAMP
    if (lane == 0)
        for (int k = 0; k < 4; k++) ctr_add(d, C_NALL + k, (unsigned long long)st_[k]);
#endif
#undef CSR_STAMP
#undef CSR_ACC
    const bool mine = valid && fl == 0;
    const uint32_t nmine = (uint32_t)__popcll(__ballot(mine));
    if (lane == 0 && nmine) ctr_add(d, C_X_CS_ROWS, (unsigned long long)nmine);   // rows this launch hashed
    if (!valid) return;
    if (!mine) {                                                    // left to the production kernels
        const uint32_t at = atomicAdd(a.fb_cnt, 1u);
        a.fb_list[at] = id;
        // by reason (swimsim_checksum_path_stats): short, entry/run capacity, window plan, record capacity, slots
        const uint32_t r = (fl & CSD_F_SHORT) ? 0u : (fl & CSD_F_ECAP) ? 1u : (fl & CSR_F_PLAN) ? 2u : (fl & CSR_F_RCAP) ? 3u
                         : (fl & CSR_F_SLOTS) ? 4u : 6u;
        atomicAdd(a.fb_cnt + 1 + r, 1u);
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

// ---------------------------------------------------------------------------------------------------------------
// k_csr2: the chains with the h lane in a wave of its own (round 5). A block is 12 VALU instructions over three
// lanes of one row, of which h is independent of the coupled g and f. With one lane per row, 65,536 rows fill the
// chip's 1,024 SIMDs at one wave each, and a lone wave issues at best one instruction every ~5 cycles and waits
// ~10 for a dependent one: k_csr ran its 12-instruction block at ~93 cycles from LDS. Here each 64-row group has
// a g/f wave (8 instructions a block, a 5-deep dependent chain) and an h wave (4, 4 deep) on the same SIMD (waves w
// and w + 4 of the workgroup), so the SIMD interleaves two chains at the same instruction count. Each role stages its
// own half of the window (EA for g/f, EB for h), decodes the same records into its own codes (no code table in LDS:
// a record's 32 u16 codes are unpacked in registers, exception codes patched to the wave's slots), and writes its
// own half of the exception entries. The h wave hands its final state to the g/f wave through LDS at the end.
// ---------------------------------------------------------------------------------------------------------------
template <int W, int ROLE>                                           // ROLE 0: g/f lanes, 1: h lanes
__device__ __forceinline__ void csr2_role(const DS &d, const uint32_t *list, const uint32_t cnt, const CsrArgs &a,
                                          const CsrPlan &p, uint4 (*EA)[CSR_ENT], uint2 (*EB)[CSR_ENT], uint32_t *XH,
                                          const uint32_t *phs) {
    constexpr bool GF = ROLE == 0;
    constexpr uint32_t CSH = GF ? 0u : 1u;                           // EA entries are 16 B, EB entries 8 B
    const uint32_t tid = threadIdx.x & (CSR_ROWS - 1), rwave = tid >> 6;
    const uint32_t g0 = blockIdx.x * CSR_ROWS;
    const uint32_t gi = g0 + tid;
    const bool valid = gi < cnt;
    const uint32_t id = list[valid ? gi : g0];
    const bool is_row = id < d.NL;
    const uint32_t *row = csd_row(d, id);
    const CsdRow ri = a.rinfo[valid ? gi : g0];
    const uint32_t nrec = valid ? a.nrec[gi] : 0u;
    const uint32_t len = csd_len(d, id);
    const uint32_t iters = len > 24 ? (len - 1) / 20 : 0u;
    uint32_t fl = !valid ? 0u : ri.flags ? ri.flags : !p.feasible || ri.ecnt > p.ecmax ? CSR_F_PLAN
                : nrec == 0xFFFFFFFFu ? CSR_F_RCAP : 0u;
    if (valid && !fl && iters == 0) fl = CSD_F_SHORT;
    const bool live = valid && fl == 0;
    const uint32_t myit = live ? iters : 0u;
    const uint32_t T_ = p.feasible ? (p.maxit + CSR_SB - 1) / CSR_SB : 0u;
    const CsrRec *rec = a.rec + (size_t)(valid ? gi : g0) * a.rcap;
    const uint4 *ent = a.ent + (size_t)(valid ? gi : g0) * a.ecap * 2;
    const uint32_t nr = live ? nrec : 0u;

    FH fh{0, 0, 0};
    uint32_t it2 = 0;
    const bool ok = cs_prologue<W>(d, id, is_row, row, fh, it2);
    uint32_t X0 = GF ? fh.g + ri.b0 : fh.h + ri.a0;                  // Xg, or Xh
    uint32_t X1 = GF ? fh.f + ri.c0 : 0u;                            // Xf
    int32_t s = 0;
    uint32_t base = csr_base(p, 0);

    // records, one ahead (as k_csr: whole vector registers, unconditional loads from clamped indices)
    uint32_t rcur = 0, ecur = 0;
    bool rv = false;
    u32x4 R0, R1, R2, R3, R4;
    typedef typename std::conditional<GF, u32x4, u32x2>::type EV;   // this role's half of an exception entry
    EV RE0, RE1, RE2, RE3;
    auto ent_half = [&](uint32_t e) -> EV {
        if constexpr (GF) return *(const u32x4 *)(ent + 2 * e);
        else return *(const u32x2 *)(ent + 2 * e + 1);
    };
    auto load_rec = [&](uint32_t q, uint32_t e0) {
        const u32x4 *rp = (const u32x4 *)(rec + min(q, a.rcap - 1u));
        R0 = rp[0]; R1 = rp[1]; R2 = rp[2]; R3 = rp[3]; R4 = rp[4];
        const uint32_t eb = min(e0, a.ecap - (uint32_t)CSR_EREG);
        RE0 = ent_half(eb); RE1 = ent_half(eb + 1); RE2 = ent_half(eb + 2); RE3 = ent_half(eb + 3);
        rv = q < nr;
    };
    load_rec(0, 0);

    // window staging: entries u = tid + 256 v, this role's half, two register sets (super step u -> set u & 1)
    constexpr int WV = CSR_WINMAX / CSR_ROWS;
    EV wA[WV], wB[WV];
    const uint32_t nwin = p.nph * p.Wn;
    const uint4 *wsrc[WV];
    int32_t wk0[WV];
#pragma unroll
    for (int v = 0; v < WV; v++) {
        const uint32_t u = tid + (uint32_t)CSR_ROWS * v;
        const uint32_t ps = u < nwin ? u / p.Wn : 0u, w = u < nwin ? u - ps * p.Wn : 0u;
        wsrc[v] = a.P + 2 * (size_t)phs[min(ps, 19u)] * a.KP + (GF ? 0 : 1);
        wk0[v] = u < nwin ? (int32_t)w - p.cmax : 0x40000000;
    }
    auto wload = [&](EV (&wst)[WV], uint32_t t) {
#pragma unroll
        for (int v = 0; v < WV; v++) {
            const int32_t k = min(max(wk0[v] + (int32_t)(t * CSR_SB), 0), (int32_t)a.KP - 1);
            wst[v] = *(const EV *)(wsrc[v] + 2 * (uint32_t)k);
        }
    };
    auto put = [&](uint32_t b, uint32_t e, const EV &x) {
        if constexpr (GF) *(u32x4 *)&EA[b][e] = x;
        else *(u32x2 *)&EB[b][e] = x;
    };
    auto wstore = [&](const EV (&wst)[WV], uint32_t b) {
#pragma unroll
        for (int v = 0; v < WV; v++) put(b, tid + (uint32_t)CSR_ROWS * v, wst[v]);
    };

    uint32_t code[CSR_SB];
    auto set_base = [&]() {
        const uint32_t ba = (base * CSR_ESZ) >> CSH;
#pragma unroll
        for (int i = 0; i < CSR_SB; i++) code[i] = ba + (((uint32_t)i * CSR_ESZ) >> CSH);
    };
    if (live) set_base();
    else {
#pragma unroll
        for (int i = 0; i < CSR_SB; i++) code[i] = 0u;
    }
    bool was = false;
    auto prep = [&](uint32_t t, uint32_t b) {
        const bool has = live && rv && R0.x == t;
        if (__ballot(has)) {
            uint32_t ne = has ? R0.w : 0u, tot = 0;
            const uint32_t sb = wscan_excl(ne, tot);              // this row's first slot in the wave's area
            const uint32_t xb = (uint32_t)CSR_WINMAX + rwave * CSR_EXW + sb;
            if (has && sb + ne > (uint32_t)CSR_EXW) fl |= CSR_F_SLOTS;
            if (has) {
                const uint32_t xa = xb * CSR_ESZ;
                auto dec = [&](uint32_t c) -> uint32_t {          // a record code -> this role's LDS offset
                    return ((c & CSR_EXC) ? xa + (c & 0x7FFFu) * CSR_ESZ : c) >> CSH;
                };
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const u32x4 Rq = q == 0 ? R1 : q == 1 ? R2 : q == 2 ? R3 : R4;
                    code[8 * q + 0] = dec(Rq.x & 0xFFFFu); code[8 * q + 1] = dec(Rq.x >> 16);
                    code[8 * q + 2] = dec(Rq.y & 0xFFFFu); code[8 * q + 3] = dec(Rq.y >> 16);
                    code[8 * q + 4] = dec(Rq.z & 0xFFFFu); code[8 * q + 5] = dec(Rq.z >> 16);
                    code[8 * q + 6] = dec(Rq.w & 0xFFFFu); code[8 * q + 7] = dec(Rq.w >> 16);
                }
                if (!(fl & CSR_F_SLOTS)) {
                    if (ne > 0) put(b, xb + 0, RE0);
                    if (ne > 1) put(b, xb + 1, RE1);
                    if (ne > 2) put(b, xb + 2, RE2);
                    if (ne > 3) put(b, xb + 3, RE3);
                    for (uint32_t k = CSR_EREG; k < ne; k++) put(b, xb + k, ent_half(ecur + k));   // (rare)
                }
                s = (int32_t)R0.y;
            }
        }
        if (was && !has) set_base();
        was = has;
    };

    // super step 0
    wload(wA, 0);
    wstore(wA, 0);
    wload(wB, 1);
    prep(0, 0);
    if (live && rv && R0.x == 0) { base = csr_base(p, s); rcur++; ecur += R0.w; load_rec(rcur, ecur); }
    lds_barrier();
    auto iter = [&](uint32_t t, auto BC) {
        constexpr uint32_t b = decltype(BC)::value;
        const uint32_t K0 = t * CSR_SB;
        if constexpr (b) wload(wB, t + 2);
        else wload(wA, t + 2);
        const bool full = __all(myit == 0u || K0 + CSR_SB <= myit);
        const char *Eb = GF ? (const char *)EA[b] : (const char *)EB[b];
        auto run = [&](auto FULLC) {
            constexpr bool FULL = decltype(FULLC)::value;
            EV va[CSR_PF + 1];
            auto fetch = [&](int i) { va[i % (CSR_PF + 1)] = *(const EV *)(Eb + code[i]); };
#pragma unroll
            for (int i = 0; i < CSR_PF; i++) fetch(i);
#pragma unroll
            for (int i = 0; i < CSR_SB; i++) {
                if (i + CSR_PF < CSR_SB) fetch(i + CSR_PF);
                const EV A = va[i % (CSR_PF + 1)];
                uint32_t n0 = X0, n1 = X1;
                if constexpr (GF) csd_gf_step(n0, n1, A.x, A.y, A.z, A.w);
                else csd_h_step(n0, A.x, A.y);
                if (FULL) {
                    X0 = n0; X1 = n1;
                } else {
                    const bool act = K0 + (uint32_t)i < myit;
                    X0 = act ? n0 : X0;
                    X1 = act ? n1 : X1;
                }
            }
        };
        if (full) run(std::integral_constant<bool, true>{});
        else run(std::integral_constant<bool, false>{});
        asm volatile("" ::: "memory");
        if constexpr (b) wstore(wA, 0u);                           // super step t + 1 (even) -> buffer 0
        else wstore(wB, 1u);
        prep(t + 1, b ^ 1u);
        const bool adv = live && rv && R0.x == t + 1;
        if (adv) { base = csr_base(p, s); rcur++; ecur += R0.w; }
        if (__ballot(adv)) load_rec(rcur, ecur);
        lds_barrier();
    };
    uint32_t t = 0;
    for (; t + 1 < T_; t += 2) {
        iter(t, std::integral_constant<uint32_t, 0>{});
        iter(t + 1, std::integral_constant<uint32_t, 1>{});
    }
    if (t < T_) iter(t, std::integral_constant<uint32_t, 0>{});

    if constexpr (!GF) XH[tid] = X0;
    lds_barrier();
    if constexpr (GF) {
        const bool mine = valid && fl == 0;
        const uint32_t nmine = (uint32_t)__popcll(__ballot(mine));
        if ((threadIdx.x & 63u) == 0 && nmine) ctr_add(d, C_X_CS_ROWS, (unsigned long long)nmine);
        if (!valid) return;
        if (!mine) {                                                // left to the production kernels
            const uint32_t at = atomicAdd(a.fb_cnt, 1u);
            a.fb_list[at] = id;
            const uint32_t r = (fl & CSD_F_SHORT) ? 0u : (fl & CSD_F_ECAP) ? 1u : (fl & CSR_F_PLAN) ? 2u : (fl & CSR_F_RCAP) ? 3u
                             : 4u;
            atomicAdd(a.fb_cnt + 1 + r, 1u);
            return;
        }
        fh.h = XH[tid]; fh.g = X0; fh.f = X1;
        const uint32_t hv = ok ? fh.fin() : 0u;
        if (is_row) {
            d.cs[id] = hv;
            d.dirty[id] = 0;
        } else {
            d.dense_cs[id - d.NL] = hv;
        }
    }
}

template <int W>
__global__ void __launch_bounds__(2 * CSR_ROWS) k_csr2(DS d, const uint32_t *list, const uint32_t *count, CsrArgs a) {
    __shared__ uint4 EA[2][CSR_ENT];
    __shared__ uint2 EB[2][CSR_ENT];
    __shared__ uint32_t XH[CSR_ROWS];
    __shared__ uint32_t phs[20];
    const uint32_t cnt = *count;
    if (blockIdx.x * CSR_ROWS >= cnt) return;
    const CsrPlan p = a.plan[blockIdx.x];
    if (threadIdx.x < 20 && ((p.phm >> threadIdx.x) & 1u)) phs[__popc(p.phm & ((1u << threadIdx.x) - 1u))] = threadIdx.x;
    __syncthreads();
    // waves 0-3: g/f lanes of rows 64 w .. 64 w + 63; waves 4-7: their h lanes (wave w + 4 shares wave w's SIMD)
    if (threadIdx.x < CSR_ROWS) csr2_role<W, 0>(d, list, cnt, a, p, EA, EB, XH, phs);
    else csr2_role<W, 1>(d, list, cnt, a, p, EA, EB, XH, phs);
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
        hipLaunchKernelGGL(k_csr_rec, dim3((n + 3) / 4), dim3(256), 0, s, d, list, n, a);
    } else if (part == 4) {
        hipLaunchKernelGGL((k_csr2<W>), dim3((n + CSR_ROWS - 1) / CSR_ROWS), dim3(2 * CSR_ROWS), 0, s, d, list, count, a);
    } else {                                                        // (round 4's one-wave chains, for comparison)
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
