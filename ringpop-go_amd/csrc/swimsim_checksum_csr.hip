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
//                 32 codes (u16: a clean block's window entry as an LDS byte address), the shift after it and the
//                 mask of its exception blocks
//   k_csr3        the chains (below): 256 rows per workgroup, four waves per SIMD (the rows' g/f lanes, their h lanes,
//                 a record stager that fills their codes and exception entries and a window stager), handed over
//                 through LDS counters
// Rows the path cannot take (scan flags, an infeasible window, a super step with more exception entries than a
// ring) are listed and hashed by the production kernels (k_checksum3 / k_checksum_q16): bit-exact either way.

constexpr int CSR_ROWS = 256;          // rows per workgroup (4 row groups of 64)
constexpr int CSR_SB = 32;             // blocks per super step
constexpr int CSR_WINMAX = 1024;       // window entries per buffer: phases in use x Wn
constexpr int C3_NB = 3;               // k_csr3's window and code table buffers (super step t: buffer t % 3)
#ifndef C3_CTR_AT_DEF
#define C3_CTR_AT_DEF 26
#endif
// the chain block at which a chain wave reads the next super step's hand-over counters (26: 4.66 / 7.41 ms on real
// cascade rounds 14 / 18 at 65,536 rows, against 4.79 / 7.45 read before block 0 and 4.62 / 7.44 at block 16; a read
// that comes too early finds the stagers short and costs a wait of an LDS round trip)
constexpr int C3_CTR_AT = C3_CTR_AT_DEF;
constexpr uint32_t CSR_ESZ = 16;       // a code's unit: an entry's byte offset in each of the two entry arrays
constexpr int CSR_EREG = 4;            // exception entries of a record prefetched with it
#ifndef CSR_PF_DEF
#define CSR_PF_DEF 6
#endif
constexpr int CSR_PF = CSR_PF_DEF;     // blocks the chain's LDS reads run ahead of its arithmetic (6: 7.37 / 11.52 ms
                                       // on rounds 14 / 18 against 7.48 / 11.69 with 4 and 8.00 / 12.00 with 2)
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
    uint32_t xmask, ne;    // its exception blocks (bit i: block i; their entries in block order), their number
    uint32_t code[16];     // 32 u16 codes, block i in the low half of code[i / 2] for even i: the byte address of a
                           // clean block's entry in k_csr3's window buffer t % 3 (0 for an exception block)
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
    uint32_t exw;                 // k_csr3: cap on a row group's exception ring entries (~0; tests lower it to 8,
                                  // swimsim_tuning.fault_inject bit 4)
    uint32_t stprio;              // k_csr3: stager waves at issue priority 1 (tests: fault_inject bit 16, a schedule
                                  // that let one kind of chain wave run super steps ahead of the other)
    uint32_t jitter;              // k_csr3 (tests: fault_inject 64): 0 off; else bits 0-3 the roles to delay (g/f, h,
                                  // record stager, window stager), bits 8-31 the seed of their delays
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int32_t csr_ceil20(int32_t x) { return x >= 0 ? (x + 19) / 20 : -((-x) / 20); }

// The window of a super step holds, for every phase in use (slot ps of nph) and window position w (0 .. Wn-1), the
// premixed entry of S_B block 32 t - cmax + w at that phase, phase-interleaved: entry w nph + ps. A row at shift s
// reads position cmax - ceil(s / 20) + i for block i, so its entry is const + nph i - s / 2 (for even shifts; nph = 10
// with every even phase in use): rows at nearby shifts read nearby entries, in distinct LDS banks. (Round 4's
// phase-major layout, entry ps Wn + w, put rows 18 bytes apart on one bank: 1.05e9 bank-conflict cycles per heavy
// launch, half of the LDS's active cycles.)
// The entry of block 0 of a super step for a row at shift s (clamped into the window: a shift with no clean block
// after it, i.e. past the row's last exception run, is only ever read by predicated blocks beyond the row's chain);
// block i's entry is that + i nph.
__device__ __forceinline__ uint32_t csr_base(const CsrPlan &p, int32_t s) {
    const uint32_t phi = csd_phase(s);
    const uint32_t ps = (uint32_t)__popc(p.phm & ((1u << phi) - 1u));
    const int32_t w = min(max(p.cmax - csr_ceil20(s), 0), (int32_t)p.Wn - CSR_SB);
    return (uint32_t)w * p.nph + ps;
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
            p.Wn = (uint32_t)(CSR_SB + (p.cmax - csr_ceil20(smin)) + 1);
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
                    const uint32_t wbase = (t % C3_NB) * p.nph * p.Wn;     // (k_csr3's window buffer t % 3)
                    uint32_t q = lane, kn = h.x, pos = 0;
                    for (uint32_t b = 0; b < (uint32_t)CSR_SB; b++) {
                        const uint32_t j = K0 + b;
                        uint32_t c;
                        if (q < gend && kn == j) {
                            c = 0;
                            pos |= 1u << b;
                            s = (int32_t)hd[wv][q].y;
                            q++;
                            kn = q < gend ? hd[wv][q].x : 0xFFFFFFFFu;
                        } else {
                            c = j < iters ? (wbase + csr_base(p, s) + b * p.nph) * CSR_ESZ : 0u;
                        }
                        if (b & 1u) r.code[b >> 1] |= c << 16;
                        else r.code[b >> 1] = c;
                    }
                    r.t = t;
                    r.s_end = s;
                    r.xmask = pos;
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

// ---------------------------------------------------------------------------------------------------------------
// k_csr3: chain waves that only run chains (round 5). k_csr2's waves spent 39 % (light rounds) to 55 % (heavy) of
// their loop outside the chain: staging the next super step's window, unpacking records, writing exception entries,
// and waiting at the per-super-step barrier for the slowest of the eight (shader-clock stamps, tools/csr_stamps.py).
// Here two more waves per SIMD do all of that ahead of the chains, the record stager (lane = row: codes, exception
// entries) and the window stager (a quarter of the window, three super steps ahead), and no barrier is left in the
// loop. The window and the codes are triple-buffered (window buffer and code table t % 3) and the exception entries
// live in a ring per row group, so a record stager runs up to two super steps ahead of its chains (the stamps of the
// double-buffered version: its chains waited 30 % of a heavy round for it while it waited 45 % of the time for them,
// one super step of slack against records that come in bursts). LDS counters hand the buffers over: readyw[b] (window
// stagers that filled window buffer b: 4 per super step), done[k][b] (chain waves of kind k, g/f or h, done with it: 4
// per super step, which the window stagers wait for), readyr[g] (super steps group g's record stager has staged) and
// doner[k][g] (super steps group g's chain wave of kind k has finished: a group's codes and ring are its own, so its
// record stager waits only for them). Done counts are kept per kind because a kind's waves can run super steps ahead
// of the other's. Codes are u16 byte offsets into the entry arrays (window buffers 0, 1 and 2, then the four rings), so
// base codes do not depend on which window buffer a code buffer meets.
// A chain wave waits only until the stagers have filled the super step it needs, reads its row's 32 codes (base(s) + i
// in its window buffer, or a record's codes with its exceptions patched to ring slots) and runs the chain. Roles:
// waves 0-3 g/f lanes, 4-7 h lanes, 8-11 record stagers, 12-15 window stagers; waves w, w + 4, w + 8 and w + 12 share
// a SIMD and rows 64 w .. 64 w + 63. The kernel's one barrier after the loops (every role reaches it from the same
// call site) hands the h lanes' state and the stagers' flags to the g/f waves' epilogue.
// Tests perturb the hand-over (CsrArgs::jitter, swimsim_tuning.fault_inject 64): seeded sleeps before every counter
// wait and signal of the selected roles, so one kind of chain wave runs ahead of the other, or a stager falls behind.
// ---------------------------------------------------------------------------------------------------------------
constexpr int C3_ENT = 4096;               // entries: 3 windows of nwin entries, then 4 rings share the rest
static_assert(C3_NB * CSR_WINMAX + 4 * 256 <= C3_ENT, "rings of at least 256 entries");
static_assert(C3_ENT * CSR_ESZ <= 65536, "codes are u16 byte offsets");

struct Csr3Lds {
    // (EB first: both arrays then start below 64 KB, so an entry's base folds into the LDS reads' immediate offset;
    // with EB at 64 KB every h-lane read took a v_or of its base)
    uint2 EB[C3_ENT];                      // {Mh, KH} per entry: window buffers 0 and 1, then the rings
    uint4 EA[C3_ENT];                      // {Mg, D, Mf, PF}
    uint4 TC[C3_NB][4][CSR_ROWS];         // codes: TC[k][q][row] = u16 codes 8q .. 8q + 7 of the row (lane-contiguous)
    uint32_t XH[CSR_ROWS];                 // h lanes' final state
    uint32_t FLX[CSR_ROWS];                // rows the stagers flagged (exception slots)
    uint32_t readyw[C3_NB];                // window stagers that filled buffer b (4 a super step)
    uint32_t done[2][C3_NB];               // [g/f, h] chain waves done with buffer b (4 a super step each)
    uint32_t readyr[4], doner[2][4];       // per row group: super steps staged by its record stager; done by its g/f
                                           // and its h wave (one count per kind: one kind's waves can run steps ahead
                                           // of the other's, and a shared count let the leader's steps stand in for
                                           // the laggard's, which was still reading the buffer)
    uint32_t phs[20];
};

__device__ __forceinline__ void c3_wait(const uint32_t *ctr, uint32_t target) {
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
}
// both kinds of chain wave (g/f: ctr[0][i], h: ctr[1][i]) have reached target
template <int NI>
__device__ __forceinline__ void c3_wait2(const uint32_t (&ctr)[2][NI], uint32_t i, uint32_t target) {
#ifdef C3_T_SHAREDDONE
    c3_wait(&ctr[0][i], 2u * target);                                // (test build: round 5's racy shared count)
#else
    c3_wait(&ctr[0][i], target);
    c3_wait(&ctr[1][i], target);
#endif
}
__device__ __forceinline__ void c3_signal(uint32_t *ctr) {
    if ((threadIdx.x & 63u) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// tests only (CsrArgs::jitter): a seeded, wave-uniform delay before a hand-over wait or signal of role `role` at super
// step t (site: which wait or signal). With probability 3/8 the wave sleeps 0 .. 127 x 128 clocks, up to several super
// steps of chain, so every order of the four roles around a buffer reuse occurs somewhere in a launch.
__device__ __forceinline__ void c3_jitter(uint32_t jit, uint32_t role, uint32_t t, uint32_t site) {
    if (!((jit >> role) & 1u)) return;
    const uint32_t x = fmix32((jit >> 8) * 0x9E3779B9u ^ blockIdx.x * 0x85EBCA6Bu ^ (threadIdx.x >> 6) * 0xC2B2AE35u ^
                              t * 0x27D4EB2Fu ^ site * 0x165667B1u);
    if ((x & 7u) < 3u)
        for (uint32_t k = (x >> 8) & 127u; k; k--) __builtin_amdgcn_s_sleep(2);
}

struct C3Row {                                                      // what every role knows of its row
    uint32_t gi, id, fl, iters, nrec;
    bool valid, is_row, live;
    CsdRow ri;
};
__device__ __forceinline__ C3Row c3_row(const DS &d, const uint32_t *list, uint32_t cnt, const CsrArgs &a,
                                        const CsrPlan &p, uint32_t tid) {
    C3Row r;
    const uint32_t g0 = blockIdx.x * CSR_ROWS;
    r.gi = g0 + tid;
    r.valid = r.gi < cnt;
    r.id = list[r.valid ? r.gi : g0];
    r.is_row = r.id < d.NL;
    r.ri = a.rinfo[r.valid ? r.gi : g0];
    r.nrec = r.valid ? a.nrec[r.gi] : 0u;
    const uint32_t len = csd_len(d, r.id);
    r.iters = len > 24 ? (len - 1) / 20 : 0u;
    r.fl = !r.valid ? 0u : r.ri.flags ? r.ri.flags : !p.feasible || r.ri.ecnt > p.ecmax ? CSR_F_PLAN
         : r.nrec == 0xFFFFFFFFu ? CSR_F_RCAP : 0u;
    if (r.valid && !r.fl && r.iters == 0) r.fl = CSD_F_SHORT;
    r.live = r.valid && r.fl == 0;
    return r;
}

// the record stager of rows 64 w .. 64 w + 63 (lane = row): their codes and exception entries, up to two super steps
// ahead of the group's chains
__device__ __forceinline__ void c3_stage(const DS &d, const uint32_t *list, uint32_t cnt, const CsrArgs &a, const CsrPlan &p,
                                         Csr3Lds &L, uint32_t T_) {
    const uint32_t tid = threadIdx.x & (CSR_ROWS - 1), rwave = tid >> 6;
#if defined(C3_SPRIO) && C3_SPRIO > 0
    __builtin_amdgcn_s_setprio(C3_SPRIO);
#endif
    if (a.stprio) __builtin_amdgcn_s_setprio(1);
    C3Row r = c3_row(d, list, cnt, a, p, tid);
    const CsrRec *rec = a.rec + (size_t)(r.valid ? r.gi : blockIdx.x * CSR_ROWS) * a.rcap;
    const uint4 *ent = a.ent + (size_t)(r.valid ? r.gi : blockIdx.x * CSR_ROWS) * a.ecap * 2;
    const uint32_t nr = r.live ? r.nrec : 0u;
    uint32_t rcur = 0, ecur = 0;
    bool rv = false;
    u32x4 R0, R1, R2, R3, R4;
    u32x4 EA0, EA1, EA2, EA3;
    u32x2 EB0, EB1, EB2, EB3;
    auto load_rec = [&](uint32_t q, uint32_t e0) {
        const u32x4 *rp = (const u32x4 *)(rec + min(q, a.rcap - 1u));
        R0 = rp[0]; R1 = rp[1]; R2 = rp[2]; R3 = rp[3]; R4 = rp[4];
        // (no clamp: the entry array has CSR_EREG spare entries past its last row, csr_alloc, so a record whose entries
        // start within CSR_EREG of a row's cap loads its own entries; what lies past them is never stored)
        const u32x4 *ep = (const u32x4 *)(ent + 2 * e0);
        EA0 = ep[0]; EB0 = *(const u32x2 *)(ep + 1);
        EA1 = ep[2]; EB1 = *(const u32x2 *)(ep + 3);
        EA2 = ep[4]; EB2 = *(const u32x2 *)(ep + 5);
        EA3 = ep[6]; EB3 = *(const u32x2 *)(ep + 7);
        rv = q < nr;
    };
    load_rec(0, 0);
    int32_t s = 0;
    uint32_t base = csr_base(p, 0);
    // what TC[k][.][row] holds: base codes (base), or a record (~0)
    uint32_t tg0 = 0xFFFFFFFEu, tg1 = 0xFFFFFFFEu, tg2 = 0xFFFFFFFEu;
    // the group's ring: the entries past the three windows (nwin each), a quarter each; alloc counts the entries handed
    // out (monotone), e1 .. e3 what it was after super steps u - 1 .. u - 3, rpos the next free one
    const uint32_t nwin = p.nph * p.Wn, Rf = ((uint32_t)C3_ENT - C3_NB * nwin) / 4u, R = min(Rf, a.exw);
    const uint32_t ring0 = C3_NB * nwin + rwave * Rf;
    uint32_t alloc = 0, e1 = 0, e2 = 0, e3 = 0, rpos = 0;
    // (k is a compile-time constant: the loop is unrolled by the 3 buffers, so the tags stay in registers)
    auto tag_ref = [&](auto KC) -> uint32_t & {
        constexpr uint32_t k = decltype(KC)::value;
        if constexpr (k == 0) return tg0;
        else if constexpr (k == 1) return tg1;
        else return tg2;
    };
    // one super step's codes and exceptions of this row into code buffer k (window buffer b)
#ifdef CSR_DIAG_NE
    uint64_t dg_[4] = {0, 0, 0, 0};
#endif
    auto prep = [&](uint32_t t, uint32_t b, auto KC) {
        constexpr uint32_t k = decltype(KC)::value;
#ifdef C3_T_NOREC
        const bool has = false;
#else
        const bool has = r.live && rv && R0.x == t;
#endif
        if (__ballot(has)) {
            uint32_t ne = has && !(r.fl & CSR_F_SLOTS) ? R0.w : 0u, tot = 0;
#ifdef CSR_DIAG_NE
            {                                                       // (diagnostics: record super steps, long ones)
                const uint64_t bh = __ballot(has), bl = __ballot(ne > (uint32_t)CSR_EREG);
                dg_[0]++;
                dg_[1] += (uint64_t)__popcll(bh);
                dg_[2] += bl ? 1u : 0u;
                dg_[3] += (uint64_t)__popcll(bl);
            }
#endif
            const uint32_t sb = wscan_excl(ne, tot);
            // ring slots for the wave's exceptions; rows past the ring's size are left to the production kernels
            const bool over = has && ne > 0 && sb + ne > R;
            const uint32_t need = tot > R ? wmin(over ? sb : 0xFFFFFFFFu) : tot;
            if (over) r.fl |= CSR_F_SLOTS;
            const uint32_t skip = rpos + need > R ? R - rpos : 0u;
            // the slots of super steps t - 2 and t - 1 may still be read (those of t - 3 are free: the step's wait)
            if (alloc + skip + need - e3 > R) {
                if (t >= 2) c3_wait2(L.doner, rwave, t - 1u);
                if (alloc + skip + need - e2 > R && t >= 1) c3_wait2(L.doner, rwave, t);
            }
            const uint32_t xb = ring0 + (skip ? 0u : rpos) + sb;
            alloc += skip + need;
            rpos = (skip ? 0u : rpos) + need;
            if (rpos >= R) rpos = 0;
            if (has) {
                // (the record's codes address window buffer t % 3 = k already; its exception blocks are patched below)
                L.TC[k][0][tid] = make_uint4(R1.x, R1.y, R1.z, R1.w);
                L.TC[k][1][tid] = make_uint4(R2.x, R2.y, R2.z, R2.w);
                L.TC[k][2][tid] = make_uint4(R3.x, R3.y, R3.z, R3.w);
                L.TC[k][3][tid] = make_uint4(R4.x, R4.y, R4.z, R4.w);
                tag_ref(KC) = 0xFFFFFFFFu;
                if (!(r.fl & CSR_F_SLOTS)) {
                    const uint32_t xa = xb * CSR_ESZ;
                    // exception codes -> the ring's slots (u16 stores into the row's codes): block i lives in
                    // TC[k][i / 8][row], halfword i % 8
                    auto patch = [&](uint32_t i, uint32_t ord) {
                        uint16_t *c16 = (uint16_t *)&L.TC[k][i >> 3][tid] + (i & 7u);
                        *c16 = (uint16_t)(xa + ord * CSR_ESZ);
                    };
                    uint32_t m = R0.z;                             // exception blocks, their entries in block order
                    if (ne > 0) { patch((uint32_t)__builtin_ctz(m), 0); m &= m - 1u; }
                    if (ne > 1) { patch((uint32_t)__builtin_ctz(m), 1); m &= m - 1u; }
                    if (ne > 2) { patch((uint32_t)__builtin_ctz(m), 2); m &= m - 1u; }
                    if (ne > 3) { patch((uint32_t)__builtin_ctz(m), 3); m &= m - 1u; }
                    for (uint32_t ord = CSR_EREG; m; ord++, m &= m - 1u) patch((uint32_t)__builtin_ctz(m), ord);   // (rare)
                    auto putx = [&](uint32_t e, const u32x4 &x, const u32x2 &y) {
                        *(u32x4 *)&L.EA[e] = x;
                        *(u32x2 *)&L.EB[e] = y;
                    };
                    if (ne > 0) putx(xb + 0, EA0, EB0);
                    if (ne > 1) putx(xb + 1, EA1, EB1);
                    if (ne > 2) putx(xb + 2, EA2, EB2);
                    if (ne > 3) putx(xb + 3, EA3, EB3);
                    for (uint32_t j = CSR_EREG; j < ne; j++) {      // more than CSR_EREG: synchronous loads (rare)
                        const uint4 *ep = ent + 2 * (ecur + j);
                        putx(xb + j, *(const u32x4 *)ep, *(const u32x2 *)(ep + 1));
                    }
                }
                s = (int32_t)R0.y;
            }
        }
        if (!has) {
            const uint32_t want = r.live ? base : 0xFFFFFFFDu;      // (rows not hashed read entry 0)
            if (tag_ref(KC) != want) {
                const uint32_t c0 = r.live ? (k * nwin + base) * CSR_ESZ : 0u;
                const uint32_t st1 = r.live ? p.nph * CSR_ESZ : 0u, st2 = 2u * st1;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t c = c0 + (uint32_t)(4 * q) * st2;
                    L.TC[k][q][tid] = make_uint4(c | ((c + st1) << 16), (c + st2) | ((c + st2 + st1) << 16),
                                                 (c + 2 * st2) | ((c + 2 * st2 + st1) << 16),
                                                 (c + 3 * st2) | ((c + 3 * st2 + st1) << 16));
                }
                tag_ref(KC) = want;
            }
        }
        const bool adv = has;
        if (adv) { base = csr_base(p, s); rcur++; ecur += R0.w; }
        if (__ballot(adv)) load_rec(rcur, ecur);
    };
#ifdef CSR_DIAG_STAMP
    // (diagnostic build only: the stagers' shader-clock stamps into diagnostic counters 4-7: waiting for the chains,
    // the window, the rows' codes and exceptions, the hand-over)
    uint64_t st_[4] = {0, 0, 0, 0};
    auto stamp = [&]() -> uint64_t {
        uint64_t tt;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tt) :: "memory");
        __builtin_amdgcn_sched_barrier(0);
        return tt;
    };
#define C3S_STAMP(v) const uint64_t v = stamp()
#define C3S_ACC(k, x) st_[k] += (x)
#else
#define C3S_STAMP(v)
#define C3S_ACC(k, x)
#endif
    auto step = [&](uint32_t u, auto BC, auto KC) {
        constexpr uint32_t b = decltype(BC)::value;
        C3S_STAMP(s0);
        c3_jitter(a.jitter, 2, u, 0);
        if (u >= 3) c3_wait2(L.doner, rwave, u - 2u);               // this group's chains are done with super step u - 3
        C3S_STAMP(s1);
#ifdef CSR_DIAG_STAMP
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");            // (diagnostics: slot 1 = the record loads' wait)
#endif
        C3S_STAMP(s2);
        prep(u, b, KC);
        e3 = e2; e2 = e1; e1 = alloc;
        C3S_STAMP(s3);
        c3_jitter(a.jitter, 2, u, 1);
        c3_signal(&L.readyr[rwave]);
        C3S_STAMP(s4);
        C3S_ACC(0, s1 - s0);
#ifndef CSR_DIAG_WINDOW
        C3S_ACC(1, s2 - s1);
#endif
        C3S_ACC(2, s3 - s2);
#ifndef CSR_DIAG_WINDOW
        C3S_ACC(3, s4 - s3);
#endif
    };
    using I0 = std::integral_constant<uint32_t, 0>;
    using I1 = std::integral_constant<uint32_t, 1>;
    using I2 = std::integral_constant<uint32_t, 2>;
    for (uint32_t u = 0; u < T_; u += 3) {                          // (super step u + j: buffers j)
        step(u, I0{}, I0{});
        if (u + 1 >= T_) break;
        step(u + 1, I1{}, I1{});
        if (u + 2 >= T_) break;
        step(u + 2, I2{}, I2{});
    }
#ifdef CSR_DIAG_STAMP
    if ((threadIdx.x & 63u) == 0)
        for (int k = 0; k < 4; k++) ctr_add(d, C_NALL + 4 + k, (unsigned long long)st_[k]);
#endif
#undef C3S_STAMP
#undef C3S_ACC
#ifdef CSR_DIAG_NE
    if ((threadIdx.x & 63u) == 0)
        for (int k = 0; k < 4; k++) ctr_add(d, C_NALL + 4 + k, (unsigned long long)dg_[k]);
#endif
    L.FLX[tid] = r.fl;
}

// the window stager (role 3): a quarter of every super step's window, entries u = tid + 256 v (both halves), from
// three register sets (super step u -> set u % 3) loaded three super steps ahead. A wave of its own since round 5's
// stamps: in the record stager's loop the window took 34-43 % of the chain waves' loop, and the chains waited for it.
__device__ __forceinline__ void c3_wstage(const CsrArgs &a, const CsrPlan &p, Csr3Lds &L, uint32_t T_) {
    const uint32_t tid = threadIdx.x & (CSR_ROWS - 1);
#if defined(C3_WPRIO) && C3_WPRIO > 0
    __builtin_amdgcn_s_setprio(C3_WPRIO);
#endif
    if (a.stprio) __builtin_amdgcn_s_setprio(1);
    // window: entries u = tid + 256 v (both halves), two register sets (super step u -> set u & 1), loaded two ahead
    constexpr int WV = CSR_WINMAX / CSR_ROWS;
    u32x4 wA0[WV], wB0[WV], wC0[WV];
    u32x2 wA1[WV], wB1[WV], wC1[WV];
    const uint32_t nwin = p.nph * p.Wn;
    uint32_t wsrc[WV];                                               // (phase rows of P as entry offsets: 32-bit)
    int32_t wk0[WV];
#pragma unroll
    for (int v = 0; v < WV; v++) {
        const uint32_t u = tid + (uint32_t)CSR_ROWS * v;
        const uint32_t w = u < nwin ? u / p.nph : 0u, ps = u < nwin ? u - w * p.nph : 0u;   // (phase-interleaved)
        wsrc[v] = L.phs[min(ps, 19u)] * a.KP;
        wk0[v] = u < nwin ? (int32_t)w - p.cmax : 0x40000000;
    }
    auto wload = [&](u32x4 (&w0)[WV], u32x2 (&w1)[WV], uint32_t t) {
#pragma unroll
        for (int v = 0; v < WV; v++) {
            const int32_t k = min(max(wk0[v] + (int32_t)(t * CSR_SB), 0), (int32_t)a.KP - 1);
            const uint4 *src = a.P + 2 * (size_t)(wsrc[v] + (uint32_t)k);
#ifdef C3_T_NOWIN
            w0[v] = u32x4{(uint32_t)k, 1u, 2u, 3u}; w1[v] = u32x2{(uint32_t)k, 5u}; (void)src;
#else
            w0[v] = *(const u32x4 *)src;
            w1[v] = *(const u32x2 *)(src + 1);
#endif
        }
    };
    auto wstore = [&](const u32x4 (&w0)[WV], const u32x2 (&w1)[WV], uint32_t b) {
#pragma unroll
        for (int v = 0; v < WV; v++) {
            const uint32_t u = tid + (uint32_t)CSR_ROWS * v;
            if (u < nwin) {
                *(u32x4 *)&L.EA[b * nwin + u] = w0[v];
                *(u32x2 *)&L.EB[b * nwin + u] = w1[v];
            }
        }
    };
    wload(wA0, wA1, 0);
    wload(wB0, wB1, 1);
    wload(wC0, wC1, 2);
    // super step u = 3 j + b: register set and buffer b, loaded three super steps ahead
    auto step = [&](uint32_t u, uint32_t j, auto BC) {
        constexpr uint32_t b = decltype(BC)::value;
        c3_jitter(a.jitter, 3, u, 0);
        if (j > 0) c3_wait2(L.done, b, 4u * j);                      // every chain is done with super step u - 3
        if constexpr (b == 0) { wstore(wA0, wA1, 0u); wload(wA0, wA1, u + 3); }
        else if constexpr (b == 1) { wstore(wB0, wB1, 1u); wload(wB0, wB1, u + 3); }
        else { wstore(wC0, wC1, 2u); wload(wC0, wC1, u + 3); }
        c3_jitter(a.jitter, 3, u, 1);
        c3_signal(&L.readyw[b]);
    };
    for (uint32_t u = 0, j = 0; u < T_; u += 3, j++) {
        step(u, j, std::integral_constant<uint32_t, 0>{});
        if (u + 1 >= T_) break;
        step(u + 1, j, std::integral_constant<uint32_t, 1>{});
        if (u + 2 >= T_) break;
        step(u + 2, j, std::integral_constant<uint32_t, 2>{});
    }
}

template <int W, int ROLE>                                          // ROLE 0: g/f lanes, 1: h lanes
__device__ __forceinline__ void c3_chain(const DS &d, const uint32_t *list, uint32_t cnt, const CsrArgs &a, const CsrPlan &p,
                                         Csr3Lds &L, uint32_t T_, uint3 &out) {
    constexpr bool GF = ROLE == 0;
    typedef typename std::conditional<GF, u32x4, u32x2>::type EV;
    const uint32_t tid = threadIdx.x & (CSR_ROWS - 1), grp = tid >> 6;
    const C3Row r = c3_row(d, list, cnt, a, p, tid);
    const uint32_t myit = r.live ? r.iters : 0u;
    const uint32_t *row = csd_row(d, r.id);
    FH fh{0, 0, 0};
    uint32_t it2 = 0;
    const bool ok = cs_prologue<W>(d, r.id, r.is_row, row, fh, it2);
    uint32_t X0 = GF ? fh.g + r.ri.b0 : fh.h + r.ri.a0;             // Xg, or Xh
    uint32_t X1 = GF ? fh.f + r.ri.c0 : 0u;                         // Xf
#ifdef CSR_DIAG_STAMP
    // (diagnostic build only: shader-clock stamps of the g/f waves, summed into the diagnostic counters: 0 chain,
    // 1 waiting for the stagers, 2 codes, 3 whole loop)
    uint64_t st_[4] = {0, 0, 0, 0};
    auto stamp = [&]() -> uint64_t {
        uint64_t tt;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tt) :: "memory");
        __builtin_amdgcn_sched_barrier(0);
        return tt;
    };
#define C3_STAMP(v) const uint64_t v = stamp()
#define C3_ACC(k, x) st_[k] += (x)
#else
#define C3_STAMP(v)
#define C3_ACC(k, x)
#endif
    C3_STAMP(tl0);
    uint32_t code[CSR_SB];
    uint32_t pr = 0, pw = 0;                                         // the hand-over counters, as last read
    // super step t = 3 j + b: window and code buffer b
    auto step = [&](uint32_t t, uint32_t j, auto BC) {
        constexpr uint32_t b = decltype(BC)::value;
        const uint32_t K0 = t * CSR_SB;
        C3_STAMP(ta);
        c3_jitter(a.jitter, ROLE, t, 0);
        // this group's record stager has staged super step t, and the window stagers its window: the counters were
        // read near the end of the last super step's chain (an LDS round trip per read, 10 % of a light round's loop
        // when read here); only when they were short is there a wait, then an acquire fence for what they hand over
        if (pr < t + 1u) c3_wait(&L.readyr[grp], t + 1u);
#ifdef CSR_DIAG_SPLITWAIT
        C3_STAMP(tw);                                               // (diagnostics: slot 2 = the window's wait)
#endif
        if (pw < 4u * (j + 1u)) c3_wait(&L.readyw[b], 4u * (j + 1u));
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        C3_STAMP(tb);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 v = L.TC[b][q][tid];
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if constexpr (GF) { code[8 * q + 2 * j] = w4[j] & 0xFFFFu; code[8 * q + 2 * j + 1] = w4[j] >> 16; }
                else { code[8 * q + 2 * j] = __builtin_amdgcn_ubfe(w4[j], 1, 15); code[8 * q + 2 * j + 1] = w4[j] >> 17; }
            }
        }
        C3_STAMP(tc);
        const bool full = __all(myit == 0u || K0 + CSR_SB <= myit);
        const char *Eb = GF ? (const char *)L.EA : (const char *)L.EB;
        auto run = [&](auto FULLC) {
            constexpr bool FULL = decltype(FULLC)::value;
            EV va[CSR_PF + 1];
            auto fetch = [&](int i) { va[i % (CSR_PF + 1)] = *(const EV *)(Eb + code[i]); };
#pragma unroll
            for (int i = 0; i < CSR_PF; i++) fetch(i);
#pragma unroll
            for (int i = 0; i < CSR_SB; i++) {
                if (i + CSR_PF < CSR_SB) fetch(i + CSR_PF);
                if (i == C3_CTR_AT) {                                   // the next super step's hand-over counters
                    pr = __hip_atomic_load(&L.readyr[grp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    pw = __hip_atomic_load(&L.readyw[b == 2u ? 0u : b + 1u], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                }
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
        c3_jitter(a.jitter, ROLE, t, 1);
#ifdef C3_T_SHAREDDONE
        c3_signal(&L.done[0][b]);
        c3_signal(&L.doner[0][grp]);
#else
        c3_signal(&L.done[ROLE][b]);
        c3_signal(&L.doner[ROLE][grp]);
#endif
        C3_STAMP(td);
        C3_ACC(0, td - tc);
#ifdef CSR_DIAG_SPLITWAIT
        C3_ACC(1, tw - ta);
        C3_ACC(2, tb - tw);
#else
        C3_ACC(1, tb - ta);
#endif
#if !defined(CSR_DIAG_WINDOW) && !defined(CSR_DIAG_SPLITWAIT)
        C3_ACC(2, tc - tb);
#endif
    };
    for (uint32_t t = 0, j = 0; t < T_; t += 3, j++) {
        step(t, j, std::integral_constant<uint32_t, 0>{});
        if (t + 1 >= T_) break;
        step(t + 1, j, std::integral_constant<uint32_t, 1>{});
        if (t + 2 >= T_) break;
        step(t + 2, j, std::integral_constant<uint32_t, 2>{});
    }
    C3_STAMP(tl1);
    C3_ACC(3, tl1 - tl0);
#ifdef CSR_DIAG_STAMP
    if (GF && (threadIdx.x & 63u) == 0)
        for (int k = 0; k < 4; k++) ctr_add(d, C_NALL + k, (unsigned long long)st_[k]);
#endif
#undef C3_STAMP
#undef C3_ACC
    if constexpr (!GF) L.XH[tid] = X0;
    out = make_uint3(X0, X1, ok ? 1u : 0u);
}

// the g/f waves' epilogue, after k_csr3's barrier: the h lanes' state (XH) and the stagers' flags (FLX) are in LDS
template <int W>
__device__ __forceinline__ void c3_finish(const DS &d, const uint32_t *list, uint32_t cnt, const CsrArgs &a, const CsrPlan &p,
                                          Csr3Lds &L, uint3 X) {
    const uint32_t tid = threadIdx.x & (CSR_ROWS - 1);
    const C3Row r = c3_row(d, list, cnt, a, p, tid);
    const uint32_t fl = r.fl | L.FLX[tid];
    const bool mine = r.valid && fl == 0;
    const uint32_t nmine = (uint32_t)__popcll(__ballot(mine));
    if ((threadIdx.x & 63u) == 0 && nmine) ctr_add(d, C_X_CS_ROWS, (unsigned long long)nmine);
    if (!r.valid) return;
    if (!mine) {                                                    // left to the production kernels
        const uint32_t at = atomicAdd(a.fb_cnt, 1u);
        a.fb_list[at] = r.id;
        const uint32_t rr = (fl & CSD_F_SHORT) ? 0u : (fl & CSD_F_ECAP) ? 1u : (fl & CSR_F_PLAN) ? 2u
                          : (fl & CSR_F_RCAP) ? 3u : 4u;
        atomicAdd(a.fb_cnt + 1 + rr, 1u);
        return;
    }
    FH fh{L.XH[tid], X.x, X.y};
    const uint32_t hv = X.z ? fh.fin() : 0u;                        // (X.z: the row's string is longer than 24 bytes)
    if (r.is_row) {
        d.cs[r.id] = hv;
        d.dirty[r.id] = 0;
    } else {
        d.dense_cs[r.id - d.NL] = hv;
    }
}

template <int W>
__global__ void __launch_bounds__(4 * CSR_ROWS) k_csr3(DS d, const uint32_t *list, const uint32_t *count, CsrArgs a) {
    __shared__ Csr3Lds L;
    const uint32_t cnt = *count;
    if (blockIdx.x * CSR_ROWS >= cnt) return;
    const CsrPlan p = a.plan[blockIdx.x];
    if (threadIdx.x < 20 && ((p.phm >> threadIdx.x) & 1u)) L.phs[__popc(p.phm & ((1u << threadIdx.x) - 1u))] = threadIdx.x;
    if (threadIdx.x < C3_NB) { L.readyw[threadIdx.x] = 0; L.done[0][threadIdx.x] = 0; L.done[1][threadIdx.x] = 0; }
    if (threadIdx.x < 4) { L.readyr[threadIdx.x] = 0; L.doner[0][threadIdx.x] = 0; L.doner[1][threadIdx.x] = 0; }
    __syncthreads();
    const uint32_t T_ = p.feasible ? (p.maxit + CSR_SB - 1) / CSR_SB : 0u;
    const uint32_t role = threadIdx.x / CSR_ROWS;
    uint3 X = make_uint3(0u, 0u, 0u);
    if (role == 0) c3_chain<W, 0>(d, list, cnt, a, p, L, T_, X);
    else if (role == 1) c3_chain<W, 1>(d, list, cnt, a, p, L, T_, X);
    else if (role == 2) c3_stage(d, list, cnt, a, p, L, T_);
    else {
        c3_wstage(a, p, L, T_);
#if defined(CSR_DIAG_STAMP) && defined(CSR_DIAG_WINDOW)
        if (threadIdx.x == 3 * CSR_ROWS) {                          // (diagnostics: window geometry per super step)
            ctr_add(d, C_NALL + 2, (unsigned long long)T_);
            ctr_add(d, C_NALL + 5, (unsigned long long)T_ * p.nph * p.Wn);
            ctr_add(d, C_NALL + 7, (unsigned long long)T_ * p.nph);
        }
#endif
    }
    __syncthreads();                                                // (every role: XH and the stagers' FLX)
    if (role == 0) c3_finish<W>(d, list, cnt, a, p, L, X);
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
        hipLaunchKernelGGL((k_csr3<W>), dim3((n + CSR_ROWS - 1) / CSR_ROWS), dim3(4 * CSR_ROWS), 0, s, d, list, count, a);
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
