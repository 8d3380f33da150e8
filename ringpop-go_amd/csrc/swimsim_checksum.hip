// swimsim_checksum.hip — phase C: the membership checksum (memberlist.go:83-128), i.e. go-farm
// Fingerprint32 = FarmHash-32 "mk" over addr ‖ status ‖ decimal(inc) ‖ ';' of every non-tombstone
// member in index order. Fixed-width ascending addresses make the sorted order the index order, so
// the string is generated on the fly and never sorted. Included by swimsim_kernels.hip.
//
// The FarmHash chain is sequential within a row, so a row's hash is one lane's (or one lane quad's) work and a
// launch's latency is at least one row's chain (≈1.9 blocks of 20 bytes per member). Two production kernels:
//   k_checksum3    (swimsim_checksum3.hip): launches of many rows, 64 rows per workgroup (lane = row), a
//                  formatter wave and a hasher wave;
//   k_checksum_q16 (swimsim_checksum4.hip): launches of at most CS_NARROW_ROWS rows (latency-bound), 16 rows per
//                  workgroup, the chain in carried-sum form on lane quads fed by premix and formatter waves.
// Superseded kernels (the 4-wave k_checksum, k_checksum_n16, k_checksum2) and every diagnostic variant live in
// tools/diag/swimsim_checksum_diag.hip and are compiled only into the diagnostics library
// (make -C ringpop-go_amd diag -> tools/libswimsim_diag.so), never into libswimsim.so.
// The string length and the last included member (the FarmHash-mk prologue hashes the last 20
// bytes before the chain) come from per-row values kept current by the merges.

#include <type_traits>

// address widths the checksum kernels are instantiated for (W = 13..20 bytes; a development build with
// -DSWIMSIM_DEV_W19 compiles W = 19 only, the workloads' width, in a third of the time)
#ifdef SWIMSIM_DEV_W19
#define CS_W_CASES(X) X(19)
#else
#define CS_W_CASES(X) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20)
#endif

constexpr int CS_ROWS = 64;                     // rows per workgroup of the wide kernel
constexpr int CS_PRE = 12;                      // spill area in front of a row's ring (narrow kernel)
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

// narrow kernel geometry (swimsim_checksum4.hip): 16 rows per workgroup, ring words [0, CN_MIR) mirrored behind
// the ring end
constexpr int CN_ROWS = 16;
constexpr int CN_MIR = 20;

// wide kernel geometry (swimsim_checksum3.hip)
constexpr int C2_ROWS = 64;
constexpr int C2_IT = 4;                         // members per step
// for records of at most RMAX bytes: blocks one step can complete, words per buffer per lane (the last record
// of a step starts at most 19 + 3 * RMAX bytes past the buffer's base and writes NO words)
constexpr int c2_nb(int rmax) { return (19 + C2_IT * rmax) / 20; }
constexpr int c2_bw(int rmax, int no) {     // and every hasher / carry read of NB blocks stays inside
    return (19 + (C2_IT - 1) * rmax) / 4 + no + 1 > 5 * c2_nb(rmax) + 5 ? (19 + (C2_IT - 1) * rmax) / 4 + no + 1
                                                                       : 5 * c2_nb(rmax) + 5;
}

// NO for the address width W and the longest record tail of the handle's incarnation table
constexpr int cs_no(int W, int maxtail) { return (3 + W + maxtail + 3) / 4; }

#include "swimsim_checksum3.hip"
#include "swimsim_checksum4.hip"
#include "swimsim_checksum_ref.hip"
#include "swimsim_checksum_csr.hip"
#ifdef SWIMSIM_DIAG                            // tools/diag (diagnostics library only): the reference-row path
#include "swimsim_checksum_delta.hip"          // (off by default in round 3, not a win over the cascade), the 3-wave
#include "swimsim_checksum5.hip"               // and fast-path experiments and every superseded kernel
#include "swimsim_checksum6.hip"
#include "swimsim_checksum_diag.hip"
#endif

// up to CS_NARROW_ROWS rows (measured crossover) the launch is latency-bound: k_checksum_q16 (16 rows per
// workgroup; 16 records per step up to 4,096 rows, 8 above); above, the 64-row throughput kernel k_checksum3
constexpr uint32_t CS_NARROW_ROWS = 8192;
// phase-C launches of at most CS_ASYNC_ROWS rows (after dedup) run on the side stream, overlapping the next round
// (swimsim_engine.hip checksum_dirty); the kernel is still chosen by row count
constexpr uint32_t CS_ASYNC_ROWS = 12288;
static uint32_t g_csq16_groups = 256;                  // q16 row groups up to which 16 records per step are used

enum CsKind { CS_NONE = 0, CS_WIDE = 1, CS_NARROW = 2 };

// which production kernel a launch of n rows uses (narrow_rows: the handle's crossover, swimsim_tuning)
inline CsKind cs_kind(uint32_t n, uint32_t narrow_rows = CS_NARROW_ROWS) {
    return n == 0 ? CS_NONE : n <= narrow_rows ? CS_NARROW : CS_WIDE;
}

// one launch of the production kernel `kind` over the listed rows (count on the device; n = at most that many)
void launch_checksum_kind(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t n, CsKind kind, hipStream_t s) {
    if (kind == CS_WIDE) {
        const uint32_t grid = (n + CS_ROWS - 1) / CS_ROWS;
        switch (d.W) {
#define CS_CASE(Wv) case Wv: launch_cs3_w<Wv>(d, list, count, grid, s); break;
            CS_W_CASES(CS_CASE)
#undef CS_CASE
        default: break;
        }
    } else if (kind == CS_NARROW) {
        const uint32_t ngrid = (n + CN_ROWS - 1) / CN_ROWS;
        switch (d.W) {
#define CS_CASE(Wv)                                                                         \
    case Wv:                                                                                \
        if (ngrid <= g_csq16_groups) launch_csq_w<Wv, 16>(d, list, count, ngrid, s);        \
        else launch_csq_w<Wv, 8>(d, list, count, ngrid, s);                                 \
        break;
            CS_W_CASES(CS_CASE)
#undef CS_CASE
        default: break;
        }
    }
}

// the wide kernel with 4 row groups per workgroup and SIMD-placed roles (k_checksum3<..., G = 4>)
void launch_checksum_wide4(const DS &d, const uint32_t *list, const uint32_t *count, uint32_t n, hipStream_t s) {
    const uint32_t grid = (n + 4 * CS_ROWS - 1) / (4 * CS_ROWS);
    switch (d.W) {
#define CS_CASE(Wv) case Wv: launch_cs3_w<Wv, 0, 4>(d, list, count, grid, s); break;
        CS_W_CASES(CS_CASE)
#undef CS_CASE
    default: break;
    }
}


