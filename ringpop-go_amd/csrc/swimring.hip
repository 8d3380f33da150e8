// swimring.hip — the consistent-hash ring Ringpop feeds from swim's applied changes
// (include/swimring.h states the semantics and the reference lines).
//
// HBM layout: the ring is one ascending array of u64 points (hash << 32 | server id); hashes are
// unique in it (a collision keeps the first inserter, rbtree.go:122-126). Server names live in a
// device byte pool (offset, length per id). An AddRemoveServers batch runs as:
//   k_ring_points   one lane per (added server, replica): Fingerprint32(name ‖ decimal(i)),
//                   key = hash << 32 | batch sequence (insertion order: server order, then i)
//   radix sort      by (hash, sequence)
//   k_ring_keep     keep the first point of each hash that the ring does not already hold
//   select + sort   append the kept points to the ring, sort the u64 points
//   k_ring_points   replica hashes of the removed servers (hash only), radix sort
//   k_ring_drop     drop every ring point whose hash is one of them (rbtree Delete by value)
// Lookups: one lane per key hashes it and binary-searches the ring (lower bound, wrap to 0).
#include "../../include/swimring.h"
#include "../../include/swimsim.h"
#include "swimsim_device.h"
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

using namespace swimdev;

namespace {

constexpr uint32_t RING_NAME_MAX = 240;     // longest server name a replica string is built from
constexpr uint32_t RING_STR_MAX = RING_NAME_MAX + 10;

// ---------------------------------------------------------------------------------------------
// go-farm Fingerprint32 (FarmHash-32 "mk", glide.lock:18-19), one string per lane. Bytes come from
// a per-lane buffer, so the length paths select only arithmetic.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ld32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t fmix_fh(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

__device__ uint32_t fp32_dev(const uint8_t *s, uint32_t len) {
    if (len <= 4) {                                               // Hash32Len0to4
        uint32_t b = 0, c = 9;
        for (uint32_t i = 0; i < len; i++) {
            b = b * FH_C1 + (uint32_t)(int32_t)(int8_t)s[i];
            c ^= b;
        }
        return fmix_fh(fh_mur(b, fh_mur(len, c)));
    }
    if (len <= 12) {                                              // Hash32Len5to12
        uint32_t a = len, b = len * 5, c = 9, d = b;
        a += ld32(s);
        b += ld32(s + len - 4);
        c += ld32(s + ((len >> 1) & 4));
        return fmix_fh(fh_mur(c, fh_mur(b, fh_mur(a, d))));
    }
    if (len <= 24) {                                              // Hash32Len13to24
        uint32_t a = ld32(s - 4 + (len >> 1)), b = ld32(s + 4), c = ld32(s + len - 8);
        uint32_t d = ld32(s + (len >> 1)), e = ld32(s), f = ld32(s + len - 4);
        uint32_t h = d * FH_C1 + len;
        a = ror32(a, 12) + f;
        h = fh_mur(c, h) + a;
        a = ror32(a, 3) + c;
        h = fh_mur(e, h) + a;
        a = ror32(a + f, 12) + d;
        h = fh_mur(b, h) + a;
        return fmix_fh(h);
    }
    FH fh;                                                        // len > 24: prologue, 20-byte blocks
    fh.init(len, ld32(s + len - 20), ld32(s + len - 16), ld32(s + len - 12), ld32(s + len - 8), ld32(s + len - 4));
    const uint32_t iters = (len - 1) / 20;
    for (uint32_t k = 0; k < iters; k++, s += 20)
        fh.block(ld32(s), ld32(s + 4), ld32(s + 8), ld32(s + 12), ld32(s + 16));
    return fh.fin();
}

// name ‖ decimal(i) into buf; returns its length (fmt.Sprintf("%s%v", server, i), hashring.go:151)
__device__ __forceinline__ uint32_t replica_string(const uint8_t *name, uint32_t nlen, uint32_t i, uint8_t *buf) {
    for (uint32_t k = 0; k < nlen; k++) buf[k] = name[k];
    uint8_t dig[10];
    uint32_t nd = 0;
    do { dig[nd++] = (uint8_t)('0' + i % 10u); i /= 10u; } while (i);
    for (uint32_t k = 0; k < nd; k++) buf[nlen + k] = dig[nd - 1 - k];
    return nlen + nd;
}

// one lane per (server of the batch, replica): keys[j] = hash << 32 | j, vals[j] = server id
__global__ void k_ring_points(const uint8_t *names, const uint64_t *noff, const uint32_t *nlen, const int32_t *ids,
                              uint32_t nsrv, uint32_t R, unsigned long long *keys, uint32_t *vals) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nsrv * R) return;
    const uint32_t k = j / R, i = j - k * R;
    const int32_t id = ids[k];
    uint8_t buf[RING_STR_MAX + 4];
    const uint32_t len = replica_string(names + noff[id], nlen[id], i, buf);
    buf[len] = buf[len + 1] = buf[len + 2] = buf[len + 3] = 0;
    keys[j] = ((unsigned long long)fp32_dev(buf, len) << 32) | j;
    vals[j] = (uint32_t)id;
}

__device__ __forceinline__ uint32_t lower_bound_u64(const unsigned long long *a, uint32_t n, unsigned long long x) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ bool ring_has(const unsigned long long *ring, uint32_t P, uint32_t h) {
    const uint32_t p = lower_bound_u64(ring, P, (unsigned long long)h << 32);
    return p < P && (uint32_t)(ring[p] >> 32) == h;
}

// sorted new points: keep the first of each hash unless the ring already has it; out = hash << 32 | id
__global__ void k_ring_keep(const unsigned long long *skeys, const uint32_t *svals, uint32_t n,
                            const unsigned long long *ring, uint32_t P, uint8_t *flag, unsigned long long *out) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t h = (uint32_t)(skeys[j] >> 32);
    const bool first = j == 0 || (uint32_t)(skeys[j - 1] >> 32) != h;
    flag[j] = first && !ring_has(ring, P, h) ? 1 : 0;
    out[j] = ((unsigned long long)h << 32) | svals[j];
}

// ring points whose hash is a removed server's replica hash are dropped (sorted delete keys)
__global__ void k_ring_drop(const unsigned long long *ring, uint32_t P, const unsigned long long *dkeys, uint32_t nd,
                            uint8_t *flag) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const uint32_t h = (uint32_t)(ring[p] >> 32);
    const uint32_t q = lower_bound_u64(dkeys, nd, (unsigned long long)h << 32);
    flag[p] = (q < nd && (uint32_t)(dkeys[q] >> 32) == h) ? 0 : 1;
}

__global__ void k_fp32_batch(const uint8_t *bytes, const uint64_t *off, uint32_t n, uint32_t *out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint64_t a = off[k], len = off[k + 1] - a;
    out[k] = fp32_dev(bytes + a, (uint32_t)len);                  // the ld32 tail reads stay inside the
}                                                                 // padded byte buffer

// Lookup: owner of the first point >= Fingerprint32(key), wrapping to the first point
__global__ void k_ring_lookup(const uint8_t *bytes, const uint64_t *off, uint32_t n, const unsigned long long *ring,
                              uint32_t P, int32_t *out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    if (P == 0) { out[k] = -1; return; }
    const uint64_t a = off[k];
    const uint32_t h = fp32_dev(bytes + a, (uint32_t)(off[k + 1] - a));
    uint32_t p = lower_bound_u64(ring, P, (unsigned long long)h << 32);
    if (p == P) p = 0;
    out[k] = (int32_t)(uint32_t)ring[p];
}

// LookupN: distinct owners walking up from the key's hash, then from 0 (rbtree.go:262-286). One workgroup:
// its threads clear a seen-bitmap over server ids, then one lane walks the ring (O(P) at worst, one bit test
// per point; the order of first occurrences decides which n owners are taken)
__global__ void k_ring_lookup_n(const uint8_t *key, uint32_t len, const unsigned long long *ring, uint32_t P, uint32_t n,
                                int32_t *out, uint32_t *nout, uint32_t *seen, uint32_t seen_words) {
    if (blockIdx.x) return;
    for (uint32_t i = threadIdx.x; i < seen_words; i += blockDim.x) seen[i] = 0;
    __syncthreads();
    if (threadIdx.x) return;
    uint32_t got = 0;
    const uint32_t h = fp32_dev(key, len);
    const uint32_t start = lower_bound_u64(ring, P, (unsigned long long)h << 32);
    for (int pass = 0; pass < 2 && got < n; pass++) {
        for (uint32_t p = pass ? 0 : start; p < P && got < n; p++) {
            const uint32_t o = (uint32_t)ring[p];
            const uint32_t bit = 1u << (o & 31);
            if (seen[o >> 5] & bit) continue;
            seen[o >> 5] |= bit;
            out[got++] = (int32_t)o;
        }
    }
    *nout = got;
}

uint32_t grid_for(uint64_t n) { return (uint32_t)std::max<uint64_t>(1, (n + 255) / 256); }

}  // namespace

struct swimring {
    uint32_t R = 100;
    int device = 0;
    hipStream_t s = nullptr;
    std::string err;
    // server table (host) and its device copy
    std::unordered_map<std::string, int32_t> ids;
    std::vector<std::string> names;
    std::vector<uint8_t> in_set;
    uint32_t nset = 0;
    uint8_t *dnames = nullptr;
    uint64_t *dnoff = nullptr;
    uint32_t *dnlen = nullptr;
    size_t names_bytes_dev = 0, names_cap = 0, ids_cap = 0, ids_dev = 0;
    std::vector<uint64_t> hnoff;
    std::vector<uint32_t> hnlen;
    // ring
    unsigned long long *ring = nullptr, *ring2 = nullptr;
    uint32_t *seen = nullptr;                                     // LookupN's seen-bitmap over server ids
    size_t seen_cap = 0;
    uint32_t P = 0;
    size_t ring_cap = 0;
    uint32_t checksum = 0;
    // scratch
    unsigned long long *k0 = nullptr, *k1 = nullptr, *kept = nullptr;
    uint32_t *v0 = nullptr, *v1 = nullptr, *nsel = nullptr;
    uint8_t *flag = nullptr;
    int32_t *bid = nullptr;
    size_t scr_cap = 0, bid_cap = 0;
    void *cub = nullptr;
    size_t cub_cap = 0;
    uint8_t *bytes = nullptr;
    uint64_t *boff = nullptr;
    size_t bytes_cap = 0, boff_cap = 0;
    int32_t *iout = nullptr;
    uint32_t *uout = nullptr;
    size_t out_cap = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    double t_add = 0, t_look = 0;

    int fail(int code, const char *fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
};

#define RCHK(r, x)                                                                               \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) return (r)->fail(SWIMSIM_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

namespace {

template <typename T>
int grow(swimring *r, T **p, size_t *cap, size_t need, bool keep = false, size_t keep_elems = 0) {
    if (need <= *cap) return 0;
    size_t c = std::max<size_t>(need + need / 2, 1024);
    T *q = nullptr;
    if (hipMalloc(&q, c * sizeof(T)) != hipSuccess) return r->fail(SWIMSIM_ENOMEM, "hipMalloc(%zu bytes)", c * sizeof(T));
    if (keep && *p && keep_elems)
        if (hipMemcpyAsync(q, *p, keep_elems * sizeof(T), hipMemcpyDeviceToDevice, r->s) != hipSuccess)
            return r->fail(SWIMSIM_EHIP, "ring copy");
    if (*p) {
        hipStreamSynchronize(r->s);
        hipFree(*p);
    }
    *p = q;
    *cap = c;
    return 0;
}

int intern(swimring *r, const char *s, int32_t *id) {
    auto it = r->ids.find(s);
    if (it != r->ids.end()) { *id = it->second; return 0; }
    const size_t len = strlen(s);
    if (len > RING_NAME_MAX) return r->fail(SWIMSIM_EINVAL, "server name longer than %u bytes", RING_NAME_MAX);
    *id = (int32_t)r->names.size();
    r->ids.emplace(s, *id);
    r->names.emplace_back(s);
    r->in_set.push_back(0);
    r->hnoff.push_back(r->hnoff.empty() ? 0 : r->hnoff.back() + r->hnlen.back());
    r->hnlen.push_back((uint32_t)len);
    return 0;
}

// upload server names interned since the last upload (append-only)
int sync_names(swimring *r) {
    const size_t n = r->names.size();
    if (n == r->ids_dev) return 0;
    const size_t total = r->hnoff.back() + r->hnlen.back();
    size_t cap = r->names_cap;
    if (int rc = grow(r, &r->dnames, &cap, total + 8, true, r->names_bytes_dev)) return rc;
    r->names_cap = cap;
    size_t icap = r->ids_cap, icap2 = r->ids_cap;
    if (int rc = grow(r, &r->dnoff, &icap, n, true, r->ids_dev)) return rc;
    if (int rc = grow(r, &r->dnlen, &icap2, n, true, r->ids_dev)) return rc;
    r->ids_cap = icap;
    std::string blob;
    for (size_t i = r->ids_dev; i < n; i++) blob += r->names[i];
    const size_t b0 = r->names_bytes_dev;
    if (!blob.empty()) RCHK(r, hipMemcpyAsync(r->dnames + b0, blob.data(), blob.size(), hipMemcpyHostToDevice, r->s));
    RCHK(r, hipMemcpyAsync(r->dnoff + r->ids_dev, r->hnoff.data() + r->ids_dev, (n - r->ids_dev) * 8, hipMemcpyHostToDevice, r->s));
    RCHK(r, hipMemcpyAsync(r->dnlen + r->ids_dev, r->hnlen.data() + r->ids_dev, (n - r->ids_dev) * 4, hipMemcpyHostToDevice, r->s));
    RCHK(r, hipStreamSynchronize(r->s));                         // the blob is a host temporary
    r->names_bytes_dev = total;
    r->ids_dev = n;
    return 0;
}

int ensure_scratch(swimring *r, size_t n) {
    size_t c;
    c = r->scr_cap; if (int rc = grow(r, &r->k0, &c, n)) return rc;
    c = r->scr_cap; if (int rc = grow(r, &r->k1, &c, n)) return rc;
    c = r->scr_cap; if (int rc = grow(r, &r->kept, &c, n)) return rc;
    c = r->scr_cap; if (int rc = grow(r, &r->v0, &c, n)) return rc;
    c = r->scr_cap; if (int rc = grow(r, &r->v1, &c, n)) return rc;
    c = r->scr_cap; if (int rc = grow(r, &r->flag, &c, n)) return rc;
    r->scr_cap = std::max(r->scr_cap, c);
    return 0;
}

int ensure_cub(swimring *r, size_t bytes) {
    size_t c = r->cub_cap;
    if (int rc = grow(r, (uint8_t **)&r->cub, &c, bytes)) return rc;
    r->cub_cap = c;
    return 0;
}

// replica points of the listed servers, sorted by (hash, insertion sequence) into k1 / v1
int hash_replicas(swimring *r, const std::vector<int32_t> &list) {
    const size_t n = list.size() * r->R;
    if (int rc = ensure_scratch(r, n)) return rc;
    size_t c = r->bid_cap;
    if (int rc = grow(r, &r->bid, &c, list.size())) return rc;
    r->bid_cap = c;
    RCHK(r, hipMemcpyAsync(r->bid, list.data(), list.size() * 4, hipMemcpyHostToDevice, r->s));
    hipLaunchKernelGGL(k_ring_points, dim3(grid_for(n)), dim3(256), 0, r->s, r->dnames, r->dnoff, r->dnlen, r->bid,
                       (uint32_t)list.size(), r->R, r->k0, r->v0);
    size_t tb = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, tb, r->k0, r->k1, r->v0, r->v1, (int)n, 0, 64, r->s);
    if (int rc = ensure_cub(r, tb)) return rc;
    RCHK(r, hipcub::DeviceRadixSort::SortPairs(r->cub, tb, r->k0, r->k1, r->v0, r->v1, (int)n, 0, 64, r->s));
    RCHK(r, hipStreamSynchronize(r->s));                         // list is a host temporary
    return 0;
}

int upload_keys(swimring *r, const uint8_t *keys, const uint64_t *off, size_t nkeys) {
    const size_t nb = off[nkeys];
    size_t c = r->bytes_cap;
    if (int rc = grow(r, &r->bytes, &c, nb + 8)) return rc;
    r->bytes_cap = c;
    c = r->boff_cap;
    if (int rc = grow(r, &r->boff, &c, nkeys + 1)) return rc;
    r->boff_cap = c;
    c = r->out_cap;
    size_t c2 = r->out_cap;
    if (int rc = grow(r, &r->iout, &c, std::max<size_t>(nkeys, 64))) return rc;
    if (int rc = grow(r, &r->uout, &c2, std::max<size_t>(nkeys, 64))) return rc;
    r->out_cap = c;
    if (nb) RCHK(r, hipMemcpyAsync(r->bytes, keys, nb, hipMemcpyHostToDevice, r->s));
    RCHK(r, hipMemsetAsync(r->bytes + nb, 0, 8, r->s));
    RCHK(r, hipMemcpyAsync(r->boff, off, (nkeys + 1) * 8, hipMemcpyHostToDevice, r->s));
    return 0;
}

int compute_checksum(swimring *r) {
    std::vector<const std::string *> v;
    for (size_t i = 0; i < r->names.size(); i++)
        if (r->in_set[i]) v.push_back(&r->names[i]);
    std::sort(v.begin(), v.end(), [](const std::string *a, const std::string *b) { return *a < *b; });
    std::string joined;
    for (size_t i = 0; i < v.size(); i++) {
        if (i) joined += ';';
        joined += *v[i];
    }
    const uint64_t off[2] = {0, joined.size()};
    if (int rc = upload_keys(r, (const uint8_t *)joined.data(), off, 1)) return rc;
    hipLaunchKernelGGL(k_fp32_batch, dim3(1), dim3(64), 0, r->s, r->bytes, r->boff, 1u, r->uout);
    RCHK(r, hipMemcpyAsync(&r->checksum, r->uout, 4, hipMemcpyDeviceToHost, r->s));
    RCHK(r, hipStreamSynchronize(r->s));
    return 0;
}

}  // namespace

extern "C" {

int swimring_create(uint32_t replica_points, int32_t device, swimring_t **out) {
    if (!out || replica_points == 0) return SWIMSIM_EINVAL;
    *out = nullptr;
    swimring *r = new swimring;
    r->R = replica_points;
    r->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&r->s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&r->e0) != hipSuccess || hipEventCreate(&r->e1) != hipSuccess) {
        delete r;
        return SWIMSIM_EHIP;
    }
    *out = r;                                                     // checksum 0 until the first change (Go zero value)
    return SWIMSIM_OK;
}

int swimring_destroy(swimring_t *r) {
    if (!r) return SWIMSIM_OK;
    if (r->s) hipStreamSynchronize(r->s);
    void *bufs[] = {r->dnames, r->dnoff, r->dnlen, r->ring, r->ring2, r->k0, r->k1, r->kept, r->v0, r->v1, r->nsel,
                    r->flag, r->bid, r->cub, r->bytes, r->boff, r->iout, r->uout, r->seen};
    for (void *p : bufs)
        if (p) hipFree(p);
    if (r->e0) hipEventDestroy(r->e0);
    if (r->e1) hipEventDestroy(r->e1);
    if (r->s) hipStreamDestroy(r->s);
    delete r;
    return SWIMSIM_OK;
}

const char *swimring_last_error(swimring_t *r) { return r ? r->err.c_str() : "null handle"; }

// the device half of AddRemoveServers: hash and insert the added servers' points, then drop the removed
// servers' points. *adds_done tells a failing caller whether the adds reached the ring
static int ring_apply(swimring *r, const std::vector<int32_t> &A, const std::vector<int32_t> &D, bool *adds_done) {
    RCHK(r, hipEventRecord(r->e0, r->s));
    size_t c;
    if (!A.empty()) {
        if (int rc = hash_replicas(r, A)) return rc;
        const uint32_t n = (uint32_t)(A.size() * r->R);
        hipLaunchKernelGGL(k_ring_keep, dim3(grid_for(n)), dim3(256), 0, r->s, r->k1, r->v1, n, r->ring, r->P, r->flag,
                           r->kept);
        c = r->ring_cap;
        const size_t need = (size_t)r->P + n;
        size_t c2 = r->ring_cap;
        if (int rc = grow(r, &r->ring, &c, need, true, r->P)) return rc;
        if (int rc = grow(r, &r->ring2, &c2, need)) return rc;
        r->ring_cap = std::min(c, c2);
        if (!r->nsel) RCHK(r, hipMalloc(&r->nsel, 16));
        size_t tb = 0;
        hipcub::DeviceSelect::Flagged(nullptr, tb, r->kept, r->flag, r->ring + r->P, r->nsel, (int)n, r->s);
        if (int rc = ensure_cub(r, tb)) return rc;
        RCHK(r, hipcub::DeviceSelect::Flagged(r->cub, tb, r->kept, r->flag, r->ring + r->P, r->nsel, (int)n, r->s));
        uint32_t nk = 0;
        RCHK(r, hipMemcpyAsync(&nk, r->nsel, 4, hipMemcpyDeviceToHost, r->s));
        RCHK(r, hipStreamSynchronize(r->s));
        const uint32_t P2 = r->P + nk;
        tb = 0;
        hipcub::DeviceRadixSort::SortKeys(nullptr, tb, r->ring, r->ring2, (int)P2, 0, 64, r->s);
        if (int rc = ensure_cub(r, tb)) return rc;
        RCHK(r, hipcub::DeviceRadixSort::SortKeys(r->cub, tb, r->ring, r->ring2, (int)P2, 0, 64, r->s));
        std::swap(r->ring, r->ring2);
        r->P = P2;
    }
    *adds_done = true;
    if (!D.empty() && r->P) {
        const uint32_t nd = (uint32_t)(D.size() * r->R);
        if (int rc = ensure_scratch(r, std::max<size_t>(r->P, nd))) return rc;   // before k1 is filled
        if (int rc = hash_replicas(r, D)) return rc;
        hipLaunchKernelGGL(k_ring_drop, dim3(grid_for(r->P)), dim3(256), 0, r->s, r->ring, r->P, r->k1, nd, r->flag);
        if (!r->nsel) RCHK(r, hipMalloc(&r->nsel, 16));
        size_t tb = 0;
        hipcub::DeviceSelect::Flagged(nullptr, tb, r->ring, r->flag, r->ring2, r->nsel, (int)r->P, r->s);
        if (int rc = ensure_cub(r, tb)) return rc;
        RCHK(r, hipcub::DeviceSelect::Flagged(r->cub, tb, r->ring, r->flag, r->ring2, r->nsel, (int)r->P, r->s));
        uint32_t nk = 0;
        RCHK(r, hipMemcpyAsync(&nk, r->nsel, 4, hipMemcpyDeviceToHost, r->s));
        RCHK(r, hipStreamSynchronize(r->s));
        std::swap(r->ring, r->ring2);
        r->P = nk;
    }
    RCHK(r, hipEventRecord(r->e1, r->s));
    RCHK(r, hipEventSynchronize(r->e1));
    float ms = 0;
    hipEventElapsedTime(&ms, r->e0, r->e1);
    r->t_add = ms;
    return 0;
}

int swimring_add_remove(swimring_t *r, const char *const *add, size_t nadd, const char *const *remove, size_t nremove,
                        int32_t *changed) {
    if (!r || (nadd && !add) || (nremove && !remove)) return SWIMSIM_EINVAL;
    if (changed) *changed = 0;
    // every name is checked and interned before the server set changes, so a bad name leaves the ring as
    // it was; a HIP failure further down rolls the set back to the servers the device ring holds
    for (size_t i = 0; i < nadd; i++)
        if (!add[i] || strlen(add[i]) > RING_NAME_MAX) return r->fail(SWIMSIM_EINVAL, "bad server name in the add list");
    for (size_t i = 0; i < nremove; i++)
        if (!remove[i]) return SWIMSIM_EINVAL;
    std::vector<int32_t> aid(nadd);
    for (size_t i = 0; i < nadd; i++)
        if (int rc = intern(r, add[i], &aid[i])) return rc;
    std::vector<int32_t> A, D;
    for (size_t i = 0; i < nadd; i++) {                          // addServerNoLock: skip servers in the set
        const int32_t id = aid[i];
        if (r->in_set[id]) continue;
        r->in_set[id] = 1;
        r->nset++;
        A.push_back(id);
    }
    for (size_t i = 0; i < nremove; i++) {                       // removeServerNoLock: skip unknown ones
        auto it = r->ids.find(remove[i]);
        if (it == r->ids.end() || !r->in_set[it->second]) continue;
        r->in_set[it->second] = 0;
        r->nset--;
        D.push_back(it->second);
    }
    if (A.empty() && D.empty()) return SWIMSIM_OK;
    if (changed) *changed = 1;
    auto undo = [&](bool adds, int rc) {
        if (adds)
            for (int32_t id : A) { r->in_set[id] = 0; r->nset--; }
        for (int32_t id : D) { r->in_set[id] = 1; r->nset++; }
        if (changed) *changed = 0;
        return rc;
    };
    if (int rc = sync_names(r)) return undo(true, rc);
    bool adds_done = false;
    if (int rc = ring_apply(r, A, D, &adds_done)) return undo(!adds_done, rc);
    return compute_checksum(r);
}

int swimring_checksum(swimring_t *r, uint32_t *out) {
    if (!r || !out) return SWIMSIM_EINVAL;
    *out = r->checksum;
    return SWIMSIM_OK;
}

int swimring_server_count(swimring_t *r, uint32_t *out) {
    if (!r || !out) return SWIMSIM_EINVAL;
    *out = r->nset;
    return SWIMSIM_OK;
}

int swimring_has_server(swimring_t *r, const char *server, int32_t *out) {
    if (!r || !server || !out) return SWIMSIM_EINVAL;
    auto it = r->ids.find(server);
    *out = it != r->ids.end() && r->in_set[it->second] ? 1 : 0;
    return SWIMSIM_OK;
}

int swimring_lookup_batch(swimring_t *r, const uint8_t *keys, const uint64_t *off, size_t nkeys, int32_t *out) {
    if (!r || !off || !out || (nkeys && !keys && off[nkeys])) return SWIMSIM_EINVAL;
    if (nkeys == 0) return SWIMSIM_OK;
    if (int rc = upload_keys(r, keys, off, nkeys)) return rc;
    RCHK(r, hipEventRecord(r->e0, r->s));
    hipLaunchKernelGGL(k_ring_lookup, dim3(grid_for(nkeys)), dim3(256), 0, r->s, r->bytes, r->boff, (uint32_t)nkeys,
                       r->ring, r->P, r->iout);
    RCHK(r, hipEventRecord(r->e1, r->s));
    RCHK(r, hipMemcpyAsync(out, r->iout, nkeys * 4, hipMemcpyDeviceToHost, r->s));
    RCHK(r, hipStreamSynchronize(r->s));
    float ms = 0;
    hipEventElapsedTime(&ms, r->e0, r->e1);
    r->t_look = ms;
    return SWIMSIM_OK;
}

int swimring_lookup_n(swimring_t *r, const uint8_t *key, size_t len, uint32_t n, int32_t *out, size_t *nout) {
    if (!r || (len && !key) || !out || !nout) return SWIMSIM_EINVAL;
    *nout = 0;
    if (n >= r->nset) {                                          // lookupNNoLock: every server
        for (size_t i = 0; i < r->names.size(); i++)
            if (r->in_set[i]) out[(*nout)++] = (int32_t)i;
        return SWIMSIM_OK;
    }
    if (n == 0) return SWIMSIM_OK;
    const uint64_t off[2] = {0, len};
    if (int rc = upload_keys(r, key, off, 1)) return rc;
    size_t c = r->out_cap, c2 = r->out_cap;
    if (int rc = grow(r, &r->iout, &c, n)) return rc;
    if (int rc = grow(r, &r->uout, &c2, n)) return rc;
    r->out_cap = std::min(c, c2);
    const size_t words = (r->names.size() + 31) / 32;
    if (words > r->seen_cap) {
        if (r->seen) hipFree(r->seen);
        r->seen = nullptr;
        r->seen_cap = 0;
        RCHK(r, hipMalloc(&r->seen, std::max<size_t>(words, 64) * 4));
        r->seen_cap = std::max<size_t>(words, 64);
    }
    hipLaunchKernelGGL(k_ring_lookup_n, dim3(1), dim3(256), 0, r->s, r->bytes, (uint32_t)len, r->ring, r->P, n, r->iout,
                       r->uout, r->seen, (uint32_t)words);
    uint32_t got = 0;
    RCHK(r, hipMemcpyAsync(&got, r->uout, 4, hipMemcpyDeviceToHost, r->s));
    RCHK(r, hipStreamSynchronize(r->s));
    RCHK(r, hipMemcpyAsync(out, r->iout, (size_t)got * 4, hipMemcpyDeviceToHost, r->s));
    RCHK(r, hipStreamSynchronize(r->s));
    *nout = got;
    return SWIMSIM_OK;
}

const char *swimring_server_name(swimring_t *r, int32_t id) {
    if (!r || id < 0 || (size_t)id >= r->names.size()) return nullptr;
    return r->names[id].c_str();
}

int swimring_points(swimring_t *r, uint32_t *hash, int32_t *owner, size_t cap, size_t *n) {
    if (!r || !n) return SWIMSIM_EINVAL;
    *n = r->P;
    if (!hash && !owner) return SWIMSIM_OK;
    std::vector<unsigned long long> h(r->P);
    if (r->P) RCHK(r, hipMemcpyAsync(h.data(), r->ring, (size_t)r->P * 8, hipMemcpyDeviceToHost, r->s));
    RCHK(r, hipStreamSynchronize(r->s));
    for (size_t i = 0; i < h.size() && i < cap; i++) {
        if (hash) hash[i] = (uint32_t)(h[i] >> 32);
        if (owner) owner[i] = (int32_t)(uint32_t)h[i];
    }
    return SWIMSIM_OK;
}

int swimring_fingerprint32_batch(swimring_t *r, const uint8_t *bytes, const uint64_t *off, size_t n, uint32_t *out) {
    if (!r || !off || !out) return SWIMSIM_EINVAL;
    if (n == 0) return SWIMSIM_OK;
    if (int rc = upload_keys(r, bytes, off, n)) return rc;
    hipLaunchKernelGGL(k_fp32_batch, dim3(grid_for(n)), dim3(256), 0, r->s, r->bytes, r->boff, (uint32_t)n, r->uout);
    RCHK(r, hipMemcpyAsync(out, r->uout, n * 4, hipMemcpyDeviceToHost, r->s));
    RCHK(r, hipStreamSynchronize(r->s));
    return SWIMSIM_OK;
}

int swimring_last_times(swimring_t *r, double *add_remove_ms, double *lookup_ms) {
    if (!r) return SWIMSIM_EINVAL;
    if (add_remove_ms) *add_remove_ms = r->t_add;
    if (lookup_ms) *lookup_ms = r->t_look;
    return SWIMSIM_OK;
}

}  // extern "C"
