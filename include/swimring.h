/* swimring.h — C ABI of the MI355X consistent-hash ring.
 *
 * The ring Ringpop keeps per node and feeds from the membership changes its swim node applies
 * (ringpop.go:550-563 handleChanges: alive/suspect -> add, faulty/leave/tombstone -> remove).
 * Semantics follow hashring.HashRing (hashring/hashring.go) with hashfunc = go-farm Fingerprint32
 * and replicaPoints replicas per server (options.go:337-339 default 100):
 *   - a server's replica points are Fingerprint32(server ‖ decimal(i)), i = 0..replicaPoints-1
 *     (hashring.go:148-155); on a hash collision the point inserted first keeps it
 *     (rbtree.go:122-126), and removing a server deletes every point at its replica hashes,
 *     whoever owns them (hashring.go:182-188, rbtree Delete by value);
 *   - AddRemoveServers applies every add, then every remove, and recomputes the checksum
 *     Fingerprint32(join(sort(servers), ";")) if anything changed (hashring.go:199-229, 100-118);
 *   - Lookup(key) is the owner of the first point >= Fingerprint32(key), wrapping to the first
 *     point (hashring.go:258-301, rbtree.go:262-286); LookupN returns n distinct owners the same way.
 * Points live in HBM as one sorted array of (hash << 32 | server id). Replica hashing, ring
 * rebuilds and batched lookups are HIP kernels; the server-name table and the server set (the
 * reference's serverSet map) are host bookkeeping. Errors are negative SWIMSIM_E* codes.
 */
#ifndef SWIMRING_H
#define SWIMRING_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct swimring swimring_t;

/* hashring.New(farm.Fingerprint32, replicaPoints) (hashring.go:76-88) on device `device` */
int swimring_create(uint32_t replica_points, int32_t device, swimring_t **out);
int swimring_destroy(swimring_t *r);
const char *swimring_last_error(swimring_t *r);

/* AddRemoveServers (hashring.go:199-229). Server names are NUL-terminated; *changed = 1 if the
 * server set changed. */
int swimring_add_remove(swimring_t *r, const char *const *add, size_t nadd, const char *const *remove, size_t nremove,
                        int32_t *changed);

/* Checksum (hashring.go:90-97), ServerCount (249-255), HasServer (232-238) */
int swimring_checksum(swimring_t *r, uint32_t *out);
int swimring_server_count(swimring_t *r, uint32_t *out);
int swimring_has_server(swimring_t *r, const char *server, int32_t *out);

/* Lookup (hashring.go:258-266) for a batch of keys: key k is bytes [off[k], off[k+1]) of `keys`.
 * out[k] = the owner's server id (swimring_server_name), -1 if the ring is empty. */
int swimring_lookup_batch(swimring_t *r, const uint8_t *keys, const uint64_t *off, size_t nkeys, int32_t *out);

/* LookupN (hashring.go:268-301): up to n distinct owners of key (order not significant: the
 * reference returns them from a map) */
int swimring_lookup_n(swimring_t *r, const uint8_t *key, size_t len, uint32_t n, int32_t *out, size_t *nout);

/* server id -> name (ids are stable for the handle's lifetime) */
const char *swimring_server_name(swimring_t *r, int32_t id);

/* the ring itself, ascending: hash[i], owner id[i] (diagnostics and parity tests) */
int swimring_points(swimring_t *r, uint32_t *hash, int32_t *owner, size_t cap, size_t *n);

/* batched Fingerprint32 of byte strings on the device (the hash the ring and the membership
 * checksum share): out[k] = Fingerprint32(bytes [off[k], off[k+1])) */
int swimring_fingerprint32_batch(swimring_t *r, const uint8_t *bytes, const uint64_t *off, size_t n, uint32_t *out);

/* measurement: average ms of the last swimring_add_remove's device work and of the last lookup batch */
int swimring_last_times(swimring_t *r, double *add_remove_ms, double *lookup_ms);

#ifdef __cplusplus
}
#endif
#endif
