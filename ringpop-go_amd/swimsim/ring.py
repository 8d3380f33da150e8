"""HashRing: the consistent-hash ring Ringpop feeds from swim's applied changes, on the MI355X
(include/swimring.h, csrc/swimring.hip). The method names and meanings follow hashring.HashRing
(hashring/hashring.go): AddServer / RemoveServer / AddRemoveServers / Checksum / HasServer /
ServerCount / Servers / Lookup / LookupN. There is no CPU path: the ring lives in HBM and every
hash, rebuild and lookup runs as a HIP kernel of libswimsim.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import SwimsimError, load_library, ERRORS, ALIVE, SUSPECT

_ring_sigs_done = False


def _lib():
    global _ring_sigs_done
    L = load_library()
    if not _ring_sigs_done:
        P, u32, i32, sz = C.c_void_p, C.c_uint32, C.c_int32, C.c_size_t
        sigs = {
            "swimring_create": (C.c_int, [u32, i32, C.POINTER(P)]),
            "swimring_destroy": (C.c_int, [P]),
            "swimring_last_error": (C.c_char_p, [P]),
            "swimring_add_remove": (C.c_int, [P, P, sz, P, sz, C.POINTER(i32)]),
            "swimring_checksum": (C.c_int, [P, C.POINTER(u32)]),
            "swimring_server_count": (C.c_int, [P, C.POINTER(u32)]),
            "swimring_has_server": (C.c_int, [P, C.c_char_p, C.POINTER(i32)]),
            "swimring_lookup_batch": (C.c_int, [P, P, P, sz, P]),
            "swimring_lookup_n": (C.c_int, [P, C.c_char_p, sz, u32, P, C.POINTER(sz)]),
            "swimring_server_name": (C.c_char_p, [P, i32]),
            "swimring_points": (C.c_int, [P, P, P, sz, C.POINTER(sz)]),
            "swimring_fingerprint32_batch": (C.c_int, [P, P, P, sz, P]),
            "swimring_last_times": (C.c_int, [P, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
        }
        for name, (res, args) in sigs.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _ring_sigs_done = True
    return L


def _pack(keys):
    bs = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
    off = np.zeros(len(bs) + 1, np.uint64)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs])
    blob = b"".join(bs)
    return blob, off


class HashRing:
    """hashring.New(farm.Fingerprint32, replica_points) (hashring.go:76-88) on GPU `device`."""

    def __init__(self, replica_points: int = 100, device: int = 0):
        self.h = C.c_void_p()
        rc = _lib().swimring_create(replica_points, device, C.byref(self.h))
        if rc < 0:
            raise SwimsimError(f"swimring_create: {ERRORS.get(rc, rc)}")
        self.replica_points = replica_points

    def _chk(self, rc):
        if rc < 0:
            raise SwimsimError(f"{ERRORS.get(rc, rc)}: {_lib().swimring_last_error(self.h).decode()}")
        return rc

    def close(self):
        if self.h:
            _lib().swimring_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- mutation (hashring.go:121-229) ----
    def add_remove_servers(self, add=(), remove=()) -> bool:
        a = [s.encode() for s in add]
        r = [s.encode() for s in remove]
        aa = (C.c_char_p * max(1, len(a)))(*a)
        rr = (C.c_char_p * max(1, len(r)))(*r)
        changed = C.c_int32()
        self._chk(_lib().swimring_add_remove(self.h, aa, len(a), rr, len(r), C.byref(changed)))
        return bool(changed.value)

    def add_server(self, server: str) -> bool:
        return self.add_remove_servers([server], [])

    def remove_server(self, server: str) -> bool:
        return self.add_remove_servers([], [server])

    def sync_from_row(self, status, address) -> bool:
        """Ringpop.handleChanges (ringpop.go:550-563) for a whole membership row: members alive or
        suspect are servers, every other status is not. Adds and removes go in member-index order
        (the order of a message's changes in this engine)."""
        st = np.asarray(status)
        want = (st == ALIVE) | (st == SUSPECT)
        add = [address(m) for m in np.nonzero(want)[0] if not self.has_server(address(m))]
        rem = [address(m) for m in np.nonzero(~want)[0] if self.has_server(address(m))]
        return self.add_remove_servers(add, rem)

    # ---- queries ----
    def checksum(self) -> int:
        v = C.c_uint32()
        self._chk(_lib().swimring_checksum(self.h, C.byref(v)))
        return v.value

    def server_count(self) -> int:
        v = C.c_uint32()
        self._chk(_lib().swimring_server_count(self.h, C.byref(v)))
        return v.value

    def has_server(self, server: str) -> bool:
        v = C.c_int32()
        self._chk(_lib().swimring_has_server(self.h, server.encode(), C.byref(v)))
        return bool(v.value)

    def name(self, sid: int) -> str:
        v = _lib().swimring_server_name(self.h, int(sid))
        return v.decode() if v is not None else ""

    def lookup_ids(self, keys) -> np.ndarray:
        """Lookup for a batch of keys on the device: owner server ids (-1: empty ring)."""
        blob, off = _pack(keys)
        out = np.empty(len(keys), np.int32)
        self._chk(_lib().swimring_lookup_batch(self.h, blob, off.ctypes.data, len(keys), out.ctypes.data))
        return out

    def lookup(self, key):
        sid = int(self.lookup_ids([key])[0])
        return (self.name(sid), True) if sid >= 0 else ("", False)

    def lookup_n(self, key, n: int):
        k = key.encode() if isinstance(key, str) else bytes(key)
        cap = max(1, n, self.server_count())
        out = np.empty(cap, np.int32)
        got = C.c_size_t()
        self._chk(_lib().swimring_lookup_n(self.h, k, len(k), n, out.ctypes.data, C.byref(got)))
        return [self.name(i) for i in out[:got.value]]

    def servers(self):
        return self.lookup_n(b"", self.server_count())

    def points(self):
        n = C.c_size_t()
        self._chk(_lib().swimring_points(self.h, None, None, 0, C.byref(n)))
        hs = np.empty(max(1, n.value), np.uint32)
        ow = np.empty(max(1, n.value), np.int32)
        self._chk(_lib().swimring_points(self.h, hs.ctypes.data, ow.ctypes.data, n.value, C.byref(n)))
        return hs[:n.value], ow[:n.value]

    def fingerprint32(self, strings) -> np.ndarray:
        blob, off = _pack(strings)
        out = np.empty(len(strings), np.uint32)
        self._chk(_lib().swimring_fingerprint32_batch(self.h, blob, off.ctypes.data, len(strings), out.ctypes.data))
        return out

    def last_times(self):
        a, b = C.c_double(), C.c_double()
        self._chk(_lib().swimring_last_times(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value
