"""JSON wire format of the swim RPCs, bridged to the engine's rows.

The reference sends its gossip as JSON bodies over TChannel:
  * ``Change``        swim/member.go:135-145 (``tombstone`` is omitempty; ``timestamp`` is
                      util.Timestamp, an integer Unix time in seconds, util/util.go:255-276)
  * ``ping``          swim/ping_sender.go:35-40 (a ping and its response share this body)
  * ``pingRequest``   swim/ping_request_sender.go:35-41
  * ``pingResponse``  swim/ping_request_handler.go:26-30
  * ``joinRequest``   swim/join_sender.go:58-63
  * ``joinResponse``  swim/join_handler.go:27-32

Encoding follows Go's ``encoding/json`` byte for byte: struct fields in declaration order, no
whitespace, HTML-safe string escapes, ``[]`` for an empty issued list (disseminator.go:203-205) and
``null`` for a nil slice. Decoding follows ``json.Unmarshal``: keys match exactly or else
case-insensitively, the last duplicate wins, unknown keys are ignored, ``null`` leaves a field
unchanged, and a number that is not an integer of the field's range is an error.

The engine bridge turns an observer's device state into the bodies the reference node would send
(``ping_of``, ``issue_as_sender``, ``membership_as_changes``, ``join_response``) and seeds rows from
a received membership (``seed_from_membership``). Go iterates its change map in random order
(disseminator.go:203-207) and its member slice in join order; the bridge lists members by index.
This module is host-side formatting around the C ABI; it does no protocol arithmetic itself.
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import ALIVE, FAULTY, LEAVE, SUSPECT, TOMBSTONE, UNKNOWN, STATUS_NAMES, address_of

STATUS_CODES = {v: k for k, v in STATUS_NAMES.items()}
GO_ZERO_TIME_UNIX = -62135596800        # time.Time{}.Unix(): what an unset Timestamp marshals to


class WireError(ValueError):
    pass


# ---- Go encoding/json string and number rules ---------------------------------------------------
_HEX = "0123456789abcdef"


def go_string(s: str) -> str:
    """encoding/json encodeState.string with HTML escaping (Go 1.5/1.6, .travis.yml:2-4)"""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"' or ch == "\\":
            out.append("\\" + ch)
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or ch in "<>&":
            out.append("\\u00" + _HEX[o >> 4] + _HEX[o & 15])
        elif o in (0x2028, 0x2029):
            out.append("\\u202" + _HEX[o & 15])
        elif 0xD800 <= o <= 0xDFFF:          # invalid UTF-8 (a lone surrogate here): Go writes \ufffd
            out.append("\\ufffd")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


class _Obj(list):
    """a decoded JSON object: its (key, value) pairs in document order"""


class _Float(str):
    """raw JSON number text with a fraction or exponent (Go rejects it for integer fields)"""


def _reject_constant(name):
    raise WireError(f"invalid character in JSON: {name}")


def _loads(data):
    if isinstance(data, (bytes, bytearray)):
        data = data.decode("utf-8", errors="replace")
    try:
        return json.loads(data, parse_float=_Float, parse_constant=_reject_constant,
                          object_pairs_hook=_Obj)
    except json.JSONDecodeError as e:
        raise WireError(f"invalid JSON: {e}") from None


def _int(v, lo, hi, what):
    if isinstance(v, bool) or not isinstance(v, int):
        raise WireError(f"json: cannot unmarshal {type(v).__name__} into {what}")
    if not lo <= v <= hi:
        raise WireError(f"json: cannot unmarshal number {v} into {what}")
    return v


def _i64(v, what):
    return _int(v, -(1 << 63), (1 << 63) - 1, what)


def _u32(v, what):
    return _int(v, 0, (1 << 32) - 1, what)


def _str(v, what):
    if not isinstance(v, str) or isinstance(v, _Float):
        raise WireError(f"json: cannot unmarshal {type(v).__name__} into {what} of type string")
    return str(v)


def _bool(v, what):
    if not isinstance(v, bool):
        raise WireError(f"json: cannot unmarshal {type(v).__name__} into {what} of type bool")
    return v


def _fields(pairs, names, null_is_error=()):
    """Go field matching: exact name first, else case-insensitive; last duplicate wins; null leaves a
    field unchanged, except for fields whose UnmarshalJSON receives it (null_is_error)"""
    if not isinstance(pairs, _Obj):
        raise WireError("json: cannot unmarshal non-object into a struct")
    folded = {n.lower(): n for n in names}
    got = {}
    for k, v in pairs:
        name = k if k in names else folded.get(k.lower())
        if name is None:
            continue
        if v is None:
            if name in null_is_error:
                raise WireError(f"json: {name}: UnmarshalJSON cannot parse null")
            continue
        got[name] = v
    return got


# ---- Change ----------------------------------------------------------------------------------------
@dataclass
class Change:
    """swim.Change (swim/member.go:135-145); status is the wire string ("alive" ... "tombstone")"""
    source: str = ""
    source_incarnation: int = 0
    address: str = ""
    incarnation: int = 0
    status: str = ""
    tombstone: bool = False
    timestamp: int = GO_ZERO_TIME_UNIX      # Unix seconds

    def validate_outgoing(self) -> "Change":   # member.go:160-167
        if self.status == "tombstone":
            return Change(self.source, self.source_incarnation, self.address, self.incarnation, "faulty", True,
                          self.timestamp)
        return self

    def validate_incoming(self) -> "Change":   # member.go:150-155
        if self.status == "faulty" and self.tombstone:
            return Change(self.source, self.source_incarnation, self.address, self.incarnation, "tombstone",
                          self.tombstone, self.timestamp)
        return self

    def to_json(self) -> str:
        parts = [f'"source":{go_string(self.source)}',
                 f'"sourceIncarnationNumber":{int(self.source_incarnation)}',
                 f'"address":{go_string(self.address)}',
                 f'"incarnationNumber":{int(self.incarnation)}',
                 f'"status":{go_string(self.status)}']
        if self.tombstone:
            parts.append('"tombstone":true')
        parts.append(f'"timestamp":{int(self.timestamp)}')
        return "{" + ",".join(parts) + "}"

    @classmethod
    def from_pairs(cls, pairs) -> "Change":
        f = _fields(pairs, ("source", "sourceIncarnationNumber", "address", "incarnationNumber", "status",
                            "tombstone", "timestamp"), null_is_error=("timestamp",))
        c = cls()
        if "source" in f:
            c.source = _str(f["source"], "Change.source")
        if "sourceIncarnationNumber" in f:
            c.source_incarnation = _i64(f["sourceIncarnationNumber"], "Change.sourceIncarnationNumber of type int64")
        if "address" in f:
            c.address = _str(f["address"], "Change.address")
        if "incarnationNumber" in f:
            c.incarnation = _i64(f["incarnationNumber"], "Change.incarnationNumber of type int64")
        if "status" in f:
            c.status = _str(f["status"], "Change.status")
        if "tombstone" in f:
            c.tombstone = _bool(f["tombstone"], "Change.tombstone")
        if "timestamp" in f:
            # util.Timestamp.UnmarshalJSON is strconv.Atoi of the raw bytes (util/util.go:268-276)
            c.timestamp = _int(f["timestamp"], -(1 << 63), (1 << 63) - 1, "util.Timestamp")
        return c


def _changes_json(changes: Optional[List[Change]]) -> str:
    if changes is None:
        return "null"
    return "[" + ",".join(c.to_json() for c in changes) + "]"


def _changes_from(v, what) -> List[Change]:
    if isinstance(v, _Obj) or not isinstance(v, list) or not all(isinstance(x, _Obj) for x in v):
        raise WireError(f"json: cannot unmarshal into {what} of type []swim.Change")
    return [Change.from_pairs(x) for x in v]


# ---- RPC bodies ------------------------------------------------------------------------------------
@dataclass
class Ping:
    """swim.ping (swim/ping_sender.go:35-40): request and response body of /protocol/ping"""
    changes: Optional[List[Change]] = None
    checksum: int = 0
    source: str = ""
    source_incarnation: int = 0

    def to_json(self) -> str:
        return (f'{{"changes":{_changes_json(self.changes)},"checksum":{int(self.checksum)},'
                f'"source":{go_string(self.source)},"sourceIncarnationNumber":{int(self.source_incarnation)}}}')

    @classmethod
    def from_json(cls, data) -> "Ping":
        f = _fields(_loads(data), ("changes", "checksum", "source", "sourceIncarnationNumber"))
        p = cls()
        if "changes" in f:
            p.changes = _changes_from(f["changes"], "ping.changes")
        if "checksum" in f:
            p.checksum = _u32(f["checksum"], "ping.checksum of type uint32")
        if "source" in f:
            p.source = _str(f["source"], "ping.source")
        if "sourceIncarnationNumber" in f:
            p.source_incarnation = _i64(f["sourceIncarnationNumber"], "ping.sourceIncarnationNumber of type int64")
        return p


@dataclass
class PingRequest:
    """swim.pingRequest (swim/ping_request_sender.go:35-41)"""
    source: str = ""
    source_incarnation: int = 0
    target: str = ""
    checksum: int = 0
    changes: Optional[List[Change]] = None

    def to_json(self) -> str:
        return (f'{{"source":{go_string(self.source)},"sourceIncarnationNumber":{int(self.source_incarnation)},'
                f'"target":{go_string(self.target)},"checksum":{int(self.checksum)},'
                f'"changes":{_changes_json(self.changes)}}}')

    @classmethod
    def from_json(cls, data) -> "PingRequest":
        f = _fields(_loads(data), ("source", "sourceIncarnationNumber", "target", "checksum", "changes"))
        r = cls()
        if "source" in f:
            r.source = _str(f["source"], "pingRequest.source")
        if "sourceIncarnationNumber" in f:
            r.source_incarnation = _i64(f["sourceIncarnationNumber"], "pingRequest.sourceIncarnationNumber")
        if "target" in f:
            r.target = _str(f["target"], "pingRequest.target")
        if "checksum" in f:
            r.checksum = _u32(f["checksum"], "pingRequest.checksum of type uint32")
        if "changes" in f:
            r.changes = _changes_from(f["changes"], "pingRequest.changes")
        return r


@dataclass
class PingResponse:
    """swim.pingResponse (swim/ping_request_handler.go:26-30)"""
    ok: bool = False
    target: str = ""
    changes: Optional[List[Change]] = None

    def to_json(self) -> str:
        return (f'{{"pingStatus":{"true" if self.ok else "false"},"target":{go_string(self.target)},'
                f'"changes":{_changes_json(self.changes)}}}')

    @classmethod
    def from_json(cls, data) -> "PingResponse":
        f = _fields(_loads(data), ("pingStatus", "target", "changes"))
        r = cls()
        if "pingStatus" in f:
            r.ok = _bool(f["pingStatus"], "pingResponse.pingStatus")
        if "target" in f:
            r.target = _str(f["target"], "pingResponse.target")
        if "changes" in f:
            r.changes = _changes_from(f["changes"], "pingResponse.changes")
        return r


@dataclass
class JoinRequest:
    """swim.joinRequest (swim/join_sender.go:58-63); timeout is a time.Duration in nanoseconds"""
    app: str = ""
    source: str = ""
    incarnation: int = 0
    timeout_ns: int = 0

    def to_json(self) -> str:
        return (f'{{"app":{go_string(self.app)},"source":{go_string(self.source)},'
                f'"incarnationNumber":{int(self.incarnation)},"timeout":{int(self.timeout_ns)}}}')

    @classmethod
    def from_json(cls, data) -> "JoinRequest":
        f = _fields(_loads(data), ("app", "source", "incarnationNumber", "timeout"))
        r = cls()
        if "app" in f:
            r.app = _str(f["app"], "joinRequest.app")
        if "source" in f:
            r.source = _str(f["source"], "joinRequest.source")
        if "incarnationNumber" in f:
            r.incarnation = _i64(f["incarnationNumber"], "joinRequest.incarnationNumber of type int64")
        if "timeout" in f:
            r.timeout_ns = _i64(f["timeout"], "joinRequest.timeout of type time.Duration")
        return r


@dataclass
class JoinResponse:
    """swim.joinResponse (swim/join_handler.go:27-32)"""
    app: str = ""
    coordinator: str = ""
    membership: Optional[List[Change]] = None
    checksum: int = 0

    def to_json(self) -> str:
        return (f'{{"app":{go_string(self.app)},"coordinator":{go_string(self.coordinator)},'
                f'"membership":{_changes_json(self.membership)},"membershipChecksum":{int(self.checksum)}}}')

    @classmethod
    def from_json(cls, data) -> "JoinResponse":
        f = _fields(_loads(data), ("app", "coordinator", "membership", "membershipChecksum"))
        r = cls()
        if "app" in f:
            r.app = _str(f["app"], "joinResponse.app")
        if "coordinator" in f:
            r.coordinator = _str(f["coordinator"], "joinResponse.coordinator")
        if "membership" in f:
            r.membership = _changes_from(f["membership"], "joinResponse.membership")
        if "membershipChecksum" in f:
            r.checksum = _u32(f["membershipChecksum"], "joinResponse.membershipChecksum of type uint32")
        return r


# ---- addresses <-> member indices --------------------------------------------------------------------
_ADDR = re.compile(r"^10\.(\d{3})\.(\d{3})\.(\d{3}):7000$")


def index_of(address: str) -> int:
    """inverse of swimsim.address_of (the synthetic address scheme of SURVEY.md §8(d))"""
    m = _ADDR.match(address)
    if not m:
        raise WireError(f"address {address!r} is not a simulated member address")
    a, b, c = (int(x) for x in m.groups())
    if a > 255 or b > 255 or c > 255:
        raise WireError(f"address {address!r} has an octet above 255")
    return (a << 16) | (b << 8) | c


def changes_to_arrays(changes: List[Change], n: int, index=index_of):
    """Incoming changes (validateIncoming applied) as the engine's packed columns: member u32,
    status u8, incarnation i64, source i32 (-1 when the source is not a member), sourceInc i64."""
    k = len(changes)
    member = np.empty(k, np.uint32); status = np.empty(k, np.uint8); inc = np.empty(k, np.int64)
    source = np.empty(k, np.int32); sinc = np.empty(k, np.int64)
    for i, c in enumerate(changes):
        c = c.validate_incoming()
        if c.status not in STATUS_CODES:
            raise WireError(f"change {i}: unknown status {c.status!r}")
        m = index(c.address)
        if m >= n:
            raise WireError(f"change {i}: member {m} outside a {n}-member cluster")
        member[i], status[i], inc[i] = m, STATUS_CODES[c.status], c.incarnation
        try:
            s = index(c.source)
            source[i] = s if s < n else -1
        except WireError:
            source[i] = -1
        sinc[i] = c.source_incarnation
    return {"member": member, "status": status, "incarnation": inc, "source": source, "source_incarnation": sinc}


# ---- engine bridge -------------------------------------------------------------------------------------
def issue_as_sender(cluster, o: int, timestamp: int = GO_ZERO_TIME_UNIX) -> List[Change]:
    """disseminator.issueChanges (disseminator.go:199-214) of observer o: its buffered changes with
    their recorded source, validateOutgoing applied. Reading does not bump piggyback counters."""
    st, inc = cluster.row(o)
    out = []
    for m, (_p, s, sinc) in sorted(cluster.changes(o).items()):
        # an entry can outlive its member's eviction (Evict leaves the disseminator alone,
        # memberlist.go:271-279): the change then reads (tombstone, inc), as issueChanges builds it from
        # the last applied change
        code = int(st[m])
        name = STATUS_NAMES[TOMBSTONE if code == UNKNOWN else code]
        out.append(Change(address_of(s) if s >= 0 else "", sinc, address_of(m), int(inc[m]),
                          name, False, timestamp).validate_outgoing())
    return out


def ping_of(cluster, o: int, timestamp: int = GO_ZERO_TIME_UNIX) -> Ping:
    """the ping body observer o sends now (sendPing / sendPingWithChanges, ping_sender.go:43-66)"""
    return Ping(issue_as_sender(cluster, o, timestamp), cluster.checksum(o), address_of(o),
                cluster.member(o, o)[1])


def issue_as_receiver(cluster, o: int, sender: str, sender_incarnation: int, sender_checksum: int,
                      timestamp: int = GO_ZERO_TIME_UNIX):
    """disseminator.IssueAsReceiver (disseminator.go:155-181) of observer o, read-only: the buffered
    changes minus those that came from the sender at its incarnation (filterChangesFromSender,
    185-199); if none are left and the checksums differ, the full membership and full_sync = True.
    The device's piggyback counters are not bumped (the engine bumps them inside swimsim_step)."""
    changes = [c for c in issue_as_sender(cluster, o, timestamp)
               if not (c.source == sender and c.source_incarnation == sender_incarnation)]
    if changes or cluster.checksum(o) == sender_checksum:
        return changes, False
    return membership_as_changes(cluster, o, timestamp), True


def ping_request_of(cluster, o: int, target: int, timestamp: int = GO_ZERO_TIME_UNIX) -> PingRequest:
    """the pingRequest body o sends to each helper about `target` (ping_request_sender.go:95-101)"""
    return PingRequest(address_of(o), cluster.member(o, o)[1], address_of(target), cluster.checksum(o),
                       issue_as_sender(cluster, o, timestamp))


def ping_response_of(cluster, helper: int, req: PingRequest, ok: bool,
                     timestamp: int = GO_ZERO_TIME_UNIX) -> PingResponse:
    """the helper's answer to a pingRequest (handlePingRequest, ping_request_handler.go:32-76): the
    relayed ping's outcome and IssueAsReceiver's changes, the full membership included when it falls
    back to a full sync (whose flag the handler ignores, line 69)."""
    changes, _full = issue_as_receiver(cluster, helper, req.source, req.source_incarnation, req.checksum, timestamp)
    return PingResponse(bool(ok), req.target, changes)


def membership_as_changes(cluster, o: int, timestamp: int = GO_ZERO_TIME_UNIX) -> List[Change]:
    """disseminator.MembershipAsChanges (disseminator.go:107-123): every known member, source = self"""
    st, inc = cluster.row(o)
    src, sinc = address_of(o), int(inc[o])
    return [Change(src, sinc, address_of(m), int(inc[m]), STATUS_NAMES[int(st[m])], False, timestamp).validate_outgoing()
            for m in np.nonzero(st != UNKNOWN)[0].tolist()]


def join_response(cluster, o: int, app: str, timestamp: int = GO_ZERO_TIME_UNIX) -> JoinResponse:
    """handleJoin's response body (join_handler.go:52-77) from observer o"""
    return JoinResponse(app, address_of(o), membership_as_changes(cluster, o, timestamp), cluster.checksum(o))


def seed_from_membership(cluster, o: int, changes: List[Change]) -> int:
    """Write a received membership (a joinResponse's, or a real node's) into observer o's row as its
    bootstrap state: the list applied in order by memberlist.Update's rules to an empty memberlist
    (memberlist.go:310-390). An unseen member is taken wholesale (325-334) unless the change is a
    tombstone, which Apply refuses to create (424-426); a later duplicate applies only if it overrides
    (nonLocalOverride, member.go:79-93). Members absent from the list stay unknown. No side effects (no
    dissemination entries or timers): one swimsim_set_row call. Returns the number of members written."""
    cols = changes_to_arrays(changes, cluster.n)
    status = np.full(cluster.n, UNKNOWN, np.uint8)
    inc = np.zeros(cluster.n, np.int64)
    for m, st, ic in zip(cols["member"].tolist(), cols["status"].tolist(), cols["incarnation"].tolist()):
        if status[m] == UNKNOWN:
            if st == TOMBSTONE:
                continue
        elif not (ic > inc[m] or (ic == inc[m] and st > status[m])):
            continue
        status[m], inc[m] = st, ic
    cluster.set_row(o, status, inc)
    return int(np.count_nonzero(status != UNKNOWN))


__all__ = ["Change", "Ping", "PingRequest", "PingResponse", "JoinRequest", "JoinResponse", "WireError",
           "go_string", "index_of", "changes_to_arrays", "issue_as_sender", "issue_as_receiver", "ping_of",
           "ping_request_of", "ping_response_of", "membership_as_changes",
           "join_response", "seed_from_membership", "GO_ZERO_TIME_UNIX", "STATUS_CODES",
           "ALIVE", "SUSPECT", "FAULTY", "LEAVE", "TOMBSTONE"]
