"""JSON wire format of the swim RPCs (swimsim.wire).

CPU tests pin the encoder to Go's encoding/json rules for the reference's structs and the decoder to
json.Unmarshal's; the bridge tests run against the C oracle wrapped in the engine's read-back names.
GPU tests compare the bodies built from the engine's device state with those built from the oracle
on the same workload, byte for byte, and seed engine rows from a decoded joinResponse.

Expected bytes are derived from Go's encoding rules and the struct tags (swim/member.go:135-145,
ping_sender.go:35-40, ping_request_sender.go:35-41, ping_request_handler.go:26-30,
join_sender.go:58-63, join_handler.go:27-32): no Go toolchain exists here, so they are not outputs
of the reference itself.
"""
import numpy as np
import pytest

import swimsim
from swimsim import wire as W
from swimsim import workloads as WL
from oracle_ffi import OracleSim
from swimsim import TOMBSTONE, UNKNOWN

ZERO = W.GO_ZERO_TIME_UNIX


def test_change_omits_tombstone():
    # member_test.go:127-141 (TestChangeOmitTombstone)
    c = W.Change(address="192.0.2.100:1234", incarnation=42, status="alive")
    assert c.to_json() == ('{"source":"","sourceIncarnationNumber":0,"address":"192.0.2.100:1234",'
                           '"incarnationNumber":42,"status":"alive","timestamp":-62135596800}')
    assert "tombstone" not in c.to_json()


def test_tombstone_goes_out_as_faulty_with_flag():
    # validateOutgoing / validateIncoming, member.go:150-167
    c = W.Change("10.000.000.001:7000", 7, "10.000.000.002:7000", 9, "tombstone", timestamp=1500000000)
    out = c.validate_outgoing()
    assert (out.status, out.tombstone) == ("faulty", True)
    assert out.to_json() == ('{"source":"10.000.000.001:7000","sourceIncarnationNumber":7,'
                             '"address":"10.000.000.002:7000","incarnationNumber":9,"status":"faulty",'
                             '"tombstone":true,"timestamp":1500000000}')
    back = W.Ping.from_json(W.Ping([out]).to_json()).changes[0].validate_incoming()
    assert back.status == "tombstone"
    # faulty without the flag stays faulty
    assert W.Change(status="faulty").validate_incoming().status == "faulty"


def test_bodies_field_order_and_empty_lists():
    assert W.Ping([], 3, "a", 4).to_json() == '{"changes":[],"checksum":3,"source":"a","sourceIncarnationNumber":4}'
    assert W.Ping(None).to_json() == '{"changes":null,"checksum":0,"source":"","sourceIncarnationNumber":0}'
    assert W.PingRequest("s", 1, "t", 2, []).to_json() == \
        '{"source":"s","sourceIncarnationNumber":1,"target":"t","checksum":2,"changes":[]}'
    assert W.PingResponse(True, "t", None).to_json() == '{"pingStatus":true,"target":"t","changes":null}'
    assert W.JoinRequest("ringpop", "s", 5, 1_000_000_000).to_json() == \
        '{"app":"ringpop","source":"s","incarnationNumber":5,"timeout":1000000000}'
    assert W.JoinResponse("ringpop", "c", [], 9).to_json() == \
        '{"app":"ringpop","coordinator":"c","membership":[],"membershipChecksum":9}'


@pytest.mark.parametrize("body", [
    W.Ping([W.Change("a", 1, "b", 2, "suspect", False, 3)], 4294967295, "a", -5),
    W.PingRequest("a", 1, "c", 0, [W.Change(address="x", status="leave")]),
    W.PingResponse(False, "c", [W.Change(status="faulty", tombstone=True)]),
    W.JoinRequest("app", "src", 1500000000000, 1),
    W.JoinResponse("app", "coord", [W.Change("a", 1, "b", 2, "alive")] * 3, 123456),
])
def test_round_trip(body):
    assert type(body).from_json(body.to_json()) == body
    assert type(body).from_json(body.to_json().encode()) == body


def test_go_string_escapes():
    assert W.go_string('<a&b>') == '"\\u003ca\\u0026b\\u003e"'
    assert W.go_string('q"\\\n\r\t\x01') == '"q\\"\\\\\\n\\r\\t\\u0001"'
    assert W.go_string(" x ") == '"\\u2028x\\u2029"'
    assert W.go_string("é") == '"é"'
    assert W.go_string("a\udc80b") == '"a\\ufffdb"'        # invalid UTF-8 (surrogateescape) -> \ufffd


def test_unmarshal_rules():
    # keys: exact or case-insensitive, last duplicate wins, unknown ignored, null leaves the default
    p = W.Ping.from_json('{"CHECKSUM":1,"checksum":2,"Source":"x","extra":[1,2],"changes":null,'
                         '"sourceIncarnationNumber":null}')
    assert (p.checksum, p.source, p.changes, p.source_incarnation) == (2, "x", None, 0)
    c = W.Ping.from_json('{"changes":[{"ADDRESS":"a","status":"alive","incarnationnumber":3}]}').changes[0]
    assert (c.address, c.status, c.incarnation, c.timestamp) == ("a", "alive", 3, ZERO)


@pytest.mark.parametrize("text", [
    '{"checksum":-1}', '{"checksum":4294967296}', '{"checksum":1.0}', '{"checksum":"1"}',
    '{"sourceIncarnationNumber":1e3}', '{"sourceIncarnationNumber":9223372036854775808}',
    '{"source":5}', '{"changes":{}}', '{"changes":[1]}', '{"changes":[{"timestamp":1.5}]}',
    '{"changes":[{"timestamp":null}]}', '{"changes":[{"tombstone":1}]}', '[]', '{"checksum":NaN}', '{',
])
def test_unmarshal_errors(text):
    with pytest.raises(W.WireError):
        W.Ping.from_json(text)


def test_addresses_and_columns():
    for m in (0, 1, 255, 256, 65535, 65536, (1 << 24) - 1):
        assert W.index_of(swimsim.address_of(m)) == m
    for bad in ("10.0.0.1:7000", "10.000.000.001:7001", "11.000.000.001:7000", "10.256.000.000:7000"):
        with pytest.raises(W.WireError):
            W.index_of(bad)
    cs = [W.Change(swimsim.address_of(1), 10, swimsim.address_of(5), 20, "faulty", True),
          W.Change("192.0.2.1:1", 11, swimsim.address_of(6), 21, "suspect")]
    cols = W.changes_to_arrays(cs, 8)
    assert cols["member"].tolist() == [5, 6]
    assert cols["status"].tolist() == [swimsim.TOMBSTONE, swimsim.SUSPECT]
    assert cols["source"].tolist() == [1, -1]
    assert cols["incarnation"].tolist() == [20, 21] and cols["source_incarnation"].tolist() == [10, 11]
    with pytest.raises(W.WireError):
        W.changes_to_arrays([W.Change(address=swimsim.address_of(8), status="alive")], 8)
    with pytest.raises(W.WireError):
        W.changes_to_arrays([W.Change(address=swimsim.address_of(1), status="dead")], 8)


class OracleView:
    """the C oracle under the engine's read-back names, so the bridge runs on CPU (test only)"""

    def __init__(self, ora):
        self.o, self.n = ora, ora.n

    def row(self, o):
        return self.o.row(o)

    def changes(self, o):
        return self.o.dis_entries(o)

    def checksum(self, o):
        return self.o.checksum(o)

    def member(self, o, m):
        return self.o.member(o, m)

    def set_row(self, o, status, inc):
        for m in range(self.n):
            self.o.set_member(o, m, int(status[m]), int(inc[m]))


def _oracle_after(wl, rounds):
    ora = OracleSim(wl.n)
    for r in range(rounds):
        ora.step(wl.events_for(r))
    return ora


def test_bridge_bodies_from_oracle_state():
    wl = WL.config1()
    ora = _oracle_after(wl, 3)            # member 5 killed at r=0: suspect declarations are buffered
    v = OracleView(ora)
    o = next(o for o in range(wl.n) if ora.dis_entries(o))
    ping = W.ping_of(v, o)
    assert ping.source == swimsim.address_of(o) and ping.checksum == ora.checksum(o)
    assert ping.source_incarnation == ora.member(o, o)[1]
    assert [W.index_of(c.address) for c in ping.changes] == sorted(ora.dis_entries(o))
    st, inc = ora.row(o)
    for c in ping.changes:
        m = W.index_of(c.address)
        p, s, sinc = ora.dis_entries(o)[m]
        assert (c.incarnation, W.index_of(c.source), c.source_incarnation) == (inc[m], s, sinc)
        assert W.STATUS_CODES[c.validate_incoming().status] == st[m]
    again = W.Ping.from_json(ping.to_json())
    assert again == ping
    jr = W.join_response(v, o, "ringpop")
    assert len(jr.membership) == wl.n and jr.checksum == ora.checksum(o)
    assert all(c.source == swimsim.address_of(o) for c in jr.membership)


def test_ping_request_and_response_bodies_on_oracle():
    wl = WL.config1()
    ora = _oracle_after(wl, 4)            # six observers hold buffered suspect changes
    v = OracleView(ora)
    o = next(o for o in range(wl.n) if ora.dis_entries(o))
    req = W.ping_request_of(v, o, 5)
    assert (req.source, req.target) == (swimsim.address_of(o), swimsim.address_of(5))
    assert req.changes == W.issue_as_sender(v, o) and req.checksum == ora.checksum(o)
    assert W.PingRequest.from_json(req.to_json()) == req
    # filterChangesFromSender: a helper drops what came from the requester at its incarnation
    h = next(h for h in range(wl.n) if h != o and ora.dis_entries(h))
    mine = W.issue_as_sender(v, h)
    fake = W.PingRequest(mine[0].source, mine[0].source_incarnation, swimsim.address_of(5), ora.checksum(h), [])
    res = W.ping_response_of(v, h, fake, True)
    assert res.ok and res.target == swimsim.address_of(5)
    assert res.changes == [c for c in mine if (c.source, c.source_incarnation) != (fake.source, fake.source_incarnation)]
    # nothing left and checksums differ: IssueAsReceiver falls back to the full membership
    quiet = next(q for q in range(wl.n) if q != 5 and not ora.dis_entries(q))
    ch, full = W.issue_as_receiver(v, quiet, "x", 0, ora.checksum(quiet) ^ 1)
    assert full and len(ch) == wl.n and all(c.source == swimsim.address_of(quiet) for c in ch)
    ch, full = W.issue_as_receiver(v, quiet, "x", 0, ora.checksum(quiet))
    assert (ch, full) == ([], False)


def test_seed_from_join_response_reproduces_checksum_on_oracle():
    wl = WL.config1()
    ora = _oracle_after(wl, 40)           # member 5 faulty in every live row by now
    body = W.join_response(OracleView(ora), 0, "ringpop").to_json()
    fresh = OracleSim(wl.n, init="self")
    assert W.seed_from_membership(OracleView(fresh), 3, W.JoinResponse.from_json(body).membership) == wl.n
    assert (fresh.row(3)[0] == ora.row(0)[0]).all() and (fresh.row(3)[1] == ora.row(0)[1]).all()
    assert fresh.checksum(3) == ora.checksum(0) == W.JoinResponse.from_json(body).checksum


def test_seed_skips_tombstones_of_unseen_members():
    """Apply refuses to create a member whose first state is tombstone (memberlist.go:424-426)"""
    wl = WL.config1()
    ora = _oracle_after(wl, 3)
    inc9 = ora.member(0, 9)[1]
    assert ora.make_change(0, 9, inc9, TOMBSTONE) == 1
    jr = W.join_response(OracleView(ora), 0, "ringpop")
    assert any(c.validate_incoming().status == "tombstone" for c in jr.membership)
    fresh = OracleSim(wl.n, init="self")
    assert W.seed_from_membership(OracleView(fresh), 3, jr.membership) == wl.n - 1
    assert fresh.member(3, 9)[0] == UNKNOWN and fresh.num_members(3) == wl.n - 1
    assert fresh.checksum(3) == ora.checksum(0)       # tombstones are not in the checksum string


def test_ping_of_after_eviction_keeps_buffered_tombstone():
    """An entry can outlive its member's eviction (Evict leaves the disseminator alone,
    memberlist.go:271-279): the ping then carries it as faulty + tombstone flag (issueChanges builds it
    from the last applied change; validateOutgoing, member.go:161-167)"""
    n = 8
    ora = OracleSim(n, suspect_ms=400, faulty_ms=400, tombstone_ms=400)
    v = OracleView(ora)
    ev = [(0, WL.EV_PARTITION, 0, 1)]
    found = None
    for r in range(40):
        ora.step([e for e in ev if e[0] == r])
        for o in range(1, n):
            ents = ora.dis_entries(o)
            if 0 in ents and ora.member(o, 0)[0] == UNKNOWN:
                found = o
                break
        if found is not None:
            break
    assert found is not None, "no observer held a buffered change of an evicted member"
    ping = W.ping_of(v, found)
    c0 = next(c for c in ping.changes if W.index_of(c.address) == 0)
    assert c0.status == "faulty" and c0.tombstone
    assert W.Ping.from_json(ping.to_json()) == ping


# ---- GPU: bodies from device state, byte for byte against the oracle's -------------------------------
@pytest.mark.gpu
def test_gpu_ping_and_join_bodies_match_oracle():
    wl = WL.config2(n=256, rounds=12)
    eng = swimsim.Cluster(wl.n, device=0)
    ora = OracleSim(wl.n)
    for r in range(wl.rounds):
        ev = wl.events_for(r)
        eng.step(1, ev)
        ora.step(ev)
    v = OracleView(ora)
    for o in range(0, wl.n, 17):
        assert W.ping_of(eng, o).to_json() == W.ping_of(v, o).to_json(), f"ping body of {o}"
        assert W.join_response(eng, o, "ringpop").to_json() == W.join_response(v, o, "ringpop").to_json()
        assert W.ping_request_of(eng, o, (o + 1) % wl.n).to_json() == W.ping_request_of(v, o, (o + 1) % wl.n).to_json()
        req = W.ping_request_of(v, (o + 3) % wl.n, o)
        assert W.ping_response_of(eng, o, req, True).to_json() == W.ping_response_of(v, o, req, True).to_json()


@pytest.mark.gpu
def test_gpu_seed_rows_from_join_response():
    wl = WL.config3(n=1024, rounds=40, kill_round=2)
    src = swimsim.Cluster(wl.n, device=0)
    src.run(wl.rounds, wl.events)
    dst = swimsim.Cluster(wl.n, device=0, init="self")
    for o in (0, 511, 1023):
        jr = W.JoinResponse.from_json(W.join_response(src, o, "ringpop").to_json())
        W.seed_from_membership(dst, o, jr.membership)
        s1, i1 = src.row(o)
        s2, i2 = dst.row(o)
        assert (s1 == s2).all() and (i1 == i2).all()
        assert dst.checksum(o) == src.checksum(o) == jr.checksum
        assert dst.count_reachable(o) == src.count_reachable(o)


@pytest.mark.gpu
def test_gpu_seed_refuses_foreign_incarnations():
    """the engine keeps incarnations as t0 + e*period: another value is refused, never rounded"""
    eng = swimsim.Cluster(16, device=0)
    before = eng.row(3)
    bad = [W.Change(address=swimsim.address_of(m), incarnation=swimsim.T0_MS + 1, status="alive") for m in range(16)]
    with pytest.raises(swimsim.SwimsimError):
        W.seed_from_membership(eng, 3, bad)
    st = np.full(16, 9, np.uint8)
    with pytest.raises(swimsim.SwimsimError):
        eng.set_row(3, st, np.full(16, swimsim.T0_MS, np.int64))
    after = eng.row(3)
    assert (before[0] == after[0]).all() and (before[1] == after[1]).all(), "a refused row write changed the row"


def test_round_trip_properties():
    """random bodies: the encoding is valid JSON carrying the same values, and decodes to the body"""
    import json
    from hypothesis import given, settings, strategies as st

    text = st.text(st.characters(blacklist_categories=("Cs",)), max_size=12)
    i64 = st.integers(-(1 << 63), (1 << 63) - 1)
    change = st.builds(W.Change, text, i64, text, i64, st.sampled_from(["alive", "suspect", "faulty", "leave"]),
                       st.booleans(), i64)

    @settings(max_examples=200, deadline=None)
    @given(st.lists(change, max_size=5) | st.none(), st.integers(0, (1 << 32) - 1), text, i64)
    def check(changes, checksum, source, sinc):
        p = W.Ping(changes, checksum, source, sinc)
        j = p.to_json()
        plain = json.loads(j)
        assert (plain["checksum"], plain["source"], plain["sourceIncarnationNumber"]) == (checksum, source, sinc)
        assert list(plain) == ["changes", "checksum", "source", "sourceIncarnationNumber"]
        if changes:
            assert [c["address"] for c in plain["changes"]] == [c.address for c in changes]
            assert all(("tombstone" in c) == x.tombstone for c, x in zip(plain["changes"], changes))
        assert W.Ping.from_json(j) == p

    check()
