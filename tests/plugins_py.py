"""Stand-ins for two of the reference's process plugins, as ipxg_plugin callbacks (TEST
INFRASTRUCTURE: the real plugins are C++ objects behind the StoragePlugin shim; these restate
only the decisions that change flow boundaries, so the engine's bridge and the oracle can be
driven by the same hooks and checked against the reference's own goldens).

  DnsFlush   dns.cpp:97-127, 650-682: post_create / post_update on a port-53 packet return
             FLOW_FLUSH when parse_dns accepts the payload (header checks and the name walks
             that throw, dns.cpp:148-206, 429-660; an overflow *returns* success).
  HttpReinsert  http.cpp:100-140, 233-300, 400-450: a second request (or response) line in
             a flow that already holds one returns FLOW_FLUSH_WITH_REINSERT from pre_update;
             the first one is kept in the flow's extension (here: bits of the ext handle).
"""
import ctypes

import numpy as np

import pcaputil
from ipfixprobe_amd.engine import (FLOW_FLUSH, FLOW_FLUSH_WITH_REINSERT, FLOW_HOOK_FN, PRE_CREATE_FN,
                                   PRE_EXPORT_FN, Plugin)


class _Throw(Exception):
    pass


def _rec(ptr):
    return np.frombuffer((ctypes.c_uint8 * pcaputil.FLOW_DTYPE.itemsize).from_address(ptr),
                         dtype=pcaputil.FLOW_DTYPE)[0]


def _pkt(view):
    v = view.contents
    p = np.frombuffer((ctypes.c_uint8 * pcaputil.PARSED_DTYPE.itemsize).from_address(v.pkt),
                      dtype=pcaputil.PARSED_DTYPE)[0]
    off, n = int(p["payload_off"]), int(p["payload_len"])
    # Packet::payload_len can run past the captured bytes (uint16_t wraps of malformed lengths,
    # parser.cpp:780-797; the reference reads whatever follows): bytes at or past caplen read as 0
    cap = int(v.caplen)
    end = min(off + n, cap)
    data = (bytes(v.data[off:end]) if end > off else b"") + bytes(max(0, off + n - max(end, off))) if n else b""
    return p, data


class PyPlugin:
    """Base: builds the ctypes Plugin (rule + callbacks) and keeps the callbacks alive."""
    proto_mask = 3
    ports = ()
    prefixes = ()

    def __init__(self):
        self.calls = {"pre_create": 0, "post_create": 0, "pre_update": 0, "post_update": 0, "pre_export": 0}
        self._cb = [PRE_CREATE_FN(self._pre_create), FLOW_HOOK_FN(self._post_create), FLOW_HOOK_FN(self._pre_update),
                    FLOW_HOOK_FN(self._post_update), PRE_EXPORT_FN(self._pre_export)]
        s = Plugin()
        s.proto_mask = self.proto_mask
        s.n_ports = len(self.ports)
        for k, port in enumerate(self.ports):
            s.ports[k] = port
        s.n_prefixes = len(self.prefixes)
        for q, pre in enumerate(self.prefixes):
            s.prefix_len[q] = len(pre)
            for k, b in enumerate(pre):
                s.prefix[q][k] = b
        s.pre_create, s.post_create, s.pre_update, s.post_update, s.pre_export = self._cb
        self.struct = s

    def _pre_create(self, ctx, view):
        self.calls["pre_create"] += 1
        return 0

    def _post_create(self, ctx, flow, view):
        self.calls["post_create"] += 1
        p, data = _pkt(view)
        return self.post_create(_rec(flow), p, data)

    def _pre_update(self, ctx, flow, view):
        self.calls["pre_update"] += 1
        p, data = _pkt(view)
        return self.pre_update(_rec(flow), p, data)

    def _post_update(self, ctx, flow, view):
        self.calls["post_update"] += 1
        p, data = _pkt(view)
        return self.post_update(_rec(flow), p, data)

    def _pre_export(self, ctx, flow):
        self.calls["pre_export"] += 1

    def post_create(self, rec, p, data):
        return 0

    def pre_update(self, rec, p, data):
        return 0

    def post_update(self, rec, p, data):
        return 0


# ---- DNS ------------------------------------------------------------------------------------
MAX_LABEL_CNT = 127


def _b(d, i):
    return d[i] if 0 <= i < len(d) else 0


def _get_name_length(d, i, n):  # dns.cpp:148-169
    ln = 0
    while True:
        if i + 1 > n:
            raise _Throw()
        if not _b(d, i):
            break
        if (_b(d, i) & 0xC0) == 0xC0:
            return ln + 2
        ln += _b(d, i) + 1
        i += _b(d, i) + 1
    return ln + 1


def _get_name(d, i, n):  # dns.cpp:175-206 (only whether it throws)
    cnt = 0
    if i > n:
        raise _Throw()
    while _b(d, i):
        c = _b(d, i)
        if (c & 0xC0) == 0xC0:
            i = ((c & 0x3F) << 8) | _b(d, i + 1)
            if cnt > MAX_LABEL_CNT or i > n:
                raise _Throw()
            cnt += 1
            continue
        if cnt > MAX_LABEL_CNT or c > 63 or i + c + 2 > n:
            raise _Throw()
        cnt += 1
        i += c + 1


def _rdata(d, i, atype, n):  # process_rdata's name walks (dns.cpp:250-320) for the first answer
    if atype in (2, 5, 12, 39):  # NS, CNAME, PTR, DNAME
        _get_name(d, i, n)
    elif atype == 6:  # SOA
        _get_name(d, i, n)
        i += _get_name_length(d, i, n)
        _get_name(d, i, n)
        _get_name_length(d, i, n)
    elif atype == 15:  # MX: preference, then the exchange name
        _get_name(d, i + 2, n)


def dns_valid(payload, tcp):
    """parse_dns (dns.cpp:429-660): False when it would return false (or throw)."""
    d = payload
    n = len(d)
    if tcp:
        n = (n - 2) & 0xFFFFFFFF
        if ((_b(d, 0) << 8) | _b(d, 1)) != n:
            return False
        d = d[2:]
    if n < 12:
        return False
    be16 = lambda i: (_b(d, i) << 8) | _b(d, i + 1)  # noqa: E731
    qd, an, ns, ar = be16(4), be16(6), be16(8), be16(10)
    i = 12
    try:
        for _ in range(qd):
            _get_name(d, i, n)
            i += _get_name_length(d, i, n)
            if i + 4 > n:
                return True
            i += 4
        for k in range(an):
            i += _get_name_length(d, i, n)
            if i + 10 > n or i + 10 + be16(i + 8) > n:
                return True
            atype, rdl = be16(i), be16(i + 8)
            i += 10
            if k == 0:
                _rdata(d, i, atype, n)
            i += rdl
        for _ in range(ns + ar):
            i += _get_name_length(d, i, n)
            if i + 10 > n or i + 10 + be16(i + 8) > n:
                return True
            i += 10 + be16(i + 8)
    except _Throw:
        return False
    return True


class DnsFlush(PyPlugin):
    ports = (53,)

    def _dns(self, rec, p, data):
        return dns_valid(data, int(p["ip_proto"]) == 6)

    def post_create(self, rec, p, data):
        if 53 in (int(p["src_port"]), int(p["dst_port"])):
            if self._dns(rec, p, data):
                rec["ext"] = 1  # RecordExtDNS attached
                return FLOW_FLUSH
        return 0

    def post_update(self, rec, p, data):
        if 53 in (int(p["src_port"]), int(p["dst_port"])):
            if rec["ext"] == 0:
                if self._dns(rec, p, data):
                    rec["ext"] = 1
                    return FLOW_FLUSH
                return 0
            return FLOW_FLUSH  # parse_dns into the existing extension, then flush
        return 0


# ---- HTTP -----------------------------------------------------------------------------------
METHODS = (b"GET ", b"POST", b"PUT ", b"HEAD", b"DELE", b"TRAC", b"OPTI", b"CONN", b"PATC")


def _request_line(data):
    """parse_http_request's checks up to the method copy (http.cpp:233-290)."""
    sp = data.find(b" ")
    if sp < 0:
        return False
    sp2 = data.find(b" ", sp + 1)
    return sp2 >= 0 and data[sp2 + 1:sp2 + 5] == b"HTTP"


def _response_line(data):
    """parse_http_response's checks up to the code (http.cpp:400-445)."""
    sp = data.find(b" ")
    if sp < 0:
        return False
    sp2 = data.find(b" ", sp + 1)
    if sp2 < 0:
        return False
    try:
        return int(data[sp + 1:sp2]) > 0
    except ValueError:
        return False


class HttpReinsert(PyPlugin):
    proto_mask = 1
    prefixes = METHODS + (b"HTTP",)
    REQ, RESP = 2, 4  # ext bits: request / response stored (bit 0: extension present)

    def _kind(self, data):
        if len(data) >= 4 and data[:4] in METHODS:
            return "req"
        if len(data) >= 4 and data[:4] == b"HTTP":
            return "resp"
        return None

    def post_create(self, rec, p, data):
        k = self._kind(data)
        if k == "req" and _request_line(data):
            rec["ext"] = 1 | self.REQ
        elif k == "resp" and _response_line(data):
            rec["ext"] = 1 | self.RESP
        return 0

    def pre_update(self, rec, p, data):
        k = self._kind(data)
        if k is None:
            return 0
        ext = int(rec["ext"])
        bit, ok = (self.REQ, _request_line(data)) if k == "req" else (self.RESP, _response_line(data))
        if not ext:
            if ok:
                rec["ext"] = 1 | bit
            return 0
        if ok and ext & bit:
            return FLOW_FLUSH_WITH_REINSERT  # flow_flush: the flow already holds one
        if ok:
            rec["ext"] = ext | bit
        return 0


# ---- NTP ------------------------------------------------------------------------------------
class NtpFlush(PyPlugin):
    """ntp.cpp:80-90: post_create on a port-123 packet always returns FLOW_FLUSH."""
    ports = (123,)

    def post_create(self, rec, p, data):
        if 123 in (int(p["src_port"]), int(p["dst_port"])):
            rec["ext"] = 1
            return FLOW_FLUSH
        return 0


# ---- SIP ------------------------------------------------------------------------------------
def _le32(s):
    return int.from_bytes(s, "little")


SIP_T1 = {_le32(b"REGI"): 5, _le32(b"INVI"): 1, _le32(b"OPTI"): 6, _le32(b"NOTI"): 8, _le32(b"CANC"): 3,
          _le32(b"INFO"): 9}
SIP_T2 = {_le32(b"SIP/"): 99, _le32(b"ACK "): 2, _le32(b"BYE "): 4, _le32(b"SUBS"): 10, _le32(b"PUBL"): 7}


def _sip_filter(first, test):
    """sip.cpp:125-135 on amd64: uint32 check against the 64-bit MAGIC_BITS (sip.hpp:293-296)."""
    check = (first ^ test) & 0xFFFFFFFF
    t = ((check + 0x7efefefe7efefeff) & 0xFFFFFFFFFFFFFFFF) ^ (~check & 0xFFFFFFFF)
    return (t & 0x8101010181010100) != 0


def sip_msg_type(d):
    """SIPPlugin::parse_msg_type (sip.cpp:107-185): 0 = SIP_MSG_TYPE_INVALID."""
    if len(d) < 64:  # payload_len == 0 or < SIP_MIN_MSG_LEN
        return 0
    first = _le32(d[0:4])
    if _sip_filter(first, _le32(b"IATI")):
        t = SIP_T1.get(first)
        if t == 6:
            return 6 if d[4:8] == b"ONS " and d[8:12] == b"sip:" else 0
        if t == 8:
            return 0 if d[4:8] == b"FY *" and d[8:12] == b" HTT" else 8
        if t:
            return t
    if _sip_filter(first, _le32(b"SIB ")):
        t = SIP_T2.get(first)
        if t:
            return t
    return 0


class SipReinsert(PyPlugin):
    """sip.cpp:66-95: pre_update on a SIP message returns FLOW_FLUSH_WITH_REINSERT."""
    prefixes = (b"REGI", b"INVI", b"OPTI", b"NOTI", b"CANC", b"INFO", b"SIP/", b"ACK ", b"BYE ", b"SUBS", b"PUBL")

    def post_create(self, rec, p, data):
        if sip_msg_type(data):
            rec["ext"] = 1
        return 0

    def pre_update(self, rec, p, data):
        return FLOW_FLUSH_WITH_REINSERT if sip_msg_type(data) else 0
