"""A small IPFIX (RFC 7011) message-stream decoder for the tests: message headers, template
sets, data sets decoded through their templates into FLOW_DTYPE records (the basic templates'
fields only).  Independent of the engine and of the oracle: it checks the structure every
message must have (lengths, set padding, sequence numbers) and gives back the records."""
import struct

import numpy as np

from pcaputil import FLOW_DTYPE

# (enterprise, element id) -> how a basic-template field lands in a FLOW_DTYPE record
_EPOCH = 2208988800


def _ntp_to_tv(v):
    sec = (v >> 32) - _EPOCH
    frac = v & 0xFFFFFFFF
    # MK_NTP_TS: frac = floor(usec * 2^32 / 1e6), so usec = ceil(frac * 1e6 / 2^32)
    usec = (frac * 1000000 + (1 << 32) - 1) >> 32
    return sec & 0xFFFFFFFF, usec


def decode(stream, templates=None):
    """-> (messages [dict], templates {id: [(en, id, len)]}, records FLOW_DTYPE array,
    per-record message index, dir_bit_field values seen).  templates: known from an earlier
    part of the session."""
    b = bytes(stream)
    o = 0
    msgs, recs, where, dirs = [], [], [], set()
    templates = dict(templates or {})
    while o < len(b):
        ver, length, etime, seq, odid = struct.unpack(">HHIII", b[o:o + 16])
        assert ver == 10, "not an IPFIX message at %d" % o
        assert 16 <= length and o + length <= len(b)
        m = {"offset": o, "length": length, "export_time": etime, "sequence": seq, "odid": odid, "sets": [],
             "records": 0}
        p = o + 16
        while p < o + length:
            sid, slen = struct.unpack(">HH", b[p:p + 4])
            assert slen >= 4 and p + slen <= o + length
            body = b[p + 4:p + slen]
            m["sets"].append((sid, slen))
            if sid == 2:  # template set
                q = 0
                while q + 4 <= len(body):
                    tid, cnt = struct.unpack(">HH", body[q:q + 4])
                    q += 4
                    fields = []
                    for _ in range(cnt):
                        eid, flen = struct.unpack(">HH", body[q:q + 4])
                        q += 4
                        en = 0
                        if eid & 0x8000:
                            en = struct.unpack(">I", body[q:q + 4])[0]
                            q += 4
                        fields.append((en, eid & 0x7FFF, flen))
                    templates[tid] = fields
            elif sid >= 256:
                fields = templates[sid]
                rl = sum(f[2] for f in fields)
                assert len(body) % rl == 0, "data set of template %d: %d bytes" % (sid, len(body))
                for k in range(len(body) // rl):
                    r, d = _record(body[k * rl:(k + 1) * rl], fields)
                    recs.append(r)
                    where.append(len(msgs))
                    dirs.add(d)
                    m["records"] += 1
            p += slen
        assert p == o + length
        msgs.append(m)
        o += length
    out = np.zeros(len(recs), dtype=FLOW_DTYPE)
    for i, r in enumerate(recs):
        for k, v in r.items():
            out[i][k] = v
    return msgs, templates, out, np.array(where, dtype=np.int64), dirs


def _record(raw, fields):
    r = {}
    d = None
    q = 0
    for en, eid, ln in fields:
        v = raw[q:q + ln]
        q += ln
        u = int.from_bytes(v, "big")
        key = (en, eid)
        if key == (0, 136):
            r["end_reason"] = u
        elif key == (0, 1):
            r["src_bytes"] = u
        elif key == (29305, 1):
            r["dst_bytes"] = u
        elif key == (0, 2):
            r["src_packets"] = u
        elif key == (29305, 2):
            r["dst_packets"] = u
        elif key == (0, 154):
            r["time_first_sec"], r["time_first_usec"] = _ntp_to_tv(u)
        elif key == (0, 155):
            r["time_last_sec"], r["time_last_usec"] = _ntp_to_tv(u)
        elif key == (0, 60):
            r["ip_version"] = u
        elif key == (0, 4):
            r["ip_proto"] = u
        elif key == (0, 6):
            r["src_tcp_flags"] = u
        elif key == (29305, 6):
            r["dst_tcp_flags"] = u
        elif key == (0, 7):
            r["src_port"] = u
        elif key == (0, 11):
            r["dst_port"] = u
        elif key == (0, 10):
            d = u
        elif key in ((0, 8), (0, 27)):
            a = np.zeros(16, np.uint8)
            a[:ln] = np.frombuffer(v, np.uint8)
            r["src_ip"] = a
        elif key in ((0, 12), (0, 28)):
            a = np.zeros(16, np.uint8)
            a[:ln] = np.frombuffer(v, np.uint8)
            r["dst_ip"] = a
        elif key == (0, 56):
            r["src_mac"] = np.frombuffer(v, np.uint8)
        elif key == (0, 80):
            r["dst_mac"] = np.frombuffer(v, np.uint8)
    return r, d


# the record fields the basic templates carry (flow_hash and vlan_id are not exported)
BASIC_FIELDS = ["end_reason", "src_bytes", "dst_bytes", "src_packets", "dst_packets", "time_first_sec",
                "time_first_usec", "time_last_sec", "time_last_usec", "ip_version", "ip_proto", "src_tcp_flags",
                "dst_tcp_flags", "src_port", "dst_port", "src_ip", "dst_ip", "src_mac", "dst_mac"]


def basic_view(recs):
    """Records reduced to the exported fields (IPv4 addresses past byte 4 zeroed), as a sortable
    list of tuples."""
    out = []
    for r in recs:
        t = []
        for f in BASIC_FIELDS:
            v = r[f]
            if f in ("src_ip", "dst_ip"):
                v = bytes(v[:4]) + b"\0" * 12 if int(r["ip_version"]) == 4 else bytes(v)
            elif f in ("src_mac", "dst_mac"):
                v = bytes(v)
            else:
                v = int(v)
            t.append(v)
        out.append(tuple(t))
    return sorted(out)
