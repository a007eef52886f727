"""Comparison helpers for flow-record multisets (parity contract)."""
from collections import Counter

import numpy as np

# every field of ipxg_flow_record except end_reason (secondary: it depends on when the
# reference's per-packet sweep happens to visit the slot) and the reserved bytes
CONTRACT_FIELDS = ["flow_hash", "time_first_sec", "time_first_usec", "time_last_sec",
                   "time_last_usec", "src_bytes", "dst_bytes", "src_packets", "dst_packets",
                   "src_tcp_flags", "dst_tcp_flags", "ip_version", "ip_proto", "src_port",
                   "dst_port", "src_ip", "dst_ip", "src_mac", "dst_mac", "vlan_id"]


def rec_key(r, fields=CONTRACT_FIELDS):
    out = []
    for f in fields:
        v = r[f]
        out.append(bytes(v) if isinstance(v, np.ndarray) else int(v))
    return tuple(out)


def multiset(recs, fields=CONTRACT_FIELDS):
    return Counter(rec_key(r, fields) for r in recs)


def diff(a, b, fields=CONTRACT_FIELDS, limit=5):
    """Human-readable difference of two record multisets ('' when equal)."""
    ma, mb = multiset(a, fields), multiset(b, fields)
    if ma == mb:
        return ""
    only_a = list((ma - mb).elements())[:limit]
    only_b = list((mb - ma).elements())[:limit]
    lines = ["%d vs %d records; only in first: %d, only in second: %d"
             % (len(a), len(b), sum((ma - mb).values()), sum((mb - ma).values()))]
    for x in only_a:
        lines.append("  - " + repr(dict(zip(fields, x))))
    for x in only_b:
        lines.append("  + " + repr(dict(zip(fields, x))))
    return "\n".join(lines)
