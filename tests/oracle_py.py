"""ctypes wrapper around oracle/liboracle.so -- the CPU checker (test infrastructure).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes
import os

import numpy as np

from pcaputil import FLOW_DTYPE, PARSED_DTYPE, STATS_FIELDS, VLAN_IDS, VLAN_STATS_DTYPE

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_ROOT, "oracle", "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        vp, u8p = ctypes.c_void_p, ctypes.c_void_p
        L.oracle_xxh64.restype = ctypes.c_uint64
        L.oracle_xxh64.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint64]
        L.oracle_xxh64_batch.argtypes = [vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64, vp]
        L.oracle_parse.restype = ctypes.c_int
        L.oracle_parse.argtypes = [u8p, ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_uint32, vp,
                                   ctypes.POINTER(ctypes.c_int)]
        L.oracle_cache_new.restype = vp
        L.oracle_cache_new.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_int, ctypes.c_int,
                                                               ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_cache_free.argtypes = [vp]
        L.oracle_cache_run.argtypes = [vp, u8p, vp, ctypes.c_size_t, ctypes.c_uint32]
        L.oracle_cache_export_expired.argtypes = [vp, ctypes.c_int64]
        L.oracle_cache_finish.argtypes = [vp]
        L.oracle_cache_pending.restype = ctypes.c_size_t
        L.oracle_cache_pending.argtypes = [vp]
        L.oracle_cache_take.restype = ctypes.c_size_t
        L.oracle_cache_take.argtypes = [vp, vp, ctypes.c_size_t]
        L.oracle_ipfix_basic.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint32, vp, vp]
        L.oracle_cache_stats.argtypes = [vp, vp]
        L.oracle_cache_parser_stats.argtypes = [vp, vp, vp, vp]
        L.oracle_cache_add_plugin.argtypes = [vp, vp]
        L.oracle_ipfix_export.restype = ctypes.c_size_t
        L.oracle_ipfix_export.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_bench_mt.restype = ctypes.c_double
        L.oracle_bench_mt.argtypes = [vp, vp, vp, vp, ctypes.c_int, vp, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        _LIB = L
    return _LIB


def xxh64(data: bytes, seed=0):
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    return lib().oracle_xxh64(buf, len(data), seed)


def xxh64_batch(keys: np.ndarray, keylen: int, seed=0):
    """XXH64 of each keylen-byte key of the flat uint8 array keys (as Engine.xxh64, on the CPU)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n = len(keys) // keylen
    out = np.empty(n, dtype=np.uint64)
    lib().oracle_xxh64_batch(keys.ctypes.data, keylen, n, seed, out.ctypes.data)
    return out


def parse(frame: bytes, caplen=None, wirelen=None, datalink=1, sec=0, usec=0):
    """Returns (parsed record as numpy void, beyond_caplen flag)."""
    out = np.zeros(1, dtype=PARSED_DTYPE)
    cl = len(frame) if caplen is None else caplen
    wl = cl if wirelen is None else wirelen
    buf = ctypes.create_string_buffer(bytes(frame), max(len(frame), 1))
    beyond = ctypes.c_int(0)
    lib().oracle_parse(buf, cl, wl, sec, usec, datalink, out.ctypes.data, ctypes.byref(beyond))
    return out[0], bool(beyond.value)


def parse_batch(arena, desc, datalink=1):
    out = np.zeros(len(desc), dtype=PARSED_DTYPE)
    beyond = np.zeros(len(desc), dtype=bool)
    L = lib()
    rec = np.zeros(1, dtype=PARSED_DTYPE)
    b = ctypes.c_int(0)
    base = arena.ctypes.data
    for i, d in enumerate(desc):
        L.oracle_parse(ctypes.c_void_p(base + int(d["offset"])), int(d["caplen"]),
                       int(d["wirelen"]), int(d["ts_sec"]), int(d["ts_usec"]), datalink,
                       rec.ctypes.data, ctypes.byref(b))
        out[i] = rec[0]
        beyond[i] = bool(b.value)
    return out, beyond


class OracleCache:
    """NHTFlowCache restatement; defaults are the reference's (cache.hpp:52-64, :91-102)."""

    def __init__(self, cache_exp=17, line_exp=4, active=300, inactive=30, split_biflow=False,
                 frag_enable=True, frag_size=10007, frag_timeout=3):
        self._c = lib().oracle_cache_new(cache_exp, line_exp, active, inactive,
                                         int(split_biflow), int(frag_enable), frag_size,
                                         frag_timeout)
        if not self._c:
            raise MemoryError("oracle_cache_new failed")

    def run(self, arena, desc, datalink=1):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        desc = np.ascontiguousarray(desc)
        lib().oracle_cache_run(self._c, arena.ctypes.data, desc.ctypes.data, len(desc), datalink)

    def export_expired(self, ts):
        lib().oracle_cache_export_expired(self._c, ts)

    def finish(self):
        lib().oracle_cache_finish(self._c)

    def take(self):
        n = lib().oracle_cache_pending(self._c)
        out = np.zeros(n, dtype=FLOW_DTYPE)
        if n:
            lib().oracle_cache_take(self._c, out.ctypes.data, n)
        return out

    def stats(self):
        arr = (ctypes.c_uint64 * len(STATS_FIELDS))()
        lib().oracle_cache_stats(self._c, arr)
        return dict(zip(STATS_FIELDS, list(arr)))

    def add_plugin(self, plugin):
        """The same ipxg_plugin callbacks the engine's bridge calls (ctypes Plugin struct)."""
        lib().oracle_cache_add_plugin(self._c, ctypes.addressof(plugin))

    def parser_stats(self):
        """(tcp port frequencies, udp port frequencies, VlanStats per VLAN id)"""
        tcp = np.zeros(65536, dtype=np.uint64)
        udp = np.zeros(65536, dtype=np.uint64)
        vl = np.zeros(VLAN_IDS, dtype=VLAN_STATS_DTYPE)
        lib().oracle_cache_parser_stats(self._c, tcp.ctypes.data, udp.ctypes.data, vl.ctypes.data)
        return tcp, udp, vl

    def close(self):
        if self._c:
            lib().oracle_cache_free(self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ipfix_basic(recs, dir_bit_field=0):
    """IPFIXExporter::fill_basic_flow restated (oracle): (bytes uint8 array, offsets[n+1])."""
    recs = np.ascontiguousarray(recs, dtype=FLOW_DTYPE)
    out = np.zeros(max(len(recs), 1) * 105, dtype=np.uint8)
    off = np.zeros(len(recs) + 1, dtype=np.uint64)
    lib().oracle_ipfix_basic(recs.ctypes.data, len(recs), dir_bit_field, out.ctypes.data, off.ctypes.data)
    return out[: int(off[-1])], off


class IpfixExporterState(ctypes.Structure):
    """ipxg_ipfix_exporter (include/ipxg.h) for the oracle's exporter."""
    _fields_ = [("odid", ctypes.c_uint32), ("dir_bit_field", ctypes.c_uint32), ("export_time", ctypes.c_uint32),
                ("sequence", ctypes.c_uint32), ("mtu", ctypes.c_uint16), ("templates_sent", ctypes.c_uint16)]


def ipfix_exporter(odid=0, dir_bit_field=0, export_time=0, mtu=1458):
    x = IpfixExporterState()
    x.odid, x.dir_bit_field, x.export_time, x.mtu = odid, dir_bit_field, export_time, mtu
    return x


def ipfix_export(x, recs):
    """IPFIXExporter::export_flow per record in the given order, then flush() (oracle): (bytes,
    messages); x (IpfixExporterState) is updated like the exporter's state."""
    recs = np.ascontiguousarray(recs, dtype=FLOW_DTYPE)
    cap = 196 + len(recs) * 125 + 64
    out = np.zeros(cap, dtype=np.uint8)
    nm = ctypes.c_size_t()
    n = lib().oracle_ipfix_export(ctypes.byref(x), recs.ctypes.data if len(recs) else None, len(recs),
                                  out.ctypes.data, cap, ctypes.byref(nm))
    assert n != ctypes.c_size_t(-1).value
    return out[:n], nm.value


def run_capture(arena, desc, datalink=1, finish=True, plugins=(), **kw):
    c = OracleCache(**kw)
    for pl in plugins:
        c.add_plugin(pl)
    c.run(arena, desc, datalink)
    if finish:
        c.finish()
    recs = c.take()
    st = c.stats()
    c.close()
    return recs, st


def bench_mt(arena, desc, shard, nshards, cpus=None, cache_exp=17, datalink=1):
    """oracle/cpu_baseline.c: nshards pinned threads, thread k runs parse + put_pkt + finish
    over the packets with shard == k (in arrival order) with its own cache.  Returns
    (wall seconds, records, NO_RES exports)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    order = np.argsort(shard, kind="stable")
    grouped = np.ascontiguousarray(desc[order])
    count = np.bincount(shard, minlength=nshards).astype(np.uint64)
    first = np.concatenate([[0], np.cumsum(count)[:-1]]).astype(np.uint64)
    cp = None if cpus is None else np.ascontiguousarray(cpus, dtype=np.int32)
    rec, nr = ctypes.c_uint64(), ctypes.c_uint64()
    dt = lib().oracle_bench_mt(arena.ctypes.data, grouped.ctypes.data, first.ctypes.data, count.ctypes.data,
                               nshards, None if cp is None else cp.ctypes.data, cache_exp, datalink,
                               ctypes.byref(rec), ctypes.byref(nr))
    if dt < 0:
        raise RuntimeError("oracle_bench_mt failed")
    return dt, rec.value, nr.value
