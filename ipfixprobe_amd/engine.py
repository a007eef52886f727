"""ctypes bindings of libipxg (include/ipxg.h) for the tests and bench.py.

The product surface above the C-ABI is C++ (ipfixprobe_amd/host: the GpuFlowCache storage
plugin and the ipxg_probe tool).  This module is plumbing: it loads the in-tree
libipxg.so -- and fails loudly if it is missing or no GPU is present; there is no CPU
fallback anywhere in the product path.
"""
import atexit
import ctypes
import os
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# IPXG_LIB: an alternative build of the same library (tuning experiments, tools/variants.sh)
LIB_PATH = os.environ.get("IPXG_LIB") or os.path.join(_HERE, "libipxg.so")

DLT_EN10MB, DLT_RAW, DLT_LINUX_SLL, DLT_LINUX_SLL2 = 1, 12, 113, 276
BATCH_DEVICE = 0x1
BATCH_ASYNC = 0x2
BATCH_OFFSET16 = 0x4  # descriptor offsets count 16-byte units (arenas up to 64 GiB)
MAX_BATCH = 16 * 1024 * 1024 - 1

DESC_DTYPE = np.dtype([("offset", "<u4"), ("caplen", "<u2"), ("wirelen", "<u2"),
                       ("ts_sec", "<u4"), ("ts_usec", "<u4")])
FLOW_DTYPE = np.dtype([
    ("flow_hash", "<u8"),
    ("time_first_sec", "<u4"), ("time_first_usec", "<u4"),
    ("time_last_sec", "<u4"), ("time_last_usec", "<u4"),
    ("src_bytes", "<u8"), ("dst_bytes", "<u8"),
    ("src_packets", "<u4"), ("dst_packets", "<u4"),
    ("src_tcp_flags", "u1"), ("dst_tcp_flags", "u1"), ("ip_version", "u1"), ("ip_proto", "u1"),
    ("src_port", "<u2"), ("dst_port", "<u2"),
    ("src_ip", "u1", (16,)), ("dst_ip", "u1", (16,)),
    ("src_mac", "u1", (6,)), ("dst_mac", "u1", (6,)),
    ("vlan_id", "<u2"), ("end_reason", "u1"), ("reserved0", "u1"), ("reserved", "u1", (8,)),
    ("ext", "<u8"), ("reserved2", "u1", (8,)),
])
PARSED_DTYPE = np.dtype([
    ("valid", "u1"), ("ip_version", "u1"), ("ip_proto", "u1"), ("tcp_flags", "u1"),
    ("ethertype", "<u2"), ("ip_len", "<u2"), ("src_port", "<u2"), ("dst_port", "<u2"),
    ("frag_off", "<u2"), ("more_fragments", "u1"), ("ip_ttl", "u1"),
    ("vlan_id", "<u4"), ("frag_id", "<u4"), ("mpls_top", "<u4"), ("tcp_mss", "<u4"),
    ("tcp_options", "<u8"),
    ("src_ip", "u1", (16,)), ("dst_ip", "u1", (16,)),
    ("src_mac", "u1", (6,)), ("dst_mac", "u1", (6,)),
    ("ip_tos", "u1"), ("ip_flags", "u1"), ("tcp_window", "<u2"),
    ("tcp_seq", "<u4"), ("tcp_ack", "<u4"),
    ("hash_fwd", "<u8"), ("hash_inv", "<u8"),
    ("payload_off", "<u2"), ("payload_len", "<u2"), ("reserved2", "<u4"),
])
STATS_FIELDS = [
    "seen_packets", "parsed_packets", "unknown_packets", "ipv4_packets", "ipv6_packets",
    "tcp_packets", "udp_packets", "mpls_packets", "pppoe_packets", "trill_packets",
    "vlan_packets", "ipv4_bytes", "ipv6_bytes", "end_inactive", "end_active", "end_eof",
    "end_forced", "end_no_res", "flows_in_cache", "total_exported", "keyless_packets",
    "fragmented_packets", "fragments_filled", "complex_flows", "table_capacity",
    "table_rehashes", "batches", "spilled_packets", "slow_path_packets",
    "aggregated_packets", "walked_packets", "flows_1_packet", "flows_2_5_packets", "flows_6_10_packets",
    "flows_11_20_packets", "flows_21_50_packets", "flows_51_plus_packets",
]


class Config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "cache_exp", "line_exp", "active_s", "inactive_s", "split_biflow", "frag_enable",
        "frag_size", "frag_timeout_s")] + [("device_id", ctypes.c_int32)] + \
        [(n, ctypes.c_uint32) for n in ("batch_pkts", "datalink", "flags")]


class Batch(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("arena_len", ctypes.c_uint64),
                ("desc", ctypes.c_void_p), ("n", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class Timing(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in ("ingest_ms", "ingest_slow_ms", "reduce_ms", "fin_ms",
                                               "finalize_ms", "slow_ms", "finish_ms")] + \
        [(n, ctypes.c_uint64) for n in ("ingest_launches", "reduce_launches", "finalize_launches",
                                        "slow_launches", "finish_launches", "ingest_packets")] + \
        [("plugin_ms", ctypes.c_double)] + [(n, ctypes.c_uint64) for n in ("plugin_flows", "plugin_packets",
                                                                             "plugin_bytes", "plugin_extra_bytes",
                                                                             "plugin_overlapped", "slow_redos",
                                                                             "plugin_d2h_bytes", "ex_compactions")]


class Capture(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("arena_len", ctypes.c_uint64),
                ("desc", ctypes.c_void_p), ("n", ctypes.c_uint32), ("datalink", ctypes.c_uint32)]


IPFIX_V4_LEN, IPFIX_V6_LEN = 81, 105  # IPXG_IPFIX_V4_LEN / _V6_LEN


class IpfixExporter(ctypes.Structure):
    """ipxg_ipfix_exporter: the IPFIX exporter's state (include/ipxg.h)."""
    _fields_ = [("odid", ctypes.c_uint32), ("dir_bit_field", ctypes.c_uint32), ("export_time", ctypes.c_uint32),
                ("sequence", ctypes.c_uint32), ("mtu", ctypes.c_uint16), ("templates_sent", ctypes.c_uint16)]

EXPORTED_SYMBOLS = [
    "ipxg_config_default", "ipxg_config_parse", "ipxg_create", "ipxg_destroy",
    "ipxg_last_error", "ipxg_stream", "ipxg_submit", "ipxg_expire", "ipxg_finish",
    "ipxg_reset", "ipxg_pending_exports", "ipxg_poll_exports", "ipxg_device_exports",
    "ipxg_clear_exports", "ipxg_get_stats", "ipxg_parse_batch", "ipxg_xxh64_batch",
    "ipxg_capture_load", "ipxg_capture_free", "ipxg_profile", "ipxg_get_timing",
    "ipxg_probe_counters", "ipxg_ipfix_basic", "ipxg_poll_ipfix", "ipxg_ipfix_exporter_init",
    "ipxg_ipfix_bound", "ipxg_ipfix_export", "ipxg_poll_ipfix_messages", "ipxg_device_ipfix_messages",
    "ipxg_device_ipfix_counts", "ipxg_ipfix_stream",
    "ipxg_parser_stats", "ipxg_top_ports", "ipxg_add_plugin", "ipxg_set_walk_threads",
    "ipxg_demux", "ipxg_demux_arena_bytes", "ipxg_demux_split",
]

FLOW_FLUSH = 0x1
FLOW_FLUSH_WITH_REINSERT = 0x3


class PacketView(ctypes.Structure):
    """include/ipxg.h ipxg_packet_view: what a process-plugin hook sees of the packet."""
    _fields_ = [("pkt", ctypes.c_void_p), ("data", ctypes.POINTER(ctypes.c_uint8)), ("caplen", ctypes.c_uint32),
                ("wirelen", ctypes.c_uint32), ("ts_sec", ctypes.c_uint32), ("ts_usec", ctypes.c_uint32),
                ("index", ctypes.c_uint32), ("source_pkt", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 3)]


PRE_CREATE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(PacketView))
FLOW_HOOK_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(PacketView))
PRE_EXPORT_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)
ERROR_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p)  # const char* (a C string the plugin keeps)
PLUGIN_ERROR = -1  # IPXG_PLUGIN_ERROR: a hook's PluginError


class Plugin(ctypes.Structure):
    """include/ipxg.h ipxg_plugin: a process plugin's pre-classifier rule and hooks."""
    _fields_ = [("ctx", ctypes.c_void_p), ("proto_mask", ctypes.c_uint32), ("n_ports", ctypes.c_uint32),
                ("ports", ctypes.c_uint16 * 16), ("n_prefixes", ctypes.c_uint32),
                ("prefix_len", ctypes.c_uint8 * 16), ("prefix", (ctypes.c_uint8 * 16) * 16),
                ("pre_create", PRE_CREATE_FN), ("post_create", FLOW_HOOK_FN), ("pre_update", FLOW_HOOK_FN),
                ("post_update", FLOW_HOOK_FN), ("pre_export", PRE_EXPORT_FN),
                ("masked", ctypes.c_uint32), ("follow_packets", ctypes.c_uint32),
                ("prefix_mask", (ctypes.c_uint8 * 16) * 16),
                ("copy_ctx", ctypes.c_void_p), ("free_ctx", ctypes.c_void_p),  # ABI 3 (C function pointers)
                ("error", ERROR_FN),  # ABI 4
                ("all_packets", ctypes.c_uint32),  # ABI 6
                ("follow_bytes", ctypes.c_uint32)]  # ABI 7

# ipxg_vlan_stats (VlanStats, parser-stats.hpp:126-160) and ipxg_port_stat (TopPorts::PortStats)
VLAN_STATS_DTYPE = np.dtype([("ipv4_packets", "<u8"), ("ipv6_packets", "<u8"), ("ipv4_bytes", "<u8"),
                             ("ipv6_bytes", "<u8"), ("tcp_packets", "<u8"), ("udp_packets", "<u8"),
                             ("total_packets", "<u8"), ("total_bytes", "<u8"),
                             ("hist_packets", "<u8", (10,)), ("hist_bytes", "<u8", (10,))])
PORT_STAT_DTYPE = np.dtype([("port", "<u2"), ("protocol", "u1"), ("reserved", "u1", (5,)), ("frequency", "<u8")])
VLAN_IDS = 4096

_LIB = None


class IpxgError(RuntimeError):
    pass


def lib():
    """Load the in-tree libipxg.so.  Raises if it has not been built."""
    global _LIB
    if _LIB is None:
        try:
            # torch ships its own libamdhip64.so.7; loading it first makes libipxg bind to
            # that same runtime (identical soname), so one process never holds two HIP
            # runtimes when the tests/bench also use torch for device buffers.
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise IpxgError("libipxg.so not built (%s): run __graft_entry__.build()" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
        L.ipxg_config_default.argtypes = [ctypes.POINTER(Config)]
        L.ipxg_config_parse.argtypes = [ctypes.c_char_p, ctypes.POINTER(Config)]
        L.ipxg_create.argtypes = [ctypes.POINTER(Config), ctypes.POINTER(vp)]
        L.ipxg_destroy.argtypes = [vp]
        L.ipxg_last_error.argtypes = [vp]
        L.ipxg_last_error.restype = ctypes.c_char_p
        L.ipxg_stream.argtypes = [vp]
        L.ipxg_stream.restype = vp
        L.ipxg_submit.argtypes = [vp, ctypes.POINTER(Batch)]
        L.ipxg_expire.argtypes = [vp, ctypes.c_int64]
        L.ipxg_finish.argtypes = [vp]
        L.ipxg_reset.argtypes = [vp]
        L.ipxg_pending_exports.argtypes = [vp, ctypes.POINTER(sz)]
        L.ipxg_poll_exports.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
        L.ipxg_device_exports.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(sz)]
        L.ipxg_clear_exports.argtypes = [vp]
        L.ipxg_get_stats.argtypes = [vp, vp]
        L.ipxg_parse_batch.argtypes = [vp, ctypes.POINTER(Batch), vp]
        L.ipxg_xxh64_batch.argtypes = [vp, vp, u32, u32, ctypes.c_uint64, vp]
        L.ipxg_capture_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.POINTER(Capture))]
        L.ipxg_capture_free.argtypes = [ctypes.POINTER(Capture)]
        L.ipxg_profile.argtypes = [vp, ctypes.c_int]
        L.ipxg_get_timing.argtypes = [vp, ctypes.POINTER(Timing)]
        L.ipxg_probe_counters.argtypes = [vp, vp]
        L.ipxg_ipfix_basic.argtypes = [vp, vp, sz, u32, vp, vp]
        L.ipxg_poll_ipfix.argtypes = [vp, u32, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]
        px = ctypes.POINTER(IpfixExporter)
        L.ipxg_ipfix_exporter_init.argtypes = [px]
        L.ipxg_ipfix_exporter_init.restype = None
        L.ipxg_ipfix_bound.argtypes = [ctypes.c_uint64]
        L.ipxg_ipfix_bound.restype = ctypes.c_uint64
        L.ipxg_ipfix_export.argtypes = [vp, px, vp, sz, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]
        L.ipxg_poll_ipfix_messages.argtypes = [vp, px, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(sz),
                                               ctypes.POINTER(sz)]
        L.ipxg_parser_stats.argtypes = [vp, vp, vp, vp]
        L.ipxg_add_plugin.argtypes = [vp, ctypes.POINTER(Plugin)]
        L.ipxg_set_walk_threads.argtypes = [vp, u32]
        L.ipxg_top_ports.argtypes = [vp, sz, vp, ctypes.POINTER(sz)]
        L.ipxg_device_ipfix_messages.argtypes = [vp, px, ctypes.POINTER(vp), ctypes.POINTER(sz),
                                                 ctypes.POINTER(sz), ctypes.POINTER(sz)]
        L.ipxg_device_ipfix_counts.argtypes = [vp, ctypes.POINTER(vp)]
        L.ipxg_ipfix_stream.argtypes = [vp]
        L.ipxg_ipfix_stream.restype = vp
        L.ipxg_demux.argtypes = [ctypes.POINTER(Batch), u32, u32, vp, vp]
        L.ipxg_demux_arena_bytes.argtypes = [ctypes.POINTER(Batch), vp, u32]
        L.ipxg_demux_arena_bytes.restype = ctypes.c_uint64
        L.ipxg_demux_split.argtypes = [ctypes.POINTER(Batch), vp, u32, vp, vp, ctypes.POINTER(u32)]
        for name in EXPORTED_SYMBOLS:
            if name not in ("ipxg_last_error", "ipxg_stream", "ipxg_ipfix_stream", "ipxg_config_default",
                            "ipxg_demux_arena_bytes",
                            "ipxg_capture_free", "ipxg_ipfix_exporter_init", "ipxg_ipfix_bound"):
                getattr(L, name).restype = ctypes.c_int
        _LIB = L
    return _LIB


STD_LIB_PATH = os.path.join(_HERE, "libipxg_stdplugins.so")
_STD = None


class StdPlugin:
    """A native stand-in process plugin (include/ipxg_stdplugins.h: "dns", "http", "tls", "quic"),
    its ipxg_plugin in .struct (pass it to Engine.add_plugin or the oracle)."""

    def __init__(self, name):
        global _STD
        if _STD is None:
            if not os.path.exists(STD_LIB_PATH):
                raise IpxgError("libipxg_stdplugins.so not built: run __graft_entry__.build()")
            _STD = ctypes.CDLL(STD_LIB_PATH)
            _STD.ipxg_std_plugin.argtypes = [ctypes.c_char_p, ctypes.POINTER(Plugin)]
            _STD.ipxg_std_plugin_free.argtypes = [ctypes.POINTER(Plugin)]
            _STD.ipxg_std_plugin_calls.argtypes = [ctypes.POINTER(Plugin), ctypes.c_void_p]
        self.name = name
        self.struct = Plugin()
        if _STD.ipxg_std_plugin(name.encode(), ctypes.byref(self.struct)):
            raise IpxgError("unknown stand-in plugin %r" % name)

    def calls(self):
        out = np.zeros(6, dtype=np.uint64)
        _STD.ipxg_std_plugin_calls(ctypes.byref(self.struct), out.ctypes.data)
        return dict(zip(("pre_create", "post_create", "pre_update", "post_update", "pre_export", "flushes"),
                        (int(x) for x in out)))

    def __del__(self):
        try:
            _STD.ipxg_std_plugin_free(ctypes.byref(self.struct))
        except Exception:
            pass


def make_config(params: str = "", **kw) -> Config:
    """Reference defaults, then the cache option string, then keyword overrides."""
    cfg = Config()
    lib().ipxg_config_default(ctypes.byref(cfg))
    if params:
        rc = lib().ipxg_config_parse(params.encode(), ctypes.byref(cfg))
        if rc:
            raise IpxgError("invalid option string %r (rc %d)" % (params, rc))
    for k, v in kw.items():
        setattr(cfg, k, int(v))
    return cfg


def load_capture(path):
    """pcap/pcapng -> (arena uint8 ndarray, desc DESC_DTYPE ndarray, datalink) via libipxg."""
    p = ctypes.POINTER(Capture)()
    rc = lib().ipxg_capture_load(os.fsencode(path), ctypes.byref(p))
    if rc:
        raise IpxgError("ipxg_capture_load(%s) failed: %d" % (path, rc))
    c = p.contents
    try:
        arena = np.ctypeslib.as_array(ctypes.cast(c.arena, ctypes.POINTER(ctypes.c_uint8)),
                                      shape=(c.arena_len,)).copy()
        if c.n:
            raw = np.ctypeslib.as_array(ctypes.cast(c.desc, ctypes.POINTER(ctypes.c_uint8)),
                                        shape=(c.n * 16,)).copy()
            desc = raw.view(DESC_DTYPE)
        else:
            desc = np.zeros(0, dtype=DESC_DTYPE)
        return arena, desc, int(c.datalink)
    finally:
        lib().ipxg_capture_free(p)


def demux(arena, desc, n_shards, datalink=DLT_EN10MB, offset16=False):
    """Host symmetric demux (ipxg_demux / ipxg_demux_split): one (arena, desc) batch per shard,
    packets in arrival order, each shard's frames copied into its own arena -- the per-GPU rings
    of the end-to-end multi-GPU path (offsets counted as the input's: offset16, 16-byte units).
    Returns (batches, shard_of)."""
    b = Engine._batch(arena, desc, offset16=offset16)
    n = int(b.n)
    shard_of = np.zeros(n, dtype=np.uint32)
    counts = np.zeros(n_shards, dtype=np.uint32)
    rc = lib().ipxg_demux(ctypes.byref(b), datalink, n_shards, shard_of.ctypes.data, counts.ctypes.data)
    if rc:
        raise IpxgError("ipxg_demux failed: %d" % rc)
    out = []
    for k in range(n_shards):
        nb = int(lib().ipxg_demux_arena_bytes(ctypes.byref(b), shard_of.ctypes.data, k))
        a = np.zeros(max(nb, 16), dtype=np.uint8)
        d = np.zeros(int(counts[k]), dtype=DESC_DTYPE)
        got = ctypes.c_uint32(0)
        rc = lib().ipxg_demux_split(ctypes.byref(b), shard_of.ctypes.data, k, a.ctypes.data, d.ctypes.data,
                                    ctypes.byref(got))
        if rc or got.value != counts[k]:
            raise IpxgError("ipxg_demux_split failed: %d" % rc)
        out.append((a, d))
    return out, shard_of


# Engines still open at interpreter exit are destroyed before the module's objects are: an engine
# frees its walk threads' copies of the registered plugins, which the plugins' owners (StdPlugin,
# the adapter) must outlive -- at exit after an exception the objects would go in any order.
_LIVE = weakref.WeakSet()


@atexit.register
def _close_live_engines():
    for e in list(_LIVE):
        try:
            e.close()
        except Exception:
            pass


class Engine:
    """One ipxg engine (one HIP stream on one device) -- the StoragePlugin-shaped lifecycle:
    submit = put_pkt for a whole batch, expire = export_expired, finish = finish."""

    def __init__(self, params: str = "", **kw):
        self.cfg = make_config(params, **kw)
        h = ctypes.c_void_p()
        rc = lib().ipxg_create(ctypes.byref(self.cfg), ctypes.byref(h))
        if rc:
            raise IpxgError("ipxg_create failed (rc %d): no usable HIP device?" % rc)
        self._h = h
        _LIVE.add(self)

    def _check(self, rc, what):
        if rc:
            msg = lib().ipxg_last_error(self._h).decode(errors="replace")
            err = IpxgError("%s failed (rc %d): %s" % (what, rc, msg))
            err.rc = rc
            raise err

    @property
    def handle(self):
        return self._h

    def stream(self):
        return lib().ipxg_stream(self._h)

    @staticmethod
    def _batch(arena, desc, device=False, asynchronous=False, offset16=False):
        b = Batch()
        if device or hasattr(arena, "data_ptr"):  # torch tensors: on the GPU, or (pinned) host
            b.arena = arena.data_ptr()
            b.arena_len = arena.numel() * arena.element_size()
            b.desc = desc.data_ptr()
            b.n = desc.numel() * desc.element_size() // 16
            b.flags = (BATCH_DEVICE if device else 0) | (BATCH_ASYNC if asynchronous else 0)
            b._keep = (arena, desc)
        else:
            arena = np.ascontiguousarray(arena, dtype=np.uint8)
            desc = np.ascontiguousarray(desc)
            b.arena = arena.ctypes.data
            b.arena_len = arena.nbytes
            b.desc = desc.ctypes.data
            b.n = len(desc)
            b.flags = BATCH_ASYNC if asynchronous else 0
            b._keep = (arena, desc)
        if offset16:
            b.flags |= BATCH_OFFSET16
        return b

    def submit(self, arena, desc, device=False, asynchronous=False, wait_producer=True, offset16=False):
        """offset16: the descriptors' offsets count 16-byte units (IPXG_BATCH_OFFSET16: arenas
        up to 64 GiB, every frame 16-byte aligned).
        asynchronous: may return before the batch is applied; keep the arrays / tensors alive
        and unchanged until the next call on the engine (host batches: pinned memory lets the
        copy overlap the previous batch's kernels).  wait_producer (device
        torch tensors): the engine's stream first waits for the work queued so far on torch's
        current stream (the kernels that wrote the batch) -- the engine's stream is a
        non-blocking stream, unordered with respect to torch's; pass False when the caller has
        synchronised already."""
        if device and wait_producer and hasattr(arena, "data_ptr"):
            import torch
            dev = arena.device
            if getattr(self, "_ext_stream", None) is None:
                self._ext_stream = torch.cuda.ExternalStream(self.stream(), device=dev)
            self._ext_stream.wait_stream(torch.cuda.current_stream(dev))
        b = self._batch(arena, desc, device, asynchronous, offset16)
        self._keep_async = b._keep if asynchronous else None
        self._check(lib().ipxg_submit(self._h, ctypes.byref(b)), "ipxg_submit")

    def submit_all(self, arena, desc, batch=None):
        """Host capture in arrival order, cut into batches of at most `batch` packets."""
        batch = batch or int(self.cfg.batch_pkts)
        for s in range(0, len(desc), batch):
            self.submit(arena, desc[s:s + batch])

    def expire(self, now_sec):
        self._check(lib().ipxg_expire(self._h, int(now_sec)), "ipxg_expire")

    def finish(self):
        self._check(lib().ipxg_finish(self._h), "ipxg_finish")

    def reset(self):
        self._check(lib().ipxg_reset(self._h), "ipxg_reset")

    def pending(self):
        n = ctypes.c_size_t()
        self._check(lib().ipxg_pending_exports(self._h, ctypes.byref(n)), "ipxg_pending_exports")
        return n.value

    def poll(self):
        n = self.pending()
        out = np.zeros(n, dtype=FLOW_DTYPE)
        got = ctypes.c_size_t()
        self._check(lib().ipxg_poll_exports(self._h, out.ctypes.data if n else None, n,
                                            ctypes.byref(got)), "ipxg_poll_exports")
        return out[:got.value]

    def device_exports(self):
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._check(lib().ipxg_device_exports(self._h, ctypes.byref(p), ctypes.byref(n)),
                    "ipxg_device_exports")
        return p.value, n.value

    def clear_exports(self):
        self._check(lib().ipxg_clear_exports(self._h), "ipxg_clear_exports")

    def stats(self):
        arr = (ctypes.c_uint64 * len(STATS_FIELDS))()
        self._check(lib().ipxg_get_stats(self._h, arr), "ipxg_get_stats")
        return dict(zip(STATS_FIELDS, list(arr)))

    def add_plugin(self, plugin):
        """Register a Plugin (ctypes struct); the caller keeps it (and its callbacks) alive."""
        self._check(lib().ipxg_add_plugin(self._h, ctypes.byref(plugin)), "ipxg_add_plugin")

    def set_walk_threads(self, n):
        """Threads of the plugin flows' host walk (0 = default, 1 = the calling thread)."""
        self._check(lib().ipxg_set_walk_threads(self._h, int(n)), "ipxg_set_walk_threads")

    def parser_stats(self):
        """(tcp port frequencies [65536], udp [65536], VlanStats [4096]) -- engine made with ps=true."""
        tcp = np.zeros(65536, dtype=np.uint64)
        udp = np.zeros(65536, dtype=np.uint64)
        vl = np.zeros(VLAN_IDS, dtype=VLAN_STATS_DTYPE)
        self._check(lib().ipxg_parser_stats(self._h, tcp.ctypes.data, udp.ctypes.data, vl.ctypes.data),
                    "ipxg_parser_stats")
        return tcp, udp, vl

    def top_ports(self, n):
        out = np.zeros(max(n, 1), dtype=PORT_STAT_DTYPE)
        got = ctypes.c_size_t()
        self._check(lib().ipxg_top_ports(self._h, n, out.ctypes.data, ctypes.byref(got)), "ipxg_top_ports")
        return out[:got.value]

    def profile(self, enable=True, every=1):
        """HIP-event stage timing (ipxg_profile): level 1/2/3 (True = 1), on one batch of every
        `every` (each event record costs the stream a packet of its own)."""
        self._check(lib().ipxg_profile(self._h, int(enable) | (int(every) << 8)), "ipxg_profile")

    def timing(self):
        t = Timing()
        self._check(lib().ipxg_get_timing(self._h, ctypes.byref(t)), "ipxg_get_timing")
        return {f: getattr(t, f) for f, _ in Timing._fields_}

    def probe_counters(self):
        out = np.zeros(16, dtype=np.uint64)
        self._check(lib().ipxg_probe_counters(self._h, out.ctypes.data), "ipxg_probe_counters")
        return out

    def ipfix_basic(self, recs, dir_bit_field=0):
        """IPFIX basic-template data records of `recs` (FLOW_DTYPE) formatted on the device:
        (bytes uint8 array, offsets[n + 1])."""
        recs = np.ascontiguousarray(recs, dtype=FLOW_DTYPE)
        out = np.zeros(max(len(recs), 1) * IPFIX_V6_LEN, dtype=np.uint8)
        off = np.zeros(len(recs) + 1, dtype=np.uint64)
        self._check(lib().ipxg_ipfix_basic(self._h, recs.ctypes.data, len(recs), dir_bit_field,
                                           out.ctypes.data, off.ctypes.data), "ipxg_ipfix_basic")
        return out[: int(off[-1])], off

    def poll_ipfix(self, dir_bit_field=0, cap=None):
        """Pending exports as IPFIX basic-template records (consumed): (bytes, records)."""
        if cap is None:
            cap = self.pending() * IPFIX_V6_LEN
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        n, nb = ctypes.c_size_t(), ctypes.c_size_t()
        self._check(lib().ipxg_poll_ipfix(self._h, dir_bit_field, out.ctypes.data, cap, ctypes.byref(n),
                                          ctypes.byref(nb)), "ipxg_poll_ipfix")
        return out[: nb.value], n.value

    @staticmethod
    def ipfix_exporter(odid=0, dir_bit_field=0, export_time=0, mtu=1458):
        x = IpfixExporter()
        lib().ipxg_ipfix_exporter_init(ctypes.byref(x))
        x.odid, x.dir_bit_field, x.export_time, x.mtu = odid, dir_bit_field, export_time, mtu
        return x

    def ipfix_export(self, x, recs):
        """Host records (FLOW_DTYPE) through the exporter state x: (message bytes, messages)."""
        recs = np.ascontiguousarray(recs, dtype=FLOW_DTYPE)
        cap = int(lib().ipxg_ipfix_bound(len(recs)))
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        nb, nm = ctypes.c_size_t(), ctypes.c_size_t()
        self._check(lib().ipxg_ipfix_export(self._h, ctypes.byref(x), recs.ctypes.data if len(recs) else None,
                                            len(recs), out.ctypes.data, cap, ctypes.byref(nb), ctypes.byref(nm)),
                    "ipxg_ipfix_export")
        return out[:nb.value], nm.value

    def poll_ipfix_messages(self, x):
        """Pending exports as IPFIX messages (consumed): (bytes, records, messages)."""
        cap = int(lib().ipxg_ipfix_bound(self.pending()))
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        nr, nb, nm = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        self._check(lib().ipxg_poll_ipfix_messages(self._h, ctypes.byref(x), out.ctypes.data, cap, ctypes.byref(nr),
                                                   ctypes.byref(nb), ctypes.byref(nm)), "ipxg_poll_ipfix_messages")
        return out[:nb.value], nr.value, nm.value

    def device_ipfix_messages(self, x):
        """Pending exports as IPFIX messages in an engine-owned device buffer (consumed):
        (device pointer, bytes, records, messages); valid until the next engine call."""
        p = ctypes.c_void_p()
        nr, nb, nm = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        self._check(lib().ipxg_device_ipfix_messages(self._h, ctypes.byref(x), ctypes.byref(p), ctypes.byref(nr),
                                                     ctypes.byref(nb), ctypes.byref(nm)), "ipxg_device_ipfix_messages")
        return p.value, nb.value, nr.value, nm.value

    def ipfix_stream(self):
        """The stream device_ipfix_messages formats on (hipStream_t as an int)."""
        return lib().ipxg_ipfix_stream(self._h)

    def device_ipfix_counts(self):
        """Device pointer to the {bytes, records} (2 x uint64) of the last device_ipfix_messages
        call, written on the engine's stream (no host round trip for the gather's header)."""
        p = ctypes.c_void_p()
        self._check(lib().ipxg_device_ipfix_counts(self._h, ctypes.byref(p)), "ipxg_device_ipfix_counts")
        return p.value

    def parse(self, arena, desc, offset16=False):
        b = self._batch(arena, desc, offset16=offset16)
        out = np.zeros(b.n, dtype=PARSED_DTYPE)
        self._check(lib().ipxg_parse_batch(self._h, ctypes.byref(b), out.ctypes.data),
                    "ipxg_parse_batch")
        return out

    def xxh64(self, keys: np.ndarray, keylen: int, seed: int = 0):
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        n = keys.size // keylen if keylen else len(keys)
        out = np.zeros(n, dtype=np.uint64)
        self._check(lib().ipxg_xxh64_batch(self._h, keys.ctypes.data, keylen, n, seed,
                                           out.ctypes.data), "ipxg_xxh64_batch")
        return out

    def close(self):
        if getattr(self, "_h", None):
            lib().ipxg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def run_capture(arena, desc, datalink=DLT_EN10MB, params="", batch=None, finish=True, plugins=(), **kw):
    """Whole capture through the engine, returns (records, stats)."""
    with Engine(params, datalink=datalink, **kw) as e:
        for pl in plugins:
            e.add_plugin(pl)
        e.submit_all(arena, desc, batch)
        if finish:
            e.finish()
        recs = e.poll()
        st = e.stats()
    return recs, st
