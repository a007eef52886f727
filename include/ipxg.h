/*
 * ipxg.h -- C-ABI of the MI355X-native packet -> biflow engine.
 *
 * This is the drop-in boundary for ipfixprobe's per-packet hot path:
 *
 *   parse_packet()              /root/reference/src/plugins/input/parser/parser.cpp:673-805
 *                               (declared parser.hpp:87-93)
 *   NHTFlowCache::put_pkt()     /root/reference/src/plugins/storage/cache/src/cache.cpp:322-491
 *   create_hash_key() + XXH64() cache.cpp:525-574, xxhash.h:2885-2901
 *   FragmentationCache          cache/src/fragmentationCache/fragmentationCache.cpp:46-100
 *   StoragePlugin virtuals      /root/reference/include/ipfixprobe/storagePlugin.hpp:54-72
 *
 * Plain C, plain pointers and sizes.  Every entry point returns 0 on success or a
 * negative IPXG_E* code; no exception ever crosses this boundary (the reference throws
 * PluginError, plugin.hpp:81-91 -- the C++ shim in ipfixprobe_amd/host maps codes back).
 *
 * Threading: one engine per input pipeline, called from one thread (the reference builds
 * one NHTFlowCache per input thread, ipfixprobe.cpp:381-464).  An engine owns one HIP
 * stream on one device.
 */
#ifndef IPXG_H
#define IPXG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IPXG_ABI_VERSION 9 /* 2: ipxg_plugin gained masked prefixes and follow_packets;
                              3: ipxg_plugin gained copy_ctx / free_ctx (multi-threaded walk);
                              4: hooks report PluginError (IPXG_PLUGIN_ERROR, ipxg_plugin.error);
                              5: ipxg_timing gained plugin_overlapped
                              6: ipxg_profile takes a sampling period; ipxg_timing gained
                                 slow_redos; ipxg_plugin gained all_packets
                              7: ipxg_plugin gained follow_bytes; ipxg_timing gained
                                 plugin_d2h_bytes
                              8: IPXG_BATCH_OFFSET16 (arenas up to 64 GiB)
                              9: ipxg_timing gained ex_compactions */

/* ---- error codes ------------------------------------------------------------------- */
#define IPXG_OK 0
#define IPXG_EINVAL (-1)   /* bad argument / option string                               */
#define IPXG_ENOMEM (-2)   /* device or host allocation failed                           */
#define IPXG_EDEVICE (-3)  /* HIP runtime error (message in ipxg_last_error)             */
#define IPXG_EALIGN (-4)   /* a frame offset is not 16-byte aligned                      */
#define IPXG_ETOOBIG (-5)  /* batch larger than IPXG_MAX_BATCH, or arena > 4 GiB (64 GiB
                              with IPXG_BATCH_OFFSET16)                                  */
#define IPXG_EIO (-6)      /* file could not be read / unsupported capture format        */
#define IPXG_ESTATE (-7)   /* call not valid in the engine's current state               */
#define IPXG_EPLUGIN (-8)  /* a process plugin's hook failed -- the reference's PluginError
                              (plugin.hpp:81-91), which its input worker catches and reports
                              through WorkerResult (workers.cpp:107-112): the message is in
                              ipxg_last_error, the batch is lost, and the engine accepts only
                              ipxg_reset / ipxg_destroy / ipxg_last_error until reset        */

#define IPXG_MAX_BATCH (16u * 1024u * 1024u - 1u) /* per-batch counters are 24-bit     */

/* Link types (pcap LINKTYPE / libpcap DLT numbers), reference pcap.cpp:178-200 and
 * parser.cpp:704-726. */
#define IPXG_DLT_EN10MB 1
#define IPXG_DLT_RAW 12        /* libpcap DLT_RAW; LINKTYPE_RAW (101) is mapped to it    */
#define IPXG_DLT_LINUX_SLL 113
#define IPXG_DLT_LINUX_SLL2 276

/* Flow end reasons, reference flowifc.hpp:236-240 */
#define IPXG_FLOW_END_INACTIVE 0x01
#define IPXG_FLOW_END_ACTIVE 0x02
#define IPXG_FLOW_END_EOF 0x03
#define IPXG_FLOW_END_FORCED 0x04
#define IPXG_FLOW_END_NO_RES 0x05

/* ---- input: one packet descriptor (16 B), frames live in a byte arena ---------------
 * Replaces the (ts, data, len, caplen) argument tuple of parse_packet (parser.cpp:673-679).
 * caplen/wirelen are uint16_t exactly as parse_packet's parameters (the pcap plugin passes
 * pcap_pkthdr's 32-bit lengths into them, pcap.cpp:54-70, i.e. truncated mod 2^16).
 * Timestamps are timeval split into unsigned 32-bit seconds and microseconds (the classic
 * pcap record header's own width).  Frames at 16-byte aligned offsets take the register
 * parsers; others the general one.  With IPXG_BATCH_OFFSET16 offset counts 16-byte units. */
typedef struct ipxg_pkt_desc {
    uint32_t offset;  /* byte offset of the frame inside the batch arena (16-byte units
                         with IPXG_BATCH_OFFSET16)                                      */
    uint16_t caplen;  /* captured bytes present in the arena                            */
    uint16_t wirelen; /* original length on the wire                                    */
    uint32_t ts_sec;
    uint32_t ts_usec;
} ipxg_pkt_desc;

#define IPXG_BATCH_DEVICE 0x1u /* arena and desc are device pointers (already in HBM)   */
#define IPXG_BATCH_ASYNC 0x2u  /* ipxg_submit may return before the batch is applied (its
                                * kernels enqueued); the batch's buffers must stay unchanged
                                * until the next call on the engine, which completes it
                                * (ipxg_finish right behind it then costs one host round
                                * trip instead of two).  Host batches: copied into one of two
                                * device staging slots on a copy stream while the previous
                                * batch is in the kernels (pinned host memory for overlap) */
#define IPXG_BATCH_OFFSET16 0x4u /* every descriptor's offset counts 16-byte units: frames
                                  * start 16-byte aligned and the arena may hold up to
                                  * 64 GiB - 4 KiB (the 32-bit byte offsets cap it at 4 GiB,
                                  * 5M frames of the configs[4] mix).  Every frame must lie in
                                  * the arena (offset + caplen <= arena_len): the ingest reads
                                  * one past it as zeros (a keyless packet), with either
                                  * offset form, and never reads outside the arena there */

typedef struct ipxg_batch {
    const uint8_t* arena;       /* frame bytes                                          */
    uint64_t arena_len;         /* bytes valid in arena (<= 4 GiB; IPXG_BATCH_OFFSET16:
                                   <= 64 GiB - 4 KiB)                                   */
    const ipxg_pkt_desc* desc;  /* n descriptors in arrival order                       */
    uint32_t n;                 /* packets in this batch, <= IPXG_MAX_BATCH             */
    uint32_t flags;             /* IPXG_BATCH_*                                          */
} ipxg_batch;

/* ---- output: one exported biflow record (128 B POD) ----------------------------------
 * Mirrors ipxp::Flow (flowifc.hpp:245-268) minus the RecordExt chain, plus vlan_id (part
 * of the flow key, cache.hpp:29-46) and end_reason.  IPv4 addresses occupy the first 4
 * bytes of src_ip/dst_ip in network order (ipaddr_t.v4), the rest are zero. */
typedef struct ipxg_flow_record {
    uint64_t flow_hash;       /* XXH64 of the creating packet's forward key            */
    uint32_t time_first_sec;
    uint32_t time_first_usec;
    uint32_t time_last_sec;
    uint32_t time_last_usec;
    uint64_t src_bytes;
    uint64_t dst_bytes;
    uint32_t src_packets;
    uint32_t dst_packets;
    uint8_t src_tcp_flags;
    uint8_t dst_tcp_flags;
    uint8_t ip_version;
    uint8_t ip_proto;
    uint16_t src_port;
    uint16_t dst_port;
    uint8_t src_ip[16];
    uint8_t dst_ip[16];
    uint8_t src_mac[6];
    uint8_t dst_mac[6];
    uint16_t vlan_id;
    uint8_t end_reason;       /* IPXG_FLOW_END_*                                        */
    uint8_t reserved0;        /* IPXG_REC_PRE_EXPORTED, else zero                        */
    uint8_t reserved[8];      /* zero on export                                          */
    uint64_t ext;             /* the process plugins' per-flow handle (Flow::m_exts,
                                 see ipxg_plugin): zero on a record the engine creates,
                                 kept while the flow lives, exported with the record   */
    uint8_t reserved2[8];
} ipxg_flow_record;

/* ---- per-packet parse result (debug / parity entry point) ----------------------------
 * The flow-relevant subset of ipxp::Packet (packet.hpp:46-147) after parse_packet. */
typedef struct ipxg_parsed_pkt {
    uint8_t valid;            /* parse_packet accepted the packet (pblock->cnt++)        */
    uint8_t ip_version;
    uint8_t ip_proto;
    uint8_t tcp_flags;
    uint16_t ethertype;
    uint16_t ip_len;
    uint16_t src_port;
    uint16_t dst_port;
    uint16_t frag_off;
    uint8_t more_fragments;
    uint8_t ip_ttl;
    uint32_t vlan_id;
    uint32_t frag_id;
    uint32_t mpls_top;
    uint32_t tcp_mss;
    uint64_t tcp_options;
    uint8_t src_ip[16];
    uint8_t dst_ip[16];
    uint8_t src_mac[6];
    uint8_t dst_mac[6];
    uint8_t ip_tos;
    uint8_t ip_flags;
    uint16_t tcp_window;
    uint32_t tcp_seq;
    uint32_t tcp_ack;
    uint64_t hash_fwd;        /* XXH64(key), 0 when the packet has no flow key          */
    uint64_t hash_inv;        /* XXH64(inverse key)                                     */
    uint16_t payload_off;     /* Packet::payload - packet (data_offset, parser.cpp:797)  */
    uint16_t payload_len;     /* Packet::payload_len (parser.cpp:780-796: padding trim)  */
    uint32_t reserved2;
} ipxg_parsed_pkt;

/* ---- engine ------------------------------------------------------------------------ */
typedef struct ipxg_config {
    uint32_t cache_exp;       /* s=  initial table capacity 2^s slots (4..30)          */
    uint32_t line_exp;        /* l=  line size 2^l (strict=true; otherwise accepted)    */
    uint32_t active_s;        /* a=  active timeout, seconds (default 300)             */
    uint32_t inactive_s;      /* i=  inactive timeout, seconds (default 30)            */
    uint32_t split_biflow;    /* S   1 = uniflows                                      */
    uint32_t frag_enable;     /* fe= fragmentation cache on (default 1)                */
    uint32_t frag_size;       /* fs= buckets (default 10007)                           */
    uint32_t frag_timeout_s;  /* ft= seconds (default 3)                               */
    int32_t device_id;        /* dev= HIP device ordinal                               */
    uint32_t batch_pkts;      /* batch= max packets per submit (staging size)          */
    uint32_t datalink;        /* IPXG_DLT_*                                            */
    uint32_t flags;           /* IPXG_CFG_*                                            */
} ipxg_config;

/* ipxg_config.flags */
#define IPXG_CFG_ATOMIC_INGEST 0x1u /* ingest=atomic: fold every packet into the table with
                                       device atomics (one kernel) instead of the binned
                                       two-phase ingest; kept for A/B measurement          */
#define IPXG_CFG_WALK_WIDE 0x2u     /* walk=wide: k_bin loads 96 bytes per frame and parses
                                       VLAN/QinQ, IPv6 and TCP-timestamp frames from
                                       registers too; default walk=auto picks per batch
                                       from the previous batch's mix                        */
#define IPXG_CFG_WALK_NARROW 0x4u   /* walk=narrow: k_bin parses the plain Eth/IPv4/UDP|TCP
                                       shape only (48-byte loads), the rest goes through
                                       the slow list (k_bin_slow)                           */
#define IPXG_CFG_PARSER_STATS 0x8u  /* ps=true: the parser's side statistics -- TCP/UDP port
                                       frequencies (TopPorts) and per-VLAN counters with the
                                       packet-size histogram (VlanStats), parser-stats.hpp
                                       :126-201 -- kept on the device (ipxg_parser_stats) */
#define IPXG_CFG_STRICT 0x10u       /* strict=true: the reference's table exactly -- 2^s records
                                       in lines of 2^l (l <= 4, at most 32768 lines), move to
                                       front, FLOW_END_NO_RES eviction with insertion at the
                                       middle, the per-packet sweep (cache.cpp:322-523) --
                                       replayed on the device in packet order per line
                                       (ipxg_strict.hip); ipxg_expire is then one
                                       export_expired(now) step.  Not with ingest=atomic, ps=true
                                       or process plugins. */

typedef struct ipxg_stats {
    /* parser counters, reference parser-stats.hpp:126-201 (the subset on the path) */
    uint64_t seen_packets;
    uint64_t parsed_packets;  /* pblock->cnt increments                                */
    uint64_t unknown_packets;
    uint64_t ipv4_packets;
    uint64_t ipv6_packets;
    uint64_t tcp_packets;
    uint64_t udp_packets;
    uint64_t mpls_packets;
    uint64_t pppoe_packets;
    uint64_t trill_packets;
    uint64_t vlan_packets;
    uint64_t ipv4_bytes;
    uint64_t ipv6_bytes;
    /* cache counters, reference cache.cpp:618-665 */
    uint64_t end_inactive;
    uint64_t end_active;
    uint64_t end_eof;
    uint64_t end_forced;
    uint64_t end_no_res;
    uint64_t flows_in_cache;
    uint64_t total_exported;
    uint64_t keyless_packets; /* valid packets without a flow key (create_hash_key false) */
    uint64_t fragmented_packets;
    uint64_t fragments_filled;
    uint64_t complex_flows;   /* flow-batches resolved on the sequential device path    */
    uint64_t table_capacity;
    uint64_t table_rehashes;
    uint64_t batches;
    uint64_t spilled_packets; /* packets that fell back from the binned ingest to direct
                                 device atomics (partition region or LDS table full)    */
    uint64_t slow_path_packets; /* packets k_bin left to the general parser (k_bin_slow)  */
    uint64_t aggregated_packets; /* packets folded into per-tile flow aggregates (skew)   */
    uint64_t walked_packets;  /* packets of the wide walk's extra shapes (VLAN, IPv6, TCP
                                 timestamp option) parsed from registers by k_bin     */
    /* FlowRecordStats (cache.cpp:601-616, counted in export_flow :262-267): exported records
       by src_packets + dst_packets = 1, 2-5, 6-10, 11-20, 21-50, anything else (51+) */
    uint64_t flows_1_packet;
    uint64_t flows_2_5_packets;
    uint64_t flows_6_10_packets;
    uint64_t flows_11_20_packets;
    uint64_t flows_21_50_packets;
    uint64_t flows_51_plus_packets;
} ipxg_stats;

/* VlanStats (parser-stats.hpp:126-160) for one VLAN id; sizes are packet_len = caplen,
   histogram buckets 0-64, 65-127, 128-255, 256-511, 512-1023, 1024-1517, 1518-2047,
   2048-4095, 4096-8191, 8192+ (PacketSizeHistogram, parser-stats.hpp:42-95). */
#define IPXG_VLAN_IDS 4096
#define IPXG_SIZE_BUCKETS 10
typedef struct ipxg_vlan_stats {
    uint64_t ipv4_packets;
    uint64_t ipv6_packets;
    uint64_t ipv4_bytes;
    uint64_t ipv6_bytes;
    uint64_t tcp_packets;
    uint64_t udp_packets;
    uint64_t total_packets;
    uint64_t total_bytes;
    uint64_t hist_packets[IPXG_SIZE_BUCKETS];
    uint64_t hist_bytes[IPXG_SIZE_BUCKETS];
} ipxg_vlan_stats;

/* One entry of TopPorts::get_top_ports (topPorts.cpp): protocol 6 (TCP) or 17 (UDP). */
typedef struct ipxg_port_stat {
    uint16_t port;
    uint8_t protocol;
    uint8_t reserved[5];
    uint64_t frequency;
} ipxg_port_stat;

typedef struct ipxg_engine ipxg_engine;

/* Fill *cfg with the reference defaults (cache.hpp:52-64, :91-102). */
void ipxg_config_default(ipxg_config* cfg);
/* Parse the reference cache option string ("s=20;a=300;i=30;S;fe=false;..."), plus
 * dev= / batch= / dlt=, into *cfg (reference CacheOptParser, cache.hpp:81-221). */
int ipxg_config_parse(const char* params, ipxg_config* cfg);

int ipxg_create(const ipxg_config* cfg, ipxg_engine** out);
/* Release the engine.  Pending exports are dropped; no hook of a registered plugin is called --
 * only free_ctx, once for every copy the engine made (copy_ctx) -- also after IPXG_EPLUGIN /
 * IPXG_ESTATE.  A registered ipxg_plugin (its ctx, hooks and free_ctx) must stay valid until this
 * call returns; the caller frees its own instance after it (tests/plugin_lifetime.cpp). */
int ipxg_destroy(ipxg_engine* eng);
const char* ipxg_last_error(const ipxg_engine* eng);
/* hipStream_t the engine launches on (for event timing by the caller). */
void* ipxg_stream(ipxg_engine* eng);

/* Parse + hash + biflow-cache update for one batch, in arrival order
 * (= for each packet: parse_packet, then NHTFlowCache::put_pkt).  Host batches are
 * staged to HBM with hipMemcpyAsync; device batches are read in place.  Returns after the
 * batch has been applied (the stream is synchronised). */
int ipxg_submit(ipxg_engine* eng, const ipxg_batch* batch);
/* Export every flow idle for >= inactive seconds at now_sec (reference export_expired,
 * cache.cpp:508-523, whole table at once). */
int ipxg_expire(ipxg_engine* eng, int64_t now_sec);
/* Export every remaining flow as FLOW_END_FORCED and empty the cache (cache.cpp:276-288). */
int ipxg_finish(ipxg_engine* eng);
/* Drop all state without exporting (engine reuse). */
int ipxg_reset(ipxg_engine* eng);
/* Number of exported records waiting in the device export buffer. */
int ipxg_pending_exports(ipxg_engine* eng, size_t* n);
/* Copy up to cap exported records to host memory out and remove them from the buffer. */
int ipxg_poll_exports(ipxg_engine* eng, ipxg_flow_record* out, size_t cap, size_t* n);
/* Device pointer to the export buffer and its current count (no copy; valid until the next
 * engine call).  The device-side consumers of the exports -- this call, ipxg_poll_ipfix_messages and
 * ipxg_device_ipfix_messages -- do not call the plugins' pre_export (host code) on the records the
 * device exported: with process plugins holding per-flow state (ext), consume the exports through
 * ipxg_poll_exports, which does (IPXG_REC_PRE_EXPORTED).  A pre_export failure there (the instance's
 * error()) fails that call with IPXG_EPLUGIN after handing the records over. */
int ipxg_device_exports(ipxg_engine* eng, const ipxg_flow_record** dptr, size_t* n);
/* Forget the pending exports without copying them (caller consumed them on device). */
int ipxg_clear_exports(ipxg_engine* eng);
int ipxg_get_stats(ipxg_engine* eng, ipxg_stats* out);
/* Parser side statistics (engine created with ps=true, else IPXG_EINVAL): TopPorts' TCP and
 * UDP frequency arrays (65536 entries each; parser.cpp:484-485, 563-564) and VlanStats for
 * every VLAN id (IPXG_VLAN_IDS entries; parser.cpp:798); any output may be null. */
int ipxg_parser_stats(ipxg_engine* eng, uint64_t* tcp_ports, uint64_t* udp_ports, ipxg_vlan_stats* vlans);
/* TopPorts::get_top_ports (topPorts.cpp): up to n most frequent ports, TCP then UDP, ties in
 * port order, *got entries written. */
int ipxg_top_ports(ipxg_engine* eng, size_t n, ipxg_port_stat* out, size_t* got);

/* ---- process-plugin bridge (processPlugin.hpp:42-119; call sites cache.cpp:290-491) ---- */
#define IPXG_FLOW_FLUSH 0x1               /* FLOW_FLUSH (processPlugin.hpp:27)                 */
#define IPXG_FLOW_FLUSH_WITH_REINSERT 0x3 /* FLOW_FLUSH_WITH_REINSERT (processPlugin.hpp:36)   */
#define IPXG_PLUGIN_MAX_PORTS 16
#define IPXG_PLUGIN_MAX_PREFIXES 16
#define IPXG_PLUGIN_PREFIX_LEN 16

/* What a hook sees of ipxp::Packet (packet.hpp:46-147): the parsed fields (payload_off /
 * payload_len locate Packet::payload in data), the captured bytes, the timestamp and
 * source_pkt (set before post_create / pre_update / post_update, cache.cpp:428). */
typedef struct ipxg_packet_view {
    const ipxg_parsed_pkt* pkt;
    const uint8_t* data;
    uint32_t caplen;
    uint32_t wirelen;
    uint32_t ts_sec;
    uint32_t ts_usec;
    uint32_t index;           /* position of the packet in its batch                   */
    uint8_t source_pkt;
    uint8_t reserved[3];
} ipxg_packet_view;

/* A process plugin: the device pre-classifier rule (a packet is the plugin's when it is
 * TCP/UDP -- proto_mask bit 0 TCP, bit 1 UDP -- with its source or destination port in
 * ports[], or its payload starts with one of prefixes[]: byte k equal to prefix[q][k], or, when
 * bit q of `masked` is set, equal under prefix_mask[q][k] -- e.g. QUIC's long-header bit,
 * mask 0x80), and the hooks.  Contract: on the packets outside the rule every hook returns 0
 * and changes nothing (so flows with none of the plugin's packets in a batch stay on the
 * device) -- except, for a plugin with follow_packets > 0, on a flow whose record carries a
 * non-zero ext while it holds fewer than follow_packets packets: such a flow stays on the host
 * walk with all its packets, batch after batch, until it reaches follow_packets (QUIC stores
 * every packet's type for the first QUIC_MAX_ELEMCOUNT packets of a flow it detected,
 * quic.cpp:340-346,494-498).  A flow with one of them has all its packets of the batch replayed
 * in order on the host, through these hooks at put_pkt_recursive's call sites.  The record's
 * ext field (a 64-bit handle) is the plugins' per-flow state -- Flow::m_exts: zero on a new
 * record, cleared by erase/reuse, carried by the exported record.  Hooks return 0 or
 * IPXG_FLOW_FLUSH / IPXG_FLOW_FLUSH_WITH_REINSERT, or a negative value (IPXG_PLUGIN_ERROR) where
 * the reference plugin throws PluginError: the walk stops and the call that ran it fails with
 * IPXG_EPLUGIN.  No C++ exception may leave a hook (the adapter of INTEGRATION.md catches them). */
#define IPXG_PLUGIN_ERROR (-1)
/* reserved0 of an exported record: the plugins' pre_export has been dealt with.  The reference
 * calls plugins_pre_export on every export but a flush (cache.cpp:280,406,455,466,514; not in
 * :290-320).  The host walk calls it at those sites for the flows it replays and marks every
 * record it exports; a record the device exported (k_fin_list's evictions and timeouts,
 * k_finish, k_expire) with a non-zero ext gets the registered plugins' pre_export, in
 * registration order, on the calling thread inside ipxg_poll_exports -- then it carries the
 * mark too.  (A device record with ext == 0 holds no plugin state: pre_export is not called.) */
#define IPXG_REC_PRE_EXPORTED 0x01
typedef struct ipxg_plugin {
    void* ctx;
    uint32_t proto_mask;
    uint32_t n_ports;
    uint16_t ports[IPXG_PLUGIN_MAX_PORTS];
    uint32_t n_prefixes;
    uint8_t prefix_len[IPXG_PLUGIN_MAX_PREFIXES];
    uint8_t prefix[IPXG_PLUGIN_MAX_PREFIXES][IPXG_PLUGIN_PREFIX_LEN];
    int (*pre_create)(void* ctx, ipxg_packet_view* pkt);
    int (*post_create)(void* ctx, ipxg_flow_record* flow, const ipxg_packet_view* pkt);
    int (*pre_update)(void* ctx, ipxg_flow_record* flow, ipxg_packet_view* pkt);
    int (*post_update)(void* ctx, ipxg_flow_record* flow, const ipxg_packet_view* pkt);
    void (*pre_export)(void* ctx, ipxg_flow_record* flow);
    /* ABI 2 */
    uint32_t masked;          /* bit q: prefix q compares under prefix_mask[q]                 */
    uint32_t follow_packets;  /* see above; 0 = the rule alone decides                          */
    uint8_t prefix_mask[IPXG_PLUGIN_MAX_PREFIXES][IPXG_PLUGIN_PREFIX_LEN];
    /* ABI 3: ProcessPlugin::copy() (processPlugin.hpp:50).  The host walk splits a batch's
     * plugin flows over several threads (ipxg_set_walk_threads), each calling the hooks of its
     * own instance of every plugin -- as the reference gives every storage pipeline its own copy
     * of each process plugin (ipfixprobe.cpp:430-436).  copy_ctx returns a new context for another
     * walk thread (NULL: out of memory), free_ctx releases one.  The engine copies a plugin when
     * it is registered (and in ipxg_set_walk_threads), before any walk has used it -- copy()
     * copies a plugin's state, and the reference copies its prototypes before the pipelines
     * start -- and frees the copies in ipxg_destroy, so the original ctx must outlive the
     * engine.  A NULL copy_ctx on any registered plugin keeps the walk on one thread. */
    void* (*copy_ctx)(void* ctx);
    void (*free_ctx)(void* ctx);
    /* ABI 4: the message of a failure of this instance since the previous call, or NULL
     * (optional; the string stays valid until the instance fails again).  The engine calls it
     * after a hook returned IPXG_PLUGIN_ERROR, and after every walk of a batch -- pre_export
     * returns nothing, so a failure there is reported only here. */
    const char* (*error)(void* ctx);
    /* ABI 6: 1 = the plugin's hooks act on every packet of every flow (pstats, phists, bstats and
     * any plugin whose packets no port / prefix rule describes): every flow the batch touches is
     * walked on the host -- the reference's behaviour (its hooks see every packet), at the host
     * walk's rate.  The rule fields are then unused. */
    uint32_t all_packets;
    /* ABI 7: 0 = the hooks may read any byte of a walked packet (its whole frame crosses to the
     * host).  N > 0 = on a packet outside this plugin's rule (a packet of a flow it follows, or of
     * a flow another plugin walks) the hooks read at most the first N payload bytes -- QUIC reads
     * the first byte of a short-header packet and nothing more (quic.cpp:494-498,
     * quic_parser.cpp:1105-1117, 1160-1167).  When every registered plugin declares N > 0 and none
     * acts on all packets, a walked packet that matches no rule crosses with its headers and the
     * largest N payload bytes; the view's caplen and the parsed fields stay the packet's own. */
    uint32_t follow_bytes;
} ipxg_plugin;

/* Register a plugin (the order of registration is the order of the hook calls).  The struct is
 * copied; its ctx stays the caller's and must outlive the engine (ipxg_destroy). */
int ipxg_add_plugin(ipxg_engine* eng, const ipxg_plugin* plugin);
/* Threads of the plugin flows' host walk: 0 = default (the host's hardware threads, at most
 * 16), 1 = the calling thread only.  Raising it after the first plugin walk fails with
 * IPXG_ESTATE (the new copies would copy used plugin instances).  Flows are independent (the walk replays each flow's
 * packets in order on one thread), so the records are the same for any thread count; the export
 * order of the walked flows is the concatenation of the threads' (contiguous flow ranges in
 * order of each flow's first packet). */
int ipxg_set_walk_threads(ipxg_engine* eng, uint32_t threads);

/* ---- stage timing (HIP events on the engine's stream) --------------------------------- */
typedef struct ipxg_timing {
    double ingest_ms;          /* k_bin: parse + hash + partition (atomic mode: k_ingest)  */
    double ingest_slow_ms;     /* k_bin_slow: frames for the general parser                */
    double reduce_ms;          /* k_reduce: per-flow aggregation + table merge             */
    double fin_ms;             /* k_fin_list: split rules on the flows k_reduce completed  */
    double finalize_ms;        /* k_finalize table scan (only when k_reduce could not)     */
    double slow_ms;            /* fragment / overflow / complex-flow paths                 */
    double finish_ms;          /* k_finish + table clear                                   */
    uint64_t ingest_launches;
    uint64_t reduce_launches;
    uint64_t finalize_launches;
    uint64_t slow_launches;
    uint64_t finish_launches;
    uint64_t ingest_packets;   /* packets covered by the timed ingest launches             */
    /* the process-plugin bridge's host walk (wall clock, always counted; zeroed by ipxg_profile) */
    double plugin_ms;          /* plugin flows: pack, copies of their packets, the walk, write-back */
    uint64_t plugin_flows;     /* flow-batches walked on the host                               */
    uint64_t plugin_packets;   /* packets handed to the hooks                                   */
    uint64_t plugin_bytes;     /* their captured bytes (full caplen, copied to the host)        */
    uint64_t plugin_extra_bytes; /* of which past each frame's first 128 (full caplen
                                    for packets handed to process plugins)                    */
    uint64_t plugin_overlapped;  /* IPXG_BATCH_ASYNC device batches whose k_bin / k_bin_slow ran
                                    during the previous batch's host walk                      */
    /* ABI 6 (always counted; zeroed by ipxg_profile): batches launched without k_bin_slow (the
       previous batch had no slow-list packet) whose k_bin listed some -- run again from k_bin_slow */
    uint64_t slow_redos;
    /* ABI 7: bytes the plugin walk copied to the host -- frames (whole, or their byte budget:
       ipxg_plugin.follow_bytes), packet and flow records, per-flow arrays */
    uint64_t plugin_d2h_bytes;
    /* ABI 9 (always counted; zeroed by ipxg_profile): finishes fused into a batch's finalise pass whose
       reserved export records had holes (flows that turned complex or found no slot), closed by a
       compaction of the export buffer before the records were handed out */
    uint64_t ex_compactions;
} ipxg_timing;

/* Per-phase shader-clock sums of the last batch's k_bin, k_reduce and k_bin_slow (16 values;
 * all zero unless the library was built with -DIPXG_PROBE -- a tuning aid). */
int ipxg_probe_counters(ipxg_engine* eng, uint64_t* out);
/* Event timing: 1 = every stage, 2 = the ingest kernel only (two events per batch, the
 * least host overhead), 3 = k_bin and k_bin_slow (three events), 0 = off; enabling also
 * zeroes the accumulators.  ABI 6: bits 8..23 of `enable` = a period p -- the events are
 * recorded on one batch of every p (0 or 1: every batch; each event record is a packet of its
 * own on the engine's stream, ~4-5 us of GPU time on MI355X), and the timing counts those. */
int ipxg_profile(ipxg_engine* eng, int enable);
int ipxg_get_timing(ipxg_engine* eng, ipxg_timing* out);

/* ---- IPFIX export formatting --------------------------------------
 * Data records of the reference IPFIX output plugin's basic templates (BASIC_TMPLT_V4 /
 * BASIC_TMPLT_V6, include/ipfixprobe/ipfix-elements.hpp:328-366) as
 * IPFIXExporter::fill_basic_flow writes them (src/plugins/output/ipfix/src/ipfix.cpp:1470-1516,
 * field encoding IPFIX_FILL_FIELD :77-96): big-endian, flow times as 64-bit NTP timestamps
 * (MK_NTP_TS, ipfix-elements.hpp:50-60), INPUT_INTERFACE = the exporter's dir_bit_field.
 * IPXG_IPFIX_V4_LEN bytes for ip_version 4, IPXG_IPFIX_V6_LEN otherwise, back to back in
 * record order.  Formatted on the device. */
#define IPXG_IPFIX_V4_LEN 81
#define IPXG_IPFIX_V6_LEN 105
/* n host records -> out (>= n * 105 bytes), offsets[n + 1] byte offsets (offsets[n] = total). */
int ipxg_ipfix_basic(ipxg_engine* eng, const ipxg_flow_record* recs, size_t n, uint32_t dir_bit_field,
                     uint8_t* out, uint64_t* offsets);
/* The pending exports straight from the device export buffer, consumed like
 * ipxg_poll_exports: the longest prefix of whole records fitting `cap` bytes; *n records,
 * *bytes written. */
int ipxg_poll_ipfix(ipxg_engine* eng, uint32_t dir_bit_field, uint8_t* out, size_t cap, size_t* n,
                    size_t* bytes);

/* ---- IPFIX messages: the IPFIX output plugin's wire format ---------
 * The message stream IPFIXExporter (src/plugins/output/ipfix/src/ipfix.cpp) sends for a run of
 * export_flow() calls followed by flush(): the template message (the basic templates, ids 258
 * for IPv4 and 259 for IPv6, create_template ipfix.cpp:537-656, create_template_packet
 * :671-728) once per exporter, then data messages of at most `mtu` bytes, each a 16-byte
 * header (fill_ipfix_header :475-486: version 10, length, export time, sequence number =
 * records in earlier data messages, observation domain) and one data set per template whose
 * buffer fits (create_data_packet :739-795), a template's buffer flushing when its next record
 * would pass mtu - 16 bytes (fill_basic_flow :1470-1516, export_flow :385-398).  The records
 * are fed to that exporter in export-buffer order with the IPv4 records first (a stable
 * partition by template -- export order is not part of the flow contract), formatted and
 * packed on the device.  The caller keeps the exporter state. */
#define IPXG_IPFIX_DEFAULT_MTU 1458 /* ipfix.hpp:34 */
typedef struct ipxg_ipfix_exporter {
    uint32_t odid;            /* observationDomainId (ipfix plugin id=)                    */
    uint32_t dir_bit_field;   /* INPUT_INTERFACE value (ipfix plugin dir=)                 */
    uint32_t export_time;     /* header exportTime (the reference: time(NULL) at send)     */
    uint32_t sequence;        /* in/out: records carried by earlier data messages          */
    uint16_t mtu;             /* message size limit, >= 125 (ipfix plugin mtu=)            */
    uint16_t templates_sent;  /* in/out: the template message has gone out                 */
} ipxg_ipfix_exporter;

void ipxg_ipfix_exporter_init(ipxg_ipfix_exporter* x);
/* Upper bound of the message bytes for n records (templates included). */
uint64_t ipxg_ipfix_bound(uint64_t n);
/* n host records, in this order, through the exporter -> out (cap bytes, IPXG_ETOOBIG and
 * nothing written if short); *bytes written, *msgs messages. */
int ipxg_ipfix_export(ipxg_engine* eng, ipxg_ipfix_exporter* x, const ipxg_flow_record* recs, size_t n,
                      uint8_t* out, size_t cap, size_t* bytes, size_t* msgs);
/* The pending exports (consumed, like ipxg_poll_exports) as messages into host memory. */
int ipxg_poll_ipfix_messages(ipxg_engine* eng, ipxg_ipfix_exporter* x, uint8_t* out, size_t cap, size_t* n_records,
                             size_t* bytes, size_t* msgs);
/* The same into a device buffer owned by the engine, for gathering the per-GPU message streams
 * with RCCL.  Two buffers alternate: a stream stays valid until the second
 * ipxg_device_ipfix_messages call after the one that produced it (a consumer may send stream k
 * while the engine formats stream k+1).  Formatted on ipxg_ipfix_stream(eng), a side stream forked
 * from the engine's stream (so it runs beside the next batch's first kernels); the engine's stream
 * joins it before anything that appends exports.  A consumer waits for ipxg_ipfix_stream.  Called
 * with an asynchronous batch in flight (ipxg_submit with IPXG_BATCH_ASYNC, nothing since), it
 * formats the exports of the batches completed before it and leaves that batch running. */
int ipxg_device_ipfix_messages(ipxg_engine* eng, ipxg_ipfix_exporter* x, const uint8_t** dptr, size_t* n_records,
                               size_t* bytes, size_t* msgs);
/* The {stream bytes, records} of the last ipxg_device_ipfix_messages call as two uint64 in device
 * memory, written in order on ipxg_ipfix_stream with the messages: a consumer on
 * another stream that waits for the engine's reads them without a host round trip (the header of
 * the multi-GPU stream gather).  They sit at the tail of that call's message buffer (8-byte aligned
 * past the stream), so they stay valid exactly as long as the messages: until the call after the
 * next ipxg_device_ipfix_messages -- a consumer must make the engine's stream wait for its reads
 * before that call.  IPXG_ESTATE before the first call. */
int ipxg_device_ipfix_counts(ipxg_engine* eng, const uint64_t** dptr);
/* The stream ipxg_device_ipfix_messages formats on (hipStream_t; the engine's own stream before
 * the first call). */
void* ipxg_ipfix_stream(ipxg_engine* eng);

/* ---- stateless device entry points (parity tests, tools) ---------------------------- */
/* Run the device parser on a batch; out receives n records (host pointer). */
int ipxg_parse_batch(ipxg_engine* eng, const ipxg_batch* batch, ipxg_parsed_pkt* out);
/* XXH64(seed) of n keys of keylen bytes each, packed back to back, on the device. */
int ipxg_xxh64_batch(ipxg_engine* eng, const uint8_t* keys, uint32_t keylen, uint32_t n,
                     uint64_t seed, uint64_t* out);

/* ---- host ingestion (pcap / pcapng files) -------------------------------------------
 * Reads a whole capture into a host batch: frames at 16-byte aligned offsets, lengths
 * truncated to 16 bits exactly as the reference passes them to parse_packet, nanosecond
 * captures scaled to microseconds by integer division (libpcap's behaviour). */
typedef struct ipxg_capture {
    uint8_t* arena;
    uint64_t arena_len;
    ipxg_pkt_desc* desc;
    uint32_t n;
    uint32_t datalink;        /* IPXG_DLT_* of the capture                              */
} ipxg_capture;

int ipxg_capture_load(const char* path, ipxg_capture** out);
void ipxg_capture_free(ipxg_capture* cap);

/* ---- multi-GPU host demux (SURVEY 8(e) "input distribution", 8(f) row 3) ---------------
 * The host side of the end-to-end multi-GPU path: which engine (one per GPU, each with its
 * own table) takes each packet of a host batch -- the analogue of the NIC's symmetric RSS
 * into per-queue rings (dpdkDevice.cpp:230-262; one pipeline per queue, ipfixprobe.cpp:381-464).
 * shard = a symmetric hash of the outermost IP address pair, found through Ethernet, VLAN/QinQ
 * tags, MPLS labels and PPPoE (the link types of ipxg_batch; SLL/SLL2/RAW too), so both
 * directions of a biflow and every fragment of a datagram go to the same engine; frames
 * without an IP header go to shard 0.  Reads at most the first 64 header bytes per frame.
 * shard_of[i] (n entries) receives packet i's shard; counts[k] (n_shards) the shard sizes.
 * ipxg_demux_split then gathers shard k's frames into its own batch (arena at 16-byte aligned
 * offsets, descriptors in arrival order; offsets counted as in's are, bytes or 16-byte units
 * with IPXG_BATCH_OFFSET16): arena_out must hold ipxg_demux_arena_bytes(...). */
int ipxg_demux(const ipxg_batch* in, uint32_t datalink, uint32_t n_shards, uint32_t* shard_of, uint32_t* counts);
uint64_t ipxg_demux_arena_bytes(const ipxg_batch* in, const uint32_t* shard_of, uint32_t shard);
int ipxg_demux_split(const ipxg_batch* in, const uint32_t* shard_of, uint32_t shard, uint8_t* arena_out,
                     ipxg_pkt_desc* desc_out, uint32_t* n_out);

#ifdef __cplusplus
}
#endif

#endif /* IPXG_H */
