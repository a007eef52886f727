/*
 * ipxg_oracle.h -- CPU restatement of ipfixprobe's parse -> hash -> biflow-cache path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libipxg, the host shim, the CLI)
 * includes, links or calls this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it, as the checker.
 *
 * It restates, function by function, the reference sources under /root/reference:
 *   parser     src/plugins/input/parser/parser.cpp:68-805 (+ headers.hpp)
 *   hash key   src/plugins/storage/cache/src/cache.cpp:525-574, cache.hpp:29-46
 *   XXH64      src/plugins/storage/cache/src/xxhash.h:2725-2901 (xxHash 0.8.1)
 *   frag cache src/plugins/storage/cache/src/fragmentationCache/{.cpp,.hpp}
 *   NHT cache  src/plugins/storage/cache/src/cache.cpp:52-152, 262-523 (lines, move-to-
 *              front, NO_RES eviction at the last slot / insertion at the middle slot, the
 *              per-packet cyclic expiry sweep, inactive/active/SYN-after-FIN splits)
 *
 * Pinning: the restatement reproduces the reference's own golden outputs
 * (tests/functional/outputs/basic from mixed.pcap, outputs/vlan from vlan.pcap, and the
 * basic columns of the other plugin goldens), see tests/test_oracle_golden.py; XXH64 is
 * checked against the reference's xxhash.c compiled into oracle/_ref and against python
 * xxhash 3.8.1.  The parser/cache sources themselves are not buildable here (they include
 * the third-party <telemetry.hpp>, absent), see DESIGN.md.
 *
 * Reads past caplen: the reference reads whatever memory follows the captured bytes in a
 * few places (undefined behaviour).  The oracle defines such bytes as 0 and sets
 * `beyond_caplen` so tests can tell those packets apart.
 */
#ifndef IPXG_ORACLE_H
#define IPXG_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/ipxg.h"

#ifdef __cplusplus
extern "C" {
#endif

uint64_t oracle_xxh64(const void* data, size_t len, uint64_t seed);
void oracle_xxh64_batch(const uint8_t* keys, size_t keylen, size_t n, uint64_t seed, uint64_t* out);

/* Parse one frame; returns 1 if parse_packet would append it to the block (valid). */
int oracle_parse(const uint8_t* data, uint16_t caplen, uint16_t wirelen, uint32_t ts_sec,
                 uint32_t ts_usec, uint32_t datalink, ipxg_parsed_pkt* out,
                 int* beyond_caplen);

typedef struct oracle_cache oracle_cache;

/* cache_exp = s=, line_exp = l= (reference defaults 17 and 4). */
oracle_cache* oracle_cache_new(uint32_t cache_exp, uint32_t line_exp, uint32_t active_s,
                               uint32_t inactive_s, int split_biflow, int frag_enable,
                               uint32_t frag_size, uint32_t frag_timeout_s);
void oracle_cache_free(oracle_cache* c);
/* Process-plugin hooks at the reference's call sites (cache.cpp:290-491; the same
 * ipxg_plugin callbacks the engine's bridge calls); up to 8, called in order. */
void oracle_cache_add_plugin(oracle_cache* c, const ipxg_plugin* p);
/* parse_packet + NHTFlowCache::put_pkt for each packet of a batch, in order. */
void oracle_cache_run(oracle_cache* c, const uint8_t* arena, const ipxg_pkt_desc* desc,
                      size_t n, uint32_t datalink);
void oracle_cache_export_expired(oracle_cache* c, int64_t ts_sec);
void oracle_cache_finish(oracle_cache* c);
size_t oracle_cache_pending(const oracle_cache* c);
/* Move up to cap exported records into out; returns the number moved. */
size_t oracle_cache_take(oracle_cache* c, ipxg_flow_record* out, size_t cap);
void oracle_cache_stats(const oracle_cache* c, ipxg_stats* out);
/* The parser's side statistics over every packet run so far (parser.cpp:484-485, 563-564,
 * 798): TCP/UDP port frequencies (65536 each) and VlanStats per VLAN id; outputs may be null. */
void oracle_cache_parser_stats(const oracle_cache* c, uint64_t* tcp_ports, uint64_t* udp_ports,
                               ipxg_vlan_stats* vlans);

/* IPFIXExporter::fill_basic_flow (ipfix.cpp:1470-1516) for each of n records: the basic
 * template's data records back to back into out, byte offsets into offsets[n + 1]. */
void oracle_ipfix_basic(const ipxg_flow_record* recs, size_t n, uint32_t dir_bit_field, uint8_t* out,
                        uint64_t* offsets);

/* IPFIXExporter::export_flow for each record in order, then flush(): the message bytes into
 * out (returns their length, (size_t)-1 if cap is short); updates x->sequence and
 * x->templates_sent like the exporter's state. */
size_t oracle_ipfix_export(ipxg_ipfix_exporter* x, const ipxg_flow_record* recs, size_t n, uint8_t* out, size_t cap,
                           size_t* msgs);

#ifdef __cplusplus
}
#endif

#endif
