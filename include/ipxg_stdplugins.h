/*
 * ipxg_stdplugins.h -- native stand-ins of four of ipfixprobe's process plugins as ipxg_plugin
 * rules + hooks (ipfixprobe_amd/host/ipxg_stdplugins.c).
 *
 * They restate what each reference plugin decides at put_pkt_recursive's hook call sites that
 * can change flow boundaries or the plugin's claim on a flow -- not the enrichment itself
 * (SNI, DNS answers, ...), which stays with the real plugin behind the adapter of
 * INTEGRATION.md.  Uses: the bench's configs[2] / configs[4] runs with their process plugins
 * registered (the bridge's cost measured with native hooks), and device-vs-oracle parity on the
 * synthetic mixes (the oracle calls the same hooks for every packet).  The real plugins are
 * pinned against the reference goldens through the adapter (tests/test_ref_plugins.py).
 *
 *   "dns"   dns.cpp:97-127,650-682: port 53; post_create / post_update FLOW_FLUSH when
 *           parse_dns accepts the payload, or always once the flow holds a DNS extension
 *   "http"  http.cpp:100-140: a second request (response) in a flow holding one ->
 *           FLOW_FLUSH_WITH_REINSERT from pre_update
 *   "tls"   tls.cpp:101-122: claims a flow on a TLS handshake record (16 03 xx, ClientHello /
 *           ServerHello); never ends a flow
 *   "quic"  quic.cpp:350-549: a long-header QUIC packet of a supported version claims the flow;
 *           version negotiation -> FLOW_FLUSH; follows the first QUIC_MAX_ELEMCOUNT (30) packets
 *           of a claimed flow (its per-packet type list, quic.cpp:340-346,494-498)
 *
 * Each plugin owns bits of the record's ext handle (its "RecordExt"): dns 0x1, http 0x2/0x4/0x8
 * (present / request / response), tls 0x10, quic 0x20.
 */
#ifndef IPXG_STDPLUGINS_H
#define IPXG_STDPLUGINS_H

#include <stdint.h>

#include "ipxg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define IPXG_STD_EXT_DNS 0x1ull
#define IPXG_STD_EXT_HTTP 0x2ull
#define IPXG_STD_EXT_HTTP_REQ 0x4ull
#define IPXG_STD_EXT_HTTP_RESP 0x8ull
#define IPXG_STD_EXT_TLS 0x10ull
#define IPXG_STD_EXT_QUIC 0x20ull

/* Fill *out with the named plugin ("dns", "http", "tls", "quic"): rule, hooks and a fresh
 * context (freed by ipxg_std_plugin_free).  0, or IPXG_EINVAL for an unknown name. */
int ipxg_std_plugin(const char* name, ipxg_plugin* out);
void ipxg_std_plugin_free(ipxg_plugin* pl);
/* Hook calls so far: pre_create, post_create, pre_update, post_update, pre_export, flushes
 * returned (6 counters). */
void ipxg_std_plugin_calls(const ipxg_plugin* pl, uint64_t* out6);

#ifdef __cplusplus
}
#endif

#endif /* IPXG_STDPLUGINS_H */
