// plugin_adapter.hpp -- a reference process plugin (ipxp::ProcessPlugin, include/ipfixprobe/
// processPlugin.hpp:42-119) behind the engine's process-plugin bridge (ipxg_plugin,
// include/ipxg.h): the Adapter of INTEGRATION.md, for the gpucache storage plugin a maintainer
// adds in the reference tree.  Header-only; compiles against the reference's unmodified
// headers (processPlugin.hpp, packet.hpp, flowifc.hpp -- none of them includes the absent
// third-party telemetry.hpp), which only the reference tree has, so it is built here only by the
// test recipe oracle/Makefile (ref_plugins: the reference's own dns/http/tls/quic plugin sources
// through this adapter, checked against the reference goldens).
//
//   ipxg hook (include/ipxg.h)          -> ProcessPlugin virtual, as put_pkt_recursive calls it
//   pre_create(view)                       pre_create(Packet&)                  cache.cpp:332
//   post_create(rec, view)                 post_create(Flow&, const Packet&)    cache.cpp:443
//   pre_update(rec, view)                  pre_update(Flow&, Packet&)           cache.cpp:474
//   post_update(rec, view)                 post_update(Flow&, const Packet&)    cache.cpp:480
//   pre_export(rec)                        pre_export(Flow&)                    cache.cpp:455,466,514
//
// The record's ext handle is the address of a heap ipxp::Flow that holds the flow's RecordExt
// chain (Flow::m_exts, flowifc.hpp:146-234) -- shared by every plugin registered on the engine,
// each finding its own extension by id, as on a reference Flow.  A flow no plugin has attached
// an extension to keeps ext = 0 (hooks run on a scratch Flow), so the engine's notion of a
// claimed flow (ipxg_plugin.follow_packets) is the reference's (an extension exists).  The
// consumer of an exported record owns its Flow (take it with flow_of(ext), delete it).
#pragma once

#include <sys/time.h>

#include <cstdint>
#include <cstring>
#include <string>

#include <ipfixprobe/flowifc.hpp>
#include <ipfixprobe/packet.hpp>
#include <ipfixprobe/processPlugin.hpp>

#include "../../include/ipxg.h"

namespace ipxg_ref {

inline ipxp::Flow* flow_of(uint64_t ext) { return reinterpret_cast<ipxp::Flow*>(static_cast<uintptr_t>(ext)); }

// ipxp::Packet from what the hook sees (packet.hpp:46-147; parse_packet fills the same fields,
// parser.cpp:673-805).  payload_len_wire is the captured payload (the view carries no wire length
// of the payload); none of the bridged plugins reads it.
inline void fill_packet(ipxp::Packet& k, const ipxg_packet_view& v) {
    const ipxg_parsed_pkt& p = *v.pkt;
    k.ts.tv_sec = v.ts_sec;
    k.ts.tv_usec = v.ts_usec;
    std::memcpy(k.dst_mac, p.dst_mac, 6);
    std::memcpy(k.src_mac, p.src_mac, 6);
    k.ethertype = p.ethertype;
    k.ip_len = p.ip_len;
    k.ip_version = p.ip_version;
    k.ip_ttl = p.ip_ttl;
    k.ip_proto = p.ip_proto;
    k.ip_tos = p.ip_tos;
    k.ip_flags = p.ip_flags;
    std::memcpy(&k.src_ip, p.src_ip, 16);
    std::memcpy(&k.dst_ip, p.dst_ip, 16);
    k.vlan_id = p.vlan_id;
    k.frag_id = p.frag_id;
    k.frag_off = p.frag_off;
    k.more_fragments = p.more_fragments != 0;
    k.src_port = p.src_port;
    k.dst_port = p.dst_port;
    k.tcp_flags = p.tcp_flags;
    k.tcp_window = p.tcp_window;
    k.tcp_options = p.tcp_options;
    k.tcp_mss = p.tcp_mss;
    k.tcp_seq = p.tcp_seq;
    k.tcp_ack = p.tcp_ack;
    k.mplsTop = p.mpls_top;
    k.packet = v.data;
    k.packet_len = (uint16_t)v.caplen;
    k.packet_len_wire = (uint16_t)v.wirelen;
    k.payload = v.data + p.payload_off;
    // (payload_len can run past the captured bytes on malformed lengths -- parser.cpp:780-797 in
    // uint16_t; the reference's plugins then read past the frame: here the view ends at caplen)
    const uint32_t cap_left = p.payload_off < v.caplen ? v.caplen - p.payload_off : 0u;
    k.payload_len = (uint16_t)(p.payload_len < cap_left ? p.payload_len : cap_left);
    k.payload_len_wire = k.payload_len;
    k.source_pkt = v.source_pkt != 0;
}

// the record's basic fields into the Flow the hooks see (flowifc.hpp:245-268)
inline void fill_flow(ipxp::Flow& f, const ipxg_flow_record& r) {
    f.flow_hash = r.flow_hash;
    f.time_first.tv_sec = r.time_first_sec;
    f.time_first.tv_usec = r.time_first_usec;
    f.time_last.tv_sec = r.time_last_sec;
    f.time_last.tv_usec = r.time_last_usec;
    f.src_bytes = r.src_bytes;
    f.dst_bytes = r.dst_bytes;
    f.src_packets = r.src_packets;
    f.dst_packets = r.dst_packets;
    f.src_tcp_flags = r.src_tcp_flags;
    f.dst_tcp_flags = r.dst_tcp_flags;
    f.ip_version = r.ip_version;
    f.ip_proto = r.ip_proto;
    f.src_port = r.src_port;
    f.dst_port = r.dst_port;
    std::memcpy(&f.src_ip, r.src_ip, 16);
    std::memcpy(&f.dst_ip, r.dst_ip, 16);
    std::memcpy(f.src_mac, r.src_mac, 6);
    std::memcpy(f.dst_mac, r.dst_mac, 6);
    f.end_reason = r.end_reason;
}

// The pre-classifier rule of a plugin kind: the packets its hooks act on (a superset).
//   dns   port 53                        dns.cpp:97-127 (src_port / dst_port == 53)
//   http  method / "HTTP" prefixes, TCP  http.cpp:100-140 (is_request / is_response)
//   tls   payload 16 03 (handshake)      tls_parser.cpp:102-124 (record type 22, major 3)
//   quic  UDP, long-header bit           quic_parser.cpp:1058-1117; follows 30 packets of a
//                                        detected flow (QUIC_MAX_ELEMCOUNT, quic.cpp:340-346)
//   ntp   port 123                       ntp.cpp:82-90 (post_create only, FLOW_FLUSH)
//   sip   the 11 message-type prefixes   sip.cpp:105-172 (parse_msg_type: the payload's first
//                                        4 bytes; post_create claims, pre_update flushes)
//   wg    UDP, message types 1-4         wg.cpp:69-100, 140-147 (type byte, 3 zero bytes);
//                                        follows every packet of a claimed flow (pre_update
//                                        parses each: possible_wg, FLOW_FLUSH_WITH_REINSERT)
//   any other plugin (pstats, phists, bstats, mqtt, rtsp -- 17 prefixes, more than a rule holds --,
//   smtp, ...): every packet of every flow (ipxg_plugin.all_packets), as the reference calls
//   every hook for every packet: correct for any plugin, at the host walk's rate.
inline bool rule_for(const std::string& name, ipxg_plugin& q) {
    auto prefix = [&q](const char* s, uint8_t n) {
        q.prefix_len[q.n_prefixes] = n;
        std::memcpy(q.prefix[q.n_prefixes], s, n);
        q.n_prefixes++;
    };
    if (name == "dns") {
        q.proto_mask = 3;
        q.n_ports = 1;
        q.ports[0] = 53;
        q.follow_bytes = 1;  // (dns.cpp reads a payload only on port 53)
    } else if (name == "http") {
        q.proto_mask = 1;
        for (const char* m : {"GET ", "POST", "PUT ", "HEAD", "DELE", "TRAC", "OPTI", "CONN", "PATC", "HTTP"})
            prefix(m, 4);
    } else if (name == "tls") {
        q.proto_mask = 3;
        prefix("\x16\x03", 2);
    } else if (name == "quic") {
        q.proto_mask = 2;
        prefix("\x80", 1);
        q.masked = 1;
        q.prefix_mask[0][0] = 0x80;
        q.follow_packets = 30;
        // outside the rule (short header) QUICPlugin reads the payload's first byte only:
        // quic_parse_quic_bit and quic_long_header_packet's long-header test (quic_parser.cpp
        // :1160-1167, :1105-1117) before it gives up (quic.cpp:494-498)
        q.follow_bytes = 1;
    } else if (name == "ntp") {
        q.proto_mask = 3;
        q.n_ports = 1;
        q.ports[0] = 123;
    } else if (name == "sip") {
        q.proto_mask = 3;
        for (const char* m : {"INVI", "REGI", "NOTI", "OPTI", "CANC", "INFO", "SIP/", "ACK ", "BYE ", "SUBS", "PUBL"})
            prefix(m, 4);
    } else if (name == "wg") {
        q.proto_mask = 2;
        for (const char* m : {"\x01\0\0\0", "\x02\0\0\0", "\x03\0\0\0", "\x04\0\0\0"}) prefix(m, 4);
        q.follow_packets = 0xFFFFFFFFu;
    } else {
        q.all_packets = 1;
    }
    return true;
}

class Adapter {
public:
    explicit Adapter(ipxp::ProcessPlugin* p, bool owns = false) : m_p(p), m_owns(owns) {}
    ~Adapter() {
        if (m_owns) delete m_p;
    }
    Adapter(const Adapter&) = delete;
    Adapter& operator=(const Adapter&) = delete;

    // The ipxg_plugin of this adapter (ctx = this): the rule of `kind` and the five hooks.
    bool make(const std::string& kind, ipxg_plugin& q) {
        std::memset(&q, 0, sizeof(q));
        if (!rule_for(kind, q)) return false;
        q.ctx = this;
        // Every virtual is called inside guard(): a PluginError (plugin.hpp:81-91) -- or any other
        // exception -- must not cross the engine's C ABI; it becomes IPXG_PLUGIN_ERROR with the
        // message kept for q.error, and the engine fails the call with IPXG_EPLUGIN as the
        // reference's input worker reports it (workers.cpp:107-112).
        q.pre_create = [](void* c, ipxg_packet_view* v) -> int {
            Adapter* a = static_cast<Adapter*>(c);
            return a->guard([&] {
                ipxp::Packet k;
                fill_packet(k, *v);
                return a->m_p->pre_create(k);
            });
        };
        q.post_create = [](void* c, ipxg_flow_record* r, const ipxg_packet_view* v) -> int {
            return static_cast<Adapter*>(c)->call(r, v, [](ipxp::ProcessPlugin* p, ipxp::Flow& f, ipxp::Packet& k) {
                return p->post_create(f, k);
            });
        };
        q.pre_update = [](void* c, ipxg_flow_record* r, ipxg_packet_view* v) -> int {
            return static_cast<Adapter*>(c)->call(r, v, [](ipxp::ProcessPlugin* p, ipxp::Flow& f, ipxp::Packet& k) {
                return p->pre_update(f, k);
            });
        };
        q.post_update = [](void* c, ipxg_flow_record* r, const ipxg_packet_view* v) -> int {
            return static_cast<Adapter*>(c)->call(r, v, [](ipxp::ProcessPlugin* p, ipxp::Flow& f, ipxp::Packet& k) {
                return p->post_update(f, k);
            });
        };
        q.pre_export = [](void* c, ipxg_flow_record* r) {
            Adapter* a = static_cast<Adapter*>(c);
            (void)a->guard([&] {
                ipxp::Flow& f = a->flow(*r);
                a->m_p->pre_export(f);
                a->adopt(*r, f);
                return 0;
            });
        };
        q.error = [](void* c) -> const char* {  // a failure since the last call, taken
            Adapter* a = static_cast<Adapter*>(c);
            if (!a->m_fresh) return nullptr;
            a->m_fresh = false;
            return a->m_err.c_str();  // (valid until this instance fails again)
        };
        // a walk thread's own instance: ProcessPlugin::copy() (processPlugin.hpp:50), as the
        // reference copies every process plugin per storage pipeline (ipfixprobe.cpp:430-436)
        q.copy_ctx = [](void* c) -> void* {
            try {
                return new Adapter(static_cast<Adapter*>(c)->m_p->copy(), true);
            } catch (...) {
                return nullptr;
            }
        };
        q.free_ctx = [](void* c) { delete static_cast<Adapter*>(c); };
        return true;
    }

private:
    ipxp::Flow& flow(const ipxg_flow_record& r) {
        ipxp::Flow& f = r.ext ? *flow_of(r.ext) : m_scratch;
        fill_flow(f, r);
        return f;
    }
    // a first extension on a flow without one: the chain moves to a Flow of its own
    void adopt(ipxg_flow_record& r, ipxp::Flow& f) {
        if (!r.ext && f.m_exts) {
            ipxp::Flow* own = new ipxp::Flow(m_scratch);
            own->m_exts = m_scratch.m_exts;
            m_scratch.m_exts = nullptr;
            r.ext = reinterpret_cast<uintptr_t>(own);
        }
    }
    template <class F>
    int call(ipxg_flow_record* r, const ipxg_packet_view* v, F hook) {
        return guard([&] {
            ipxp::Packet k;
            fill_packet(k, *v);
            ipxp::Flow& f = flow(*r);
            const int ret = hook(m_p, f, k);
            adopt(*r, f);
            return ret;
        });
    }
    template <class F>
    int guard(F&& body) {
        std::string msg;
        try {
            return body();
        } catch (const ipxp::PluginError& x) {
            msg = std::string("PluginError: ") + x.what();
        } catch (const std::exception& x) {
            msg = x.what();
        } catch (...) {
            msg = "unknown exception";
        }
        if (!m_fresh) {  // the first failure since error() last took one
            m_err = msg;
            m_fresh = true;
        }
        return IPXG_PLUGIN_ERROR;
    }

    ipxp::ProcessPlugin* m_p;
    bool m_owns;
    std::string m_err;     // the first failure since q.error last took one
    bool m_fresh = false;  // m_err not taken yet
    ipxp::Flow m_scratch{};  // the hooks' Flow for a record without extensions
};

}  // namespace ipxg_ref
