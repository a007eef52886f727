// gpucache.hpp -- the "gpucache" storage plugin: ipfixprobe's StoragePlugin lifecycle
// (include/ipfixprobe/storagePlugin.hpp:33-172) over the ipxg C-ABI.
//
// Reference interface it replaces: NHTFlowCache (src/plugins/storage/cache/src/cache.hpp:
// 246-320) -- same option string (CacheOptParser, cache.hpp:81-221) plus dev=/batch=/dlt=,
// same entry points:
//   init(params)         -> ipxg_config_parse + ipxg_create       (cache.cpp:182-242)
//   put_pkt(Packet&)     -> buffer the raw frame; a full batch goes to ipxg_submit
//                           (the CPU parser's results in Packet are not used)
//   export_expired(ts)   -> flush the partial batch, ipxg_expire  (cache.cpp:508-523)
//   finish()             -> flush, ipxg_finish                    (cache.cpp:276-288)
// Exported records are handed to an ExportSink, the analogue of ipx_ring_push(&flow)
// (cache.cpp:270); INTEGRATION.md shows the adapter that fills ipxp::Flow and pushes it to
// the reference's ring.  Errors are thrown as PluginError, like the reference (plugin.hpp:81-91).
#pragma once

#include <sys/time.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ipxg.h"

namespace ipxp {

class PluginError : public std::runtime_error {
public:
    explicit PluginError(const std::string& m) : std::runtime_error(m) {}
};

// Raw-frame view of ipxp::Packet (packet.hpp:46-147): the fields the engine consumes.
struct RawPacket {
    struct timeval ts;
    const uint8_t* packet;     // Packet::packet
    uint16_t packet_len;       // Packet::packet_len (caplen)
    uint16_t packet_len_wire;  // Packet::packet_len_wire
};

class ExportSink {
public:
    virtual ~ExportSink() {}
    virtual void push(const ipxg_flow_record& rec) = 0;
};

// IPFIX output formatted on the device: the message stream the reference's IPFIX output
// plugin would send for the exported flows (ipxg_poll_ipfix_messages), handed over whole.
class MessageSink {
public:
    virtual ~MessageSink() {}
    virtual void messages(const uint8_t* data, size_t bytes, size_t records, size_t msgs) = 0;
};

class GpuFlowCache {
public:
    GpuFlowCache(const std::string& params, ExportSink* sink);
    ~GpuFlowCache();
    void init(const char* params);
    void close();
    std::string get_name() const { return "gpucache"; }
    int put_pkt(const RawPacket& pkt);
    void export_expired(time_t ts);
    void finish();
    void set_queue(ExportSink* sink) { m_sink = sink; }
    // exports go out as IPFIX messages (exporter state x: odid, mtu, dir, export time)
    void set_ipfix(MessageSink* sink, const ipxg_ipfix_exporter& x) {
        m_msg_sink = sink;
        m_ipfix = x;
    }
    ipxg_stats stats();
    // whole pre-built batch (arena + descriptors), bypassing the per-packet buffer
    void put_batch(const ipxg_batch& b);

private:
    void flush_batch();
    void drain();
    void check(int rc, const char* what);

    ipxg_engine* m_eng = nullptr;
    ipxg_config m_cfg;
    ExportSink* m_sink = nullptr;
    MessageSink* m_msg_sink = nullptr;
    ipxg_ipfix_exporter m_ipfix;
    std::vector<uint8_t> m_msg;
    std::vector<uint8_t> m_arena;
    std::vector<ipxg_pkt_desc> m_desc;
    std::vector<ipxg_flow_record> m_out;
};

}  // namespace ipxp
