// gpucache.cpp -- see gpucache.hpp.
#include "gpucache.hpp"

#include <cstring>

namespace ipxp {

GpuFlowCache::GpuFlowCache(const std::string& params, ExportSink* sink) : m_sink(sink) {
    ipxg_ipfix_exporter_init(&m_ipfix);
    init(params.c_str());
}

GpuFlowCache::~GpuFlowCache() { close(); }

void GpuFlowCache::check(int rc, const char* what) {
    if (rc != IPXG_OK) {
        std::string msg = std::string("gpucache: ") + what + " failed (" + std::to_string(rc) + ")";
        if (m_eng) msg += ": " + std::string(ipxg_last_error(m_eng));
        throw PluginError(msg);
    }
}

void GpuFlowCache::init(const char* params) {
    ipxg_config_default(&m_cfg);
    if (ipxg_config_parse(params, &m_cfg) != IPXG_OK) throw PluginError("gpucache: invalid option string");
    if (m_sink == nullptr) throw PluginError("output queue must be set before init");  // cache.cpp:200-202
    check(ipxg_create(&m_cfg, &m_eng), "ipxg_create");
    m_arena.reserve((size_t)m_cfg.batch_pkts * 128);
    m_desc.reserve(m_cfg.batch_pkts);
}

void GpuFlowCache::close() {
    if (m_eng) {
        ipxg_destroy(m_eng);
        m_eng = nullptr;
    }
}

int GpuFlowCache::put_pkt(const RawPacket& pkt) {
    ipxg_pkt_desc d;
    d.offset = (uint32_t)m_arena.size();
    d.caplen = pkt.packet_len;
    d.wirelen = pkt.packet_len_wire;
    d.ts_sec = (uint32_t)pkt.ts.tv_sec;
    d.ts_usec = (uint32_t)pkt.ts.tv_usec;
    const size_t padded = ((size_t)pkt.packet_len + 15) & ~(size_t)15;
    if (m_arena.size() + padded > 0xFFFFFFF0ull) flush_batch();
    d.offset = (uint32_t)m_arena.size();
    m_arena.resize(m_arena.size() + padded, 0);
    std::memcpy(m_arena.data() + d.offset, pkt.packet, pkt.packet_len);
    m_desc.push_back(d);
    if (m_desc.size() >= m_cfg.batch_pkts) flush_batch();
    return 0;
}

void GpuFlowCache::put_batch(const ipxg_batch& b) {
    flush_batch();
    check(ipxg_submit(m_eng, &b), "ipxg_submit");
    drain();
}

void GpuFlowCache::flush_batch() {
    if (m_desc.empty()) return;
    ipxg_batch b;
    b.arena = m_arena.data();
    b.arena_len = m_arena.size();
    b.desc = m_desc.data();
    b.n = (uint32_t)m_desc.size();
    b.flags = 0;
    check(ipxg_submit(m_eng, &b), "ipxg_submit");
    m_arena.clear();
    m_desc.clear();
    drain();
}

void GpuFlowCache::drain() {
    size_t n = 0;
    check(ipxg_pending_exports(m_eng, &n), "ipxg_pending_exports");
    if (!n) return;
    if (m_msg_sink) {  // IPFIX messages formatted and packed on the device
        m_msg.resize(ipxg_ipfix_bound(n));
        size_t recs = 0, bytes = 0, msgs = 0;
        check(ipxg_poll_ipfix_messages(m_eng, &m_ipfix, m_msg.data(), m_msg.size(), &recs, &bytes, &msgs),
              "ipxg_poll_ipfix_messages");
        m_msg_sink->messages(m_msg.data(), bytes, recs, msgs);
        return;
    }
    m_out.resize(n);
    size_t got = 0;
    check(ipxg_poll_exports(m_eng, m_out.data(), n, &got), "ipxg_poll_exports");
    if (m_sink)
        for (size_t i = 0; i < got; ++i) m_sink->push(m_out[i]);
}

void GpuFlowCache::export_expired(time_t ts) {
    flush_batch();
    check(ipxg_expire(m_eng, (int64_t)ts), "ipxg_expire");
    drain();
}

void GpuFlowCache::finish() {
    flush_batch();
    check(ipxg_finish(m_eng), "ipxg_finish");
    drain();
}

ipxg_stats GpuFlowCache::stats() {
    ipxg_stats s;
    check(ipxg_get_stats(m_eng, &s), "ipxg_get_stats");
    return s;
}

}  // namespace ipxp
