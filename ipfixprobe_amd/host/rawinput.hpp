// rawinput.hpp -- the input side of the device path: input plugins
// that hand raw frames to the gpucache storage plugin without running the CPU parser.
//
// The reference's input plugins call parse_packet on every frame they read (pcap.cpp:258-293,
// dpdk.cpp:196-225, ndp.cpp:123-185) and fill the 200-byte Packet; with the device engine
// behind the storage plugin those parsed fields are never used (GpuFlowCache::put_pkt takes
// Packet::packet / packet_len / packet_len_wire / ts only), so:
//   RawPcapReader   "pcapraw": InputPlugin::get(PacketBlock&) of the pcap plugin with the parse
//                   left out -- a block of raw frames per call, Result::PARSED until
//                   Result::END_OF_FILE (pcap.cpp:258-293); the capture read by the engine's
//                   own pcap/pcapng reader (ipxg_capture_load: classic µs/ns, pcapng, the
//                   link types of pcap.cpp:178-200);
//   burst_to_block  a DPDK rx burst (rte_eth_rx_burst's rte_mbuf* array) as a raw block: frame
//                   = rte_pktmbuf_mtod(m) (buf_addr + data_off), length = rte_pktmbuf_data_len(m)
//                   for both caplen and wire length, the device's timestamp of each mbuf
//                   (DpdkDevice::getPacketTimestamp: NIC or system time) -- exactly what
//                   DpdkReader::get passes to parse_packet (dpdk.cpp:206-214).  A template over
//                   the mbuf type: DPDK is absent here, so it is compiled and tested against a
//                   struct with rte_mbuf's field names (ipxg_probe --mbuf); in the reference tree
//                   it takes struct rte_mbuf itself.
// The driver loop is input_storage_worker's (workers.cpp:66-122): get a block, put_pkt each
// frame, finish at END_OF_FILE (ipxg_probe.cpp).
#pragma once

#include <sys/time.h>

#include <cstdint>
#include <string>
#include <vector>

#include "gpucache.hpp"

namespace ipxp {

// InputPlugin::Result (inputPlugin.hpp:43-49)
enum class InputResult { TIMEOUT = 0, PARSED, NOT_PARSED, END_OF_FILE, ERROR };

// PacketBlock (packet.hpp:149-164) of raw frames
struct RawPacketBlock {
    std::vector<RawPacket> pkts;
    size_t cnt = 0;
    size_t bytes = 0;
    explicit RawPacketBlock(size_t size) : pkts(size) {}
    size_t size() const { return pkts.size(); }
};

class RawPcapReader {
public:
    RawPcapReader() = default;
    explicit RawPcapReader(const std::string& params) { init(params.c_str()); }
    ~RawPcapReader() { close(); }
    RawPcapReader(const RawPcapReader&) = delete;
    RawPcapReader& operator=(const RawPcapReader&) = delete;

    // "file=PATH" / "f=PATH" (the pcap plugin's option names, pcap.hpp PcapOptParser)
    void init(const char* params) {
        std::string p = params ? params : "", file;
        size_t at = 0;
        while (at <= p.size()) {
            const size_t end = p.find(';', at);
            const std::string tok = p.substr(at, end == std::string::npos ? std::string::npos : end - at);
            const size_t eq = tok.find('=');
            const std::string k = tok.substr(0, eq), v = eq == std::string::npos ? "" : tok.substr(eq + 1);
            if (k == "file" || k == "f") file = v;
            else if (!k.empty()) throw PluginError("pcapraw: unknown option " + k);
            if (end == std::string::npos) break;
            at = end + 1;
        }
        if (file.empty()) throw PluginError("pcapraw: no file= given");
        close();
        const int rc = ipxg_capture_load(file.c_str(), &m_cap);
        if (rc != IPXG_OK) throw PluginError("pcapraw: cannot read " + file + " (" + std::to_string(rc) + ")");
        m_next = 0;
    }
    void close() {
        if (m_cap) ipxg_capture_free(m_cap);
        m_cap = nullptr;
    }
    std::string get_name() const { return "pcapraw"; }
    // link type of the capture (IPXG_DLT_*): the storage plugin's dlt=
    uint32_t datalink() const { return m_cap ? m_cap->datalink : IPXG_DLT_EN10MB; }

    InputResult get(RawPacketBlock& block) {
        if (!m_cap) throw PluginError("pcapraw: no file opened");
        block.cnt = 0;
        block.bytes = 0;
        while (block.cnt < block.size() && m_next < m_cap->n) {
            const ipxg_pkt_desc& d = m_cap->desc[m_next++];
            RawPacket& p = block.pkts[block.cnt++];
            p.ts.tv_sec = d.ts_sec;
            p.ts.tv_usec = d.ts_usec;
            p.packet = m_cap->arena + d.offset;
            p.packet_len = d.caplen;
            p.packet_len_wire = d.wirelen;
            block.bytes += d.wirelen;  // pblock->bytes += len (parser.cpp:804)
        }
        m_seen += block.cnt;
        return block.cnt ? InputResult::PARSED : InputResult::END_OF_FILE;
    }
    uint64_t seen() const { return m_seen; }

private:
    ipxg_capture* m_cap = nullptr;
    uint32_t m_next = 0;
    uint64_t m_seen = 0;
};

// rte_pktmbuf_mtod / rte_pktmbuf_data_len on any mbuf type with rte_mbuf's fields
template <class Mbuf>
inline const uint8_t* mbuf_data(const Mbuf* m) {
    return static_cast<const uint8_t*>(m->buf_addr) + m->data_off;
}

// A burst of n mbufs (arrival order) into block: DpdkReader::get without parse_packet.
// ts_of(const Mbuf*) -> timeval: the packet's timestamp (DpdkDevice::getPacketTimestamp).
template <class Mbuf, class TsOf>
inline InputResult burst_to_block(Mbuf* const* mbufs, uint16_t n, TsOf ts_of, RawPacketBlock& block) {
    block.cnt = 0;
    block.bytes = 0;
    if (!n) return InputResult::TIMEOUT;  // nothing received (dpdk.cpp:202-204)
    if (block.size() < n) block.pkts.resize(n);
    for (uint16_t i = 0; i < n; ++i) {
        RawPacket& p = block.pkts[block.cnt++];
        p.ts = ts_of(mbufs[i]);
        p.packet = mbuf_data(mbufs[i]);
        p.packet_len = mbufs[i]->data_len;
        p.packet_len_wire = mbufs[i]->data_len;
        block.bytes += mbufs[i]->data_len;
    }
    return InputResult::PARSED;
}

}  // namespace ipxp
