// ipxg_probe -- minimal pipeline driver: pcap/pcapng file -> gpucache -> flow records.
//
//   ipxg_probe -i FILE [-s "s=20;a=300;i=30;..."] [-o csv|csv-vlan|ipfix:PATH] [--odid N]
//              [--export-time SEC] [--mtu N] [-q BLOCK] [--mbuf]
//
// The input side is ipfixprobe's input_storage_worker (workers.cpp:40-140) over the raw-ingest
// input plugin "pcapraw" (rawinput.hpp: the pcap plugin without the CPU parser): blocks of -q
// frames (default 64, ipfixprobe.cpp:56) in arrival order, each frame handed to the storage
// plugin (put_pkt); at end of file the storage is finished (workers.cpp:136).  --mbuf: every
// block goes through the DPDK burst adapter instead (burst_to_block), the frames copied into
// mbufs of rte_mbuf's layout (a 128-byte headroom, data_off / data_len) as rte_eth_rx_burst
// returns them.  Output is
// the basic biflow columns in the text form of the reference's functional tests (UniRec
// logger, tests/functional/scripts/run_test.sh), one line per exported flow, or (ipfix:PATH)
// the IPFIX message stream of the reference's IPFIX output plugin (basic templates), written
// to PATH as sent on the wire -- formatted and packed on the device.
#include <arpa/inet.h>
#include <sys/time.h>
#include <time.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "gpucache.hpp"
#include "rawinput.hpp"

namespace {

struct CsvSink : ipxp::ExportSink {
    FILE* f;
    bool vlan;
    size_t n = 0;
    explicit CsvSink(FILE* out, bool with_vlan) : f(out), vlan(with_vlan) {}
    static std::string ip(const uint8_t* a, int ver) {
        char b[INET6_ADDRSTRLEN];
        inet_ntop(ver == 4 ? AF_INET : AF_INET6, a, b, sizeof(b));
        return b;
    }
    static std::string mac(const uint8_t* m) {
        char b[32];
        snprintf(b, sizeof(b), "%02x:%02x:%02x:%02x:%02x:%02x", m[0], m[1], m[2], m[3], m[4], m[5]);
        return b;
    }
    static std::string tm(uint32_t s, uint32_t us) {
        time_t t = s;
        struct tm g;
        gmtime_r(&t, &g);
        char b[64];
        strftime(b, sizeof(b), "%Y-%m-%dT%H:%M:%S", &g);
        char o[80];
        snprintf(o, sizeof(o), "%s.%06u", b, us);
        return o;
    }
    void push(const ipxg_flow_record& r) override {
        n++;
        fprintf(f, "%s,%s,%llu,%llu,0,%s,%s,%s,%s,%u,%u,%u,%u,", ip(r.dst_ip, r.ip_version).c_str(),
                ip(r.src_ip, r.ip_version).c_str(), (unsigned long long)r.src_bytes, (unsigned long long)r.dst_bytes,
                tm(r.time_first_sec, r.time_first_usec).c_str(), tm(r.time_last_sec, r.time_last_usec).c_str(),
                mac(r.dst_mac).c_str(), mac(r.src_mac).c_str(), r.src_packets, r.dst_packets, r.dst_port, r.src_port);
        if (vlan) fprintf(f, "%u,", r.vlan_id);
        fprintf(f, "0,%u,%u,%u\n", r.ip_proto, r.src_tcp_flags, r.dst_tcp_flags);
    }
};

struct FileMessages : ipxp::MessageSink {
    FILE* f;
    size_t records = 0, msgs = 0;
    explicit FileMessages(FILE* out) : f(out) {}
    void messages(const uint8_t* data, size_t bytes, size_t n, size_t m) override {
        if (bytes && fwrite(data, 1, bytes, f) != bytes) throw ipxp::PluginError("ipxg_probe: write failed");
        records += n;
        msgs += m;
    }
};

// rte_mbuf's fields that the burst adapter reads (rte_mbuf_core.h: buf_addr, data_off,
// data_len, pkt_len), plus where this driver keeps the packet's timestamp (DPDK: a dynfield)
struct MockMbuf {
    void* buf_addr;
    uint16_t data_off;
    uint16_t data_len;
    uint32_t pkt_len;
    struct timeval ts;
    uint8_t room[128 + 65536];  // RTE_PKTMBUF_HEADROOM + data
};

void usage() {
    fprintf(stderr, "usage: ipxg_probe -i FILE [-s CACHE_OPTIONS] [-o csv|csv-vlan|ipfix:PATH] [--odid N] "
                    "[--export-time SEC] [--mtu N] [--stats] [-q BLOCK] [--mbuf]\n");
}

}  // namespace

int main(int argc, char** argv) {
    std::string in, opts, fmt = "csv";
    bool stats = false, mbuf = false;
    size_t qsize = 64;
    ipxg_ipfix_exporter x;
    ipxg_ipfix_exporter_init(&x);
    x.export_time = (uint32_t)time(nullptr);
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "-i" && i + 1 < argc) in = argv[++i];
        else if (a == "-s" && i + 1 < argc) opts = argv[++i];
        else if (a == "-o" && i + 1 < argc) fmt = argv[++i];
        else if (a == "--odid" && i + 1 < argc) x.odid = (uint32_t)strtoul(argv[++i], nullptr, 0);
        else if (a == "--export-time" && i + 1 < argc) x.export_time = (uint32_t)strtoul(argv[++i], nullptr, 0);
        else if (a == "--mtu" && i + 1 < argc) x.mtu = (uint16_t)strtoul(argv[++i], nullptr, 0);
        else if (a == "--stats") stats = true;
        else if (a == "-q" && i + 1 < argc) qsize = std::max<size_t>(1, strtoul(argv[++i], nullptr, 0));
        else if (a == "--mbuf") mbuf = true;
        else {
            usage();
            return 2;
        }
    }
    if (in.empty()) {
        usage();
        return 2;
    }
    ipxp::RawPcapReader input;
    try {
        input.init(("file=" + in).c_str());
    } catch (const ipxp::PluginError& e) {
        fprintf(stderr, "ipxg_probe: %s\n", e.what());
        return 1;
    }
    // the capture's link type, unless the option string names one
    ipxg_config probe_cfg;
    ipxg_config_default(&probe_cfg);
    probe_cfg.datalink = 0;
    if (ipxg_config_parse(opts.c_str(), &probe_cfg) != IPXG_OK) {
        fprintf(stderr, "ipxg_probe: invalid option string\n");
        return 2;
    }
    if (probe_cfg.datalink == 0) opts += (opts.empty() ? "" : ";") + std::string("dlt=") + std::to_string(input.datalink());
    CsvSink sink(stdout, fmt == "csv-vlan");
    FILE* ipfix_out = nullptr;
    if (fmt.rfind("ipfix:", 0) == 0) {
        ipfix_out = fopen(fmt.c_str() + 6, "wb");
        if (!ipfix_out) {
            fprintf(stderr, "ipxg_probe: cannot write %s\n", fmt.c_str() + 6);
            return 1;
        }
    }
    FileMessages msink(ipfix_out);
    try {
        ipxp::GpuFlowCache cache(opts, &sink);
        if (ipfix_out) cache.set_ipfix(&msink, x);
        ipxp::RawPacketBlock block(qsize), burst(qsize);
        std::vector<MockMbuf> pool(mbuf ? qsize : 0);
        std::vector<MockMbuf*> rx(mbuf ? qsize : 0);
        for (;;) {  // input_storage_worker (workers.cpp:66-122)
            const ipxp::InputResult r = input.get(block);
            if (r == ipxp::InputResult::END_OF_FILE) break;
            const ipxp::RawPacketBlock* b = &block;
            if (mbuf) {  // the frames as an rx burst of mbufs, back through the DPDK adapter
                for (size_t k = 0; k < block.cnt; ++k) {
                    MockMbuf& m = pool[k];
                    m.buf_addr = m.room;
                    m.data_off = 128;
                    m.data_len = block.pkts[k].packet_len;
                    m.pkt_len = block.pkts[k].packet_len_wire;
                    m.ts = block.pkts[k].ts;
                    std::memcpy(m.room + 128, block.pkts[k].packet, m.data_len);
                    rx[k] = &m;
                }
                ipxp::burst_to_block(rx.data(), (uint16_t)block.cnt, [](const MockMbuf* m) { return m->ts; }, burst);
                b = &burst;
            }
            for (size_t k = 0; k < b->cnt; ++k) cache.put_pkt(b->pkts[k]);
        }
        cache.finish();
        if (stats) {
            ipxg_stats s = cache.stats();
            fprintf(stderr, "packets seen %llu parsed %llu flows exported %llu (forced %llu, inactive %llu, "
                    "active %llu, eof %llu)\n",
                    (unsigned long long)s.seen_packets, (unsigned long long)s.parsed_packets,
                    (unsigned long long)s.total_exported, (unsigned long long)s.end_forced,
                    (unsigned long long)s.end_inactive, (unsigned long long)s.end_active,
                    (unsigned long long)s.end_eof);
        }
    } catch (const ipxp::PluginError& e) {
        fprintf(stderr, "ipxg_probe: %s\n", e.what());
        if (ipfix_out) fclose(ipfix_out);
        return 1;
    }
    if (ipfix_out) {
        fclose(ipfix_out);
        if (stats) fprintf(stderr, "ipfix: %zu records in %zu messages\n", msink.records, msink.msgs);
    }
    return 0;
}
