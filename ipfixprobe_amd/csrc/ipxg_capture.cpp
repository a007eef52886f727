// ipxg_capture.cpp -- host ingestion: classic pcap (us/ns, either byte order) and pcapng
// (EPB/SPB/PB, per-interface if_tsresol) into an ipxg batch.
//
// Mirrors what the reference's pcap input hands parse_packet (pcap.cpp:54-70, 258-293):
// libpcap opens files at microsecond precision, so nanosecond and other sub-us resolutions
// are scaled down by integer division; caplen/len are passed into uint16_t parameters, i.e.
// truncated mod 2^16.  Link types accepted are those PcapReader::check_datalink allows
// (pcap.cpp:178-200): EN10MB, LINUX_SLL, LINUX_SLL2, RAW (LINKTYPE_RAW 101 -> DLT_RAW 12).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/ipxg.h"

namespace {

struct Pkt {
    uint32_t sec, usec, caplen, wirelen;
    size_t off;  // into file buffer
};

uint32_t rd32(const uint8_t* p, bool swap) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}
uint16_t rd16(const uint8_t* p, bool swap) {
    uint16_t v;
    std::memcpy(&v, p, 2);
    return swap ? __builtin_bswap16(v) : v;
}

int map_linktype(uint32_t lt) {
    switch (lt) {
    case 1: return IPXG_DLT_EN10MB;
    case 101: case 12: case 14: return IPXG_DLT_RAW;
    case 113: return IPXG_DLT_LINUX_SLL;
    case 276: return IPXG_DLT_LINUX_SLL2;
    default: return -1;
    }
}

bool read_pcap(const std::vector<uint8_t>& d, std::vector<Pkt>& out, int& dlt) {
    if (d.size() < 24) return false;
    uint32_t m;
    std::memcpy(&m, d.data(), 4);
    bool swap = (m == 0xD4C3B2A1u || m == 0x4D3CB2A1u);
    bool nano = (m == 0xA1B23C4Du || m == 0x4D3CB2A1u);
    dlt = map_linktype(rd32(&d[20], swap) & 0x0FFFFFFF);
    size_t o = 24;
    while (o + 16 <= d.size()) {
        Pkt p;
        p.sec = rd32(&d[o], swap);
        uint32_t frac = rd32(&d[o + 4], swap);
        p.usec = nano ? frac / 1000 : frac;
        p.caplen = rd32(&d[o + 8], swap);
        p.wirelen = rd32(&d[o + 12], swap);
        o += 16;
        if (o + p.caplen > d.size()) break;  // truncated file
        p.off = o;
        o += p.caplen;
        out.push_back(p);
    }
    return true;
}

bool read_pcapng(const std::vector<uint8_t>& d, std::vector<Pkt>& out, int& dlt) {
    struct Iface {
        int dlt;
        uint64_t res;  // units per second
        bool dec;      // a power of ten (else a power of two)
    };
    std::vector<Iface> ifs;
    bool swap = false;
    size_t o = 0;
    dlt = -1;
    while (o + 12 <= d.size()) {
        uint32_t bt = rd32(&d[o], swap);
        if (bt == 0x0A0D0D0Au) {
            uint32_t bom;
            std::memcpy(&bom, &d[o + 8], 4);
            swap = (bom != 0x1A2B3C4Du);
            ifs.clear();
        }
        uint32_t bl = rd32(&d[o + 4], swap);
        if (bl < 12 || o + bl > d.size()) break;
        const uint8_t* body = &d[o + 8];
        size_t blen = bl - 12;
        if (bt == 1 && blen >= 8) {  // IDB
            Iface f{map_linktype(rd16(body, swap)), 1000000, true};
            size_t p = 8;
            while (p + 4 <= blen) {
                uint16_t code = rd16(body + p, swap), ol = rd16(body + p + 2, swap);
                if (code == 0) break;
                if (code == 9 && ol >= 1 && p + 5 <= blen) {  // if_tsresol
                    const uint8_t v = body[p + 4], ex = v & 0x7F;
                    f.dec = !(v & 0x80);
                    // a resolution that does not fit 64 bits (10^20, 2^64) cannot be a
                    // timestamp unit: reject the capture instead of dividing by zero
                    if (f.dec ? ex > 19 : ex > 63) return false;
                    f.res = 1;
                    for (int i = 0; i < ex; ++i) f.res *= f.dec ? 10 : 2;
                }
                p += 4 + ((ol + 3u) & ~3u);
            }
            ifs.push_back(f);
            if (dlt < 0) dlt = f.dlt;
        } else if ((bt == 6 || bt == 2) && blen >= 20) {  // EPB / obsolete PB
            uint32_t iid = bt == 6 ? rd32(body, swap) : rd16(body, swap);
            uint64_t t = ((uint64_t)rd32(body + 4, swap) << 32) | rd32(body + 8, swap);
            Pkt p;
            p.caplen = rd32(body + 12, swap);
            p.wirelen = rd32(body + 16, swap);
            if (iid >= ifs.size() || 20 + (size_t)p.caplen > blen) break;
            // libpcap's conversion to microseconds: a decimal resolution finer than 1 us divides
            // by the power of ten, anything else scales frac * 10^6 / res (128-bit: exact)
            const uint64_t res = ifs[iid].res;
            uint64_t sec = t / res, frac = t % res;
            if (ifs[iid].dec && res >= 1000000) frac /= (res / 1000000);
            else frac = (uint64_t)((unsigned __int128)frac * 1000000u / res);
            p.sec = (uint32_t)sec;
            p.usec = (uint32_t)frac;
            p.off = (size_t)(body + 20 - d.data());
            out.push_back(p);
        } else if (bt == 3 && blen >= 4) {  // SPB: no timestamp
            Pkt p;
            p.wirelen = rd32(body, swap);
            p.caplen = std::min<uint32_t>(p.wirelen, (uint32_t)(blen - 4));
            p.sec = p.usec = 0;
            p.off = (size_t)(body + 4 - d.data());
            out.push_back(p);
        }
        o += bl;
    }
    return dlt >= 0 || out.empty();
}

}  // namespace

extern "C" int ipxg_capture_load(const char* path, ipxg_capture** out) {
    if (!path || !out) return IPXG_EINVAL;
    *out = nullptr;
    FILE* f = std::fopen(path, "rb");
    if (!f) return IPXG_EIO;
    std::vector<uint8_t> d;
    uint8_t buf[1 << 16];
    size_t r;
    while ((r = std::fread(buf, 1, sizeof(buf), f)) > 0) d.insert(d.end(), buf, buf + r);
    std::fclose(f);
    if (d.size() < 4) return IPXG_EIO;
    uint32_t m;
    std::memcpy(&m, d.data(), 4);
    std::vector<Pkt> pk;
    int dlt = -1;
    bool ok;
    if (m == 0xA1B2C3D4u || m == 0xA1B23C4Du || m == 0xD4C3B2A1u || m == 0x4D3CB2A1u) ok = read_pcap(d, pk, dlt);
    else if (m == 0x0A0D0D0Au) ok = read_pcapng(d, pk, dlt);
    else return IPXG_EIO;
    if (!ok || dlt < 0) return IPXG_EIO;
    ipxg_capture* c = (ipxg_capture*)std::calloc(1, sizeof(ipxg_capture));
    if (!c) return IPXG_ENOMEM;
    uint64_t total = 0;
    for (auto& p : pk) total += ((uint64_t)(p.caplen & 0xFFFF) + 15) & ~15ull;
    if (total > (1ull << 32)) {
        std::free(c);
        return IPXG_ETOOBIG;
    }
    c->n = (uint32_t)pk.size();
    c->datalink = (uint32_t)dlt;
    c->arena_len = total ? total : 16;
    c->arena = (uint8_t*)std::aligned_alloc(64, (c->arena_len + 63) & ~63ull);
    c->desc = (ipxg_pkt_desc*)std::calloc(pk.size() ? pk.size() : 1, sizeof(ipxg_pkt_desc));
    if (!c->arena || !c->desc) {
        ipxg_capture_free(c);
        return IPXG_ENOMEM;
    }
    std::memset(c->arena, 0, (c->arena_len + 63) & ~63ull);
    uint64_t o = 0;
    for (size_t i = 0; i < pk.size(); ++i) {
        const uint32_t cl = pk[i].caplen & 0xFFFF;  // uint16_t parameter of parse_packet
        std::memcpy(c->arena + o, &d[pk[i].off], cl);
        c->desc[i].offset = (uint32_t)o;
        c->desc[i].caplen = (uint16_t)cl;
        c->desc[i].wirelen = (uint16_t)(pk[i].wirelen & 0xFFFF);
        c->desc[i].ts_sec = pk[i].sec;
        c->desc[i].ts_usec = pk[i].usec;
        o += ((uint64_t)cl + 15) & ~15ull;
    }
    *out = c;
    return IPXG_OK;
}

extern "C" void ipxg_capture_free(ipxg_capture* c) {
    if (!c) return;
    std::free(c->arena);
    std::free(c->desc);
    std::free(c);
}
