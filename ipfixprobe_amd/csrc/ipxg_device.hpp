// ipxg_device.hpp -- device-side building blocks of the MI355X packet -> biflow engine.
//
// * byte sources: the parser reads a frame through one of two sources --
//     LdsWin : the first IPXG_WIN bytes of the frame staged in LDS by the loading lane
//              (dword-interleaved across the block so a wave's same-offset reads hit 64
//              consecutive banks), falling back to global memory past the window;
//     GlobalSrc: byte-addressed reads straight from HBM (creator re-parse, slow path).
//   Both return 0 for bytes at or beyond caplen (the reference reads whatever memory
//   follows in those cases -- undefined behaviour, outside the parity contract).
// * xxh64_16 / xxh64_40: XXH64 (xxhash.h:2725-2901) specialised for the 16 B IPv4 and
//   40 B IPv6 flow keys and the 40 B fragmentation key, on 64-bit words in registers.
// * parse_frame<FULL>: parse_packet (parser.cpp:673-805) as an iterative state machine
//   (the reference recurses IPv4 -> GRE -> IPv4/IPv6/MPLS/PPPoE and MPLS -> Eth); every
//   bounds check, uint16_t wrap and quirk is kept (see DESIGN.md "parser quirks").
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ipxg.h"

#define IPXG_BLOCK 256        // packets per tile (one lane each)
#define IPXG_WIN 128          // header bytes staged in LDS per packet (B_pkt)
#define IPXG_WIN_DW (IPXG_WIN / 4)
#define IPXG_MAX_L3_HOPS 64   // bound on the GRE/MPLS/PPPoE header chain (reference: recursion)
#define IPXG_MAX_EXT_STEPS 4096  // bound on the IPv6 extension-header walk (reference: may not return)

namespace ipxg {

// ---- protocol constants (reference headers.hpp:35-62, parser.hpp:41-57) ---------------
constexpr uint16_t ETH_P_8021AD = 0x88A8, ETH_P_8021Q = 0x8100, ETH_P_IP = 0x0800,
                   ETH_P_IPV6 = 0x86DD, ETH_P_MPLS_UC = 0x8847, ETH_P_MPLS_MC = 0x8848,
                   ETH_P_PPP_SES = 0x8864, ETH_P_TRILL = 0x22F3;
constexpr uint16_t GRE_CHECKSUM = 0x8000, GRE_KEY = 0x2000, GRE_SEQNUM = 0x1000;

// ---- byte sources ---------------------------------------------------------------------
__device__ __forceinline__ uint16_t bswap16(uint32_t x) { return (uint16_t)(((x & 0xFF) << 8) | ((x >> 8) & 0xFF)); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

struct GlobalSrc {
    const uint8_t* p;
    uint32_t cap;
    __device__ __forceinline__ uint32_t b(uint32_t o) const { return o < cap ? (uint32_t)p[o] : 0u; }
    // 4 bytes starting at o, memory order (byte o in bits 0..7)
    __device__ __forceinline__ uint32_t le32(uint32_t o) const {
        return b(o) | (b(o + 1) << 8) | (b(o + 2) << 16) | (b(o + 3) << 24);
    }
};

// Bytes past the staged window (deep header chains only): out of line, so the ~60 read sites of
// the parser do not each carry an inlined copy of the byte loads (code size: the slow pass's
// kernel outgrew the instruction cache).
__device__ __noinline__ uint32_t far_le32(const uint8_t* p, uint32_t cap, uint32_t o) {
    const GlobalSrc g{p, cap};
    return g.le32(o);
}

// Per-lane view of the LDS-staged window.  win points at dword 0 of this lane's column;
// dword d lives at win[d * IPXG_BLOCK].
struct LdsWin {
    const uint32_t* win;
    GlobalSrc g;
    __device__ __forceinline__ uint32_t dw(uint32_t d) const { return win[d * IPXG_BLOCK]; }
    __device__ __forceinline__ uint32_t le32(uint32_t o) const {
        if (o + 4 <= IPXG_WIN) {
            uint32_t d = o >> 2, sh = o & 3;
            uint32_t lo = dw(d);
            if (sh == 0) return lo;
            uint32_t hi = (d + 1 < IPXG_WIN_DW) ? dw(d + 1) : 0u;
            return __builtin_amdgcn_alignbyte(hi, lo, sh);
        }
        return far_le32(g.p, g.cap, o);
    }
    __device__ __forceinline__ uint32_t b(uint32_t o) const {
        if (o < IPXG_WIN) return (dw(o >> 2) >> ((o & 3) * 8)) & 0xFF;
        return far_le32(g.p, g.cap, o) & 0xFF;
    }
};

template <class S> __device__ __forceinline__ uint32_t rd8(const S& s, uint32_t o) { return s.b(o); }
template <class S> __device__ __forceinline__ uint32_t rd16(const S& s, uint32_t o) { return bswap16(s.le32(o)); }
template <class S> __device__ __forceinline__ uint32_t rd32(const S& s, uint32_t o) { return bswap32(s.le32(o)); }

// ---- XXH64 (xxhash.h:2725-2901) ---------------------------------------------------------
constexpr uint64_t XP1 = 0x9E3779B185EBCA87ULL, XP2 = 0xC2B2AE3D27D4EB4FULL,
                   XP3 = 0x165667B19E3779F9ULL, XP4 = 0x85EBCA77C2B2AE63ULL,
                   XP5 = 0x27D4EB2F165667C5ULL;
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xx_round(uint64_t acc, uint64_t in) {
    acc += in * XP2;
    acc = rotl64(acc, 31);
    return acc * XP1;
}
__device__ __forceinline__ uint64_t xx_merge(uint64_t acc, uint64_t v) {
    acc ^= xx_round(0, v);
    return acc * XP1 + XP4;
}
__device__ __forceinline__ uint64_t xx_aval(uint64_t h) {
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}
// len 16, seed 0: h = P5 + 16, two 8-byte finalize rounds (xxhash.h:2804-2810)
__device__ __forceinline__ uint64_t xxh64_16(uint64_t w0, uint64_t w1) {
    uint64_t h = XP5 + 16;
    h ^= xx_round(0, w0);
    h = rotl64(h, 27) * XP1 + XP4;
    h ^= xx_round(0, w1);
    h = rotl64(h, 27) * XP1 + XP4;
    return xx_aval(h);
}
// len 40, seed 0: one 32-byte stripe (:2849-2873) + one 8-byte tail round
__device__ __forceinline__ uint64_t xxh64_40(uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3,
                                             uint64_t w4) {
    uint64_t v1 = XP1 + XP2, v2 = XP2, v3 = 0, v4 = 0 - XP1;
    v1 = xx_round(v1, w0);
    v2 = xx_round(v2, w1);
    v3 = xx_round(v3, w2);
    v4 = xx_round(v4, w3);
    uint64_t h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xx_merge(h, v1);
    h = xx_merge(h, v2);
    h = xx_merge(h, v3);
    h = xx_merge(h, v4);
    h += 40;
    h ^= xx_round(0, w4);
    h = rotl64(h, 27) * XP1 + XP4;
    return xx_aval(h);
}
// generic length (tests / tools)
__device__ inline uint64_t xxh64_any(const uint8_t* p, uint32_t len, uint64_t seed) {
    auto r64 = [](const uint8_t* q) {
        uint64_t v = 0;
        for (int i = 7; i >= 0; --i) v = (v << 8) | q[i];
        return v;
    };
    uint64_t h;
    const uint8_t* s = p;
    if (len >= 32) {
        const uint8_t* limit = p + len - 31;
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        do {
            v1 = xx_round(v1, r64(s));
            v2 = xx_round(v2, r64(s + 8));
            v3 = xx_round(v3, r64(s + 16));
            v4 = xx_round(v4, r64(s + 24));
            s += 32;
        } while (s < limit);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xx_merge(h, v1);
        h = xx_merge(h, v2);
        h = xx_merge(h, v3);
        h = xx_merge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += len;
    uint32_t rem = len & 31;
    while (rem >= 8) {
        h ^= xx_round(0, r64(s));
        s += 8;
        h = rotl64(h, 27) * XP1 + XP4;
        rem -= 8;
    }
    if (rem >= 4) {
        uint32_t v = s[0] | (s[1] << 8) | (s[2] << 16) | ((uint32_t)s[3] << 24);
        h ^= (uint64_t)v * XP1;
        s += 4;
        h = rotl64(h, 23) * XP2 + XP3;
        rem -= 4;
    }
    while (rem > 0) {
        h ^= (uint64_t)(*s++) * XP5;
        h = rotl64(h, 11) * XP1;
        --rem;
    }
    return xx_aval(h);
}

// ---- parsed packet (flow-relevant subset of ipxp::Packet, packet.hpp:46-147) -----------
struct DevPkt {
    uint32_t sip[4], dip[4];   // address bytes in memory order, 4 per word
    uint32_t vlan_id;
    uint32_t frag_id;
    uint16_t ethertype, ip_len, src_port, dst_port, frag_off;
    uint8_t ip_version, ip_proto, tcp_flags, more_fragments;
    uint8_t l4;  // 6 / 17: parse_tcp_hdr / parse_udp_hdr read the ports (TopPorts counted them,
                 // parser.cpp:484-485, 563-564) -- for TCP even when the packet is then dropped
    // FULL-only fields
    uint32_t mac_lo, mac_mid, mac_hi;  // dst_mac[0..5] src_mac[0..5] packed in memory order
    uint32_t mpls_top, tcp_seq, tcp_ack, tcp_mss;
    uint64_t tcp_options;
    uint16_t tcp_window;
    uint8_t ip_ttl, ip_tos, ip_flags;
    uint16_t ip_payload_len;            // Packet::ip_payload_len (parser.cpp:332, 412, 436)
    uint16_t payload_off, payload_len;  // Packet::payload / payload_len (parser.cpp:780-797)
};

// parser counters kept per lane and reduced per block (parser-stats.hpp:126-201)
struct ParseCounts {
    uint32_t seen, parsed, unknown, ipv4, ipv6, tcp, udp, mpls, pppoe, trill, vlan;
    uint32_t ipv4_bytes, ipv6_bytes;
};

// Ethernet header (parse_eth_hdr parser.cpp:68-155).  Returns hdr_len, 0 + err on throw.
template <bool FULL, class S>
__device__ __forceinline__ uint32_t parse_eth(const S& s, uint32_t base, uint32_t data_len,
                                              uint32_t& ethertype, uint32_t& vlan_id, DevPkt* macs,
                                              bool& err) {
    if (14 > data_len) { err = true; return 0; }
    uint32_t hdr_len = 14;
    uint32_t et = rd16(s, base + 12);
    if (FULL && macs) {
        macs->mac_lo = s.le32(base);
        macs->mac_mid = s.le32(base + 4);
        macs->mac_hi = s.le32(base + 8);
    }
    vlan_id = 0;
    if (et == ETH_P_8021AD || et == ETH_P_8021Q) {
        if (4 > (int)data_len - (int)hdr_len) { err = true; return 0; }
        vlan_id = rd16(s, base + hdr_len) & 0x0FFF;
        hdr_len += 4;
        et = rd16(s, base + hdr_len - 2);
    }
    while (et == ETH_P_8021Q) {
        if (4 > (int)data_len - (int)hdr_len) { err = true; return 0; }
        hdr_len += 4;
        et = rd16(s, base + hdr_len - 2);
    }
    ethertype = et;
    return hdr_len & 0xFFFF;
}

// IPv4 header fields (parse_ipv4_hdr parser.cpp:328-339)
template <bool FULL, class S>
__device__ __forceinline__ void ipv4_fields(const S& s, uint32_t base, uint32_t ihl, uint32_t proto,
                                            DevPkt& p) {
    p.ip_version = 4;
    p.ip_proto = (uint8_t)proto;
    p.ip_len = (uint16_t)rd16(s, base + 2);
    uint32_t fo = rd16(s, base + 6);
    p.sip[0] = s.le32(base + 12);
    p.dip[0] = s.le32(base + 16);
    p.sip[1] = p.sip[2] = p.sip[3] = 0;
    p.dip[1] = p.dip[2] = p.dip[3] = 0;
    p.frag_id = rd16(s, base + 4);
    p.frag_off = (uint16_t)(fo & 0x1FFF);
    p.more_fragments = (fo & 0x2000) ? 1 : 0;
    if (FULL) {
        p.ip_tos = (uint8_t)rd8(s, base + 1);
        p.ip_ttl = (uint8_t)rd8(s, base + 8);
        p.ip_flags = (uint8_t)((fo & 0xE000) >> 13);
        p.ip_payload_len = (uint16_t)(p.ip_len - ihl);
    }
}

// IPv6 header + extension-header walk (parse_ipv6_hdr :423-460, skip_ipv6_ext_hdrs :365-414).
// Returns the header length (u16), sets err on throw.
template <bool FULL, class S>
__device__ __forceinline__ uint32_t parse_ipv6(const S& s, uint32_t base, uint32_t data_len, DevPkt& p,
                                               bool& err) {
    if (40 > data_len) { err = true; return 0; }
    p.ip_version = 6;
    uint32_t proto = rd8(s, base + 6);
    p.ip_proto = (uint8_t)proto;
    uint32_t plen = rd16(s, base + 4);
    p.ip_len = (uint16_t)(plen + 40);
    for (int k = 0; k < 4; ++k) {
        p.sip[k] = s.le32(base + 8 + 4 * k);
        p.dip[k] = s.le32(base + 24 + 4 * k);
    }
    if (FULL) {
        p.ip_tos = (uint8_t)((rd32(s, base) & 0x0ff00000) >> 20);
        p.ip_ttl = (uint8_t)rd8(s, base + 7);
        p.ip_flags = 0;
        p.ip_payload_len = (uint16_t)plen;
    }
    uint32_t hdr_len = 40;
    if (proto != 6 && proto != 17) {
        const uint32_t eb = base + 40;
        const uint32_t dl = (data_len - 40) & 0xFFFF;
        uint32_t ext = eb, next_hdr = proto, hdrs_len = 0;
        for (int step = 0;; ++step) {
            if (hdrs_len > dl || 2u > dl - hdrs_len) { err = true; return 0; }
            if (step >= IPXG_MAX_EXT_STEPS) { err = true; return 0; }  // AH +2/-2 cycle, see oracle
            if (next_hdr == 0 || next_hdr == 60) {
                hdrs_len += (rd8(s, ext + 1) << 3) + 8;
            } else if (next_hdr == 43) {
                hdrs_len += (rd8(s, eb + hdrs_len + 1) << 3) + 8;
            } else if (next_hdr == 51) {
                hdrs_len += (uint32_t)(((int)rd8(s, ext + 1) << 2) - 2);  // AH quirk :382
            } else if (next_hdr == 44) {
                uint32_t fr = eb + hdrs_len;
                p.frag_id = rd32(s, fr + 4);
                uint32_t fo = rd16(s, fr + 2);
                p.frag_off = (uint16_t)(fo & 0xFFF8);
                p.more_fragments = (fo & 0x1) ? 1 : 0;
                hdrs_len += 8;
            } else if (next_hdr == 135) {
                hdrs_len += (rd8(s, ext + 1) << 3) + 8;
                if (rd8(s, ext) == 59) {
                    p.ip_proto = 59;
                    break;
                }
            } else {
                break;
            }
            if (hdrs_len > 65535u) { err = true; return 0; }
            next_hdr = rd8(s, ext);
            ext = eb + hdrs_len;
            p.ip_proto = (uint8_t)next_hdr;
        }
        if (hdrs_len > 65535u) { err = true; return 0; }
        hdr_len = (hdr_len + hdrs_len) & 0xFFFF;
        if (FULL) p.ip_payload_len = (uint16_t)(p.ip_payload_len - hdrs_len);
    }
    return hdr_len;
}

enum L3Kind : uint32_t { L3_IPV4, L3_IPV6, L3_GRE, L3_MPLS, L3_PPPOE, L3_DONE };

// The L3 chain reached from ethertype dispatch (parser.cpp:734-748): IPv4 -> GRE ->
// {IPv4, IPv6, MPLS, PPPoE}, MPLS -> {IPv4, IPv6, EoMPLS}, PPPoE -> {IPv4, IPv6}.  Each
// reference function returns its own length plus its callee's, as uint16_t; the sum is
// accumulated mod 2^16 here (EoMPLS *replaces* the running MPLS length, parser.cpp:625).
template <bool FULL, class S>
__device__ __forceinline__ uint32_t parse_l3(const S& s, uint32_t kind, uint32_t base, uint32_t dl,
                                             uint32_t caplen, DevPkt& p, bool& err) {
    uint32_t total = 0;
    for (int hop = 0; hop < IPXG_MAX_L3_HOPS; ++hop) {
        dl &= 0xFFFF;
        if (kind == L3_IPV4) {
            if (20 > dl) { err = true; return 0; }
            uint32_t ihl = (rd8(s, base) & 0x0F) << 2;
            uint32_t proto = rd8(s, base + 9);
            if (proto == 47) {
                if (dl < ihl) { err = true; return 0; }
                total += ihl;
                base += ihl;
                dl -= ihl;
                kind = L3_GRE;
                continue;
            }
            ipv4_fields<FULL>(s, base, ihl, proto, p);
            return (total + ihl) & 0xFFFF;
        } else if (kind == L3_IPV6) {
            uint32_t r = parse_ipv6<FULL>(s, base, dl, p, err);
            if (err) return 0;
            return (total + r) & 0xFFFF;
        } else if (kind == L3_GRE) {  // parse_gre :256-302
            uint32_t gre_len = 4;
            if (dl < gre_len) { err = true; return 0; }
            uint32_t flags = rd16(s, base), type = rd16(s, base + 2);
            if (flags & GRE_CHECKSUM) gre_len += 4;
            if (flags & GRE_KEY) gre_len += 4;
            if (flags & GRE_SEQNUM) gre_len += 4;
            if (dl < gre_len) { err = true; return 0; }
            base += gre_len;
            dl -= gre_len;
            if (type == ETH_P_IP) kind = L3_IPV4;
            else if (type == ETH_P_IPV6) kind = L3_IPV6;
            else if (type == ETH_P_MPLS_UC || type == ETH_P_MPLS_MC) kind = L3_MPLS;
            else if (type == ETH_P_PPP_SES) kind = L3_PPPOE;
            else {
                p.ip_proto = 47;  // IPPROTO_GRE; GRE itself contributes 0 (:298-300)
                return total & 0xFFFF;
            }
            total += gre_len;
        } else if (kind == L3_MPLS) {  // process_mpls :611-634, process_mpls_stack :581-602
            if (FULL) p.mpls_top = rd32(s, base);
            uint32_t length = 0, w;
            do {
                uint32_t m = base + length;
                length = (length + 4) & 0xFFFF;
                if (0 > (int)dl - (int)length) { err = true; return 0; }
                if (m + 4 > caplen) { err = true; return 0; }  // see oracle process_mpls_stack
                w = rd32(s, m);
            } while (!(w & 0x100));
            uint32_t nh = (rd8(s, base + length) & 0xF0) >> 4;
            if (nh == 4 || nh == 6) {
                total += length;
                base += length;
                dl = (dl - length) & 0xFFFF;
                kind = nh == 4 ? L3_IPV4 : L3_IPV6;
            } else if (nh == 0) {
                length = (length + 4) & 0xFFFF;
                uint32_t tmp_et, tmp_vlan;
                uint32_t L = parse_eth<false>(s, base + length, (dl - length) & 0xFFFF, tmp_et,
                                              tmp_vlan, nullptr, err);
                if (err) return 0;
                total += L;  // `length = parse_eth_hdr(...)` drops the stack length
                if (tmp_et == ETH_P_IP || tmp_et == ETH_P_IPV6) {
                    base += L;
                    dl = (dl - L) & 0xFFFF;
                    kind = tmp_et == ETH_P_IP ? L3_IPV4 : L3_IPV6;
                } else {
                    return total & 0xFFFF;
                }
            } else {
                return (total + length) & 0xFFFF;
            }
        } else {  // L3_PPPOE, process_pppoe :643-671
            if (8 > dl) { err = true; return 0; }
            uint32_t nh = rd16(s, base + 6);
            total += 8;
            if (rd8(s, base + 1) != 0) return total & 0xFFFF;
            if (nh == 0x0021) kind = L3_IPV4;
            else if (nh == 0x0057) kind = L3_IPV6;
            else return total & 0xFFFF;
            base += 8;
            dl -= 8;
        }
    }
    err = true;  // header chain deeper than IPXG_MAX_L3_HOPS
    return 0;
}

// parse_tcp_hdr :469-543.  Returns hdr_len, err on throw.
template <bool FULL, class S>
__device__ __forceinline__ uint32_t parse_tcp(const S& s, uint32_t base, uint32_t data_len, DevPkt& p,
                                              bool& err) {
    if (20 > data_len) { err = true; return 0; }
    uint32_t w0 = s.le32(base);
    p.src_port = bswap16(w0);
    p.dst_port = bswap16(w0 >> 16);
    p.l4 = 6;
    uint32_t w3 = s.le32(base + 12);
    p.tcp_flags = (uint8_t)(w3 >> 8);
    if (FULL) {
        p.tcp_seq = rd32(s, base + 4);
        p.tcp_ack = rd32(s, base + 8);
        p.tcp_window = bswap16(w3 >> 16);
    }
    int hdr_len = (int)((w3 & 0xFF) >> 4) << 2;
    int hdr_opt_len = hdr_len - 20;
    if (hdr_len > (int)data_len) { err = true; return 0; }
    int i = 0;
    while (i < hdr_opt_len) {
        uint32_t opt = base + 20 + (uint32_t)i;
        uint32_t kind = rd8(s, opt);
        if (i + 1 >= hdr_opt_len) {
            if (kind <= 1) return (uint32_t)hdr_len;
            err = true;
            return 0;
        }
        uint32_t opt_len = kind <= 1 ? 1 : rd8(s, opt + 1);
        if (FULL) p.tcp_options |= 1ULL << (((kind & 0xF8) + (7 - (kind & 7))) & 63);
        if (kind == 0) break;
        if (FULL && kind == 2) p.tcp_mss = rd32(s, opt + 2);
        if (opt_len == 0) { err = true; return 0; }
        i += (int)opt_len;
    }
    return (uint32_t)hdr_len;
}

// parse_packet :673-805 with parse_all = false.  Returns valid (pblock->cnt++).
template <bool FULL, class S>
__device__ __forceinline__ bool parse_frame(const S& s, uint32_t caplen, uint32_t dlt, DevPkt& p,
                                            ParseCounts& c) {
    p.ip_version = 0; p.ip_proto = 0; p.tcp_flags = 0; p.more_fragments = 0;
    p.ethertype = 0; p.ip_len = 0; p.src_port = 0; p.dst_port = 0; p.frag_off = 0;
    p.vlan_id = 0; p.frag_id = 0; p.l4 = 0;
    for (int k = 0; k < 4; ++k) p.sip[k] = p.dip[k] = 0;
    if (FULL) {
        p.mac_lo = p.mac_mid = p.mac_hi = 0;
        p.mpls_top = p.tcp_seq = p.tcp_ack = p.tcp_mss = 0;
        p.tcp_options = 0;
        p.tcp_window = 0;
        p.ip_ttl = p.ip_tos = p.ip_flags = 0;
        p.ip_payload_len = p.payload_off = p.payload_len = 0;
    }
    c.seen++;
    bool err = false;
    uint32_t off = 0, et = 0;
    if (dlt == 0 || dlt == IPXG_DLT_EN10MB) {
        uint32_t vl;
        off = parse_eth<FULL>(s, 0, caplen, et, vl, &p, err);
        if (err) return false;
        p.vlan_id = vl;
    } else if (dlt == IPXG_DLT_LINUX_SLL) {  // parse_sll :165-189
        if (16 > caplen) return false;
        if (FULL) {
            uint32_t ha = rd16(s, 2);
            uint32_t a0 = s.le32(6), a1 = s.le32(10);
            p.mac_lo = 0;
            p.mac_mid = ha == 1 ? (a0 << 16) : 0;
            p.mac_hi = ha == 1 ? ((a0 >> 16) | (a1 << 16)) : 0;
        }
        et = rd16(s, 14);
        off = 16;
    } else if (dlt == IPXG_DLT_LINUX_SLL2) {  // parse_sll2 :192-217
        if (20 > caplen) return false;
        if (FULL) {
            uint32_t ha = rd16(s, 8);
            uint32_t a0 = s.le32(12), a1 = s.le32(16);
            p.mac_lo = 0;
            p.mac_mid = ha == 1 ? (a0 << 16) : 0;
            p.mac_hi = ha == 1 ? ((a0 >> 16) | (a1 << 16)) : 0;
        }
        et = rd16(s, 0);
        off = 20;
    } else if (dlt == IPXG_DLT_RAW) {
        uint32_t v = rd8(s, 0) & 0xF0;
        et = v == 0x40 ? ETH_P_IP : (v == 0x60 ? ETH_P_IPV6 : 0);
    } else {
        c.unknown++;
        return false;
    }
    if (et == ETH_P_TRILL) {  // :728-732
        uint32_t dl = (caplen - off) & 0xFFFF;
        if (6 > dl) return false;
        uint32_t b0 = rd8(s, off), b1 = rd8(s, off + 1);
        uint32_t op_len = (((b0 & 7) << 2) | (b1 >> 6)) & 0xFF;
        off = (off + 6 + ((op_len * 4) & 0xFF)) & 0xFFFF;
        c.trill++;
        uint32_t vl;
        uint32_t r = parse_eth<FULL>(s, off, (caplen - off) & 0xFFFF, et, vl, &p, err);
        if (err) return false;
        p.vlan_id = vl;
        off = (off + r) & 0xFFFF;
    }
    p.ethertype = (uint16_t)et;
    const uint32_t l3_off = off;
    uint32_t kind;
    if (et == ETH_P_IP) kind = L3_IPV4;
    else if (et == ETH_P_IPV6) kind = L3_IPV6;
    else if (et == ETH_P_MPLS_UC || et == ETH_P_MPLS_MC) kind = L3_MPLS;
    else if (et == ETH_P_PPP_SES) kind = L3_PPPOE;
    else {
        c.unknown++;
        return false;
    }
    uint32_t r = parse_l3<FULL>(s, kind, off, (caplen - off) & 0xFFFF, caplen, p, err);
    if (err) return false;
    c.mpls += kind == L3_MPLS ? 1u : 0u;
    c.pppoe += kind == L3_PPPOE ? 1u : 0u;
    off = (off + r) & 0xFFFF;
    const uint32_t l4_off = off;
    if (p.frag_off == 0) {
        if (p.ip_proto == 6) {
            const uint32_t h = parse_tcp<FULL>(s, off, (caplen - off) & 0xFFFF, p, err);
            if (err) return false;
            off = (off + h) & 0xFFFF;
        } else if (p.ip_proto == 17) {  // parse_udp_hdr :552-573
            if (8 > ((caplen - off) & 0xFFFF)) return false;
            uint32_t w0 = s.le32(off);
            p.src_port = bswap16(w0);
            p.dst_port = bswap16(w0 >> 16);
            p.l4 = 17;
            off = (off + 8) & 0xFFFF;
        }
    }
    c.tcp += p.l4 == 6 ? 1u : 0u;  // (branch-free: see the counters below)
    c.udp += p.l4 == 17 ? 1u : 0u;
    if (FULL) {  // payload, parser.cpp:780-797 (uint16_t arithmetic as there)
        uint32_t pkt_len = caplen, wire;
        if (l4_off != l3_off) {
            if (l4_off + p.ip_payload_len < 64) pkt_len = (l4_off + p.ip_payload_len) & 0xFFFF;
            wire = (p.ip_payload_len - (off - l4_off)) & 0xFFFF;
        } else {
            wire = (pkt_len - off) & 0xFFFF;
        }
        uint32_t plen = wire;
        if (plen + off > pkt_len) plen = (pkt_len - off) & 0xFFFF;
        p.payload_off = (uint16_t)off;
        p.payload_len = (uint16_t)plen;
    }
    // branch-free counter updates: with if/else the compiler merged them into one update at a
    // selected field offset, which put the whole ParseCounts in scratch memory
    const uint32_t is4 = et == ETH_P_IP ? 1u : 0u, is6 = et == ETH_P_IPV6 ? 1u : 0u;
    c.vlan += p.vlan_id ? 1u : 0u;
    c.ipv4 += is4;
    c.ipv4_bytes += is4 ? caplen : 0u;
    c.ipv6 += is6;
    c.ipv6_bytes += is6 ? caplen : 0u;
    c.parsed++;
    return true;
}

// ---- flow key words (cache.hpp:29-46 packed layout, little-endian 64-bit words) ---------
struct FlowKey {
    uint64_t w[5];
    uint32_t len;  // 16, 40 or 0
};

__device__ __forceinline__ void build_keys(const DevPkt& p, FlowKey& fwd, FlowKey& inv) {
    const uint64_t vl = (uint64_t)(p.vlan_id & 0xFFFF);
    const uint64_t sp = p.src_port, dp = p.dst_port, pr = p.ip_proto;
    if (p.ip_version == 4) {
        fwd.len = inv.len = 16;
        fwd.w[0] = sp | (dp << 16) | (pr << 32) | (4ull << 40) | ((uint64_t)(p.sip[0] & 0xFFFF) << 48);
        fwd.w[1] = (uint64_t)(p.sip[0] >> 16) | ((uint64_t)p.dip[0] << 16) | (vl << 48);
        inv.w[0] = dp | (sp << 16) | (pr << 32) | (4ull << 40) | ((uint64_t)(p.dip[0] & 0xFFFF) << 48);
        inv.w[1] = (uint64_t)(p.dip[0] >> 16) | ((uint64_t)p.sip[0] << 16) | (vl << 48);
    } else if (p.ip_version == 6) {
        fwd.len = inv.len = 40;
        const uint32_t* s = p.sip;
        const uint32_t* d = p.dip;
        auto mk = [&](FlowKey& k, uint64_t a, uint64_t b, const uint32_t* x, const uint32_t* y) {
            k.w[0] = a | (b << 16) | (pr << 32) | (6ull << 40) | ((uint64_t)(x[0] & 0xFFFF) << 48);
            k.w[1] = (uint64_t)(x[0] >> 16) | ((uint64_t)x[1] << 16) | ((uint64_t)(x[2] & 0xFFFF) << 48);
            k.w[2] = (uint64_t)(x[2] >> 16) | ((uint64_t)x[3] << 16) | ((uint64_t)(y[0] & 0xFFFF) << 48);
            k.w[3] = (uint64_t)(y[0] >> 16) | ((uint64_t)y[1] << 16) | ((uint64_t)(y[2] & 0xFFFF) << 48);
            k.w[4] = (uint64_t)(y[2] >> 16) | ((uint64_t)y[3] << 16) | (vl << 48);
        };
        mk(fwd, sp, dp, s, d);
        mk(inv, dp, sp, d, s);
    } else {
        fwd.len = inv.len = 0;
    }
}

__device__ __forceinline__ uint64_t key_hash(const FlowKey& k) {
    return k.len == 16 ? xxh64_16(k.w[0], k.w[1]) : xxh64_40(k.w[0], k.w[1], k.w[2], k.w[3], k.w[4]);
}

// FragmentationKey (fragmentationKeyData.hpp:49-82), 40 B packed, hashed with XXH64
__device__ __forceinline__ uint64_t frag_key_hash(const DevPkt& p) {
    const uint64_t ver = p.ip_version;
    const uint32_t* s = p.sip;
    const uint32_t* d = p.dip;
    uint64_t w0 = ver | ((uint64_t)s[0] << 16) | ((uint64_t)(s[1] & 0xFFFF) << 48);
    uint64_t w1 = (uint64_t)(s[1] >> 16) | ((uint64_t)s[2] << 16) | ((uint64_t)(s[3] & 0xFFFF) << 48);
    uint64_t w2 = (uint64_t)(s[3] >> 16) | ((uint64_t)d[0] << 16) | ((uint64_t)(d[1] & 0xFFFF) << 48);
    uint64_t w3 = (uint64_t)(d[1] >> 16) | ((uint64_t)d[2] << 16) | ((uint64_t)(d[3] & 0xFFFF) << 48);
    uint64_t w4 = (uint64_t)(d[3] >> 16) | ((uint64_t)p.frag_id << 16) | ((uint64_t)(p.vlan_id & 0xFFFF) << 48);
    return xxh64_40(w0, w1, w2, w3, w4);
}

}  // namespace ipxg
