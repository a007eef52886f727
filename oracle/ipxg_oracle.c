/*
 * ipxg_oracle.c -- CPU restatement of ipfixprobe's parse -> XXH64 -> NHTFlowCache path.
 * TEST INFRASTRUCTURE ONLY (see ipxg_oracle.h).  Each function cites the reference
 * file:line it restates; paths are relative to /root/reference.
 */
#include "ipxg_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ===================================================================================== */
/* XXH64 -- src/plugins/storage/cache/src/xxhash.h:2725-2901 (xxHash 0.8.1)             */
/* ===================================================================================== */
#define XP1 0x9E3779B185EBCA87ULL /* xxhash.h:2725 */
#define XP2 0xC2B2AE3D27D4EB4FULL
#define XP3 0x165667B19E3779F9ULL
#define XP4 0x85EBCA77C2B2AE63ULL
#define XP5 0x27D4EB2F165667C5ULL

static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t rd64le(const uint8_t* p)
{
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}
static uint32_t rd32le(const uint8_t* p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
/* XXH64_round xxhash.h:2754-2760 */
static uint64_t xx_round(uint64_t acc, uint64_t in)
{
    acc += in * XP2;
    acc = rotl64(acc, 31);
    return acc * XP1;
}
/* XXH64_mergeRound :2762-2768 */
static uint64_t xx_merge(uint64_t acc, uint64_t val)
{
    val = xx_round(0, val);
    acc ^= val;
    return acc * XP1 + XP4;
}
/* XXH64_avalanche :2771-2778 */
static uint64_t xx_aval(uint64_t h)
{
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}

/* XXH64_endian_align + XXH64_finalize, xxhash.h:2799-2873 */
uint64_t oracle_xxh64(const void* data, size_t len, uint64_t seed)
{
    const uint8_t* p = (const uint8_t*)data;
    uint64_t h;
    if (len >= 32) {
        const uint8_t* limit = p + len - 31;
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        do {
            v1 = xx_round(v1, rd64le(p));
            v2 = xx_round(v2, rd64le(p + 8));
            v3 = xx_round(v3, rd64le(p + 16));
            v4 = xx_round(v4, rd64le(p + 24));
            p += 32;
        } while (p < limit);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xx_merge(h, v1);
        h = xx_merge(h, v2);
        h = xx_merge(h, v3);
        h = xx_merge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += (uint64_t)len;
    size_t rem = len & 31;
    while (rem >= 8) {
        h ^= xx_round(0, rd64le(p));
        p += 8;
        h = rotl64(h, 27) * XP1 + XP4;
        rem -= 8;
    }
    if (rem >= 4) {
        h ^= (uint64_t)rd32le(p) * XP1;
        p += 4;
        h = rotl64(h, 23) * XP2 + XP3;
        rem -= 4;
    }
    while (rem > 0) {
        h ^= (uint64_t)(*p++) * XP5;
        h = rotl64(h, 11) * XP1;
        --rem;
    }
    return xx_aval(h);
}

/* n keys of keylen bytes, back to back -> XXH64 of each (test helper: flow-hash shards of a
 * synthetic mix on the CPU) */
void oracle_xxh64_batch(const uint8_t* keys, size_t keylen, size_t n, uint64_t seed, uint64_t* out)
{
    for (size_t i = 0; i < n; ++i) out[i] = oracle_xxh64(keys + i * keylen, keylen, seed);
}

/* ===================================================================================== */
/* Parser -- src/plugins/input/parser/parser.cpp                                         */
/* Offsets are absolute byte offsets into the frame; "data_len" values are uint16_t     */
/* exactly where the reference passes uint16_t parameters (so they wrap identically).   */
/* A `throw` of the reference is modelled by setting c->err and unwinding.              */
/* ===================================================================================== */
#define ETH_P_8021AD 0x88A8 /* headers.hpp:35 */
#define ETH_P_8021Q 0x8100
#define ETH_P_IP 0x0800
#define ETH_P_IPV6 0x86DD
#define ETH_P_MPLS_UC 0x8847
#define ETH_P_MPLS_MC 0x8848
#define ETH_P_PPP_SES 0x8864
#define ETH_P_TRILL 0x22F3 /* parser.hpp:57 */
#define GRE_CHECKSUM 0x8000 /* headers.hpp:60-62 */
#define GRE_KEY 0x2000
#define GRE_SEQNUM 0x1000
#define IPV6_FRAGMENT_OFFSET 0xFFF8 /* headers.hpp:53-54 */
#define IPV6_MORE_FRAGMENTS 0x1
#define IPXG_MAX_EXT_STEPS 4096

typedef struct {
    uint16_t ethertype;
    uint32_t vlan_id;
    uint8_t src_mac[6];
    uint8_t dst_mac[6];
} eth_out;

/* ParserStats' side counters (parser-stats.hpp:126-201, topPorts.hpp) */
typedef struct {
    uint64_t tcp[65536], udp[65536];
    ipxg_vlan_stats vlan[IPXG_VLAN_IDS];
} pstats;

typedef struct {
    const uint8_t* d;
    uint32_t cap;
    int beyond;
    int err;
    ipxg_parsed_pkt* p;
    uint16_t ip_payload_len;
    ipxg_stats* st;
    pstats* ps; /* may be null */
} pctx;

static uint8_t B8(pctx* c, uint32_t o)
{
    if (o < c->cap) return c->d[o];
    c->beyond = 1;
    return 0;
}
static uint16_t BE16(pctx* c, uint32_t o) { return (uint16_t)((B8(c, o) << 8) | B8(c, o + 1)); }
static uint32_t BE32(pctx* c, uint32_t o)
{
    return ((uint32_t)B8(c, o) << 24) | ((uint32_t)B8(c, o + 1) << 16) | ((uint32_t)B8(c, o + 2) << 8) |
           B8(c, o + 3);
}
static void COPY(pctx* c, uint8_t* dst, uint32_t o, int n)
{
    for (int i = 0; i < n; ++i) dst[i] = B8(c, o + (uint32_t)i);
}
#define THROW(c)         \
    do {                 \
        (c)->err = 1;    \
        return 0;        \
    } while (0)
#define CHK(c)               \
    do {                     \
        if ((c)->err) return 0; \
    } while (0)

/* parse_eth_hdr parser.cpp:68-155 */
static uint16_t parse_eth_hdr(pctx* c, uint32_t base, uint16_t data_len, eth_out* e)
{
    if (14 > data_len) THROW(c);
    uint16_t hdr_len = 14;
    uint16_t ethertype = BE16(c, base + 12);
    COPY(c, e->dst_mac, base, 6);
    COPY(c, e->src_mac, base + 6, 6);
    e->vlan_id = 0;
    if (ethertype == ETH_P_8021AD || ethertype == ETH_P_8021Q) {
        if (4 > (int)data_len - (int)hdr_len) THROW(c);
        uint16_t vlan = BE16(c, base + hdr_len);
        e->vlan_id = vlan & 0x0FFF;
        hdr_len += 4;
        ethertype = BE16(c, base + hdr_len - 2);
    }
    while (ethertype == ETH_P_8021Q) {
        if (4 > (int)data_len - (int)hdr_len) THROW(c);
        hdr_len += 4;
        ethertype = BE16(c, base + hdr_len - 2);
    }
    e->ethertype = ethertype;
    return hdr_len;
}

static void eth_to_pkt(const eth_out* e, ipxg_parsed_pkt* p)
{
    memcpy(p->dst_mac, e->dst_mac, 6);
    memcpy(p->src_mac, e->src_mac, 6);
    p->vlan_id = e->vlan_id;
    p->ethertype = e->ethertype;
}

/* parse_sll parser.cpp:165-189 (struct sll_header: pkttype, hatype, halen, addr[8], protocol) */
static uint16_t parse_sll(pctx* c, uint16_t data_len)
{
    if (16 > data_len) THROW(c);
    if (BE16(c, 2) == 1) COPY(c, c->p->src_mac, 6, 6); /* ARPHRD_ETHER */
    else memset(c->p->src_mac, 0, 6);
    memset(c->p->dst_mac, 0, 6);
    c->p->ethertype = BE16(c, 14);
    return 16;
}

/* parse_sll2 parser.cpp:192-217 (struct sll2_header: protocol, mbz, if_index, hatype,
 * pkttype, halen, addr[8]) */
static uint16_t parse_sll2(pctx* c, uint16_t data_len)
{
    if (20 > data_len) THROW(c);
    if (BE16(c, 8) == 1) COPY(c, c->p->src_mac, 12, 6);
    else memset(c->p->src_mac, 0, 6);
    memset(c->p->dst_mac, 0, 6);
    c->p->ethertype = BE16(c, 0);
    return 20;
}

/* parse_trill parser.cpp:228-249; trill_hdr little-endian bitfields headers.hpp:230-246 */
static uint16_t parse_trill(pctx* c, uint32_t base, uint16_t data_len)
{
    if (6 > data_len) THROW(c);
    uint8_t b0 = B8(c, base), b1 = B8(c, base + 1);
    uint8_t op_len = (uint8_t)(((b0 & 0x7) << 2) | (b1 >> 6));
    uint8_t op_len_bytes = (uint8_t)(op_len * 4);
    return (uint16_t)(6 + op_len_bytes);
}

static uint16_t parse_ipv4_hdr(pctx* c, uint32_t base, uint16_t data_len);
static uint16_t parse_ipv6_hdr(pctx* c, uint32_t base, uint16_t data_len);
static uint16_t process_mpls(pctx* c, uint32_t base, uint16_t data_len);
static uint16_t process_pppoe(pctx* c, uint32_t base, uint16_t data_len);

/* parse_gre parser.cpp:256-302 */
static uint16_t parse_gre(pctx* c, uint32_t base, uint16_t data_len)
{
    int gre_len = 4;
    if (data_len < gre_len) THROW(c);
    uint16_t flags = BE16(c, base);
    uint16_t type = BE16(c, base + 2);
    if (flags & GRE_CHECKSUM) gre_len += 4;
    if (flags & GRE_KEY) gre_len += 4;
    if (flags & GRE_SEQNUM) gre_len += 4;
    if (data_len < gre_len) THROW(c);
    base += (uint32_t)gre_len;
    data_len = (uint16_t)(data_len - gre_len);
    uint16_t r;
    switch (type) {
    case ETH_P_IP:
        r = parse_ipv4_hdr(c, base, data_len);
        CHK(c);
        return (uint16_t)(r + gre_len);
    case ETH_P_IPV6:
        r = parse_ipv6_hdr(c, base, data_len);
        CHK(c);
        return (uint16_t)(r + gre_len);
    case ETH_P_MPLS_UC:
    case ETH_P_MPLS_MC:
        r = process_mpls(c, base, data_len);
        CHK(c);
        return (uint16_t)(r + gre_len);
    case ETH_P_PPP_SES:
        r = process_pppoe(c, base, data_len);
        CHK(c);
        return (uint16_t)(r + gre_len);
    default:
        c->p->ip_proto = 47; /* IPPROTO_GRE */
        return 0;
    }
}

/* parse_ipv4_hdr parser.cpp:311-356 */
static uint16_t parse_ipv4_hdr(pctx* c, uint32_t base, uint16_t data_len)
{
    if (20 > data_len) THROW(c);
    const int ihl = (B8(c, base) & 0x0F) << 2;
    uint8_t protocol = B8(c, base + 9);
    if (protocol == 47) {
        if (data_len < ihl) THROW(c);
        uint16_t r = parse_gre(c, base + (uint32_t)ihl, (uint16_t)(data_len - ihl));
        CHK(c);
        return (uint16_t)(r + ihl);
    }
    ipxg_parsed_pkt* p = c->p;
    p->ip_version = 4;
    p->ip_proto = protocol;
    p->ip_tos = B8(c, base + 1);
    p->ip_len = BE16(c, base + 2);
    c->ip_payload_len = (uint16_t)(p->ip_len - ihl);
    p->ip_ttl = B8(c, base + 8);
    uint16_t fo = BE16(c, base + 6);
    p->ip_flags = (uint8_t)((fo & 0xE000) >> 13);
    memset(p->src_ip, 0, 16);
    memset(p->dst_ip, 0, 16);
    COPY(c, p->src_ip, base + 12, 4);
    COPY(c, p->dst_ip, base + 16, 4);
    p->frag_id = BE16(c, base + 4);
    p->frag_off = fo & 0x1FFF;
    p->more_fragments = (fo & 0x2000) ? 1 : 0;
    return (uint16_t)ihl;
}

/* skip_ipv6_ext_hdrs parser.cpp:365-414 */
static uint16_t skip_ipv6_ext_hdrs(pctx* c, uint32_t base, uint16_t data_len)
{
    ipxg_parsed_pkt* p = c->p;
    uint32_t ext = base;
    uint8_t next_hdr = p->ip_proto;
    uint32_t hdrs_len = 0;
    for (int step = 0;; ++step) {
        if (hdrs_len > data_len || 2u > (uint32_t)data_len - hdrs_len) THROW(c);
        /* AH with length 1 then 0 moves the walk +2/-2 forever (parser.cpp:382): the
         * reference never returns.  Walks longer than IPXG_MAX_EXT_STEPS are malformed here. */
        if (step >= IPXG_MAX_EXT_STEPS) {
            c->beyond = 1;
            THROW(c);
        }
        if (next_hdr == 0 || next_hdr == 60) { /* HOPOPTS, DSTOPTS */
            hdrs_len += ((uint32_t)B8(c, ext + 1) << 3) + 8;
        } else if (next_hdr == 43) { /* ROUTING */
            hdrs_len += ((uint32_t)B8(c, base + hdrs_len + 1) << 3) + 8;
        } else if (next_hdr == 51) { /* AH: (len << 2) - 2, parser.cpp:382 */
            hdrs_len += (uint32_t)(((int)B8(c, ext + 1) << 2) - 2);
        } else if (next_hdr == 44) { /* FRAGMENT */
            uint32_t fr = base + hdrs_len;
            p->frag_id = BE32(c, fr + 4);
            uint16_t fo = BE16(c, fr + 2);
            p->frag_off = fo & IPV6_FRAGMENT_OFFSET;
            p->more_fragments = (fo & IPV6_MORE_FRAGMENTS) ? 1 : 0;
            hdrs_len += 8;
        } else if (next_hdr == 135) { /* MH */
            hdrs_len += ((uint32_t)B8(c, ext + 1) << 3) + 8;
            if (B8(c, ext) == 59) {
                p->ip_proto = 59;
                break;
            }
        } else {
            break;
        }
        if (hdrs_len > 65535u) THROW(c);
        next_hdr = B8(c, ext);
        ext = base + hdrs_len;
        p->ip_proto = next_hdr;
    }
    if (hdrs_len > 65535u) THROW(c);
    c->ip_payload_len = (uint16_t)(c->ip_payload_len - hdrs_len);
    return (uint16_t)hdrs_len;
}

/* parse_ipv6_hdr parser.cpp:423-460 */
static uint16_t parse_ipv6_hdr(pctx* c, uint32_t base, uint16_t data_len)
{
    uint16_t hdr_len = 40;
    if (40 > data_len) THROW(c);
    ipxg_parsed_pkt* p = c->p;
    p->ip_version = 6;
    p->ip_tos = (uint8_t)((BE32(c, base) & 0x0ff00000) >> 20);
    p->ip_proto = B8(c, base + 6);
    p->ip_ttl = B8(c, base + 7);
    p->ip_flags = 0;
    c->ip_payload_len = BE16(c, base + 4);
    p->ip_len = (uint16_t)(c->ip_payload_len + 40);
    COPY(c, p->src_ip, base + 8, 16);
    COPY(c, p->dst_ip, base + 24, 16);
    if (p->ip_proto != 6 && p->ip_proto != 17) {
        uint16_t r = skip_ipv6_ext_hdrs(c, base + hdr_len, (uint16_t)(data_len - hdr_len));
        CHK(c);
        hdr_len = (uint16_t)(hdr_len + r);
    }
    return hdr_len;
}

/* parse_tcp_hdr parser.cpp:469-543 */
static uint16_t parse_tcp_hdr(pctx* c, uint32_t base, uint16_t data_len)
{
    if (20 > data_len) THROW(c);
    ipxg_parsed_pkt* p = c->p;
    p->src_port = BE16(c, base);
    p->dst_port = BE16(c, base + 2);
    p->tcp_seq = BE32(c, base + 4);
    p->tcp_ack = BE32(c, base + 8);
    p->tcp_flags = B8(c, base + 13);
    p->tcp_window = BE16(c, base + 14);
    if (c->ps) { /* top_ports.increment_tcp_frequency, parser.cpp:484-485 (before the doff check) */
        c->ps->tcp[p->src_port]++;
        c->ps->tcp[p->dst_port]++;
    }
    int hdr_len = (B8(c, base + 12) >> 4) << 2;
    int hdr_opt_len = hdr_len - 20;
    int i = 0;
    if (hdr_len > data_len) THROW(c);
    while (i < hdr_opt_len) {
        uint32_t opt = base + 20 + (uint32_t)i;
        uint8_t kind = B8(c, opt);
        if (i + 1 >= hdr_opt_len) {
            if (kind <= 1) return (uint16_t)hdr_len;
            THROW(c);
        }
        uint8_t opt_len = (uint8_t)(kind <= 1 ? 1 : B8(c, opt + 1));
        /* shift count taken mod 64, as the x86-64 / gfx950 shifters do (parser.cpp:528) */
        p->tcp_options |= 1ULL << (((kind & 0xF8) + (7 - (kind & 7))) & 63);
        if (kind == 0) break;
        if (kind == 2) p->tcp_mss = BE32(c, opt + 2);
        if (opt_len == 0) THROW(c);
        i += opt_len;
    }
    return (uint16_t)hdr_len;
}

/* parse_udp_hdr parser.cpp:552-573 */
static uint16_t parse_udp_hdr(pctx* c, uint32_t base, uint16_t data_len)
{
    if (8 > data_len) THROW(c);
    c->p->src_port = BE16(c, base);
    c->p->dst_port = BE16(c, base + 2);
    if (c->ps) { /* parser.cpp:563-564 */
        c->ps->udp[c->p->src_port]++;
        c->ps->udp[c->p->dst_port]++;
    }
    return 8;
}

/* process_mpls_stack parser.cpp:581-602 */
static uint16_t process_mpls_stack(pctx* c, uint32_t base, uint16_t data_len)
{
    uint16_t length = 0;
    uint32_t w;
    do {
        uint32_t m = base + length;
        length = (uint16_t)(length + 4);
        if (0 > (int)data_len - (int)length) THROW(c);
        /* A label word past caplen is only reachable through a wrapped data_len (the
         * reference then reads out of bounds, and with zero fill would never see BoS):
         * defined here as malformed. */
        if (m + 4 > c->cap) {
            c->beyond = 1;
            THROW(c);
        }
        w = BE32(c, m);
    } while (!(w & 0x100));
    return length;
}

/* process_mpls parser.cpp:611-634 (EoMPLS keeps the reference's `length =` at :625) */
static uint16_t process_mpls(pctx* c, uint32_t base, uint16_t data_len)
{
    c->p->mpls_top = BE32(c, base);
    uint16_t length = process_mpls_stack(c, base, data_len);
    CHK(c);
    uint8_t next_hdr = (uint8_t)((B8(c, base + length) & 0xF0) >> 4);
    uint16_t r;
    if (next_hdr == 4) {
        r = parse_ipv4_hdr(c, base + length, (uint16_t)(data_len - length));
        CHK(c);
        length = (uint16_t)(length + r);
    } else if (next_hdr == 6) {
        r = parse_ipv6_hdr(c, base + length, (uint16_t)(data_len - length));
        CHK(c);
        length = (uint16_t)(length + r);
    } else if (next_hdr == 0) {
        eth_out tmp;
        memset(&tmp, 0, sizeof(tmp));
        length = (uint16_t)(length + 4);
        length = parse_eth_hdr(c, base + length, (uint16_t)(data_len - length), &tmp);
        CHK(c);
        if (tmp.ethertype == ETH_P_IP) {
            r = parse_ipv4_hdr(c, base + length, (uint16_t)(data_len - length));
            CHK(c);
            length = (uint16_t)(length + r);
        } else if (tmp.ethertype == ETH_P_IPV6) {
            r = parse_ipv6_hdr(c, base + length, (uint16_t)(data_len - length));
            CHK(c);
            length = (uint16_t)(length + r);
        }
    }
    return length;
}

/* process_pppoe parser.cpp:643-671 */
static uint16_t process_pppoe(pctx* c, uint32_t base, uint16_t data_len)
{
    if (8 > data_len) THROW(c);
    uint16_t next_hdr = BE16(c, base + 6);
    uint16_t length = 8;
    if (B8(c, base + 1) != 0) return length; /* code */
    uint16_t r;
    if (next_hdr == 0x0021) {
        r = parse_ipv4_hdr(c, base + length, (uint16_t)(data_len - length));
        CHK(c);
        length = (uint16_t)(length + r);
    } else if (next_hdr == 0x0057) {
        r = parse_ipv6_hdr(c, base + length, (uint16_t)(data_len - length));
        CHK(c);
        length = (uint16_t)(length + r);
    }
    return length;
}

/* parse_packet parser.cpp:673-805 (parse_all = false, as every input plugin passes) */
static int parse_packet(pctx* c, uint16_t caplen, uint32_t datalink)
{
    ipxg_parsed_pkt* p = c->p;
    ipxg_stats* st = c->st;
    uint16_t data_offset = 0;
    uint32_t l3_hdr_offset, l4_hdr_offset;
    eth_out e;
    st->seen_packets++;
    if (datalink == 0 || datalink == IPXG_DLT_EN10MB) {
        data_offset = parse_eth_hdr(c, 0, caplen, &e);
        if (c->err) return 0;
        eth_to_pkt(&e, p);
    } else if (datalink == IPXG_DLT_LINUX_SLL) {
        data_offset = parse_sll(c, caplen);
        if (c->err) return 0;
    } else if (datalink == IPXG_DLT_LINUX_SLL2) {
        data_offset = parse_sll2(c, caplen);
        if (c->err) return 0;
    } else if (datalink == IPXG_DLT_RAW) {
        uint8_t v = B8(c, 0) & 0xF0;
        if (v == 0x40) p->ethertype = ETH_P_IP;
        else if (v == 0x60) p->ethertype = ETH_P_IPV6;
    } else {
        st->unknown_packets++;
        return 0;
    }
    if (p->ethertype == ETH_P_TRILL) {
        data_offset = (uint16_t)(data_offset + parse_trill(c, data_offset, (uint16_t)(caplen - data_offset)));
        if (c->err) return 0;
        st->trill_packets++;
        uint16_t r = parse_eth_hdr(c, data_offset, (uint16_t)(caplen - data_offset), &e);
        if (c->err) return 0;
        eth_to_pkt(&e, p);
        data_offset = (uint16_t)(data_offset + r);
    }
    uint16_t r;
    l3_hdr_offset = data_offset;
    if (p->ethertype == ETH_P_IP) {
        r = parse_ipv4_hdr(c, data_offset, (uint16_t)(caplen - data_offset));
        if (c->err) return 0;
        data_offset = (uint16_t)(data_offset + r);
    } else if (p->ethertype == ETH_P_IPV6) {
        r = parse_ipv6_hdr(c, data_offset, (uint16_t)(caplen - data_offset));
        if (c->err) return 0;
        data_offset = (uint16_t)(data_offset + r);
    } else if (p->ethertype == ETH_P_MPLS_UC || p->ethertype == ETH_P_MPLS_MC) {
        r = process_mpls(c, data_offset, (uint16_t)(caplen - data_offset));
        if (c->err) return 0;
        data_offset = (uint16_t)(data_offset + r);
        st->mpls_packets++;
    } else if (p->ethertype == ETH_P_PPP_SES) {
        r = process_pppoe(c, data_offset, (uint16_t)(caplen - data_offset));
        if (c->err) return 0;
        data_offset = (uint16_t)(data_offset + r);
        st->pppoe_packets++;
    } else {
        st->unknown_packets++;
        return 0;
    }
    l4_hdr_offset = data_offset;
    if (p->frag_off == 0) {
        if (p->ip_proto == 6) {
            r = parse_tcp_hdr(c, data_offset, (uint16_t)(caplen - data_offset));
            if (c->err) return 0;
            data_offset = (uint16_t)(data_offset + r);
            st->tcp_packets++;
        } else if (p->ip_proto == 17) {
            r = parse_udp_hdr(c, data_offset, (uint16_t)(caplen - data_offset));
            if (c->err) return 0;
            data_offset = (uint16_t)(data_offset + r);
            st->udp_packets++;
        }
    }
    { /* payload, parser.cpp:780-797 */
        uint16_t pkt_len = caplen, wire;
        if (l4_hdr_offset != l3_hdr_offset) {
            if (l4_hdr_offset + c->ip_payload_len < 64) pkt_len = (uint16_t)(l4_hdr_offset + c->ip_payload_len);
            wire = (uint16_t)(c->ip_payload_len - (data_offset - l4_hdr_offset));
        } else {
            wire = (uint16_t)(pkt_len - data_offset);
        }
        uint16_t plen = wire;
        if (plen + data_offset > pkt_len) plen = (uint16_t)(pkt_len - data_offset);
        p->payload_off = data_offset;
        p->payload_len = plen;
    }
    if (p->vlan_id) st->vlan_packets++;
    if (p->ethertype == ETH_P_IP) {
        st->ipv4_packets++;
        st->ipv4_bytes += caplen;
    } else if (p->ethertype == ETH_P_IPV6) {
        st->ipv6_packets++;
        st->ipv6_bytes += caplen;
    }
    st->parsed_packets++;
    if (c->ps) { /* vlan_stats[vlan_id].update(*pkt), parser.cpp:798 + VlanStats::update */
        ipxg_vlan_stats* v = &c->ps->vlan[p->vlan_id & 0xFFF];
        const uint16_t len = caplen; /* packet_len = caplen (parser.cpp:771) */
        if (p->ip_version == 4) {
            v->ipv4_packets++;
            v->ipv4_bytes += len;
        } else if (p->ip_version == 6) {
            v->ipv6_packets++;
            v->ipv6_bytes += len;
        }
        if (p->ip_proto == 6) v->tcp_packets++;
        else if (p->ip_proto == 17) v->udp_packets++;
        v->total_packets++;
        v->total_bytes += len;
        /* PacketSizeHistogram::update (parser-stats.hpp:42-80) */
        int b = len <= 64 ? 0 : len < 128 ? 1 : len < 256 ? 2 : len < 512 ? 3 : len < 1024 ? 4
              : len < 1518 ? 5 : len < 2048 ? 6 : len < 4096 ? 7 : len < 8192 ? 8 : 9;
        v->hist_packets[b]++;
        v->hist_bytes[b] += len;
    }
    return 1;
}

/* ---- flow key (cache.hpp:29-46, create_hash_key cache.cpp:525-574) ------------------ */
/* Builds the packed key and its inverse; returns the key length (0 = no key). */
static int build_keys(const ipxg_parsed_pkt* p, uint8_t* key, uint8_t* inv)
{
    uint16_t vlan = (uint16_t)p->vlan_id;
    if (p->ip_version == 4) {
        key[0] = p->src_port & 0xFF;
        key[1] = p->src_port >> 8;
        key[2] = p->dst_port & 0xFF;
        key[3] = p->dst_port >> 8;
        key[4] = p->ip_proto;
        key[5] = 4;
        memcpy(key + 6, p->src_ip, 4);
        memcpy(key + 10, p->dst_ip, 4);
        key[14] = vlan & 0xFF;
        key[15] = vlan >> 8;
        inv[0] = p->dst_port & 0xFF;
        inv[1] = p->dst_port >> 8;
        inv[2] = p->src_port & 0xFF;
        inv[3] = p->src_port >> 8;
        inv[4] = p->ip_proto;
        inv[5] = 4;
        memcpy(inv + 6, p->dst_ip, 4);
        memcpy(inv + 10, p->src_ip, 4);
        inv[14] = vlan & 0xFF;
        inv[15] = vlan >> 8;
        return 16;
    }
    if (p->ip_version == 6) {
        key[0] = p->src_port & 0xFF;
        key[1] = p->src_port >> 8;
        key[2] = p->dst_port & 0xFF;
        key[3] = p->dst_port >> 8;
        key[4] = p->ip_proto;
        key[5] = 6;
        memcpy(key + 6, p->src_ip, 16);
        memcpy(key + 22, p->dst_ip, 16);
        key[38] = vlan & 0xFF;
        key[39] = vlan >> 8;
        inv[0] = p->dst_port & 0xFF;
        inv[1] = p->dst_port >> 8;
        inv[2] = p->src_port & 0xFF;
        inv[3] = p->src_port >> 8;
        inv[4] = p->ip_proto;
        inv[5] = 6;
        memcpy(inv + 6, p->dst_ip, 16);
        memcpy(inv + 22, p->src_ip, 16);
        inv[38] = vlan & 0xFF;
        inv[39] = vlan >> 8;
        return 40;
    }
    return 0;
}

int oracle_parse(const uint8_t* data, uint16_t caplen, uint16_t wirelen, uint32_t ts_sec,
                 uint32_t ts_usec, uint32_t datalink, ipxg_parsed_pkt* out, int* beyond_caplen)
{
    (void)wirelen;
    (void)ts_sec;
    (void)ts_usec;
    ipxg_stats st;
    memset(&st, 0, sizeof(st));
    memset(out, 0, sizeof(*out));
    pctx c = {data, caplen, 0, 0, out, 0, &st, NULL};
    int ok = parse_packet(&c, caplen, datalink);
    out->valid = (uint8_t)ok;
    if (ok) {
        uint8_t k[40], ki[40];
        int kl = build_keys(out, k, ki);
        if (kl) {
            out->hash_fwd = oracle_xxh64(k, (size_t)kl, 0);
            out->hash_inv = oracle_xxh64(ki, (size_t)kl, 0);
        }
    }
    if (beyond_caplen) *beyond_caplen = c.beyond;
    return ok;
}

/* ===================================================================================== */
/* Fragmentation cache -- fragmentationCache.cpp:46-100, fragmentationTable.cpp:37-61,  */
/* fragmentationKeyData.hpp:49-136, ringBuffer.hpp:212-227 (RING_SIZE 4)                 */
/* ===================================================================================== */
typedef struct {
    uint8_t key[40];
    uint16_t sport, dport;
    uint32_t sec, usec;
} frag_entry;

typedef struct {
    frag_entry e[4]; /* e[0] oldest .. e[n-1] newest */
    uint32_t n;
} frag_ring;

static void frag_key(const ipxg_parsed_pkt* p, uint8_t* k)
{
    memset(k, 0, 40);
    k[0] = p->ip_version; /* uint16_t ip_version, little-endian */
    k[1] = 0;
    memcpy(k + 2, p->src_ip, 16);
    memcpy(k + 18, p->dst_ip, 16);
    k[34] = (uint8_t)p->frag_id;
    k[35] = (uint8_t)(p->frag_id >> 8);
    k[36] = (uint8_t)(p->frag_id >> 16);
    k[37] = (uint8_t)(p->frag_id >> 24);
    k[38] = (uint8_t)p->vlan_id;
    k[39] = (uint8_t)(p->vlan_id >> 8);
}

/* ===================================================================================== */
/* NHTFlowCache -- cache.cpp                                                              */
/* ===================================================================================== */
typedef struct {
    uint64_t hash; /* m_hash, 0 = empty (cache.cpp:84-87) */
    ipxg_flow_record f;
} orec;

struct oracle_cache {
    uint32_t cache_size, line_size, line_mask, line_new_idx, timeout_idx;
    uint32_t active, inactive;
    int split, frag_enable;
    uint32_t frag_size, frag_timeout;
    orec* recs;
    uint32_t* tab; /* m_flow_table: slot -> record */
    frag_ring* frings;
    ipxg_flow_record* ex;
    size_t ex_head, ex_n, ex_cap;
    ipxg_stats st;
    uint64_t flows_in_cache;
    pstats* ps;
    ipxg_plugin plugins[8];
    int n_plugins;
};

void oracle_cache_add_plugin(oracle_cache* c, const ipxg_plugin* p)
{
    if (c->n_plugins < 8) c->plugins[c->n_plugins++] = *p;
}

/* plugins_* (cache.cpp:596-655 / storagePlugin.hpp:97-158): every plugin's hook, OR of the
 * returns */
static int hook_pre_create(oracle_cache* c, ipxg_packet_view* v)
{
    int r = 0;
    for (int k = 0; k < c->n_plugins; ++k)
        if (c->plugins[k].pre_create) r |= c->plugins[k].pre_create(c->plugins[k].ctx, v);
    return r;
}
static int hook_post_create(oracle_cache* c, ipxg_flow_record* f, const ipxg_packet_view* v)
{
    int r = 0;
    for (int k = 0; k < c->n_plugins; ++k)
        if (c->plugins[k].post_create) r |= c->plugins[k].post_create(c->plugins[k].ctx, f, v);
    return r;
}
static int hook_pre_update(oracle_cache* c, ipxg_flow_record* f, ipxg_packet_view* v)
{
    int r = 0;
    for (int k = 0; k < c->n_plugins; ++k)
        if (c->plugins[k].pre_update) r |= c->plugins[k].pre_update(c->plugins[k].ctx, f, v);
    return r;
}
static int hook_post_update(oracle_cache* c, ipxg_flow_record* f, const ipxg_packet_view* v)
{
    int r = 0;
    for (int k = 0; k < c->n_plugins; ++k)
        if (c->plugins[k].post_update) r |= c->plugins[k].post_update(c->plugins[k].ctx, f, v);
    return r;
}
static void hook_pre_export(oracle_cache* c, ipxg_flow_record* f)
{
    for (int k = 0; k < c->n_plugins; ++k)
        if (c->plugins[k].pre_export) c->plugins[k].pre_export(c->plugins[k].ctx, f);
}
static void ext_clear(ipxg_flow_record* f) { memset(f->reserved + 8, 0, 8); } /* remove_extensions */

oracle_cache* oracle_cache_new(uint32_t cache_exp, uint32_t line_exp, uint32_t active_s,
                               uint32_t inactive_s, int split_biflow, int frag_enable,
                               uint32_t frag_size, uint32_t frag_timeout_s)
{
    oracle_cache* c = (oracle_cache*)calloc(1, sizeof(*c));
    if (!c) return NULL;
    /* NHTFlowCache::init cache.cpp:191-198 */
    c->cache_size = 1u << cache_exp;
    c->line_size = 1u << line_exp;
    c->line_mask = (c->cache_size - 1) & ~(c->line_size - 1);
    c->line_new_idx = c->line_size / 2;
    c->active = active_s;
    c->inactive = inactive_s;
    c->split = split_biflow;
    c->frag_enable = frag_enable;
    c->frag_size = frag_size ? frag_size : 10007;
    c->frag_timeout = frag_timeout_s;
    c->recs = (orec*)calloc(c->cache_size, sizeof(orec));
    c->ps = (pstats*)calloc(1, sizeof(pstats));
    c->tab = (uint32_t*)malloc(sizeof(uint32_t) * c->cache_size);
    c->frings = (frag_ring*)calloc(c->frag_size, sizeof(frag_ring));
    c->ex_cap = 1024;
    c->ex = (ipxg_flow_record*)malloc(sizeof(ipxg_flow_record) * c->ex_cap);
    if (!c->recs || !c->tab || !c->frings || !c->ex || !c->ps) {
        oracle_cache_free(c);
        return NULL;
    }
    for (uint32_t i = 0; i < c->cache_size; ++i) c->tab[i] = i;
    return c;
}

void oracle_cache_free(oracle_cache* c)
{
    if (!c) return;
    free(c->recs);
    free(c->tab);
    free(c->frings);
    free(c->ex);
    free(c->ps);
    free(c);
}

/* FlowRecord::erase cache.cpp:52-71 (MACs are left in place, as the reference does) */
static void rec_erase(orec* r)
{
    r->hash = 0;
    uint8_t sm[6], dm[6];
    memcpy(sm, r->f.src_mac, 6);
    memcpy(dm, r->f.dst_mac, 6);
    uint8_t reason = r->f.end_reason;
    memset(&r->f, 0, sizeof(r->f));
    memcpy(r->f.src_mac, sm, 6);
    memcpy(r->f.dst_mac, dm, 6);
    r->f.end_reason = reason;
}

/* FlowRecord::create cache.cpp:94-132 */
static void rec_create(orec* r, const ipxg_parsed_pkt* p, uint32_t sec, uint32_t usec, uint64_t hash)
{
    ipxg_flow_record* f = &r->f;
    f->src_packets = 1;
    r->hash = hash;
    f->time_first_sec = f->time_last_sec = sec;
    f->time_first_usec = f->time_last_usec = usec;
    f->flow_hash = hash;
    memcpy(f->src_mac, p->src_mac, 6);
    memcpy(f->dst_mac, p->dst_mac, 6);
    f->vlan_id = (uint16_t)p->vlan_id;
    if (p->ip_version == 4) {
        f->ip_version = 4;
        f->ip_proto = p->ip_proto;
        memcpy(f->src_ip, p->src_ip, 4);
        memcpy(f->dst_ip, p->dst_ip, 4);
        f->src_bytes = p->ip_len;
    } else if (p->ip_version == 6) {
        f->ip_version = 6;
        f->ip_proto = p->ip_proto;
        memcpy(f->src_ip, p->src_ip, 16);
        memcpy(f->dst_ip, p->dst_ip, 16);
        f->src_bytes = p->ip_len;
    }
    if (p->ip_proto == 6) {
        f->src_port = p->src_port;
        f->dst_port = p->dst_port;
        f->src_tcp_flags = p->tcp_flags;
    } else if (p->ip_proto == 17 || p->ip_proto == 1 || p->ip_proto == 58) {
        f->src_port = p->src_port;
        f->dst_port = p->dst_port;
    }
}

/* FlowRecord::update cache.cpp:134-152 */
static void rec_update(orec* r, const ipxg_parsed_pkt* p, uint32_t sec, uint32_t usec, int src)
{
    ipxg_flow_record* f = &r->f;
    f->time_last_sec = sec;
    f->time_last_usec = usec;
    if (src) {
        f->src_packets++;
        f->src_bytes += p->ip_len;
        if (p->ip_proto == 6) f->src_tcp_flags |= p->tcp_flags;
    } else {
        f->dst_packets++;
        f->dst_bytes += p->ip_len;
        if (p->ip_proto == 6) f->dst_tcp_flags |= p->tcp_flags;
    }
}

/* export_flow cache.cpp:262-274: hand the record to the export queue, empty the slot */
static void export_flow(oracle_cache* c, uint32_t index, uint8_t reason)
{
    orec* r = &c->recs[c->tab[index]];
    r->f.end_reason = reason;
    switch (reason) {
    case IPXG_FLOW_END_INACTIVE: c->st.end_inactive++; break;
    case IPXG_FLOW_END_ACTIVE: c->st.end_active++; break;
    case IPXG_FLOW_END_EOF: c->st.end_eof++; break;
    case IPXG_FLOW_END_FORCED: c->st.end_forced++; break;
    case IPXG_FLOW_END_NO_RES: c->st.end_no_res++; break;
    }
    c->st.total_exported++;
    { /* update_flow_record_stats cache.cpp:601-616 (0 packets: the final else) */
        const uint64_t n = (uint64_t)r->f.src_packets + r->f.dst_packets;
        uint64_t* b = n == 1 ? &c->st.flows_1_packet : (n >= 2 && n <= 5) ? &c->st.flows_2_5_packets
                    : (n >= 6 && n <= 10) ? &c->st.flows_6_10_packets : (n >= 11 && n <= 20) ? &c->st.flows_11_20_packets
                    : (n >= 21 && n <= 50) ? &c->st.flows_21_50_packets : &c->st.flows_51_plus_packets;
        (*b)++;
    }
    c->flows_in_cache--;
    if (c->ex_head + c->ex_n == c->ex_cap) {
        if (c->ex_head > 0) {
            memmove(c->ex, c->ex + c->ex_head, c->ex_n * sizeof(*c->ex));
            c->ex_head = 0;
        } else {
            c->ex_cap *= 2;
            c->ex = (ipxg_flow_record*)realloc(c->ex, c->ex_cap * sizeof(*c->ex));
        }
    }
    c->ex[c->ex_head + c->ex_n++] = r->f;
    rec_erase(r);
}

/* get_export_reason cache.cpp:498-506 */
static uint8_t export_reason(const ipxg_flow_record* f)
{
    return ((f->src_tcp_flags | f->dst_tcp_flags) & (0x01 | 0x04)) ? IPXG_FLOW_END_EOF
                                                                   : IPXG_FLOW_END_INACTIVE;
}

/* export_expired cache.cpp:508-523 */
void oracle_cache_export_expired(oracle_cache* c, int64_t ts)
{
    for (uint32_t i = c->timeout_idx; i < c->timeout_idx + c->line_new_idx; ++i) {
        orec* r = &c->recs[c->tab[i]];
        if (r->hash != 0 && ts - (int64_t)r->f.time_last_sec >= (int64_t)c->inactive) {
            r->f.end_reason = export_reason(&r->f);
            hook_pre_export(c, &r->f);
            export_flow(c, i, r->f.end_reason);
        }
    }
    c->timeout_idx = (c->timeout_idx + c->line_new_idx) & (c->cache_size - 1);
}

/* flush cache.cpp:290-320.  FLOW_FLUSH_WITH_REINSERT: the record goes to the export ring as
 * it is (FORCED; ipx_ring_push only -- no export statistics), and the slot continues with a
 * copy of it: extensions removed, reuse() (time_first = time_last, counters zero), update()
 * with the packet, then post_create (whose flush recurses).  FLOW_FLUSH: export_flow, FORCED. */
static void flush(oracle_cache* c, uint32_t fi, int ret, ipxg_packet_view* v, const ipxg_parsed_pkt* p, uint32_t sec,
                  uint32_t usec, int source_flow)
{
    orec* r = &c->recs[c->tab[fi]];
    if (ret == IPXG_FLOW_FLUSH_WITH_REINSERT) {
        r->f.end_reason = IPXG_FLOW_END_FORCED;
        if (c->ex_head + c->ex_n == c->ex_cap) {
            if (c->ex_head > 0) {
                memmove(c->ex, c->ex + c->ex_head, c->ex_n * sizeof(*c->ex));
                c->ex_head = 0;
            } else {
                c->ex_cap *= 2;
                c->ex = (ipxg_flow_record*)realloc(c->ex, c->ex_cap * sizeof(*c->ex));
            }
        }
        c->ex[c->ex_head + c->ex_n++] = r->f;
        ext_clear(&r->f);
        r->f.time_first_sec = r->f.time_last_sec; /* FlowRecord::reuse cache.cpp:73-83 */
        r->f.time_first_usec = r->f.time_last_usec;
        r->f.src_packets = r->f.dst_packets = 0;
        r->f.src_bytes = r->f.dst_bytes = 0;
        r->f.src_tcp_flags = r->f.dst_tcp_flags = 0;
        rec_update(r, p, sec, usec, source_flow);
        ret = hook_post_create(c, &r->f, v);
        if (ret & IPXG_FLOW_FLUSH) flush(c, fi, ret, v, p, sec, usec, source_flow);
    } else {
        export_flow(c, fi, IPXG_FLOW_END_FORCED);
    }
}

/* put_pkt_recursive cache.cpp:330-491, with the process-plugin hooks at their call sites */
static void put_pkt_recursive(oracle_cache* c, const ipxg_parsed_pkt* p, uint32_t sec, uint32_t usec,
                              ipxg_packet_view* v)
{
    if (c->n_plugins) hook_pre_create(c, v); /* its return is not used (:332) */
    uint8_t key[40], inv[40];
    int keylen = build_keys(p, key, inv);
    if (!keylen) return;
    uint64_t hashval = oracle_xxh64(key, (size_t)keylen, 0);
    int found = 0, source_flow = 1;
    uint32_t line_index = (uint32_t)(hashval & c->line_mask);
    uint32_t next_line = line_index + c->line_size;
    uint32_t fi;
    for (fi = line_index; fi < next_line; ++fi)
        if (c->recs[c->tab[fi]].hash == hashval) {
            found = 1;
            break;
        }
    if (!found && !c->split) {
        uint64_t hinv = oracle_xxh64(inv, (size_t)keylen, 0);
        uint32_t li = (uint32_t)(hinv & c->line_mask);
        for (fi = li; fi < li + c->line_size; ++fi)
            if (c->recs[c->tab[fi]].hash == hinv) {
                found = 1;
                source_flow = 0;
                hashval = hinv;
                line_index = li;
                break;
            }
    }
    if (found) { /* move to front, :375-391 */
        uint32_t flow = c->tab[fi];
        for (uint32_t j = fi; j > line_index; --j) c->tab[j] = c->tab[j - 1];
        c->tab[line_index] = flow;
        fi = line_index;
    } else {
        for (fi = line_index; fi < next_line; ++fi)
            if (c->recs[c->tab[fi]].hash == 0) {
                found = 1;
                break;
            }
        if (!found) { /* line full: evict the last slot, insert at the middle, :400-419 */
            fi = next_line - 1;
            hook_pre_export(c, &c->recs[c->tab[fi]].f);
            export_flow(c, fi, IPXG_FLOW_END_NO_RES);
            uint32_t new_idx = line_index + c->line_new_idx;
            uint32_t flow = c->tab[fi];
            for (uint32_t j = fi; j > new_idx; --j) c->tab[j] = c->tab[j - 1];
            fi = new_idx;
            c->tab[new_idx] = flow;
        }
    }
    if (v) v->source_pkt = (uint8_t)source_flow; /* :428 */
    orec* r = &c->recs[c->tab[fi]];
    uint8_t flw_flags = source_flow ? r->f.src_tcp_flags : r->f.dst_tcp_flags;
    if ((p->tcp_flags & 0x02) && (flw_flags & (0x01 | 0x04))) { /* :431-438 */
        export_flow(c, fi, IPXG_FLOW_END_EOF);
        put_pkt_recursive(c, p, sec, usec, v);
        return;
    }
    if (r->hash == 0) {
        c->flows_in_cache++;
        rec_create(r, p, sec, usec, hashval);
        if (c->n_plugins && (hook_post_create(c, &r->f, v) & IPXG_FLOW_FLUSH)) /* :443-449 */
            export_flow(c, fi, r->f.end_reason);  /* end_reason as the record holds it */
    } else {
        if ((int64_t)sec - (int64_t)r->f.time_last_sec >= (int64_t)c->inactive) { /* :453 */
            r->f.end_reason = export_reason(&r->f);
            hook_pre_export(c, &r->f);
            export_flow(c, fi, r->f.end_reason);
            put_pkt_recursive(c, p, sec, usec, v);
            return;
        }
        if ((int64_t)sec - (int64_t)r->f.time_first_sec >= (int64_t)c->active) { /* :464 */
            r->f.end_reason = IPXG_FLOW_END_ACTIVE;
            hook_pre_export(c, &r->f);
            export_flow(c, fi, IPXG_FLOW_END_ACTIVE);
            put_pkt_recursive(c, p, sec, usec, v);
            return;
        }
        if (c->n_plugins) {
            int ret = hook_pre_update(c, &r->f, v); /* :474-486 */
            if (ret & IPXG_FLOW_FLUSH) {
                flush(c, fi, ret, v, p, sec, usec, source_flow);
                return;
            }
            rec_update(r, p, sec, usec, source_flow);
            ret = hook_post_update(c, &r->f, v);
            if (ret & IPXG_FLOW_FLUSH) {
                flush(c, fi, ret, v, p, sec, usec, source_flow);
                return;
            }
        } else {
            rec_update(r, p, sec, usec, source_flow);
        }
    }
    oracle_cache_export_expired(c, (int64_t)sec); /* :489 */
}

/* FragmentationCache::process_packet fragmentationCache.cpp:46-100 */
static void frag_process(oracle_cache* c, ipxg_parsed_pkt* p, uint32_t sec, uint32_t usec)
{
    if (!(p->frag_off || p->more_fragments)) return;
    c->st.fragmented_packets++;
    uint8_t k[40];
    frag_key(p, k);
    frag_ring* ring = &c->frings[oracle_xxh64(k, 40, 0) % c->frag_size];
    if (!p->frag_off && p->more_fragments) { /* first fragment: insert (ring push_back) */
        if (ring->n == 4) {
            memmove(&ring->e[0], &ring->e[1], 3 * sizeof(frag_entry));
            ring->n = 3;
        }
        frag_entry* e = &ring->e[ring->n++];
        memcpy(e->key, k, 40);
        e->sport = p->src_port;
        e->dport = p->dst_port;
        e->sec = sec;
        e->usec = usec;
        return;
    }
    for (int i = (int)ring->n - 1; i >= 0; --i) { /* find, newest first */
        frag_entry* e = &ring->e[i];
        if (memcmp(e->key, k, 40) != 0) continue;
        /* timeout check: packet.ts > data.timestamp + timeout (timevalUtils.hpp) */
        uint64_t lim_sec = (uint64_t)e->sec + c->frag_timeout;
        uint64_t lim_usec = e->usec;
        if (lim_usec >= 1000000) {
            lim_sec++;
            lim_usec -= 1000000;
        }
        int later = (sec == lim_sec) ? (usec > lim_usec) : (sec > lim_sec);
        if (!later) {
            p->src_port = e->sport;
            p->dst_port = e->dport;
            c->st.fragments_filled++;
        }
        return;
    }
}

void oracle_cache_run(oracle_cache* c, const uint8_t* arena, const ipxg_pkt_desc* desc, size_t n,
                      uint32_t datalink)
{
    for (size_t i = 0; i < n; ++i) {
        const ipxg_pkt_desc* d = &desc[i];
        ipxg_parsed_pkt p;
        memset(&p, 0, sizeof(p));
        pctx pc = {arena + d->offset, d->caplen, 0, 0, &p, 0, &c->st, c->ps};
        if (!parse_packet(&pc, d->caplen, datalink)) continue;
        if (c->frag_enable) frag_process(c, &p, d->ts_sec, d->ts_usec);
        if (p.ip_version != 4 && p.ip_version != 6) c->st.keyless_packets++;
        ipxg_packet_view v = {&p, arena + d->offset, d->caplen, d->wirelen, d->ts_sec, d->ts_usec, (uint32_t)i, 0, {0}};
        put_pkt_recursive(c, &p, d->ts_sec, d->ts_usec, &v);
    }
}

/* finish cache.cpp:276-288 */
void oracle_cache_finish(oracle_cache* c)
{
    for (uint32_t i = 0; i < c->cache_size; ++i)
        if (c->recs[c->tab[i]].hash != 0) {
            hook_pre_export(c, &c->recs[c->tab[i]].f);
            export_flow(c, i, IPXG_FLOW_END_FORCED);
        }
}

size_t oracle_cache_pending(const oracle_cache* c) { return c->ex_n; }

size_t oracle_cache_take(oracle_cache* c, ipxg_flow_record* out, size_t cap)
{
    size_t k = c->ex_n < cap ? c->ex_n : cap;
    memcpy(out, c->ex + c->ex_head, k * sizeof(*out));
    c->ex_head += k;
    c->ex_n -= k;
    if (c->ex_n == 0) c->ex_head = 0;
    return k;
}

void oracle_cache_parser_stats(const oracle_cache* c, uint64_t* tcp_ports, uint64_t* udp_ports,
                               ipxg_vlan_stats* vlans)
{
    if (tcp_ports) memcpy(tcp_ports, c->ps->tcp, sizeof(c->ps->tcp));
    if (udp_ports) memcpy(udp_ports, c->ps->udp, sizeof(c->ps->udp));
    if (vlans) memcpy(vlans, c->ps->vlan, sizeof(c->ps->vlan));
}

void oracle_cache_stats(const oracle_cache* c, ipxg_stats* out)
{
    *out = c->st;
    out->flows_in_cache = c->flows_in_cache;
    out->table_capacity = c->cache_size;
}

/* ===================================================================================== */
/* IPFIX basic templates -- src/plugins/output/ipfix/src/ipfix.cpp,                       */
/* include/ipfixprobe/ipfix-elements.hpp                                                  */
/* ===================================================================================== */
/* One template element: enterprise number, element id, length (ipfix-elements.hpp FIELD
 * macro order) and which Flow member it reads. */
enum ipfix_src {
    S_END_REASON, S_BYTES, S_BYTES_REV, S_PACKETS, S_PACKETS_REV, S_START, S_END, S_L3, S_L4,
    S_FLAGS, S_FLAGS_REV, S_SPORT, S_DPORT, S_DIR, S_SRC4, S_DST4, S_SRC6, S_DST6, S_SMAC, S_DMAC
};
typedef struct {
    uint32_t en, id;
    int len;
    enum ipfix_src src;
} ipfix_elem;

/* BASIC_TMPLT_V4 / _V6 (ipfix-elements.hpp:328-366) with the element definitions of
 * ipfix-elements.hpp:71-119 (FLOW_START/END are the USEC variants, IPXP_TS_MSEC unset). */
static const ipfix_elem basic_v4[] = {
    {0, 136, 1, S_END_REASON}, {0, 1, 8, S_BYTES},       {29305, 1, 8, S_BYTES_REV},
    {0, 2, 8, S_PACKETS},      {29305, 2, 8, S_PACKETS_REV}, {0, 154, 8, S_START},
    {0, 155, 8, S_END},        {0, 60, 1, S_L3},         {0, 4, 1, S_L4},
    {0, 6, 1, S_FLAGS},        {29305, 6, 1, S_FLAGS_REV}, {0, 7, 2, S_SPORT},
    {0, 11, 2, S_DPORT},       {0, 10, 4, S_DIR},        {0, 8, 4, S_SRC4},
    {0, 12, 4, S_DST4},        {0, 56, 6, S_SMAC},       {0, 80, 6, S_DMAC}};
static const ipfix_elem basic_v6[] = {
    {0, 136, 1, S_END_REASON}, {0, 1, 8, S_BYTES},       {29305, 1, 8, S_BYTES_REV},
    {0, 2, 8, S_PACKETS},      {29305, 2, 8, S_PACKETS_REV}, {0, 154, 8, S_START},
    {0, 155, 8, S_END},        {0, 60, 1, S_L3},         {0, 4, 1, S_L4},
    {0, 6, 1, S_FLAGS},        {29305, 6, 1, S_FLAGS_REV}, {0, 7, 2, S_SPORT},
    {0, 11, 2, S_DPORT},       {0, 10, 4, S_DIR},        {0, 27, 16, S_SRC6},
    {0, 28, 16, S_DST6},       {0, 56, 6, S_SMAC},       {0, 80, 6, S_DMAC}};

/* MK_NTP_TS (ipfix-elements.hpp:50-60): (tv_sec + EPOCH_DIFF) << 32 | usec * 2^32 / 1e6 */
static uint64_t ntp_ts(uint32_t sec, uint32_t usec)
{
    return (((uint64_t)sec + 2208988800ULL) << 32) | (uint64_t)(uint32_t)(((uint64_t)usec << 32) / 1000000);
}

/* the element's source value in host byte order (integers) or its bytes (addresses, MACs),
 * as the FIELD macro's SRC pointer would read it */
static void ipfix_source(const ipxg_flow_record* r, uint32_t dir, enum ipfix_src s, uint64_t* v,
                         const uint8_t** bytes)
{
    *bytes = NULL;
    switch (s) {
    case S_END_REASON: *v = r->end_reason; break;
    case S_BYTES: *v = r->src_bytes; break;
    case S_BYTES_REV: *v = r->dst_bytes; break;
    case S_PACKETS: *v = (uint64_t)r->src_packets; break;  /* temp = (uint64_t) flow.src_packets */
    case S_PACKETS_REV: *v = (uint64_t)r->dst_packets; break;
    case S_START: *v = ntp_ts(r->time_first_sec, r->time_first_usec); break;
    case S_END: *v = ntp_ts(r->time_last_sec, r->time_last_usec); break;
    case S_L3: *v = r->ip_version; break;
    case S_L4: *v = r->ip_proto; break;
    case S_FLAGS: *v = r->src_tcp_flags; break;
    case S_FLAGS_REV: *v = r->dst_tcp_flags; break;
    case S_SPORT: *v = r->src_port; break;
    case S_DPORT: *v = r->dst_port; break;
    case S_DIR: *v = dir; break;                               /* &this->dir_bit_field */
    case S_SRC4: case S_SRC6: *bytes = r->src_ip; break;        /* network order in memory */
    case S_DST4: case S_DST6: *bytes = r->dst_ip; break;
    case S_SMAC: *bytes = r->src_mac; break;
    case S_DMAC: *bytes = r->dst_mac; break;
    }
}

/* IPFIX_FILL_FIELD (ipfix.cpp:77-96): len 1 copy; len 2 htons; the IPv4 addresses (en 0,
 * ids 8/12) copied as stored; other len 4 htonl; len 8 byte swap; anything else memcpy. */
static uint8_t* ipfix_fill_field(uint8_t* t, const ipfix_elem* e, const ipxg_flow_record* r, uint32_t dir)
{
    uint64_t v = 0;
    const uint8_t* b;
    ipfix_source(r, dir, e->src, &v, &b);
    if (e->len == 1) {
        t[0] = (uint8_t)v;
    } else if (e->len == 2) {
        t[0] = (uint8_t)(v >> 8);
        t[1] = (uint8_t)v;
    } else if (e->en == 0 && (e->id == 8 || e->id == 12)) {
        memcpy(t, b, 4);
    } else if (e->len == 4) {
        for (int k = 0; k < 4; ++k) t[k] = (uint8_t)(v >> (24 - 8 * k));
    } else if (e->len == 8) {
        for (int k = 0; k < 8; ++k) t[k] = (uint8_t)(v >> (56 - 8 * k));
    } else {
        memcpy(t, b, (size_t)e->len);
    }
    return t + e->len;
}

/* fill_basic_flow: ip_version == IP::v4 selects BASIC_TMPLT_V4, anything else _V6
 * (ipfix.cpp:1478-1509; get_template :289 likewise) */
void oracle_ipfix_basic(const ipxg_flow_record* recs, size_t n, uint32_t dir_bit_field, uint8_t* out,
                        uint64_t* offsets)
{
    uint8_t* p = out;
    offsets[0] = 0;
    for (size_t i = 0; i < n; ++i) {
        const ipxg_flow_record* r = &recs[i];
        const ipfix_elem* t = r->ip_version == 4 ? basic_v4 : basic_v6;
        const size_t ne = r->ip_version == 4 ? sizeof(basic_v4) / sizeof(basic_v4[0])
                                             : sizeof(basic_v6) / sizeof(basic_v6[0]);
        for (size_t k = 0; k < ne; ++k) p = ipfix_fill_field(p, &t[k], r, dir_bit_field);
        offsets[i + 1] = (uint64_t)(p - out);
    }
}

/* ===================================================================================== */
/* IPFIX messages -- IPFIXExporter (src/plugins/output/ipfix/src/ipfix.cpp) over the       */
/* basic templates, TCP transport (templates sent once, no refresh: ipfix.hpp:52,66)      */
/* ===================================================================================== */
typedef struct {
    uint16_t id;
    uint8_t rec[128]; /* templateRecord */
    uint16_t rec_size;
    uint8_t buf[65536]; /* template buffer: data set header + records */
    uint32_t buf_size, count;
    int exported;
} otmpl;

typedef struct {
    ipxg_ipfix_exporter* x;
    otmpl t[2];  /* the template list: [0] = IPv6 (259, created second, list head), [1] = IPv4 */
    int have;    /* templates created (get_template on the first flow) */
    uint8_t* out;
    size_t cap, len, msgs;
    int overflow;
} oexp;

static void be16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void be32(uint8_t* p, uint32_t v)
{
    for (int k = 0; k < 4; ++k) p[k] = (uint8_t)(v >> (24 - 8 * k));
}

/* create_template ipfix.cpp:537-656 (fields from the template-file table = ipfix-elements.hpp) */
static void otmpl_create(otmpl* t, uint16_t id, const ipfix_elem* el, size_t ne, uint32_t mtu)
{
    memset(t, 0, sizeof(*t));
    t->id = id;
    be16(t->rec, id);
    uint16_t sz = 4;
    for (size_t k = 0; k < ne; ++k) {
        be16(t->rec + sz, el[k].id | (el[k].en ? 0x8000 : 0));
        be16(t->rec + sz + 2, (uint32_t)el[k].len);
        sz += 4;
        if (el[k].en) {
            be32(t->rec + sz, el[k].en);
            sz += 4;
        }
    }
    be16(t->rec + 2, (uint32_t)ne);
    t->rec_size = sz;
    be16(t->buf, id); /* init_template_buffer :414-417 */
    t->buf_size = 4;
    (void)mtu;
}

static void oexp_emit(oexp* e, const uint8_t* msg, size_t n)
{
    if (e->len + n > e->cap) {
        e->overflow = 1;
    } else {
        memcpy(e->out + e->len, msg, n);
    }
    e->len += n;
    e->msgs++;
}

/* fill_ipfix_header :475-486 */
static void ohdr(oexp* e, uint8_t* p, uint32_t size)
{
    be16(p, 10);
    be16(p + 2, size);
    be32(p + 4, e->x->export_time);
    be32(p + 8, e->x->sequence);
    be32(p + 12, e->x->odid);
}

/* flush :846-853 = send_templates (create_template_packet :671-728) + send_data
 * (create_data_packet :739-795 until it returns 0); send_packet adds packet->flows to the
 * sequence number (:945) */
static void oexp_flush(oexp* e)
{
    static uint8_t msg[65536];
    if (!e->have) return;
    uint32_t total = 0;
    for (int k = 0; k < 2; ++k)
        if (!e->t[k].exported) total += e->t[k].rec_size;
    if (total) {
        total += 16 + 4;
        ohdr(e, msg, total);
        be16(msg + 16, 2); /* TEMPLATE_SET_ID */
        be16(msg + 18, total - 16);
        uint32_t p = 20;
        for (int k = 0; k < 2; ++k)
            if (!e->t[k].exported) {
                memcpy(msg + p, e->t[k].rec, e->t[k].rec_size);
                p += e->t[k].rec_size;
                e->t[k].exported = 1;
            }
        oexp_emit(e, msg, total);
        e->x->templates_sent = 1;
    }
    for (;;) {
        uint32_t size = 16, flows = 0;
        for (int k = 0; k < 2; ++k) {
            otmpl* t = &e->t[k];
            if (t->count > 0 && size + t->buf_size <= e->x->mtu) {
                memcpy(msg + size, t->buf, t->buf_size);
                be16(msg + size + 2, t->buf_size);
                size += t->buf_size;
                t->buf_size = 4;
                flows += t->count;
                t->count = 0;
            }
        }
        if (size == 16) break;
        ohdr(e, msg, size);
        oexp_emit(e, msg, size);
        e->x->sequence += flows;
    }
}

/* fill_template :350-382 / fill_basic_flow :1470-1516: -1 when the record passes the buffer
 * limit mtu - IPFIX_HEADER_SIZE */
static int oexp_fill(oexp* e, otmpl* t, const ipxg_flow_record* r)
{
    const uint32_t len = r->ip_version == 4 ? 81 : 105;
    if (t->buf_size + len > (uint32_t)e->x->mtu - 16) return -1;
    uint64_t off[2];
    oracle_ipfix_basic(r, 1, e->x->dir_bit_field, t->buf + t->buf_size, off);
    t->buf_size += len;
    t->count++;
    return 0;
}

size_t oracle_ipfix_export(ipxg_ipfix_exporter* x, const ipxg_flow_record* recs, size_t n, uint8_t* out, size_t cap,
                           size_t* msgs)
{
    static oexp e; /* test infrastructure: one exporter at a time */
    memset(&e, 0, sizeof(e));
    e.x = x;
    e.out = out;
    e.cap = cap;
    /* get_template :287-323 creates both basic templates on the first flow: v4 first (id 258),
     * then v6 (259), each pushed at the list head */
    if (n) {
        otmpl_create(&e.t[1], 258, basic_v4, sizeof(basic_v4) / sizeof(basic_v4[0]), x->mtu);
        otmpl_create(&e.t[0], 259, basic_v6, sizeof(basic_v6) / sizeof(basic_v6[0]), x->mtu);
        e.t[0].exported = e.t[1].exported = x->templates_sent;
        e.have = 1;
    }
    for (size_t i = 0; i < n; ++i) { /* export_flow :385-398 */
        otmpl* t = recs[i].ip_version == 6 ? &e.t[0] : &e.t[1];
        if (oexp_fill(&e, t, &recs[i]) != 0) {
            oexp_flush(&e);
            oexp_fill(&e, t, &recs[i]);
        }
    }
    oexp_flush(&e); /* the output worker's flush when its queue runs dry (workers.cpp:176-183) */
    if (msgs) *msgs = e.msgs;
    return e.overflow ? (size_t)-1 : e.len;
}
