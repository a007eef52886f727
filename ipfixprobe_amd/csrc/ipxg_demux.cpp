// ipxg_demux.cpp -- host-side symmetric demux of a packet batch into one batch per engine/GPU
// (the NIC's symmetric RSS into per-queue rings: dpdkDevice.cpp:230-262, one input pipeline and
// cache per queue: ipfixprobe.cpp:381-464).  The shard depends only on the unordered pair of
// the outermost IP addresses, so both directions of a biflow -- and non-first fragments, which
// carry no ports -- land on the same engine, and the engines never exchange flow state.
#include <cstring>

#include "../../include/ipxg.h"

namespace {

constexpr uint32_t HDR_MAX = 64;  // header bytes the walk may read

uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }

// splitmix64 finaliser over the address bytes (commutative combination below)
uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t addr_hash(const uint8_t* a, uint32_t len) {
    uint64_t w[2] = {0, 0};
    std::memcpy(w, a, len);
    return mix(w[0] ^ mix(w[1] + len));
}

// byte offset of the IP header and its version (4/6), or 0 when the walk finds none
uint32_t find_ip(const uint8_t* f, uint32_t cap, uint32_t dlt, uint32_t& ver) {
    ver = 0;
    cap = cap < HDR_MAX ? cap : HDR_MAX;
    uint32_t off = 0, et = 0;
    if (dlt == 0 || dlt == IPXG_DLT_EN10MB) {
        if (cap < 14) return 0;
        et = be16(f + 12);
        off = 14;
        for (int k = 0; k < 2 && (et == 0x8100 || et == 0x88A8); ++k) {
            if (off + 4 > cap) return 0;
            et = be16(f + off + 2);
            off += 4;
        }
    } else if (dlt == IPXG_DLT_LINUX_SLL) {
        if (cap < 16) return 0;
        et = be16(f + 14);
        off = 16;
    } else if (dlt == IPXG_DLT_LINUX_SLL2) {
        if (cap < 20) return 0;
        et = be16(f);
        off = 20;
    } else if (dlt == IPXG_DLT_RAW) {
        if (cap < 1) return 0;
        et = (f[0] >> 4) == 4 ? 0x0800 : ((f[0] >> 4) == 6 ? 0x86DD : 0);
    }
    if (et == 0x8864) {  // PPPoE session: 6 bytes + PPP protocol
        if (off + 8 > cap) return 0;
        const uint32_t pp = be16(f + off + 6);
        et = pp == 0x0021 ? 0x0800 : (pp == 0x0057 ? 0x86DD : 0);
        off += 8;
    } else if (et == 0x8847 || et == 0x8848) {  // MPLS: labels up to bottom of stack, then the IP nibble
        for (;;) {
            if (off + 4 > cap) return 0;
            const bool bos = f[off + 2] & 1;
            off += 4;
            if (bos) break;
        }
        if (off >= cap) return 0;
        et = (f[off] >> 4) == 4 ? 0x0800 : ((f[off] >> 4) == 6 ? 0x86DD : 0);
    }
    if (et == 0x0800 && off + 20 <= cap) ver = 4;
    else if (et == 0x86DD && off + 40 <= cap) ver = 6;
    return ver ? off : 0;
}

uint32_t shard_of_frame(const uint8_t* f, uint32_t cap, uint32_t dlt, uint32_t n_shards) {
    uint32_t ver;
    const uint32_t off = find_ip(f, cap, dlt, ver);
    if (!ver) return 0;
    const uint64_t h = ver == 4 ? addr_hash(f + off + 12, 4) + addr_hash(f + off + 16, 4)
                                : addr_hash(f + off + 8, 16) + addr_hash(f + off + 24, 16);
    return (uint32_t)(((unsigned __int128)mix(h) * n_shards) >> 64);
}

}  // namespace

int ipxg_demux(const ipxg_batch* in, uint32_t datalink, uint32_t n_shards, uint32_t* shard_of, uint32_t* counts) {
    if (!in || !shard_of || !counts || n_shards == 0 || (in->n && (!in->arena || !in->desc))) return IPXG_EINVAL;
    if (in->flags & IPXG_BATCH_DEVICE) return IPXG_EINVAL;  // a host ring's batch
    std::memset(counts, 0, n_shards * sizeof(uint32_t));
    const uint32_t sh = (in->flags & IPXG_BATCH_OFFSET16) ? 4u : 0u;
    for (uint32_t i = 0; i < in->n; ++i) {
        const ipxg_pkt_desc& d = in->desc[i];
        const uint64_t fo = (uint64_t)d.offset << sh;
        if (fo + d.caplen > in->arena_len) return IPXG_EINVAL;
        const uint32_t s = shard_of_frame(in->arena + fo, d.caplen, datalink, n_shards);
        shard_of[i] = s;
        counts[s]++;
    }
    return IPXG_OK;
}

uint64_t ipxg_demux_arena_bytes(const ipxg_batch* in, const uint32_t* shard_of, uint32_t shard) {
    if (!in || !shard_of) return 0;
    uint64_t b = 0;
    for (uint32_t i = 0; i < in->n; ++i)
        if (shard_of[i] == shard) b += ((uint64_t)in->desc[i].caplen + 15) & ~15ull;
    return b;
}

int ipxg_demux_split(const ipxg_batch* in, const uint32_t* shard_of, uint32_t shard, uint8_t* arena_out,
                     ipxg_pkt_desc* desc_out, uint32_t* n_out) {
    if (!in || !shard_of || !n_out || (in->n && (!arena_out || !desc_out))) return IPXG_EINVAL;
    uint64_t off = 0;
    uint32_t k = 0;
    // the shard's descriptors count offsets as the input's do (bytes, or 16-byte units)
    const uint32_t sh = (in->flags & IPXG_BATCH_OFFSET16) ? 4u : 0u;
    for (uint32_t i = 0; i < in->n; ++i) {
        if (shard_of[i] != shard) continue;
        ipxg_pkt_desc d = in->desc[i];
        if ((off >> sh) > 0xFFFFFFFFull) return IPXG_ETOOBIG;  // descriptor offsets are 32-bit
        std::memcpy(arena_out + off, in->arena + ((uint64_t)d.offset << sh), d.caplen);
        const uint32_t pad = ((d.caplen + 15u) & ~15u) - d.caplen;
        if (pad) std::memset(arena_out + off + d.caplen, 0, pad);
        d.offset = (uint32_t)(off >> sh);
        desc_out[k++] = d;
        off += ((uint64_t)d.caplen + 15) & ~15ull;
    }
    *n_out = k;
    return IPXG_OK;
}
