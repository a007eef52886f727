/* ipxg_stdplugins.c -- native stand-ins of the dns / http / tls / quic process plugins as
 * ipxg_plugin rules + hooks (include/ipxg_stdplugins.h): the decisions of each reference
 * plugin that end a flow or claim it, restated from its source (cited per function).  Not the
 * enrichment -- the real plugins run behind the adapter of INTEGRATION.md. */
#include "../../include/ipxg_stdplugins.h"

#include <stdlib.h>
#include <string.h>

#include <pthread.h>

#include <openssl/evp.h>
#include <openssl/sha.h>

enum { C_PRE_CREATE, C_POST_CREATE, C_PRE_UPDATE, C_POST_UPDATE, C_PRE_EXPORT, C_FLUSH, C_N };

/* A plugin instance's counters.  The walk threads' copies (copy_ctx, ProcessPlugin::copy) hang
 * off the instance they were copied from; ipxg_std_plugin_calls sums them, and a copy released
 * by the engine (free_ctx) folds its counts into it.  Copies are made and released by the
 * engine's calling thread, between walks. */
typedef struct std_ctx {
    uint64_t calls[C_N];
    struct std_ctx* root;   /* NULL on the instance ipxg_std_plugin made */
    struct std_ctx* next;   /* root: first copy; copy: next copy of the same root */
    struct std_ctx* prev;
    EVP_CIPHER_CTX* ecb;    /* QUIC: the instance's cipher contexts, made on first use and kept */
    EVP_CIPHER_CTX* gcm;    /* (walk threads each hold their own copy) */
} std_ctx;

static void std_ctx_release(std_ctx* c) {
    if (c->ecb) EVP_CIPHER_CTX_free(c->ecb);
    if (c->gcm) EVP_CIPHER_CTX_free(c->gcm);
    free(c);
}

static void* std_copy(void* ctx) {
    std_ctx* r = (std_ctx*)ctx;
    if (r->root) r = r->root;
    std_ctx* c = (std_ctx*)calloc(1, sizeof(std_ctx));
    if (!c) return NULL;
    c->root = r;
    c->next = r->next;
    c->prev = r;
    if (r->next) r->next->prev = c;
    r->next = c;
    return c;
}

static void std_free_copy(void* ctx) {
    std_ctx* c = (std_ctx*)ctx;
    if (!c || !c->root) return; /* the original belongs to ipxg_std_plugin_free */
    for (int k = 0; k < C_N; ++k) c->root->calls[k] += c->calls[k];
    c->prev->next = c->next;
    if (c->next) c->next->prev = c->prev;
    std_ctx_release(c);
}

static const uint8_t* payload(const ipxg_packet_view* v, uint32_t* n) {
    const ipxg_parsed_pkt* p = v->pkt;
    uint32_t off = p->payload_off, len = p->payload_len;
    if (off > v->caplen) off = v->caplen;
    if (off + len > v->caplen) len = v->caplen - off;
    *n = len;
    return v->data + off;
}

static int count(void* ctx, int idx, int ret) {
    std_ctx* c = (std_ctx*)ctx;
    c->calls[idx]++;
    if (ret) c->calls[C_FLUSH]++;
    return ret;
}

static int hook_pre_create(void* ctx, ipxg_packet_view* v) {
    (void)v;
    return count(ctx, C_PRE_CREATE, 0);
}
static void hook_pre_export(void* ctx, ipxg_flow_record* f) {
    (void)f;
    count(ctx, C_PRE_EXPORT, 0);
}

/* ---- DNS: parse_dns (dns.cpp:429-660), only whether it returns true ------------------------- */
#define MAX_LABEL_CNT 127

typedef struct {
    const uint8_t* d;
    uint32_t n;   /* bytes the parser may read (length check bound) */
    uint32_t avail;
} dns_buf;

static uint32_t db(const dns_buf* b, uint32_t i) { return i < b->avail ? b->d[i] : 0u; }
static uint32_t be16(const dns_buf* b, uint32_t i) { return (db(b, i) << 8) | db(b, i + 1); }

/* get_name_length (dns.cpp:148-169): -1 when it throws */
static int64_t name_length(const dns_buf* b, uint32_t i) {
    int64_t len = 0;
    for (;;) {
        if (i + 1 > b->n) return -1;
        const uint32_t c = db(b, i);
        if (!c) break;
        if ((c & 0xC0) == 0xC0) return len + 2;
        len += c + 1;
        i += c + 1;
    }
    return len + 1;
}

/* get_name (dns.cpp:175-206): 0 when it throws */
static int name_ok(const dns_buf* b, uint32_t i) {
    uint32_t cnt = 0;
    if (i > b->n) return 0;
    while (db(b, i)) {
        const uint32_t c = db(b, i);
        if ((c & 0xC0) == 0xC0) {
            i = ((c & 0x3F) << 8) | db(b, i + 1);
            if (cnt > MAX_LABEL_CNT || i > b->n) return 0;
            cnt++;
            continue;
        }
        if (cnt > MAX_LABEL_CNT || c > 63 || i + c + 2 > b->n) return 0;
        cnt++;
        i += c + 1;
    }
    return 1;
}

/* process_rdata's name walks (dns.cpp:250-320) for the first answer */
static int rdata_ok(const dns_buf* b, uint32_t i, uint32_t type) {
    if (type == 2 || type == 5 || type == 12 || type == 39) return name_ok(b, i);
    if (type == 6) {
        if (!name_ok(b, i)) return 0;
        const int64_t l = name_length(b, i);
        if (l < 0) return 0;
        i += (uint32_t)l;
        if (!name_ok(b, i)) return 0;
        return name_length(b, i) >= 0;
    }
    if (type == 15) return name_ok(b, i + 2);
    return 1;
}

static int dns_valid(const uint8_t* d, uint32_t len, int tcp) {
    dns_buf b = {d, len, len};
    if (tcp) {
        const uint32_t n = (len - 2) & 0xFFFFFFFFu;
        if (((uint32_t)db(&b, 0) << 8 | db(&b, 1)) != n) return 0;
        b.d = d + 2;
        b.n = n;
        b.avail = len >= 2 ? len - 2 : 0;
    }
    if (b.n < 12) return 0;
    const uint32_t qd = be16(&b, 4), an = be16(&b, 6), ns = be16(&b, 8), ar = be16(&b, 10);
    uint32_t i = 12;
    for (uint32_t q = 0; q < qd; ++q) {
        if (!name_ok(&b, i)) return 0;
        const int64_t l = name_length(&b, i);
        if (l < 0) return 0;
        i += (uint32_t)l;
        if (i + 4 > b.n) return 1;
        i += 4;
    }
    for (uint32_t k = 0; k < an; ++k) {
        const int64_t l = name_length(&b, i);
        if (l < 0) return 0;
        i += (uint32_t)l;
        if (i + 10 > b.n || i + 10 + be16(&b, i + 8) > b.n) return 1;
        const uint32_t type = be16(&b, i), rdl = be16(&b, i + 8);
        i += 10;
        if (k == 0 && !rdata_ok(&b, i, type)) return 0;
        i += rdl;
    }
    for (uint32_t k = 0; k < ns + ar; ++k) {
        const int64_t l = name_length(&b, i);
        if (l < 0) return 0;
        i += (uint32_t)l;
        if (i + 10 > b.n || i + 10 + be16(&b, i + 8) > b.n) return 1;
        i += 10 + be16(&b, i + 8);
    }
    return 1;
}

static int dns_port(const ipxg_packet_view* v) { return v->pkt->src_port == 53 || v->pkt->dst_port == 53; }

/* DNSPlugin::post_create / post_update (dns.cpp:97-127) */
static int dns_post_create(void* ctx, ipxg_flow_record* f, const ipxg_packet_view* v) {
    int r = 0;
    if (dns_port(v)) {
        uint32_t n;
        const uint8_t* d = payload(v, &n);
        if (dns_valid(d, n, v->pkt->ip_proto == 6)) {
            f->ext |= IPXG_STD_EXT_DNS;
            r = IPXG_FLOW_FLUSH;
        }
    }
    return count(ctx, C_POST_CREATE, r);
}
static int dns_post_update(void* ctx, ipxg_flow_record* f, const ipxg_packet_view* v) {
    int r = 0;
    if (dns_port(v)) {
        if (f->ext & IPXG_STD_EXT_DNS) {
            r = IPXG_FLOW_FLUSH;  /* parse into the existing extension, then flush */
        } else {
            uint32_t n;
            const uint8_t* d = payload(v, &n);
            if (dns_valid(d, n, v->pkt->ip_proto == 6)) {
                f->ext |= IPXG_STD_EXT_DNS;
                r = IPXG_FLOW_FLUSH;
            }
        }
    }
    return count(ctx, C_POST_UPDATE, r);
}
static int noop_pre_update(void* ctx, ipxg_flow_record* f, ipxg_packet_view* v) {
    (void)f;
    (void)v;
    return count(ctx, C_PRE_UPDATE, 0);
}
static int noop_post_update(void* ctx, ipxg_flow_record* f, const ipxg_packet_view* v) {
    (void)f;
    (void)v;
    return count(ctx, C_POST_UPDATE, 0);
}

/* ---- HTTP (http.cpp:100-140, parse_http_request :233-290, parse_http_response :400-445) ----- */
static const char* const METHODS[] = {"GET ", "POST", "PUT ", "HEAD", "DELE", "TRAC", "OPTI", "CONN", "PATC"};

static const uint8_t* find_sp(const uint8_t* d, uint32_t n, uint32_t from) {
    for (uint32_t k = from; k < n; ++k)
        if (d[k] == ' ') return d + k;
    return NULL;
}
static int request_line(const uint8_t* d, uint32_t n) {
    const uint8_t* a = find_sp(d, n, 0);
    if (!a) return 0;
    const uint8_t* b = find_sp(d, n, (uint32_t)(a - d) + 1);
    if (!b) return 0;
    const uint32_t o = (uint32_t)(b - d) + 1;
    return o + 4 <= n && memcmp(d + o, "HTTP", 4) == 0;
}
static int response_line(const uint8_t* d, uint32_t n) {
    const uint8_t* a = find_sp(d, n, 0);
    if (!a) return 0;
    const uint8_t* b = find_sp(d, n, (uint32_t)(a - d) + 1);
    if (!b) return 0;
    long code = 0;
    int digits = 0;
    for (const uint8_t* p = a + 1; p < b; ++p) {
        if (*p < '0' || *p > '9') return 0;
        code = code * 10 + (*p - '0');
        if (++digits > 9) return 0;
    }
    return digits > 0 && code > 0;
}
/* 1 request, 2 response, 0 neither */
static int http_kind(const uint8_t* d, uint32_t n) {
    if (n < 4) return 0;
    for (unsigned k = 0; k < sizeof(METHODS) / sizeof(METHODS[0]); ++k)
        if (memcmp(d, METHODS[k], 4) == 0) return 1;
    return memcmp(d, "HTTP", 4) == 0 ? 2 : 0;
}
static int http_post_create(void* ctx, ipxg_flow_record* f, const ipxg_packet_view* v) {
    uint32_t n;
    const uint8_t* d = payload(v, &n);
    const int k = http_kind(d, n);
    if (k == 1 && request_line(d, n)) f->ext |= IPXG_STD_EXT_HTTP | IPXG_STD_EXT_HTTP_REQ;
    else if (k == 2 && response_line(d, n)) f->ext |= IPXG_STD_EXT_HTTP | IPXG_STD_EXT_HTTP_RESP;
    return count(ctx, C_POST_CREATE, 0);
}
static int http_pre_update(void* ctx, ipxg_flow_record* f, ipxg_packet_view* v) {
    uint32_t n;
    const uint8_t* d = payload(v, &n);
    const int k = http_kind(d, n);
    int r = 0;
    if (k) {
        const uint64_t bit = k == 1 ? IPXG_STD_EXT_HTTP_REQ : IPXG_STD_EXT_HTTP_RESP;
        const int ok = k == 1 ? request_line(d, n) : response_line(d, n);
        if (!(f->ext & IPXG_STD_EXT_HTTP)) {
            if (ok) f->ext |= IPXG_STD_EXT_HTTP | bit;
        } else if (ok && (f->ext & bit)) {
            r = IPXG_FLOW_FLUSH_WITH_REINSERT;  /* the flow already holds one */
        } else if (ok) {
            f->ext |= bit;
        }
    }
    return count(ctx, C_PRE_UPDATE, r);
}

/* ---- TLS (tls.cpp:101-122, add_tls_record :410-425; TLSParser::parse tls_parser.cpp:72-100) ---
 * The extension is attached when TLSPlugin::parse_tls accepts a ClientHello (a ServerHello never
 * attaches one: parse_tls returns false after it, tls.cpp:392-401): the record header (type 22,
 * version 3.0-3.3, :102-124), the handshake (ClientHello / ServerHello, version 3.1-3.3,
 * :126-154), then every length check of the session id (:156-170), cipher suites (:172-203),
 * compression methods (:205-223) and the extensions section (has_valid_extension_length,
 * :413-427) -- a hello cut short by the capture (the configs[2] mix's 64-byte-class frames hold
 * 43 bytes of it) attaches nothing.  Bytes at or past the payload's end read as 0 (the reference
 * reads whatever follows; DESIGN.md section 2 rule 1).  Nothing ends a flow. */
static uint32_t tls_b(const uint8_t* d, uint32_t n, uint32_t i) { return i < n ? d[i] : 0u; }
static int tls_hello(const uint8_t* d, uint32_t n) {
    if (n < 5 || d[0] != 22 || d[1] != 3 || d[2] > 3) return 0;  /* parse_tls_header */
    if (5 + 6 > n) return 0;                                       /* parse_tls_handshake */
    const uint8_t t = d[5];
    if (t != 1 && t != 2) return 0;
    if (!(d[9] == 3 && d[10] >= 1 && d[10] <= 3)) return 0;
    const uint32_t sid_off = 5 + 6 + 32;                           /* parse_session_id */
    if (sid_off > n) return 0;
    const uint32_t sid_sec = 1 + tls_b(d, n, sid_off);
    if (sid_off + sid_sec > n) return 0;
    const uint32_t cs_off = sid_off + sid_sec;                     /* parse_cipher_suites */
    if (cs_off + 2 > n) return 0;
    uint32_t cs_sec = 2;
    if (t == 1) {
        const uint32_t cl = (tls_b(d, n, cs_off) << 8) | tls_b(d, n, cs_off + 1);
        if (cs_off + 2 + cl > n) return 0;
        cs_sec = 2 + cl;
    }
    const uint32_t cm_off = cs_off + cs_sec;                       /* parse_compression_methods */
    if (cm_off > n) return 0;
    uint32_t cm_sec = 1;
    if (t == 1) {
        const uint32_t cm = tls_b(d, n, cm_off);
        if (1 + cm > n) return 0;  /* (the reference compares with the whole length) */
        cm_sec = 1 + cm;
    }
    if (t != 1) return 0;                                          /* only a ClientHello attaches */
    const uint32_t ext_off = cm_off + cm_sec;                      /* has_valid_extension_length */
    if (ext_off > n) return 0;
    const uint32_t el = (tls_b(d, n, ext_off) << 8) | tls_b(d, n, ext_off + 1);
    return ext_off + el <= n;
}
static int tls_post_create(void* ctx, ipxg_flow_record* f, const ipxg_packet_view* v) {
    uint32_t n;
    const uint8_t* d = payload(v, &n);
    if (tls_hello(d, n)) f->ext |= IPXG_STD_EXT_TLS;
    return count(ctx, C_POST_CREATE, 0);
}
static int tls_pre_update(void* ctx, ipxg_flow_record* f, ipxg_packet_view* v) {
    if (!(f->ext & IPXG_STD_EXT_TLS)) {
        uint32_t n;
        const uint8_t* d = payload(v, &n);
        if (tls_hello(d, n)) f->ext |= IPXG_STD_EXT_TLS;
    }
    return count(ctx, C_PRE_UPDATE, 0);
}

/* ---- QUIC (quic.cpp:350-549, QUICPlugin::add_quic :515-540; QUICParser quic_parser.cpp) -------
 * The extension is attached when process_quic detects QUIC (QUIC_DETECTED): the datagram's first
 * packet passes quic_long_header_packet (:1105-1117: UDP, long-header bit, >= 8 bytes, a version
 * quic_draft_version knows, :313-393) and quic_parse_headers (:1287-1377), which fails unless a TLS
 * handshake header was parsed by the time the first packet is done (quic_set_server_port,
 * :1379-1407) -- i.e. the first packet is a client Initial whose protection comes off with the
 * initial secrets of its version's salt and its DCID (RFC 9001 5.2-5.4: HKDF, AES-128-ECB header
 * protection, AES-128-GCM), whose CRYPTO frames reassemble (:1009-1043) and start with a TLS
 * ClientHello / ServerHello handshake header of version 3.1-3.3 (TLSParser::parse_tls_handshake).
 * The version-negotiation FLOW_FLUSH of quic.cpp:400-403 is never reached (its datagram carries no
 * handshake: quic_set_server_port fails first), so nothing ends a flow.  Bytes the reference would
 * read past the datagram read as 0 here.  OpenSSL's libcrypto does the primitives, as it does for
 * the plugin. */
#define QUIC_BUF 1500u   /* CURRENT_BUFFER_SIZE, quic_parser.hpp:45 */
#define QUIC_MAX_HDR 323u /* MAX_HEADER_LEN (67 + 256) */

/* quic_draft_version (:313-393): 0 = unknown; *v2 for QUIC version 2 */
static unsigned quic_draft(uint32_t v, int* v2) {
    *v2 = 0;
    const unsigned dv = v & 0xFF;
    if ((v >> 8) == 0xff0000u && dv >= 1 && dv <= 34) return dv;
    if ((v & 0x0F0F0F0Fu) == 0x0a0a0a0au) return 35;
    switch (v & 0xfffffff0u) {
        case 0xabcd0000u: return 29;
        case 0xf0f0f0f0u: case 0xf0f0f1f0u: case 0x07007000u: case 0xf0f0f2f0u: case 0x5c100000u: return 35;
        case 0xf123f0c0u: return 14;
    }
    switch (v & 0xffffff00u) {
        case 0x45474700u: return dv;
        case 0x51474f00u: case 0x91c17000u: return 35;
    }
    switch (v) {
        case 0x00000000u: return 1;
        case 0xfaceb000u: return 20;
        case 0xfaceb001u: return 22;
        case 0xfaceb002u: case 0xfaceb00du: case 0xfaceb00fu: case 0xfaceb00eu: case 0xfaceb011u:
        case 0xfaceb013u: case 0xfaceb010u: case 0xfaceb012u: return 27;
        case 0x00000001u: return 35;
        case 0x50435130u: case 0x50435131u: return 36;
        case 0xff020000u: case 0x709a50c4u: *v2 = 1; return 100;
        case 0x6b3343cfu: *v2 = 1; return 101;
        default: return 255;
    }
}

/* quic_obtain_version's salt (:403-474); NULL: none (version negotiation, or unsupported) */
static const uint8_t* quic_salt(uint32_t v) {
    static const uint8_t d7[20] = {0xaf, 0xc8, 0x24, 0xec, 0x5f, 0xc7, 0x7e, 0xca, 0x1e, 0x9d,
                                   0x36, 0xf3, 0x7f, 0xb2, 0xd4, 0x65, 0x18, 0xc3, 0x66, 0x39};
    static const uint8_t d10[20] = {0x9c, 0x10, 0x8f, 0x98, 0x52, 0x0a, 0x5c, 0x5c, 0x32, 0x96,
                                    0x8e, 0x95, 0x0e, 0x8a, 0x2c, 0x5f, 0xe0, 0x6d, 0x6c, 0x38};
    static const uint8_t d17[20] = {0xef, 0x4f, 0xb0, 0xab, 0xb4, 0x74, 0x70, 0xc4, 0x1b, 0xef,
                                    0xcf, 0x80, 0x31, 0x33, 0x4f, 0xae, 0x48, 0x5e, 0x09, 0xa0};
    static const uint8_t d21[20] = {0x7f, 0xbc, 0xdb, 0x0e, 0x7c, 0x66, 0xbb, 0xe9, 0x19, 0x3a,
                                    0x96, 0xcd, 0x21, 0x51, 0x9e, 0xbd, 0x7a, 0x02, 0x64, 0x4a};
    static const uint8_t d23[20] = {0xc3, 0xee, 0xf7, 0x12, 0xc7, 0x2e, 0xbb, 0x5a, 0x11, 0xa7,
                                    0xd2, 0x43, 0x2b, 0xb4, 0x63, 0x65, 0xbe, 0xf9, 0xf5, 0x02};
    static const uint8_t d29[20] = {0xaf, 0xbf, 0xec, 0x28, 0x99, 0x93, 0xd2, 0x4c, 0x9e, 0x97,
                                    0x86, 0xf1, 0x9c, 0x61, 0x11, 0xe0, 0x43, 0x90, 0xa8, 0x99};
    static const uint8_t s1[20] = {0x38, 0x76, 0x2c, 0xf7, 0xf5, 0x59, 0x34, 0xb3, 0x4d, 0x17,
                                   0x9a, 0xe6, 0xa4, 0xc8, 0x0c, 0xad, 0xcc, 0xbb, 0x7f, 0x0a};
    static const uint8_t v2p[20] = {0xa7, 0x07, 0xc2, 0x03, 0xa5, 0x9b, 0x47, 0x18, 0x4a, 0x1d,
                                    0x62, 0xca, 0x57, 0x04, 0x06, 0xea, 0x7a, 0xe3, 0xe5, 0xd3};
    static const uint8_t v2s[20] = {0x0d, 0xed, 0xe3, 0xde, 0xf7, 0x00, 0xa6, 0xdb, 0x81, 0x93,
                                    0x81, 0xbe, 0x6e, 0x26, 0x9d, 0xcb, 0xf9, 0xbd, 0x2e, 0xd9};
    static const uint8_t pico[20] = {0x30, 0x67, 0x16, 0xd7, 0x63, 0x75, 0xd5, 0x55, 0x4b, 0x2f,
                                     0x60, 0x5e, 0xef, 0x78, 0xd8, 0x33, 0x3d, 0xc1, 0xca, 0x36};
    int v2;
    const unsigned d = quic_draft(v, &v2);
    if (v == 0) return NULL;
    if (!v2 && v == 1) return s1;
    if (!v2 && d && d <= 9) return d7;
    if (!v2 && d && d <= 16) return d10;
    if (!v2 && d && d <= 20) return d17;
    if (!v2 && d && d <= 22) return d21;
    if (!v2 && d && d <= 28) return d23;
    if (!v2 && d && d <= 32) return d29;
    if (!v2 && d && d <= 35) return s1;
    if (!v2 && d && d <= 36) return pico;
    if (v2 && d && d <= 100) return v2p;
    if (v2 && d && d <= 101) return v2s;
    return NULL;
}

/* SHA-256 (FIPS 180-4) and HMAC-SHA256 (RFC 2104) for the Initial secrets (RFC 9001 §5.2): a
 * few hundred bytes per flow, where OpenSSL 3's one-shot HMAC() fetches its algorithms on every
 * call and serialises the walk threads on the provider's locks. */
typedef struct {
    uint32_t h[8];
    uint8_t b[64];
    uint64_t n;
} sha256_t;

/* one 64-byte block: OpenSSL's low-level transform (its SHA-NI / AVX2 code, no provider lookup or
 * lock: 88 ns a block on the container's Xeon against 630 ns for the portable C it replaced, which
 * made 75 % of an Initial's detection) */
static void sha256_block(uint32_t h[8], const uint8_t* p) {
    SHA256_CTX c;
    memcpy(c.h, h, 32);
    SHA256_Transform(&c, p);
    memcpy(h, c.h, 32);
}

static void sha256_init(sha256_t* s) {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(s->h, iv, sizeof(iv));
    s->n = 0;
}

static void sha256_put(sha256_t* s, const uint8_t* p, size_t n) {
    while (n) {
        const size_t at = s->n & 63, k = 64 - at < n ? 64 - at : n;
        memcpy(s->b + at, p, k);
        s->n += k;
        p += k;
        n -= k;
        if ((s->n & 63) == 0) sha256_block(s->h, s->b);
    }
}

static void sha256_end(sha256_t* s, uint8_t out[32]) {
    const uint64_t bits = s->n * 8;
    static const uint8_t pad[64] = {0x80};
    sha256_put(s, pad, 1 + ((119 - (s->n & 63)) & 63));
    uint8_t l[8];
    for (int i = 0; i < 8; ++i) l[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha256_put(s, l, 8);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(s->h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(s->h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(s->h[i] >> 8);
        out[4 * i + 3] = (uint8_t)s->h[i];
    }
}

/* HMAC-SHA256 with a key of at most 64 bytes (the salts and secrets here: 20 / 32) */
static void hmac_sha256(const uint8_t* key, size_t kl, const uint8_t* msg, size_t ml, uint8_t out[32]) {
    uint8_t ip[64], op[64], inner[32];
    memset(ip, 0x36, 64);
    memset(op, 0x5c, 64);
    for (size_t i = 0; i < kl; ++i) {
        ip[i] ^= key[i];
        op[i] ^= key[i];
    }
    sha256_t s;
    sha256_init(&s);
    sha256_put(&s, ip, 64);
    sha256_put(&s, msg, ml);
    sha256_end(&s, inner);
    sha256_init(&s);
    sha256_put(&s, op, 64);
    sha256_put(&s, inner, 32);
    sha256_end(&s, out);
}

/* HKDF-Expand-Label(secret, "tls13 " + label, "", len) for len <= 32 (one HMAC-SHA256 block) */
static void quic_expand(const uint8_t secret[32], const char* label, unsigned len, uint8_t* out) {
    uint8_t info[64];
    const unsigned ll = (unsigned)strlen(label);
    info[0] = 0;
    info[1] = (uint8_t)len;
    info[2] = (uint8_t)(6 + ll);
    memcpy(info + 3, "tls13 ", 6);
    memcpy(info + 9, label, ll);
    info[9 + ll] = 0;     /* context length */
    info[10 + ll] = 1;    /* HKDF-Expand block counter */
    uint8_t t[32];
    hmac_sha256(secret, 32, info, 11 + ll, t);
    memcpy(out, t, len);
}

/* The ciphers, fetched once per process (an implicit fetch per EVP_*Init_ex call is the other
 * provider-lock hot spot of OpenSSL 3) */
static EVP_CIPHER* g_aes_ecb;
static EVP_CIPHER* g_aes_gcm;
static pthread_once_t g_aes_once = PTHREAD_ONCE_INIT;
static void aes_fetch(void) {
    g_aes_ecb = EVP_CIPHER_fetch(NULL, "AES-128-ECB", NULL);
    g_aes_gcm = EVP_CIPHER_fetch(NULL, "AES-128-GCM", NULL);
}

/* quic_get_variable_length (:206-251) over a buffer of at least QUIC_BUF + 8 bytes */
static uint64_t quic_varint(const uint8_t* b, uint64_t* off) {
    const uint64_t o = *off;
    const unsigned n = 1u << (b[o < QUIC_BUF ? o : 0] >> 6);
    if (o >= QUIC_BUF - n || (n == 1 && o >= QUIC_BUF - 1)) {
        *off = o + n;
        return 0;
    }
    uint64_t v = b[o] & 0x3F;
    for (unsigned k = 1; k < n; ++k) v = (v << 8) | b[o + k];
    *off = o + n;
    return v;
}

/* TLSParser::parse with is_quic (no record header, tls_parser.cpp:72-100) on the reassembled
 * CRYPTO data: 0 nothing, 1 the handshake header parsed (what quic_set_server_port needs), 2 the
 * whole hello and its extensions' length (quic_parse_tls succeeded: QUICParser::parsed_initial) */
static int quic_tls(const uint8_t* d, uint32_t n) {
    if (6 > n) return 0;
    const uint8_t t = d[0];
    if (t != 1 && t != 2) return 0;
    if (!(d[4] == 3 && d[5] >= 1 && d[5] <= 3)) return 0;
    const uint32_t sid_off = 6 + 32;
    if (sid_off > n) return 1;
    const uint32_t sid_sec = 1 + tls_b(d, n, sid_off);
    if (sid_off + sid_sec > n) return 1;
    const uint32_t cs_off = sid_off + sid_sec;
    if (cs_off + 2 > n) return 1;
    uint32_t cs_sec = 2;
    if (t == 1) {
        const uint32_t cl = (tls_b(d, n, cs_off) << 8) | tls_b(d, n, cs_off + 1);
        if (cs_off + 2 + cl > n) return 1;
        cs_sec = 2 + cl;
    }
    const uint32_t cm_off = cs_off + cs_sec;
    if (cm_off > n) return 1;
    uint32_t cm_sec = 1;
    if (t == 1) {
        const uint32_t cm = tls_b(d, n, cm_off);
        if (1 + cm > n) return 1;
        cm_sec = 1 + cm;
    }
    const uint32_t ext_off = cm_off + cm_sec;  /* parse_extensions' has_valid_extension_length */
    if (ext_off > n) return 1;
    const uint32_t el = (tls_b(d, n, ext_off) << 8) | tls_b(d, n, ext_off + 1);
    return ext_off + el <= n ? 2 : 1;
}

/* quic_parse_initial (:1430-1470) of the Initial whose packet number starts at pkt[pn] with the
 * Length field's value plen: 0 failed, 1 the TLS handshake header parsed, 2 parsed_initial */
static int quic_open_initial(std_ctx* cx, const uint8_t* pkt, uint64_t pn, uint64_t plen, const uint8_t* salt,
                             int v2, const uint8_t* dcid, unsigned dcl) {
    uint8_t sec[32], cis[32], key[16], iv[12], hp[16];
    hmac_sha256(salt, 20, dcid, dcl, sec);  /* HKDF-Extract */
    quic_expand(sec, "client in", 32, cis);
    quic_expand(cis, v2 ? "quicv2 key" : "quic key", 16, key);
    quic_expand(cis, v2 ? "quicv2 iv" : "quic iv", 12, iv);
    quic_expand(cis, v2 ? "quicv2 hp" : "quic hp", 16, hp);
    pthread_once(&g_aes_once, aes_fetch);
    if (!g_aes_ecb || !g_aes_gcm) return 0;
    if (!cx->ecb && !(cx->ecb = EVP_CIPHER_CTX_new())) return 0;
    if (!cx->gcm && !(cx->gcm = EVP_CIPHER_CTX_new())) return 0;
    /* header protection (quic_decrypt_initial_header :780-842): AES-128-ECB of the sample */
    uint8_t mask[16];
    int ol = 0, fl = 0;
    EVP_CIPHER_CTX* c = cx->ecb;
    int ok = EVP_EncryptInit_ex(c, g_aes_ecb, NULL, hp, NULL) && EVP_CIPHER_CTX_set_padding(c, 0) &&
             EVP_EncryptUpdate(c, mask, &ol, pkt + pn + 4, 16) && EVP_EncryptFinal_ex(c, mask + ol, &fl);
    if (!ok) return 0;
    const uint8_t first = pkt[0] ^ (mask[0] & 0x0f);
    const unsigned pnl = (first & 3u) + 1;
    const uint64_t body = pn + pnl;
    uint64_t len = plen - pnl;  /* (unsigned: a Length below the packet number wraps and fails) */
    if (len > QUIC_BUF) return 0;
    if (body > QUIC_MAX_HDR) return 0;
    uint8_t hdr[QUIC_MAX_HDR];
    memcpy(hdr, pkt, body);
    hdr[0] = first;
    uint64_t pnum = 0;
    for (unsigned i = 0; i < pnl; ++i) pnum |= (uint64_t)(pkt[pn + i] ^ mask[1 + i]) << (8 * (pnl - 1 - i));
    for (unsigned i = 0; i < pnl; ++i) hdr[body - 1 - i] = (uint8_t)(pnum >> (8 * i));
    for (unsigned i = 0; i < 8; ++i) iv[4 + i] ^= (uint8_t)(pnum >> (8 * (7 - i)));
    /* payload (quic_decrypt_payload :844-905): AES-128-GCM, the last 16 bytes the tag */
    if (len <= 16) return 0;
    len -= 16;
    uint8_t dec[QUIC_BUF + 16];
    memset(dec, 0, sizeof(dec));
    c = cx->gcm;
    ok = EVP_DecryptInit_ex(c, g_aes_gcm, NULL, NULL, NULL) &&
         EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL) && EVP_DecryptInit_ex(c, NULL, NULL, key, iv) &&
         EVP_DecryptUpdate(c, NULL, &ol, hdr, (int)body) && EVP_DecryptUpdate(c, dec, &ol, pkt + body, (int)len) &&
         EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, 16, (void*)(pkt + body + len)) &&
         EVP_DecryptFinal_ex(c, dec + ol, &fl) > 0;
    if (!ok) return 0;
    /* CRYPTO frames (quic_reassemble_frames :1009-1043) */
    uint8_t asm_[QUIC_BUF + 16];
    memset(asm_, 0, sizeof(asm_));
    uint32_t cstart = 0xFFFF, clen = 0;
    uint64_t off = 0;
    while (off < len) {
        const uint8_t ft = dec[off];
        if (ft == 0x06) {
            off++;
            uint32_t fo = (uint32_t)quic_varint(dec, &off), fln = (uint32_t)quic_varint(dec, &off);
            if (off > len) {
                clen += fln;
                off += fln;
                continue;
            }
            if (fo > QUIC_BUF - 1) fo = QUIC_BUF - 1;
            if (fln > QUIC_BUF - 1 - fo) fln = QUIC_BUF - 1 - fo;
            if (fln > len - off) fln = (uint32_t)(len - off);
            memcpy(asm_ + fo, dec + off, fln);
            if (fo < cstart) cstart = fo;
            clen += fln;
            off += fln;
        } else if (ft == 0x02 || ft == 0x03) {  /* ACK */
            off++;
            (void)quic_varint(dec, &off);
            (void)quic_varint(dec, &off);
            const uint64_t rc = quic_varint(dec, &off);
            (void)quic_varint(dec, &off);
            for (uint64_t x = 0; x < rc && off < QUIC_BUF; ++x) {
                (void)quic_varint(dec, &off);
                (void)quic_varint(dec, &off);
            }
            if (ft == 0x03)
                for (int k = 0; k < 3; ++k) (void)quic_varint(dec, &off);
        } else if (ft == 0x1C || ft == 0x1D) {  /* CONNECTION_CLOSE */
            off++;
            (void)quic_varint(dec, &off);
            if (ft == 0x1C) (void)quic_varint(dec, &off);
            off += quic_varint(dec, &off);
        } else if (ft == 0x00 || ft == 0x01) {  /* PADDING, PING */
            off++;
        } else {
            return 0;
        }
        if (off >= QUIC_BUF) break;  /* (past the decrypted buffer: the reference's loop ends too) */
    }
    if (cstart == 0xFFFF) return 0;
    uint32_t n = clen;
    if (cstart + n > QUIC_BUF) n = QUIC_BUF - cstart;  /* (reads past the buffer: zeros here) */
    return quic_tls(asm_ + cstart, n);
}

/* QUICParser::quic_check_quic_long_header_packet (:1409-1428) for a new flow (no stored DCID) */
static int quic_detected(std_ctx* cx, const uint8_t* d, uint32_t n) {
    if (n < 8 || !(d[0] & 0x80)) return 0;  /* quic_long_header_packet: long header, >= 8 bytes */
    int v2;
    const uint32_t ver0 = ((uint32_t)d[1] << 24) | ((uint32_t)d[2] << 16) | ((uint32_t)d[3] << 8) | d[4];
    const unsigned dv0 = quic_draft(ver0, &v2);
    if (dv0 == 0 || dv0 >= 255) return 0;
    const uint8_t packets0 = (d[0] & 0x40) ? 0x80 : 0;  /* quic_parse_quic_bit: F_QUIC_BIT */
    /* the datagram, zero past its end: every read the reference makes beyond it sees 0 here */
    const size_t cap = (size_t)n + QUIC_BUF + 64;
    uint8_t stackbuf[4096];
    uint8_t* pk = cap <= sizeof(stackbuf) ? stackbuf : (uint8_t*)malloc(cap);
    if (!pk) return 0;
    memset(pk, 0, cap);
    memcpy(pk, d, n);
    uint8_t packets = packets0;
    int hs = 0, parsed = 0, result = -1;
    uint64_t off = 0;
    while (off + 8 <= n) {  /* quic_parse_headers (:1287-1377), coalesced packets */
        /* quic_parse_header (:1216-1285) */
        if (!(off < n) || !(pk[off] & 0x80)) break;
        const uint8_t b0 = pk[off];
        const uint32_t ver = ((uint32_t)pk[off + 1] << 24) | ((uint32_t)pk[off + 2] << 16) | ((uint32_t)pk[off + 3] << 8) | pk[off + 4];
        const uint8_t* salt = quic_salt(ver);
        quic_draft(ver, &v2);
        if (!salt && ver != 0) break;  /* quic_obtain_version */
        const unsigned dcl = pk[off + 5];
        uint64_t o = off + 6;
        if (!(o < n)) break;
        if (dcl > 20) break;
        const uint8_t* dcid = pk + o;
        o += dcl;
        if (!(o < n)) break;
        const unsigned scl = pk[o];
        o += 1;
        if (!(o < n)) break;
        if (scl > 20) break;
        o += scl;
        if (!(o < n)) break;
        unsigned type = (b0 & 0x30) >> 4;  /* quic_parse_packet_type */
        if (ver == 0) type = 4;          /* VERSION_NEGOTIATION */
        else if (v2) type = type == 1 ? 0 : (type == 2 ? 1 : (type == 3 ? 2 : 3));
        packets |= ver == 0 ? 0x01 : (type == 0 ? 0x02 : (type == 1 ? 0x04 : (type == 2 ? 0x08 : 0x10)));
        if (type == 1) {  /* ZERO_RTT */
            o += quic_varint(pk, &o);
        } else if (type == 2) {  /* HANDSHAKE */
            const uint64_t l = quic_varint(pk, &o);
            if (l > QUIC_BUF) { result = 0; break; }
            o += l;
        } else if (type == 0) {  /* INITIAL: quic_parse_initial_header (:1119-1158) */
            const uint64_t tl = quic_varint(pk, &o);
            if (!(o < n)) { result = 0; break; }
            o += tl;
            if (!(o < n)) { result = 0; break; }
            const uint64_t plen = quic_varint(pk, &o);
            if (plen > QUIC_BUF) { result = 0; break; }
            if (!(o < n)) { result = 0; break; }
            if (!(o + 4 < n)) { result = 0; break; }
            if (!parsed) {
                /* the first attempt with the flow's first DCID, then with this packet's: one DCID
                 * for a new flow (a flow whose later Initial only opens with the DCID of its first
                 * one -- after a Retry -- is decided on this packet's alone: not restated) */
                const int r = quic_open_initial(cx, pk + off, o - off, plen, salt ? salt : pk, v2, dcid, dcl);
                if (r >= 1) hs = 1;
                if (r == 2) parsed = 1;
            }
            o += plen;
        } else if (type == 3) {  /* RETRY */
            if (n < o + 16) { result = 0; break; }  /* (a negative token length: the pointer check fails) */
            o = n - 16;
            if (!(o < n)) { result = 0; break; }
        }
        if (!hs) { result = 0; break; }  /* quic_set_server_port: no TLS handshake parsed */
        off = o;
        if (type == 3) break;
    }
    if (pk != stackbuf) free(pk);
    if (result == 0) return 0;
    return packets != 0;
}

static int quic_add(void* ctx, ipxg_flow_record* f, const ipxg_packet_view* v, int idx) {
    uint32_t n;
    const uint8_t* d = payload(v, &n);
    /* add_quic: a flow without the extension gets it when QUIC is detected; with it, nothing
     * changes the flow (the packet types it records are enrichment) */
    if (!(f->ext & IPXG_STD_EXT_QUIC) && v->pkt->ip_proto == 17 && quic_detected((std_ctx*)ctx, d, n)) f->ext |= IPXG_STD_EXT_QUIC;
    return count(ctx, idx, 0);
}
static int quic_post_create(void* ctx, ipxg_flow_record* f, const ipxg_packet_view* v) {
    return quic_add(ctx, f, v, C_POST_CREATE);
}
static int quic_post_update(void* ctx, ipxg_flow_record* f, const ipxg_packet_view* v) {
    return quic_add(ctx, f, v, C_POST_UPDATE);
}

int ipxg_std_plugin(const char* name, ipxg_plugin* out) {
    if (!name || !out) return IPXG_EINVAL;
    memset(out, 0, sizeof(*out));
    out->pre_create = hook_pre_create;
    out->pre_export = hook_pre_export;
    out->pre_update = noop_pre_update;
    out->post_update = noop_post_update;
    if (strcmp(name, "dns") == 0) {
        out->proto_mask = 3;
        out->n_ports = 1;
        out->ports[0] = 53;
        out->follow_bytes = 1;  /* (outside port 53 the hooks read no payload byte) */
        out->post_create = dns_post_create;
        out->post_update = dns_post_update;
    } else if (strcmp(name, "http") == 0) {
        out->proto_mask = 1;
        const unsigned nm = sizeof(METHODS) / sizeof(METHODS[0]);
        for (unsigned k = 0; k < nm; ++k) {
            out->prefix_len[k] = 4;
            memcpy(out->prefix[k], METHODS[k], 4);
        }
        out->prefix_len[nm] = 4;
        memcpy(out->prefix[nm], "HTTP", 4);
        out->n_prefixes = nm + 1;
        out->post_create = http_post_create;
        out->pre_update = http_pre_update;
    } else if (strcmp(name, "tls") == 0) {
        out->proto_mask = 3;
        out->n_prefixes = 1;
        out->prefix_len[0] = 2;
        out->prefix[0][0] = 22;
        out->prefix[0][1] = 3;
        out->post_create = tls_post_create;
        out->pre_update = tls_pre_update;
    } else if (strcmp(name, "quic") == 0) {
        out->proto_mask = 2;
        out->n_prefixes = 1;
        out->prefix_len[0] = 1;
        out->prefix[0][0] = 0x80;
        out->masked = 1;
        out->prefix_mask[0][0] = 0x80;
        out->follow_packets = 30;  /* QUIC_MAX_ELEMCOUNT, quic.hpp:58 */
        /* outside the rule (a short header, bit 7 clear) the hooks read the payload's first byte
           only (quic_detected above; quic_long_header_packet :1105-1117) */
        out->follow_bytes = 1;
        out->post_create = quic_post_create;
        out->post_update = quic_post_update;
    } else {
        return IPXG_EINVAL;
    }
    out->copy_ctx = std_copy;
    out->free_ctx = std_free_copy;
    out->ctx = calloc(1, sizeof(std_ctx));
    return out->ctx ? IPXG_OK : IPXG_ENOMEM;
}

void ipxg_std_plugin_free(ipxg_plugin* pl) {
    if (pl && pl->ctx) {
        std_ctx* r = (std_ctx*)pl->ctx;
        while (r->next) { /* copies an engine still held (destroy the engine first) */
            std_ctx* c = r->next;
            r->next = c->next;
            std_ctx_release(c);
        }
        std_ctx_release(r);
        pl->ctx = NULL;
    }
}

void ipxg_std_plugin_calls(const ipxg_plugin* pl, uint64_t* out6) {
    if (!pl || !pl->ctx || !out6) return;
    const std_ctx* r = (const std_ctx*)pl->ctx;
    memcpy(out6, r->calls, sizeof(uint64_t) * C_N);
    for (const std_ctx* c = r->next; c; c = c->next)
        for (int k = 0; k < C_N; ++k) out6[k] += c->calls[k];
}
