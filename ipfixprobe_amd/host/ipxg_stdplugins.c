/* ipxg_stdplugins.c -- native stand-ins of the dns / http / tls / quic process plugins as
 * ipxg_plugin rules + hooks (include/ipxg_stdplugins.h): the decisions of each reference
 * plugin that end a flow or claim it, restated from its source (cited per function).  Not the
 * enrichment -- the real plugins run behind the adapter of INTEGRATION.md. */
#include "../../include/ipxg_stdplugins.h"

#include <stdlib.h>
#include <string.h>

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
} std_ctx;

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
    free(c);
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

/* ---- QUIC (quic.cpp:350-549; QUICParser::quic_long_header_packet quic_parser.cpp:1105-1117,
 * quic_draft_version :313-380) -- a long-header packet (first payload bit), UDP, >= 8 bytes, a
 * version the parser knows (here: 1, version negotiation 0, IETF drafts ff0000xx 1-34) claims
 * the flow; version negotiation ends it (FLOW_FLUSH, quic.cpp:400-403). */
static int quic_version_ok(uint32_t v) {
    return v == 0 || v == 1 || ((v >> 8) == 0xff0000u && (v & 0xFF) >= 1 && (v & 0xFF) <= 34);
}
static int quic_add(void* ctx, ipxg_flow_record* f, const ipxg_packet_view* v, int idx) {
    uint32_t n;
    const uint8_t* d = payload(v, &n);
    int r = 0;
    if (v->pkt->ip_proto == 17 && n >= 8 && (d[0] & 0x80)) {
        const uint32_t ver = ((uint32_t)d[1] << 24) | ((uint32_t)d[2] << 16) | ((uint32_t)d[3] << 8) | d[4];
        if (quic_version_ok(ver)) {
            f->ext |= IPXG_STD_EXT_QUIC;
            if (ver == 0) r = IPXG_FLOW_FLUSH;
        }
    }
    return count(ctx, idx, r);
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
            free(c);
        }
        free(r);
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
