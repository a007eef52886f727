// The plugin-lifetime contract at the C ABI (include/ipxg.h, ipxg_add_plugin / ipxg_destroy;
// VERDICT r5 item 7), from a C++ caller as the reference's storage plugin would be one: a process
// plugin fails (IPXG_PLUGIN_ERROR on its n-th hook call, the reference's PluginError), the batch
// fails with IPXG_EPLUGIN, the engine refuses work (IPXG_ESTATE), then ipxg_destroy -- which may call
// only free_ctx, once per copy it made -- and only then the caller frees the plugin itself.
// Built with AddressSanitizer on this (host) code by tests/Makefile: a hook or free_ctx reaching a
// freed context, or a copy freed twice, is reported by ASan; the counters below check the rest.
// Exit 0: contract held; 77: no GPU (ipxg_create failed); anything else: a failure (printed).
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../include/ipxg.h"

namespace {

struct Counts {
    int live = 0;           // contexts alive: the original + the engine's copies
    int copies = 0;         // copies made
    int frees = 0;          // copies released through free_ctx
    long hooks = 0;         // hook calls over every instance
    bool destroyed = false;  // set after ipxg_destroy returned: no call may follow
    int late_calls = 0;      // calls that arrived after it anyway
};

struct Ctx {
    Counts* c;
    long calls = 0;
    long fail_at;
    std::string msg;
    bool failed = false;
    explicit Ctx(Counts* k, long n) : c(k), fail_at(n) { c->live++; }
    Ctx(const Ctx& o) : c(o.c), calls(0), fail_at(o.fail_at) { c->live++; }
    ~Ctx() { c->live--; }
    int hook() {
        if (c->destroyed) c->late_calls++;
        c->hooks++;
        if (++calls == fail_at) {
            failed = true;
            msg = "lifetime test plugin: hook call " + std::to_string(calls);
            return IPXG_PLUGIN_ERROR;
        }
        return 0;
    }
};

ipxg_plugin make_plugin(Ctx* ctx) {
    ipxg_plugin q;
    std::memset(&q, 0, sizeof q);
    q.ctx = ctx;
    q.proto_mask = 2;  // UDP
    q.n_ports = 1;
    q.ports[0] = 53;
    q.pre_create = [](void* c, ipxg_packet_view*) { return static_cast<Ctx*>(c)->hook(); };
    q.post_create = [](void* c, ipxg_flow_record*, const ipxg_packet_view*) { return static_cast<Ctx*>(c)->hook(); };
    q.pre_update = [](void* c, ipxg_flow_record*, ipxg_packet_view*) { return static_cast<Ctx*>(c)->hook(); };
    q.post_update = [](void* c, ipxg_flow_record*, const ipxg_packet_view*) { return static_cast<Ctx*>(c)->hook(); };
    q.pre_export = [](void* c, ipxg_flow_record*) { (void)static_cast<Ctx*>(c)->hook(); };
    q.copy_ctx = [](void* c) -> void* {
        Ctx* o = static_cast<Ctx*>(c);
        if (o->c->destroyed) o->c->late_calls++;
        o->c->copies++;
        return new Ctx(*o);
    };
    q.free_ctx = [](void* c) {
        Ctx* o = static_cast<Ctx*>(c);
        if (o->c->destroyed) o->c->late_calls++;
        o->c->frees++;
        delete o;
    };
    q.error = [](void* c) -> const char* {
        Ctx* o = static_cast<Ctx*>(c);
        if (!o->failed) return nullptr;
        o->failed = false;
        return o->msg.c_str();
    };
    return q;
}

// n packets of 64-byte Ethernet/IPv4/UDP frames over `flows` flows, all to port 53
void udp53_batch(uint32_t n, uint32_t flows, std::vector<uint8_t>& arena, std::vector<ipxg_pkt_desc>& desc) {
    arena.assign((size_t)n * 64, 0);
    desc.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t* f = &arena[(size_t)i * 64];
        const uint32_t fl = i % flows;
        f[0] = 2, f[6] = 4, f[12] = 0x08, f[14] = 0x45, f[17] = 50, f[22] = 64, f[23] = 17;
        f[26] = 10, f[27] = (uint8_t)(fl >> 16), f[28] = (uint8_t)(fl >> 8), f[29] = (uint8_t)fl;
        f[30] = 192, f[31] = 168, f[32] = 0, f[33] = 1;
        f[34] = (uint8_t)((1024 + fl % 50000) >> 8), f[35] = (uint8_t)(1024 + fl % 50000);
        f[36] = 0, f[37] = 53, f[39] = 30;
        desc[i] = ipxg_pkt_desc{i * 64u, 64, 64, 1700000000u + i / 1000u, (i % 1000u) * 1000u};
    }
}

int fail(const char* what, int rc, ipxg_engine* e) {
    std::printf("FAIL: %s (rc %d: %s)\n", what, rc, e ? ipxg_last_error(e) : "");
    return 1;
}

}  // namespace

int main() {
    Counts counts;
    Ctx* original = new Ctx(&counts, 500);  // fails on the 500th hook call of an instance
    ipxg_config cfg;
    ipxg_config_default(&cfg);
    if (ipxg_config_parse("s=16", &cfg) != IPXG_OK) return fail("config", -1, nullptr);
    ipxg_engine* e = nullptr;
    if (ipxg_create(&cfg, &e) != IPXG_OK) {
        std::printf("no GPU: ipxg_create failed\n");
        delete original;
        return counts.live == 0 ? 77 : 1;
    }
    int rc;
    if ((rc = ipxg_set_walk_threads(e, 4)) != IPXG_OK) return fail("walk threads", rc, e);
    const ipxg_plugin q = make_plugin(original);
    if ((rc = ipxg_add_plugin(e, &q)) != IPXG_OK) return fail("add plugin", rc, e);
    std::vector<uint8_t> arena;
    std::vector<ipxg_pkt_desc> desc;
    udp53_batch(20000, 400, arena, desc);
    const ipxg_batch b{arena.data(), arena.size(), desc.data(), (uint32_t)desc.size(), 0};
    rc = ipxg_submit(e, &b);
    if (rc != IPXG_EPLUGIN) return fail("the batch should fail with IPXG_EPLUGIN", rc, e);
    if (!std::strstr(ipxg_last_error(e), "lifetime test plugin: hook call 500"))
        return fail("the plugin's message in ipxg_last_error", rc, e);
    rc = ipxg_submit(e, &b);
    if (rc != IPXG_ESTATE) return fail("a failed engine should refuse work with IPXG_ESTATE", rc, e);
    rc = ipxg_finish(e);
    if (rc != IPXG_ESTATE) return fail("ipxg_finish after the failure should give IPXG_ESTATE", rc, e);
    const long hooks_before = counts.hooks;
    if ((rc = ipxg_destroy(e)) != IPXG_OK) return fail("destroy", rc, nullptr);
    counts.destroyed = true;
    if (counts.hooks != hooks_before) return fail("ipxg_destroy called a hook of a failed plugin", -1, nullptr);
    if (counts.copies < 1) return fail("no walk copies were made (4 walk threads)", -1, nullptr);
    if (counts.frees != counts.copies) return fail("ipxg_destroy did not release every copy exactly once", -1, nullptr);
    if (counts.live != 1) return fail("copies still alive after ipxg_destroy", -1, nullptr);
    delete original;  // the caller's instance, freed only now (the contract)
    if (counts.live != 0 || counts.late_calls) return fail("a call after ipxg_destroy returned", -1, nullptr);
    std::printf("ok: IPXG_EPLUGIN then IPXG_ESTATE; destroy released %d copies (%ld hook calls before it), "
                "none after\n", counts.copies, counts.hooks);
    return 0;
}
