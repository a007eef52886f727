// ref_plugins.cpp -- TEST INFRASTRUCTURE.  The reference's own process plugins (the 23 with a
// functional test: their unmodified sources under /root/reference/src/plugins/process, built by
// oracle/Makefile into oracle/_ref/libref_plugins.so together with this file) behind the
// product's plugin adapter (ipfixprobe_amd/host/plugin_adapter.hpp), as ipxg_plugin structs the
// engine's bridge (ipxg_add_plugin) and the oracle take alike.  Nothing in the product links
// or loads this; tests/test_ref_plugins.py does.
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>

#include <ipfixprobe/pluginFactory/pluginFactory.hpp>
#include <ipfixprobe/processPlugin.hpp>

#include "../ipfixprobe_amd/host/plugin_adapter.hpp"

namespace {

struct Held {
    std::unique_ptr<ipxp::ProcessPlugin> plugin;
    std::unique_ptr<ipxg_ref::Adapter> adapter;
};

std::map<void*, Held*>& held() {
    static std::map<void*, Held*> m;  // adapter (the ipxg_plugin's ctx) -> what it keeps alive
    return m;
}

// A process plugin that throws the reference's PluginError (plugin.hpp:81-91) on its nth
// post_create / post_update call -- each instance counts its own calls, so every walk thread's
// copy fails on its nth -- behind the same adapter, with dns's rule (port 53): the failure path
// of the bridge, where the reference's input worker catches the error and
// reports it through WorkerResult (workers.cpp:107-112).
class FailingPlugin : public ipxp::ProcessPlugin {
public:
    FailingPlugin(int id, int nth) : ipxp::ProcessPlugin(id), m_nth(nth) {}
    ipxp::ProcessPlugin* copy() override { return new FailingPlugin(*this); }
    ipxp::OptionsParser* get_parser() const override { return nullptr; }
    std::string get_name() const override { return "failing"; }
    int post_create(ipxp::Flow&, const ipxp::Packet&) override { return step(); }
    int post_update(ipxp::Flow&, const ipxp::Packet&) override { return step(); }

private:
    int step() {
        if (++m_calls == m_nth) throw ipxp::PluginError("failing plugin: hook call " + std::to_string(m_nth));
        return 0;
    }
    int m_nth, m_calls = 0;
};

}  // namespace

extern "C" {

// FailingPlugin(nth) behind an adapter with dns's rule: *out is its ipxg_plugin (release it with
// ref_plugin_destroy).  0, or -1.
int ref_failing_plugin_create(int nth, ipxg_plugin* out) {
    auto h = std::make_unique<Held>();
    h->plugin = std::make_unique<FailingPlugin>(0, nth);
    h->adapter = std::make_unique<ipxg_ref::Adapter>(h->plugin.get());
    if (!h->adapter->make("dns", *out)) return -1;
    held()[out->ctx] = h.release();
    return 0;
}

// A fresh instance of the reference plugin `name` (its registrar's factory entry, as ipfixprobe's
// process_plugin_args creates it, ipfixprobe.cpp:300-308) behind an adapter: *out is its
// ipxg_plugin.  0; -1 unknown plugin or no rule for it; -2 the plugin threw.
int ref_plugin_create(const char* name, const char* params, ipxg_plugin* out) {
    try {
        const int id = ipxp::ProcessPluginIDGenerator::instance().generatePluginID();
        auto h = std::make_unique<Held>();
        h->plugin = ipxp::ProcessPluginFactory::getInstance().createUnique(name, std::string(params ? params : ""), id);
        h->adapter = std::make_unique<ipxg_ref::Adapter>(h->plugin.get());
        if (!h->adapter->make(name, *out)) return -1;
        held()[out->ctx] = h.release();
        return 0;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "ref_plugin_create(%s): %s\n", name, e.what());
        return -2;
    }
}

void ref_plugin_destroy(ipxg_plugin* pl) {
    auto it = held().find(pl->ctx);
    if (it == held().end()) return;
    delete it->second;
    held().erase(it);
    pl->ctx = nullptr;
}

// The extensions an exported record carries (its ext handle): RecordExt::get_text()
// per extension in chain order, separated by '\n', into out (cap bytes, NUL-terminated); the
// length (or the length needed when cap is short).  0 for ext = 0.
int ref_ext_text(uint64_t ext, char* out, int cap) {
    std::string s;
    if (ext) {
        for (ipxp::RecordExt* e = ipxg_ref::flow_of(ext)->m_exts; e; e = e->m_next) {
            if (!s.empty()) s += '\n';
            s += e->get_text();  // (ids differ between plugin instances: not printed)
        }
    }
    if (out && cap > 0) {
        const size_t n = std::min<size_t>(s.size(), (size_t)cap - 1);
        std::memcpy(out, s.data(), n);
        out[n] = 0;
    }
    return (int)s.size();
}

// The number of extensions an exported record carries: the reference's UniRec output sends one
// record per extension (a second of the same type flushes the first, unirec.cpp:361-397), so a
// flow with k extensions is k lines of a functional-test golden, and one with none is no line.
int ref_ext_count(uint64_t ext) {
    int n = 0;
    if (ext)
        for (ipxp::RecordExt* e = ipxg_ref::flow_of(ext)->m_exts; e; e = e->m_next) ++n;
    return n;
}

// The consumer's release of an exported record's Flow (and its extension chain).
void ref_ext_free(uint64_t ext) {
    if (ext) delete ipxg_ref::flow_of(ext);
}

}  // extern "C"
