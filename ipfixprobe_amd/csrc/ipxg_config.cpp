// ipxg_config.cpp -- the reference cache plugin's option string, restated for the engine.
//
// "s=EXP;l=EXP;a=SEC;i=SEC;S;fe=true|false;fs=N;ft=SEC" with the long names "size", "line",
// "active", "inactive", "split", "frag-enable", "frag-size", "frag-timeout"
// (CacheOptParser, cache.hpp:81-221; OptionsParser::parse, options.cpp:62-160: ';'-separated
// tokens, "name=value" or "name" followed by its value as the next token), plus the GPU keys
// "dev"/"device", "batch", "dlt" (EN10MB | RAW | LINUX_SLL | LINUX_SLL2 or a number) and
// "ingest" (binned | atomic), "walk" (auto | wide | narrow: which k_bin variant walks
// the header chains), "ps"/"parser-stats" (true | false: TopPorts + VlanStats) and "strict"
// (true | false: the reference's line table replayed exactly, ipxg_strict.hip).
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ipxg.h"

namespace {

bool to_u32(const std::string& s, uint32_t& v) {
    if (s.empty()) return false;
    char* end = nullptr;
    unsigned long long x = std::strtoull(s.c_str(), &end, 10);
    if (*end != 0 || x > 0xFFFFFFFFull) return false;
    v = (uint32_t)x;
    return true;
}

}  // namespace

extern "C" int ipxg_config_parse(const char* params, ipxg_config* cfg) {
    if (!cfg) return IPXG_EINVAL;
    if (!params || !*params) return IPXG_OK;
    std::vector<std::string> tok;
    std::string cur;
    for (const char* p = params;; ++p) {
        if (*p == ';' || *p == 0) {
            size_t eq = cur.find('=');
            tok.push_back(cur.substr(0, eq));
            if (eq != std::string::npos) tok.push_back("=" + cur.substr(eq + 1));
            cur.clear();
            if (*p == 0) break;
        } else {
            cur.push_back(*p);
        }
    }
    for (size_t i = 0; i < tok.size(); ++i) {
        const std::string name = tok[i];
        if (name.empty()) continue;
        auto arg = [&](std::string& a) -> bool {
            if (i + 1 < tok.size() && !tok[i + 1].empty() && tok[i + 1][0] == '=') {
                a = tok[++i].substr(1);
                return true;
            }
            if (i + 1 < tok.size()) {
                a = tok[++i];
                return true;
            }
            return false;
        };
        std::string a;
        uint32_t v;
        if (name == "S" || name == "split") {
            cfg->split_biflow = 1;
            if (i + 1 < tok.size() && !tok[i + 1].empty() && tok[i + 1][0] == '=') ++i;
        } else if (name == "s" || name == "size") {
            if (!arg(a) || !to_u32(a, v) || v < 4 || v > 30) return IPXG_EINVAL;
            cfg->cache_exp = v;
        } else if (name == "l" || name == "line") {
            if (!arg(a) || !to_u32(a, v) || v > 30) return IPXG_EINVAL;
            cfg->line_exp = v;
        } else if (name == "a" || name == "active") {
            if (!arg(a) || !to_u32(a, v)) return IPXG_EINVAL;
            cfg->active_s = v;
        } else if (name == "i" || name == "inactive") {
            if (!arg(a) || !to_u32(a, v)) return IPXG_EINVAL;
            cfg->inactive_s = v;
        } else if (name == "fe" || name == "frag-enable") {
            if (!arg(a)) return IPXG_EINVAL;
            if (a == "true") cfg->frag_enable = 1;
            else if (a == "false") cfg->frag_enable = 0;
            else return IPXG_EINVAL;
        } else if (name == "fs" || name == "frag-size") {
            if (!arg(a) || !to_u32(a, v) || v == 0) return IPXG_EINVAL;
            cfg->frag_size = v;
        } else if (name == "ft" || name == "frag-timeout") {
            if (!arg(a) || !to_u32(a, v)) return IPXG_EINVAL;
            cfg->frag_timeout_s = v;
        } else if (name == "dev" || name == "device") {
            if (!arg(a) || !to_u32(a, v)) return IPXG_EINVAL;
            cfg->device_id = (int32_t)v;
        } else if (name == "batch") {
            if (!arg(a) || !to_u32(a, v) || v == 0 || v > IPXG_MAX_BATCH) return IPXG_EINVAL;
            cfg->batch_pkts = v;
        } else if (name == "ingest") {
            if (!arg(a)) return IPXG_EINVAL;
            if (a == "atomic") cfg->flags |= IPXG_CFG_ATOMIC_INGEST;
            else if (a == "binned") cfg->flags &= ~IPXG_CFG_ATOMIC_INGEST;
            else return IPXG_EINVAL;
        } else if (name == "strict") {
            if (!arg(a)) return IPXG_EINVAL;
            if (a == "true") cfg->flags |= IPXG_CFG_STRICT;
            else if (a == "false") cfg->flags &= ~IPXG_CFG_STRICT;
            else return IPXG_EINVAL;
        } else if (name == "ps" || name == "parser-stats") {
            if (!arg(a)) return IPXG_EINVAL;
            if (a == "true") cfg->flags |= IPXG_CFG_PARSER_STATS;
            else if (a == "false") cfg->flags &= ~IPXG_CFG_PARSER_STATS;
            else return IPXG_EINVAL;
        } else if (name == "walk") {
            if (!arg(a)) return IPXG_EINVAL;
            cfg->flags &= ~(IPXG_CFG_WALK_WIDE | IPXG_CFG_WALK_NARROW);
            if (a == "wide") cfg->flags |= IPXG_CFG_WALK_WIDE;
            else if (a == "narrow") cfg->flags |= IPXG_CFG_WALK_NARROW;
            else if (a != "auto") return IPXG_EINVAL;
        } else if (name == "dlt") {
            if (!arg(a)) return IPXG_EINVAL;
            if (a == "EN10MB") cfg->datalink = IPXG_DLT_EN10MB;
            else if (a == "RAW") cfg->datalink = IPXG_DLT_RAW;
            else if (a == "LINUX_SLL") cfg->datalink = IPXG_DLT_LINUX_SLL;
            else if (a == "LINUX_SLL2") cfg->datalink = IPXG_DLT_LINUX_SLL2;
            else if (to_u32(a, v)) cfg->datalink = v;
            else return IPXG_EINVAL;
        } else {
            return IPXG_EINVAL;  // "invalid option" (options.cpp:120-122)
        }
    }
    return IPXG_OK;
}
