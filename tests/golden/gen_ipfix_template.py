"""Writes tests/golden/ipfix_basic_templates.json from the reference's own header: compiles a
tiny C++ program that includes /root/reference/include/ipfixprobe/ipfix-elements.hpp and
expands BASIC_TMPLT_V4 / BASIC_TMPLT_V6 into (enterprise, element id, length) triples, plus
MK_NTP_TS of a few timestamps.  Run in the build container (the reference is not on the GPU box);
the JSON is the committed fixture.  The header is macros only: nothing else is needed."""
import json
import os
import subprocess
import tempfile

REF = "/root/reference/include/ipfixprobe/ipfix-elements.hpp"
HERE = os.path.dirname(os.path.abspath(__file__))

SRC = r'''
#include <cstdint>
#include <cstdio>
#include <sys/time.h>
#include "%s"
#define TRIPLE(EN, ID, LEN, SRC) std::printf("[%%d, %%d, %%d],", (int)(EN), (int)(ID), (int)(LEN));
#define EXPAND(FIELD) FIELD(TRIPLE)
int main() {
    std::printf("{\"BASIC_TMPLT_V4\": [");
    BASIC_TMPLT_V4(EXPAND)
    std::printf("null], \"BASIC_TMPLT_V6\": [");
    BASIC_TMPLT_V6(EXPAND)
    std::printf("null], \"MK_NTP_TS\": [");
    const long ts[][2] = {{0, 0}, {1600000000, 1}, {1700000000, 999999}, {4000000000L, 500000}, {1234567890, 123456}};
    for (auto& t : ts) {
        struct timeval tv;
        tv.tv_sec = t[0];
        tv.tv_usec = t[1];
        std::printf("[%%ld, %%ld, \"%%016llx\"],", t[0], t[1], (unsigned long long)MK_NTP_TS(tv));
    }
    std::printf("null]}\n");
}
''' % REF


def main():
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.cpp")
        exe = os.path.join(d, "t")
        with open(c, "w") as f:
            f.write(SRC)
        subprocess.run(["g++", "-std=c++17", "-o", exe, c], check=True)
        out = subprocess.run([exe], check=True, stdout=subprocess.PIPE, text=True).stdout
    js = json.loads(out)
    for k in js:
        js[k] = [v for v in js[k] if v is not None]
    js["source"] = "expanded from " + REF + " (BASIC_TMPLT_V4/V6, IPXP_TS_MSEC unset; MK_NTP_TS)"
    with open(os.path.join(HERE, "ipfix_basic_templates.json"), "w") as f:
        json.dump(js, f)
    print("fields v4 %d v6 %d" % (len(js["BASIC_TMPLT_V4"]), len(js["BASIC_TMPLT_V6"])))


if __name__ == "__main__":
    main()
