// Host-side checks of the walk's thread pool (ipfixprobe_amd/csrc/ipxg_walkpool.hpp), built and
// run by tests/test_walkpool.py under AddressSanitizer and under ThreadSanitizer.  The job of each
// run writes a per-walk array sized by the run's thread count, indexed by t -- the shape of the
// round-3 fault (pool threads t >= T writing past plugin_walk's per-walk arrays), which ASan
// reports as a heap overflow if the pool ever hands a job a t outside [0, n).
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <vector>

#include "../ipfixprobe_amd/csrc/ipxg_walkpool.hpp"

#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                 \
        }                                                                 \
    } while (0)

int main() {
    using ipxg::WalkPool;
    {
        WalkPool p(16);
        CHECK(p.size() == 16);
        // every n from 1 to past the pool's size, many times over: each t < n exactly once
        for (int rep = 0; rep < 200; ++rep)
            for (unsigned n = 1; n <= 18; ++n) {
                std::vector<int>* per = new std::vector<int>(n < 16 ? n : 16, 0);  // heap: ASan bounds
                int* a = per->data();
                const unsigned ran = p.run([a](unsigned t) { a[t] += 1; }, n);
                CHECK(ran == (n < 16 ? n : 16));
                for (unsigned t = 0; t < ran; ++t) CHECK(a[t] == 1);
                delete per;
            }
        CHECK(!p.take_escaped());
        CHECK(p.run([](unsigned) { CHECK(false); }, 0) == 0);
        // a worker that raises: recorded, the run still completes every other share
        std::vector<int> hit(8, 0);
        p.run([&](unsigned t) {
            hit[t] = 1;
            if (t == 5) throw std::runtime_error("hook");
        }, 8);
        for (int h : hit) CHECK(h == 1);
        CHECK(p.take_escaped());
        CHECK(!p.take_escaped());  // (take semantics)
        // the caller's own share raising: held until the workers are done with the job
        std::vector<int> hit2(16, 0);
        p.run([&](unsigned t) {
            if (t == 0) throw 7;
            hit2[t] = 1;
        }, 16);
        for (unsigned t = 1; t < 16; ++t) CHECK(hit2[t] == 1);
        CHECK(p.take_escaped());
    }
    {
        WalkPool p(1);  // no worker threads: the caller walks alone
        int x = 0;
        CHECK(p.run([&](unsigned t) { x += 1 + (int)t; }, 4) == 1);
        CHECK(x == 1);
    }
    {
        WalkPool p(4);  // destroyed idle, never run
    }
    std::puts("walkpool ok");
    return 0;
}
