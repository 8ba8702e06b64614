// Host-only test of the shim's request combiner (include/pcp_pcl.hpp detail::Combiner): T
// threads submit single requests concurrently; every request must come back with its own
// result exactly once, batches must actually merge requests, and a failing batch must re-throw
// in every thread whose request it held.  No GPU: the batch function is a stand-in.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <stdexcept>
#include <thread>
#include <vector>

#include "pcp_pcl.hpp"

struct Req {
    long v;
    long out = 0;
    bool done = false;
    std::exception_ptr err;
};

int main() {
    using cloud_blend_double::detail::Combiner;
    int fails = 0;
    {
        Combiner<Req> c;
        std::atomic<long> batches{0}, items{0}, bad{0}, maxb{0};
        std::vector<std::thread> th;
        const int T = 16, N = 4000;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                for (int i = 0; i < N; i++) {
                    Req r{(long)t * 1000000 + i};
                    c.submit(&r, [&](std::vector<Req*>& b) {
                        batches++;
                        items += (long)b.size();
                        long m = maxb.load();
                        while ((long)b.size() > m && !maxb.compare_exchange_weak(m, (long)b.size())) {}
                        std::this_thread::sleep_for(std::chrono::microseconds(50));
                        for (Req* x : b) x->out += x->v * 2 + 1;  // += : a request run twice is caught
                    });
                    bad += r.out != r.v * 2 + 1;
                }
            });
        for (auto& x : th) x.join();
        std::printf("combiner: %ld requests in %ld batches (mean %.2f, max %ld), %ld wrong\n", (long)items,
                    (long)batches, (double)items / (double)batches, (long)maxb, (long)bad);
        if (bad != 0 || items != (long)T * N) fails++;
        if ((double)items / (double)batches < 2.0) fails++;  // 16 busy threads must merge
    }
    {
        Combiner<Req> c;
        std::atomic<long> thrown{0}, ok{0};
        std::vector<std::thread> th;
        for (int t = 0; t < 8; t++)
            th.emplace_back([&, t] {
                for (int i = 0; i < 500; i++) {
                    Req r{(long)t * 1000 + i};
                    try {
                        c.submit(&r, [&](std::vector<Req*>& b) {
                            for (Req* x : b)
                                if (x->v % 7 == 0) throw std::runtime_error("batch failed");
                            for (Req* x : b) x->out = 1;
                        });
                        ok += r.out == 1;
                    } catch (const std::runtime_error&) {
                        thrown++;
                    }
                }
            });
        for (auto& x : th) x.join();
        std::printf("combiner errors: %ld thrown, %ld completed, of %d\n", (long)thrown, (long)ok, 8 * 500);
        if (thrown + ok != 8 * 500 || thrown == 0) fails++;
    }
    std::printf(fails ? "combiner_test: FAILED\n" : "combiner_test: all checks passed\n");
    return fails ? 1 : 0;
}
