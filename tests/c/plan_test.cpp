// plan_test.cpp -- CPU unit test of tv_plan.h (the resident payload under a device budget, tv_set_layout): the
// allocation retry loop ends on every input, with a fake allocator that fails above a capacity.
// Built and run by tests/test_plan.py (g++; no HIP).
#include <cstdio>
#include <cstdlib>

#include <algorithm>

#include "../../torrent_amd/csrc/tv_plan.h"

using tvi::PayloadPlan;

static int failures = 0;
#define CHECK(cond)                                                         \
    do {                                                                    \
        if (!(cond)) {                                                      \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);     \
            failures++;                                                     \
        }                                                                   \
    } while (0)

// allocate under a device that holds `capacity` bytes; returns the status, the plan, the tries
static int run(uint64_t count, uint64_t stride, uint64_t budget, uint64_t capacity, PayloadPlan* plan, int* tries,
               uint64_t* held_budget, int bufs = tvi::kWinBufsDefault) {
    const uint64_t slack = 256;
    *tries = 0;
    uint64_t failed = 0;
    return tvi::allocate_payload(
        count, stride, slack, budget,
        [&](const PayloadPlan& p, uint64_t) -> int {
            if (++*tries > 1000) {  // a loop that does not end
                std::printf("FAIL: more than 1000 tries (count %llu stride %llu capacity %llu)\n",
                            (unsigned long long)count, (unsigned long long)stride, (unsigned long long)capacity);
                std::exit(1);
            }
            return p.bytes <= capacity ? 0 : 1;
        },
        plan, held_budget, &failed, bufs);
}

int main() {
    const uint64_t MiB = 1ull << 20, GiB = 1ull << 30;
    PayloadPlan p;
    int tries;
    uint64_t b;
    // cfg2 on an idle MI355X: the whole shard
    CHECK(run(16384, MiB + 256, 280 * GiB, 288 * GiB, &p, &tries, &b) == 0 && !p.win && tries == 1);
    CHECK(p.bytes == 16384 * (MiB + 256) + 256);
    // a budget below the shard: the default window buffers within the budget, a multiple of 64 pieces
    CHECK(run(16384, MiB + 256, 2 * GiB, 288 * GiB, &p, &tries, &b) == 0 && p.win && p.bufs == tvi::kWinBufsDefault);
    CHECK(p.bytes <= 2 * GiB && p.win_n % 64 == 0 && p.win_n >= 256);
    // two buffers asked for: two windows of twice the pieces
    CHECK(run(16384, MiB + 256, 2 * GiB, 288 * GiB, &p, &tries, &b, 2) == 0 && p.win && p.bufs == 2);
    CHECK(p.bytes <= 2 * GiB && p.win_n == 1024 - 64);
    // a budget of three one-piece windows asks for four buffers: three (one piece each)
    CHECK(run(100, MiB + 256, 3 * (MiB + 512), 288 * GiB, &p, &tries, &b, 4) == 0 && p.bufs == 3 && p.win_n == 1);
    // more buffers than windows are never allocated
    CHECK(run(3, MiB + 256, 3 * MiB, 288 * GiB, &p, &tries, &b, 8) == 0 && p.win && p.win_n * p.bufs <= 3 + 2);
    for (int B = 1; B <= tvi::kWinBufsMax + 2; B++) {
        CHECK(run(16384, MiB + 256, GiB / 2, 288 * GiB, &p, &tries, &b, B) == 0 && p.win && p.bytes <= GiB / 2);
        CHECK(p.bufs == std::min(B, tvi::kWinBufsMax));
    }
    // the budget says yes, the device says no: retried with smaller windows until one fits
    CHECK(run(51200, 4 * MiB + 256, 200 * GiB, 3 * GiB, &p, &tries, &b) == 0 && p.win && p.bytes <= 3 * GiB);
    CHECK(tries > 1 && b < 200 * GiB);
    // pieces larger than what the device has left -- a one-piece window cannot shrink: out of memory,
    // after a bounded number of tries (it looped forever)
    CHECK(run(10, 128 * MiB + 256, 2 * GiB, 100 * MiB, &p, &tries, &b) == 1 && tries < 64);
    CHECK(run(3, 512 * MiB + 256, 0, 0, &p, &tries, &b) == 1 && tries < 64);
    CHECK(run(1, 1024 * MiB + 256, 4 * GiB, 0, &p, &tries, &b) == 1 && tries < 64);
    // small requests are not retried
    CHECK(run(4, MiB + 256, 64 * MiB, 0, &p, &tries, &b) == 1 && tries == 1);
    // every shape ends, and a success is within the capacity
    using U = uint64_t;
    for (U count : {U(1), U(7), U(255), U(4096), U(51200)})
        for (U stride : {U(320), MiB + 256, 4 * MiB + 256, 64 * MiB + 256, 300 * MiB + 256})
            for (U cap : {U(0), MiB, 100 * MiB, GiB, 64 * GiB})
                for (U budget : {U(0), 10 * MiB, GiB, 512 * GiB}) {
                    const int r = run(count, stride, budget, cap, &p, &tries, &b);
                    CHECK(r == 0 || r == 1);
                    if (r == 0) CHECK(p.bytes <= cap && p.bytes > 0 && (p.win ? p.win_n >= 1 : true));
                    CHECK(tries < 64);
                }
    // an error other than out of memory is not retried
    uint64_t failed = 0;
    int calls = 0;
    CHECK(tvi::allocate_payload(100, MiB, 256, GiB, [&](const PayloadPlan&, uint64_t) { calls++; return 2; }, &p, &b,
                                &failed) == 2 && calls == 1);
    if (failures) return 1;
    std::printf("ok\n");
    return 0;
}
