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
    // a stream's geometry under a device budget (stream_geometry: tv_stream_file_table, tv_verify_host)
    {
        const uint64_t slot = 64 * MiB, slack = 256, KiB = 1024;
        uint64_t col = 0, win = 0;
        auto geo = [&](uint64_t L, uint64_t count, uint64_t budget, uint64_t min_win) {
            tvi::stream_geometry(L, count, budget, min_win, slot, slack, &col, &win);
        };
        geo(MiB, 16384, GiB / 2, 2048);   // cfg2 at 0.5 GiB: 124 KiB rows, 9 columns
        CHECK(col == 124 * KiB && win == 2048);
        geo(MiB, 16384, 2 * GiB, 2048);   // each chunk buffer at most 256 MiB: the same geometry
        CHECK(col == 124 * KiB && win == 2048);
        geo(MiB, 16384, GiB / 4, 2048);   // 0.25 GiB: 60 KiB
        CHECK(col == 60 * KiB && win == 2048);
        geo(MiB, 16384, GiB, 512);        // a cold shard's 512-piece windows: 4 x longer rows
        CHECK(col == 508 * KiB && win == 512);
        geo(4096, 5000, GiB, 2048);       // whole pieces fit: one window of the shard
        CHECK(col == 4096 && win == 5000);
        geo(4096, 5000, 2 * (2048 * (1024 + 256) + 256), 2048);   // tests/test_gpu_fuzz.py: 3 windows x 4 columns
        CHECK(col == 1024 && win == 2048);
        geo(4096, 5000, 1, 2048);         // no room: 64-byte columns
        CHECK(col == 64 && win == 2048);
        geo(MiB, 160, 2 * (160 * (256 * KiB + 256) + 256), 64);   // tests/test_gpu_cold.py: 640 KiB, 2 columns
        CHECK(col == 640 * KiB && win == 64);
        geo(1 << 30, 3, GiB, 2048);       // a piece larger than a ring slot: rows of one slot
        CHECK(col == slot && win == 3);
        // invariants over a sweep: columns a multiple of 64 (of 4 KiB from 4 KiB up) within a slot and the piece,
        // windows a multiple of 64 or the whole shard, both chunk buffers within the budget whenever it has room
        uint64_t seed = 1;
        for (int t = 0; t < 20000; t++) {
            seed = seed * 6364136223846793005ull + 1442695040888963407ull;
            const uint64_t L = 1 + (seed >> 33) % (96 * MiB), count = 1 + (seed >> 13) % 70000;
            const uint64_t budget = (seed >> 7) % (8 * GiB), mw = (t & 1) ? 2048 : 512;
            geo(L, count, budget, mw);
            const uint64_t lpad = std::min<uint64_t>((L + 63) / 64 * 64, slot);
            CHECK(col >= 64 && col % 64 == 0 && col <= lpad && (col < 4096 || col % 4096 == 0 || col == lpad));
            CHECK(win >= 1 && win <= count && (win == count || win % 64 == 0));
            if (col > 64)
                CHECK((col + 256) * win + slack <= std::min<uint64_t>(budget / 2, tvi::kStreamChunkMax));
        }
    }
    if (failures) return 1;
    std::printf("ok\n");
    return 0;
}
