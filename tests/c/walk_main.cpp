// walk_main.cpp -- runs tv_plan.h's walk_file_table (tv_stage_file_table's Storage.get walk) on the CPU for
// tests/test_plan.py: stdin "n lo hi L" then n file lengths; stdout one "file file_offset linear len" line per
// segment, then "reached <offset>"; or "overflow <file>".  Built with g++ (no HIP).
#include <cstdio>
#include <vector>

#include "../../torrent_amd/csrc/tv_plan.h"

int main() {
    unsigned long long n = 0, lo = 0, hi = 0, L = 0;
    if (std::scanf("%llu %llu %llu %llu", &n, &lo, &hi, &L) != 4) return 2;
    std::vector<uint64_t> lengths(n);
    for (auto& v : lengths) {
        unsigned long long x = 0;
        if (std::scanf("%llu", &x) != 1) return 2;
        v = x;
    }
    std::vector<tvi::TableSeg> segs;
    uint64_t bad = 0, reached = 0;
    if (!tvi::walk_file_table(n, lengths.data(), lo, hi, L, &segs, &bad, &reached)) {
        std::printf("overflow %llu\n", (unsigned long long)bad);
        return 0;
    }
    for (const auto& g : segs)
        std::printf("%llu %llu %llu %llu\n", (unsigned long long)g.file, (unsigned long long)g.file_offset,
                    (unsigned long long)g.linear, (unsigned long long)g.len);
    std::printf("reached %llu\n", (unsigned long long)reached);
    return 0;
}
