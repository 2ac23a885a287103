// mix_probe: diagnostics of the MIX work-queue launch (tv_launch_mix) outside the library.
// Runs one hash-mode MIX launch over P synthetic pieces with a per-unit trace, checks its digests against
// the lane kernel's, and prints the unit timeline: per worker kind the unit durations and the waits.
// Build (tools/build_mix_probe.sh): hipcc links it with torrent_amd/csrc/tv_kernels.hip.o.
// usage: mix_probe L P last_len [pair_wgs pair_lds_bufs lane_wgs lane_waves_per_wg lane_lds seg_blocks verify
//                                 cumask [trace.csv]]
// cumask: 0 none; 1 pairs on the low half of the CU mask bits, lanes on the high half; 2 pairs on even
// bits, lanes on odd bits; 3 pairs on bits with (i / 4) even (CU quads), lanes on the others.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../torrent_amd/csrc/tv_internal.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); exit(2); } } while (0)

// Clock sampler: one wave per workgroup records (s_memtime, s_memrealtime) every ~0.5 ms for `ms`
// milliseconds of wall time, then exits (the exit condition is wall time only, so every wave reaches it).
__global__ __launch_bounds__(64) void clock_kernel(uint64_t* out, uint32_t samples, uint32_t ms) {
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t k = 0;
    for (;;) {
        const uint64_t t = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime();
        if (k < samples && threadIdx.x == 0) {
            out[2ull * (blockIdx.x * samples + k)] = t;
            out[2ull * (blockIdx.x * samples + k) + 1] = r;
        }
        k++;
        if (r - r0 > 100000ull * ms) break;
        for (int i = 0; i < 6; i++) __builtin_amdgcn_s_sleep(127);   // ~50k cycles
    }
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: mix_probe L P last_len [pair_wgs pair_lds_bufs lane_wgs lane_waves_per_wg lane_lds "
                        "seg_blocks verify cumask [trace.csv]]\n");
        return 1;
    }
    const uint64_t L = strtoull(argv[1], 0, 0), P = strtoull(argv[2], 0, 0), last = strtoull(argv[3], 0, 0);
    TvMixShape m{};
    m.pair_wgs = argc > 4 ? atoi(argv[4]) : 256;
    m.pair_lds_bufs = argc > 5 ? atoi(argv[5]) : 5;
    m.lane_wgs = argc > 6 ? atoi(argv[6]) : 256;
    m.lane_waves_per_wg = argc > 7 ? atoi(argv[7]) : 2;
    m.lane_lds = argc > 8 ? atoi(argv[8]) : 0;
    const uint32_t seg_blocks = argc > 9 ? atoi(argv[9]) : 1024;
    const bool verify = argc > 10 ? atoi(argv[10]) != 0 : false;
    const int cumask = argc > 11 ? atoi(argv[11]) : 0;
    const char* csv = argc > 12 ? argv[12] : nullptr;
    if (!L || !P || !last || last > L || P > (1u << 30)) { fprintf(stderr, "bad geometry\n"); return 1; }
    const uint64_t stride = (L + 63) / 64 * 64 + 256;
    uint8_t* data;
    CK(hipMalloc((void**)&data, stride * P + 4096));
    hipStream_t sa, sb, sp = nullptr, sl = nullptr;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    if (cumask) {
        std::vector<uint32_t> ma((cus + 31) / 32, 0), mb((cus + 31) / 32, 0);
        for (int i = 0; i < cus; i++) {
            const bool pair = cumask == 1 ? i < cus / 2 : cumask == 2 ? (i % 2 == 0) : ((i / 4) % 2 == 0);
            (pair ? ma : mb)[i / 32] |= 1u << (i % 32);
        }
        CK(hipExtStreamCreateWithCUMask(&sp, (uint32_t)ma.size(), ma.data()));
        CK(hipExtStreamCreateWithCUMask(&sl, (uint32_t)mb.size(), mb.data()));
    }
    CK(tv_launch_fill(data, stride, 0, (uint32_t)P, L, 7, sa));
    uint32_t *state, *dig, *outd, *outd_lane, *qbuf;
    uint64_t *out64, *trace;
    CK(hipMalloc((void**)&state, 20 * P));
    CK(hipMalloc((void**)&dig, 20 * P));
    CK(hipMalloc((void**)&outd, 20 * P));
    CK(hipMalloc((void**)&outd_lane, 20 * P));
    CK(hipMalloc((void**)&out64, ((P + 255) / 256) * 32));
    TvPieces p{};
    p.data = data; p.stride = stride; p.L = L; p.last_len = last;
    p.blk_end = UINT64_MAX; p.n = (uint32_t)P; p.n_main = last < L ? (uint32_t)P - 1 : (uint32_t)P;
    p.last_idx = (uint32_t)P - 1; p.finalize = 1; p.dcount = (uint32_t)P;
    p.state = state; p.digests = dig; p.out64 = out64;
    TvQueue q{};
    q.groups = (p.n_main + 63) / 64 + (p.n_main < p.n ? 1 : 0);
    q.seg_blocks = seg_blocks;
    q.segs = (uint32_t)((((L + 8) / 64 + 1) + seg_blocks - 1) / seg_blocks);
    const uint64_t units = (uint64_t)q.groups * q.segs;
    q.units = (uint32_t)units;
    q.ring = q.groups;
    const uint64_t qbytes = 16 + 8ull * q.ring;
    CK(hipMalloc((void**)&qbuf, qbytes));
    CK(hipMalloc((void**)&trace, units * 32));
    q.head = qbuf; q.tail = qbuf + 1; q.error = qbuf + 2; q.slots = reinterpret_cast<uint64_t*>(qbuf + 4);
    q.trace = trace;

    // reference: the lane kernel in hash mode
    p.out_digests = outd_lane;
    CK(tv_launch_verify(p, TV_KERNEL_LANE, true, sa));
    hipEvent_t e0, e1, ej;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
    CK(hipEventRecord(e0, sa));
    CK(tv_launch_verify(p, TV_KERNEL_LANE, true, sa));
    CK(hipEventRecord(e1, sa));
    CK(hipStreamSynchronize(sa));
    float lane_ms = 0;
    CK(hipEventElapsedTime(&lane_ms, e0, e1));

    // lane-kernel verify of the same launch, timed (digests all zero: every bit 0, same work), with the
    // shader clock sampled beside it on a third stream (8 one-wave workgroups, mostly asleep)
    float lane_verify_ms = 0;
    const uint32_t csamples = 4096, cwgs = 8;
    uint64_t* cbuf;
    CK(hipMalloc((void**)&cbuf, 16ull * csamples * cwgs));
    CK(hipMemset(cbuf, 0, 16ull * csamples * cwgs));
    hipStream_t sc;
    CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
    const uint32_t cms = (uint32_t)std::min<double>(1500.0, lane_ms * 1.5 + 20);
    hipLaunchKernelGGL(clock_kernel, dim3(cwgs), dim3(64), 0, sc, cbuf, csamples, cms);
    CK(hipGetLastError());
    CK(hipEventRecord(e0, sa));
    CK(tv_launch_verify(p, TV_KERNEL_LANE, false, sa));
    CK(hipEventRecord(e1, sa));
    CK(hipStreamSynchronize(sa));
    CK(hipStreamSynchronize(sc));
    CK(hipEventElapsedTime(&lane_verify_ms, e0, e1));
    {
        std::vector<uint64_t> cb(2ull * csamples * cwgs);
        CK(hipMemcpy(cb.data(), cbuf, cb.size() * 8, hipMemcpyDeviceToHost));
        // per workgroup: clock over successive ~10 ms windows; print min / median / max over windows
        std::vector<double> mhz;
        for (uint32_t w = 0; w < cwgs; w++) {
            const uint64_t* c = cb.data() + 2ull * w * csamples;
            uint32_t i = 0;
            while (i + 1 < csamples && c[2 * (i + 1) + 1]) {
                uint32_t j = i + 1;
                while (j + 1 < csamples && c[2 * (j + 1) + 1] && c[2 * j + 1] - c[2 * i + 1] < 1000000) j++;
                if (c[2 * j + 1] - c[2 * i + 1] >= 500000) {
                    mhz.push_back((double)(c[2 * j] - c[2 * i]) / (double)(c[2 * j + 1] - c[2 * i + 1]) * 100.0);
                    if (w == 0) printf("  clock t=%.1f..%.1f ms %.0f MHz\n", (c[2 * i + 1] - c[1]) / 1e5,
                                       (c[2 * j + 1] - c[1]) / 1e5, mhz.back());
                }
                i = j;
            }
        }
        std::sort(mhz.begin(), mhz.end());
        if (!mhz.empty())
            printf("shader clock over ~10 ms windows during the lane verify (+ idle tail): min %.0f med %.0f max %.0f MHz (%zu)\n",
                   mhz.front(), mhz[mhz.size() / 2], mhz.back(), mhz.size());
    }

    p.out_digests = outd;
    CK(hipMemsetAsync(out64, 0, ((P + 255) / 256) * 32, sa));
    CK(hipMemsetAsync(qbuf, 0, qbytes, sa));
    CK(hipMemsetAsync(trace, 0, units * 32, sa));
    CK(hipEventRecord(e0, sa));
    CK(hipStreamWaitEvent(sb, e0, 0));
    if (cumask) {
        CK(hipStreamWaitEvent(sp, e0, 0));
        CK(hipStreamWaitEvent(sl, e0, 0));
        CK(tv_launch_mix(p, q, !verify, sp, sl, m));
        CK(hipEventRecord(ej, sp));
        CK(hipStreamWaitEvent(sb, ej, 0));
        CK(hipEventRecord(ej, sl));
        CK(hipStreamWaitEvent(sb, ej, 0));
    } else {
        CK(tv_launch_mix(p, q, !verify, sa, sb, m));
    }
    CK(hipEventRecord(ej, sb));
    CK(hipStreamWaitEvent(sa, ej, 0));
    CK(hipEventRecord(e1, sa));
    CK(hipStreamSynchronize(sa));
    float mix_ms = 0;
    CK(hipEventElapsedTime(&mix_ms, e0, e1));

    uint32_t hq[3];
    CK(hipMemcpy(hq, qbuf, 12, hipMemcpyDeviceToHost));
    std::vector<uint32_t> a(5 * P), b(5 * P);
    CK(hipMemcpy(a.data(), outd, 20 * P, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), outd_lane, 20 * P, hipMemcpyDeviceToHost));
    std::vector<uint64_t> t(4 * units);
    CK(hipMemcpy(t.data(), trace, units * 32, hipMemcpyDeviceToHost));
    uint64_t mism = 0;
    if (!verify)
        for (uint64_t i = 0; i < 5 * P; i++) mism += a[i] != b[i];
    std::vector<uint64_t> bits((P + 255) / 256 * 4);
    CK(hipMemcpy(bits.data(), out64, bits.size() * 8, hipMemcpyDeviceToHost));
    uint64_t ones = 0;
    for (uint64_t w : bits) ones += __builtin_popcountll(w);

    uint64_t tmin = UINT64_MAX, tmax = 0, done = 0;
    for (uint64_t u = 0; u < units; u++)
        if (t[4 * u + 2]) { tmin = std::min(tmin, t[4 * u]); tmax = std::max(tmax, t[4 * u + 2]); done++; }
    std::vector<double> dur[2], wait[2];
    for (uint64_t u = 0; u < units; u++) {
        if (!t[4 * u + 2]) continue;
        const int k = t[4 * u + 3] >= 0x10000 ? 1 : 0;
        dur[k].push_back((t[4 * u + 2] - t[4 * u + 1]) / 100.0);   // us (100 MHz ticks)
        wait[k].push_back((t[4 * u + 1] - t[4 * u + 0]) / 100.0);
    }
    printf("L=%llu P=%llu last=%llu groups=%u segs=%u units=%llu pairs=%u (lds bufs %u) lane_wgs=%u x %u waves "
           "lds=%u seg_blocks=%u mode=%s cumask=%d cus=%d\n",
           (unsigned long long)L, (unsigned long long)P, (unsigned long long)last, q.groups, q.segs,
           (unsigned long long)units, m.pair_wgs, m.pair_lds_bufs, m.lane_wgs, m.lane_waves_per_wg, m.lane_lds,
           seg_blocks, verify ? "verify" : "hash", cumask, cus);
    const uint64_t bytes = L * (P - 1) + last;
    printf("lane hash %.3f ms (%.1f GB/s) verify %.3f ms (%.1f GB/s); mix %.3f ms (%.1f GB/s); error=%u "
           "pops=%u pushes=%u done=%llu digest_mismatch_words=%llu bits_set=%llu trace_span=%.3f ms\n",
           lane_ms, bytes / (lane_ms * 1e6), lane_verify_ms, bytes / (lane_verify_ms * 1e6), mix_ms,
           bytes / (mix_ms * 1e6), hq[2], hq[0], hq[1], (unsigned long long)done, (unsigned long long)mism,
           (unsigned long long)ones, done ? (tmax - tmin) / 1e5 : 0.0);
    const char* kind[2] = {"pair", "lane"};
    for (int k = 0; k < 2; k++) {
        if (dur[k].empty()) continue;
        std::sort(dur[k].begin(), dur[k].end());
        std::sort(wait[k].begin(), wait[k].end());
        const size_t n = dur[k].size();
        printf("%s units=%zu dur_us min/med/p99/max %.1f %.1f %.1f %.1f  wait_us med/p99/max %.1f %.1f %.1f\n",
               kind[k], n, dur[k][0], dur[k][n / 2], dur[k][n * 99 / 100], dur[k][n - 1], wait[k][n / 2],
               wait[k][n * 99 / 100], wait[k][n - 1]);
    }
    if (csv) {
        FILE* f = fopen(csv, "w");
        if (f) {
            fprintf(f, "unit,seg,group,claim_us,start_us,end_us,worker\n");
            for (uint64_t u = 0; u < units; u++)
                if (t[4 * u + 2])
                    fprintf(f, "%llu,%llu,%llu,%.2f,%.2f,%.2f,%llu\n", (unsigned long long)u,
                            (unsigned long long)(u / q.groups), (unsigned long long)(u % q.groups),
                            (t[4 * u] - tmin) / 100.0, (t[4 * u + 1] - tmin) / 100.0, (t[4 * u + 2] - tmin) / 100.0,
                            (unsigned long long)t[4 * u + 3]);
            fclose(f);
        }
    }
    return (mism || hq[2] || ones || done != units) ? 3 : 0;
}
