// dma_rows_probe.hip -- how fast row-sized host-to-device DMAs go when many threads queue them: T host threads, each
// with B reused page-locked buffers of `row` bytes, queue hipMemcpyAsync(row) into a 1 GiB device buffer on S shared
// streams (thread t on stream t % S), an event per buffer, each buffer reused after its event (as a reader that reads
// a row into its own buffer and DMAs it from there would).  No file I/O: the DMA-side ceiling of such a design.
//   build: hipcc --offload-arch=gfx950 -O2 tools/dma_rows_probe.hip -o dma_rows_probe
//   usage: dma_rows_probe THREADS ROW_BYTES STREAMS [BUFS_PER_THREAD=2] [TOTAL_GIB=16] [GROUP=1]
// GROUP > 1: each DMA is a 2D copy of GROUP rows from a GROUP x row buffer (fewer, larger submissions).
// Prints {"threads":..,"row":..,"streams":..,"gbps":..}.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const int T = atoi(argv[1]);
    const size_t row = strtoull(argv[2], nullptr, 10);
    const int S = atoi(argv[3]);
    const int B = argc > 4 ? atoi(argv[4]) : 2;
    const double gib = argc > 5 ? atof(argv[5]) : 16.0;
    const int G = argc > 6 ? atoi(argv[6]) : 1;
    if (T < 1 || S < 1 || B < 1 || G < 1 || row < 64) return 2;
    const size_t dev_bytes = 1ull << 30, pitch = row + 256;
    const size_t slots = dev_bytes / (pitch * G);
    const uint64_t total_rows = (uint64_t)(gib * (1ull << 30)) / row / G * G;
    CK(hipSetDevice(0));
    uint8_t* dev = nullptr;
    CK(hipMalloc((void**)&dev, dev_bytes));
    std::vector<hipStream_t> st(S);
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<std::vector<uint8_t*>> buf(T, std::vector<uint8_t*>(B));
    std::vector<std::vector<hipEvent_t>> ev(T, std::vector<hipEvent_t>(B));
    for (int t = 0; t < T; t++)
        for (int b = 0; b < B; b++) {
            CK(hipHostMalloc((void**)&buf[t][b], row * G, 0));
            for (size_t o = 0; o < row * G; o += 4096) buf[t][b][o] = (uint8_t)o;
            CK(hipEventCreateWithFlags(&ev[t][b], hipEventDisableTiming));
        }
    std::atomic<uint64_t> next{0};
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            std::vector<char> rec(B, 0);
            int k = 0;
            hipStream_t s = st[t % S];
            for (;;) {
                const uint64_t g = next.fetch_add(1);
                if (g * G >= total_rows) break;
                if (rec[k]) CK(hipEventSynchronize(ev[t][k]));
                uint8_t* d = dev + (g % slots) * pitch * G;
                if (G == 1)
                    CK(hipMemcpyAsync(d, buf[t][k], row, hipMemcpyHostToDevice, s));
                else
                    CK(hipMemcpy2DAsync(d, pitch, buf[t][k], row, row, G, hipMemcpyHostToDevice, s));
                CK(hipEventRecord(ev[t][k], s));
                rec[k] = 1;
                k = (k + 1) % B;
            }
        });
    for (auto& x : th) x.join();
    for (auto& s : st) CK(hipStreamSynchronize(s));
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"threads\": %d, \"row\": %zu, \"streams\": %d, \"bufs\": %d, \"group\": %d, \"gbps\": %.2f}\n", T, row, S,
           B, G, total_rows * row / sec / 1e9);
    return 0;
}
