// Host -> device upload strategies for shadowtopo_create's edge list (cold
// start): a 1.14 GB pageable source (C2's 47.5 M edges x 24 B) into device memory.
// Prints one JSON line per strategy: ms for setup (allocation / registration), copy, teardown.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <thread>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

int main(int argc, char** argv) {
    const size_t N = argc > 1 ? strtoull(argv[1], nullptr, 10) : (size_t)1140 << 20;
    char* src = (char*)malloc(N);
    for (size_t i = 0; i < N; i += 4096) src[i] = (char)i;  // fault the pages in
    memset(src, 1, N);
    CK(hipFree(nullptr));  // runtime initialised before anything is timed
    void* dst = nullptr;
    {  // first touch of fresh device memory: by the copy's DMA, or by a memset kernel first
        // (three buffers held at once, so none reuses another's pages); the source is warm
        // (pinned by a first copy) so only the device side differs
        void *d0 = nullptr, *d1 = nullptr, *d2 = nullptr;
        CK(hipMalloc(&d0, N));
        CK(hipMemcpy(d0, src, N, hipMemcpyHostToDevice));  // warms the source (and d0)
        auto t0 = clk::now();
        CK(hipMemcpy(d0, src, N, hipMemcpyHostToDevice));
        auto t1 = clk::now();
        CK(hipMalloc(&d1, N));
        auto t2 = clk::now();
        CK(hipMemcpy(d1, src, N, hipMemcpyHostToDevice));
        auto t3 = clk::now();
        CK(hipMalloc(&d2, N));
        auto t4 = clk::now();
        CK(hipMemset(d2, 0, N));
        CK(hipDeviceSynchronize());
        auto t5 = clk::now();
        CK(hipMemcpy(d2, src, N, hipMemcpyHostToDevice));
        auto t6 = clk::now();
        printf("{\"strategy\": \"device_first_touch\", \"bytes\": %zu, \"warm_copy_ms\": %.2f, \"fresh_dma_copy_ms\": %.2f, "
               "\"fresh_memset_ms\": %.2f, \"copy_after_memset_ms\": %.2f}\n", N, ms(t0, t1), ms(t2, t3), ms(t4, t5), ms(t5, t6));
        CK(hipFree(d0));
        CK(hipFree(d1));
        CK(hipFree(d2));
        void* hsrc = nullptr;
        auto t7 = clk::now();
        CK(hipHostMalloc(&hsrc, (size_t)32 << 20, hipHostMallocDefault));
        auto t8 = clk::now();
        printf("{\"strategy\": \"hipHostMalloc_32MB\", \"ms\": %.2f}\n", ms(t7, t8));
        CK(hipHostFree(hsrc));
        char* src2 = (char*)malloc(N);  // a fresh source, as the first copy of a new edge list sees
        memset(src2, 2, N);
        free(src);
        src = src2;
    }
    CK(hipMalloc(&dst, N));
    CK(hipMemset(dst, 0, N));
    CK(hipDeviceSynchronize());
    auto report = [&](const char* name, double setup, double copy, double teardown) {
        printf("{\"strategy\": \"%s\", \"bytes\": %zu, \"setup_ms\": %.2f, \"copy_ms\": %.2f, \"teardown_ms\": %.2f, "
               "\"total_ms\": %.2f, \"copy_GBps\": %.1f}\n",
               name, N, setup, copy, teardown, setup + copy + teardown, N / copy / 1e6);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        {  // 1. plain hipMemcpy from pageable memory
            auto t0 = clk::now();
            CK(hipMemcpy(dst, src, N, hipMemcpyHostToDevice));
            auto t1 = clk::now();
            report("pageable_hipMemcpy", 0, ms(t0, t1), 0);
        }
        {  // 2. register the source in place, copy, unregister
            auto t0 = clk::now();
            CK(hipHostRegister(src, N, hipHostRegisterDefault));
            auto t1 = clk::now();
            CK(hipMemcpy(dst, src, N, hipMemcpyHostToDevice));
            auto t2 = clk::now();
            CK(hipHostUnregister(src));
            auto t3 = clk::now();
            report("hostRegister", ms(t0, t1), ms(t1, t2), ms(t2, t3));
        }
        for (int W : {1, 2, 4, 8}) {  // 3. pinned staging ring, W threads filling it, one stream
            constexpr size_t CH = (size_t)8 << 20;
            const int NB = 2 * W;
            auto t0 = clk::now();
            std::vector<void*> buf(NB);
            std::vector<hipEvent_t> ev(NB);
            hipStream_t st;
            CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            for (int k = 0; k < NB; ++k) {
                CK(hipHostMalloc(&buf[k], CH, hipHostMallocDefault));
                CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
            }
            auto t1 = clk::now();
            // chunk c -> buffer c % NB; thread w fills chunks w, w + W, ...; the copy of chunk c
            // is issued by its filler on the shared stream in chunk order (a ticket)
            const size_t nch = (N + CH - 1) / CH;
            std::vector<std::thread> th;
            std::atomic<size_t> ticket{0};
            std::vector<char> used(NB, 0);
            auto work = [&](int w) {
                CK(hipSetDevice(0));
                for (size_t c = w; c < nch; c += W) {
                    const int k = (int)(c % NB);
                    if (c >= (size_t)NB) CK(hipEventSynchronize(ev[k]));  // recorded for chunk c - NB
                    const size_t o = c * CH, n = std::min(CH, N - o);
                    memcpy(buf[k], src + o, n);
                    while (ticket.load(std::memory_order_acquire) != c) std::this_thread::yield();
                    CK(hipMemcpyAsync((char*)dst + o, buf[k], n, hipMemcpyHostToDevice, st));
                    CK(hipEventRecord(ev[k], st));
                    ticket.store(c + 1, std::memory_order_release);
                }
            };
            for (int w = 1; w < W; ++w) th.emplace_back(work, w);
            work(0);
            for (auto& t : th) t.join();
            CK(hipStreamSynchronize(st));
            auto t2 = clk::now();
            for (int k = 0; k < NB; ++k) {
                CK(hipHostFree(buf[k]));
                CK(hipEventDestroy(ev[k]));
            }
            CK(hipStreamDestroy(st));
            auto t3 = clk::now();
            char name[64];
            snprintf(name, sizeof name, "staged_ring_W%d", W);
            report(name, ms(t0, t1), ms(t1, t2), ms(t2, t3));
        }
        for (int W : {2, 4, 8}) {  // 4. W threads, each hipMemcpyAsync of its pageable slice on its stream
            auto t0 = clk::now();
            std::vector<hipStream_t> sts(W);
            for (auto& s : sts) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            auto t1 = clk::now();
            std::vector<std::thread> th;
            for (int w = 0; w < W; ++w)
                th.emplace_back([&, w] {
                    CK(hipSetDevice(0));
                    const size_t a = N * w / W, z = N * (w + 1) / W;
                    CK(hipMemcpyAsync((char*)dst + a, src + a, z - a, hipMemcpyHostToDevice, sts[w]));
                    CK(hipStreamSynchronize(sts[w]));
                });
            for (auto& t : th) t.join();
            auto t2 = clk::now();
            for (auto& s : sts) CK(hipStreamDestroy(s));
            auto t3 = clk::now();
            char name[64];
            snprintf(name, sizeof name, "pageable_parallel_W%d", W);
            report(name, ms(t0, t1), ms(t1, t2), ms(t2, t3));
        }
    }
    return 0;
}
