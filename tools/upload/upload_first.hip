// The FIRST host -> device transfer of a process, as shadowtopo_create's edge upload is:
// a fresh 1.2 GB pageable source (C2's edge list), fresh device memory, one strategy per
// process (argv[1]: pageable | ring1 | ring2 | register).  Prints one JSON line.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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
    const std::string mode = argc > 1 ? argv[1] : "pageable";
    const size_t N = (size_t)1140 << 20;
    CK(hipFree(nullptr));
    char* src = (char*)malloc(N);
    memset(src, 1, N);
    void* dst = nullptr;
    CK(hipMalloc(&dst, N));
    double setup = 0, copy = 0;
    auto t0 = clk::now();
    if (mode == "pageable") {
        CK(hipMemcpy(dst, src, N, hipMemcpyHostToDevice));
        copy = ms(t0, clk::now());
    } else if (mode == "register") {
        CK(hipHostRegister(src, N, hipHostRegisterDefault));
        auto t1 = clk::now();
        CK(hipMemcpy(dst, src, N, hipMemcpyHostToDevice));
        setup = ms(t0, t1);
        copy = ms(t1, clk::now());
    } else {
        const int W = mode == "ring2" ? 2 : 1;
        constexpr size_t CH = (size_t)8 << 20;
        constexpr int NB = 4;
        void* buf[NB];
        hipEvent_t ev[NB];
        hipStream_t st;
        CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        for (int k = 0; k < NB; ++k) {
            CK(hipHostMalloc(&buf[k], CH, hipHostMallocDefault));
            CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
        }
        auto t1 = clk::now();
        const size_t nch = (N + CH - 1) / CH;
        std::atomic<size_t> ticket{0};
        auto work = [&](int w) {
            CK(hipSetDevice(0));
            for (size_t c = w; c < nch; c += W) {
                const int k = (int)(c % NB);
                if (c >= (size_t)NB) CK(hipEventSynchronize(ev[k]));
                const size_t o = c * CH, n = std::min(CH, N - o);
                memcpy(buf[k], src + o, n);
                while (ticket.load(std::memory_order_acquire) != c) std::this_thread::yield();
                CK(hipMemcpyAsync((char*)dst + o, buf[k], n, hipMemcpyHostToDevice, st));
                CK(hipEventRecord(ev[k], st));
                ticket.store(c + 1, std::memory_order_release);
            }
        };
        std::vector<std::thread> th;
        for (int w = 1; w < W; ++w) th.emplace_back(work, w);
        work(0);
        for (auto& t : th) t.join();
        CK(hipStreamSynchronize(st));
        setup = ms(t0, t1);
        copy = ms(t1, clk::now());
    }
    printf("{\"strategy\": \"first_%s\", \"bytes\": %zu, \"setup_ms\": %.2f, \"copy_ms\": %.2f, \"total_ms\": %.2f}\n",
           mode.c_str(), N, setup, copy, setup + copy);
    return 0;
}
