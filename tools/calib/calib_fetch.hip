// calib_fetch.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// shapes of the sparse relax kernels (k_relax / k_relax_wl in shadow_amd/csrc/engine.hip)
// against known byte counts.  MI355X_MICROARCH.md documents FETCH_SIZE = 1/2 of the bytes
// only for 16 B/lane streaming reads; every other width is uncalibrated there.
//
// Each kernel touches a table far larger than the 256 MB Infinity Cache exactly once, so
// every byte it asks for crosses the L2's memory side once.  Run it three times: plain
// (prints known bytes and HIP-event times), under `rocprofv3 --pmc FETCH_SIZE` and under
// `rocprofv3 --pmc WRITE_SIZE`; tools/calib/calib_summary.py divides.
//
//   shape        access per wave-instruction                      as in
//   stream16     16 B/lane, contiguous 1 KB                       the guide's reference case
//   rows8        8 B/lane, one 512-B row (64 sources x f64)       relax_visit's D row loads
//   rows4        4 B/lane, one 256-B row (64 sources x u32)       D32 / H rows
//   lanes8       8 B/lane, every lane its own row (lane column)   finish_vertex's pred H/R gathers
//   store8       8 B/lane stores, one 512-B row                   finish_vertex's state stores
//   bytes1       1-B stores at scattered vertices                 activation flags
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                            \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int64_t ROWS = 4 << 20;  // 4 Mi rows
constexpr int RIF = 8;             // rows in flight per wave (relax_visit's chunk of 8 arcs)

__global__ __launch_bounds__(256) void k_stream16(const float4* __restrict__ t, int64_t n, float* __restrict__ sink) {
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = t[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == -1.f) sink[threadIdx.x] = acc;
}

// 8 rows per wave, all loads in flight before the first use (relax_visit's shape)
__global__ __launch_bounds__(256) void k_rows8(const double* __restrict__ t, const int32_t* __restrict__ perm,
                                               int64_t nrows, double* __restrict__ sink) {
    const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (w * RIF >= nrows) return;
    int32_t r[RIF];
    double v[RIF];
#pragma unroll
    for (int k = 0; k < RIF; ++k) r[k] = __builtin_amdgcn_readfirstlane(perm[w * RIF + k]);
#pragma unroll
    for (int k = 0; k < RIF; ++k) v[k] = t[(size_t)r[k] * 64 + lane];
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < RIF; ++k) acc += v[k];
    if (acc == -1.0) sink[lane] = acc;
}

__global__ __launch_bounds__(256) void k_rows4(const uint32_t* __restrict__ t, const int32_t* __restrict__ perm,
                                               int64_t nrows, uint32_t* __restrict__ sink) {
    const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (w * RIF >= nrows) return;
    int32_t r[RIF];
    uint32_t v[RIF];
#pragma unroll
    for (int k = 0; k < RIF; ++k) r[k] = __builtin_amdgcn_readfirstlane(perm[w * RIF + k]);
#pragma unroll
    for (int k = 0; k < RIF; ++k) v[k] = t[(size_t)r[k] * 64 + lane];
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < RIF; ++k) acc ^= v[k];
    if (acc == 0xdeadbeefu) sink[lane] = acc;
}

// every lane reads its own column of a row of its own: one 8-byte word per 512-B row, the
// rows a permutation so that every (row, lane) word is read once over the launch
__global__ __launch_bounds__(256) void k_lanes8(const double* __restrict__ t, const int32_t* __restrict__ perm,
                                                int64_t nrows, double* __restrict__ sink) {
    const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (w * RIF >= nrows) return;
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < RIF; ++k) {
        // lane l of wave w, step k reads word l of row perm[(w*RIF + k + l*stride) mod nrows]:
        // over the launch row i's word l is read once (a bijection per lane)
        const int64_t j = (w * RIF + k + (int64_t)lane * (nrows / 64)) % nrows;
        acc += t[(size_t)perm[j] * 64 + lane];
    }
    if (acc == -1.0) sink[lane] = acc;
}

__global__ __launch_bounds__(256) void k_store8(double* __restrict__ t, const int32_t* __restrict__ perm, int64_t nrows) {
    const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (w * RIF >= nrows) return;
#pragma unroll
    for (int k = 0; k < RIF; ++k) {
        const int32_t r = __builtin_amdgcn_readfirstlane(perm[w * RIF + k]);
        t[(size_t)r * 64 + lane] = (double)(r + lane);
    }
}

// 1-byte flag stores: each lane one byte at a scattered position of a table of `n` bytes
__global__ __launch_bounds__(256) void k_bytes1(uint8_t* __restrict__ t, const int32_t* __restrict__ perm, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    t[perm[i]] = 1;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    const size_t row8 = 512, row4 = 256;
    double* t8 = nullptr;
    uint32_t* t4 = nullptr;
    float4* ts = nullptr;
    int32_t* perm = nullptr;
    double* sink = nullptr;
    CK(hipMalloc(&t8, ROWS * row8));
    CK(hipMalloc(&t4, ROWS * row4));
    CK(hipMalloc(&perm, ROWS * sizeof(int32_t)));
    CK(hipMalloc(&sink, 4096));
    ts = reinterpret_cast<float4*>(t8);
    CK(hipMemset(t8, 0, ROWS * row8));
    CK(hipMemset(t4, 0, ROWS * row4));
    std::vector<int32_t> h(ROWS);
    for (int64_t i = 0; i < ROWS; ++i) h[i] = (int32_t)i;
    uint64_t x = 88172645463325252ull;
    for (int64_t i = ROWS - 1; i > 0; --i) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        std::swap(h[i], h[x % (uint64_t)(i + 1)]);
    }
    CK(hipMemcpy(perm, h.data(), ROWS * sizeof(int32_t), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // a 1 GB write between kernels evicts the Infinity Cache
    uint8_t* flush = nullptr;
    CK(hipMalloc(&flush, (size_t)1 << 30));
    auto evict = [&]() { CK(hipMemsetAsync(flush, reps, (size_t)1 << 30, 0)); };
    const int64_t waves = ROWS / RIF;
    const dim3 gw((uint32_t)(waves * 64 / 256)), blk(256);
    const int64_t nbytes_flags = ROWS;  // 4 MB flag table, one store per byte
    printf("{\"rows\": %lld, \"rows_in_flight\": %d, \"kernels\": [\n", (long long)ROWS, RIF);
    for (int r = 0; r < reps; ++r) {
        struct K {
            const char* name;
            double bytes;
            const char* dir;
        };
        const K ks[] = {{"k_stream16", (double)ROWS * row8, "read"},
                        {"k_rows8", (double)ROWS * row8, "read"},
                        {"k_rows4", (double)ROWS * row4, "read"},
                        {"k_lanes8", (double)ROWS * row8, "read"},
                        {"k_store8", (double)ROWS * row8, "write"},
                        {"k_bytes1", (double)nbytes_flags, "write"}};
        for (int k = 0; k < 6; ++k) {
            evict();
            CK(hipEventRecord(a, 0));
            switch (k) {
                case 0: hipLaunchKernelGGL(k_stream16, dim3(8192), blk, 0, 0, ts, (int64_t)(ROWS * row8 / 16), (float*)sink); break;
                case 1: hipLaunchKernelGGL(k_rows8, gw, blk, 0, 0, t8, perm, ROWS, sink); break;
                case 2: hipLaunchKernelGGL(k_rows4, gw, blk, 0, 0, t4, perm, ROWS, (uint32_t*)sink); break;
                case 3: hipLaunchKernelGGL(k_lanes8, gw, blk, 0, 0, t8, perm, ROWS, sink); break;
                case 4: hipLaunchKernelGGL(k_store8, gw, blk, 0, 0, t8, perm, ROWS); break;
                case 5: hipLaunchKernelGGL(k_bytes1, dim3((uint32_t)(nbytes_flags / 256)), blk, 0, 0, (uint8_t*)t4, perm, nbytes_flags); break;
            }
            CK(hipGetLastError());
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("  {\"rep\": %d, \"kernel\": \"%s\", \"dir\": \"%s\", \"known_bytes\": %.0f, \"index_bytes\": %lld, \"ms\": %.4f, \"GBps\": %.1f}%s\n",
                   r, ks[k].name, ks[k].dir, ks[k].bytes, (long long)(k == 0 ? 0 : ROWS * 4), ms, ks[k].bytes / ms / 1e6,
                   (r == reps - 1 && k == 5) ? "" : ",");
        }
    }
    printf("]}\n");
    CK(hipDeviceSynchronize());
    return 0;
}
