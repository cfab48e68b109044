// graph_build.hip -- the engine's resident graph, built on the GPU (see graph_build.h).
//
// What it restates (reference: /root/reference/src/main/routing/topology.c and igraph's
// storage):
//  * igraph edge storage: undirected edges keep from = max(u, v), to = min(u, v);
//  * the relaxation in-CSR: non-loop arcs u -> v sorted by (v, u, eid), parallel arcs merged
//    to their minimum latency, reliability and id of the lowest-id edge (get_eid,
//    topology.c:401-444), a multigraph flag when that edge is not the minimum;
//  * igraph_incident(OUT) order (topology.c:495, :1559): edges with from == v by (to, eid),
//    then, undirected, edges with to == v by (from, eid) -- a self-loop twice;
//  * _topology_isComplete (topology.c:450-552): every vertex has >= V incident edges
//    (undirected: one less when it has a self-loop).
// Every sort is hipCUB's stable LSD radix sort over 64-bit (primary << 32 | secondary) keys
// with the edge or arc index as the value, so ties keep edge-id order exactly as the
// host's counting sorts did; tables are then filled by segment-boundary kernels.
#include "graph_build.h"

#include <hipcub/hipcub.hpp>

#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <limits>

namespace graph_build {
namespace {

#define GB_TRY(expr)                      \
    do {                                  \
        hipError_t e_ = (expr);           \
        if (e_ != hipSuccess) return e_;  \
    } while (0)

template <typename T>
hipError_t dalloc(std::vector<void*>& owner, T** p, size_t n) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, (n ? n : 1) * sizeof(T));
    if (e != hipSuccess) return e;
    owner.push_back(q);
    *p = static_cast<T*>(q);
    return hipSuccess;
}

// the build's scratch allocations, recorded in the caller's list (it frees them)
struct Scratch {
    std::vector<void*>& v;
};

inline unsigned grid_of(int64_t n, int bs = 256) {
    const int64_t b = (n + bs - 1) / bs;
    return (unsigned)(b < 1 ? 1 : (b > 1048576 ? 1048576 : b));
}

int bitlen(uint64_t x) {
    int b = 0;
    while (x) {
        ++b;
        x >>= 1;
    }
    return b;
}

// igraph storage, 1 - loss, the lowest self-loop, and the relaxation arcs (key v << 32 | u,
// value eid); a loop's arcs get the sentinel head V, which sorts them past every real arc
// in place: efrom / eto / erel may be src / dst / loss themselves (each element is read, then
// written, by the same thread)
__global__ void k_edges(int64_t E, int32_t V, int directed, const int32_t* src, const int32_t* dst,
                        const double* loss, int32_t* efrom, int32_t* eto, double* erel, int32_t* loop_min,
                        uint64_t* akey, int32_t* aval) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t a = src[e], b = dst[e];
        int32_t f = a, t = b;
        if (!directed && a < b) {
            f = b;
            t = a;
        }
        efrom[e] = f;
        eto[e] = t;
        erel[e] = 1.0 - loss[e];
        const bool loop = f == t;
        if (loop) atomicMin(&loop_min[f], (int32_t)e);
        const uint64_t sentinel = (uint64_t)V << 32;
        if (directed) {
            akey[e] = loop ? sentinel : ((uint64_t)t << 32 | (uint32_t)f);
            aval[e] = (int32_t)e;
        } else {
            akey[2 * e] = loop ? sentinel : ((uint64_t)t << 32 | (uint32_t)f);
            akey[2 * e + 1] = loop ? sentinel : ((uint64_t)f << 32 | (uint32_t)t);
            aval[2 * e] = (int32_t)e;
            aval[2 * e + 1] = (int32_t)e;
        }
    }
}

__global__ void k_loop_fix(int32_t V, int32_t* loop_eid) {
    for (int32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < V; v += gridDim.x * blockDim.x)
        if (loop_eid[v] == INT_MAX) loop_eid[v] = -1;
}

// run heads of the sorted arc keys
__global__ void k_heads(int64_t n, const uint64_t* __restrict__ key, int32_t* head) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        head[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}

// one merged arc per run: minimum latency, the lowest-id (first, stable order) edge's
// reliability and id (topology.c:401-444, get_eid)
__global__ void k_merge(int64_t n, const uint64_t* __restrict__ key, const int32_t* __restrict__ val,
                        const int32_t* __restrict__ head, const int32_t* __restrict__ pos,
                        const double* __restrict__ elat, const double* __restrict__ erel, int32_t* in_src,
                        double* in_w, float* in_w32, double* in_r, int32_t* in_eid, int32_t* arc_v,
                        int32_t* multigraph) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!head[i]) continue;
        const uint64_t k = key[i];
        const int32_t low = val[i];
        double w = elat[low];
        for (int64_t j = i + 1; j < n && key[j] == k; ++j) w = fmin(w, elat[val[j]]);
        const int32_t p = pos[i];
        in_src[p] = (int32_t)(uint32_t)k;
        in_w[p] = w;
        in_w32[p] = __double2float_rd(w);  // the f32 filter key (engine.hip f32_key)
        in_r[p] = erel[low];
        in_eid[p] = low;
        arc_v[p] = (int32_t)(k >> 32);
        if (w != elat[low]) atomicOr(multigraph, 1);
    }
}

__global__ void k_pad(int64_t M, int pad, int32_t* in_src, double* in_w, float* in_w32, double* in_r,
                      int32_t* in_eid) {
    const int k = threadIdx.x;
    if (k >= pad) return;
    in_src[M + k] = 0;
    in_w[M + k] = __longlong_as_double(0x7ff0000000000000LL);
    in_w32[M + k] = __int_as_float(0x7f800000);
    in_r[M + k] = 0.0;
    in_eid[M + k] = -1;
}

// CSR row pointer [V+1] from a sorted array of row ids (n entries): ptr[x] = first index with
// row >= x
__global__ void k_bounds(int64_t n, int32_t V, const int32_t* __restrict__ row, int64_t* ptr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n == 0) {
        for (int64_t x = i; x <= V; x += (int64_t)gridDim.x * blockDim.x) ptr[x] = 0;
        return;
    }
    for (int64_t p = i; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int32_t lo = p == 0 ? 0 : row[p - 1] + 1;
        for (int32_t x = lo; x <= row[p]; ++x) ptr[x] = p;
        if (p == n - 1)
            for (int64_t x = (int64_t)row[p] + 1; x <= V; ++x) ptr[x] = n;
    }
}

// high / low halves of sorted 64-bit keys
__global__ void k_split(int64_t n, const uint64_t* __restrict__ key, int32_t* hi, int32_t* lo) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (hi) hi[i] = (int32_t)(key[i] >> 32);
        if (lo) lo[i] = (int32_t)(uint32_t)key[i];
    }
}

__global__ void k_outkey(int64_t M, const int32_t* __restrict__ in_src, const int32_t* __restrict__ arc_v,
                         uint64_t* key) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < M; p += (int64_t)gridDim.x * blockDim.x)
        key[p] = (uint64_t)(uint32_t)in_src[p] << 32 | (uint32_t)arc_v[p];
}

// incidence sort keys: out-list (from, to), in-list (to, from); value = eid
__global__ void k_inckeys(int64_t E, const int32_t* __restrict__ efrom, const int32_t* __restrict__ eto,
                          uint64_t* okey, uint64_t* ikey, int32_t* val) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        okey[e] = (uint64_t)(uint32_t)efrom[e] << 32 | (uint32_t)eto[e];
        if (ikey) ikey[e] = (uint64_t)(uint32_t)eto[e] << 32 | (uint32_t)efrom[e];
        val[e] = (int32_t)e;
    }
}

__global__ void k_inc_count(int32_t V, const int64_t* __restrict__ os, const int64_t* __restrict__ is, int64_t* cnt) {
    for (int32_t v = blockIdx.x * blockDim.x + threadIdx.x; v <= V; v += gridDim.x * blockDim.x)
        cnt[v] = v == V ? 0 : (os[v + 1] - os[v]) + (is ? is[v + 1] - is[v] : 0);
}

__global__ void k_inc_fill(int64_t E, const int32_t* __restrict__ row, const int32_t* __restrict__ eid,
                           const int64_t* __restrict__ seg, const int64_t* __restrict__ os,
                           const int64_t* __restrict__ inc_ptr, int after_out, int32_t* inc_eid,
                           const double* __restrict__ elat, double* inc_lat) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < E; x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = row[x];
        const int64_t base = inc_ptr[v] + (after_out ? os[v + 1] - os[v] : 0);
        const int32_t e = eid[x];
        inc_eid[base + (x - seg[v])] = e;
        inc_lat[base + (x - seg[v])] = elat[e];
    }
}

// topology.c:450-552: complete iff every vertex's incident count (undirected: minus one for
// a self-loop) reaches V
__global__ void k_complete(int32_t V, int directed, const int64_t* __restrict__ inc_ptr,
                           const int32_t* __restrict__ loop_eid, int32_t* ok) {
    bool short_list = false;
    for (int32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < V; v += gridDim.x * blockDim.x) {
        int64_t c = inc_ptr[v + 1] - inc_ptr[v];
        if (!directed && loop_eid[v] >= 0) c -= 1;
        short_list |= c < V;
    }
    // one atomic per wave (one per vertex serialised 8.7e5 atomics on one word: 9.9 ms on C5)
    if (__ballot(short_list) != 0ull && (threadIdx.x & 63) == 0) atomicAnd(ok, 0);
}

__global__ void k_dense_fill(int64_t n, int32_t* WI) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        WI[i] = -1;
}

// the arcs' ids at their TRANSPOSED cells WI[v][u]: the in-CSR lists each head v's arcs by
// ascending tail u, so consecutive arcs write neighbouring words (the direct cell [u][v]
// would be one line per arc, Vp * 4 bytes apart: 4.8 ms on C2 against 0.1 ms)
__global__ void k_dense_scatter_t(int64_t M, int32_t Vp, const int32_t* __restrict__ in_src,
                                  const int32_t* __restrict__ arc_v, int32_t* WI) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < M; p += (int64_t)gridDim.x * blockDim.x)
        WI[(size_t)arc_v[p] * Vp + in_src[p]] = (int32_t)p;
}

// WI transposed in place, 64 x 64 tiles: block (I, J), I <= J, holds tiles (I, J) and (J, I)
// in LDS and writes each one's transpose over the other, with the W / W32 / WR cells of both
// from the arcs' latency and reliability (the arcs of one tile's column are consecutive, so
// the gathers stay within a few lines per column)
constexpr int DTT = 64;
__global__ __launch_bounds__(256) void k_dense_tr(int32_t Vp, int32_t* WI, const double* __restrict__ in_w,
                                                  const double* __restrict__ in_r, double* __restrict__ W,
                                                  float* __restrict__ W32, double* __restrict__ WR) {
    __shared__ int32_t sa[DTT][DTT + 1], sb[DTT][DTT + 1];
    const int32_t I = blockIdx.x, J = blockIdx.y;
    if (I > J) return;
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
    const size_t a0 = (size_t)I * DTT * Vp + (size_t)J * DTT, b0 = (size_t)J * DTT * Vp + (size_t)I * DTT;
    for (int r = r0; r < DTT; r += 4) {
        sa[r][c] = WI[a0 + (size_t)r * Vp + c];
        if (I != J) sb[r][c] = WI[b0 + (size_t)r * Vp + c];
    }
    __syncthreads();
    auto put = [&](size_t o, int32_t a) {
        const double w = a >= 0 ? in_w[a] : __longlong_as_double(0x7ff0000000000000LL);
        WI[o] = a;
        W[o] = w;
        W32[o] = a >= 0 ? __double2float_rd(w) : __int_as_float(0x7fc00000);
        WR[o] = a >= 0 ? in_r[a] : 0.0;
    };
    for (int r = r0; r < DTT; r += 4) {
        put(b0 + (size_t)r * Vp + c, sa[c][r]);  // cell (J*64 + r, I*64 + c) = transposed (I, J) tile
        if (I != J) put(a0 + (size_t)r * Vp + c, sb[c][r]);
    }
}

hipError_t sort_pairs(Scratch& sc, const uint64_t* kin, uint64_t* kout, const int32_t* vin, int32_t* vout, int64_t n,
                      int end_bit, hipStream_t s) {
    if (n == 0) return hipSuccess;
    size_t tmp = 0;
    GB_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, kin, kout, vin, vout, (int)n, 0, end_bit, s));
    void* t = nullptr;
    GB_TRY(hipMalloc(&t, tmp));
    sc.v.push_back(t);
    return hipcub::DeviceRadixSort::SortPairs(t, tmp, kin, kout, vin, vout, (int)n, 0, end_bit, s);
}

hipError_t sort_keys(Scratch& sc, const uint64_t* kin, uint64_t* kout, int64_t n, int end_bit, hipStream_t s) {
    if (n == 0) return hipSuccess;
    size_t tmp = 0;
    GB_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, kin, kout, (int)n, 0, end_bit, s));
    void* t = nullptr;
    GB_TRY(hipMalloc(&t, tmp));
    sc.v.push_back(t);
    return hipcub::DeviceRadixSort::SortKeys(t, tmp, kin, kout, (int)n, 0, end_bit, s);
}

template <typename T>
hipError_t exclusive_sum(Scratch& sc, const T* in, T* out, int64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    size_t tmp = 0;
    GB_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, (int)n, s));
    void* t = nullptr;
    GB_TRY(hipMalloc(&t, tmp));
    sc.v.push_back(t);
    return hipcub::DeviceScan::ExclusiveSum(t, tmp, in, out, (int)n, s);
}

}  // namespace

hipError_t build(int32_t V, int64_t E, int64_t n_loops, bool directed, int pad, int32_t* d_src, int32_t* d_dst,
                 double* d_lat, double* d_loss, hipStream_t s, Built& g, std::vector<void*>& allocs,
                 std::vector<void*>& scratch) {
    const bool tr = getenv("SHADOWTOPO_TRACE_BUILD") != nullptr;
    auto t_ph = std::chrono::steady_clock::now();
    auto stamp = [&](const char* what) {
        if (!tr) return;
        (void)hipStreamSynchronize(s);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[graph_build] %s %.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_ph).count());
        t_ph = t;
    };
    Scratch sc{scratch};
    const int dir = directed ? 1 : 0;
    const int64_t NA = directed ? E : 2 * E;           // arcs before dropping loops
    const int64_t NL = NA - (directed ? 1 : 2) * n_loops;  // non-loop arcs
    if (NA >= INT_MAX) return hipErrorInvalidValue;      // hipCUB item counts are int
    // igraph storage, in the uploaded buffers themselves
    g.efrom = d_src;
    g.eto = d_dst;
    g.elat = d_lat;
    g.erel = d_loss;
    GB_TRY(dalloc(allocs, &g.loop_eid, V));
    {
        // loop_eid starts at INT_MAX (atomicMin), then -1 where no loop
        std::vector<int32_t> init((size_t)V, INT_MAX);
        GB_TRY(hipMemcpyAsync(g.loop_eid, init.data(), sizeof(int32_t) * V, hipMemcpyHostToDevice, s));
        GB_TRY(hipStreamSynchronize(s));
    }
    uint64_t *ak = nullptr, *ak2 = nullptr;
    int32_t *av = nullptr, *av2 = nullptr;
    GB_TRY(dalloc(sc.v, &ak, NA));
    GB_TRY(dalloc(sc.v, &ak2, NA));
    GB_TRY(dalloc(sc.v, &av, NA));
    GB_TRY(dalloc(sc.v, &av2, NA));
    if (E)
        hipLaunchKernelGGL(k_edges, dim3(grid_of(E)), dim3(256), 0, s, E, V, dir, d_src, d_dst, d_loss, g.efrom, g.eto,
                           g.erel, g.loop_eid, ak, av);
    hipLaunchKernelGGL(k_loop_fix, dim3(grid_of(V)), dim3(256), 0, s, V, g.loop_eid);
    GB_TRY(hipGetLastError());
    const int kbits = 32 + bitlen((uint64_t)V);
    stamp("edges");
    GB_TRY(sort_pairs(sc, ak, ak2, av, av2, NA, kbits, s));
    stamp("arc sort");
    // merge runs of parallel arcs
    int32_t *head = nullptr, *pos = nullptr, *d_mg = nullptr;
    GB_TRY(dalloc(sc.v, &head, NL));
    GB_TRY(dalloc(sc.v, &pos, NL));
    GB_TRY(dalloc(sc.v, &d_mg, 1));
    GB_TRY(hipMemsetAsync(d_mg, 0, sizeof(int32_t), s));
    int64_t M = 0;
    if (NL > 0) {
        hipLaunchKernelGGL(k_heads, dim3(grid_of(NL)), dim3(256), 0, s, NL, ak2, head);
        GB_TRY(exclusive_sum(sc, head, pos, NL, s));
        int32_t last[2] = {0, 0};
        GB_TRY(hipMemcpyAsync(&last[0], pos + NL - 1, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        GB_TRY(hipMemcpyAsync(&last[1], head + NL - 1, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        GB_TRY(hipStreamSynchronize(s));
        M = (int64_t)last[0] + last[1];
    }
    g.n_arcs = M;
    GB_TRY(dalloc(allocs, &g.in_src, M + pad));
    GB_TRY(dalloc(allocs, &g.in_w, M + pad));
    GB_TRY(dalloc(allocs, &g.in_w32, M + pad));
    GB_TRY(dalloc(allocs, &g.in_r, M + pad));
    GB_TRY(dalloc(allocs, &g.in_eid, M + pad));
    GB_TRY(dalloc(allocs, &g.in_ptr, (size_t)V + 1));
    GB_TRY(dalloc(allocs, &g.arc_v, M));
    if (NL > 0)
        hipLaunchKernelGGL(k_merge, dim3(grid_of(NL)), dim3(256), 0, s, NL, ak2, av2, head, pos, g.elat, g.erel,
                           g.in_src, g.in_w, g.in_w32, g.in_r, g.in_eid, g.arc_v, d_mg);
    if (pad > 0) hipLaunchKernelGGL(k_pad, dim3(1), dim3(64), 0, s, M, pad, g.in_src, g.in_w, g.in_w32, g.in_r, g.in_eid);
    hipLaunchKernelGGL(k_bounds, dim3(grid_of(M > 0 ? M : V + 1)), dim3(256), 0, s, M, V, g.arc_v, g.in_ptr);
    GB_TRY(hipGetLastError());
    stamp("merge");
    // out-CSR (directed): merged arcs by (u, v)
    if (directed) {
        GB_TRY(dalloc(allocs, &g.out_ptr, (size_t)V + 1));
        GB_TRY(dalloc(allocs, &g.out_dst, M + pad));
        GB_TRY(hipMemsetAsync(g.out_dst, 0, sizeof(int32_t) * (M + pad), s));
        int32_t* ou = nullptr;
        GB_TRY(dalloc(sc.v, &ou, M));
        if (M > 0) {
            hipLaunchKernelGGL(k_outkey, dim3(grid_of(M)), dim3(256), 0, s, M, g.in_src, g.arc_v, ak);
            GB_TRY(sort_keys(sc, ak, ak2, M, 32 + bitlen((uint64_t)V), s));
            hipLaunchKernelGGL(k_split, dim3(grid_of(M)), dim3(256), 0, s, M, ak2, ou, g.out_dst);
        }
        hipLaunchKernelGGL(k_bounds, dim3(grid_of(M > 0 ? M : V + 1)), dim3(256), 0, s, M, V, ou, g.out_ptr);
        GB_TRY(hipGetLastError());
    }
    stamp("out-csr");
    // igraph_incident(OUT) order
    GB_TRY(dalloc(allocs, &g.inc_ptr, (size_t)V + 1));
    int64_t *os = nullptr, *is = nullptr, *cnt = nullptr;
    int32_t *orow = nullptr, *irow = nullptr, *oval = nullptr, *ival = nullptr;
    GB_TRY(dalloc(sc.v, &os, (size_t)V + 1));
    GB_TRY(dalloc(sc.v, &cnt, (size_t)V + 1));
    GB_TRY(dalloc(sc.v, &orow, E));
    GB_TRY(dalloc(sc.v, &oval, E));
    if (!directed) {
        GB_TRY(dalloc(sc.v, &is, (size_t)V + 1));
        GB_TRY(dalloc(sc.v, &irow, E));
        GB_TRY(dalloc(sc.v, &ival, E));
    }
    // reuse the arc buffers (NA >= E): okey in ak, ikey in ak + E (undirected: NA = 2E)
    uint64_t* okey = ak;
    uint64_t* ikey = directed ? nullptr : ak + E;
    uint64_t* okey2 = ak2;
    uint64_t* ikey2 = directed ? nullptr : ak2 + E;
    if (E > 0) {
        hipLaunchKernelGGL(k_inckeys, dim3(grid_of(E)), dim3(256), 0, s, E, g.efrom, g.eto, okey, ikey, av);
        GB_TRY(sort_pairs(sc, okey, okey2, av, oval, E, kbits, s));
        hipLaunchKernelGGL(k_split, dim3(grid_of(E)), dim3(256), 0, s, E, okey2, orow, nullptr);
        if (!directed) {
            GB_TRY(sort_pairs(sc, ikey, ikey2, av, ival, E, kbits, s));
            hipLaunchKernelGGL(k_split, dim3(grid_of(E)), dim3(256), 0, s, E, ikey2, irow, nullptr);
        }
    }
    hipLaunchKernelGGL(k_bounds, dim3(grid_of(E > 0 ? E : V + 1)), dim3(256), 0, s, E, V, orow, os);
    if (!directed) hipLaunchKernelGGL(k_bounds, dim3(grid_of(E > 0 ? E : V + 1)), dim3(256), 0, s, E, V, irow, is);
    hipLaunchKernelGGL(k_inc_count, dim3(grid_of((int64_t)V + 1)), dim3(256), 0, s, V, os, is, cnt);
    GB_TRY(hipGetLastError());
    GB_TRY(exclusive_sum(sc, cnt, g.inc_ptr, (int64_t)V + 1, s));
    const int64_t ninc = directed ? E : 2 * E;
    GB_TRY(dalloc(allocs, &g.inc_eid, ninc));
    GB_TRY(dalloc(allocs, &g.inc_lat, ninc));
    if (E > 0) {
        hipLaunchKernelGGL(k_inc_fill, dim3(grid_of(E)), dim3(256), 0, s, E, orow, oval, os, os, g.inc_ptr, 0, g.inc_eid,
                           g.elat, g.inc_lat);
        if (!directed)
            hipLaunchKernelGGL(k_inc_fill, dim3(grid_of(E)), dim3(256), 0, s, E, irow, ival, is, os, g.inc_ptr, 1,
                               g.inc_eid, g.elat, g.inc_lat);
    }
    stamp("incidence");
    int32_t* d_ok = nullptr;
    GB_TRY(dalloc(sc.v, &d_ok, 1));
    const int32_t one = 1;
    GB_TRY(hipMemcpyAsync(d_ok, &one, sizeof(int32_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_complete, dim3(grid_of(V)), dim3(256), 0, s, V, dir, g.inc_ptr, g.loop_eid, d_ok);
    GB_TRY(hipGetLastError());
    int32_t flags[2] = {0, 0};
    GB_TRY(hipMemcpyAsync(&flags[0], d_mg, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    GB_TRY(hipMemcpyAsync(&flags[1], d_ok, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    GB_TRY(hipStreamSynchronize(s));
    stamp("tail");
    g.multigraph = flags[0];
    g.complete = flags[1];
    return hipSuccess;
}

hipError_t preload() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_edges));
}

hipError_t build_dense(int32_t Vp, const Built& g, double* W, int32_t* WI, float* W32, double* WR, hipStream_t s) {
    if (Vp % DTT) return hipErrorInvalidValue;
    const int64_t n = (int64_t)Vp * Vp;
    const bool tr = getenv("SHADOWTOPO_TRACE_BUILD") != nullptr;
    auto t_ph = std::chrono::steady_clock::now();
    auto stamp = [&](const char* what) {
        if (!tr) return;
        (void)hipStreamSynchronize(s);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[graph_build] %s %.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_ph).count());
        t_ph = t;
    };
    stamp("dense start");
    hipLaunchKernelGGL(k_dense_fill, dim3(grid_of(n)), dim3(256), 0, s, n, WI);
    stamp("dense fill");
    if (g.n_arcs > 0)
        hipLaunchKernelGGL(k_dense_scatter_t, dim3(grid_of(g.n_arcs)), dim3(256), 0, s, g.n_arcs, Vp, g.in_src,
                           g.arc_v, WI);
    stamp("dense scatter");
    hipLaunchKernelGGL(k_dense_tr, dim3(Vp / DTT, Vp / DTT), dim3(256), 0, s, Vp, WI, g.in_w, g.in_r, W, W32, WR);
    GB_TRY(hipGetLastError());
    stamp("dense transpose");
    return hipStreamSynchronize(s);
}

}  // namespace graph_build
