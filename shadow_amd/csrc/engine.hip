// engine.hip -- libshadowtopo_hip: batched many-source shortest-latency routing for
// Shadow's topology (gfx950 / MI355X).  C ABI: include/shadowtopo.h.
//
// What this replaces in the reference (/root/reference/src/main/routing/topology.c):
// one igraph Dijkstra per unique attached source, run lazily on a cache miss under the
// global graphLock (:1655-1875, :1747-1781), followed by a per-target path walk that
// re-fetches every hop's edge with igraph_get_eid (:1407-1523), the self-path rule
// (:1545-1653), the direct-path rule (:1877-1927) and the dispatch of
// _topology_getPathEntry (:2019-2031).
//
// How (see DESIGN.md for the full argument):
//  * A batch = 64 sources = one wavefront's lanes.  Per-batch state is laid out
//    [vertex][lane] (source-minor), so the 64 distances of one vertex are one 512-byte
//    row: every relaxation step is one fully coalesced global_load_dwordx2 per wave.
//  * k_relax: pull-style label-correcting rounds.  One wave owns one destination v and
//    walks v's in-arcs (scalar loads: the arc list is wave-uniform); each lane keeps the
//    lexicographic minimum of (fl(d(u)+w), d(u)).  In exact IEEE arithmetic every
//    relaxation order converges to the same fixed point as igraph's Dijkstra, and the
//    (candidate, d(u)) minimum is igraph's "first popped predecessor" whenever no two
//    candidates share d(u) -- that case is flagged (tie taint) and resolved by k_replay,
//    a heap-exact re-execution of igraph's algorithm on the device.
//  * Hop count and the reliability product are carried along the predecessor tree in
//    the same rounds (H, R), so the common case needs no path walk at all.
//  * Frontier: a vertex is recomputed only when an in-neighbour changed (byte flags).
//  * k_compose applies the reference's pair dispatch and writes the attached-pair rows
//    through an LDS transpose (coalesced row stores).
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "graph_build.h"
#include "shadowtopo.h"

namespace {

constexpr int KL = 64;                    // sources per batch = wave width
constexpr int SPEC_MAX = 4;               // dense: most leading rounds enqueued without a read-back
constexpr int CNT_ROWS = SPEC_MAX + 4;    // change-count rows per batch slot (run_rounds: cnt_row)
constexpr uint32_t TAINT = 0x80000000u;   // H bit: tree path crosses a heap-order tie
constexpr uint32_t LTIE = 0x40000000u;    // H bit: the tie is at this vertex (its own predecessor choice)
constexpr uint32_t HMASK = 0x3fffffffu;
constexpr int REPLAY_SLOTS = 64;

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return fail(SHADOWTOPO_EDEVICE, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                                     \
    } while (0)

struct GraphDev {
    int32_t V;
    uint32_t flags;
    int32_t multigraph;
    int32_t Vp;              // state rows per batch slot: V rounded up to 64
    const int64_t* in_ptr;   // [V+1] relaxation in-CSR (no loops, parallel edges merged)
    const int32_t* in_src;   // [arcs] tail u, ascending within a row
    const double* in_w;      // [arcs] min latency over the merged parallel edges
    const float* in_w32;     // [arcs] in_w rounded toward -inf (the f32 filter key; padding arcs +inf)
    const double* in_r;      // [arcs] 1 - packetloss of the get_eid edge
    const int32_t* in_eid;   // [arcs] get_eid edge (lowest edge id)
    const int64_t* out_ptr;  // [V+1] out-neighbours (== in-CSR for undirected graphs)
    const int32_t* out_dst;
    const int64_t* inc_ptr;  // [V+1] igraph_incident(OUT) order, loops included
    const int32_t* inc_eid;
    const double* inc_lat;   // [inc] elat in that order (k_self's contiguous scan)
    const int32_t* efrom;    // igraph storage (undirected: from = max, to = min)
    const int32_t* eto;
    const double* elat;
    const double* erel;      // 1.0 - packetloss (topology.c:437)
    const double* vfac;      // 1.0 - vertex packetloss, 1.0 when absent (topology.c:1441-1462)
    const int32_t* loop_eid; // lowest-id self-loop per vertex, -1 if none
};

// Per-batch state lives in contiguous pools (slot b at offset b * vk), addressed from the
// kernel argument itself: no dependent load of a descriptor before the first useful load.
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) uint32_t guint;
typedef __attribute__((address_space(1))) int32_t gint;
typedef __attribute__((address_space(1))) uint8_t gbyte;

// The tree record of a (vertex, source) pair: reliability fold, hops | TAINT | LTIE and the
// predecessor in-arc, interleaved in 16 bytes, so the predecessor gather of a changed pair
// (finish_vertex: one lane, one scattered record) touches one cache line instead of two,
// and a visit reads / writes its own record with one 16-byte access per lane.
struct __attribute__((aligned(16))) Rec {
    double r;
    uint32_t h;
    int32_t p;
};
typedef __attribute__((address_space(1))) Rec gRec;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ Rec rec_load(const gRec* q) {
    const u32x4 v = *(const gu32x4*)q;
    Rec x;
    x.r = __longlong_as_double((long long)(((unsigned long long)v.y << 32) | v.x));
    x.h = v.z;
    x.p = (int32_t)v.w;
    return x;
}

__device__ __forceinline__ void rec_store(gRec* q, double r, uint32_t h, int32_t p) {
    const unsigned long long rb = (unsigned long long)__double_as_longlong(r);
    *(gu32x4*)q = u32x4{(uint32_t)rb, (uint32_t)(rb >> 32), h, (uint32_t)p};
}

struct Pools {
    double* D;          // [slot][Vp][64] distance
    Rec* Q;             // [slot][Vp][64] tree record {reliability fold, hops | TAINT, predecessor in-arc}
    uint8_t* act;       // [slot][2][Vp] frontier flags, alternating rounds
    int32_t* srcv;      // [slot][64] source vertex per lane (-1 = unused lane)
    int32_t* row;       // [slot][64] attached row per lane (-1 = none)
    unsigned long long* mask;  // [slot] lanes whose rows need the heap-exact replay
    double* BDU;        // dense mode: [slot][Vp][64] d(pred) of the recorded predecessor (lex key)
    unsigned long long* chm;   // dense mode: [slot][2][Vp] lanes whose (v, source) state changed, per round parity
    float* D32;         // dense mode: [slot][Vp][64] f32 filter key (distance rounded down, NaN unreached)
    unsigned long long* err;   // compose: nonzero when a path walk left the predecessor tree (the word
                               // before mask[0]: reset and read back together with the masks)
    int32_t* P32;       // lean sparse rounds (Q = NULL): [slot][Vp][64] predecessor arc | LT_BIT (local tie)
    uint8_t* stamp;     // lean sparse rounds: [slot][Vp] round (mod 256) of a vertex's last distance change
    int64_t vk;         // Vp * 64
    int32_t Vp;
    int32_t inc;        // incremental lean rounds (OPT_CSR_INCREMENTAL): 0 = off, else the in-degree
                        // above which a visit reads only the fresh tails
};
// the pendant-pruned relaxation view's device arrays (ensure_pruned), allocated at the graph's
// sizes once and refilled per attached set
struct ViewBufs {
    int32_t *nid = nullptr, *cnt = nullptr, *loop = nullptr, *att = nullptr, *src = nullptr, *eid = nullptr;
    int64_t* ptr = nullptr;
    double *vf = nullptr, *w = nullptr, *r = nullptr;
    float* w32 = nullptr;
};
constexpr int32_t LT_BIT = (int32_t)0x80000000u;  // P32: the predecessor choice here is a heap-order tie
constexpr int32_t P_MASK = 0x7fffffff;
constexpr uint8_t STAMP_NONE = 0x80;  // stamp of a vertex no round has changed (a stale match only costs a re-read)

struct BatchDev {
    gdouble* D;
    gRec* Q;
    gbyte* act0;
    gbyte* act1;
    const int32_t* srcv;
    const int32_t* row;
    unsigned long long* mask;
    gdouble* BDU;
    unsigned long long* chm0;
    unsigned long long* chm1;
    gfloat* D32;
    gint* P32;  // lean rounds only (Q NULL)
    gbyte* st;  // incremental lean rounds only: per-vertex change stamps
    int32_t inc_min;  // incremental lean rounds: in-degree above which a visit reads fresh tails only
    __device__ gbyte* act(int32_t parity) const { return parity ? act1 : act0; }
    __device__ unsigned long long* chm(int32_t parity) const { return parity ? chm1 : chm0; }
};

__device__ __forceinline__ BatchDev batch_view(const Pools& p, int32_t b) {
    BatchDev B;
    const size_t o = (size_t)b * (size_t)p.vk;
    B.D = (gdouble*)(p.D + o);
    B.Q = p.Q ? (gRec*)(p.Q + o) : nullptr;  // NULL with lean rounds (P32 instead)
    B.act0 = (gbyte*)(p.act + (size_t)b * 2 * p.Vp);
    B.act1 = B.act0 + p.Vp;
    B.srcv = p.srcv + (size_t)b * KL;
    B.row = p.row + (size_t)b * KL;
    B.mask = p.mask + b;
    B.BDU = p.BDU ? (gdouble*)(p.BDU + o) : nullptr;
    B.chm0 = p.chm ? p.chm + (size_t)b * 2 * p.Vp : nullptr;
    B.chm1 = B.chm0 ? B.chm0 + p.Vp : nullptr;
    B.D32 = p.D32 ? (gfloat*)(p.D32 + o) : nullptr;
    B.P32 = p.P32 ? (gint*)(p.P32 + o) : nullptr;
    B.st = p.inc && p.stamp ? (gbyte*)(p.stamp + (size_t)b * p.Vp) : nullptr;
    B.inc_min = p.inc;
    return B;
}

struct ReplayDev {
    double* dist;     // [slot][V]
    int32_t* parent;  // [slot][V] parent edge id
    double* hdata;    // [slot][V] heap keys
    int32_t* hidx;    // [slot][V] heap position -> vertex
    int32_t* hidx2;   // [slot][V] vertex -> position + 2 (0 = not in heap)
    uint8_t* tgt;     // [slot][V]
    int32_t srcv[REPLAY_SLOTS];
    int32_t row[REPLAY_SLOTS];
};

constexpr int CSR_PAD = 16;  // in_src / in_w carry 16 padding arcs (u = 0, w = +inf) so chunk loads never clamp

__device__ __forceinline__ double dinf() { return __longlong_as_double(0x7ff0000000000000LL); }
inline double dinf_host() { return std::numeric_limits<double>::infinity(); }
__device__ __forceinline__ double dmax() { return __longlong_as_double(0x7fefffffffffffffLL); }

// Block -> (group, tile) with every XCD busy whatever the group count: the grid has
// 8 * S blocks, S = ceil(groups * tiles / 8), and XCD x (blockIdx % 8) takes the contiguous
// range [x*S, (x+1)*S) of the group-major (group, tile) order -- so a group's tiles share
// one XCD (its [V][64] state stays in that L2) when there are >= 8 groups, and a group is
// spread over several XCDs when there are fewer.  Placement is a speed hint only.
__device__ __forceinline__ bool xcd_tile(int64_t L, int32_t ngroups, int32_t ntiles, int32_t& grp, int32_t& tile) {
    const int64_t S = ((int64_t)ngroups * ntiles + 7) / 8;
    if ((L >> 3) >= S) return false;  // padding blocks of a 2-D grid (grid_of)
    const int64_t i = (L & 7) * S + (L >> 3);
    grp = (int32_t)(i / ntiles);
    tile = (int32_t)(i - (int64_t)grp * ntiles);
    return grp < ngroups;
}

// Linear block id of a grid from grid_of: a launch's work-item count is a 32-bit field of
// the dispatch packet, so grids past 2^24 blocks of 256 go 2-D (x a multiple of 8, so
// flat & 7 is still the XCD the block runs on).
__device__ __forceinline__ int64_t flat_block() { return (int64_t)blockIdx.y * gridDim.x + blockIdx.x; }

// f32 filter key of a distance: rounded toward -inf, NaN when unreached (see k_relax_dense_f)
__device__ __forceinline__ float f32_key(double d) {
    return d < dinf() ? __double2float_rd(d) : __int_as_float(0x7fc00000);
}

// conservative f32 threshold of a running best bc: rounded up plus 4 ulps (+inf when
// unreached); fl32(D32 + W32) <= it whenever fl64(d + w) <= bc (see k_relax_dense_f)
__device__ __forceinline__ float f32_thr(double bc) {
    if (!(bc < dmax())) return __int_as_float(0x7f800000);  // unreached: any finite candidate passes
    const float r = __double2float_ru(bc);
    // 4 ulps up, saturating at +inf: past FLT_MAX the bit pattern would be a NaN, which
    // never passes a filter (a lane would silently lose its candidates)
    if (!(r < __int_as_float(0x7f7ffffc))) return __int_as_float(0x7f800000);
    return __int_as_float(__float_as_int(r) + 4);
}

__device__ __forceinline__ double readlane_d(double x, int l) {
    const long long b = __double_as_longlong(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long x, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ int64_t find_arc(const GraphDev& g, int32_t v, int32_t u) {
    int64_t lo = g.in_ptr[v], end = g.in_ptr[v + 1], hi = end;
    while (lo < hi) {
        int64_t mid = lo + ((hi - lo) >> 1);
        if (g.in_src[mid] < u)
            lo = mid + 1;
        else
            hi = mid;
    }
    return (lo < end && g.in_src[lo] == u) ? lo : -1;
}

// igraph_get_eid(from, to, directed=graph's, error=FALSE) -- topology.c:416-420
__device__ __forceinline__ int32_t get_eid(const GraphDev& g, int32_t from, int32_t to) {
    if (from == to) return g.loop_eid[from];
    int64_t a = find_arc(g, to, from);
    return a < 0 ? -1 : g.in_eid[a];
}

// ---------------------------------------------------------------- batch state init
// D = +inf is the whole unreached state for the FULL and MASKED rounds: H, R and P of a
// (vertex, source) are read only once its D is finite, i.e. after a round wrote all four,
// so `tree` (set for the kernels that read them eagerly) is the only reason to write them.
__global__ void k_init(Pools pools, int32_t V, int32_t tree) {
    const BatchDev B = batch_view(pools, blockIdx.y);
    const size_t total = (size_t)V * KL;
    const double inf = dinf();
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        B.D[i] = inf;
        if (tree) {
            rec_store(B.Q + i, 0.0, 0u, -1);
        }
    }
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)V; i += (size_t)gridDim.x * blockDim.x) {
        B.act0[i] = 0;
        B.act1[i] = 0;
        if (B.st) B.st[i] = STAMP_NONE;
    }
    if (B.chm0) {
        if (tree)
            for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
                if (B.BDU) B.BDU[i] = inf;
                if (B.D32) B.D32[i] = __int_as_float(0x7fc00000);
            }
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)V; i += (size_t)gridDim.x * blockDim.x) {
            B.chm0[i] = 0;
            B.chm1[i] = 0;
        }
    }
}

// sources: d(s) = 0, R(s) = 1*(1-loss_v(s)) (topology.c:1441-1445); activate out-neighbours
__global__ void k_seed(GraphDev g, Pools pools) {
    const BatchDev B = batch_view(pools, blockIdx.y);
    const int j = blockIdx.x;
    const int32_t s = B.srcv[j];
    if (s < 0) return;
    if (threadIdx.x == 0) {
        const size_t idx = (size_t)s * KL + j;
        B.D[idx] = 0.0;
        if (B.Q) rec_store(B.Q + idx, g.vfac[s], 0u, -1);  // lean rounds: the source's P32 is never read
        if (B.st) B.st[s] = 0xFF;  // changed in round -1: round 0's visits read the source's row
        // dense mode: f32 filter key NaN (the source's own row never passes a dense filter:
        // its seed candidate starts every lexicographic state, k_relax_dense_f), and the
        // first delta round reads the change masks of a virtual round -1
        if (B.D32) B.D32[idx] = __int_as_float(0x7fc00000);
        if (B.chm1) atomicOr(&B.chm1[s], 1ull << j);
    }
    for (int64_t x = g.out_ptr[s] + threadIdx.x; x < g.out_ptr[s + 1]; x += blockDim.x) B.act0[g.out_dst[x]] = 1;
}

// Record the new best for (v, lane): hop count / reliability carried from the predecessor
// (topology.c:1499 totalReliability *= edgeReliability), the taint bit from the
// predecessor's path or a tie here.  cur* were prefetched at kernel entry.
__device__ __forceinline__ bool finish_vertex(const BatchDev& B, int lane, int32_t v, int32_t arc, int32_t u, double bc,
                                              double bdu, bool tie, const double* __restrict__ in_r, double curD,
                                              uint32_t curH, double curR, int32_t curP) {
    const size_t idx = (size_t)v * KL + lane;
    if (B.P32) {  // lean rounds: D and the predecessor arc with its local tie bit, nothing folded
        const int32_t np = arc | ((tie || bdu == bc) ? LT_BIT : 0);
        if (bc != curD || np != curP) {
            B.D[idx] = bc;
            B.P32[idx] = np;
            return true;
        }
        return false;
    }
    const size_t uidx = (size_t)u * KL + lane;
    const Rec qu = rec_load(B.Q + uidx);  // the predecessor's record: one line per lane
    const uint32_t hu = qu.h;
    const double ru = qu.r;
    // local tie: two candidates share (fl(d(u)+w), d(u)), or the degenerate d(u) == d(v)
    const uint32_t taint = (hu & TAINT) | ((tie || bdu == bc) ? (TAINT | LTIE) : 0u);
    const uint32_t h = (((hu & HMASK) + 1u) & HMASK) | taint;
    const double r = ru * in_r[arc];
    if (bc != curD || h != curH || r != curR || arc != curP) {
        B.D[idx] = bc;
        if (B.D32) B.D32[idx] = f32_key(bc);
        rec_store(B.Q + idx, r, h, arc);
        return true;
    }
    return false;
}

__device__ __forceinline__ void relax_arc(double du, double w, int32_t e, int32_t u, double& bc, double& bdu,
                                          int32_t& be, int32_t& bu, bool& tie) {
    const double c = du + w;  // igraph: altdist = mindist + weights[edge]
    if (c <= bc) {
        if (c < bc || du < bdu) {
            bc = c;
            bdu = du;
            be = e;
            bu = u;
            tie = false;
        } else if (du == bdu) {
            tie = true;  // two predecessors at the same d(u): heap pop order decides
        }
    }
}

// One relaxation round over every active destination vertex of every batch in flight
// (CSR form, any density).  One wave = one destination v; the in-arc list is walked in
// chunks of 8: one s_load_dwordx8 of tails, one s_load_dwordx16 of weights (the arrays
// carry CSR_PAD padding arcs, so a chunk never clamps; arcs past the row get weight +inf)
// and 8 row loads, all in flight before the first compare.
// Grid: 1-D, remapped so that all blocks sharing an XCD (blockIdx % 8) work on the same
// batch (its [V][64] state then stays in that XCD's L2).  Placement is a speed hint only.
// one visit of destination v in batch b (the body of k_relax / k_relax_wl)
__device__ __forceinline__ void relax_visit(const int64_t* __restrict__ in_ptr, const int32_t* __restrict__ in_src,
                                            const double* __restrict__ in_w, const double* __restrict__ in_r,
                                            const int64_t* __restrict__ out_ptr, const int32_t* __restrict__ out_dst,
                                            const BatchDev& B, int32_t b, int32_t v, int lane, int32_t round,
                                            int32_t* __restrict__ cnt, unsigned long long* __restrict__ prof) {
    const int32_t parity = round & 1;
    const int32_t beg = (int32_t)in_ptr[v], end = (int32_t)in_ptr[v + 1];
    const int32_t sv = B.srcv[lane];
    const size_t idx = (size_t)v * KL + lane;
    const double curD = B.D[idx];
    uint32_t curH = 0;
    double curR = 0.0;
    int32_t curP;
    if (B.P32) {
        curP = B.P32[idx];
    } else {
        const Rec cur = rec_load(B.Q + idx);
        curH = cur.h;
        curR = cur.r;
        curP = cur.p;
    }
    const gdouble* Dl = B.D + lane;
    // (unlike the dense kernel, the running best is not seeded with curD here: rows are
    // short, and seeding would put curD's load latency in front of the first row loads)
    double bc = dmax(), bdu = dinf();
    int32_t be = -1, bu = -1;
    bool tie = false;
    for (int32_t e = beg; e < end; e += 8) {
        int32_t u[8];
        double w[8], du[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            u[k] = in_src[e + k];
            w[k] = in_w[e + k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (e + k >= end) w[k] = dinf();
            du[k] = e + k < end ? Dl[(size_t)u[k] * KL] : 0.0;  // no row loads past the list
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) relax_arc(du[k], w[k], e + k, u[k], bc, bdu, be, bu, tie);
    }

    bool ch = false;
    if (be >= 0 && sv >= 0 && sv != v) ch = finish_vertex(B, lane, v, be, bu, bc, bdu, tie, in_r, curD, curH, curR, curP);
    // lean rounds: only a distance change reaches the out-neighbours (their candidates depend
    // on d alone; with the tree fold in the rounds a changed hop count or reliability has to)
    if (B.P32) ch = ch && bc != curD;
    if (__ballot(ch)) {
        gbyte* act_nxt = B.act(parity ^ 1);
        for (int64_t x = out_ptr[v] + lane; x < out_ptr[v + 1]; x += 64) act_nxt[out_dst[x]] = 1;
        if (lane == 0) {
            cnt[b] = 1;  // idempotent flag, no atomic contention
            if (B.st) B.st[v] = (uint8_t)round;  // incremental lean rounds: v's row is fresh
        }
        if (prof && lane == 0) atomicAdd(&prof[2 * (8 * b + (blockIdx.x & 7)) + 1], 1ull);
    }
    if (prof && lane == 0) atomicAdd(&prof[2 * (8 * b + (blockIdx.x & 7))], 1ull);
}

// Incremental lean visit (OPT_CSR_INCREMENTAL).  The state (d, predecessor arc | tie bit) of
// (v, lane) is already the lexicographic minimum over every in-arc at the values its tail had
// when last read, and distances only fall; so a visit only has to fold in the arcs whose tail
// changed since: a change in round q stamps the tail (u, batch) with q and activates v for
// round q + 1, whose visit reads the tails stamped q or q + 1 (a later change stamps and
// activates again).  A tail's row is loaded only when its stamp is fresh -- one byte per
// (tail, batch) instead of 512 bytes per arc.  The running best starts from the stored state;
// its d(pred), the second key, is gathered only when a candidate meets it at an equal
// distance.  The tie bit is carried while the key holds and cleared when a strictly better
// candidate replaces it: an arc that ties the final key is read at its final value after its
// tail's last change, which is when that key is already the running best or becomes it, so
// no tie the full visit finds is lost; a bit that outlives its tie (the predecessor's d fell
// at the same fl sum) only sends the source to the heap-exact replay.  Same distances, same
// predecessor wherever the path is untied.
__device__ __forceinline__ void relax_arc_inc(const int32_t* __restrict__ in_src, const gdouble* Dl, double du,
                                              double w, int32_t e, double& bc, double& bdu, int32_t& be, bool& tie,
                                              bool& known) {
    const double c = du + w;
    if (c < bc) {
        bc = c;
        bdu = du;
        be = e;
        tie = false;
        known = true;
    } else if (c == bc && e != be) {
        if (!known) {  // the stored predecessor's d, now (only ever falls: a stale key is re-decided)
            bdu = Dl[(size_t)in_src[be] * KL];
            known = true;
        }
        if (du < bdu) {
            bdu = du;
            be = e;
            tie = false;
        } else if (du == bdu) {
            tie = true;
        }
    }
}

__device__ __forceinline__ void relax_visit_inc(const int64_t* __restrict__ in_ptr, const int32_t* __restrict__ in_src,
                                                const double* __restrict__ in_w, const double* __restrict__ in_r,
                                                const int64_t* __restrict__ out_ptr,
                                                const int32_t* __restrict__ out_dst, const BatchDev& B, int32_t b,
                                                int32_t v, int lane, int32_t round, int32_t* __restrict__ cnt,
                                                unsigned long long* __restrict__ prof) {
    const int32_t beg = (int32_t)in_ptr[v], end = (int32_t)in_ptr[v + 1];
    // a short in-list costs one chunk of row loads either way: the full visit (it stamps too)
    // has one dependent load fewer than the stamp filter
    if (end - beg <= B.inc_min) {
        relax_visit(in_ptr, in_src, in_w, in_r, out_ptr, out_dst, B, b, v, lane, round, cnt, prof);
        return;
    }
    const int32_t sv = B.srcv[lane];
    const size_t idx = (size_t)v * KL + lane;
    const double curD = B.D[idx];
    const int32_t curP = B.P32[idx];
    const gdouble* Dl = B.D + lane;
    const uint32_t s_prev = (uint32_t)(round - 1) & 0xffu, s_cur = (uint32_t)round & 0xffu;
    double bc = dmax(), bdu = dinf();
    int32_t be = -1;
    bool tie = false, known = true;
    const int32_t a0 = curP & P_MASK;
    if (curD < dinf() && sv >= 0 && sv != v && a0 >= beg && a0 < end) {
        bc = curD;
        be = a0;
        tie = curP < 0;  // LT_BIT
        known = false;
    }
    // 64 in-arcs at a time: lane i reads arc i's tail, weight and the tail's stamp; the ballot
    // is the fresh-arc mask, whose arcs then go 8 rows in flight
    for (int32_t e0 = beg; e0 < end; e0 += 64) {
        const int32_t e = e0 + lane;
        int32_t ul = 0;
        double wl = 0.0;
        bool fresh = false;
        if (e < end) {
            ul = in_src[e];
            wl = in_w[e];
            const uint32_t t = B.st[ul];
            fresh = t == s_prev || t == s_cur;
        }
        uint64_t m = __ballot(fresh);
        while (m) {
            int32_t uq[8], eq[8];
            double wq[8], dq[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                eq[q] = -1;
                uq[q] = 0;
                wq[q] = 0.0;
                if (m) {
                    const int i = __builtin_ctzll(m);
                    m &= m - 1;
                    eq[q] = e0 + i;
                    uq[q] = __builtin_amdgcn_readlane(ul, i);
                    wq[q] = readlane_d(wl, i);
                }
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) dq[q] = eq[q] >= 0 ? Dl[(size_t)uq[q] * KL] : 0.0;
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (eq[q] >= 0) relax_arc_inc(in_src, Dl, dq[q], wq[q], eq[q], bc, bdu, be, tie, known);
        }
    }
    bool ch = false;
    if (be >= 0 && sv >= 0 && sv != v) {
        const int32_t np = be | ((tie || (known && bdu == bc)) ? LT_BIT : 0);
        if (bc != curD) {
            B.D[idx] = bc;
            B.P32[idx] = np;
            ch = true;
        } else if (np != curP) {
            B.P32[idx] = np;  // a tie found at the same distance: no activation
        }
    }
    if (__ballot(ch)) {
        gbyte* act_nxt = B.act((round & 1) ^ 1);
        for (int64_t x = out_ptr[v] + lane; x < out_ptr[v + 1]; x += 64) act_nxt[out_dst[x]] = 1;
        if (lane == 0) {
            B.st[v] = (uint8_t)round;
            cnt[b] = 1;
        }
        if (prof && lane == 0) atomicAdd(&prof[2 * (8 * b + (blockIdx.x & 7)) + 1], 1ull);
    }
    if (prof && lane == 0) atomicAdd(&prof[2 * (8 * b + (blockIdx.x & 7))], 1ull);
}

template <bool INC>
__device__ __forceinline__ void relax_visit_any(const int64_t* __restrict__ in_ptr, const int32_t* __restrict__ in_src,
                                                const double* __restrict__ in_w, const double* __restrict__ in_r,
                                                const int64_t* __restrict__ out_ptr,
                                                const int32_t* __restrict__ out_dst, const BatchDev& B, int32_t b,
                                                int32_t v, int lane, int32_t round, int32_t* __restrict__ cnt,
                                                unsigned long long* __restrict__ prof) {
    if (INC)
        relax_visit_inc(in_ptr, in_src, in_w, in_r, out_ptr, out_dst, B, b, v, lane, round, cnt, prof);
    else
        relax_visit(in_ptr, in_src, in_w, in_r, out_ptr, out_dst, B, b, v, lane, round, cnt, prof);
}

// one wave per (destination, batch) of the whole grid; inactive pairs exit after their flag.
// INC: incremental lean visits (the batch views carry stamps; see relax_visit_inc)
template <bool INC>
__global__ __launch_bounds__(256) void k_relax(const int64_t* __restrict__ in_ptr, const int32_t* __restrict__ in_src,
                                               const double* __restrict__ in_w, const double* __restrict__ in_r,
                                               const int64_t* __restrict__ out_ptr,
                                               const int32_t* __restrict__ out_dst, Pools pools,
                                               int32_t V, int32_t nb, int32_t nvb, int32_t round,
                                               int32_t* __restrict__ cnt, unsigned long long* __restrict__ prof) {
    int32_t b, vt;
    if (!xcd_tile(flat_block(), nb, nvb, b, vt)) return;
    const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int32_t v = vt * 4 + wave;
    if (v >= V) return;
    const int lane = threadIdx.x & 63;
    const BatchDev B = batch_view(pools, b);
    gbyte* act_cur = B.act(round & 1);
    if (act_cur[v] == 0) return;
    if (lane == 0) act_cur[v] = 0;
    relax_visit_any<INC>(in_ptr, in_src, in_w, in_r, out_ptr, out_dst, B, b, v, lane, round, cnt, prof);
}

// Frontier worklists (default for sparse graphs): the active destinations of each batch for
// the next round, compacted from the activity flags into one list per batch.  Without them
// every round launches a wave for every (vertex, batch) pair -- 1.6e7 on C4 -- and each
// inactive one still pays a flag load; rounds where most pairs are active use the grid.
constexpr int WL_SPAN = 4096;  // vertices per compaction block: 16 flags per thread, one atomic per block
__global__ __launch_bounds__(256) void k_compact(Pools pools, int32_t V, int32_t parity, int4* __restrict__ wl,
                                                 uint32_t* __restrict__ wlcnt, const int64_t* __restrict__ in_ptr) {
    __shared__ uint32_t sc[256];
    __shared__ uint32_t sbase;
    const int32_t b = blockIdx.y;
    const int32_t v0 = blockIdx.x * WL_SPAN + threadIdx.x * 16;
    const BatchDev B = batch_view(pools, b);
    // 16 flags in one 16-byte load (the flag arrays are 64-aligned and padded to Vp, zero past V)
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (v0 < V) {
        const uint4 f = *(const uint4*)((const uint8_t*)B.act(parity) + v0);
        w[0] = f.x;
        w[1] = f.y;
        w[2] = f.z;
        w[3] = f.w;
    }
    uint32_t bits = 0;  // bit i: vertex v0 + i active
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) bits |= ((w[q] >> (8 * i)) & 0xFFu) ? 1u << (4 * q + i) : 0u;
    const uint32_t n = (uint32_t)__popc(bits);
    // block inclusive scan of the counts (Hillis-Steele in LDS)
    sc[threadIdx.x] = n;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const uint32_t add = threadIdx.x >= (unsigned)off ? sc[threadIdx.x - off] : 0u;
        __syncthreads();
        sc[threadIdx.x] += add;
        __syncthreads();
    }
    const uint32_t incl = sc[threadIdx.x];
    if (threadIdx.x == 255) sbase = incl ? atomicAdd(&wlcnt[b], incl) : 0u;
    __syncthreads();
    uint32_t pos = sbase + incl - n;
    int4* out = wl + (size_t)b * pools.Vp;
    // an entry carries the vertex's in-arc range too: the relax wave starts its arc loads
    // from the entry instead of a dependent in_ptr load
    while (bits) {
        const int i = __builtin_ctz(bits);
        bits &= bits - 1;
        const int32_t v = v0 + i;
        out[pos++] = make_int4(v, (int32_t)in_ptr[v], (int32_t)in_ptr[v + 1], 0);
    }
}

// batch of worklist item i: the last b with prefix[b] <= i (prefix non-decreasing) -- one
// coalesced load of the prefix per 64 batches and a wave ballot, instead of a binary search
// of dependent loads
__device__ __forceinline__ int32_t wl_batch(const int64_t* __restrict__ prefix, int32_t nb, int64_t i, int lane) {
    int32_t c = 0;
    for (int32_t q = 0; q < nb; q += 64) {
        const int32_t j = q + lane;
        c += __popcll(__ballot(j < nb && prefix[j] <= i));
    }
    return c - 1;
}

// one wave per listed (vertex, batch): the T items of all batches in batch-major order
// (prefix[b] = items before batch b), XCD x (block % 8) takes the contiguous slice
// [x*S, (x+1)*S) -- a batch's state stays in one XCD's L2, as with xcd_tile
template <bool INC>
__global__ __launch_bounds__(256) void k_relax_wl(const int64_t* __restrict__ in_ptr, const int32_t* __restrict__ in_src,
                                                  const double* __restrict__ in_w, const double* __restrict__ in_r,
                                                  const int64_t* __restrict__ out_ptr,
                                                  const int32_t* __restrict__ out_dst, Pools pools, int32_t round,
                                                  const int4* __restrict__ wl, const int64_t* __restrict__ prefix,
                                                  int32_t nb, int64_t S, int32_t* __restrict__ cnt,
                                                  unsigned long long* __restrict__ prof) {
    const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t L = flat_block();
    const int64_t i = (L & 7) * S + (L >> 3) * 4 + wave;
    const int64_t T = prefix[nb];
    if ((L >> 3) * 4 + wave >= S || i >= T) return;
    const int lane = threadIdx.x & 63;
    const int32_t b = __builtin_amdgcn_readfirstlane(wl_batch(prefix, nb, i, lane));
    // wave-uniform (one item per wave): the arc list then streams through scalar loads into
    // SGPRs, as in k_relax, instead of occupying VGPRs (84 -> occupancy 5 of 8)
    const int32_t v = __builtin_amdgcn_readfirstlane(wl[(size_t)b * pools.Vp + (size_t)(i - prefix[b])].x);
    const BatchDev B = batch_view(pools, b);
    relax_visit_any<INC>(in_ptr, in_src, in_w, in_r, out_ptr, out_dst, B, b, v, lane, round, cnt, prof);
    // cleared after the visit (this round sets only the other parity's flags): a store ahead
    // of the arc-list loads would keep them off the scalar unit (they could alias it)
    if (lane == 0) B.act(round & 1)[v] = 0;
}

// Device-driven worklist rounds (graphs whose batches x vertices fit OPT_DEVICE_ROUNDS'
// bound, e.g. C3): the round's item count never visits the host.  k_scan_wl turns the
// per-batch counts of k_compact into the prefix the worklist kernel reads, and logs the
// total per round (tlog[round]: the host reads a block of rounds at once and stops at the
// first empty one, which is convergence: no change, no activation).  It also zeroes the
// counts for the next round's k_compact (one memset launch fewer per round).
__global__ __launch_bounds__(256) void k_scan_wl(uint32_t* __restrict__ wlcnt, int32_t nb,
                                                 int64_t* __restrict__ prefix, int64_t* __restrict__ tlog,
                                                 int32_t round) {
    __shared__ int64_t sc[256];
    constexpr int PER = 4;  // nb <= 1024
    int64_t v[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int32_t b = threadIdx.x * PER + k;
        v[k] = 0;
        if (b < nb) {
            v[k] = (int64_t)wlcnt[b];
            wlcnt[b] = 0u;
        }
        sum += v[k];
    }
    sc[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const int64_t add = threadIdx.x >= (unsigned)off ? sc[threadIdx.x - off] : 0;
        __syncthreads();
        sc[threadIdx.x] += add;
        __syncthreads();
    }
    int64_t run = sc[threadIdx.x] - sum;  // items before this thread's batches
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int32_t b = threadIdx.x * PER + k;
        if (b < nb) prefix[b] = run;
        run += v[k];
    }
    if (threadIdx.x == 255) {
        prefix[nb] = sc[255];
        tlog[round] = sc[255];
    }
}

// k_relax_wl with a fixed grid (G blocks, G / 8 per XCD) that loops over the round's items:
// XCD x (block % 8) takes the slice [x*S, (x+1)*S) of the batch-major list, S = ceil(T / 8),
// its waves striding through it; an empty round's blocks exit at once.  A heavy round (at
// least half the pairs active, where the host-driven rounds launch the grid kernel) walks the
// virtual grid of k_relax instead -- block vb = blockIdx.x + k * gridDim.x, the same XCD
// (vb % 8) and xcd_tile mapping, one activity flag per (vertex, batch): a worklist entry load
// in front of every visit made these rounds 22-25 % slower (r04l, C4 groups of 20 / 40 batches)
template <bool INC>
__global__ __launch_bounds__(256) void k_relax_wlp(const int64_t* __restrict__ in_ptr, const int32_t* __restrict__ in_src,
                                                   const double* __restrict__ in_w, const double* __restrict__ in_r,
                                                   const int64_t* __restrict__ out_ptr,
                                                   const int32_t* __restrict__ out_dst, Pools pools, int32_t round,
                                                   const int4* __restrict__ wl, const int64_t* __restrict__ prefix,
                                                   int32_t nb, int32_t* __restrict__ cnt,
                                                   unsigned long long* __restrict__ prof, int32_t V) {
    const int64_t T = prefix[nb];
    if (T == 0) return;
    const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (T * 2 >= (int64_t)nb * V) {
        const int32_t nvb = (V + 3) / 4;
        const int64_t nvblocks = 8 * (((int64_t)nb * nvb + 7) / 8);
        for (int64_t vb = blockIdx.x; vb < nvblocks; vb += gridDim.x) {
            int32_t b, vt;
            if (!xcd_tile(vb, nb, nvb, b, vt)) continue;
            const int32_t v = vt * 4 + wave;
            if (v >= V) continue;
            const BatchDev B = batch_view(pools, b);
            gbyte* act_cur = B.act(round & 1);
            if (act_cur[v] == 0) continue;
            relax_visit_any<INC>(in_ptr, in_src, in_w, in_r, out_ptr, out_dst, B, b, v, lane, round, cnt, prof);
            if (lane == 0) act_cur[v] = 0;  // cleared after the visit, as k_relax_wl does
        }
        return;
    }
    const int64_t S = (T + 7) / 8;
    const int64_t x = blockIdx.x & 7;
    const int64_t waves_per_xcd = (int64_t)(gridDim.x >> 3) * 4;
    for (int64_t j = (int64_t)(blockIdx.x >> 3) * 4 + wave; j < S; j += waves_per_xcd) {
        const int64_t i = x * S + j;
        if (i >= T) break;
        const int32_t b = __builtin_amdgcn_readfirstlane(wl_batch(prefix, nb, i, lane));
        const int32_t v = __builtin_amdgcn_readfirstlane(wl[(size_t)b * pools.Vp + (size_t)(i - prefix[b])].x);
        const BatchDev B = batch_view(pools, b);
        relax_visit_any<INC>(in_ptr, in_src, in_w, in_r, out_ptr, out_dst, B, b, v, lane, round, cnt, prof);
        if (lane == 0) B.act(round & 1)[v] = 0;
    }
}

// ---------------------------------------------------------------- push rounds (CSR_PUSH)
// SHADOWTOPO_CSR_PUSH (undirected CSR graphs): the north star's push relaxation, as an
// alternative to the pull rounds above.  Three phases:
//  1. distances only: every (u, source) pair that changed last round pushes fl(d(u) + w)
//     along u's out-arcs (= its in-list, undirected) with a 64-bit atomicMin on the f64 bit
//     pattern (non-negative doubles order like their bits); a plain load of the head's row
//     first, so only lanes that improve on what they see reach the atomic unit (a stale
//     value is never lower than the current one: values only fall).  The lanes that changed
//     are OR-ed into the head's change mask for the next round (chm, the dense mode's masks).
//     Same least fixed point as the pull rounds, so the same distances.
//  2. k_pred_pass: one exact pull pass over every reached (vertex, batch) with the final
//     distances: the lexicographic (fl(d(u)+w), d(u)) minimum and the heap-order tie flag,
//     exactly relax_visit's, gives P and the local tie bit (H = HNOT | LTIE until folded).
//  3. k_fold level rounds: round k finishes every pair whose predecessor finished before round
//     k (its hop count is < k: a pair finished in round k has k hops, so a same-round write is
//     never used), carrying hops, taint and the reliability product down the tree as
//     finish_vertex does; a pair that finishes activates its out-neighbours.
constexpr uint32_t HNOT = HMASK;  // H hop field of a reached pair whose tree fold is pending

__device__ __forceinline__ unsigned long long* gen_u64(gdouble* p) {
    return (unsigned long long*)(double*)p;
}

__device__ __forceinline__ void push_visit(const int32_t* __restrict__ in_src, const double* __restrict__ in_w,
                                           int32_t beg, int32_t end, const BatchDev& B, int32_t b, int32_t u, int lane,
                                           int32_t parity, int32_t* __restrict__ cnt) {
    unsigned long long* chm_cur = B.chm(parity);
    const unsigned long long m = readlane_u64(chm_cur[u], 0);
    if (m == 0ull) return;
    if (lane == 0) chm_cur[u] = 0ull;  // reused two rounds on; this round's pushes go to the other parity
    const bool on = (m >> lane) & 1ull;
    const double du = B.D[(size_t)u * KL + lane];
    unsigned long long* chm_nxt = B.chm(parity ^ 1);
    gbyte* act_nxt = B.act(parity ^ 1);
    bool any = false;
    for (int32_t e = beg; e < end; e += 8) {
        int32_t v[8];
        double w[8], dv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            v[k] = in_src[e + k];
            w[k] = in_w[e + k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) dv[k] = (on && e + k < end) ? B.D[(size_t)v[k] * KL + lane] : 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double c = du + w[k];
            const bool imp = on && e + k < end && c < dv[k];
            if (imp) {
                // no-return atomic: the lane is marked changed whether or not a concurrent push
                // got lower first (it then pushes its current, lower value next round: harmless)
                (void)__hip_atomic_fetch_min(gen_u64(B.D + (size_t)v[k] * KL + lane),
                                             (unsigned long long)__double_as_longlong(c), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
            }
            const unsigned long long bal = __ballot(imp);
            if (bal) {
                any = true;
                if (lane == 0) {
                    atomicOr(&chm_nxt[v[k]], bal);
                    act_nxt[v[k]] = 1;
                }
            }
        }
    }
    if (any && lane == 0) cnt[b] = 1;
}

__global__ __launch_bounds__(256) void k_push(const int64_t* __restrict__ in_ptr, const int32_t* __restrict__ in_src,
                                              const double* __restrict__ in_w, Pools pools, int32_t V, int32_t nb,
                                              int32_t nvb, int32_t parity, int32_t* __restrict__ cnt) {
    int32_t b, vt;
    if (!xcd_tile(flat_block(), nb, nvb, b, vt)) return;
    const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int32_t u = vt * 4 + wave;
    if (u >= V) return;
    const int lane = threadIdx.x & 63;
    const BatchDev B = batch_view(pools, b);
    gbyte* act_cur = B.act(parity);
    if (act_cur[u] == 0) return;
    if (lane == 0) act_cur[u] = 0;
    push_visit(in_src, in_w, (int32_t)in_ptr[u], (int32_t)in_ptr[u + 1], B, b, u, lane, parity, cnt);
}

__global__ __launch_bounds__(256) void k_push_wl(const int32_t* __restrict__ in_src, const double* __restrict__ in_w,
                                                 Pools pools, int32_t parity, const int4* __restrict__ wl,
                                                 const int64_t* __restrict__ prefix, int32_t nb, int64_t S,
                                                 int32_t* __restrict__ cnt) {
    const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t L = flat_block();
    const int64_t i = (L & 7) * S + (L >> 3) * 4 + wave;
    const int64_t T = prefix[nb];
    if ((L >> 3) * 4 + wave >= S || i >= T) return;
    const int lane = threadIdx.x & 63;
    const int32_t b = __builtin_amdgcn_readfirstlane(wl_batch(prefix, nb, i, lane));
    const int4 it = wl[(size_t)b * pools.Vp + (size_t)(i - prefix[b])];
    const int32_t u = __builtin_amdgcn_readfirstlane(it.x);
    const int32_t beg = __builtin_amdgcn_readfirstlane(it.y), end = __builtin_amdgcn_readfirstlane(it.z);
    const BatchDev B = batch_view(pools, b);
    push_visit(in_src, in_w, beg, end, B, b, u, lane, parity, cnt);
    if (lane == 0) B.act(parity)[u] = 0;
}

// phase 1 seed: d(s) = 0, the source's tree record (k_seed's), its lane in the change mask
__global__ void k_seed_push(GraphDev g, Pools pools) {
    const BatchDev B = batch_view(pools, blockIdx.y);
    const int j = threadIdx.x;
    if (j >= KL) return;
    const int32_t s = B.srcv[j];
    if (s < 0) return;
    const size_t idx = (size_t)s * KL + j;
    B.D[idx] = 0.0;
    rec_store(B.Q + idx, g.vfac[s], 0u, -1);
    atomicOr(&B.chm0[s], 1ull << j);
    B.act0[s] = 1;
}

// phase 2: P and the local tie bit of every reached (vertex, source) pair from the final
// distances; the sources activate their out-neighbours for fold round 1 (act parity 1)
__global__ __launch_bounds__(256) void k_pred_pass(const int64_t* __restrict__ in_ptr, const int32_t* __restrict__ in_src,
                                                   const double* __restrict__ in_w, Pools pools, int32_t V, int32_t nb,
                                                   int32_t nvb) {
    int32_t b, vt;
    if (!xcd_tile(flat_block(), nb, nvb, b, vt)) return;
    const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int32_t v = vt * 4 + wave;
    if (v >= V) return;
    const int lane = threadIdx.x & 63;
    const BatchDev B = batch_view(pools, b);
    const int32_t sv = B.srcv[lane];
    const size_t idx = (size_t)v * KL + lane;
    const double dv = B.D[idx];
    const bool src = sv == v;
    if (__ballot(src)) {  // a source vertex of some lane: fold round 1 starts at its out-neighbours
        for (int64_t x = in_ptr[v] + lane; x < in_ptr[v + 1]; x += 64) B.act1[in_src[x]] = 1;
    }
    if (!(dv < dinf()) && !src) B.Q[idx].h = 0u;  // unreached: never folded (k_fold tests H alone)
    if (!__ballot(dv < dinf() && !src)) return;
    const int32_t beg = (int32_t)in_ptr[v], end = (int32_t)in_ptr[v + 1];
    const gdouble* Dl = B.D + lane;
    double bc = dmax(), bdu = dinf();
    int32_t be = -1, bu = -1;
    bool tie = false;
    for (int32_t e = beg; e < end; e += 8) {
        int32_t u[8];
        double w[8], du[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            u[k] = in_src[e + k];
            w[k] = in_w[e + k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (e + k >= end) w[k] = dinf();
            du[k] = e + k < end ? Dl[(size_t)u[k] * KL] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) relax_arc(du[k], w[k], e + k, u[k], bc, bdu, be, bu, tie);
    }
    if (dv < dinf() && !src && sv >= 0) {
        // bc == dv: the distances are the fixed point of exactly this minimum
        B.Q[idx].p = be;
        B.Q[idx].h = HNOT | ((tie || bdu == bc) ? LTIE : 0u);
    }
}

// phase 3, fold round k: pairs whose predecessor's hop count is < k (finished in an earlier
// round; its H / R written by an earlier launch) take H = H(u) + 1 (+ taint) and
// R = R(u) * r(arc); a vertex with a finished lane activates its out-neighbours
__device__ __forceinline__ void fold_visit(const int32_t* __restrict__ in_src, const double* __restrict__ in_r,
                                           const int64_t* __restrict__ out_ptr, const int32_t* __restrict__ out_dst,
                                           const BatchDev& B, int32_t b, int32_t v, int lane, int32_t parity,
                                           uint32_t k, int32_t* __restrict__ cnt) {
    const size_t idx = (size_t)v * KL + lane;
    const Rec qv = rec_load(B.Q + idx);
    const uint32_t hv = qv.h;
    bool fin = false;
    if ((hv & HMASK) == HNOT) {
        const int32_t arc = qv.p;
        const int32_t u = in_src[arc];
        const Rec qu = rec_load(B.Q + (size_t)u * KL + lane);
        const uint32_t hu = qu.h;
        if ((hu & HMASK) < k) {
            const uint32_t taint = (hu & TAINT) | ((hv & LTIE) ? (TAINT | LTIE) : 0u);
            rec_store(B.Q + idx, qu.r * in_r[arc], (((hu & HMASK) + 1u) & HMASK) | taint, arc);
            fin = true;
        }
    }
    if (__ballot(fin)) {
        gbyte* act_nxt = B.act(parity ^ 1);
        for (int64_t x = out_ptr[v] + lane; x < out_ptr[v + 1]; x += 64) act_nxt[out_dst[x]] = 1;
        if (lane == 0) cnt[b] = 1;
    }
}

__global__ __launch_bounds__(256) void k_fold(const int32_t* __restrict__ in_src, const double* __restrict__ in_r,
                                              const int64_t* __restrict__ out_ptr, const int32_t* __restrict__ out_dst,
                                              Pools pools, int32_t V, int32_t nb, int32_t nvb, int32_t parity, uint32_t k,
                                              int32_t* __restrict__ cnt) {
    int32_t b, vt;
    if (!xcd_tile(flat_block(), nb, nvb, b, vt)) return;
    const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int32_t v = vt * 4 + wave;
    if (v >= V) return;
    const int lane = threadIdx.x & 63;
    const BatchDev B = batch_view(pools, b);
    gbyte* act_cur = B.act(parity);
    if (act_cur[v] == 0) return;
    if (lane == 0) act_cur[v] = 0;
    fold_visit(in_src, in_r, out_ptr, out_dst, B, b, v, lane, parity, k, cnt);
}

__global__ __launch_bounds__(256) void k_fold_wl(const int32_t* __restrict__ in_src, const double* __restrict__ in_r,
                                                 const int64_t* __restrict__ out_ptr, const int32_t* __restrict__ out_dst,
                                                 Pools pools, int32_t parity, uint32_t k, const int4* __restrict__ wl,
                                                 const int64_t* __restrict__ prefix, int32_t nb, int64_t S,
                                                 int32_t* __restrict__ cnt) {
    const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t L = flat_block();
    const int64_t i = (L & 7) * S + (L >> 3) * 4 + wave;
    const int64_t T = prefix[nb];
    if ((L >> 3) * 4 + wave >= S || i >= T) return;
    const int lane = threadIdx.x & 63;
    const int32_t b = __builtin_amdgcn_readfirstlane(wl_batch(prefix, nb, i, lane));
    const int32_t v = __builtin_amdgcn_readfirstlane(wl[(size_t)b * pools.Vp + (size_t)(i - prefix[b])].x);
    const BatchDev B = batch_view(pools, b);
    fold_visit(in_src, in_r, out_ptr, out_dst, B, b, v, lane, parity, k, cnt);
    if (lane == 0) B.act(parity)[v] = 0;
}

// Lexicographic (candidate, d(u)) minimum with heap-order tie detection, branch-free so the
// compiler keeps the per-destination state in scalars (a branchy form made it copy whole
// <8 x double> vectors around the control flow).
__device__ __forceinline__ void lex_update(double c, double du, int32_t u, double& bc, double& bdu, int32_t& bu,
                                           uint32_t& tie, uint32_t bit) {
    const bool same_c = c == bc;
    const bool take = (c < bc) | (same_c & (du < bdu));
    const bool eq = same_c & (du == bdu);
    bc = take ? c : bc;
    bdu = take ? du : bdu;
    bu = take ? u : bu;
    tie = take ? (tie & ~bit) : (eq ? (tie | bit) : tie);
}

// Dense form for complete-ish graphs (arcs >= V^2/4): W[u][v] = merged latency of arc
// u -> v (+inf if none), WI[u][v] = its in-arc index, rows padded to Vp = roundup(V, 8).
// One wave owns DT = 8 consecutive destinations and streams every u: one 512-byte row
// load of d(u) for the 64 sources feeds 8 candidates (8x less cache traffic than the CSR
// walk), the 8 weights arrive as one 64-byte scalar load.  A batch's tiles are all
// recomputed in a round iff any vertex of that batch changed in the previous round (in a
// complete-ish graph every vertex is an in-neighbour of every other).
constexpr int DT = 8;

__device__ __forceinline__ void relax_u(double du, double w, int32_t u, double& bc, double& bdu, int32_t& bu,
                                        uint32_t& tie, uint32_t bit) {
    const double c = du + w;
    if (c <= bc) {
        if (c < bc || du < bdu) {
            bc = c;
            bdu = du;
            bu = u;
            tie &= ~bit;
        } else if (du == bdu) {
            tie |= bit;
        }
    }
}

// Dense-tile epilogue shared by the full sweeps: record each destination's new best,
// its lex key d(pred) (BDU, read by the delta rounds), and the per-vertex change mask of
// the round (lane = source) that the next delta round walks; the batch counter gets the
// number of changed (vertex, source) pairs.
// Seed (pruned sweep, optional): the lane's rows of the permuted arc-index and reliability
// tables, WIp / WRp + srow, and R(s) = 1 - loss_v(s) of its source: when the seed candidate
// won (the predecessor is the source itself, whose record is H 0, R vfac(s): k_seed), the
// new record comes from one segment of those rows instead of the scattered WI / H / R
// gathers of finish_vertex.
struct SeedRows {
    const int32_t* WIp = nullptr;
    const double* WRp = nullptr;
    size_t srow = 0;
    double rs = 0.0;
};

template <int TDT = DT>
__device__ __forceinline__ void dense_epilogue(const BatchDev& B, int lane, int32_t sv, int32_t v0, int32_t V,
                                               const double* bc, const double* bdu, const int32_t* bu, uint32_t tie,
                                               const int32_t* __restrict__ WI, int32_t Vp,
                                               const double* __restrict__ in_r, int32_t parity,
                                               int32_t* __restrict__ cnt, int32_t b,
                                               const int32_t* vids = nullptr, const SeedRows& sr = SeedRows{},
                                               float* __restrict__ mdc = nullptr, bool seeded = false) {
    unsigned long long* chn = B.chm(parity);
    int32_t nch = 0;
    // mdc (the chained rounds' pruned delta round 1): the lane's minimum new D32 over its
    // changed pairs of these destinations, folded into the chunk's minDc entry (k_min_d32c's
    // value, computed here instead of in a pass over the change masks after the sweep)
    float mlo = __int_as_float(0x7f800000);
#pragma unroll
    for (int t = 0; t < TDT; ++t) {
        const int32_t v = vids ? vids[t] : v0 + t;  // vids: the pruned sweep's permuted tile
        if (v >= V) break;
        bool ch = false;
        if (bu[t] >= 0 && sv >= 0 && sv != v) {
            const size_t idx = (size_t)v * KL + lane;
            const uint32_t taint = (((tie >> t) & 1u) || bdu[t] == bc[t]) ? (TAINT | LTIE) : 0u;
            if (sr.WIp && bu[t] == sv && seeded && !taint) {
                // the seed candidate won untainted and the stored state is still the seed's
                // (k_seed_dense_t: d 0 + w, D32, {vfac(s) * WR, h 1, arc}, BDU 0): the record
                // below would equal it field for field, so nothing is read or written
            } else if (sr.WIp && bu[t] == sv) {
                // finish_vertex with hu = 0, ru = vfac(s): h = 1 (+ a local tie), r = vfac(s) * in_r[arc]
                // (WRp holds in_r of the same arc, the same double)
                const int32_t arc = sr.WIp[sr.srow + v0 + t];
                const double r = sr.rs * sr.WRp[sr.srow + v0 + t];
                const uint32_t h = 1u | taint;
                const Rec cur = rec_load(B.Q + idx);
                if (bc[t] != B.D[idx] || h != cur.h || r != cur.r || arc != cur.p) {
                    B.D[idx] = bc[t];
                    if (B.D32) B.D32[idx] = f32_key(bc[t]);
                    rec_store(B.Q + idx, r, h, arc);
                    ch = true;
                }
                B.BDU[idx] = bdu[t];
            } else {
                const int32_t arc = WI[(size_t)bu[t] * Vp + v];
                const Rec cur = rec_load(B.Q + idx);
                ch = finish_vertex(B, lane, v, arc, bu[t], bc[t], bdu[t], (tie >> t) & 1u, in_r, B.D[idx],
                                   cur.h, cur.r, cur.p);
                B.BDU[idx] = bdu[t];
            }
        }
        if (mdc && ch) mlo = fminf(mlo, f32_key(bc[t]));
        const unsigned long long m = __ballot(ch);
        if (lane == 0) chn[v] = m;
        nch += __popcll(m);
        __builtin_amdgcn_sched_barrier(0);  // keep the epilogues from being hoisted together (VGPRs)
    }
    if (nch && lane == 0) atomicAdd(&cnt[b], nch);
    // finite D32 >= 0: the bit patterns order like the values, and the NaN reset (0x7fc00000)
    // is above every one of them
    if (mdc && mlo < __int_as_float(0x7f800000)) atomicMin((int*)(mdc + lane), __float_as_int(mlo));
}

__global__ __launch_bounds__(256) void k_relax_dense(const double* __restrict__ W, const int32_t* __restrict__ WI,
                                                     int32_t Vp, const double* __restrict__ in_r,
                                                     Pools pools, int32_t V, int32_t nb,
                                                     int32_t ntb, int32_t parity, int32_t thresh,
                                                     const int32_t* __restrict__ cnt_prev,
                                                     int32_t* __restrict__ cnt) {
    int32_t b, vt;
    if (!xcd_tile(blockIdx.x, nb, ntb, b, vt)) return;
    if (cnt_prev[b] <= thresh) return;  // converged (0) or left to the delta round
    const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int32_t v0 = (vt * 4 + wave) * DT;
    if (v0 >= V) return;
    const int lane = threadIdx.x & 63;
    const BatchDev B = batch_view(pools, b);
    const int32_t sv = B.srcv[lane];
    const gdouble* Dl = B.D + lane;
    double bc[DT], bdu[DT];
    int32_t bu[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) {
        const double cd = B.D[(size_t)(v0 + t) * KL + lane];  // padding rows are +inf
        // the current distance bounds the new minimum from above (distances only decrease
        // and the stored predecessor still offers a candidate <= cd): seed the running best
        // with it so that only candidates c <= cd take the slow path (bdu = +inf: an equal
        // candidate is accepted as the first of its key)
        bc[t] = cd < dinf() ? cd : dmax();
        bdu[t] = dinf();
        bu[t] = -1;
    }
    uint32_t tie = 0;
    // DR rows per iteration: their DR row loads and DR 64-byte weight loads are all in
    // flight before the first compare (rows V.. are +inf padding; Vp is a multiple of 64)
    constexpr int DR = 4;
    for (int32_t u = 0; u < V; u += DR) {
        double du[DR], w[DR][DT];
#pragma unroll
        for (int r = 0; r < DR; ++r) {
            du[r] = Dl[(size_t)(u + r) * KL];
#pragma unroll
            for (int t = 0; t < DT; ++t) w[r][t] = W[(size_t)(u + r) * Vp + v0 + t];
        }
#pragma unroll
        for (int r = 0; r < DR; ++r) {
            double c[DT];
            unsigned long long hit = 0;  // wave-wide: the compares go straight to SGPR masks
#pragma unroll
            for (int t = 0; t < DT; ++t) {
                c[t] = du[r] + w[r][t];
                hit |= __ballot(c[t] <= bc[t]);
            }
            if (hit) {  // rare once the running bests sit at the current distances
#pragma unroll
                for (int t = 0; t < DT; ++t) lex_update(c[t], du[r], u + r, bc[t], bdu[t], bu[t], tie, 1u << t);
            }
        }
    }
    dense_epilogue(B, lane, sv, v0, V, bc, bdu, bu, tie, WI, Vp, in_r, parity, cnt, b);
}

// f32-filtered full sweep (default for dense graphs).  Every candidate is first tested in
// f32 against a conservative threshold: D32 = d rounded down (NaN when unreached), W32 = w
// rounded down (NaN when no arc), thr = bc rounded up plus 4 ulps (+inf when unreached).
// fl32(D32 + W32) <= thr is implied by fl64(d + w) <= bc (the roundings lose < 2^-22
// relative), so a failing filter proves the exact candidate cannot beat or tie the running
// best and the lane can skip it; rows where any lane passes redo the exact f64
// lexicographic update.  The f32 stream costs half the VALU cycles of f64 add + compare and
// half the bytes per row.

// One full sweep, f32-filtered and LDS-staged.  A 256-thread block owns 4*TDT consecutive
// destinations (wave w: TDT of them) of one batch; the rows u stream through LDS in chunks
// of SRS rows, double-buffered: the block's global loads of chunk k+1 (D32 rows, lane =
// source, and the block's W32 columns) are in flight while chunk k is filtered.
//  * lexicographic state starts at the seed candidate (source -> v arc: fl(0 + w), d = 0,
//    u = s), so row u = s is skipped for that lane instead of re-offered;
//  * filter per row: a lane passes iff D32(u) <= max_t fl32(thr_t - W32(u, v_t)), one
//    subtraction per candidate plus a max tree (conservative: see f32_thr);
//  * rows where any lane passes are collected and, at the end of the chunk, re-evaluated
//    exactly in f64 (D and W from global memory) in row order -- the same lexicographic
//    minimum and tie flag as a sequential scan.
constexpr int SRS = 32;  // rows per LDS chunk
constexpr int FTDT = 8;  // f32 full sweep: destinations per wave (block: 4 * FTDT; 4 was slower: 4.63 vs 3.8 ms on C2;
                         // 16: 122 VGPRs and 4 waves per SIMD in the chunk loop, spills in the exact pass)

// Occupancy: LDS (24 KB per block) allows 6 blocks = 6 waves per SIMD, and 80 VGPRs fit 6
// (the kernel wants 82, i.e. 5 waves); waves_per_eu(6) spills 3 dwords outside the chunk
// loop and buys a sixth wave: 3.89 -> 3.68 ms on C2 together with the unrolls below.
// H16 (OPT_DENSE_W16, chunk loop only): the filter key is the 16-bit W16p table (latency rounded
// toward -inf to fp16, saturating at 65504; NaN if no arc) instead of W32p: half the LDS slab
// (8 blocks per CU instead of 6) and half the table (202 MB on C2, inside the Infinity Cache).
// W16 <= W32 <= w keeps the filter conservative; a passing row tightens the
// thresholds with an upper bound of w (one fp16 ulp up; +inf past the saturation).
// GL (r06, OPT_SWEEP_GLDS, chunk loop only): the chunk's D32 rows and W32 slab go straight from
// global memory into the LDS slot with global_load_lds_dwordx4 (LDS-DMA), issued for chunk
// k + 1 into the free slot right after the barrier that ends chunk k - 1; the same two slots and
// the same LDS image as the register staging (one wave-instruction fills 4 contiguous D32 rows,
// or 8 W32 slab rows), no staging VGPRs and no ds_write pass.
template <int TDT, int XR, int TB, bool PR, int PH = 0, int NW = 4, bool H16 = false, bool GL = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(TB == 1 ? (NW == 8 ? 8 : 6) : 1))) void k_relax_dense_f(const float* __restrict__ W32, const double* __restrict__ W,
                                                       const int32_t* __restrict__ WI, int32_t Vp,
                                                       const double* __restrict__ in_r, Pools pools, int32_t V,
                                                       int32_t nb, int32_t ntb, int32_t parity, int32_t thresh,
                                                       const int32_t* __restrict__ cnt_prev,
                                                       int32_t* __restrict__ cnt,
                                                       unsigned long long* __restrict__ prof,
                                                       uint32_t* __restrict__ hitlog,
                                                       const int32_t* __restrict__ perm,
                                                       const float* __restrict__ minW,
                                                       const float* __restrict__ minD,
                                                       const int32_t* __restrict__ ipos,
                                                       const int32_t* __restrict__ WIp,
                                                       const double* __restrict__ WRp,
                                                       const double* __restrict__ vfac, int32_t spiral,
                                                       int32_t win1, float* __restrict__ mdc_out,
                                                       const int32_t* __restrict__ border = nullptr,
                                                       uint32_t* __restrict__ bweight = nullptr,
                                                       float* __restrict__ thr_io = nullptr, int32_t seeded = 0) {
    // PR (pruned): rows, columns, W32 and W are in the locality order `perm` (W32 and W here are
    // the permuted copies W32p[i][j] = W32[perm i][perm j], Wp likewise; ipos = perm's inverse):
    // a lane's seed weights W(s, v_t) over the wave's 8 destinations are then one 64-byte
    // segment, not 8 scattered lines, and so is a logged row's W(u, v_0..v_7).  A wave skips a chunk outright when no
    // lane can pass any of its rows: min D32 over the chunk's rows (minD, per lane) exceeds
    // max_t fl32(thr_t - minW_t), minW_t = min W32 over the chunk's rows in column v_t.  Every
    // row's filter bound max_t fl32(thr_t - W32(u, v_t)) is <= that (rounding is monotone), and
    // D32(u) >= min D32, so the skip is exact; minD is taken before the sweep, which is the
    // same as having read those rows' pre-sweep values (later changes reach the delta round
    // through the change masks).
    // NW waves per block: 4.  (8 for the split chunk loop -- one staged D32 chunk for 8 waves,
    // 8 waves per SIMD -- measured 3.57 vs 3.42-3.43 ms on C2, r03s: a block-wide chunk skip
    // then needs all 8 waves dead, so more chunks are staged.)
    static_assert(NW == 4 || (NW == 8 && PH == 1), "8-wave blocks only for the chunk loop");
    static_assert(!H16 || (PH == 1 && PR && TB == 1 && NW == 4 && TDT == 8), "W16: the pruned chunk loop alone");
    static_assert(!GL || (PH == 1 && PR && TB == 1 && !H16), "LDS-DMA staging: the pruned f32 chunk loop alone");
    constexpr int NT = 64 * NW;  // threads per block
    constexpr int BW = NW * TDT;  // block columns
    constexpr int WQ = BW / 4;   // float4 per W32 chunk row
    // all of the kernel's LDS in ONE __shared__ object: beside LDS-DMA (GL), a second object
    // made hipcc wait for every outstanding DMA (vmcnt(0)) before the chunk's first LDS read
    struct SweepLds {
        float d[2][TB][SRS * KL];
        float w[2][H16 ? SRS * BW / 2 : SRS * BW];
        unsigned long long win[2];
    };
    __shared__ __attribute__((aligned(16))) SweepLds slds;
    auto& sD = slds.d;
    auto& sW = slds.w;
    int32_t grp, vt;
    // heavy-first (PH 1): border maps the hardware block to a (batch, tile) item of the same
    // XCD, the items of each XCD in decreasing chunk counts of the previous sweep (k_heavy_order),
    // so the longest blocks start first and the ragged tail shrinks; any order is exact
    const int64_t Lb = border ? (int64_t)border[blockIdx.x] : (int64_t)blockIdx.x;
    if (!xcd_tile(Lb, (nb + TB - 1) / TB, ntb, grp, vt)) return;  // block-uniform exits only (barriers below)
    const int32_t b0 = grp * TB;  // this block's TB batches
    bool live[TB];
    int32_t first = -1;
#pragma unroll
    for (int k = 0; k < TB; ++k) {
        live[k] = b0 + k < nb && cnt_prev[b0 + k] > thresh;
        if (live[k] && first < 0) first = b0 + k;
    }
    if (first < 0 || vt * BW >= V) {
        if (PH == 1 && bweight && threadIdx.x == 0) bweight[Lb] = 0u;
        return;
    }
    const int32_t vb = vt * BW;
    const int32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int32_t v0 = vb + wave * TDT;
    int32_t vid[TDT];  // this wave's destinations (vertex ids)
#pragma unroll
    for (int t = 0; t < TDT; ++t) vid[t] = PR ? perm[v0 + t] : v0 + t;
    // PH: 0 = the whole sweep in one kernel; 1 = the f32 chunk loop alone (the hit log out);
    // 2 = the exact f64 pass and epilogue alone (the hit log in).  Split, the chunk loop holds
    // no f64 lexicographic state (40 VGPRs) and the exact pass no staging registers.
    BatchDev B[TB];
    int32_t sv[TB];
    double bc[TB][TDT], bdu[TB][TDT];
    int32_t bu[TB][TDT];
    float thr[TB][TDT];
    uint32_t tie[TB];
#pragma unroll
    for (int k = 0; k < TB; ++k) {
        // a batch of the group that is past nb or left to the delta round stages a live
        // batch's rows with NaN thresholds: it never passes and is never written
        B[k] = batch_view(pools, live[k] ? b0 + k : first);
        sv[k] = B[k].srcv[lane];
        tie[k] = 0;
        const size_t wrow = (size_t)(PR ? (sv[k] >= 0 ? ipos[sv[k]] : 0) : sv[k]) * Vp;  // the source's W row
#pragma unroll
        for (int t = 0; t < TDT; ++t) {
            const int32_t v = vid[t];
            const double ws = (sv[k] >= 0 && sv[k] != v) ? W[wrow + (PR ? v0 + t : v)] : dinf();
            if (ws < dinf()) {
                bc[k][t] = 0.0 + ws;
                bdu[k][t] = 0.0;
                bu[k][t] = sv[k];
            } else {
                bc[k][t] = dmax();
                bdu[k][t] = dinf();
                bu[k][t] = -1;
            }
            if constexpr (PH != 2) {
                const double cd = B[k].D[(size_t)v * KL + lane];  // padding rows are +inf
                // a lane without a source (a partial batch) never passes: NaN, so it cannot hold a
                // pruned wave's chunk skip back either
                thr[k][t] = live[k] && sv[k] >= 0 ? f32_thr(cd < bc[k][t] ? cd : bc[k][t]) : __int_as_float(0x7fc00000);
            }
        }
    }
    const int32_t nrows = (V + SRS - 1) / SRS * SRS;  // <= Vp: rows past V are NaN padding
    const int32_t nchunks = nrows / SRS;
    // this wave's hit log [TB][nchunks] of row masks, indexed by (batch group, wave tile) so the
    // exact-pass kernel finds it whatever block shape wrote it
    // per batch and wave tile: the log rows of batch b0 + k (the same place whatever TB the
    // chunk loop ran with, so the exact pass may run one batch per wave)
    const auto hl_at = [&](int k) { return ((size_t)(b0 + k) * (size_t)(Vp / TDT) + (size_t)(v0 / TDT)) * nchunks; };
    if constexpr (PH != 2) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const f4 gf4;
    // chunk fill: TB x D32 rows = SRS*64 floats each (2 float4 per thread), W32 = SRS*BW floats
    constexpr int DQ = SRS * KL / 4 / NT;       // float4 of one batch's D32 chunk per thread
    constexpr int WQT = (SRS * WQ + NT - 1) / NT;  // float4 of W32 per thread
    static_assert(DQ * NT * 4 == SRS * KL, "the D32 chunk is whole float4s per thread");
    f4 pd[TB][DQ], pw[WQT];  // register staging (unused with GL)
    // W16: a chunk's W16 slab is SRS rows x BW halves = SRS * BW / 8 16-byte pieces
    constexpr int WQ16 = BW / 8;
    constexpr int WQT16 = (SRS * WQ16 + NT - 1) / NT;
    // PR: the chunk's skip bounds (md: min D32 per lane and batch, mw: min W32 of the
    // wave's tile columns)
    float mdn[TB], mdc[TB], mwn[TDT], mwc[TDT];
    const int32_t ncol = Vp;  // columns per chunk row of minW
    // PR: chunks in the order vt, vt+1, .., wrapping: the block's own tile (its destinations'
    // nearest rows) first, which gives unreached and arc-less (t, s) pairs a tight threshold
    // before the far chunks are tested
    const int32_t c0 = PR ? (int32_t)((int64_t)vt * BW / SRS % nchunks) : 0;  // the chunk holding the tile
    // spiral: c0, c0+1, c0-1, c0+2, c0-2, .. (the nearest rows on both sides of the tile
    // first), then the longer side's remaining chunks; otherwise c0, c0+1, .. wrapping
    const int32_t sL = c0, sR = nchunks - 1 - c0, sM = sL < sR ? sL : sR;
    auto chunk_of = [&](int32_t j) {
        if (!PR) return j;
        if (!spiral) return (c0 + j) % nchunks;
        if (j <= 2 * sM) return j == 0 ? c0 : ((j & 1) ? c0 + (j + 1) / 2 : c0 - j / 2);
        return sR > sL ? c0 + j - sM : c0 - (j - sM);
    };
    // PR: the vertices of this thread's rows of the chunk of order index j (perm, an
    // L2-resident 40 KB table).  Loaded one chunk ahead of the fetch that uses them, so the
    // D32 row loads never wait on a dependent perm load.
    auto perm_of = [&](int32_t j, int32_t* prow) {
        if (PR) {
            const int32_t u0 = chunk_of(j) * SRS;
#pragma unroll
            for (int i = 0; i < DQ; ++i) prow[i] = perm[u0 + (threadIdx.x + i * NT) / (KL / 4)];
        }
    };
    // fetch the chunk of order index j into registers (rows in the locality order: prow
    // holds each row's vertex, from perm_of)
    // GL: the same chunk straight into LDS slot `buf` (wave-uniform LDS bases, lane-linear)
    auto fetch_gl = [&](int32_t j, const int32_t* prow, int buf) {
        if constexpr (GL) {
            typedef __attribute__((address_space(1))) void gv;
            typedef __attribute__((address_space(3))) void lv;
            const int32_t c = chunk_of(j);
            const int32_t u0 = c * SRS;
            const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
            for (int i = 0; i < DQ; ++i)  // rows w*4 + 16i .. +3: 1 KB of the slot per wave-instruction
                __builtin_amdgcn_global_load_lds((gv*)(B[0].D32 + (size_t)prow[i] * KL + (size_t)(l % (KL / 4)) * 4),
                                                 (lv*)&sD[buf][0][(w * 4 + 16 * i) * KL], 16, 0, 0);
            static_assert(WQT == 1 && SRS * WQ == NT, "one W32 slab piece per thread");
            __builtin_amdgcn_global_load_lds((gv*)((const gfloat*)W32 + (size_t)(u0 + (int)threadIdx.x / WQ) * Vp + vb +
                                                   ((int)threadIdx.x % WQ) * 4),
                                             (lv*)&sW[buf][w * 256], 16, 0, 0);
            mdn[0] = minD[((size_t)(live[0] ? b0 : first) * nchunks + c) * KL + lane];
#pragma unroll
            for (int t = 0; t < TDT; ++t) mwn[t] = minW[(size_t)c * ncol + v0 + t];
        }
    };
    auto fetch = [&](int32_t j, const int32_t* prow) {
        if constexpr (GL) return;
        const int32_t c = chunk_of(j);
        const int32_t u0 = c * SRS;
#pragma unroll
        for (int k = 0; k < TB; ++k)
#pragma unroll
            for (int i = 0; i < DQ; ++i) {
                const int e = threadIdx.x + i * NT;  // float4 index within the chunk
                if (PR)
                    pd[k][i] = *(gf4*)(B[k].D32 + (size_t)prow[i] * KL + (size_t)(e % (KL / 4)) * 4);
                else
                    pd[k][i] = *(gf4*)(B[k].D32 + (size_t)u0 * KL + (size_t)e * 4);
            }
        if (PR) {
#pragma unroll
            for (int k = 0; k < TB; ++k)
                mdn[k] = minD[((size_t)(live[k] ? b0 + k : first) * nchunks + c) * KL + lane];
#pragma unroll
            for (int t = 0; t < TDT; ++t) mwn[t] = minW[(size_t)c * ncol + v0 + t];
        }
        if constexpr (H16) {
#pragma unroll
            for (int i = 0; i < WQT16; ++i) {
                const int e = threadIdx.x + i * NT;
                if (e < SRS * WQ16) {
                    const int r = e / WQ16, c = e % WQ16;
                    typedef __attribute__((address_space(1))) const uint16_t gu16;
                    pw[i] = *(gf4*)((gu16*)W32 + (size_t)(u0 + r) * Vp + vb + c * 8);
                }
            }
        } else {
#pragma unroll
        for (int i = 0; i < WQT; ++i) {
            const int e = threadIdx.x + i * NT;
            if (e < SRS * WQ) {
                const int r = e / WQ, c = e % WQ;
                pw[i] = *(gf4*)((const gfloat*)W32 + (size_t)(u0 + r) * Vp + vb + c * 4);
            }
        }
        }
    };
    auto stash = [&](int buf) {
        if constexpr (GL) return;
#pragma unroll
        for (int k = 0; k < TB; ++k)
#pragma unroll
            for (int i = 0; i < DQ; ++i) *(f4*)&sD[buf][k][(threadIdx.x + i * NT) * 4] = pd[k][i];
        if constexpr (H16) {
#pragma unroll
            for (int i = 0; i < WQT16; ++i) {
                const int e = threadIdx.x + i * NT;
                if (e < SRS * WQ16) *(f4*)&sW[buf][e * 4] = pw[i];
            }
        } else {
#pragma unroll
        for (int i = 0; i < WQT; ++i) {
            const int e = threadIdx.x + i * NT;
            if (e < SRS * WQ) *(f4*)&sW[buf][e * 4] = pw[i];
        }
        }
    };
    auto advance = [&]() {
        if (PR) {
#pragma unroll
            for (int k = 0; k < TB; ++k) mdc[k] = mdn[k];
#pragma unroll
            for (int t = 0; t < TDT; ++t) mwc[t] = mwn[t];
        }
    };
    // PR: block-wide chunk skipping.  Most chunk iterations of a pruned sweep are dead for
    // all four waves of a block at once (C2: 71 %), and a dead iteration still cost a load
    // round trip and a barrier.  So the block decides, for a window of chunks at a time and
    // with its current thresholds, which chunks any of its waves can pass (the per-wave chunk
    // bound below, evaluated for the window: lane = source, one minD load per chunk), ORs the
    // four waves' masks in LDS and loads, stages and visits only those.  Thresholds only
    // tighten during the sweep, so a chunk dead at the window's evaluation is dead for the
    // rest of it: the skip is exact (the per-wave test inside a live chunk still uses the
    // newest thresholds).  Window 0 is the block's own chunk alone (it tightens the
    // thresholds most), then windows of 64.  A dead chunk's hit log entries are zeroed at
    // the evaluation.
    auto& sWin = slds.win;
    if (PR && threadIdx.x == 0) sWin[0] = sWin[1] = 0ull;
    __syncthreads();
    int32_t cur_win = -1;
    unsigned long long cur_live = 0ull;
    // win1 (bits 0-7) > 0: window 1 is the win1 chunks next in the order (the tile's nearest
    // neighbours), so the far windows are evaluated with the thresholds they left; bits 8-15:
    // the far windows' size (0 = 64, the live mask's width)
    const int32_t w1 = (win1 & 0xff) < 64 ? (win1 & 0xff) : 0;
    const int32_t wf = ((win1 >> 8) & 0xff) > 0 && ((win1 >> 8) & 0xff) < 64 ? (win1 >> 8) & 0xff : 64;
    auto win_of = [&](int32_t j) {
        if (j == 0) return 0;
        if (w1) return j <= w1 ? 1 : 2 + (j - 1 - w1) / wf;
        return 1 + (j - 1) / wf;
    };
    auto win_base = [&](int32_t wi) {
        if (wi == 0) return 0;
        if (w1) return wi == 1 ? 1 : 1 + w1 + (wi - 2) * wf;
        return 1 + (wi - 1) * wf;
    };
    auto win_size = [&](int32_t wi) { return wi == 0 ? 1 : (w1 && wi == 1 ? w1 : wf); };
    constexpr int WG = 4;  // chunks whose bounds are in flight at once in a window evaluation (8: 64 SGPRs of
                           // minW, 149 SGPR spills reloaded by readlane in the chunk loop, sweep +6 %)
    auto eval_window = [&](int32_t wi) -> unsigned long long {
        const int32_t base = win_base(wi);
        const int32_t nw = nchunks - base < win_size(wi) ? nchunks - base : win_size(wi);
        unsigned long long wm = 0ull;
        // lane i's chunk of the window, computed once in VGPRs (r06: the spiral order's index
        // arithmetic per chunk in SGPRs was ~50 scalar instructions, about a third of the
        // chunk loop's instruction stream); each chunk's index is then one readlane
        const int32_t cl = chunk_of(base + (lane < nw ? lane : 0));
        for (int32_t j0 = 0; j0 < nw; j0 += WG) {
            float md[TB][WG], mw8[WG][TDT];
#pragma unroll
            for (int jj = 0; jj < WG; ++jj) {
                const int32_t c = __builtin_amdgcn_readlane(cl, j0 + jj < nw ? j0 + jj : 0);
#pragma unroll
                for (int k = 0; k < TB; ++k)
                    md[k][jj] = minD[((size_t)(live[k] ? b0 + k : first) * nchunks + c) * KL + lane];
#pragma unroll
                for (int t = 0; t < TDT; ++t) mw8[jj][t] = minW[(size_t)c * ncol + v0 + t];
            }
#pragma unroll
            for (int jj = 0; jj < WG; ++jj) {
                bool p = false;
#pragma unroll
                for (int k = 0; k < TB; ++k) {
                    float tm = thr[k][0] - mw8[jj][0];
#pragma unroll
                    for (int t = 1; t < TDT; ++t) tm = fmaxf(tm, thr[k][t] - mw8[jj][t]);
                    p |= md[k][jj] <= tm;
                }
                if (__ballot(p) && j0 + jj < nw) wm |= 1ull << (j0 + jj);
            }
        }
        if (threadIdx.x == 0) sWin[(wi + 1) & 1] = 0ull;  // the next window's slot: nobody ORs into it before this barrier
        if (lane == 0 && wm) atomicOr(&sWin[wi & 1], wm);
        __syncthreads();
        const unsigned long long lv =
            ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(sWin[wi & 1] >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sWin[wi & 1]);
        if (lane < nw && !((lv >> lane) & 1ull)) {
            const int32_t c = cl;
#pragma unroll
            for (int k = 0; k < TB; ++k) hitlog[hl_at(k) + c] = 0u;
        }
        return lv;
    };
    // order index of the next chunk to visit at or after `from`, -1 past the end
    auto next_live = [&](int32_t from) -> int32_t {
        if (!PR) return from < nchunks ? from : -1;
        while (from < nchunks) {
            const int32_t wi = win_of(from);
            if (wi != cur_win) {
                cur_win = wi;
                cur_live = eval_window(wi);
            }
            const unsigned long long m = cur_live & (~0ull << (from - win_base(wi)));
            if (m) return win_base(wi) + __builtin_ctzll(m);
            from = win_base(wi + 1);
        }
        return -1;
    };
    // chunks in flight: itc (in LDS, filtered this iteration), itn (its loads issued this
    // iteration, staged at its end) and itn2 (its rows' perm entries loaded this iteration)
    int32_t prow_n[DQ];
    uint32_t nvis = 0;  // chunks this block staged (its weight for the next sweep's order)
    int32_t itc = next_live(0);
    if (itc >= 0) {
        perm_of(itc, prow_n);
        if constexpr (GL) fetch_gl(itc, prow_n, 0);
        fetch(itc, prow_n);
        stash(0);
        advance();
    }
    int32_t itn = itc >= 0 ? next_live(itc + 1) : -1;
    if (itn >= 0) perm_of(itn, prow_n);
    __syncthreads();
    int bufc = 0;
    while (itc >= 0) {
        const int32_t c = chunk_of(itc);
        const int32_t u0 = c * SRS;
        const int cur = bufc;
        const bool more = itn >= 0;
        if (more) {
            if constexpr (GL) fetch_gl(itn, prow_n, cur ^ 1);  // slot cur ^ 1: read last iteration, before its barrier
            fetch(itn, prow_n);
        }
        // block-uniform (a window evaluation holds a barrier); a window evaluated one chunk
        // earlier uses slightly older thresholds, which only skips less
        const int32_t itn2 = more ? next_live(itn + 1) : -1;
        if (itn2 >= 0) perm_of(itn2, prow_n);
        bool run = true;
        if (PR) {
            bool p = false;
#pragma unroll
            for (int k = 0; k < TB; ++k) {
                float tm = thr[k][0] - mwc[0];
#pragma unroll
                for (int t = 1; t < TDT; ++t) tm = fmaxf(tm, thr[k][t] - mwc[t]);
                p |= mdc[k] <= tm;
            }
            run = __ballot(p) != 0;
        }
        // per batch: bit r = row u0 + r passed the filter in some lane.  One broadcast read
        // of the row's TDT weights serves all TB batches.  A passing row tightens the
        // thresholds at once with an f32 upper bound of its candidates -- the exact f64 work
        // is deferred to after the sweep, so no wave ever waits on a global load inside the
        // chunk loop (that wait would hold the whole block at the next barrier).
        uint32_t hits[TB];
#pragma unroll
        for (int k = 0; k < TB; ++k) hits[k] = 0;
        // PH 1 (the chunk loop alone has VGPRs to spare): each row's LDS reads are issued one
        // row ahead, so they are in flight while the previous row is filtered and votes
        constexpr bool RP = PH == 1 && !H16;
        f4 wn[TDT / 4];
        float dn[TB];
        // W16: the row's 8 halves (one 16-byte LDS read), widened to f32
        auto w16_row = [&](int r, f4* out) {
            typedef _Float16 h8 __attribute__((ext_vector_type(8)));
            typedef float f8 __attribute__((ext_vector_type(8)));
            const h8 h = *(const h8*)((const uint16_t*)&sW[cur][0] + r * BW + wave * TDT);
            const f8 f = __builtin_convertvector(h, f8);
            out[0] = f4{f[0], f[1], f[2], f[3]};
            out[1] = f4{f[4], f[5], f[6], f[7]};
        };
        // RP: the W32 slab's row base in a VGPR kept live across the chunk (rows are immediate
        // offsets from it; without the pin the compiler re-materialises it from an SGPR per row)
        typedef __attribute__((address_space(3))) const f4 lf4;
        uint32_t wbase = (uint32_t)(uintptr_t)(lf4*)&sW[cur][wave * TDT];
        if constexpr (RP) asm volatile("" : "+v"(wbase));
        auto lds_row = [&](int r) {
            if constexpr (H16) {
                w16_row(r, wn);
            } else if constexpr (RP) {
#pragma unroll
            for (int j = 0; j < TDT / 4; ++j) wn[j] = *(lf4*)(uintptr_t)(wbase + (uint32_t)(r * BW + 4 * j) * 4u);
            } else {
            const f4* wr = (const f4*)&sW[cur][r * BW + wave * TDT];
#pragma unroll
            for (int j = 0; j < TDT / 4; ++j) wn[j] = wr[j];
            }
#pragma unroll
            for (int k = 0; k < TB; ++k) dn[k] = sD[cur][k][r * KL + lane];
        };
        if (RP && run) lds_row(0);
#pragma unroll 8  // rows per unrolled step (2: +3 %, 1: +6 %)
        for (int r = 0; r < (run ? SRS : 0); ++r) {
            f4 w4[TDT / 4];
            float dk[TB];
            if constexpr (RP) {
#pragma unroll
                for (int j = 0; j < TDT / 4; ++j) w4[j] = wn[j];
#pragma unroll
                for (int k = 0; k < TB; ++k) dk[k] = dn[k];
                if (r + 1 < SRS) lds_row(r + 1);
            } else if constexpr (H16) {
                w16_row(r, w4);
#pragma unroll
                for (int k = 0; k < TB; ++k) dk[k] = sD[cur][k][r * KL + lane];
            } else {
                const f4* wr = (const f4*)&sW[cur][r * BW + wave * TDT];
#pragma unroll
                for (int j = 0; j < TDT / 4; ++j) w4[j] = wr[j];
#pragma unroll
                for (int k = 0; k < TB; ++k) dk[k] = sD[cur][k][r * KL + lane];
            }
#pragma unroll
            for (int k = 0; k < TB; ++k) {
                const float du = dk[k];
                // slacks thr_t - w_t two at a time (v_pk_add_f32), their max as a chain of
                // 3-input maxima (v_max3)
                typedef float f2 __attribute__((ext_vector_type(2)));
                float x[TDT];
#pragma unroll
                for (int j = 0; j < TDT / 4; ++j) {
                    const f2 a = f2{thr[k][4 * j], thr[k][4 * j + 1]} - f2{w4[j].x, w4[j].y};
                    const f2 c = f2{thr[k][4 * j + 2], thr[k][4 * j + 3]} - f2{w4[j].z, w4[j].w};
                    x[4 * j] = a.x;
                    x[4 * j + 1] = a.y;
                    x[4 * j + 2] = c.x;
                    x[4 * j + 3] = c.y;
                }
                float g = fmaxf(fmaxf(x[0], x[1]), x[2]);
#pragma unroll
                for (int t = 3; t + 1 < TDT; t += 2) g = fmaxf(fmaxf(g, x[t]), x[t + 1]);
                if (TDT % 2 == 0) g = fmaxf(g, x[TDT - 1]);
                // (a pass tightens the thresholds at once: deferring that to the chunk's end, r06,
                // logged far more rows -- sweep 2.36 -> 2.79 ms)
                if (__ballot(du <= g)) {
                    hits[k] |= 1u << r;
                    // c_exact <= fl32(D32 + W32) * (1 + 2^-22) <= that + 5 ulps, and f32_thr
                    // adds 4 ulps: every lane may lower thr_t to bits(c32) + 9 (a no-op where
                    // the row did not pass)
#pragma unroll
                    for (int j = 0; j < TDT / 4; ++j) {
                        const float wj[4] = {w4[j].x, w4[j].y, w4[j].z, w4[j].w};
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            // branch-free (v_cndmask): an infinite or NaN candidate, or a bound
                            // that would wrap past +inf into a NaN pattern, leaves thr as it is
                            float wu = wj[i];
                            if constexpr (H16) {
                                // an upper bound of w from its fp16 round-down: one fp16 ulp up
                                // (2^13 f32 ulps), 2^-14 below the normal range, +inf at the
                                // saturation value
                                wu = wu < 6.103515625e-05f ? 6.103515625e-05f
                                     : (wu >= 65504.0f ? __int_as_float(0x7f800000)
                                                        : __int_as_float(__float_as_int(wu) + (1 << 13)));
                                wu = wj[i] == wj[i] ? wu : wj[i];  // NaN (no arc) stays NaN
                            }
                            const float c32 = du + wu;
                            const float nb = __int_as_float(__float_as_int(c32) + 9);
                            float& th = thr[k][4 * j + i];
                            th = ((c32 < __int_as_float(0x7f800000)) & (nb < th)) ? nb : th;
                        }
                    }
                }
            }
        }
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < TB; ++k) hitlog[hl_at(k) + (u0 / SRS)] = hits[k];
        }
        if (more) {
            stash(cur ^ 1);
            advance();
        }
        __syncthreads();
        bufc ^= 1;
        itc = itn;
        itn = itn2;
        ++nvis;
    }
    if (PH == 1 && bweight && threadIdx.x == 0) bweight[Lb] = nvis;
    // refilter (OPT_SWEEP_REFILTER): the final f32 thresholds go to the exact pass, which
    // re-tests every logged row against them first (rows logged while a threshold was still
    // falling mostly no longer pass)
    if (PH == 1 && thr_io) {
#pragma unroll
        for (int t = 0; t < TDT; ++t) thr_io[(hl_at(0) / nchunks * TDT + t) * KL + lane] = thr[0][t];
    }
    }  // PH != 2
    if constexpr (PH == 1) return;
#ifdef SHADOWTOPO_EXP_PH2_CAP
    int32_t exp_rows = 0;
#endif
    // exact f64 pass over the logged rows of each batch, in row order, XR rows' loads in
    // flight at once: d(u) for the 64 sources and W(u, v0..v0+TDT) (lane j holds column
    // j % TDT, broadcast by readlane).  A source's own row never passes (its D32 is NaN: the
    // seed candidate is in the lexicographic state already).
#pragma unroll
    for (int k = 0; k < TB; ++k) {
        if (!live[k]) continue;
        const uint32_t* hl = hitlog + hl_at(k);
        const gdouble* Dl = B[k].D + lane;
        float thr_f[TDT];  // refilter: the chunk loop's final thresholds of this lane
#pragma unroll
        for (int t = 0; t < TDT; ++t)
            thr_f[t] = (PH == 2 && thr_io) ? thr_io[(hl_at(k) / nchunks * TDT + t) * KL + lane] : 0.0f;
        for (int32_t c0 = 0; c0 < nchunks; c0 += 64) {
            const uint32_t e = (c0 + lane < nchunks) ? hl[c0 + lane] : 0u;
            unsigned long long cm = __ballot(e != 0u);
            while (cm) {
                const int ci = __builtin_ctzll(cm);
                cm &= cm - 1;
                unsigned long long hrows = (uint32_t)__builtin_amdgcn_readlane((int)e, ci);
                const int32_t u0 = (c0 + ci) * SRS;
                // refilter: bit r = this lane passes row u0 + r (the f64 distance is fetched
                // only for passing lanes: a failing lane's candidate exceeds the final key)
                unsigned long long lpass = ~0ull;
                if (PH == 2 && PR && TB == 1 && thr_io) {
                    // drop the logged rows that no lane passes under the chunk loop's FINAL
                    // thresholds (D32(u) <= max_t fl32(thr_t - W32(u, v_t)), the chunk loop's own
                    // filter): every row whose exact candidate meets or beats the final key
                    // passes (thr_final >= f32_thr(bc_final), k_relax_dense_f's invariant), so
                    // the rows dropped cannot change the final lexicographic state; 4 rows' loads
                    // in flight per step
                    unsigned long long keep = 0ull, todo = hrows;
                    lpass = 0ull;
                    while (todo) {
                        int32_t rr[4];
                        float dq[4], wq[4][TDT];
#pragma unroll
                        for (int x = 0; x < 4; ++x) {
                            rr[x] = -1;
                            if (todo) {
                                rr[x] = __builtin_ctzll(todo);
                                todo &= todo - 1;
                            }
                            const int32_t rp = u0 + (rr[x] >= 0 ? rr[x] : 0);
                            dq[x] = B[k].D32[(size_t)perm[rp] * KL + lane];
#pragma unroll
                            for (int t = 0; t < TDT; ++t) wq[x][t] = W32[(size_t)rp * Vp + v0 + t];
                        }
#pragma unroll
                        for (int x = 0; x < 4; ++x) {
                            float g = thr_f[0] - wq[x][0];
#pragma unroll
                            for (int t = 1; t < TDT; ++t) g = fmaxf(g, thr_f[t] - wq[x][t]);
                            const bool p = rr[x] >= 0 && dq[x] <= g;
                            if (__ballot(p)) keep |= 1ull << rr[x];
                            lpass |= p ? 1ull << (rr[x] & 63) : 0ull;
                        }
                    }
                    hrows = keep;
                }
                if (prof && lane == 0) atomicAdd(&prof[0], (unsigned long long)__popcll(hrows));
#ifdef SHADOWTOPO_EXP_PH2_NOROWS
                hrows = 0;  // timing experiment only (wrong results): the exact pass without its rows
#endif
#ifdef SHADOWTOPO_EXP_PH2_CAP
                // timing experiment only (wrong results): at most CAP exact rows per wave
                if (exp_rows >= SHADOWTOPO_EXP_PH2_CAP) hrows = 0;
                exp_rows += __popcll(hrows);
#endif
                while (hrows) {
                    int32_t ur[XR], rp[XR];
                    int nr = 0;
#pragma unroll
                    for (int x = 0; x < XR; ++x) {
                        rp[x] = u0;
                        if (hrows) {
                            rp[x] = u0 + __builtin_ctzll(hrows);
                            hrows &= hrows - 1;
                            nr = x + 1;
                        }
                        ur[x] = PR ? perm[rp[x]] : rp[x];  // row position -> vertex
                    }
                    // the row's TDT weights are wave-uniform (rp is): scalar loads into SGPRs
                    // instead of a vector load and 2 * TDT readlanes
                    double d64[XR], ws[XR][TDT];
#pragma unroll
                    for (int x = 0; x < XR; ++x) {
                        d64[x] = (lpass >> (rp[x] - u0)) & 1ull ? Dl[(size_t)ur[x] * KL] : dinf();
#pragma unroll
                        for (int t = 0; t < TDT; ++t) ws[x][t] = W[(size_t)rp[x] * Vp + v0 + t];
                    }
#pragma unroll
                    for (int x = 0; x < XR; ++x) {
                        if (x >= nr) break;
                        const int32_t u = ur[x];
                        const bool own = (u == sv[k]);
#pragma unroll
                        for (int t = 0; t < TDT; ++t) {
                            const double c = d64[x] + ws[x][t];
                            if (__ballot((c <= bc[k][t]) & !own)) {
                                if (!own) lex_update(c, d64[x], u, bc[k][t], bdu[k][t], bu[k][t], tie[k], 1u << t);
                            }
                        }
                    }
                }
            }
        }
    }
    if (v0 < V) {
#pragma unroll
        for (int k = 0; k < TB; ++k)
            if (live[k])
            {
                SeedRows sr;
                if (PR && WIp && sv[k] >= 0) {
                    sr.WIp = WIp;
                    sr.WRp = WRp;
                    sr.srow = (size_t)ipos[sv[k]] * Vp;
                    sr.rs = vfac[sv[k]];
                }
                dense_epilogue<TDT>(B[k], lane, sv[k], v0, V, bc[k], bdu[k], bu[k], tie[k], WI, Vp, in_r, parity,
                                    cnt, b0 + k, vid, sr,
                                    mdc_out ? mdc_out + ((size_t)(b0 + k) * (Vp / KL) + v0 / KL) * KL : nullptr,
                                    seeded != 0);
            }
    }
}

// Heavy-first order of a pruned chunk-loop launch (border for k_relax_dense_f<.., PH = 1>):
// block (x, part) sorts the S = nblocks / 8 items XCD x runs in that part (L = 8 j + x, j < S)
// by the chunk counts their blocks staged last time, largest first (ties by j), and writes
// order[8 r + x] = 8 j(r) + x: the hardware block of slot r on XCD x takes the item of rank r.
// A permutation whatever the weights (read while another part's sweep may rewrite them).
constexpr int HEAVY_MAX = 2048;  // items per XCD the one-block bitonic sort takes
struct HeavyArgs {
    const uint32_t* w[4];  // per part: the chunk counts of its last sweep's blocks
    int32_t* o[4];         // per part: the order buffer the next sweep reads
    int32_t slots[4];      // per part: items per XCD (0: no sort)
};
__global__ __launch_bounds__(1024) void k_heavy_order(HeavyArgs ha) {
    __shared__ unsigned long long key[HEAVY_MAX];
    const int x = blockIdx.x, part = blockIdx.y;
    const int32_t S = ha.slots[part];
    if (S <= 0) return;
    const uint32_t* w = ha.w[part];
    int32_t* ord = ha.o[part];
    int n2 = 1;
    while (n2 < S) n2 <<= 1;
    for (int j = threadIdx.x; j < n2; j += blockDim.x)
        key[j] = j < S ? ((unsigned long long)w[8 * j + x] << 32) | (uint32_t)(0xffffffffu - (uint32_t)j) : 0ull;
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1)
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            for (int i = threadIdx.x; i < n2; i += blockDim.x) {
                const int l = i ^ jj;
                if (l > i) {
                    const unsigned long long a = key[i], b = key[l];
                    const bool desc = (i & k) == 0;  // descending overall
                    if (desc ? a < b : a > b) {
                        key[i] = b;
                        key[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    for (int r = threadIdx.x; r < S; r += blockDim.x) {
        const int32_t j = (int32_t)(0xffffffffu - (uint32_t)key[r]);
        ord[8 * r + x] = 8 * j + x;
    }
}

// Pruned full sweep (k_relax_dense_f<.., PR = true>) inputs.
// W32p[i][j] = W32[perm i][perm j]: the f32 weights in the vertex locality order, one row per block
template <typename T>
__global__ __launch_bounds__(256) void k_permute_w(const T* __restrict__ W, const int32_t* __restrict__ perm,
                                                   int32_t Vp, T* __restrict__ Wp) {
    const size_t i = blockIdx.x;
    const __attribute__((address_space(1))) T* src = (const __attribute__((address_space(1))) T*)W + (size_t)perm[i] * Vp;
    for (int32_t j = threadIdx.x; j < Vp; j += 256) Wp[i * Vp + j] = src[perm[j]];
}

// minW[c][w] = min of W32p over rows [c*SRS, c*SRS+SRS) x columns [w*tdt, w*tdt+tdt), NaN (no
// arc) ignored, +inf when the tile has no arc (the pruned sweep uses tdt = 1: one per column)
// W16p for the H16 chunk loop: W32p rounded toward -inf to fp16 (latencies are positive, so
// toward zero), saturating at 65504 (never +inf: a finite weight must keep a finite key),
// NaN (no arc) kept
__global__ __launch_bounds__(256) void k_w16(const float* __restrict__ W32p, uint16_t* __restrict__ W16p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float f = W32p[i];
        uint16_t hb;
        if (f != f) {
            hb = 0x7e00;
        } else if (f >= 65504.0f) {
            hb = 0x7bff;
        } else {
            const _Float16 h = (_Float16)f;
            hb = __builtin_bit_cast(uint16_t, h);
            if ((float)h > f) hb = (uint16_t)(hb - 1);  // f >= 0: the next fp16 below
        }
        W16p[i] = hb;
    }
}

__global__ __launch_bounds__(256) void k_min_w32(const float* __restrict__ W32p, int32_t Vp, int32_t nchunks,
                                                 int32_t nwt, int32_t tdt, float* __restrict__ minW) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)nchunks * nwt) return;
    const int32_t c = (int32_t)(idx / nwt), w = (int32_t)(idx % nwt);
    float m = __int_as_float(0x7f800000);
    for (int r = 0; r < SRS; ++r)
        for (int t = 0; t < tdt; ++t) m = fminf(m, W32p[(size_t)(c * SRS + r) * Vp + w * tdt + t]);
    minW[idx] = m;
}

// minD[b][c][lane] = min of D32 over the rows perm[c*SRS .. c*SRS+SRS) of batch b, NaN
// (unreached, own source) ignored; one wave per (chunk, batch)
__global__ __launch_bounds__(256) void k_min_d32(Pools pools, const int32_t* __restrict__ perm, int32_t nchunks,
                                                 float* __restrict__ minD) {
    const BatchDev B = batch_view(pools, blockIdx.y);
    const int32_t c = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= nchunks) return;
    float m = __int_as_float(0x7f800000);
    for (int r = 0; r < SRS; ++r) m = fminf(m, B.D32[(size_t)perm[c * SRS + r] * KL + lane]);
    minD[((size_t)blockIdx.y * nchunks + c) * KL + lane] = m;
}

// Dense round 0: every destination's only finite candidate is its source's direct arc
// (d = 0 elsewhere is +inf), so the first round needs one weight per (v, source), not a
// sweep over all u.
__global__ __launch_bounds__(256) void k_seed_dense(const double* __restrict__ W, const int32_t* __restrict__ WI,
                                                    int32_t Vp, const double* __restrict__ in_r,
                                                    Pools pools, int32_t V) {
    const BatchDev B = batch_view(pools, blockIdx.y);
    const int lane = threadIdx.x & 63;
    const int32_t sv = B.srcv[lane];
    if (sv < 0) return;
    const int32_t v0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * DT;
    const Rec qs = rec_load(B.Q + (size_t)sv * KL + lane);
    const uint32_t hs = qs.h;
    const double rs = qs.r;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
        const int32_t v = v0 + t;
        if (v >= V || v == sv) continue;
        const double w = W[(size_t)sv * Vp + v];
        if (!(w < dinf())) continue;
        const size_t idx = (size_t)v * KL + lane;
        const int32_t arc = WI[(size_t)sv * Vp + v];
        B.D[idx] = 0.0 + w;
        B.D32[idx] = f32_key(0.0 + w);
        rec_store(B.Q + idx, rs * in_r[arc], ((hs & HMASK) + 1u) | (hs & TAINT), arc);
        B.BDU[idx] = 0.0;
    }
}

// WR[i] = in_r[WI[i]]: the dense reliability factors (0 where there is no arc)

// Dense round 0 in one pass: the state k_init + k_seed + k_seed_dense would leave, with
// every (v, source) entry written once.  A block owns 32 destinations [v0, v0+32) of one
// batch; the batch's source rows W[s][v0..v0+31] are loaded coalesced (256-byte segments), staged in
// LDS and read back transposed (lane = source), so the state rows [v][64] are written
// coalesced too.  Pad rows v >= V get the unreached state.
// The arcs' reliability factors come from the dense WR table (in_r[WI], built once with the
// tables): gathered from in_r by arc id they cost one scattered line per (v, source) and
// C2's seed 0.17 ms per launch against 0.07 ms without them.
constexpr int SEED_T = 16;             // destinations per block: 22 KB of LDS, 7 blocks per CU
constexpr int SEED_ST = SEED_T + 1;    // LDS row stride: the transposed reads spread over the banks
__global__ __launch_bounds__(256) void k_seed_dense_t(const double* __restrict__ W, const int32_t* __restrict__ WI,
                                                      int32_t Vp, const double* __restrict__ WR,
                                                      const double* __restrict__ vfac, Pools pools, int32_t V,
                                                      int32_t* __restrict__ cnt, int32_t cnt_rows, int32_t cnt_stride) {
    __shared__ double sw[KL * SEED_ST];
    __shared__ double sr[KL * SEED_ST];
    __shared__ int32_t si[KL * SEED_ST];
    // the rounds' change-count rows of this batch (run_rounds: cnt_row): row 0, the virtual
    // round -1, "everything changed"; the rows of the rounds enqueued without a read-back zero
    if (blockIdx.x == 0 && (int)threadIdx.x < cnt_rows)
        cnt[(size_t)threadIdx.x * cnt_stride + blockIdx.y] = threadIdx.x == 0 ? 0x7f7f7f7f : 0;
    const BatchDev B = batch_view(pools, blockIdx.y);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int32_t v0 = blockIdx.x * SEED_T;
    // the 64 sources' rows over this block's destinations: 32-element (256-byte) segments
    for (int e = threadIdx.x; e < KL * SEED_T; e += 256) {
        const int j = e / SEED_T, x = e % SEED_T;
        const int32_t s = B.srcv[j];
        double w = dinf(), r = 0.0;
        int32_t a = -1;
        if (s >= 0 && v0 + x < V) {
            w = W[(size_t)s * Vp + v0 + x];
            a = WI[(size_t)s * Vp + v0 + x];
            r = WR[(size_t)s * Vp + v0 + x];
        }
        sw[j * SEED_ST + x] = w;
        sr[j * SEED_ST + x] = r;
        si[j * SEED_ST + x] = a;
    }
    __syncthreads();
    const int32_t sv = B.srcv[lane];
    const double rs = sv >= 0 ? vfac[sv] : 0.0;  // R(s) = 1*(1-loss_v(s)) (topology.c:1441-1445)
    for (int x = wave; x < SEED_T; x += 4) {
        const int32_t v = v0 + x;
        const double w = sw[lane * SEED_ST + x];
        const int32_t arc = si[lane * SEED_ST + x];
        const double ra = sr[lane * SEED_ST + x];
        const bool own = (v == sv);
        const bool seeded = sv >= 0 && !own && v < V && w < dinf();
        double d = dinf(), r = 0.0, bdu = dinf();
        uint32_t h = 0;
        int32_t p = -1;
        float d32 = __int_as_float(0x7fc00000);  // NaN: unreached, and the source's own row
        if (own) {
            d = 0.0;
            r = rs;
        } else if (seeded) {
            d = 0.0 + w;
            d32 = f32_key(d);
            h = 1;
            r = rs * ra;
            p = arc;
            bdu = 0.0;
        }
        const size_t idx = (size_t)v * KL + lane;
        B.D[idx] = d;
        B.D32[idx] = d32;
        rec_store(B.Q + idx, r, h, p);
        B.BDU[idx] = bdu;
        const unsigned long long reach = __ballot(seeded);
        const unsigned long long srcm = __ballot(own);
        if (lane == 0) {
            B.act0[v] = reach != 0;  // k_seed: out-neighbours of the sources
            B.act1[v] = 0;
            B.chm0[v] = 0;
            B.chm1[v] = srcm;        // k_seed: round -1's change mask holds the sources
        }
    }
}

// One candidate (u -> v for source lane s) with c <= d(v): the lexicographic update of
// k_relax_dense applied incrementally against the recorded state.  The recorded lex key is
// (D, BDU); the local-tie bit LTIE stays valid while the predecessor's key is unchanged.
// Returns whether (v, s)'s D/H/R/P changed (its children must look again next round).
__device__ __forceinline__ bool delta_candidate(const BatchDev& B, int32_t v, int32_t s, int32_t u, double du,
                                                double c, double cur, const int32_t* __restrict__ WI, int32_t Vp,
                                                const int32_t* __restrict__ in_src, const double* __restrict__ in_r,
                                                double* sdcell, float* tcell = nullptr) {
    const size_t idx = (size_t)v * KL + s;
    const Rec qv = rec_load(B.Q + idx);
    const uint32_t hv = qv.h;
    uint32_t lt = 0;
    if (!(c < cur)) {  // c == d(v): the recorded predecessor refreshed, or a same-distance rival
        const int32_t pa = qv.p;
        const int32_t pu = pa >= 0 ? in_src[pa] : -1;
        const double bdu = B.BDU[idx];
        if (pu == u) {
            // same predecessor: its key only moves down; with an unchanged key the recorded
            // tie stands, a smaller key beats every unchanged rival (a changed rival with the
            // new key is a candidate of this same round and re-marks the tie)
            lt = (du == bdu) ? (hv & LTIE) : 0u;
        } else if (du == bdu) {
            const uint32_t nh = hv | LTIE | TAINT;
            if (nh == hv) return false;
            B.Q[idx].h = nh;
            return (hv & TAINT) == 0;
        } else if (du > bdu) {
            return false;
        }
    }
    if (du == c) lt = LTIE;  // degenerate d(u) == d(v): the reference order is heap-dependent
    const int32_t arc = WI[(size_t)u * Vp + v];
    const size_t uidx = (size_t)u * KL + s;
    const Rec qu = rec_load(B.Q + uidx);
    const uint32_t h = (((qu.h & HMASK) + 1u) & HMASK) | (qu.h & TAINT) | (lt ? (TAINT | LTIE) : 0u);
    const double r = qu.r * in_r[arc];
    B.BDU[idx] = du;
    if (sdcell) *sdcell = c;
    if (tcell) *tcell = f32_thr(c);
    if (c != cur || h != hv || r != qv.r || arc != qv.p) {
        B.D[idx] = c;
        B.D32[idx] = f32_key(c);
        rec_store(B.Q + idx, r, h, arc);
        return true;
    }
    return false;
}

// Dense delta round.  A (u, source) pair whose state did not change in the previous round
// was already evaluated by every destination against its final value, so only the pairs of
// the previous round's change masks can improve anything.  One wave owns 64 destinations
// (lane = v) of one batch and keeps their 64x64 current distances in LDS; it walks the
// changed rows u in groups of DG (weights W[u][v0..v0+63] and the row d(u) for all 64
// sources: 2 coalesced 512-B loads per row, all in flight together) and, per changed
// source s of row u, compares fl(d_s(u) + w(u, v)) against d_s(v) -- one f64 add, one LDS
// read and one compare for 64 destinations.  Candidates c <= d_s(v) (rare) take the exact
// lexicographic path in delta_candidate.  The host picks this kernel for a batch when the
// previous round changed at most `thresh` pairs, k_relax_dense otherwise.
// Grid: the batches of one destination chunk sit on the same XCD (shared W rows in L2).
constexpr int DG = 8;
constexpr int DW = 4;        // waves per block: wave w takes the sources [16w, 16w+16) of the tile
constexpr int SDS = KL + 1;  // LDS row stride (doubles): conflict-free transposed staging

__global__ __launch_bounds__(64 * DW) void k_relax_dense_delta(const double* __restrict__ W,
                                                               const int32_t* __restrict__ WI, int32_t Vp,
                                                               const int32_t* __restrict__ in_src,
                                                               const double* __restrict__ in_r, Pools pools,
                                                               int32_t V, int32_t nb, int32_t nvc, int32_t parity,
                                                               int32_t thresh, const int32_t* __restrict__ cnt_prev,
                                                               int32_t* __restrict__ cnt) {
    __shared__ double sD[KL * SDS];  // [s][v - v0]
    __shared__ unsigned long long sM[DW][KL];
    const int32_t L = blockIdx.x;
    const int32_t q = L >> 3;
    const int32_t b = q % nb;
    const int32_t vc = (L & 7) + 8 * (q / nb);
    if (vc >= nvc) return;  // block-uniform exits only (barriers below)
    const int32_t cp = cnt_prev[b];
    if (cp == 0 || cp > thresh) return;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int32_t v0 = vc * KL;
    const int32_t v = v0 + lane;
    const BatchDev B = batch_view(pools, b);
    const gdouble* D = B.D;
    for (int i = wave; i < KL; i += DW) sD[lane * SDS + i] = D[(size_t)(v0 + i) * KL + lane];
    __syncthreads();
    const int32_t s0 = wave * (KL / DW);
    const unsigned long long srange = (DW == 1) ? ~0ull : (((1ull << (KL / DW)) - 1ull) << s0);
    const unsigned long long* chp = B.chm(parity ^ 1);
    const bool vok = v < V;
    const double inf = dinf();
    unsigned long long mine = 0;
    for (int32_t u0 = 0; u0 < V; u0 += KL) {
        const unsigned long long mk = ((u0 + lane < V) ? chp[u0 + lane] : 0ull) & srange;
        unsigned long long nz = __ballot(mk != 0ull);
        while (nz) {
            int32_t us[DG];
            int n = 0;
#pragma unroll
            for (int i = 0; i < DG; ++i) {
                us[i] = 0;
                if (nz) {
                    us[i] = __builtin_ctzll(nz);
                    nz &= nz - 1;
                    n = i + 1;
                }
            }
            double w[DG], dr[DG];
#pragma unroll
            for (int i = 0; i < DG; ++i) {
                if (i < n) {
                    const int32_t u = u0 + us[i];
                    w[i] = W[(size_t)u * Vp + v];
                    dr[i] = D[(size_t)u * KL + s0 + (lane & (KL / DW - 1))];  // this wave's sources only
                }
            }
#pragma unroll
            for (int i = 0; i < DG; ++i) {
                if (i >= n) break;
                const int32_t u = u0 + us[i];
                unsigned long long m = readlane_u64(mk, us[i]);
                while (m) {
                    const int32_t sj = __builtin_ctzll(m);
                    m &= m - 1;
                    const double du = readlane_d(dr[i], sj - s0);
                    const double c = du + w[i];
                    double* cell = &sD[sj * SDS + lane];
                    const double cur = *cell;
                    if (c <= cur && c < inf && vok) {
                        if (delta_candidate(B, v, sj, u, du, c, cur, WI, Vp, in_src, in_r, cell)) mine |= 1ull << sj;
                    }
                }
            }
        }
    }
    sM[wave][lane] = mine;
    __syncthreads();
    if (wave == 0) {
        unsigned long long all = 0;
#pragma unroll
        for (int k = 0; k < DW; ++k) all |= sM[k][lane];
        B.chm(parity)[v] = all;
        if (all) atomicAdd(&cnt[b], (int32_t)__popcll(all));
    }
}

// Sparse delta rounds: per batch, the 64-row chunks holding a row whose change mask (the
// previous round's) is non-zero, in ascending order -- the delta round then walks only
// those chunks (a round after a round that changed few pairs is nearly free instead of
// a full walk of every chunk's slab and barriers).  One block per batch.
__global__ __launch_bounds__(256) void k_live_chunks(Pools pools, int32_t V, int32_t nvc, int32_t parity,
                                                     const int32_t* __restrict__ cnt_prev, int32_t* __restrict__ live,
                                                     int32_t* __restrict__ nlive) {
    __shared__ int32_t sbase;
    const int32_t b = blockIdx.x;
    const BatchDev B = batch_view(pools, b);
    const unsigned long long* chp = B.chm(parity ^ 1);
    if (threadIdx.x == 0) sbase = 0;
    __syncthreads();
    for (int32_t c0 = 0; c0 < nvc; c0 += 256) {
        const int32_t c = c0 + threadIdx.x;
        bool any = false;
        if (c < nvc && cnt_prev[b] != 0)
            for (int r = 0; r < KL && c * KL + r < V; ++r) any |= chp[c * KL + r] != 0ull;
        // ascending order: wave ballots, waves in turn
        const unsigned long long bal = __ballot(any);
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        __shared__ int32_t swc[4];
        if (lane == 0) swc[wave] = __popcll(bal);
        __syncthreads();
        int32_t off = sbase;
        for (int k = 0; k < wave; ++k) off += swc[k];
        if (any)
            live[(size_t)b * nvc + off + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = c;
        __syncthreads();
        if (threadIdx.x == 0) sbase += swc[0] + swc[1] + swc[2] + swc[3];
        __syncthreads();
    }
    if (threadIdx.x == 0) nlive[b] = sbase;
}

// Staged f32 dense delta round, lane = candidate pair (the round semantics of
// k_relax_dense_delta).  The block (one batch, 64 destinations, 4 waves of 16 sources) walks
// the rows in 64-row chunks; each chunk's W32 slab W32[u0..u0+63][v0..v0+63] is loaded once,
// coalesced, into LDS (register-prefetched one chunk ahead) and serves every changed pair of
// the chunk in all four waves.  A wave lists its changed (u, s) pairs of the chunk in row
// order and filters 64 of them at once, one per lane, against the thresholds
// sT[s][v] = f32_thr(d_s(v)): pass iff D32(u, s) <= max_v fl32(sT[s][v] - W32(u, v))
// (conservative, see k_relax_dense_f).  Passing pairs (rare) are settled one at a time with
// lane = destination, exactly in f64 through delta_candidate, so no two lanes ever update one
// (v, s) state.  (Gathering each pair's W32 row from global memory instead, 16 bytes per lane
// per load, cost 1.6x this kernel's time: one texture-address cycle per lane.)
constexpr int SWS = KL + 4;              // LDS row stride (floats) of the staged W32 slab and the thresholds:
                                         // rows r != r' (mod 16) on distinct bank quads
constexpr int RING_S = 512;  // ring segment (int16 entries): a chunk's pairs of one wave (at most 64 x 16) are
                             // listed and drained 512 at a time -- 46 -> 40 KB of LDS, 4 blocks per CU

constexpr int PR_CHUNKS = 640;  // pruned delta: live-chunk list capacity (dense mode keeps Vp <= 38 730: 606 chunks)

template <bool PR, bool H16 = false>
__global__ __launch_bounds__(64 * DW) void k_relax_dense_delta_s(const float* __restrict__ W32,
                                                                 const double* __restrict__ W,
                                                                 const int32_t* __restrict__ WI, int32_t Vp,
                                                                 const int32_t* __restrict__ in_src,
                                                                 const double* __restrict__ in_r, Pools pools,
                                                                 int32_t V, int32_t nb, int32_t nvc, int32_t parity,
                                                                 int32_t thresh, const int32_t* __restrict__ cnt_prev,
                                                                 int32_t* __restrict__ cnt,
                                                                 const int32_t* __restrict__ live,
                                                                 const int32_t* __restrict__ nlive,
                                                                 const int32_t* __restrict__ perm,
                                                                 const float* __restrict__ minW64,
                                                                 const float* __restrict__ minDc,
                                                                 const float* __restrict__ minWc,
                                                                 unsigned long long* __restrict__ cmask) {
    // PR (pruned): rows, destinations and W32 (here W32p) in the vertex locality order `perm`,
    // and the block walks only the chunks that can hold a passing pair: a chunk is dead when
    // for every source s, minDc(chunk, s) > fl32(maxT_s - minW64(chunk, tile)), where minDc is
    // the minimum D32 over the chunk's CHANGED (u, s) pairs (NaN: none), maxT_s the largest
    // threshold of s over the tile's destinations at the start of the round (thresholds only
    // tighten) and minW64 the smallest W32 of the chunk x tile block.  Every pair's filter
    // bound max_v fl32(sT[s][v] - W32(u, v)) is <= the chunk's (rounding is monotone), so a dead
    // chunk holds no pair the filter would pass: the skip is exact.
    // With minWc (the sweep's per-(32-row chunk, column) W32 minima) the bound is taken per
    // destination instead: the chunk is dead when minDc(chunk, s) > max_v fl32(sT[s][v] -
    // mWc(chunk, v)) for every s, mWc(chunk, v) = min W32 of the chunk's rows into v -- the
    // same argument (W32(u, v) >= mWc(chunk, v)), and never looser than the tile bound.
    // H16 (PR only, OPT_DELTA_W16, r06): the slab comes from W16p (W32p rounded toward -inf to
    // fp16, NaN kept; k_w16), half the bytes; the filter's slacks fl32(sT - W16) are >= the
    // W32 ones, so it stays conservative and the exact settle decides as before.
    static_assert(!H16 || PR, "fp16 slabs: the pruned delta round only");
    constexpr int SW = KL / DW;  // sources per wave
    constexpr int PF = KL * KL / (H16 ? 8 : 4) / (64 * DW);  // 16-byte pieces of one slab per thread
    constexpr int SWH = KL + 8;  // H16: LDS row stride (halves) of the slab
    __shared__ __attribute__((aligned(16))) float sT[KL * SWS];  // [s][v] thresholds
    // the slab (H16: halves, half the LDS; the per-destination bounds below borrow 16 rows)
    __shared__ __attribute__((aligned(16))) float sW[H16 ? KL * SWH / 2 : KL * SWS];
    static_assert(!H16 || KL * SWH / 2 >= 4 * DW * SWS, "the bounds' column minima fit the fp16 slab");
    __shared__ int16_t sP[DW][RING_S];  // (row in chunk << 6) | s
    __shared__ int16_t sL[PR ? PR_CHUNKS : 1];  // PR: the block's live chunks, ascending
    __shared__ int32_t sNL;
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const f4 gf4;
    const int32_t L = blockIdx.x;
    const int32_t q = L >> 3;
    const int32_t b = q % nb;
    const int32_t vc = (L & 7) + 8 * (q / nb);
    if (vc >= nvc) return;  // block-uniform exits only (barriers below)
    const int32_t cp = cnt_prev[b];
    if (cp == 0 || cp > thresh) return;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int32_t v0 = vc * KL;  // the tile's first column (PR: in the locality order)
    const int32_t v = PR ? perm[v0 + lane] : v0 + lane;  // this lane's destination vertex
    const BatchDev B = batch_view(pools, b);
    const gdouble* D = B.D;
    {
        // the wave's 16 threshold rows with their loads in flight together (the row vertices
        // are the lanes' own destinations)
        double dd[KL / DW];
#pragma unroll
        for (int k = 0; k < KL / DW; ++k) dd[k] = D[(size_t)__builtin_amdgcn_readlane(v, wave + k * DW) * KL + lane];
#pragma unroll
        for (int k = 0; k < KL / DW; ++k) sT[lane * SWS + wave + k * DW] = f32_thr(dd[k]);
    }
    const int32_t s0 = wave * SW;
    const unsigned long long srange = ((1ull << SW) - 1ull) << s0;
    const unsigned long long* chp = B.chm(parity ^ 1);
    const gfloat* D32 = B.D32;
    const gfloat* W32g = (const gfloat*)W32;
    const bool vok = v < V;
    const double inf = dinf();
    int16_t* ring = sP[wave];
    unsigned long long mine = 0;

    if (PR && minWc) {
        // per-destination bounds: wave w evaluates chunks w, w + DW, ... for all 64 sources
        // (lane = source) with the chunk's column minima staged in its own row of sW (free
        // until the first slab); the live flags go to sP's bytes, wave 0 lists them in order
        __syncthreads();  // thresholds staged
        uint8_t* flags = reinterpret_cast<uint8_t*>(&sP[0][0]);
        float* mrow = &sW[wave * 4 * SWS];  // 4 rows per wave
        const int32_t nc32 = (V + SRS - 1) / SRS;
        const float* md = minDc + (size_t)b * nvc * KL + lane;
        const float* trow = &sT[lane * SWS];
        // G chunks per step, their loads issued together (one chunk's dependent loads per
        // step left every step waiting out a global load)
        constexpr int G = 4;
        for (int32_t c0 = wave * G; c0 < nvc; c0 += DW * G) {
            float m0[G], m1[G], d[G];
#pragma unroll
            for (int k = 0; k < G; ++k) {
                const int32_t c = c0 + k < nvc ? c0 + k : nvc - 1;
                m0[k] = minWc[(size_t)(2 * c) * Vp + v0 + lane];
                m1[k] = 2 * c + 1 < nc32 ? minWc[(size_t)(2 * c + 1) * Vp + v0 + lane] : __int_as_float(0x7f800000);
                d[k] = md[(size_t)c * KL];
            }
#pragma unroll
            for (int k = 0; k < G; ++k) mrow[k * SWS + lane] = fminf(m0[k], m1[k]);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the rows are written
#pragma unroll
            for (int k = 0; k < G; ++k) {
                float g = __int_as_float(0x7fc00000);
#pragma unroll
                for (int j = 0; j < KL / 4; ++j) {
                    const f4 t4 = *(const f4*)&trow[4 * j];
                    const f4 w4 = *(const f4*)&mrow[k * SWS + 4 * j];
                    g = fmaxf(fmaxf(g, t4.x - w4.x), t4.y - w4.y);
                    g = fmaxf(fmaxf(g, t4.z - w4.z), t4.w - w4.w);
                }
                const unsigned long long bal = __ballot(d[k] <= g);
                if (lane == 0 && c0 + k < nvc) {
                    flags[c0 + k] = bal != 0ull;
                    // the sources that can pass in this chunk: the walk lists only their pairs
                    if (cmask) cmask[(size_t)L * PR_CHUNKS + c0 + k] = bal;
                }
            }
            __builtin_amdgcn_wave_barrier();  // every lane's reads of the rows before the next step's writes
        }
        __syncthreads();  // flags
        if (wave == 0) {
            int32_t n = 0;
            for (int32_t c0 = 0; c0 < nvc; c0 += 64) {
                const bool f = c0 + lane < nvc && flags[c0 + lane];
                const unsigned long long bal = __ballot(f);
                if (f)
                    sL[n + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] =
                        (int16_t)(c0 + lane);
                n += __popcll(bal);
            }
            if (lane == 0) sNL = n;
        }
    } else if (PR) {
        // the block's live chunks: every wave evaluates every chunk for all 64 sources (lane =
        // source) and gets the same answer; wave 0 writes the list
        __syncthreads();  // thresholds staged
        float mt = __int_as_float(0x7fc00000);
        for (int i = 0; i < KL; ++i) mt = fmaxf(mt, sT[lane * SWS + i]);
        int32_t n = 0;
        const float* md = minDc + (size_t)b * nvc * KL + lane;
        const float* mw = minW64 + vc;
        for (int32_t c0 = 0; c0 < nvc; c0 += 8) {
            float d8[8], w8[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int32_t c = c0 + k < nvc ? c0 + k : nvc - 1;
                d8[k] = md[(size_t)c * KL];
                w8[k] = mw[(size_t)c * nvc];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool ok = c0 + k < nvc && d8[k] <= mt - w8[k];
                if (__ballot(ok)) {
                    if (wave == 0 && lane == 0 && n < PR_CHUNKS) sL[n] = (int16_t)(c0 + k);
                    ++n;
                }
            }
        }
        if (wave == 0 && lane == 0) sNL = n;
    }

    f4 pw[PF];
    // The prefetch addresses are held live until the stash: the compiler must not reuse a
    // VGPR that a load in flight addresses (it would wait for that load right there, i.e. at
    // the first drain instead of after the drains).
    const gf4* pwa[PF];
    const unsigned long long* pma = chp;
    auto fetch = [&](int32_t u0) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int e = threadIdx.x + i * 64 * DW;  // float4 index within the slab: row e / 16, column 4 (e % 16)
            if constexpr (H16)  // 8 halves per piece: row e / 8, column 8 (e % 8)
                pwa[i] = (gf4*)((const __attribute__((address_space(1))) uint16_t*)W32g + (size_t)(u0 + (e >> 3)) * Vp +
                                v0 + 8 * (e & 7));
            else
                pwa[i] = (gf4*)(W32g + (size_t)(u0 + (e >> 4)) * Vp + v0 + 4 * (e & 15));
            pw[i] = *pwa[i];
        }
    };
    auto hold = [&]() {
#pragma unroll
        for (int i = 0; i < PF; ++i) asm volatile("" ::"v"(pwa[i]));
        asm volatile("" ::"v"(pma));
    };
    auto stash = [&]() {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int e = threadIdx.x + i * 64 * DW;
            if constexpr (H16)
                *(f4*)((uint16_t*)sW + (e >> 3) * SWH + 8 * (e & 7)) = pw[i];
            else
                *(f4*)&sW[(e >> 4) * SWS + 4 * (e & 15)] = pw[i];
        }
    };
    // the staged slab's weight of row r into column c (H16: fp16 -> f32, exact)
    auto slab_w = [&](int r, int c) -> float {
        if constexpr (H16) return (float)__builtin_bit_cast(_Float16, ((const uint16_t*)sW)[r * SWH + c]);
        else return sW[r * SWS + c];
    };

    // filter n <= 64 listed pairs starting at ring[h] (lane = pair), settle the passing ones;
    // urow: this lane's row vertex of the chunk (lane = row)
    auto drain = [&](int32_t u0, int32_t urow, int h, int n) {
        const bool valid = lane < n;
        const int32_t e = ring[h + (valid ? lane : n - 1)];
        const int32_t r = e >> 6, sp = e & 63;
        const int32_t ur = PR ? __shfl(urow, r) : u0 + r;
        const gfloat* dua = D32 + (size_t)ur * KL + sp;
        const float du = *dua;
        const float* trow = &sT[sp * SWS];
        // slacks two at a time (v_pk_add_f32), their maximum as a v_max3 chain; both rows are
        // read at immediate offsets from one base each
        typedef float f2 __attribute__((ext_vector_type(2)));
        float g = __int_as_float(0x7fc00000);
        if constexpr (H16) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            typedef _Float16 hh2 __attribute__((ext_vector_type(2)));
            const uint16_t* wrow = (const uint16_t*)sW + r * SWH;
#pragma unroll
            for (int j = 0; j < KL / 8; ++j) {
                const u4 w8 = *(const u4*)&wrow[8 * j];
                const f4 ta = *(const f4*)&trow[8 * j];
                const f4 tb = *(const f4*)&trow[8 * j + 4];
                const float tv[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t word = w8[k];  // a local copy: hipcc 7.2 mis-reads a bit_cast component lvalue
                    const hh2 h = __builtin_bit_cast(hh2, word);
                    const f2 a = f2{tv[2 * k], tv[2 * k + 1]} - f2{(float)h.x, (float)h.y};
                    g = fmaxf(fmaxf(g, a.x), a.y);
                }
            }
        } else {
            const float* wrow = &sW[r * SWS];
#pragma unroll
            for (int j = 0; j < KL / 4; ++j) {
                const f4 w4 = *(const f4*)&wrow[4 * j];
                const f4 t4 = *(const f4*)&trow[4 * j];
                const f2 a = f2{t4.x, t4.y} - f2{w4.x, w4.y};
                const f2 c = f2{t4.z, t4.w} - f2{w4.z, w4.w};
                g = fmaxf(fmaxf(g, a.x), a.y);
                g = fmaxf(fmaxf(g, c.x), c.y);
            }
        }
        unsigned long long pm = __ballot(valid && du <= g);
        asm volatile("" ::"v"(dua));
        while (pm) {
            const int pl = __builtin_ctzll(pm);
            pm &= pm - 1;
            const int32_t pe = __builtin_amdgcn_readlane(e, pl);
            const int32_t rr = pe >> 6, ss = pe & 63;
            const int32_t uu = PR ? __builtin_amdgcn_readlane(urow, rr) : u0 + rr;
            float* tc = &sT[ss * SWS + lane];
            const float c32 = D32[(size_t)uu * KL + ss] + slab_w(rr, lane);
            if (vok && c32 <= *tc) {
                const double du64 = D[(size_t)uu * KL + ss];
                const double c = du64 + W[(size_t)uu * Vp + v];
                const double cur = D[(size_t)v * KL + ss];
                if (c <= cur && c < inf &&
                    delta_candidate(B, v, ss, uu, du64, c, cur, WI, Vp, in_src, in_r, nullptr, tc))
                    mine |= 1ull << ss;
            }
        }
    };

    // the 64-row chunks to walk: PR, the live list above; otherwise every chunk, or (sparse
    // rounds) the batch's chunks that hold a changed row, in ascending order (k_live_chunks)
    if (PR) __syncthreads();  // the live list
    const int32_t nl = PR ? (sNL < PR_CHUNKS ? sNL : -1) : (live ? nlive[b] : (V + KL - 1) / KL);
    const bool all_chunks = PR && nl < 0;  // list overflow: walk every chunk
    const int32_t nwalk = all_chunks ? (V + KL - 1) / KL : nl;
    auto chunk_u0 = [&](int32_t i) {
        if (PR) return (all_chunks ? i : (int32_t)sL[i]) * KL;
        return (live ? live[(size_t)b * nvc + i] : i) * KL;
    };
    // PR with per-destination bounds: the chunk's passing sources (cmask, written above by the
    // evaluating wave; visible after the barrier), one chunk ahead like the change masks
    const unsigned long long* cm = (PR && minWc && cmask && !all_chunks) ? cmask + (size_t)L * PR_CHUNKS : nullptr;
    unsigned long long smk = ~0ull, smk_n = ~0ull;
    // PR: row vertices one chunk ahead of the masks that are gathered through them
    int32_t urow = 0, urow_n = 0;
    unsigned long long mnext = 0;
    if (nwalk > 0) {
        if (cm) smk = cm[chunk_u0(0) / KL];
        const int32_t f0 = chunk_u0(0);
        fetch(f0);
        stash();
        urow = PR ? perm[f0 + lane] : f0 + lane;
        mnext = chp[urow];  // rows < Vp exist; rows >= V (padding, perm maps them to themselves) are masked at use
        if (PR && nwalk > 1) urow_n = perm[chunk_u0(1) + lane];
    }
    __syncthreads();
    for (int32_t ci = 0; ci < nwalk; ++ci) {
        const int32_t u0 = chunk_u0(ci);
        const bool more = ci + 1 < nwalk;
        const int32_t un = more ? chunk_u0(ci + 1) : 0;
        const unsigned long long m = (u0 + lane < V) ? (mnext & srange & smk) : 0ull;
        // exclusive prefix sum of the per-row pair counts (<= 16, five bits) from ballots
        // and mbcnt: no cross-lane LDS round trips
        const int p = __popcll(m);
        int pos = 0, tot = 0;
#pragma unroll
        for (int bit = 0; bit < 5; ++bit) {
            const unsigned long long bm = __ballot((p >> bit) & 1);
            pos += __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u)) << bit;
            tot += __popcll(bm) << bit;
        }
        // the next chunk's change masks and W32 slab are in flight while this chunk drains
        // (issued after this chunk's masks are consumed, waited for at the stash);
        // u0 + KL + 63 < Vp when `more`
        const int32_t urow_nn = (PR && ci + 2 < nwalk) ? perm[chunk_u0(ci + 2) + lane] : 0;
        pma = chp + (PR ? (more ? urow_n : 0) : un + lane);
        mnext = *pma;
        if (cm && more) smk_n = cm[un / KL];
        if (more) fetch(un);
        for (int base = 0; base < tot; base += RING_S) {  // usually one segment (C2: ~40 pairs)
            unsigned long long mm = m;
            int q = pos;
            while (mm) {
                if (q >= base && q < base + RING_S) ring[q - base] = (int16_t)((lane << 6) | __builtin_ctzll(mm));
                ++q;
                mm &= mm - 1;
            }
            __builtin_amdgcn_wave_barrier();
            const int seg = tot - base < RING_S ? tot - base : RING_S;
            for (int h = 0; h < seg; h += KL) drain(u0, urow, h, seg - h < KL ? seg - h : KL);
            __builtin_amdgcn_wave_barrier();  // the segment is drained before the next overwrites it
        }
        hold();
        __syncthreads();  // every wave is done with this slab
        if (more) stash();
        __syncthreads();
        urow = PR ? urow_n : un + lane;
        urow_n = urow_nn;
        smk = smk_n;
    }
    // the waves' change masks, in the thresholds' LDS (every wave is past the walk's last
    // barrier: nobody reads sT any more)
    unsigned long long (*sM)[KL] = reinterpret_cast<unsigned long long (*)[KL]>(sT);
    __syncthreads();
    sM[wave][lane] = mine;
    __syncthreads();
    if (wave == 0) {
        unsigned long long all = 0;
#pragma unroll
        for (int k = 0; k < DW; ++k) all |= sM[k][lane];
        B.chm(parity)[v] = all;  // v < Vp: PR maps padding columns to themselves
        if (all) atomicAdd(&cnt[b], (int32_t)__popcll(all));
    }
}

// PR delta inputs.  minW64[c][t] = min of W32p over the 64 x 64 block (rows of chunk c,
// columns of tile t), NaN ignored (+inf: no arc)
__global__ __launch_bounds__(256) void k_min_w64(const float* __restrict__ W32p, int32_t Vp, int32_t nvc,
                                                 float* __restrict__ minW64) {
    const int64_t idx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per block of W32p
    const int lane = threadIdx.x & 63;
    if (idx >= (int64_t)nvc * nvc) return;
    const int32_t c = (int32_t)(idx / nvc), t = (int32_t)(idx % nvc);
    float m = __int_as_float(0x7f800000);
    for (int r = 0; r < KL; ++r) m = fminf(m, W32p[(size_t)(c * KL + r) * Vp + t * KL + lane]);
    for (int o = 32; o > 0; o >>= 1) m = fminf(m, __shfl_xor(m, o));
    if (lane == 0) minW64[idx] = m;
}

// minDc[b][c][lane] = min D32 over the CHANGED pairs (previous round's change masks) of the
// rows perm[c*64 .. c*64+64) of batch b; NaN when the chunk has none for the lane (a dead
// chunk for that source whatever the thresholds).  One block per (chunk, batch): each wave
// takes 16 of the rows with all their loads in flight (one wave walking the 64 rows in turn
// took 69 us per C2 delta round, latency-bound), the four minima meet in LDS.
__global__ __launch_bounds__(256) void k_min_d32c(Pools pools, const int32_t* __restrict__ perm, int32_t V,
                                                  int32_t nvc, int32_t parity, const int32_t* __restrict__ cnt_prev,
                                                  int32_t thresh, float* __restrict__ minDc) {
    __shared__ float sm[4][KL];
    constexpr int RW = KL / 4;  // rows per wave
    const int32_t b = blockIdx.y;
    const int32_t c = blockIdx.x;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const BatchDev B = batch_view(pools, b);
    float m = __int_as_float(0x7f800000);
    const int32_t cp = cnt_prev[b];
    if (cp > 0 && cp <= thresh) {  // block-uniform
        const unsigned long long* chp = B.chm(parity ^ 1);
        int32_t u[RW];
        unsigned long long mk[RW];
#pragma unroll
        for (int i = 0; i < RW; ++i) u[i] = perm[c * KL + wave * RW + i];
#pragma unroll
        for (int i = 0; i < RW; ++i) mk[i] = u[i] < V ? chp[u[i]] : 0ull;
#pragma unroll
        for (int i = 0; i < RW; ++i)
            if ((mk[i] >> lane) & 1ull) m = fminf(m, B.D32[(size_t)u[i] * KL + lane]);
    }
    sm[wave][lane] = m;
    __syncthreads();
    if (wave == 0) {
        m = fminf(fminf(sm[0][lane], sm[1][lane]), fminf(sm[2][lane], sm[3][lane]));
        minDc[((size_t)b * nvc + c) * KL + lane] = m < __int_as_float(0x7f800000) ? m : __int_as_float(0x7fc00000);
    }
}

// ---------------------------------------------------------------- self pairs
// _topology_computeShortestPathToSelf (topology.c:1545-1653): first strict minimum of the
// OUT-incident edges in igraph order, used twice; or (F_SELF_DIJKSTRA_LOOP) the [s] path
// through the source's self-loop (topology.c:1456-1499).
// Rows [i0, i1) of the attached list, run inside every computation of those rows (the
// reference computes the self path per query, so a matrix build includes it).  The
// incidence latencies are one contiguous array in igraph order (inc_lat): each thread keeps
// the first strict minimum of its strided slice (positions ascending, so a strict '<' keeps
// the first), then a reduction on (latency, position) picks the first strict minimum overall
// -- the reference's sequential rule.  BLK = true: a 256-thread block per vertex (dense
// graphs: C2's 9 500 incident edges per vertex), else one wave per vertex.
template <bool BLK>
__global__ __launch_bounds__(256) void k_self(GraphDev g, const int32_t* __restrict__ attached, int32_t i0, int32_t i1,
                                              double* self_lat, double* self_rel, uint32_t* self_hops,
                                              uint8_t* self_kind) {
    __shared__ double sl[4];
    __shared__ int64_t sp[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int32_t i = i0 + (BLK ? (int32_t)blockIdx.x : (int32_t)blockIdx.x * 4 + wave);
    if (i >= i1) return;  // uniform per block (BLK) or per wave
    const int32_t v = attached[i];
    const int tid = BLK ? (int)threadIdx.x : lane;
    constexpr int NT = BLK ? 256 : 64;
    double lat = -1.0, rel = -1.0;
    uint32_t hops = 0;
    uint8_t kind = SHADOWTOPO_KIND_NONE;
    if (g.flags & SHADOWTOPO_F_SELF_DIJKSTRA_LOOP) {
        const int32_t le = g.loop_eid[v];
        if (le >= 0) {
            lat = 0.0 + g.elat[le];
            if (lat == 0) lat = 1;
            rel = g.vfac[v] * g.erel[le];
            hops = 1;
            kind = SHADOWTOPO_KIND_DIJKSTRA;
        }
    } else {
        const int64_t beg = g.inc_ptr[v], end = g.inc_ptr[v + 1];
        if (end > beg) {
            double minl = dinf();
            int64_t pos = INT64_MAX;
            for (int64_t x = beg + tid; x < end; x += 4 * NT) {
                double l[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) l[k] = x + k * NT < end ? g.inc_lat[x + k * NT] : dinf();
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (l[k] < minl) {
                        minl = l[k];
                        pos = x + k * NT;
                    }
            }
            for (int off = 32; off > 0; off >>= 1) {
                const double ol = __shfl_xor(minl, off);
                const int64_t op = __shfl_xor(pos, off);
                if (ol < minl || (ol == minl && op < pos)) {
                    minl = ol;
                    pos = op;
                }
            }
            if (BLK) {
                if (lane == 0) {
                    sl[wave] = minl;
                    sp[wave] = pos;
                }
                __syncthreads();
                for (int w = 0; w < 4; ++w)
                    if (sl[w] < minl || (sl[w] == minl && sp[w] < pos)) {
                        minl = sl[w];
                        pos = sp[w];
                    }
            }
            // every incidence latency is finite (validated), so pos is a real entry
            const double rmin = g.erel[g.inc_eid[pos]];
            lat = 2.0 * minl;
            rel = rmin * rmin;
            hops = 2;
            kind = SHADOWTOPO_KIND_SELF;
        }
    }
    if (tid == 0) {
        self_lat[i] = lat;
        self_rel[i] = rel;
        self_hops[i] = hops;
        self_kind[i] = kind;
    }
}

// ---------------------------------------------------------------- pair dispatch
struct PairOut {
    double lat, rel;
    uint32_t hops;
    uint8_t kind;
    bool taint;
};

// _topology_lookupDirectPath (topology.c:1877-1927)
__device__ __forceinline__ void direct_pair(const GraphDev& g, int32_t s, int32_t t, PairOut& o) {
    const int32_t eid = get_eid(g, s, t);
    if (eid < 0) return;  // reference: undefined (attribute read at edge -1)
    o.lat = 0.0 + g.elat[eid];
    o.rel = (g.vfac[s] * g.vfac[t]) * g.erel[eid];
    o.hops = 1;
    o.kind = SHADOWTOPO_KIND_DIRECT;
}

// returns true if the pair is not a shortest-path pair (handled here)
__device__ __forceinline__ bool dispatch_pair(const GraphDev& g, int32_t s, int32_t t, int32_t ti,
                                              const double* self_lat, const double* self_rel,
                                              const uint32_t* self_hops, const uint8_t* self_kind, PairOut& o) {
    o.lat = -1.0;
    o.rel = -1.0;
    o.hops = 0;
    o.kind = SHADOWTOPO_KIND_NONE;
    o.taint = false;
    const bool complete = g.flags & SHADOWTOPO_F_COMPLETE;
    if (complete) {
        direct_pair(g, s, t, o);
        return true;
    }
    if (g.flags & SHADOWTOPO_F_PREFER_DIRECT) {
        if (get_eid(g, s, t) >= 0) {
            direct_pair(g, s, t, o);
            return true;
        }
    }
    if (s == t) {
        o.lat = self_lat[ti];
        o.rel = self_rel[ti];
        o.hops = self_hops[ti];
        o.kind = self_kind[ti];
        return true;
    }
    return false;
}

// forward fold over the tree path (topology.c:1473-1499): lat from 0.0, rel from
// (1-ls)*(1-lt), each hop's edge = get_eid edge; used only when the target carries vertex
// loss != 0 or the graph has parallel edges of different latency.  The path x_0 = s .. x_h = t
// is known backwards only (arc a_i = P(x_i) enters x_i from x_{i-1}), and the fold runs
// forwards, so a walk from t stores the arcs in LDS scratch (WALK_SEG per chain, stride
// COMPOSE_T) and folds them in order: h steps when h <= WALK_SEG, segments of WALK_SEG arcs
// (each re-walked from t) beyond.  Two targets' walks run in lockstep per lane (two
// independent load chains in flight: a step is a dependent record load then an arc-tail
// load).  Bounded: every step checks the arc and the vertex it leads to, and a walk must
// arrive at s after exactly h arcs and never before; a walk that fails sets an error bit
// (1: out of range, 2: hop count disagrees) for compose to report, instead of following
// garbage through memory (a non-converged state's records need not form a tree).
constexpr int WALK_SEG = 8;
struct WalkChain {
    int32_t s, t;  // source, target (relaxation view ids)
    int32_t l;     // the source's lane in its batch
    uint32_t h;    // hop count the tree recorded
    bool on;       // this chain walks
    double lat, rel;
};

// one 16-byte load per hop of a walk: the arc's tail (the next vertex), its get_eid edge (for
// a multigraph's latency) and its reliability factor in_r (k_arcinfo builds it from the view's
// in-CSR when some pair needs a walk)
struct __attribute__((aligned(16))) ArcInfo {
    int32_t u, eid;
    double r;
};

__global__ __launch_bounds__(256) void k_arcinfo(const int32_t* __restrict__ in_src, const int32_t* __restrict__ in_eid,
                                                 const double* __restrict__ in_r, int64_t n, ArcInfo* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        ArcInfo a;
        a.u = in_src[i];
        a.eid = in_eid[i];
        a.r = in_r[i];
        out[i] = a;
    }
}

// 512 threads: 8 targets per wave instead of 16 (the per-lane pair values live in registers
// until the transposes: 132 VGPRs at 16, occupancy 3)
constexpr int COMPOSE_T = 512;
__global__ __launch_bounds__(COMPOSE_T) void k_compose(GraphDev g, Pools pools,
                                                 const int32_t* __restrict__ attached, int32_t A,
                                                 const double* __restrict__ self_lat,
                                                 const double* __restrict__ self_rel,
                                                 const uint32_t* __restrict__ self_hops,
                                                 const uint8_t* __restrict__ self_kind, double* out_lat,
                                                 double* out_rel, uint32_t* out_hops, uint8_t* out_kind,
                                                 int32_t row_base, int32_t ls) {
    __shared__ double sd[64 * 65];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const BatchDev B = batch_view(pools, blockIdx.y);
    const int32_t t0 = blockIdx.x * 64;
    const int32_t s = B.srcv[lane];
    constexpr int PT = 64 / (COMPOSE_T / 64);  // targets per wave
    double vl[PT], vr[PT];
    uint32_t vh[PT];
    uint8_t vk[PT];
    bool taint_any = false;
#pragma unroll
    for (int i = 0; i < PT; ++i) {
        const int32_t ti = t0 + wave * PT + i;
        PairOut o;
        o.lat = -1.0;
        o.rel = -1.0;
        o.hops = 0;
        o.kind = 0;
        o.taint = false;
        if (ti < A && s >= 0) {
            const int32_t t = attached[ti];
            if (!dispatch_pair(g, s, t, ti, self_lat, self_rel, self_hops, self_kind, o)) {
                const size_t idx = (size_t)t * KL + lane;
                const double d = B.D[idx];
                if (d < dinf()) {
                    o.lat = (d == 0) ? 1.0 : d;  // topology.c:1848-1852
                    o.kind = SHADOWTOPO_KIND_DIJKSTRA;
                    if (B.Q) {
                        const Rec q = rec_load(B.Q + idx);
                        const uint32_t h = q.h;
                        o.taint = (h & TAINT) != 0;
                        o.hops = h & HMASK;
                        // the tree fold (k_walk re-folds the targets with vertex loss, and every
                        // pair of a multigraph, in the reference's order)
                        o.rel = q.r;
                    }  // lean rounds: hops, rel and the taint come from k_walk_lean
                }
            }
        }
        taint_any |= o.taint;
        vl[i] = o.lat;
        vr[i] = o.rel;
        vh[i] = o.hops;
        vk[i] = o.kind;
    }
    if (taint_any) atomicOr(B.mask, 1ull << lane);

    const int32_t nrow = 64;
    // lat
#pragma unroll
    for (int i = 0; i < PT; ++i) sd[lane * 65 + wave * PT + i] = vl[i];
    __syncthreads();
    for (int k = threadIdx.x; k < nrow * 64; k += COMPOSE_T) {
        const int j = k >> 6, tl = k & 63;
        const int32_t r = B.row[j], ti = t0 + tl;
        if (r >= 0 && ti < A) out_lat[((size_t)(r - row_base) * A + ti) * ls] = sd[j * 65 + tl];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PT; ++i) sd[lane * 65 + wave * PT + i] = vr[i];
    __syncthreads();
    for (int k = threadIdx.x; k < nrow * 64; k += COMPOSE_T) {
        const int j = k >> 6, tl = k & 63;
        const int32_t r = B.row[j], ti = t0 + tl;
        if (r >= 0 && ti < A) out_rel[((size_t)(r - row_base) * A + ti) * ls] = sd[j * 65 + tl];
    }
    __syncthreads();
    uint32_t* su = reinterpret_cast<uint32_t*>(sd);
#pragma unroll
    for (int i = 0; i < PT; ++i) {
        su[lane * 65 + wave * PT + i] = vh[i];
        su[64 * 65 + lane * 65 + wave * PT + i] = vk[i];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nrow * 64; k += COMPOSE_T) {
        const int j = k >> 6, tl = k & 63;
        const int32_t r = B.row[j], ti = t0 + tl;
        if (r >= 0 && ti < A) {
            if (out_hops) out_hops[(size_t)(r - row_base) * A + ti] = su[j * 65 + tl];
            if (out_kind) out_kind[(size_t)(r - row_base) * A + ti] = (uint8_t)su[64 * 65 + j * 65 + tl];
        }
    }
}

// The pairs whose path needs the reference's full fold (topology.c:1429-1499): targets that
// carry vertex loss (rel = ((1 * a_s) * a_t) * e_1 * ... -- a_t enters before the edges, so
// the tree's fold R(t) is not it), and every pair of a multigraph whose lowest-id parallel
// edge is not the minimum (lat from the get_eid edges).  After k_compose wrote the rows, this
// overwrites those pairs' rel (and lat) with the walked fold.
//  * Lane = source, as in the relaxation: the walks of a wave start at one target and paths
//    from nearby sources into it share their last hops, so a step's record loads fall in few
//    lines (lane = target measured 4.6 ms of walks on C4L against 4.0).
//  * A path x_0 = s .. x_h = t is known backwards only (arc a_i = P(x_i) enters x_i from
//    x_{i-1}) and the fold runs forwards, so a walk from t stores the factors of a segment
//    of WALK_SEG arcs in LDS (slot k: a_{k0+1+k}) and folds them in order: h steps when
//    h <= WALK_SEG, each further segment re-walked from t.  A step is two dependent loads:
//    the record's predecessor arc, then the arc's {tail, edge, factor} (ArcInfo).
//  * Each lane runs two walk chains, each its own state machine over the wave's list of
//    targets (chain c takes targets c, c + 2, ...): a chain that finishes a walk starts its
//    next target at once, so no lane waits for the wave's longest walk of a target.
//  * Bounded: every step checks the arc and the vertex it leads to, a walk must arrive at s
//    after exactly h arcs and never before; a failing walk sets an error bit (1: out of range,
//    2: hop count disagrees) that compute_rows reports, instead of following garbage through
//    memory (a non-converged state's records need not form a tree).
constexpr int WALK_T = 256;
template <bool MG, int TPW, int NC>
__global__ __launch_bounds__(WALK_T) void k_walk(GraphDev g, const ArcInfo* __restrict__ ai, Pools pools,
                                                const int32_t* __restrict__ attached,
                                                const int32_t* __restrict__ walk_ti, int32_t nw, int32_t A,
                                                double* out_lat, double* out_rel, int32_t row_base, int32_t ls) {
    __shared__ double sc[NC * WALK_SEG * WALK_T];
    __shared__ int32_t se[MG ? NC * WALK_SEG * WALK_T : 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const BatchDev B = batch_view(pools, blockIdx.y);
    const int32_t sv = B.srcv[lane], row = B.row[lane];
    const bool prefer = (g.flags & SHADOWTOPO_F_PREFER_DIRECT) != 0;
    const int64_t na = g.in_ptr[g.V];
    const double fs = sv >= 0 ? g.vfac[sv] : 1.0;
    const int32_t kb = (blockIdx.x * (WALK_T / 64) + wave) * TPW;
    const int32_t ke = min(nw, kb + TPW);
    uint32_t err = 0;
    int32_t j[NC], ti[NC], t[NC], x[NC];
    uint32_t h[NC], i[NC], k0[NC];
    double rel[NC], lat[NC];
    bool act[NC];
    // chain c's next walkable target of the list (a shortest-path pair of the dispatch's rule
    // 3: not the self pair, not a direct pair of a prefer-direct graph, reached), set up
    auto start = [&](int c) {
        act[c] = false;
        while (j[c] < ke) {
            const int32_t k = j[c];
            j[c] += NC;
            const int32_t tk = walk_ti[k], tv = attached[tk];
            if (sv < 0 || row < 0 || sv == tv || (prefer && get_eid(g, sv, tv) >= 0)) continue;
            const size_t idx = (size_t)tv * KL + lane;
            if (!(B.D[idx] < dinf())) continue;
            const uint32_t hh = B.Q[idx].h & HMASK;
            if (hh == 0 || hh > (uint32_t)g.V) {
                err |= 2u;
                continue;
            }
            ti[c] = tk;
            t[c] = x[c] = tv;
            h[c] = i[c] = hh;  // x = x_i: the next step takes a_i and moves to x_{i-1}
            k0[c] = 0;
            rel[c] = fs * g.vfac[tv];
            lat[c] = 0.0;
            act[c] = true;
            return;
        }
    };
    double* scl = sc + threadIdx.x;
    int32_t* sel = se + (MG ? threadIdx.x : 0);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        j[c] = kb + c;
        start(c);
    }
    auto any_act = [&]() {
        bool r = false;
#pragma unroll
        for (int c = 0; c < NC; ++c) r |= act[c];
        return r;
    };
    while (any_act()) {
        int32_t p[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) p[c] = act[c] ? B.Q[(size_t)x[c] * KL + lane].p : 0;
        u32x4 v[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const bool okp = p[c] >= 0 && (int64_t)p[c] < na;
            if (act[c] && !okp) err |= 1u;
            act[c] = act[c] && okp;
            if (act[c]) v[c] = *(const __attribute__((address_space(1))) u32x4*)(ai + p[c]);
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (!act[c]) continue;
            const int32_t u = (int32_t)v[c].x;
            if (i[c] <= k0[c] + WALK_SEG) {
                const size_t q = (size_t)(c * WALK_SEG + (i[c] - k0[c] - 1)) * WALK_T;
                scl[q] = __longlong_as_double((long long)(((unsigned long long)v[c].w << 32) | v[c].z));
                if (MG) sel[q] = (int32_t)v[c].y;
            }
            if (u < 0 || u >= g.V || (u == sv) != (i[c] == 1)) {
                err |= (u < 0 || u >= g.V) ? 1u : 2u;
                start(c);  // this walk is abandoned; compute_rows reports the error
                continue;
            }
            x[c] = u;
            if (--i[c] > k0[c]) continue;
            // the segment's arcs a_{k0+1} .. a_{k1} are in slots 0 .. k1 - k0 - 1: fold them forwards
            const uint32_t n = min(h[c], k0[c] + (uint32_t)WALK_SEG) - k0[c];
            for (uint32_t k = 0; k < n; ++k) {
                const size_t q = (size_t)(c * WALK_SEG + k) * WALK_T;
                rel[c] *= scl[q];
                if (MG) lat[c] += g.elat[sel[q]];
            }
            k0[c] += WALK_SEG;
            if (k0[c] < h[c]) {  // the next segment: walk again from t
                x[c] = t[c];
                i[c] = h[c];
                continue;
            }
            const size_t o = ((size_t)(row - row_base) * A + ti[c]) * ls;
            out_rel[o] = rel[c];
            if (MG) out_lat[o] = (lat[c] == 0) ? 1.0 : lat[c];
            start(c);
        }
    }
    if (err) atomicOr(pools.err, (unsigned long long)err);
}

// Lean rounds (OPT_CSR_LEAN): the rounds kept D and the predecessor arc with its local tie bit
// (P32) only, so every shortest-path pair's hop count, reliability fold and taint come from a
// walk of its tree path here, after k_compose wrote the rows (lat = d(t) and the kinds; the
// direct and self pairs are complete).  One target per wave, lane = source (as k_walk).  The
// hop count is unknown until the walk reaches s, so the first pass keeps the factors of the
// last WALK_SEG arcs it took in a ring (slot = step mod WALK_SEG): those are a_1 .. a_min(h, 8),
// the fold's first segment; paths longer than a segment re-walk from t per further segment.
// The taint is the OR of the local tie bits along the path (the rounds with the tree fold
// carry it down the tree instead).  Bounded like k_walk: every arc and vertex range-checked,
// at most V hops, an error bit instead of a wild walk.
template <bool MG, int TPW, int NC>
__global__ __launch_bounds__(WALK_T) void k_walk_lean(GraphDev g, const ArcInfo* __restrict__ ai, Pools pools,
                                                     const int32_t* __restrict__ attached, int32_t A, double* out_lat,
                                                     double* out_rel, uint32_t* out_hops, int32_t row_base,
                                                     int32_t ls) {
    // NC walks per lane in lockstep, each a state machine over the wave's TPW targets
    // (chain c takes targets c, c + NC, ...): phase 0 walks t -> s keeping the last WALK_SEG
    // factors in a ring (the hop count is unknown until s), phase 1 re-walks a further segment
    __shared__ double sc[NC * WALK_SEG * WALK_T];
    __shared__ int32_t se[MG ? NC * WALK_SEG * WALK_T : 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const BatchDev B = batch_view(pools, blockIdx.y);
    const int32_t sv = B.srcv[lane], row = B.row[lane];
    const bool prefer = (g.flags & SHADOWTOPO_F_PREFER_DIRECT) != 0;
    const int64_t na = g.in_ptr[g.V];
    const double fs = sv >= 0 ? g.vfac[sv] : 1.0;
    const int32_t kb = (blockIdx.x * (WALK_T / 64) + wave) * TPW;
    const int32_t ke = min(A, kb + TPW);
    uint32_t err = 0;
    unsigned long long tmask = 0ull;  // this lane's tainted pairs (any target): one bit, the lane's
    int32_t j[NC], ti[NC], t[NC], x[NC];
    uint32_t h[NC], i[NC], k0[NC];
    int phase[NC];
    bool act[NC], taint[NC];
    double rel[NC], lat[NC];
    auto slot = [&](int c, uint32_t k) { return (size_t)(c * WALK_SEG + k) * WALK_T + threadIdx.x; };
    // chain c's next walkable target (a shortest-path pair of the dispatch's rule 3: not the
    // self pair, not a direct pair of a prefer-direct graph, reached)
    auto start = [&](int c) {
        act[c] = false;
        while (j[c] < ke) {
            const int32_t k = j[c];
            j[c] += NC;
            const int32_t tv = attached[k];
            if (sv < 0 || row < 0 || sv == tv || (prefer && get_eid(g, sv, tv) >= 0)) continue;
            if (!(B.D[(size_t)tv * KL + lane] < dinf())) continue;
            ti[c] = k;
            t[c] = x[c] = tv;
            h[c] = 0;
            k0[c] = 0;
            phase[c] = 0;
            taint[c] = false;
            rel[c] = fs * g.vfac[tv];
            lat[c] = 0.0;
            act[c] = true;
            return;
        }
    };
    auto finish = [&](int c) {
        const size_t o = (size_t)(row - row_base) * A + ti[c];
        out_rel[o * ls] = rel[c];
        if (MG) out_lat[o * ls] = (lat[c] == 0) ? 1.0 : lat[c];
        if (out_hops) out_hops[o] = h[c];
        if (taint[c]) tmask = 1ull;
        start(c);
    };
    auto fold = [&](int c, uint32_t n, bool ring) {  // a_{k0+1} .. a_{k0+n} forwards
        for (uint32_t k = 0; k < n; ++k) {
            // ring (phase 0): a_i was taken at step h - i; segments: slot i - k0 - 1
            const size_t q = slot(c, ring ? (h[c] - 1 - k) % WALK_SEG : k);
            rel[c] *= sc[q];
            if (MG) lat[c] += g.elat[se[q]];
        }
    };
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        j[c] = kb + c;
        start(c);
    }
    for (;;) {
        bool any = false;
#pragma unroll
        for (int c = 0; c < NC; ++c) any |= act[c];
        if (!any) break;
        int32_t q[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) q[c] = act[c] ? B.P32[(size_t)x[c] * KL + lane] : 0;
        u32x4 v[NC];
        bool okp[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            okp[c] = act[c] && (int64_t)(q[c] & P_MASK) < na;
            if (okp[c]) v[c] = *(const __attribute__((address_space(1))) u32x4*)(ai + (q[c] & P_MASK));
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (!act[c]) continue;
            if (!okp[c]) {  // an arc past the range: abandoned, compute_rows reports the error
                err |= 1u;
                start(c);
                continue;
            }
            const int32_t u = (int32_t)v[c].x;
            const double r = __longlong_as_double((long long)(((unsigned long long)v[c].w << 32) | v[c].z));
            if (u < 0 || u >= g.V) {
                err |= 1u;
                start(c);
                continue;
            }
            if (phase[c] == 0) {
                taint[c] |= q[c] < 0;
                const size_t qs = slot(c, h[c] % WALK_SEG);
                sc[qs] = r;
                if (MG) se[qs] = (int32_t)v[c].y;
                ++h[c];
                if (u != sv) {
                    if (h[c] >= (uint32_t)g.V) {  // longer than any simple path: not a tree
                        err |= 2u;
                        start(c);
                    } else {
                        x[c] = u;
                    }
                    continue;
                }
                fold(c, min(h[c], (uint32_t)WALK_SEG), true);
                if (h[c] <= WALK_SEG) {
                    finish(c);
                    continue;
                }
                phase[c] = 1;  // further segments, each walked from t again
                k0[c] = WALK_SEG;
                x[c] = t[c];
                i[c] = h[c];
                continue;
            }
            // phase 1: x = x_i, taking a_i; the segment holds a_{k0+1} .. a_{k1}
            if (i[c] <= k0[c] + WALK_SEG) {
                const size_t qs = slot(c, i[c] - k0[c] - 1);
                sc[qs] = r;
                if (MG) se[qs] = (int32_t)v[c].y;
            }
            x[c] = u;
            if (--i[c] > k0[c]) continue;
            fold(c, min(h[c], k0[c] + (uint32_t)WALK_SEG) - k0[c], false);
            k0[c] += WALK_SEG;
            if (k0[c] < h[c]) {
                x[c] = t[c];
                i[c] = h[c];
            } else {
                finish(c);
            }
        }
    }
    const unsigned long long tm = __ballot(tmask != 0ull);
    if (lane == 0 && tm) atomicOr(B.mask, tm);
    if (err) atomicOr(pools.err, (unsigned long long)err);
}

// ---------------------------------------------------------------- heap-exact replay
// igraph_get_shortest_paths_dijkstra (mode OUT) re-executed exactly for one source per
// wave (lane 0): dists init -1, indexed 2-way max-heap on -dist with igraph_2wheap's
// shift_up / sink / modify, strict '<' relax in igraph_incident order, early exit once all
// attached targets are popped.  Used for sources whose tree crosses a d(u) tie.
struct Heap {
    double* data;
    int32_t* idx;
    int32_t* idx2;
    int32_t size;
};

__device__ __forceinline__ void hp_switch(Heap& h, int32_t a, int32_t b) {
    if (a == b) return;
    const double td = h.data[a];
    h.data[a] = h.data[b];
    h.data[b] = td;
    const int32_t i1 = h.idx[a], i2 = h.idx[b];
    h.idx[a] = i2;
    h.idx[b] = i1;
    h.idx2[i1] = b + 2;
    h.idx2[i2] = a + 2;
}
__device__ __forceinline__ void hp_shift_up(Heap& h, int32_t e) {
    while (!(e == 0 || h.data[e] < h.data[(e + 1) / 2 - 1])) {
        const int32_t p = (e + 1) / 2 - 1;
        hp_switch(h, e, p);
        e = p;
    }
}
__device__ __forceinline__ void hp_sink(Heap& h, int32_t head) {
    for (;;) {
        const int32_t l = (head + 1) * 2 - 1, r = (head + 1) * 2;
        if (l >= h.size) return;
        int32_t c;
        if (r == h.size || h.data[l] >= h.data[r])
            c = l;
        else
            c = r;
        if (h.data[head] < h.data[c]) {
            hp_switch(h, head, c);
            head = c;
        } else
            return;
    }
}

__global__ void k_replay(GraphDev g, ReplayDev rp, const int32_t* __restrict__ attached, int32_t A, int32_t njobs) {
    const int32_t slot = blockIdx.x;
    if (slot >= njobs || threadIdx.x != 0) return;
    const int32_t V = g.V;
    const size_t off = (size_t)slot * V;
    double* dist = rp.dist + off;
    int32_t* parent = rp.parent + off;
    uint8_t* tgt = rp.tgt + off;
    Heap h{rp.hdata + off, rp.hidx + off, rp.hidx2 + off, 0};
    for (int32_t v = 0; v < V; ++v) {
        dist[v] = -1.0;
        parent[v] = -1;
        tgt[v] = 0;
        h.idx2[v] = 0;
    }
    int32_t to_reach = A;
    for (int32_t i = 0; i < A; ++i) {
        if (!tgt[attached[i]])
            tgt[attached[i]] = 1;
        else
            to_reach--;
    }
    const int32_t s = rp.srcv[slot];
    dist[s] = 0.0;
    h.data[0] = 0.0;
    h.idx[0] = s;
    h.idx2[s] = 2;
    h.size = 1;
    while (h.size > 0 && to_reach > 0) {
        const int32_t minnei = h.idx[0];
        const double mindist = -h.data[0];
        hp_switch(h, 0, h.size - 1);
        h.size--;
        h.idx2[minnei] = 0;
        hp_sink(h, 0);
        if (tgt[minnei]) {
            tgt[minnei] = 0;
            to_reach--;
        }
        for (int64_t x = g.inc_ptr[minnei]; x < g.inc_ptr[minnei + 1]; ++x) {
            const int32_t edge = g.inc_eid[x];
            const int32_t tto = (g.efrom[edge] == minnei) ? g.eto[edge] : g.efrom[edge];
            const double altdist = mindist + g.elat[edge];
            const double curdist = dist[tto];
            if (curdist < 0) {
                dist[tto] = altdist;
                parent[tto] = edge;
                const int32_t pos = h.size++;
                h.data[pos] = -altdist;
                h.idx[pos] = tto;
                h.idx2[tto] = pos + 2;
                hp_shift_up(h, pos);
            } else if (altdist < curdist) {
                dist[tto] = altdist;
                parent[tto] = edge;
                const int32_t pos = h.idx2[tto] - 2;
                h.data[pos] = -altdist;
                hp_sink(h, pos);
                hp_shift_up(h, pos);
            }
        }
    }
}

// pair rows for replayed sources: same dispatch, shortest paths from the exact parents
__global__ void k_compose_replay(GraphDev g, ReplayDev rp, const int32_t* __restrict__ attached, int32_t A,
                                 const double* __restrict__ self_lat, const double* __restrict__ self_rel,
                                 const uint32_t* __restrict__ self_hops, const uint8_t* __restrict__ self_kind,
                                 double* out_lat, double* out_rel, uint32_t* out_hops, uint8_t* out_kind,
                                 int32_t row_base, int32_t ls) {
    const int32_t slot = blockIdx.y;
    const int32_t ti = blockIdx.x * blockDim.x + threadIdx.x;
    if (ti >= A) return;
    const int32_t s = rp.srcv[slot];
    const int32_t t = attached[ti];
    PairOut o;
    if (!dispatch_pair(g, s, t, ti, self_lat, self_rel, self_hops, self_kind, o)) {
        const size_t off = (size_t)slot * g.V;
        const double* dist = rp.dist + off;
        const int32_t* parent = rp.parent + off;
        if (dist[t] >= 0) {
            // vertex path length
            uint32_t h = 0;
            for (int32_t x = t; parent[x] >= 0; ++h) {
                const int32_t e = parent[x];
                x = (g.efrom[e] == x) ? g.eto[e] : g.efrom[e];
            }
            double lat = 0.0, rel = g.vfac[s] * g.vfac[t];
            bool ok = true;
            for (uint32_t i = 0; i < h && ok; ++i) {
                // hop i: (x_i -> x_{i+1}); walk back from t to x_{i+1}
                int32_t x = t;
                for (uint32_t k = 0; k + 1 + i < h; ++k) {
                    const int32_t e = parent[x];
                    x = (g.efrom[e] == x) ? g.eto[e] : g.efrom[e];
                }
                const int32_t e = parent[x];
                const int32_t u = (g.efrom[e] == x) ? g.eto[e] : g.efrom[e];
                const int32_t ge = get_eid(g, u, x);
                if (ge < 0) {
                    ok = false;
                    break;
                }
                lat += g.elat[ge];
                rel *= g.erel[ge];
            }
            if (ok) {
                o.lat = (lat == 0) ? 1.0 : lat;
                o.rel = rel;
                o.hops = h;
                o.kind = SHADOWTOPO_KIND_DIJKSTRA;
            }
        }
    }
    const size_t w = (size_t)(rp.row[slot] - row_base) * A + ti;
    out_lat[w * ls] = o.lat;  // ls = 2: {lat, rel} interleaved (SHADOWTOPO_MEM_HOST_LR)
    out_rel[w * ls] = o.rel;
    if (out_hops) out_hops[w] = o.hops;
    if (out_kind) out_kind[w] = o.kind;
}

// parity tooling: [V][64] -> per-source rows
__global__ void k_extract(GraphDev g, Pools pools, int32_t nsrc, double* dist, int32_t* pred,
                          uint32_t* hops, uint8_t* tie) {
    const int32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t j = blockIdx.y;
    if (v >= g.V || j >= nsrc) return;
    const BatchDev B = batch_view(pools, 0);
    const size_t idx = (size_t)v * KL + j;
    const size_t o = (size_t)j * g.V + v;
    const double d = B.D[idx];
    const bool reached = d < dinf();  // an unreached state's H / R / P were never written
    if (dist) dist[o] = d;
    if (pred) {
        const int32_t p = reached ? B.Q[idx].p : -1;
        pred[o] = p >= 0 ? g.in_src[p] : -1;
    }
    if (hops) hops[o] = reached ? B.Q[idx].h & HMASK : 0u;
    if (tie) tie[o] = (reached && (B.Q[idx].h & TAINT)) ? 1 : 0;
}

// testing (OPT_TEST_SCRAMBLE_TREE): overwrite the predecessor arc of every reached
// (vertex, source) pair but the source's own -- mode 1 past the arc range, mode 2 with the
// vertex's first in-arc (in range, but no longer a tree) -- so compose's path walks meet the
// states a convergence bug would leave; they must report an error, not fault.
__global__ void k_scramble_tree(GraphDev g, Pools pools, int32_t mode) {
    const BatchDev B = batch_view(pools, blockIdx.y);
    const int64_t na = g.in_ptr[g.V];
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)g.V * KL;
         i += (size_t)gridDim.x * blockDim.x) {
        const int32_t v = (int32_t)(i / KL);
        const int lane = (int)(i % KL);
        if (!(B.D[i] < dinf()) || B.srcv[lane] == v || B.srcv[lane] < 0) continue;
        int64_t p = na + v;
        if (mode == 2) {
            if (g.in_ptr[v + 1] == g.in_ptr[v]) continue;
            p = g.in_ptr[v];
        }
        if (B.P32)
            B.P32[i] = (int32_t)p;
        else
            B.Q[i].p = (int32_t)p;
    }
}

// ---------------------------------------------------------------- host side
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

}  // namespace

struct shadowtopo_engine {
    int32_t V = 0;
    int32_t Vp = 0;  // V rounded up to a multiple of 8 (dense tiles, padding row)
    int32_t dense = 0;
    const double* d_W = nullptr;    // dense mode: [Vp][Vp] arc latency, +inf if none
    const int32_t* d_WI = nullptr;  // dense mode: [Vp][Vp] in-arc index, -1 if none
    const double* d_WR = nullptr;   // dense mode: [Vp][Vp] in_r of that arc (the seed's reliability factors)
    const float* d_W32 = nullptr;   // dense mode: [Vp][Vp] arc latency rounded down to f32, NaN if none
    uint32_t* d_hitlog = nullptr;   // dense full sweep: per wave, per batch, per 32-row chunk: rows to settle in f64
    size_t hitlog_n = 0;
    // pruned full sweep (OPT_DENSE_PRUNE): vertex locality order and its chunk bounds
    int32_t* d_perm = nullptr;  // [Vp] row/column order (padding maps to itself)
    float* d_W32p = nullptr;    // [Vp][Vp] W32 in that order
    uint16_t* d_W16p = nullptr; // OPT_DENSE_W16: [Vp][Vp] W32p rounded down to fp16 (the chunk loop's key)
    int32_t opt_dense_w16 = 0;
    double* d_Wp = nullptr;     // [Vp][Vp] W in that order
    int32_t* d_WIp = nullptr;   // [Vp][Vp] WI in that order
    double* d_WRp = nullptr;    // [Vp][Vp] WR in that order
    int32_t* d_pos = nullptr;   // [Vp] position of each vertex in that order (perm's inverse)
    float* d_minW = nullptr;    // [nchunks][columns] min W32p over each chunk's rows
    float* d_minD = nullptr;    // [nb_cap][nchunks][64] min D32 per chunk and lane
    float* d_minW64 = nullptr;  // [nvc][nvc] min W32p over each 64 x 64 block (pruned delta rounds)
    float* d_minDc = nullptr;   // [nb_cap][nvc][64] min D32 over each 64-row chunk's changed pairs
    unsigned long long* d_cmask = nullptr;  // pruned delta: per block and live chunk, the sources that can pass
    size_t cmask_n = 0;
    size_t minDc_n = 0;
    size_t minD_n = 0;
    bool vperm_ready = false;
    std::vector<uint64_t> h_vkey;  // [V] locality key of every vertex (the order's sort key)
    int64_t E = 0;
    int64_t n_arcs = 0;
    uint32_t flags = 0;
    int32_t multigraph = 0;
    int32_t device = 0;
    GraphDev g{};
    std::vector<void*> graph_allocs;
    // Relaxation view for compute_rows (OPT_PRUNE_PENDANT): the in-CSR without the pendant
    // trees that hold no attached vertex (undirected CSR graphs), rebuilt when the attached
    // set changes; `rg` is the graph the relax rounds and compose use (g for sssp)
    GraphDev gp{};
    const GraphDev* rg = nullptr;
    std::vector<void*> prune_allocs;
    std::vector<int32_t> h_view_of;    // vertex -> its id in gp (-1 peeled); empty when gp keeps the ids
    const int32_t* d_att_view = nullptr;  // the attached list in gp's ids (a prune_allocs buffer)
    bool prune_ready = false;
    int32_t opt_prune = 1;
    int64_t pruned_vertices = 0;
    // host mirrors for shadowtopo_get_eid, copied from the device on its first call
    std::once_flag mirrors_once;
    int mirrors_rc = 0;
    std::vector<int64_t> h_in_ptr;
    std::vector<int32_t> h_in_src, h_in_eid, h_loop_eid;
    hipStream_t own_stream = nullptr;
    // attached
    int32_t A = 0;
    std::vector<int32_t> h_attached;
    std::vector<uint64_t> h_key;  // locality key per attached index (OPT_SOURCE_ORDER)
    std::vector<int32_t> h_key_order;  // attached indices sorted by h_key (stable)
    bool key_ready = false;
    int32_t opt_source_order = 1;
    int32_t opt_dense_seed = 1;
    int32_t opt_dense_prune = 1;
    int32_t* d_attached = nullptr;
    double* d_self_lat = nullptr;
    double* d_self_rel = nullptr;
    uint32_t* d_self_hops = nullptr;
    uint8_t* d_self_kind = nullptr;
    size_t att_cap = 0;       // entries d_attached / d_self_* hold
    std::vector<double> h_vfac;  // [V] 1 - vertex packetloss (1.0 when absent)
    int32_t* d_walk = nullptr;   // attached indices whose pairs k_walk re-folds
    size_t walk_cap = 0;
    int32_t n_walk = 0;
    bool walk_ready = false;
    ArcInfo* d_arcinfo = nullptr;      // k_walk's per-arc table of the relaxation graph
    size_t arcinfo_cap = 0;
    const int32_t* arcinfo_of = nullptr;
    uint64_t arcinfo_gen = 0;
    uint64_t view_gen = 0;             // ensure_pruned's rebuilds of the relaxation view
    int64_t gp_arcs = 0;               // arcs of that view
    bool self_timed = false;  // the self rule's time of this attached set was measured (self_ms)
    bool self_blk = false;    // k_self: a block per vertex (>= 128 incidence entries per vertex on average)
    hipEvent_t ev_self[2] = {nullptr, nullptr};
    hipEvent_t ev_cmp[2] = {nullptr, nullptr};  // OPT_TIMING: around k_compose
    // batch pool
    int32_t nb_cap = 0;
    Pools pools{};                       // device pools for nb_cap batch slots
    std::vector<int32_t> h_srcv, h_row;  // host staging of the per-lane tables
    std::vector<void*> batch_allocs;
    int32_t* d_cnt = nullptr;
    int32_t* h_cnt = nullptr;  // pinned
    // CSR frontier worklists (k_compact / k_relax_wl): [nb][Vp] active vertices, per-batch counts
    int4* d_wl = nullptr;  // entries {v, in_ptr[v], in_ptr[v + 1], 0}
    uint32_t* d_wlcnt = nullptr;
    uint32_t* h_wlcnt = nullptr;  // pinned [nb]
    int64_t* d_wlpre = nullptr;   // [nb + 1] item prefix, uploaded per round
    int64_t* h_wlpre = nullptr;   // pinned
    int64_t* d_tlog = nullptr;    // device-driven rounds: items per round [max rounds + 1]
    int64_t* h_tlog = nullptr;    // pinned copy of a block of rounds
    int64_t tlog_n = 0;
    int32_t opt_device_rounds = 1;  // 0 never, 1 when batches x vertices <= dev_rounds_max, 2 always
    // (r04m: C4 groups of 20 / 40 batches, 2-4 M pairs, ran 16-22 % slower device-driven: their
    // rounds take milliseconds, so the host's read-back per round is noise, while the
    // persistent kernel runs at most 7 waves per SIMD; C3, 0.77 M pairs and 0.1 ms rounds, gains)
    int64_t dev_rounds_max = (int64_t)1 << 20;
    // staging for host outputs
    void* stage = nullptr;
    size_t stage_bytes = 0;
    // pinned host destinations: group g's rows leave through staging slot g & 1 on the copy
    // stream while group g + 1 relaxes
    hipStream_t copy_stream = nullptr;
    hipEvent_t ev_comp[2] = {nullptr, nullptr}, ev_copy[2] = {nullptr, nullptr};
    // replay scratch
    ReplayDev rp{};
    bool rp_ready = false;
    std::vector<void*> rp_allocs;
    // options
    int32_t opt_nb = 0;
    int32_t opt_timing = 0;
    int64_t opt_max_rounds = 0;
    int32_t opt_force_replay = 0;
    int32_t opt_profile = 0;
    int32_t opt_dense_variant = 0;  // SHADOWTOPO_DENSE_F32 (default) or SHADOWTOPO_DENSE_F64
    int32_t opt_dense_tb = 1;       // batches per wave in the f32-filtered full sweep (1, 2 or 4)
    int32_t opt_delta_permille = 125;  // dense: delta round when a batch changed <= this share of its pairs
    int32_t opt_hbm_share = 1000;      // per mille of the batch-slot HBM budget this engine may take
    bool floor_ok = false;             // default_nb: the 24 GB budget floor was found free once
    bool floor_checked = false;        // an allocation at the floor failed once: never trust it again
    size_t pool_bytes = 0;             // device bytes the batch pools hold (ensure_batches)
    int32_t opt_worklist = 1;          // CSR rounds over compacted frontier worklists
    int32_t opt_csr_variant = SHADOWTOPO_CSR_FULL;  // CSR rounds: pull (FULL) or push (PUSH, undirected)
    int32_t trace_rounds = 0;          // SHADOWTOPO_TRACE_ROUNDS=1: one stderr line per relax round
    int32_t opt_delta_live = 2;        // dense delta rounds over live-chunk lists: 0 never, 1 always, 2 when sparse
    int32_t opt_delta_live_div = 64;   // "sparse": changed pairs <= pairs / this
    int32_t opt_delta_colbound = 2;    // pruned delta: per-destination chunk bounds (1), + per-chunk source masks (2)
    int32_t opt_sweep_spiral = 1;      // pruned sweep: chunks outward from the tile on both sides (1) or upward, wrapping (0)
    int32_t opt_sweep_win1 = 8;        // pruned sweep: size of the neighbour window after the tile's chunk (0: none);
                                       // bits 8-15: the far windows' size (0 = 64)
    int32_t opt_sweep_split = 1;       // pruned sweep as two kernels (chunk loop; exact pass + epilogue)
    int32_t opt_sweep_parts = 2;       // the split sweep's two kernels per part of the batches, one stream per part
    hipStream_t aux_stream[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_h0 = nullptr, ev_hp[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_sw[4] = {nullptr, nullptr, nullptr, nullptr};  // timing: each part's sweep end (chained rounds)
    int32_t opt_chain_parts = 1;       // the read-back-free delta rounds per sweep part, on the part's stream
    int32_t opt_fuse_mindc = 1;        // chained: round 1's chunk bounds from the exact passes' epilogues
    // part 0's share of the batches with 2 sweep parts: it is launched first and its blocks
    // take the CUs first, so an even split left part 1 finishing last (C2, 16 batches: 9 / 7
    // runs the step 3.42 -> 3.32 ms, r04zr; 10 / 6 is slower, 3.61 ms)
    int32_t opt_part0_permille = 562;
    int32_t opt_host_split = 4;        // page-locked host rows: groups a one-group computation is cut into
    int64_t opt_grid_x = (int64_t)1 << 23;  // grid_of's x limit (OPT_GRID_X)
    int32_t* d_live = nullptr;         // [nb_cap][Vp / 64] live chunk lists (k_live_chunks)
    int32_t* d_nlive = nullptr;        // [nb_cap]
    unsigned long long* d_prof = nullptr;  // = prof_buf when OPT_PROFILE is on, else NULL
    unsigned long long* prof_buf = nullptr; // [nb][8 shards][visits, changes]
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evm = nullptr, evm2 = nullptr;
    hipEvent_t ev_spin = nullptr;  // round_sync
    std::vector<hipEvent_t> ev_dev;  // device-driven rounds: one pair per round of a block
    std::vector<hipEvent_t> ev_spec;  // dense: one pair per round enqueued without a read-back
    void* d_pk_scratch = nullptr;     // row exchange codec: word counts + block sums
    size_t pk_scratch_n = 0;
    int32_t* h_cnt_spec = nullptr;    // pinned: those rounds' change counts [round][nb]
    int32_t opt_dense_spec = 2;       // dense: leading rounds enqueued without a host read-back
    int32_t opt_sweep_glds = 0;       // pruned sweep chunk loop: LDS-DMA staging (OPT_SWEEP_GLDS; r06: ties register staging)
    int32_t opt_sweep_stats = 0;      // diagnostics: staged chunks of the pruned sweeps (OPT_SWEEP_STATS)
    unsigned long long* d_sweep_hits = nullptr;  // OPT_SWEEP_STATS: the exact passes' logged rows
    int32_t opt_sweep_waves = 4;      // pruned sweep chunk loop: waves per block, 4 or 8 (OPT_SWEEP_WAVES)
    int32_t opt_sweep_refilter = 0;   // exact pass re-tests logged rows against the final thresholds (OPT_SWEEP_REFILTER)
    int32_t opt_seed_skip = 1;        // round-0 exact pass leaves untainted seed winners unread (OPT_SEED_SKIP)
    int32_t opt_delta_w16 = 1;        // pruned delta rounds filter with fp16 slabs (OPT_DELTA_W16)
    float* d_thrio = nullptr;         // refilter: the chunk loops' final thresholds [batch][Vp][64]
    size_t thrio_n = 0;
    int32_t opt_heavy_first = 1;      // pruned sweep parts: heavy-first block order (k_heavy_order)
    int32_t opt_csr_lean = 2;         // OPT_CSR_LEAN: sparse rounds with D + P32 only (1), the tree fold (0), auto (2)
    bool lean_next = false;           // the layout the next pool allocation takes (decided per computation)
    ViewBufs vb;                      // the pendant-pruned view's device buffers (kept across attached sets)
    size_t view_cap_a = 0;            // attached rows vb.att holds (0: not allocated)
    int32_t opt_host_groups = 0;      // OPT_HOST_GROUPS: page-locked host rows in this many groups (0: automatic)
    int32_t opt_spin_us = 20000;      // OPT_SPIN_US: host waits poll this long before a blocking wait (a blocking
                                      // wait's wake-up cost C3's host-delivered build 13 ms of 31, r05c3t)
    int32_t opt_spec_compose = 1;     // OPT_SPEC_COMPOSE: dense compose enqueued behind a delta round (1)
    unsigned long long* h_masks = nullptr;  // pinned: the compose's error word and tie masks, read back
    size_t h_masks_n = 0;
    int32_t opt_csr_incremental = 32; // OPT_CSR_INCREMENTAL: lean visits of vertices with more in-arcs than this
                                      // read only the tails changed since (0 = off)
    int32_t opt_walk_tpw = 1;         // k_walk shape (OPT_WALK_TPW): 1 target / 1 chain, or 2 / 2
    uint32_t* d_bweight[4] = {nullptr, nullptr, nullptr, nullptr};  // per part: chunk counts per block
    int32_t* d_border[4][2] = {};     // per part: two order buffers (ping-pong across sweeps)
    size_t heavy_cap[4] = {0, 0, 0, 0};
    int64_t heavy_key[4] = {-1, -1, -1, -1};   // shape (b0, n, ntb) the sorted order buffer is for
    int64_t heavy_next[4] = {-1, -1, -1, -1};
    int heavy_buf = 0;
    int32_t opt_test_unconverged = 0; // testing: an iteration guard hands its state to compose (OPT_TEST_UNCONVERGED)
    int32_t opt_test_scramble = 0;    // testing: predecessors overwritten before compose (OPT_TEST_SCRAMBLE_TREE)
    int32_t opt_test_pool_enomem = 0; // testing: the next pool allocation fails midway (OPT_TEST_POOL_ENOMEM)
    bool unconverged = false;         // the last rounds stopped at the guard (opt_test_unconverged)
    shadowtopo_stats st{};
};

namespace {

int dev_alloc(std::vector<void*>& owner, void** p, size_t bytes) {
    if (bytes == 0) bytes = 8;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return fail(SHADOWTOPO_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    owner.push_back(*p);
    return SHADOWTOPO_OK;
}

template <typename T>
int upload(shadowtopo_engine* eng, const std::vector<T>& h, const T** out) {
    void* p = nullptr;
    int rc = dev_alloc(eng->graph_allocs, &p, h.size() * sizeof(T));
    if (rc) return rc;
    if (!h.empty()) HIP_TRY(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    *out = static_cast<const T*>(p);
    return SHADOWTOPO_OK;
}

// host twin of f32_key for finite values: the largest float <= x
float f32_round_down(double x) {
    float f = (float)x;  // round to nearest
    if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    return f;
}

// stable counting sort of `idx` by key[idx]
void counting_sort(const std::vector<int32_t>& key, int32_t nkeys, std::vector<int64_t>& idx,
                   std::vector<int64_t>& tmp) {
    std::vector<int64_t> cnt((size_t)nkeys + 1, 0);
    for (int64_t i : idx) cnt[(size_t)key[i] + 1]++;
    for (int32_t k = 0; k < nkeys; ++k) cnt[(size_t)k + 1] += cnt[k];
    tmp.resize(idx.size());
    for (int64_t i : idx) tmp[(size_t)cnt[key[i]]++] = i;
    idx.swap(tmp);
}

void free_batches(shadowtopo_engine* eng) {
    for (void* p : eng->batch_allocs) (void)hipFree(p);
    eng->batch_allocs.clear();
    eng->pool_bytes = 0;
    eng->pools = Pools{};
    eng->d_cnt = nullptr;
    if (eng->h_cnt) (void)hipHostFree(eng->h_cnt);
    eng->h_cnt = nullptr;
    if (eng->h_cnt_spec) (void)hipHostFree(eng->h_cnt_spec);
    eng->h_cnt_spec = nullptr;
    if (eng->h_wlcnt) (void)hipHostFree(eng->h_wlcnt);
    if (eng->h_wlpre) (void)hipHostFree(eng->h_wlpre);
    eng->h_wlcnt = nullptr;
    eng->h_wlpre = nullptr;
    eng->d_wl = nullptr;
    eng->d_wlcnt = nullptr;
    eng->d_wlpre = nullptr;
    eng->d_live = nullptr;
    eng->d_nlive = nullptr;
    eng->h_srcv.clear();
    eng->h_row.clear();
    eng->nb_cap = 0;
}

// state rows per batch slot of the graph the next rounds run on (the relaxation view's, a
// renumbered pendant-pruned view being smaller than the graph)
int32_t pool_vp(const shadowtopo_engine* eng) { return eng->rg ? eng->rg->Vp : eng->Vp; }

bool state_bdu(const shadowtopo_engine* eng) { return eng->dense != 0; }
bool state_d32(const shadowtopo_engine* eng) { return eng->dense != 0; }
// bytes per (vertex, source) of the batch pools
double state_bytes(const shadowtopo_engine* eng) {
    return (eng->lean_next ? 12.0 : 24.0) + (state_bdu(eng) ? 8.0 : 0.0) + (state_d32(eng) ? 4.0 : 0.0);
}

int ensure_batches_impl(shadowtopo_engine* eng, int32_t nb);
int ensure_batches(shadowtopo_engine* eng, int32_t nb) {
    // pools with at least the rows the relaxation graph needs are kept (their row stride is
    // pools.Vp everywhere): a new attached set's pendant-pruned view differs by a few rows,
    // and reallocating C5's ~140 GB of pools for that cost 1.2 s of a fresh build (r05j)
    if (eng->nb_cap >= nb && eng->pools.Vp >= pool_vp(eng) && (eng->pools.P32 != nullptr) == eng->lean_next)
        return SHADOWTOPO_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = ensure_batches_impl(eng, nb);
    eng->st.pool_allocs++;
    eng->st.pool_alloc_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    // exactly one predecessor state: the kernels pick the tree fold or the lean form by which
    // pool pointer is set (batch_view passes an absent pool on as NULL, never as NULL + offset:
    // r05r's fault was k_seed storing a source record through such a pointer in batch >= 1)
    if (rc == SHADOWTOPO_OK && ((eng->pools.Q != nullptr) == (eng->pools.P32 != nullptr) ||
                                (eng->pools.P32 != nullptr) != eng->lean_next))
        return fail(SHADOWTOPO_EINTERNAL, "batch pools: tree records and lean predecessor state both or neither present");
    return rc;
}
int ensure_batches_impl(shadowtopo_engine* eng, int32_t nb) {
    free_batches(eng);
    const auto dev_alloc = [eng](std::vector<void*>& owner, void** p, size_t bytes) {
        // default_nb counts what the pools hold, not an estimate: only allocations that
        // succeeded (a failed one is not held, and ENOMEM's retry sizes from free + held)
        const int rc = ::dev_alloc(owner, p, bytes);
        if (rc == SHADOWTOPO_OK) eng->pool_bytes += bytes;
        return rc;
    };
    // a pruned view's rows with 1/64 headroom (another attached set's view fits the same pools)
    const int32_t pvp0 = pool_vp(eng);
    const int32_t pvp = pvp0 < eng->Vp ? std::min(eng->Vp, (pvp0 + pvp0 / 64 + 63) / 64 * 64) : pvp0;
    const size_t VK = (size_t)pvp * KL;
    Pools& P = eng->pools;
    P.vk = (int64_t)VK;
    P.Vp = pvp;
    int rc;
    if ((rc = dev_alloc(eng->batch_allocs, (void**)&P.D, VK * nb * sizeof(double)))) return rc;
    if (eng->opt_test_pool_enomem) {  // testing: HBM taken by someone else after the budget query
        eng->opt_test_pool_enomem = 0;
        return fail(SHADOWTOPO_ENOMEM, "injected pool allocation failure (OPT_TEST_POOL_ENOMEM)");
    }
    // the tree record (R, H, P: 16 B) or, for lean rounds, the predecessor arc alone (4 B)
    if ((rc = eng->lean_next ? dev_alloc(eng->batch_allocs, (void**)&P.P32, VK * nb * sizeof(int32_t))
                             : dev_alloc(eng->batch_allocs, (void**)&P.Q, VK * nb * sizeof(Rec))) ||
        (rc = dev_alloc(eng->batch_allocs, (void**)&P.act, (size_t)pvp * 2 * nb)) ||
        (eng->lean_next && (rc = dev_alloc(eng->batch_allocs, (void**)&P.stamp, (size_t)pvp * nb))) ||
        (rc = dev_alloc(eng->batch_allocs, (void**)&P.srcv, sizeof(int32_t) * KL * nb)) ||
        (rc = dev_alloc(eng->batch_allocs, (void**)&P.row, sizeof(int32_t) * KL * nb)) ||
        (rc = dev_alloc(eng->batch_allocs, (void**)&P.err, sizeof(unsigned long long) * (nb + 1))))
        return rc;
    P.mask = P.err + 1;
    // BDU (the lexicographic key) only for the kernels that fold into a recorded state, D32
    // only for the f32-filtered ones: the FULL CSR rounds keep 24 bytes per (vertex, source)
    if (state_bdu(eng) && (rc = dev_alloc(eng->batch_allocs, (void**)&P.BDU, VK * nb * sizeof(double)))) return rc;
    if ((rc = dev_alloc(eng->batch_allocs, (void**)&P.chm, sizeof(unsigned long long) * 2 * pvp * nb))) return rc;
    if (state_d32(eng) && (rc = dev_alloc(eng->batch_allocs, (void**)&P.D32, VK * nb * sizeof(float)))) return rc;
    eng->h_srcv.assign((size_t)KL * nb, -1);
    eng->h_row.assign((size_t)KL * nb, -1);
    if ((rc = dev_alloc(eng->batch_allocs, (void**)&eng->d_cnt, sizeof(int32_t) * CNT_ROWS * nb))) return rc;
    HIP_TRY(hipHostMalloc((void**)&eng->h_cnt, sizeof(int32_t) * nb, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&eng->h_cnt_spec, sizeof(int32_t) * nb * (SPEC_MAX + 1), hipHostMallocDefault));
    if (!eng->dense) {
        if ((rc = dev_alloc(eng->batch_allocs, (void**)&eng->d_wl, sizeof(int4) * VK / KL * nb)) ||
            (rc = dev_alloc(eng->batch_allocs, (void**)&eng->d_wlcnt, sizeof(uint32_t) * nb)) ||
            (rc = dev_alloc(eng->batch_allocs, (void**)&eng->d_wlpre, sizeof(int64_t) * (nb + 1))))
            return rc;
        HIP_TRY(hipHostMalloc((void**)&eng->h_wlcnt, sizeof(uint32_t) * nb, hipHostMallocDefault));
        HIP_TRY(hipHostMalloc((void**)&eng->h_wlpre, sizeof(int64_t) * (nb + 1), hipHostMallocDefault));
    }
    if ((rc = dev_alloc(eng->batch_allocs, (void**)&eng->prof_buf, sizeof(unsigned long long) * 16 * nb))) return rc;
    eng->nb_cap = nb;
    return SHADOWTOPO_OK;
}

int ensure_replay(shadowtopo_engine* eng) {
    if (eng->rp_ready) return SHADOWTOPO_OK;
    const size_t n = (size_t)REPLAY_SLOTS * eng->V;
    ReplayDev& r = eng->rp;
    int rc;
    if ((rc = dev_alloc(eng->rp_allocs, (void**)&r.dist, n * sizeof(double)))) return rc;
    if ((rc = dev_alloc(eng->rp_allocs, (void**)&r.parent, n * sizeof(int32_t)))) return rc;
    if ((rc = dev_alloc(eng->rp_allocs, (void**)&r.hdata, n * sizeof(double)))) return rc;
    if ((rc = dev_alloc(eng->rp_allocs, (void**)&r.hidx, n * sizeof(int32_t)))) return rc;
    if ((rc = dev_alloc(eng->rp_allocs, (void**)&r.hidx2, n * sizeof(int32_t)))) return rc;
    if ((rc = dev_alloc(eng->rp_allocs, (void**)&r.tgt, n))) return rc;
    eng->rp_ready = true;
    return SHADOWTOPO_OK;
}

// batch slots in flight: enough for every requested row when HBM allows.  Sparse rounds
// cost a launch + a flag read-back each, so more batches per round means fewer rounds in
// total; the budget is 55 % of the free HBM (MI355X: 288 GB) beside the resident graph, never
// under 24 GB (times the share) -- a floor that holds every requested batch skips the query
// only when it is itself within the device's capacity.
// The host's waits on the device (a round's counts decide the next launch; the copy stream's
// last rows): poll an event for up to opt_spin_us (default 20 ms) before falling back to a
// blocking wait.  A blocking synchronisation sleeps, and its wake-up added tens of
// microseconds to each of a C2 step's waits and ~0.4 ms to each of C3's host-delivered
// build's ~30 waits beside the row copies (31 -> 18 ms with a 5 ms budget, r05c3t).
// Past the first 200 us the poll yields the core between queries (r06 advisor: a multi-second
// C5 build, or 8 ranks on one host, kept a core busy that Shadow's worker threads could use);
// sched_yield returns at once when no other thread is runnable, so an idle host loses nothing.
hipError_t spin_event(const shadowtopo_engine* eng, hipEvent_t ev) {
    hipError_t e;
    const auto t0 = std::chrono::steady_clock::now();
    const auto hot = std::chrono::microseconds(std::min(eng->opt_spin_us, 200));
    const auto budget = std::chrono::microseconds(eng->opt_spin_us);
    while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
        const auto el = std::chrono::steady_clock::now() - t0;
        if (el > budget) return hipEventSynchronize(ev);
        if (el > hot) sched_yield();
    }
    return e;
}
hipError_t round_sync(shadowtopo_engine* eng, hipStream_t s) {
    hipError_t e = hipEventRecord(eng->ev_spin, s);
    if (e != hipSuccess) return e;
    return spin_event(eng, eng->ev_spin);
}

int32_t default_nb(shadowtopo_engine* eng, int32_t rows) {
    const int32_t need = std::max(1, (rows + KL - 1) / KL);
    if (eng->opt_nb > 0) return std::min(eng->opt_nb, need);
    // ensure_batches' allocations per slot: the state, act flags (2 B) and change masks
    // (16 B) per vertex, the worklist (16 B per vertex, sparse), and the per-lane tables
    const double pvp = (double)pool_vp(eng);
    const double per_batch = pvp * KL * state_bytes(eng) + 18.0 * pvp + (eng->dense ? 0.0 : 16.0 * pvp) + 8.0 * KL + 160.0;
    const double cap = eng->dense ? 16.0 : 256.0;
    // the budget is never under a 24 GB floor (times the share) once one free-memory query of
    // this engine found the floor free: when it already holds every batch, later calls (one
    // per step) answer without the driver's query
    const double floor_b = 24.0e9 * eng->opt_hbm_share / 1000.0;
    if (eng->floor_ok && std::min(cap, std::floor(floor_b / per_batch)) >= (double)need) return need;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    // the slots this engine already owns, as allocated: an estimate above the real size would
    // grow the budget from one call to the next and reallocate the pools every step (r03: C5
    // paid 1.3 s per step for that after the change-record pool was dropped)
    const double held = (double)eng->pool_bytes;
    if ((double)free_b + held >= floor_b && !eng->floor_checked) eng->floor_ok = true;
    // engines sharing one device (SHADOWTOPO_DEVICES listing it twice) split the budget
    const double budget = std::max(eng->floor_ok ? floor_b : 0.0,
                                   0.55 * ((double)free_b + held) * eng->opt_hbm_share / 1000.0);
    const int32_t nb = (int32_t)std::max(1.0, std::min(cap, std::floor(budget / per_batch)));
    return std::min(nb, need);
}

// the self rule (k_self) of attached rows [i0, i1) into l / r / h / k, on stream s, with no
// host synchronisation
hipError_t launch_self(const shadowtopo_engine* eng, const GraphDev& g, int32_t i0, int32_t i1, double* l, double* r,
                       uint32_t* h, uint8_t* k, hipStream_t s) {
    if (i1 <= i0) return hipSuccess;
    const int32_t n = i1 - i0;
    if (eng->self_blk)
        hipLaunchKernelGGL(k_self<true>, dim3((uint32_t)n), dim3(256), 0, s, g, eng->d_attached, i0, i1, l, r, h, k);
    else
        hipLaunchKernelGGL(k_self<false>, dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, s, g, eng->d_attached, i0, i1,
                           l, r, h, k);
    return hipGetLastError();
}

// the pools of batches b0, b0 + 1, ... as a pool set of their own (one part of the batches)
Pools pools_from(const Pools& in, int32_t b0) {
    Pools P = in;
    const size_t o = (size_t)b0 * (size_t)P.vk;
    P.D += o;
    if (P.Q) P.Q += o;
    if (P.P32) P.P32 += o;
    if (P.stamp) P.stamp += (size_t)b0 * P.Vp;
    P.act += (size_t)b0 * 2 * P.Vp;
    P.srcv += (size_t)b0 * KL;
    P.row += (size_t)b0 * KL;
    P.mask += b0;
    if (P.BDU) P.BDU += o;
    if (P.chm) P.chm += (size_t)b0 * 2 * P.Vp;
    if (P.D32) P.D32 += o;
    return P;
}

// W16p (OPT_DENSE_W16's chunk loop, OPT_DELTA_W16's delta slabs): W32p rounded toward -inf
// to fp16, built once on stream s (W32p never changes after ensure_vperm)
hipError_t ensure_w16p(shadowtopo_engine* eng, hipStream_t s) {
    if (eng->d_W16p) return hipSuccess;
    const size_t n = (size_t)eng->Vp * eng->Vp;
    uint16_t* p = nullptr;
    hipError_t e = hipMalloc((void**)&p, n * sizeof(uint16_t));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_w16, dim3(4096), dim3(256), 0, s, eng->d_W32p, p, n);
    if ((e = hipGetLastError()) != hipSuccess) {
        (void)hipFree(p);
        return e;
    }
    eng->d_W16p = p;  // published only once its fill is enqueued
    return hipSuccess;
}

// the number of parts (one stream each) the f32 sweep of nbg batches runs in; 1: one launch
int32_t sweep_parts(const shadowtopo_engine* eng, int32_t nbg) {
    if (eng->opt_dense_variant == SHADOWTOPO_DENSE_F64 || eng->opt_dense_tb != 1 || !eng->vperm_ready ||
        !eng->opt_dense_prune || !eng->opt_sweep_split || eng->opt_dense_w16 || eng->opt_profile)
        return 1;
    return std::max<int32_t>(1, std::min(eng->opt_sweep_parts, nbg));
}

// work a part's stream takes on after its share of the sweep, before the join (run_rounds'
// chained delta rounds): (stream, first batch, batches, part)
using PartTail = std::function<hipError_t(hipStream_t, int32_t, int32_t, int)>;

// the f32-filtered full sweep: 8 destinations per wave, exact rows settled 2 at a time
template <int TB>
hipError_t launch_dense_ft(shadowtopo_engine* eng, int32_t nbg, int32_t par, int32_t thresh,
                           const int32_t* cnt_prev, int32_t* cnt_cur, hipStream_t s, const PartTail* tail,
                           float* mdc_out, int32_t seeded) {
    constexpr int TDT = FTDT, XR = 2;
    const int32_t ntb = (eng->V + 4 * TDT - 1) / (4 * TDT);
    const int32_t ngroups = (nbg + TB - 1) / TB;
    const int64_t nblocks = 8 * (((int64_t)ngroups * ntb + 7) / 8);
    const size_t nchunks = (size_t)((eng->V + SRS - 1) / SRS);
    // hit log: per (batch group, wave tile of TDT destinations), TB x nchunks row masks
    const size_t need = (size_t)ngroups * (size_t)(eng->Vp / TDT) * TB * nchunks;
    if (eng->hitlog_n < need) {
        if (eng->d_hitlog) (void)hipFree(eng->d_hitlog);
        eng->d_hitlog = nullptr;
        eng->hitlog_n = 0;
        hipError_t e = hipMalloc((void**)&eng->d_hitlog, need * sizeof(uint32_t));
        if (e != hipSuccess) return e;
        eng->hitlog_n = need;
    }
    if (eng->vperm_ready && eng->opt_dense_prune) {
        const size_t mneed = (size_t)eng->nb_cap * nchunks * KL;
        if (eng->minD_n < mneed) {
            if (eng->d_minD) (void)hipFree(eng->d_minD);
            eng->d_minD = nullptr;
            eng->minD_n = 0;
            hipError_t e = hipMalloc((void**)&eng->d_minD, mneed * sizeof(float));
            if (e != hipSuccess) return e;
            eng->minD_n = mneed;
        }
        hipLaunchKernelGGL(k_min_d32, dim3((uint32_t)((nchunks + 3) / 4), nbg), dim3(256), 0, s, eng->pools,
                           eng->d_perm, (int32_t)nchunks, eng->d_minD);
        if (TB <= 2 && eng->opt_sweep_split) {  // the chunk loop, then the exact pass + epilogue
            if (eng->opt_dense_w16) {
                hipError_t e = ensure_w16p(eng, s);
                if (e != hipSuccess) return e;
            }
            bool w16 = false;
            if constexpr (TB == 1 && TDT == 8) {
                w16 = eng->opt_dense_w16 != 0;
                if (w16)
                    hipLaunchKernelGGL((k_relax_dense_f<TDT, XR, TB, true, 1, 4, true>), dim3((uint32_t)nblocks), dim3(256),
                                       0, s, (const float*)eng->d_W16p, eng->d_Wp, eng->d_WI, eng->Vp, eng->g.in_r,
                                       eng->pools, eng->V, nbg, ntb, par, thresh, cnt_prev, cnt_cur, eng->d_prof,
                                       eng->d_hitlog, eng->d_perm, eng->d_minW, eng->d_minD, eng->d_pos, eng->d_WIp,
                                       eng->d_WRp, eng->g.vfac, eng->opt_sweep_spiral, eng->opt_sweep_win1, nullptr);
            }
            if constexpr (TB == 1) {
                const int32_t parts = sweep_parts(eng, nbg);
                if (!w16 && parts >= 2 && !eng->d_prof) {
                    // the batches in `parts` contiguous parts, one stream each: a part's exact
                    // pass runs beside another part's chunk-loop tail (results are per batch;
                    // C2, two parts: sweep 2.92 -> 2.70 ms, r04zm)
                    hipError_t e = hipSuccess;
                    if (!eng->ev_h0) e = hipEventCreateWithFlags(&eng->ev_h0, hipEventDisableTiming);
                    for (int k = 0; k < parts - 1 && e == hipSuccess; ++k) {
                        if (!eng->aux_stream[k]) e = hipStreamCreateWithFlags(&eng->aux_stream[k], hipStreamNonBlocking);
                        if (e == hipSuccess && !eng->ev_hp[k]) e = hipEventCreateWithFlags(&eng->ev_hp[k], hipEventDisableTiming);
                    }
                    // mdc_out (chained rounds): minDc, filled by the exact passes' epilogues, reset
                    // to NaN (no changed pair) first
                    if (e == hipSuccess && mdc_out)
                        e = hipMemsetD32Async((hipDeviceptr_t)mdc_out, 0x7fc00000, (size_t)nbg * (eng->Vp / KL) * KL, s);
                    if (e == hipSuccess) e = hipEventRecord(eng->ev_h0, s);
                    for (int k = 0; k < parts - 1 && e == hipSuccess; ++k) e = hipStreamWaitEvent(eng->aux_stream[k], eng->ev_h0, 0);
                    if (e != hipSuccess) return e;
                    // heavy-first block order per part (k_heavy_order): this sweep uses order
                    // buffer `cur` (sorted after the previous sweep of the same shape), the
                    // blocks record their chunk counts, and the sort for the next sweep writes
                    // buffer cur ^ 1 (no running sweep reads it)
                    if (eng->opt_sweep_stats && !eng->d_sweep_hits &&
                        (e = hipMalloc((void**)&eng->d_sweep_hits, 2 * sizeof(unsigned long long))) != hipSuccess)
                        return e;
                    if (eng->opt_sweep_stats && (e = hipMemsetAsync(eng->d_sweep_hits, 0, 2 * sizeof(unsigned long long), s)) != hipSuccess)
                        return e;
                    if (eng->opt_sweep_refilter) {
                        const size_t need_t = (size_t)nbg * eng->Vp * KL;
                        if (eng->thrio_n < need_t) {
                            if (eng->d_thrio) (void)hipFree(eng->d_thrio);
                            eng->d_thrio = nullptr;
                            eng->thrio_n = 0;
                            if ((e = hipMalloc((void**)&eng->d_thrio, need_t * sizeof(float))) != hipSuccess) return e;
                            eng->thrio_n = need_t;
                        }
                    }
                    const int cur = eng->heavy_buf;
                    HeavyArgs ha{};
                    bool sort_any = false;
                    auto part = [&](hipStream_t st, int32_t b0, int32_t n, int k) {
                        const Pools P = pools_from(eng->pools, b0);
                        uint32_t* hl = eng->d_hitlog + (size_t)b0 * (size_t)(eng->Vp / TDT) * nchunks;
                        const float* mD = eng->d_minD + (size_t)b0 * nchunks * KL;
                        const int64_t nbl = 8 * (((int64_t)n * ntb + 7) / 8);
                        // the chunk loop's blocks: 4 waves x 8 destinations, or (OPT_SWEEP_WAVES 8)
                        // 8 waves x 8: 64 destinations per block, one staged D32 chunk for twice
                        // the columns; the exact pass keeps 4-wave blocks (hit logs are per wave tile)
                        const bool w8 = eng->opt_sweep_waves == 8;
                        const int32_t ntb1 = w8 ? (eng->V + 8 * TDT - 1) / (8 * TDT) : ntb;
                        const int64_t nbl1 = 8 * (((int64_t)n * ntb1 + 7) / 8);
                        const int64_t key = ((int64_t)b0 << 42) | ((int64_t)n << 21) | ((int64_t)w8 << 20) | ntb1;
                        bool heavy = eng->opt_heavy_first && k < 4 && nbl1 / 8 <= HEAVY_MAX;
                        if (heavy && eng->heavy_cap[k] < (size_t)nbl1) {
                            for (void* q : {(void*)eng->d_bweight[k], (void*)eng->d_border[k][0], (void*)eng->d_border[k][1]})
                                if (q) (void)hipFree(q);
                            eng->d_bweight[k] = nullptr;
                            eng->d_border[k][0] = eng->d_border[k][1] = nullptr;
                            eng->heavy_cap[k] = 0;
                            eng->heavy_key[k] = -1;
                            if (hipMalloc((void**)&eng->d_bweight[k], sizeof(uint32_t) * nbl1) != hipSuccess ||
                                hipMalloc((void**)&eng->d_border[k][0], sizeof(int32_t) * nbl1) != hipSuccess ||
                                hipMalloc((void**)&eng->d_border[k][1], sizeof(int32_t) * nbl1) != hipSuccess ||
                                hipMemsetAsync(eng->d_bweight[k], 0, sizeof(uint32_t) * nbl1, st) != hipSuccess) {
                                (void)hipGetLastError();
                                heavy = false;
                            } else {
                                eng->heavy_cap[k] = (size_t)nbl1;
                            }
                        }
                        const int32_t* ord = heavy && eng->heavy_key[k] == key ? eng->d_border[k][cur] : nullptr;
                        float* tio = eng->opt_sweep_refilter ? eng->d_thrio + (size_t)b0 * eng->Vp * KL : nullptr;
                        if (w8 && eng->opt_sweep_glds)
                            hipLaunchKernelGGL((k_relax_dense_f<TDT, XR, 1, true, 1, 8, false, true>), dim3((uint32_t)nbl1),
                                               dim3(512), 0, st, eng->d_W32p, eng->d_Wp, eng->d_WI, eng->Vp, eng->g.in_r,
                                               P, eng->V, n, ntb1, par, thresh, cnt_prev + b0, cnt_cur + b0, nullptr, hl,
                                               eng->d_perm, eng->d_minW, mD, eng->d_pos, eng->d_WIp, eng->d_WRp,
                                               eng->g.vfac, eng->opt_sweep_spiral, eng->opt_sweep_win1, nullptr, ord,
                                               heavy ? eng->d_bweight[k] : nullptr, tio);
                        else if (w8)
                            hipLaunchKernelGGL((k_relax_dense_f<TDT, XR, 1, true, 1, 8, false, false>), dim3((uint32_t)nbl1),
                                               dim3(512), 0, st, eng->d_W32p, eng->d_Wp, eng->d_WI, eng->Vp, eng->g.in_r,
                                               P, eng->V, n, ntb1, par, thresh, cnt_prev + b0, cnt_cur + b0, nullptr, hl,
                                               eng->d_perm, eng->d_minW, mD, eng->d_pos, eng->d_WIp, eng->d_WRp,
                                               eng->g.vfac, eng->opt_sweep_spiral, eng->opt_sweep_win1, nullptr, ord,
                                               heavy ? eng->d_bweight[k] : nullptr, tio);
                        else if (eng->opt_sweep_glds)
                            hipLaunchKernelGGL((k_relax_dense_f<TDT, XR, 1, true, 1, 4, false, true>), dim3((uint32_t)nbl),
                                               dim3(256), 0, st, eng->d_W32p, eng->d_Wp, eng->d_WI, eng->Vp, eng->g.in_r,
                                               P, eng->V, n, ntb, par, thresh, cnt_prev + b0, cnt_cur + b0, nullptr, hl,
                                               eng->d_perm, eng->d_minW, mD, eng->d_pos, eng->d_WIp, eng->d_WRp,
                                               eng->g.vfac, eng->opt_sweep_spiral, eng->opt_sweep_win1, nullptr, ord,
                                               heavy ? eng->d_bweight[k] : nullptr, tio);
                        else
                        hipLaunchKernelGGL((k_relax_dense_f<TDT, XR, 1, true, 1>), dim3((uint32_t)nbl), dim3(256), 0, st,
                                           eng->d_W32p, eng->d_Wp, eng->d_WI, eng->Vp, eng->g.in_r, P, eng->V, n, ntb,
                                           par, thresh, cnt_prev + b0, cnt_cur + b0, nullptr, hl, eng->d_perm,
                                           eng->d_minW, mD, eng->d_pos, eng->d_WIp, eng->d_WRp, eng->g.vfac,
                                           eng->opt_sweep_spiral, eng->opt_sweep_win1, nullptr, ord,
                                           heavy ? eng->d_bweight[k] : nullptr, tio);
                        if (heavy) {
                            ha.w[k] = eng->d_bweight[k];
                            ha.o[k] = eng->d_border[k][cur ^ 1];
                            ha.slots[k] = (int32_t)(nbl1 / 8);
                            eng->heavy_next[k] = key;
                            sort_any = true;
                        } else {
                            eng->heavy_next[k] = -1;
                        }
                        hipLaunchKernelGGL((k_relax_dense_f<TDT, XR, 1, true, 2>), dim3((uint32_t)nbl), dim3(256), 0, st,
                                           eng->d_W32p, eng->d_Wp, eng->d_WI, eng->Vp, eng->g.in_r, P, eng->V, n, ntb,
                                           par, thresh, cnt_prev + b0, cnt_cur + b0,
                                           eng->opt_sweep_stats ? eng->d_sweep_hits : nullptr, hl, eng->d_perm,
                                           eng->d_minW, mD, eng->d_pos, eng->d_WIp, eng->d_WRp, eng->g.vfac,
                                           eng->opt_sweep_spiral, eng->opt_sweep_win1,
                                           mdc_out ? mdc_out + (size_t)b0 * (eng->Vp / KL) * KL : nullptr, nullptr,
                                           nullptr, tio, seeded);
                        if (tail && e == hipSuccess) e = (*tail)(st, b0, n, k);
                    };
                    auto bound = [&](int k) {
                        if (parts == 2 && k == 1 && eng->opt_part0_permille > 0)
                            return std::max<int32_t>(1, std::min<int32_t>(nbg - 1, (int32_t)(((int64_t)nbg * eng->opt_part0_permille + 500) / 1000)));
                        return (int32_t)((int64_t)nbg * k / parts);
                    };
                    for (int k = 0; k < parts; ++k) {
                        const int32_t b0 = bound(k), b1 = bound(k + 1);
                        part(k == 0 ? s : eng->aux_stream[k - 1], b0, b1 - b0, k);
                    }
                    if (sort_any && e == hipSuccess) {
                        // on part 0's stream behind its work (the other parts may still run:
                        // their weights are then this sweep's or the last one's, either is an order)
                        hipLaunchKernelGGL(k_heavy_order, dim3(8, (uint32_t)std::min(parts, 4)), dim3(1024), 0, s, ha);
                        for (int k = 0; k < 4; ++k) eng->heavy_key[k] = k < parts ? eng->heavy_next[k] : -1;
                        eng->heavy_buf = cur ^ 1;
                    }
                    for (int k = 0; k < parts - 1 && e == hipSuccess; ++k) {
                        e = hipEventRecord(eng->ev_hp[k], eng->aux_stream[k]);
                        if (e == hipSuccess) e = hipStreamWaitEvent(s, eng->ev_hp[k], 0);
                    }
                    if (e != hipSuccess) return e;
                    if (eng->opt_sweep_stats && sort_any) {  // diagnostics: the chunks this sweep staged
                        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
                        for (int k = 0; k < parts && k < 4; ++k) {
                            if (!ha.w[k]) continue;
                            std::vector<uint32_t> wk((size_t)ha.slots[k] * 8);
                            if ((e = hipMemcpy(wk.data(), ha.w[k], wk.size() * sizeof(uint32_t), hipMemcpyDeviceToHost)) != hipSuccess)
                                return e;
                            for (uint32_t x : wk) eng->st.sweep_chunks += x;
                            const int32_t ntbs = eng->opt_sweep_waves == 8 ? (eng->V + 8 * TDT - 1) / (8 * TDT) : ntb;
                            eng->st.sweep_chunk_slots += (int64_t)(bound(k + 1) - bound(k)) * ntbs * (int64_t)nchunks;
                        }
                        unsigned long long hits = 0;
                        if ((e = hipMemcpy(&hits, eng->d_sweep_hits, sizeof hits, hipMemcpyDeviceToHost)) != hipSuccess) return e;
                        eng->st.sweep_hit_rows += (int64_t)hits;
                    }
                    return hipGetLastError();
                }
            }
            if (!w16)
            hipLaunchKernelGGL((k_relax_dense_f<TDT, XR, TB, true, 1>), dim3((uint32_t)nblocks), dim3(256), 0, s,
                               eng->d_W32p, eng->d_Wp, eng->d_WI, eng->Vp, eng->g.in_r, eng->pools, eng->V, nbg, ntb,
                               par, thresh, cnt_prev, cnt_cur, eng->d_prof, eng->d_hitlog, eng->d_perm, eng->d_minW,
                               eng->d_minD, eng->d_pos, eng->d_WIp, eng->d_WRp, eng->g.vfac, eng->opt_sweep_spiral,
                               eng->opt_sweep_win1, nullptr);
            // (4 logged rows in flight per wave instead of 2 measured the same, r03u); one batch
            // per wave whatever TB the chunk loop ran with (the f64 state of two would spill)
            const int64_t nblocks1 = 8 * (((int64_t)nbg * ntb + 7) / 8);
            hipLaunchKernelGGL((k_relax_dense_f<TDT, XR, 1, true, 2>), dim3((uint32_t)nblocks1), dim3(256), 0, s,
                               eng->d_W32p, eng->d_Wp, eng->d_WI, eng->Vp, eng->g.in_r, eng->pools, eng->V, nbg, ntb,
                               par, thresh, cnt_prev, cnt_cur, eng->d_prof, eng->d_hitlog, eng->d_perm, eng->d_minW,
                               eng->d_minD, eng->d_pos, eng->d_WIp, eng->d_WRp, eng->g.vfac, eng->opt_sweep_spiral,
                               eng->opt_sweep_win1, nullptr, nullptr, nullptr, nullptr, seeded);
            return hipGetLastError();
        }
        hipLaunchKernelGGL((k_relax_dense_f<TDT, XR, TB, true>), dim3((uint32_t)nblocks), dim3(256), 0, s,
                           eng->d_W32p, eng->d_Wp, eng->d_WI, eng->Vp, eng->g.in_r, eng->pools, eng->V, nbg, ntb, par,
                           thresh, cnt_prev, cnt_cur, eng->d_prof, eng->d_hitlog, eng->d_perm, eng->d_minW,
                           eng->d_minD, eng->d_pos, eng->d_WIp, eng->d_WRp, eng->g.vfac, eng->opt_sweep_spiral,
                               eng->opt_sweep_win1, nullptr);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((k_relax_dense_f<TDT, XR, TB, false>), dim3((uint32_t)nblocks), dim3(256), 0, s, eng->d_W32,
                       eng->d_W, eng->d_WI, eng->Vp, eng->g.in_r, eng->pools, eng->V, nbg, ntb, par, thresh, cnt_prev,
                       cnt_cur, eng->d_prof, eng->d_hitlog, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr);
    return hipGetLastError();
}

// seeded: every batch's state is k_seed_dense_t's (round 0 after the fused seed), so an exact
// pass whose seed candidate won untainted leaves the pair alone without reading it
hipError_t launch_dense_f(shadowtopo_engine* eng, int32_t nbg, int32_t par, int32_t thresh,
                          const int32_t* cnt_prev, int32_t* cnt_cur, hipStream_t s, const PartTail* tail = nullptr,
                          float* mdc_out = nullptr, bool seeded = false) {
    const int32_t sd = seeded && eng->opt_seed_skip;
    switch (eng->opt_dense_tb) {
        case 1: return launch_dense_ft<1>(eng, nbg, par, thresh, cnt_prev, cnt_cur, s, tail, mdc_out, sd);
        case 4: return launch_dense_ft<4>(eng, nbg, par, thresh, cnt_prev, cnt_cur, s, tail, mdc_out, sd);
        default: return launch_dense_ft<2>(eng, nbg, par, thresh, cnt_prev, cnt_cur, s, tail, mdc_out, sd);
    }
}

// dense delta round over the live-chunk lists (k_live_chunks): the previous round changed
// few pairs (at most 1 / opt_delta_live_div of the delta batches' pairs), or forced
bool delta_is_sparse(const shadowtopo_engine* eng, int32_t nbg, int32_t thresh) {
    if (eng->opt_delta_live != 2) return eng->opt_delta_live == 1;
    int64_t dch = 0, dpairs = 0;
    for (int32_t b = 0; b < nbg; ++b)
        if (eng->h_cnt[b] > 0 && eng->h_cnt[b] <= thresh) {
            dch += eng->h_cnt[b];
            dpairs += (int64_t)eng->V * KL;
        }
    return dch * eng->opt_delta_live_div <= dpairs;
}

// A 1-D launch of n blocks as a grid whose work-item count fits the dispatch packet's 32-bit
// fields: x up to 2^23 blocks (a multiple of 8; x 256 threads = 2^31 work-items), y the
// rest; kernels index with flat_block().  (A 1-D grid past 2^24 blocks wraps the count and
// silently drops blocks.)
dim3 grid_of(const shadowtopo_engine* eng, int64_t n) {
    const int64_t GX = eng->opt_grid_x;
    if (n <= GX) return dim3((uint32_t)std::max<int64_t>(n, 1));
    return dim3((uint32_t)GX, (uint32_t)((n + GX - 1) / GX));
}

// SHADOWTOPO_CSR_PUSH rounds (k_push / k_pred_pass / k_fold): frontier rounds over the
// activity flags (worklists when under half the pairs are active, the grid otherwise), one
// host read-back of the next round's worklist counts per round
int run_push_rounds(shadowtopo_engine* eng, int32_t nbg, hipStream_t s) {
    const GraphDev& g = eng->rg ? *eng->rg : eng->g;
    const int32_t V = g.V;
    const size_t total = (size_t)eng->pools.Vp * KL;
    const int32_t gx = (int32_t)std::min<size_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_init, dim3(gx, nbg), dim3(256), 0, s, eng->pools, eng->pools.Vp, 0);
    hipLaunchKernelGGL(k_seed_push, dim3(1, nbg), dim3(64), 0, s, g, eng->pools);
    HIP_TRY(hipGetLastError());
    const int32_t nvb = (V + 3) / 4;
    const int64_t nblocks = 8 * (((int64_t)nbg * nvb + 7) / 8);
    const int32_t ncb = (V + WL_SPAN - 1) / WL_SPAN;
    const int64_t max_rounds = eng->opt_max_rounds > 0 ? eng->opt_max_rounds : 4LL * V + 64;
    auto compact = [&](int32_t par) -> int {
        HIP_TRY(hipMemsetAsync(eng->d_wlcnt, 0, sizeof(uint32_t) * nbg, s));
        hipLaunchKernelGGL(k_compact, dim3((uint32_t)ncb, nbg), dim3(256), 0, s, eng->pools, V, par, eng->d_wl,
                           eng->d_wlcnt, g.in_ptr);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(eng->h_wlcnt, eng->d_wlcnt, sizeof(uint32_t) * nbg, hipMemcpyDeviceToHost, s));
        HIP_TRY(round_sync(eng, s));
        eng->st.host_syncs++;
        return SHADOWTOPO_OK;
    };
    int32_t* cnt = eng->d_cnt;  // written by the kernels (a batch changed), not read back
    for (int phase = 0; phase < 2; ++phase) {
        // phase 0: distance pushes from act parity 0 (the sources); phase 1: fold rounds from
        // act parity 1 (set by k_pred_pass for the sources' out-neighbours)
        if (phase == 1) {
            if (eng->opt_timing) HIP_TRY(hipEventRecord(eng->ev0, s));
            hipLaunchKernelGGL(k_pred_pass, grid_of(eng, nblocks), dim3(256), 0, s, g.in_ptr, g.in_src, g.in_w,
                               eng->pools, V, nbg, nvb);
            HIP_TRY(hipGetLastError());
            if (eng->opt_timing) {
                HIP_TRY(hipEventRecord(eng->ev1, s));
                HIP_TRY(hipEventSynchronize(eng->ev1));
                float ms = 0;
                HIP_TRY(hipEventElapsedTime(&ms, eng->ev0, eng->ev1));
                eng->st.relax_ms += ms;
                eng->st.pred_ms += ms;
            }
            eng->st.relax_launches++;
            eng->st.relax_batches += nbg;
        }
        const int32_t par0 = phase;
        int rc;
        if ((rc = compact(par0))) return rc;
        for (int64_t r = 0;; ++r) {
            if (r > max_rounds) {
                if (eng->opt_test_unconverged) return (eng->unconverged = true), SHADOWTOPO_OK;
                return fail(SHADOWTOPO_EINTERNAL, "push rounds did not converge in %lld rounds", (long long)max_rounds);
            }
            const int32_t par = (int32_t)((par0 + r) & 1);
            eng->h_wlpre[0] = 0;
            for (int32_t b = 0; b < nbg; ++b) eng->h_wlpre[b + 1] = eng->h_wlpre[b] + eng->h_wlcnt[b];
            const int64_t wl_total = eng->h_wlpre[nbg];
            if (wl_total == 0) break;
            const bool round_wl = eng->opt_worklist == 2 || (eng->opt_worklist == 1 && wl_total * 2 < (int64_t)nbg * V);
            if (round_wl)
                HIP_TRY(hipMemcpyAsync(eng->d_wlpre, eng->h_wlpre, sizeof(int64_t) * (nbg + 1), hipMemcpyHostToDevice, s));
            if (eng->opt_timing) HIP_TRY(hipEventRecord(eng->ev0, s));
            const int64_t S = (wl_total + 8 * 4 - 1) / (8 * 4) * 4;
            if (phase == 0) {
                if (round_wl)
                    hipLaunchKernelGGL(k_push_wl, grid_of(eng, 8 * (S / 4)), dim3(256), 0, s, g.in_src, g.in_w,
                                       eng->pools, par, eng->d_wl, eng->d_wlpre, nbg, S, cnt);
                else
                    hipLaunchKernelGGL(k_push, grid_of(eng, nblocks), dim3(256), 0, s, g.in_ptr, g.in_src, g.in_w,
                                       eng->pools, V, nbg, nvb, par, cnt);
            } else {
                const uint32_t k = (uint32_t)(r + 1);
                if (round_wl)
                    hipLaunchKernelGGL(k_fold_wl, grid_of(eng, 8 * (S / 4)), dim3(256), 0, s, g.in_src, g.in_r,
                                       g.out_ptr, g.out_dst, eng->pools, par, k, eng->d_wl, eng->d_wlpre, nbg, S, cnt);
                else
                    hipLaunchKernelGGL(k_fold, grid_of(eng, nblocks), dim3(256), 0, s, g.in_src, g.in_r, g.out_ptr,
                                       g.out_dst, eng->pools, V, nbg, nvb, par, k, cnt);
            }
            HIP_TRY(hipGetLastError());
            if (eng->opt_timing) HIP_TRY(hipEventRecord(eng->ev1, s));
            if ((rc = compact(par ^ 1))) return rc;
            float ms = 0;
            if (eng->opt_timing) {
                HIP_TRY(hipEventElapsedTime(&ms, eng->ev0, eng->ev1));
                eng->st.relax_ms += ms;
                if (round_wl) eng->st.wl_ms += ms;
                (phase == 0 ? eng->st.push_ms : eng->st.fold_ms) += ms;
            }
            eng->st.rounds++;
            eng->st.relax_launches++;
            eng->st.relax_batches += nbg;
            if (round_wl) eng->st.wl_launches++;
            (phase == 0 ? eng->st.push_rounds : eng->st.fold_rounds)++;
            if (eng->trace_rounds)
                fprintf(stderr, "[shadowtopo] %s round %lld batches %d items %lld%s %.3f ms\n", phase ? "fold" : "push",
                        (long long)r, nbg, (long long)wl_total, round_wl ? " (worklist)" : "", ms);
        }
    }
    return SHADOWTOPO_OK;
}

// relax rounds for the batch slots [0, nbg) until no vertex changes.  spec_compose (dense
// rounds): enqueued behind a delta round, before that round's read-back, so that the round
// that finds convergence (C2: the third) needs no second host round trip for the compose;
// *composed tells the caller whether the last enqueued compose saw the converged state (a
// compose behind a round that still changed pairs is redone, its masks and error word reset)
int run_rounds(shadowtopo_engine* eng, int32_t nbg, hipStream_t s, const std::function<int()>* spec_compose = nullptr,
               bool* composed = nullptr) {
    if (composed) *composed = false;
    const GraphDev& g = eng->rg ? *eng->rg : eng->g;
    const int32_t V = g.V;
    // incremental lean rounds (OPT_CSR_INCREMENTAL): k_init / k_seed set the change stamps the
    // relax kernels' batch views then carry
    eng->pools.inc = eng->pools.P32 && eng->pools.stamp && !eng->dense && eng->opt_csr_variant == SHADOWTOPO_CSR_FULL
                         ? eng->opt_csr_incremental
                         : 0;
    if (!eng->dense && eng->opt_csr_variant == SHADOWTOPO_CSR_PUSH && eng->d_wl) return run_push_rounds(eng, nbg, s);
    const bool fused_seed = eng->dense && eng->opt_dense_seed && eng->d_WR && eng->pools.D32 && eng->pools.BDU && eng->pools.chm;
    // dense: the first spec_rounds rounds are enqueued back to back, with no host read-back
    // between them (the full sweep, then delta rounds; C2's step is a full sweep and two delta
    // rounds, and each read-back left the GPU idle ~30 us).  A round whose decisions would
    // come from an unread count runs the delta kernel over every batch that changed at all
    // (threshold raised): exact for any set of changed pairs (the change masks hold them all),
    // a batch that would have taken another full sweep just takes a slower delta round.
    const int32_t spec_rounds = eng->dense && !eng->opt_profile ? std::min(eng->opt_dense_spec, SPEC_MAX) : 0;
    // dense change-count rows: row 0 = the virtual round -1 ("everything changed"), rows
    // 1 .. spec_rounds + 1 = rounds 0 .. spec_rounds (reset once, at the seed; read back in one
    // copy with the first read-back), then two rows alternating for the host-driven rounds
    const auto cnt_row = [&](int64_t r) {
        const int64_t i = r < 0 ? 0 : (r <= spec_rounds ? 1 + r : spec_rounds + 2 + (r & 1));
        return eng->d_cnt + i * eng->nb_cap;
    };
    if (fused_seed) {
        hipLaunchKernelGGL(k_seed_dense_t, dim3(eng->Vp / SEED_T, nbg), dim3(256), 0, s, eng->d_W, eng->d_WI, eng->Vp,
                           eng->d_WR, g.vfac, eng->pools, V, eng->d_cnt, spec_rounds + 2, eng->nb_cap);
        HIP_TRY(hipGetLastError());
    } else {
        const size_t total = (size_t)eng->pools.Vp * KL;
        int32_t gx = (int32_t)std::min<size_t>((total + 255) / 256, 4096);
        const int32_t tree = eng->dense;
        hipLaunchKernelGGL(k_init, dim3(gx, nbg), dim3(256), 0, s, eng->pools, eng->pools.Vp, tree);
        hipLaunchKernelGGL(k_seed, dim3(KL, nbg), dim3(256), 0, s, g, eng->pools);
        HIP_TRY(hipGetLastError());
    }
    const int32_t nvb = (V + 3) / 4;
    const int64_t nblocks = 8 * (((int64_t)nbg * nvb + 7) / 8);
    const int32_t ntb = (V + 4 * DT - 1) / (4 * DT);
    const int64_t nblocks_dense = 8 * (((int64_t)nbg * ntb + 7) / 8);
    if (nblocks > 0x7fffffff) return fail(SHADOWTOPO_EINVAL, "grid too large");
    const int64_t max_rounds = eng->opt_max_rounds > 0 ? eng->opt_max_rounds : 4LL * V + 64;
    eng->d_prof = eng->opt_profile ? eng->prof_buf : nullptr;
    if (eng->d_prof) HIP_TRY(hipMemsetAsync(eng->d_prof, 0, sizeof(unsigned long long) * 16 * nbg, s));
    if (eng->dense) {
        if (!fused_seed) {
            hipLaunchKernelGGL(k_seed_dense, dim3(ntb, nbg), dim3(256), 0, s, eng->d_W, eng->d_WI, eng->Vp, g.in_r,
                               eng->pools, V);
            HIP_TRY(hipGetLastError());
        }
        // round 0 consumes the change counts of a virtual round -1: every batch changed
        // everything (full sweep); k_seed_dense_t resets the rows itself
        if (!fused_seed) {
            HIP_TRY(hipMemsetAsync(cnt_row(-1), 0x7f, sizeof(int32_t) * nbg, s));
            HIP_TRY(hipMemsetAsync(cnt_row(0), 0, sizeof(int32_t) * eng->nb_cap * (spec_rounds + 1), s));
        }
        for (int32_t b = 0; b < nbg; ++b) eng->h_cnt[b] = 0x7f7f7f7f;
    }
    const int32_t nvc = eng->Vp / KL;
    const int64_t nblocks_delta = (int64_t)8 * nbg * ((nvc + 7) / 8);
    const int32_t thresh = (int32_t)std::min<int64_t>(
        0x7f7f7f7e, (int64_t)V * KL * eng->opt_delta_permille / 1000);
    std::vector<uint8_t> full_b;  // dense: batches the full sweep covers this round
    // sparse FULL rounds over compacted frontier worklists (k_compact / k_relax_wl)
    const bool use_wl = !eng->dense && eng->opt_worklist && eng->d_wl;
    const int32_t ncb = (V + WL_SPAN - 1) / WL_SPAN;
    // small graphs (C3: 110 batches x 7000 vertices): rounds driven from the device, the
    // host reading the per-round item counts once per block of DEV_K rounds instead of
    // synchronising on every round (a round of C3 is 0.1 ms of kernel and ~0.05 ms of
    // launch + read-back otherwise)
    const bool dev_rounds = use_wl && eng->opt_worklist == 1 && nbg <= 1024 &&
                            (eng->opt_device_rounds == 2 ||
                             (eng->opt_device_rounds == 1 && (int64_t)nbg * V <= eng->dev_rounds_max));
    if (dev_rounds) {
        constexpr int DEV_K = 8;
        const int64_t cap = max_rounds + DEV_K + 2;
        if (eng->tlog_n < cap) {
            if (eng->d_tlog) (void)hipFree(eng->d_tlog);
            if (eng->h_tlog) (void)hipHostFree(eng->h_tlog);
            eng->d_tlog = nullptr;
            eng->h_tlog = nullptr;
            eng->tlog_n = 0;
            HIP_TRY(hipMalloc((void**)&eng->d_tlog, sizeof(int64_t) * cap));
            HIP_TRY(hipHostMalloc((void**)&eng->h_tlog, sizeof(int64_t) * cap, hipHostMallocDefault));
            eng->tlog_n = cap;
        }
        if (eng->opt_timing && eng->ev_dev.empty()) {
            eng->ev_dev.resize(2 * DEV_K);
            for (auto& e : eng->ev_dev) HIP_TRY(hipEventCreate(&e));
        }
        // fixed grid: 2048 blocks (8192 waves).  Sized from the occupancy query instead (7
        // blocks per CU: the kernel's 106 SGPRs) it ran C3 7.29 -> 7.78 ms (r04n): the strided
        // item loop balances better over more, partly queued, blocks
        const uint32_t G = 8 * 256;
        HIP_TRY(hipMemsetAsync(eng->d_wlcnt, 0, sizeof(uint32_t) * nbg, s));
        hipLaunchKernelGGL(k_compact, dim3((uint32_t)ncb, nbg), dim3(256), 0, s, eng->pools, V, 0, eng->d_wl,
                           eng->d_wlcnt, g.in_ptr);
        hipLaunchKernelGGL(k_scan_wl, dim3(1), dim3(256), 0, s, eng->d_wlcnt, nbg, eng->d_wlpre, eng->d_tlog, 0);
        HIP_TRY(hipGetLastError());
        for (int64_t r0 = 0;; r0 += DEV_K) {
            if (r0 > max_rounds) {
                if (eng->opt_test_unconverged) return (eng->unconverged = true), SHADOWTOPO_OK;
                return fail(SHADOWTOPO_EINTERNAL, "relaxation did not converge in %lld rounds", (long long)max_rounds);
            }
            for (int64_t round = r0; round < r0 + DEV_K; ++round) {
                int32_t* cnt_cur = eng->d_cnt + (round & 1) * eng->nb_cap;  // written, not read back
                if (eng->opt_timing) HIP_TRY(hipEventRecord(eng->ev_dev[2 * (round - r0)], s));
                if (eng->pools.inc)
                    hipLaunchKernelGGL(k_relax_wlp<true>, dim3(G), dim3(256), 0, s, g.in_ptr, g.in_src, g.in_w, g.in_r,
                                       g.out_ptr, g.out_dst, eng->pools, (int32_t)round, eng->d_wl, eng->d_wlpre, nbg,
                                       cnt_cur, eng->d_prof, V);
                else
                    hipLaunchKernelGGL(k_relax_wlp<false>, dim3(G), dim3(256), 0, s, g.in_ptr, g.in_src, g.in_w, g.in_r,
                                       g.out_ptr, g.out_dst, eng->pools, (int32_t)round, eng->d_wl, eng->d_wlpre, nbg,
                                       cnt_cur, eng->d_prof, V);
                if (eng->opt_timing) HIP_TRY(hipEventRecord(eng->ev_dev[2 * (round - r0) + 1], s));
                hipLaunchKernelGGL(k_compact, dim3((uint32_t)ncb, nbg), dim3(256), 0, s, eng->pools, V,
                                   (int32_t)((round + 1) & 1), eng->d_wl, eng->d_wlcnt, g.in_ptr);
                hipLaunchKernelGGL(k_scan_wl, dim3(1), dim3(256), 0, s, eng->d_wlcnt, nbg, eng->d_wlpre, eng->d_tlog,
                                   (int32_t)(round + 1));
                HIP_TRY(hipGetLastError());
            }
            HIP_TRY(hipMemcpyAsync(eng->h_tlog + r0, eng->d_tlog + r0, sizeof(int64_t) * (DEV_K + 1),
                                   hipMemcpyDeviceToHost, s));
            HIP_TRY(round_sync(eng, s));
            eng->st.host_syncs++;
            bool done = false;
            for (int64_t round = r0; round < r0 + DEV_K; ++round) {
                const int64_t T = eng->h_tlog[round];
                if (T == 0) {  // nothing active: converged (the rest of the block were no-ops)
                    done = true;
                    break;
                }
                eng->st.rounds++;
                eng->st.relax_launches++;
                eng->st.wl_launches++;
                eng->st.relax_batches += nbg;
                float ms = 0;
                if (eng->opt_timing) {
                    HIP_TRY(hipEventElapsedTime(&ms, eng->ev_dev[2 * (round - r0)], eng->ev_dev[2 * (round - r0) + 1]));
                    eng->st.relax_ms += ms;
                    eng->st.wl_ms += ms;
                }
                if (eng->trace_rounds)
                    fprintf(stderr, "[shadowtopo] round %lld batches %d items %lld (device-driven) %.3f ms\n",
                            (long long)round, nbg, (long long)T, ms);
            }
            if (done) break;
        }
    } else {
    if (use_wl) {
        HIP_TRY(hipMemsetAsync(eng->d_wlcnt, 0, sizeof(uint32_t) * nbg, s));
        hipLaunchKernelGGL(k_compact, dim3((uint32_t)ncb, nbg), dim3(256), 0, s, eng->pools, V, 0, eng->d_wl,
                           eng->d_wlcnt, g.in_ptr);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(eng->h_wlcnt, eng->d_wlcnt, sizeof(uint32_t) * nbg, hipMemcpyDeviceToHost, s));
        HIP_TRY(round_sync(eng, s));
        eng->st.host_syncs++;
    }
    if (spec_rounds && eng->opt_timing && eng->ev_spec.empty()) {
        eng->ev_spec.resize(2 * (SPEC_MAX + 1));
        for (auto& e : eng->ev_spec) HIP_TRY(hipEventCreate(&e));
    }
    std::vector<uint8_t> spec_fb[SPEC_MAX];  // those rounds' full-sweep batches
    // f32 dense delta rounds: pruned (chunk bounds, locality order), sparse (live-chunk lists)
    // or plain; `delta_bufs` allocates the kind's scratch for all nbg batches, `enq_delta`
    // enqueues one round over batches [b0, b0 + n) on stream st (pools, cnt rows, minDc,
    // cmask and live lists offset to the part)
    enum { DK_PLAIN, DK_PRUNED, DK_SPARSE };
    const auto delta_kind = [&](bool dsparse) {
        if (eng->vperm_ready && eng->opt_dense_prune && nvc <= PR_CHUNKS && !dsparse) return (int)DK_PRUNED;
        return dsparse ? (int)DK_SPARSE : (int)DK_PLAIN;
    };
    const auto delta_bufs = [&](int kind) -> int {
        // fp16 slabs when their table can be had; without it (HBM taken) the f32 slabs serve
        if (kind == DK_PRUNED && eng->opt_delta_w16 && ensure_w16p(eng, s) != hipSuccess) (void)hipGetLastError();
        if (kind == DK_PRUNED) {
            const size_t need = (size_t)eng->nb_cap * nvc * KL;
            if (eng->minDc_n < need) {
                if (eng->d_minDc) (void)hipFree(eng->d_minDc);
                eng->d_minDc = nullptr;
                eng->minDc_n = 0;
                HIP_TRY(hipMalloc((void**)&eng->d_minDc, need * sizeof(float)));
                eng->minDc_n = need;
            }
            const size_t need_cm = (size_t)nblocks_delta * PR_CHUNKS;
            if (eng->opt_delta_colbound >= 2 && eng->cmask_n < need_cm) {
                if (eng->d_cmask) (void)hipFree(eng->d_cmask);
                eng->d_cmask = nullptr;
                eng->cmask_n = 0;
                HIP_TRY(hipMalloc((void**)&eng->d_cmask, need_cm * sizeof(unsigned long long)));
                eng->cmask_n = need_cm;
            }
        } else if (kind == DK_SPARSE && !eng->d_live) {
            int rc2;
            if ((rc2 = dev_alloc(eng->batch_allocs, (void**)&eng->d_live, sizeof(int32_t) * (size_t)eng->nb_cap * nvc)) ||
                (rc2 = dev_alloc(eng->batch_allocs, (void**)&eng->d_nlive, sizeof(int32_t) * eng->nb_cap)))
                return rc2;
        }
        return SHADOWTOPO_OK;
    };
    const auto enq_delta = [&](hipStream_t st, int32_t b0, int32_t n, int kind, int32_t par, int32_t thr,
                               const int32_t* cprev, int32_t* ccur, bool mindc_ready = false) {
        const Pools P = pools_from(eng->pools, b0);
        const int64_t c8 = (nvc + 7) / 8;
        const uint32_t nbl = (uint32_t)(8 * n * c8);
        cprev += b0;
        ccur += b0;
        if (kind == DK_PRUNED) {
            // pruned: rows and tiles in the locality order, each block walking only the chunks
            // whose changed pairs can pass (k_min_d32c bounds, minW64); a round after one that
            // changed few pairs takes the live-chunk lists instead (C2: 0.95 ms pruned vs 1.05
            // unpruned after the sweep; 0.03 vs 0.08 ms for the last round's single change).
            // cmask is per block: a part's blocks take their own region of it
            float* mdc = eng->d_minDc + (size_t)b0 * nvc * KL;
            unsigned long long* cm =
                eng->opt_delta_colbound >= 2 ? eng->d_cmask + (size_t)8 * b0 * c8 * PR_CHUNKS : nullptr;
            if (!mindc_ready)
                hipLaunchKernelGGL(k_min_d32c, dim3((uint32_t)nvc, n), dim3(256), 0, st, P, eng->d_perm, V, nvc, par,
                                   cprev, thr, mdc);
            if (eng->opt_delta_w16 && eng->d_W16p)
                hipLaunchKernelGGL((k_relax_dense_delta_s<true, true>), dim3(nbl), dim3(64 * DW), 0, st,
                                   (const float*)eng->d_W16p, eng->d_W, eng->d_WI, eng->Vp, g.in_src, g.in_r, P, V, n,
                                   nvc, par, thr, cprev, ccur, nullptr, nullptr, eng->d_perm, eng->d_minW64, mdc,
                                   eng->opt_delta_colbound ? eng->d_minW : nullptr, cm);
            else
                hipLaunchKernelGGL((k_relax_dense_delta_s<true, false>), dim3(nbl), dim3(64 * DW), 0, st, eng->d_W32p,
                                   eng->d_W, eng->d_WI, eng->Vp, g.in_src, g.in_r, P, V, n, nvc, par, thr, cprev, ccur,
                                   nullptr, nullptr, eng->d_perm, eng->d_minW64, mdc,
                                   eng->opt_delta_colbound ? eng->d_minW : nullptr, cm);
            return;
        }
        // a round after one that changed few pairs walks only the chunks holding a changed
        // row (k_live_chunks); after a full sweep nearly every chunk does
        int32_t* live = nullptr;
        int32_t* nlive = nullptr;
        if (kind == DK_SPARSE) {
            live = eng->d_live + (size_t)b0 * nvc;
            nlive = eng->d_nlive + b0;
            hipLaunchKernelGGL(k_live_chunks, dim3(n), dim3(256), 0, st, P, V, nvc, par, cprev, live, nlive);
        }
        hipLaunchKernelGGL(k_relax_dense_delta_s<false>, dim3(nbl), dim3(64 * DW), 0, st, eng->d_W32, eng->d_W,
                           eng->d_WI, eng->Vp, g.in_src, g.in_r, P, V, n, nvc, par, thr, cprev, ccur, live, nlive,
                           nullptr, nullptr, nullptr, nullptr, nullptr);
    };
    // chained: the blind rounds 1 .. spec_rounds go on each sweep part's stream right behind
    // its share of the sweep (results are per batch, so a part's delta rounds need nothing
    // from the other parts) and the parts join once, before the read-back
    const int32_t nparts = eng->dense ? sweep_parts(eng, nbg) : 1;
    const bool chain = eng->opt_chain_parts && spec_rounds > 0 && thresh != 0 && nparts >= 2 && !eng->d_prof;
    int chain_kind[SPEC_MAX + 1] = {};
    for (int32_t r = 1; chain && r <= spec_rounds; ++r) {
        chain_kind[r] = delta_kind(eng->opt_delta_live != 2 ? eng->opt_delta_live == 1 : r >= 2);
        if (int rc2 = delta_bufs(chain_kind[r])) return rc2;
    }
    // a pruned round 1 takes its chunk bounds from the sweep's exact passes (k_min_d32c's
    // values, folded in by their epilogues: the pass over the change masks after the sweep
    // waited ~0.12 ms for CUs behind the other part's kernels, r04zx)
    const bool fuse_mindc = chain && eng->opt_fuse_mindc && chain_kind[1] == DK_PRUNED;
    if (chain && eng->opt_timing)
        for (int k = 0; k < nparts; ++k)
            if (!eng->ev_sw[k]) HIP_TRY(hipEventCreate(&eng->ev_sw[k]));
    const PartTail chain_tail = [&](hipStream_t st, int32_t b0, int32_t n, int k) -> hipError_t {
        if (eng->opt_timing) {
            hipError_t e = hipEventRecord(eng->ev_sw[k], st);
            if (e != hipSuccess) return e;
        }
        for (int32_t r = 1; r <= spec_rounds; ++r)
            enq_delta(st, b0, n, chain_kind[r], (int32_t)(r & 1), 0x7f7f7f7e, cnt_row(r - 1), cnt_row(r),
                      r == 1 && fuse_mindc);
        return hipGetLastError();
    };
    for (int64_t round = 0;; ++round) {
        if (round > max_rounds) {
            if (eng->opt_test_unconverged) return (eng->unconverged = true), SHADOWTOPO_OK;
            return fail(SHADOWTOPO_EINTERNAL, "relaxation did not converge in %lld rounds", (long long)max_rounds);
        }
        const bool spec = round < spec_rounds;                   // no read-back after this round
        const bool blind = round >= 1 && round <= spec_rounds;  // decided without the last counts
        // chained rounds 1 .. spec_rounds: enqueued with round 0 (the decisions below are the
        // same blind ones, kept for the counts)
        const bool chained = chain && round >= 1 && round <= spec_rounds;
        hipEvent_t e0 = eng->ev0, e1 = eng->ev1;
        if (round <= spec_rounds && !eng->ev_spec.empty()) {
            e0 = eng->ev_spec[2 * round];
            e1 = eng->ev_spec[2 * round + 1];
        }
        int64_t wl_total = 0;
        if (use_wl) {
            eng->h_wlpre[0] = 0;
            for (int32_t b = 0; b < nbg; ++b) eng->h_wlpre[b + 1] = eng->h_wlpre[b] + eng->h_wlcnt[b];
            wl_total = eng->h_wlpre[nbg];
            if (wl_total == 0) break;  // nothing active: converged
        }
        // worklist only where it pays: a mostly-active round runs the plain grid
        const bool round_wl = use_wl && (eng->opt_worklist == 2 || wl_total * 2 < (int64_t)nbg * V);
        if (round_wl)
            HIP_TRY(hipMemcpyAsync(eng->d_wlpre, eng->h_wlpre, sizeof(int64_t) * (nbg + 1), hipMemcpyHostToDevice, s));
        int32_t* cnt_cur = eng->dense ? cnt_row(round) : eng->d_cnt + (round & 1) * eng->nb_cap;
        int32_t* cnt_prev = eng->dense ? cnt_row(round - 1) : eng->d_cnt + ((round + 1) & 1) * eng->nb_cap;
        if (!eng->dense || round > spec_rounds) HIP_TRY(hipMemsetAsync(cnt_cur, 0, sizeof(int32_t) * nbg, s));
        if (eng->opt_timing && !chained) HIP_TRY(hipEventRecord(e0, s));
        bool round_full = false, round_delta = false;
        if (eng->dense) {
            // per batch: full sweep when its previous round changed more than `thresh` pairs,
            // delta round otherwise (each kernel skips the other's batches)
            bool& any_full = round_full;
            bool& any_delta = round_delta;
            any_full = any_delta = false;
            full_b.assign((size_t)nbg, 0);
            int32_t thr = thresh;  // delta rounds: batches that changed 1 .. thr pairs
            if (blind && thresh == 0) {  // full sweeps only (OPT_DELTA_PERMILLE 0): every batch that changed
                any_full = true;
                full_b.assign((size_t)nbg, 1);
            } else if (blind) {
                any_delta = true;
                thr = 0x7f7f7f7e;
            } else {
                for (int32_t b = 0; b < nbg; ++b) {
                    full_b[b] = eng->h_cnt[b] > thresh;
                    any_full |= full_b[b] != 0;
                    any_delta |= eng->h_cnt[b] > 0 && eng->h_cnt[b] <= thresh;
                }
            }
            // live-chunk (sparse) delta rounds after a round that changed few pairs; blind: the
            // round right after the full sweep is pruned, later ones sparse (C2's pattern)
            const bool dsparse = !blind ? delta_is_sparse(eng, nbg, thr)
                                        : (eng->opt_delta_live != 2 ? eng->opt_delta_live == 1 : round >= 2);
            const int32_t par = (int32_t)(round & 1);
            if (any_full && any_delta && eng->opt_timing) HIP_TRY(hipEventRecord(eng->evm, s));
            if (any_full) {
                if (eng->opt_dense_variant == SHADOWTOPO_DENSE_F64)
                    hipLaunchKernelGGL(k_relax_dense, dim3((uint32_t)nblocks_dense), dim3(256), 0, s, eng->d_W,
                                       eng->d_WI, eng->Vp, g.in_r, eng->pools, V, nbg, ntb, par, thresh, cnt_prev,
                                       cnt_cur);
                else if (chain && round == 0) {
                    if (std::find(full_b.begin(), full_b.end(), 0) != full_b.end() || any_delta)
                        return fail(SHADOWTOPO_EINTERNAL, "chained rounds: round 0 is not a full sweep of every batch");
                    HIP_TRY(launch_dense_f(eng, nbg, par, thresh, cnt_prev, cnt_cur, s, &chain_tail,
                                           fuse_mindc ? eng->d_minDc : nullptr, fused_seed));
                } else
                    HIP_TRY(launch_dense_f(eng, nbg, par, thresh, cnt_prev, cnt_cur, s, nullptr, nullptr,
                                           fused_seed && round == 0));
                eng->st.full_sweeps++;
                for (int32_t b = 0; b < nbg; ++b) eng->st.full_batches += full_b[b];
            }
            if (any_full && any_delta && eng->opt_timing) HIP_TRY(hipEventRecord(eng->evm2, s));
            if (any_delta) {
                if (eng->opt_dense_variant == SHADOWTOPO_DENSE_F64)
                    hipLaunchKernelGGL(k_relax_dense_delta, dim3((uint32_t)nblocks_delta), dim3(64 * DW), 0, s,
                                       eng->d_W, eng->d_WI, eng->Vp, g.in_src, g.in_r, eng->pools, V, nbg, nvc, par,
                                       thr, cnt_prev, cnt_cur);
                else {
                    const int kind = delta_kind(dsparse);
                    if (!chained) {
                        if (int rc2 = delta_bufs(kind)) return rc2;
                        enq_delta(s, 0, nbg, kind, par, thr, cnt_prev, cnt_cur);
                    }
                    eng->st.pruned_deltas += kind == DK_PRUNED;
                    eng->st.sparse_deltas += kind == DK_SPARSE;
                }
                eng->st.delta_sweeps++;
            }
        } else if (round_wl) {
            eng->st.relax_batches += nbg;
            eng->st.wl_launches++;
            const int64_t S = (wl_total + 8 * 4 - 1) / (8 * 4) * 4;  // items per XCD slice, whole blocks
            if (eng->pools.inc)
                hipLaunchKernelGGL(k_relax_wl<true>, grid_of(eng, 8 * (S / 4)), dim3(256), 0, s, g.in_ptr, g.in_src,
                                   g.in_w, g.in_r, g.out_ptr, g.out_dst, eng->pools, (int32_t)round, eng->d_wl,
                                   eng->d_wlpre, nbg, S, cnt_cur, eng->d_prof);
            else
                hipLaunchKernelGGL(k_relax_wl<false>, grid_of(eng, 8 * (S / 4)), dim3(256), 0, s, g.in_ptr, g.in_src,
                                   g.in_w, g.in_r, g.out_ptr, g.out_dst, eng->pools, (int32_t)round, eng->d_wl,
                                   eng->d_wlpre, nbg, S, cnt_cur, eng->d_prof);
        } else {
            eng->st.relax_batches += nbg;
            if (eng->pools.inc)
                hipLaunchKernelGGL(k_relax<true>, grid_of(eng, nblocks), dim3(256), 0, s, g.in_ptr, g.in_src, g.in_w,
                                   g.in_r, g.out_ptr, g.out_dst, eng->pools, V, nbg, nvb, (int32_t)round, cnt_cur,
                                   eng->d_prof);
            else
                hipLaunchKernelGGL(k_relax<false>, grid_of(eng, nblocks), dim3(256), 0, s, g.in_ptr, g.in_src, g.in_w,
                                   g.in_r, g.out_ptr, g.out_dst, eng->pools, V, nbg, nvb, (int32_t)round, cnt_cur,
                                   eng->d_prof);
        }
        HIP_TRY(hipGetLastError());
        if (eng->opt_timing && !chained) HIP_TRY(hipEventRecord(e1, s));
        if (spec) {
            // no read-back: this round's counts come back with the next one (h_cnt_spec)
            spec_fb[round] = full_b;
            eng->st.relax_launches++;
            eng->st.rounds++;
            continue;
        }
        if (use_wl) {  // the next round's worklists, from the flags this round set
            HIP_TRY(hipMemsetAsync(eng->d_wlcnt, 0, sizeof(uint32_t) * nbg, s));
            hipLaunchKernelGGL(k_compact, dim3((uint32_t)ncb, nbg), dim3(256), 0, s, eng->pools, V,
                               (int32_t)((round + 1) & 1), eng->d_wl, eng->d_wlcnt, g.in_ptr);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipMemcpyAsync(eng->h_wlcnt, eng->d_wlcnt, sizeof(uint32_t) * nbg, hipMemcpyDeviceToHost, s));
        }
        // a dense delta round is usually the last: the compose goes behind it, read back with it
        const bool spec_c = spec_compose && eng->dense && !round_full && round >= 1;
        if (spec_c) {
            if (int rc2 = (*spec_compose)()) return rc2;
        }
        if (eng->dense && round == spec_rounds && spec_rounds > 0) {
            // the counts of every round since the seed, rows 1 .. spec_rounds + 1, in one copy
            HIP_TRY(hipMemcpyAsync(eng->h_cnt_spec, cnt_row(0), sizeof(int32_t) * eng->nb_cap * (spec_rounds + 1),
                                   hipMemcpyDeviceToHost, s));
        } else {
            HIP_TRY(hipMemcpyAsync(eng->h_cnt, cnt_cur, sizeof(int32_t) * nbg, hipMemcpyDeviceToHost, s));
        }
        HIP_TRY(round_sync(eng, s));
        eng->st.host_syncs++;
        if (eng->dense && round == spec_rounds && spec_rounds > 0)
            std::copy(eng->h_cnt_spec + (size_t)spec_rounds * eng->nb_cap,
                      eng->h_cnt_spec + (size_t)spec_rounds * eng->nb_cap + nbg, eng->h_cnt);
        eng->st.relax_launches++;
        eng->st.rounds++;
        if (round == spec_rounds) {
            // the rounds enqueued without a read-back: their counts and times
            for (int32_t r = 0; r < spec_rounds; ++r) {
                const int32_t* hc = eng->h_cnt_spec + (size_t)r * eng->nb_cap;
                const bool full = std::find(spec_fb[r].begin(), spec_fb[r].end(), 1) != spec_fb[r].end();
                int64_t ch = 0;
                for (int32_t b = 0; b < nbg; ++b) {
                    ch += hc[b];
                    if (!spec_fb[r].empty() && spec_fb[r][b]) eng->st.full_changes += hc[b];
                }
                float ms = 0;
                if (eng->opt_timing && chain) {
                    // round 0's events span every chained round (recorded before the fork and
                    // after the join); the sweep ends when its last part's share does
                    if (r == 0) {
                        float all = 0, sw = 0;
                        HIP_TRY(hipEventElapsedTime(&all, eng->ev_spec[0], eng->ev_spec[1]));
                        for (int k = 0; k < nparts; ++k) {
                            float t = 0;
                            HIP_TRY(hipEventElapsedTime(&t, eng->ev_spec[0], eng->ev_sw[k]));
                            sw = std::max(sw, t);
                        }
                        eng->st.relax_ms += all;
                        eng->st.full_ms += sw;
                        eng->st.delta_ms += all - sw;
                        ms = all;
                    }
                } else if (eng->opt_timing) {
                    HIP_TRY(hipEventElapsedTime(&ms, eng->ev_spec[2 * r], eng->ev_spec[2 * r + 1]));
                    eng->st.relax_ms += ms;
                    (full ? eng->st.full_ms : eng->st.delta_ms) += ms;
                }
                if (eng->trace_rounds)
                    fprintf(stderr, "[shadowtopo] round %d batches %d items %lld %s (no read-back) changed %lld %.3f ms\n",
                            r, nbg, (long long)nbg * V, full ? "full" : "delta", (long long)ch, ms);
            }
        }
        if (eng->opt_timing && !(chain && round == spec_rounds)) {  // chained: timed with round 0
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
            eng->st.relax_ms += ms;
            if (round_wl) eng->st.wl_ms += ms;
            if (eng->dense) {
                if (round_full && round_delta) {
                    float a = 0, b = 0;
                    HIP_TRY(hipEventElapsedTime(&a, eng->evm, eng->evm2));
                    HIP_TRY(hipEventElapsedTime(&b, eng->evm2, eng->ev1));
                    eng->st.full_ms += a;
                    eng->st.delta_ms += b;
                } else if (round_full) {
                    eng->st.full_ms += ms;
                } else if (round_delta) {
                    eng->st.delta_ms += ms;
                }
            }
        }
        int64_t changed = 0;
        for (int32_t b = 0; b < nbg; ++b) {
            changed += eng->h_cnt[b];
            if (round_full && full_b[b]) eng->st.full_changes += eng->h_cnt[b];
        }
        if (eng->trace_rounds) {
            float ms = 0;
            if (eng->opt_timing && !chained) (void)hipEventElapsedTime(&ms, e0, e1);
            fprintf(stderr, "[shadowtopo] round %lld batches %d items %lld%s%s%s changed %lld %.3f ms\n",
                    (long long)round, nbg, (long long)(round_wl ? wl_total : (int64_t)nbg * V),
                    round_wl ? " (worklist)" : "", round_full ? " full" : "", round_delta ? " delta" : "",
                    (long long)changed, ms);
        }
        if (eng->dense && eng->opt_profile) eng->st.changes += changed;  // changed (vertex, source) pairs
        if (changed == 0) {
            if (spec_c && composed) *composed = true;
            break;
        }
        if (spec_c) eng->st.spec_composes_lost++;
    }
    }  // host-driven rounds
    if (eng->d_prof) {
        std::vector<unsigned long long> h((size_t)16 * nbg);
        HIP_TRY(hipMemcpy(h.data(), eng->d_prof, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < h.size(); i += 2) {
            eng->st.visits += (int64_t)h[i];
            eng->st.changes += (int64_t)h[i + 1];
        }
    }
    return SHADOWTOPO_OK;
}

// landmark distances to a set of vertices: out[r][i] = dist[rows[r]][cols[i]] (rows of V)
__global__ __launch_bounds__(256) void k_gather_dist(const double* __restrict__ dist, size_t V,
                                                     const int32_t* __restrict__ rows,
                                                     const int32_t* __restrict__ cols, int32_t nc,
                                                     double* __restrict__ out) {
    const int32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nc) return;
    out[(size_t)blockIdx.y * nc + i] = dist[(size_t)rows[blockIdx.y] * V + cols[i]];
}

// Source order for the label-correcting (CSR) rounds.  A batch's wave is active at a vertex
// when ANY of its 64 sources has a changed in-neighbour there, so 64 scattered sources make
// every vertex busy in almost every round (C3: 24 visits per vertex and batch).  Sources
// that are near each other improve the same vertices in the same rounds.  The key: distances
// from eight attached landmarks (farthest-point: attached[0], then the attached vertex
// farthest from the landmarks so far), projected on their top two principal axes and
// ordered along a Hilbert curve (locality_keys), computed once per attached set with the
// engine's own rounds (C3: 13.6 ms with three landmarks in Morton order, 12.3 ms so).
// Results do not depend on it: every lane converges to its own source's fixed point.
// Morton keys of `cand` (the attached list, or every vertex for the pruned dense sweep's
// vertex order) from NL farthest-point landmarks chosen among `cand`.  embed2: instead of
// interleaving the NL distances, project the centred distance vectors on their top two
// principal axes (landmark MDS) and take the Hilbert index of those two coordinates: for
// geographic graphs that recovers a near-planar layout, whose 32-vertex chunks are far more
// compact.
int locality_keys(shadowtopo_engine* eng, hipStream_t s, const std::vector<int32_t>& cand,
                  std::vector<uint64_t>& key, int NL = 3, bool embed2 = false) {
    constexpr double HINF = std::numeric_limits<double>::infinity();
    // on the relaxation view the next rounds use (a renumbered pendant-pruned view maps the
    // candidates' vertex ids to its own)
    const GraphDev& gx = eng->rg ? *eng->rg : eng->g;
    const bool vw = eng->rg == &eng->gp && !eng->h_view_of.empty();
    auto vid = [&](int32_t v) { return vw ? eng->h_view_of[(size_t)v] : v; };
    const int32_t A = (int32_t)cand.size(), V = gx.V;
    key.assign((size_t)A, 0);
    int rc;
    if ((rc = ensure_batches(eng, std::max(1, eng->nb_cap)))) return rc;
    const shadowtopo_stats keep = eng->st;
    // dl[k][i]: the distance from landmark k to cand[i]
    std::vector<std::vector<double>> dl;
    // One batch of up to 64 sampled candidates (cand[0] first, then every (A/64)-th), and
    // farthest-point selection of the NL landmarks among them: each next landmark is the
    // sample farthest (finite) from those chosen so far.  One SSSP batch instead of NL
    // single-source runs one after another (C2 order 15.5 -> ~4 ms); any landmarks give a
    // valid order, spread ones a local one.  Two gathers leave the device: the samples'
    // distances among themselves (the selection), then the chosen landmarks' distances to the
    // candidates -- not NL whole rows of V distances (C5: 8 x 5 MB, 50 ms of the attach).
    const int32_t S = std::min<int32_t>(KL, A);
    std::vector<int32_t> samp((size_t)S), cols((size_t)std::max(A, S));
    for (int32_t i = 0; i < S; ++i) samp[i] = cand[(size_t)((int64_t)i * A / S)];
    double* d_dist = nullptr;
    double* d_out = nullptr;
    int32_t *d_rows = nullptr, *d_cols = nullptr;
    // allocation failures fall through to the common free + stats restore below (r06 advisor)
    if (hipMalloc((void**)&d_dist, sizeof(double) * (size_t)V * S) != hipSuccess ||
        hipMalloc((void**)&d_out, sizeof(double) * (size_t)std::max(A, S) * std::max(S, NL)) != hipSuccess ||
        hipMalloc((void**)&d_rows, sizeof(int32_t) * (size_t)KL) != hipSuccess ||
        hipMalloc((void**)&d_cols, sizeof(int32_t) * (size_t)std::max(A, S)) != hipSuccess)
        rc = fail(SHADOWTOPO_ENOMEM, "landmark buffers");
    for (int j = 0; j < KL; ++j) {
        eng->h_srcv[j] = j < S ? vid(samp[j]) : -1;
        eng->h_row[j] = -1;
    }
    if (rc == 0 && hipMemcpyAsync(eng->pools.srcv, eng->h_srcv.data(), sizeof(int32_t) * KL, hipMemcpyHostToDevice, s) !=
        hipSuccess)
        rc = fail(SHADOWTOPO_EDEVICE, "memcpy");
    if (rc == 0) rc = run_rounds(eng, 1, s);
    if (rc == 0) {
        hipLaunchKernelGGL(k_extract, dim3((V + 255) / 256, S), dim3(256), 0, s, gx, eng->pools, S, d_dist,
                           nullptr, nullptr, nullptr);
        if (hipGetLastError() != hipSuccess) rc = fail(SHADOWTOPO_EDEVICE, "landmark distances");
    }
    // out[r][i] = dist[rows[r]][cols[i]]
    std::vector<double> G;
    const auto gather = [&](const std::vector<int32_t>& rows, int32_t nc, std::vector<double>& out) -> int {
        const int32_t nr = (int32_t)rows.size();
        out.resize((size_t)nr * nc);
        if (hipMemcpyAsync(d_rows, rows.data(), sizeof(int32_t) * nr, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(d_cols, cols.data(), sizeof(int32_t) * nc, hipMemcpyHostToDevice, s) != hipSuccess)
            return fail(SHADOWTOPO_EDEVICE, "landmark gather");
        hipLaunchKernelGGL(k_gather_dist, dim3((uint32_t)((nc + 255) / 256), (uint32_t)nr), dim3(256), 0, s, d_dist,
                           (size_t)V, d_rows, d_cols, nc, d_out);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(out.data(), d_out, sizeof(double) * out.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
            round_sync(eng, s) != hipSuccess)
            return fail(SHADOWTOPO_EDEVICE, "landmark gather");
        return SHADOWTOPO_OK;
    };
    if (rc == 0) {
        std::vector<int32_t> all((size_t)S);
        for (int32_t j = 0; j < S; ++j) all[j] = j, cols[j] = vid(samp[j]);
        rc = gather(all, S, G);  // G[j][i]: sample j to sample i
    }
    std::vector<int32_t> land;
    {
        std::vector<double> mind((size_t)S, HINF);  // each sample's distance from the landmarks so far
        std::vector<char> taken((size_t)S, 0);
        for (int32_t li = 0, k = 0; k < NL && li >= 0 && rc == 0; ++k) {
            land.push_back(li);
            taken[li] = 1;
            double best = -1.0;
            const int32_t cur = li;
            li = -1;
            for (int32_t i = 0; i < S; ++i) {
                mind[i] = std::min(mind[i], G[(size_t)cur * S + i]);
                if (!taken[i] && mind[i] < HINF && mind[i] > best) best = mind[i], li = i;
            }
        }
    }
    if (rc == 0) {
        for (int32_t i = 0; i < A; ++i) cols[i] = vid(cand[i]);
        std::vector<double> H;
        rc = gather(land, A, H);  // H[k][i]: landmark k to cand[i]
        for (size_t k = 0; k < land.size() && rc == 0; ++k)
            dl.emplace_back(H.begin() + (ptrdiff_t)(k * A), H.begin() + (ptrdiff_t)((k + 1) * A));
    }
    (void)hipFree(d_dist);
    (void)hipFree(d_out);
    (void)hipFree(d_rows);
    (void)hipFree(d_cols);
    eng->st = keep;
    if (rc) return rc;
    if (embed2 && dl.size() >= 3) {
        const int L = (int)dl.size();
        std::vector<double> mean((size_t)L, 0.0), X((size_t)A * L);
        for (int k = 0; k < L; ++k) {
            double sum = 0.0;
            int64_t n = 0;
            for (int32_t i = 0; i < A; ++i)
                if (dl[k][i] < HINF) sum += dl[k][i], ++n;
            const double m = n ? sum / (double)n : 0.0;
            for (int32_t i = 0; i < A; ++i) {
                const double d = dl[k][i];
                X[(size_t)i * L + k] = (d < HINF ? d : m) - m;
            }
        }
        std::vector<double> C((size_t)L * L, 0.0);
        for (int32_t i = 0; i < A; ++i)
            for (int a = 0; a < L; ++a)
                for (int b = 0; b < L; ++b) C[a * L + b] += X[(size_t)i * L + a] * X[(size_t)i * L + b];
        std::vector<double> axes[2];
        for (int e = 0; e < 2; ++e) {  // power iteration with deflation
            std::vector<double> v((size_t)L), w((size_t)L);
            for (int a = 0; a < L; ++a) v[a] = 1.0 + 0.1 * a;
            double lam = 0.0;
            for (int it = 0; it < 500; ++it) {
                double nrm = 0.0;
                for (int a = 0; a < L; ++a) {
                    w[a] = 0.0;
                    for (int b = 0; b < L; ++b) w[a] += C[a * L + b] * v[b];
                    nrm += w[a] * w[a];
                }
                nrm = std::sqrt(nrm);
                if (!(nrm > 0.0)) break;
                lam = nrm;
                for (int a = 0; a < L; ++a) v[a] = w[a] / nrm;
            }
            axes[e] = v;
            for (int a = 0; a < L; ++a)
                for (int b = 0; b < L; ++b) C[a * L + b] -= lam * v[a] * v[b];
        }
        std::vector<double> y[2];
        for (int e = 0; e < 2; ++e) {
            y[e].resize((size_t)A);
            double lo = HINF, hi = -HINF;
            for (int32_t i = 0; i < A; ++i) {
                double t = 0.0;
                for (int a = 0; a < L; ++a) t += X[(size_t)i * L + a] * axes[e][a];
                y[e][i] = t;
                lo = std::min(lo, t), hi = std::max(hi, t);
            }
            const double span = hi > lo ? hi - lo : 1.0;
            for (int32_t i = 0; i < A; ++i) y[e][i] = (y[e][i] - lo) / span;
        }
        // Hilbert index of the two coordinates (no Z-order jumps: 32 consecutive vertices
        // stay one compact patch)
        constexpr int QB2 = 24;
        const uint64_t n = 1ull << QB2;
        for (int32_t i = 0; i < A; ++i) {
            uint64_t x = (uint64_t)(y[0][i] * (double)(n - 1)), z = (uint64_t)(y[1][i] * (double)(n - 1)), d = 0;
            for (uint64_t sh = n >> 1; sh > 0; sh >>= 1) {
                const uint64_t rx = (x & sh) ? 1 : 0, rz = (z & sh) ? 1 : 0;
                d += sh * sh * ((3 * rx) ^ rz);
                if (rz == 0) {
                    if (rx == 1) x = n - 1 - x, z = n - 1 - z;
                    std::swap(x, z);
                }
            }
            key[i] = d;
        }
        return SHADOWTOPO_OK;
    }
    constexpr int QB = 21;  // three 21-bit coordinates per 64-bit key
    const uint64_t qmax = (1ull << QB) - 1;
    for (size_t k = 0; k < std::min<size_t>(dl.size(), 3); ++k) {
        double lo = HINF, hi = -HINF;
        for (int32_t i = 0; i < A; ++i) {
            const double d = dl[k][i];
            if (d < HINF) lo = std::min(lo, d), hi = std::max(hi, d);
        }
        const double span = hi > lo ? hi - lo : 1.0;
        for (int32_t i = 0; i < A; ++i) {
            const double d = dl[k][i];
            const uint64_t q = d < HINF ? std::min<uint64_t>(qmax, (uint64_t)((d - lo) / span * (double)qmax)) : qmax;
            for (int b = 0; b < QB; ++b) key[i] |= ((q >> b) & 1ull) << (b * 3 + k);
        }
    }
    return SHADOWTOPO_OK;
}

// the attached rows in key order (ties by row), once per attached set: a group's lanes are
// then its rows picked out of it in one pass, instead of a sort per group and call (C2's
// 1000-row group: tens of microseconds of host time between the steps)
static void key_order(shadowtopo_engine* eng) {
    eng->h_key_order.resize((size_t)eng->A);
    for (int32_t i = 0; i < eng->A; ++i) eng->h_key_order[i] = i;
    std::stable_sort(eng->h_key_order.begin(), eng->h_key_order.end(),
                     [&](int32_t x, int32_t y) { return eng->h_key[x] < eng->h_key[y]; });
    eng->key_ready = true;
}

int ensure_locality(shadowtopo_engine* eng, hipStream_t s) {
    if (eng->key_ready) return SHADOWTOPO_OK;
    if (eng->A <= KL) {
        eng->h_key.assign((size_t)eng->A, 0);
        key_order(eng);
        return SHADOWTOPO_OK;
    }
    if (eng->vperm_ready && !eng->h_vkey.empty()) {  // the pruned sweep's vertex keys
        eng->h_key.resize((size_t)eng->A);
        for (int32_t i = 0; i < eng->A; ++i) eng->h_key[i] = eng->h_vkey[eng->h_attached[i]];
        key_order(eng);
        return SHADOWTOPO_OK;
    }
    int rc = locality_keys(eng, s, eng->h_attached, eng->h_key, 8, true);
    if (rc) return rc;
    key_order(eng);
    return SHADOWTOPO_OK;
}

// Pruned dense sweep: the vertex locality order, W32 permuted into it, and the per-chunk,
// per-wave-tile W32 minima.  Built once per engine (the landmark rounds run the unpruned
// sweep); any order gives the same results, a local one lets waves skip chunks.
int ensure_vperm(shadowtopo_engine* eng, hipStream_t s) {
    if (eng->vperm_ready || !eng->dense || !eng->opt_dense_prune || !eng->d_W32) return SHADOWTOPO_OK;
    const int32_t V = eng->V, Vp = eng->Vp;
    if (V <= SRS) return SHADOWTOPO_OK;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<int32_t> all((size_t)V);
    for (int32_t v = 0; v < V; ++v) all[v] = v;
    std::vector<uint64_t>& key = eng->h_vkey;
    int rc = locality_keys(eng, s, all, key, 8, true);
    if (rc) return rc;
    std::vector<int32_t> perm(all);
    std::stable_sort(perm.begin(), perm.end(), [&](int32_t a, int32_t b) { return key[a] < key[b]; });
    for (int32_t i = V; i < Vp; ++i) perm.push_back(i);
    constexpr int TDT = FTDT;  // launch_dense_ft's wave tile
    const int32_t nchunks = (V + SRS - 1) / SRS;
    const int32_t nwt = Vp;  // columns (every block shape's tiles stay inside Vp)
    HIP_TRY(hipMalloc((void**)&eng->d_perm, sizeof(int32_t) * (size_t)Vp));
    HIP_TRY(hipMalloc((void**)&eng->d_W32p, sizeof(float) * (size_t)Vp * Vp));
    HIP_TRY(hipMalloc((void**)&eng->d_minW, sizeof(float) * (size_t)nchunks * nwt));
    HIP_TRY(hipMemcpyAsync(eng->d_perm, perm.data(), sizeof(int32_t) * (size_t)Vp, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_permute_w<float>, dim3((uint32_t)Vp), dim3(256), 0, s, eng->d_W32, eng->d_perm, Vp,
                       eng->d_W32p);
    // the f64 weights in the same order, and the order's inverse (the sweep's seed and exact
    // row reads: one segment per lane and row instead of a line per weight)
    std::vector<int32_t> ipos((size_t)Vp);
    for (int32_t i = 0; i < Vp; ++i) ipos[(size_t)perm[i]] = i;
    HIP_TRY(hipMalloc((void**)&eng->d_Wp, sizeof(double) * (size_t)Vp * Vp));
    HIP_TRY(hipMalloc((void**)&eng->d_pos, sizeof(int32_t) * (size_t)Vp));
    HIP_TRY(hipMemcpyAsync(eng->d_pos, ipos.data(), sizeof(int32_t) * (size_t)Vp, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_permute_w<double>, dim3((uint32_t)Vp), dim3(256), 0, s, eng->d_W, eng->d_perm, Vp, eng->d_Wp);
    if (eng->d_WI && eng->d_WR) {  // the seed winners' arcs and reliability factors (dense_epilogue)
        HIP_TRY(hipMalloc((void**)&eng->d_WIp, sizeof(int32_t) * (size_t)Vp * Vp));
        HIP_TRY(hipMalloc((void**)&eng->d_WRp, sizeof(double) * (size_t)Vp * Vp));
        hipLaunchKernelGGL(k_permute_w<int32_t>, dim3((uint32_t)Vp), dim3(256), 0, s, eng->d_WI, eng->d_perm, Vp,
                           eng->d_WIp);
        hipLaunchKernelGGL(k_permute_w<double>, dim3((uint32_t)Vp), dim3(256), 0, s, eng->d_WR, eng->d_perm, Vp,
                           eng->d_WRp);
    }
    hipLaunchKernelGGL(k_min_w32, dim3((uint32_t)(((int64_t)nchunks * nwt + 255) / 256)), dim3(256), 0, s,
                       eng->d_W32p, Vp, nchunks, nwt, 1, eng->d_minW);
    const int32_t nvc = Vp / KL;
    HIP_TRY(hipMalloc((void**)&eng->d_minW64, sizeof(float) * (size_t)nvc * nvc));
    hipLaunchKernelGGL(k_min_w64, dim3((uint32_t)(((int64_t)nvc * nvc + 3) / 4)), dim3(256), 0, s, eng->d_W32p, Vp,
                       nvc, eng->d_minW64);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    eng->vperm_ready = true;
    eng->st.order_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return SHADOWTOPO_OK;
}

// page-locked host memory (hipHostMalloc / shadowtopo_host_alloc / hipHostRegister)
bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error for the caller
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Pendant trees (the attached-pair matrix never needs them).  In an
// undirected graph a non-attached vertex with at most one neighbour lies on no shortest
// path between two other vertices (entering and leaving it would repeat its neighbour; every
// latency is > 0), so peeling such vertices repeatedly leaves every attached-pair path, its
// distance, predecessor chain, hops and reliability as they were.  The relaxation view gp is
// the in-CSR restricted to the remaining vertices (rows of peeled vertices empty, arcs from
// them dropped, row order kept): their state is never activated, read or written.  Ties the
// peeled vertices could raise are the degenerate d(u) == d(v) kind at their attachment
// vertex, which igraph resolves in favour of the core (the attachment vertex is popped
// first), so only flags that were conservative disappear; the heap-exact replay keeps the
// full graph.  C5: 24 % of the vertices, 11 % of the arcs.
int ensure_mirrors(shadowtopo_engine* eng);

// the pendant-pruned view on the device.  nid[v]: v's id in the view (-1: peeled).  One wave
// per vertex: cnt[nid v] = its in-arcs from kept tails
__global__ __launch_bounds__(256) void k_view_count(const int64_t* __restrict__ in_ptr,
                                                    const int32_t* __restrict__ in_src,
                                                    const int32_t* __restrict__ nid, int32_t V,
                                                    int32_t* __restrict__ cnt) {
    const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (v >= V) return;
    const int32_t n = nid[v];
    if (n < 0) return;
    int32_t c = 0;
    for (int64_t e = in_ptr[v] + lane; e < in_ptr[v + 1]; e += 64) c += nid[in_src[e]] >= 0;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) cnt[n] = c;
}

// ptr[0] = 0, ptr[i + 1] = cnt[0] + .. + cnt[i] for i < n: one block, a contiguous segment per
// thread, the segment sums scanned in LDS
__global__ __launch_bounds__(1024) void k_view_scan(const int32_t* __restrict__ cnt, int32_t n,
                                                    int64_t* __restrict__ ptr) {
    __shared__ int64_t sc[1024];
    const int32_t per = (n + 1023) / 1024;
    const int32_t b = threadIdx.x * per, e = min(n, b + per);
    int64_t sum = 0;
    for (int32_t i = b; i < e; ++i) sum += cnt[i];
    sc[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const int64_t add = threadIdx.x >= (unsigned)off ? sc[threadIdx.x - off] : 0;
        __syncthreads();
        sc[threadIdx.x] += add;
        __syncthreads();
    }
    int64_t run = sc[threadIdx.x] - sum;
    if (threadIdx.x == 0) ptr[0] = 0;
    for (int32_t i = b; i < e; ++i) {
        run += cnt[i];
        ptr[i + 1] = run;
    }
}

// the kept arcs of each kept vertex, in row order (wave per vertex: a ballot prefix per 64 arcs)
__global__ __launch_bounds__(256) void k_view_fill(const int64_t* __restrict__ in_ptr,
                                                   const int32_t* __restrict__ in_src,
                                                   const int32_t* __restrict__ in_eid,
                                                   const double* __restrict__ in_w,
                                                   const float* __restrict__ in_w32,
                                                   const double* __restrict__ in_r,
                                                   const int32_t* __restrict__ nid, int32_t V,
                                                   const int64_t* __restrict__ ptr, int32_t* __restrict__ src,
                                                   int32_t* __restrict__ eid, double* __restrict__ w,
                                                   float* __restrict__ w32, double* __restrict__ r) {
    const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (v >= V) return;
    const int32_t n = nid[v];
    if (n < 0) return;
    int64_t o = ptr[n];
    for (int64_t e0 = in_ptr[v]; e0 < in_ptr[v + 1]; e0 += 64) {
        const int64_t e = e0 + lane;
        const int32_t t = e < in_ptr[v + 1] ? nid[in_src[e]] : -1;
        const unsigned long long m = __ballot(t >= 0);
        if (t >= 0) {
            const int64_t q = o + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            src[q] = t;
            eid[q] = in_eid[e];
            w[q] = in_w[e];
            w32[q] = in_w32[e];
            r[q] = in_r[e];
        }
        o += __popcll(m);
    }
}

// per-vertex tables in the view's ids, the attached list in them, and the builder's padding
// arcs after the na0 kept arcs (u = 0, w = +inf)
__global__ __launch_bounds__(256) void k_view_tables(const double* __restrict__ vfac,
                                                     const int32_t* __restrict__ loop_eid,
                                                     const int32_t* __restrict__ nid, int32_t V,
                                                     const int32_t* __restrict__ attached, int32_t A, int64_t na0,
                                                     double* __restrict__ vf, int32_t* __restrict__ loop,
                                                     int32_t* __restrict__ att, int32_t* __restrict__ src,
                                                     int32_t* __restrict__ eid, double* __restrict__ w,
                                                     float* __restrict__ w32, double* __restrict__ r) {
    const int32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < V) {
        const int32_t n = nid[i];
        if (n >= 0) {
            vf[n] = vfac[i];
            loop[n] = loop_eid[i];
        }
    }
    if (i < A) att[i] = nid[attached[i]];
    if (i < CSR_PAD) {
        src[na0 + i] = 0;
        eid[na0 + i] = -1;
        w[na0 + i] = dinf();
        w32[na0 + i] = __int_as_float(0x7f800000);
        r[na0 + i] = 0.0;
    }
}

int ensure_pruned(shadowtopo_engine* eng, hipStream_t s) {
    if (eng->prune_ready || !eng->opt_prune || eng->dense || (eng->flags & SHADOWTOPO_F_DIRECTED) ||
        (eng->flags & SHADOWTOPO_F_COMPLETE) || eng->n_arcs == 0)
        return SHADOWTOPO_OK;
    int rc;
    static const bool trace_prep = getenv("SHADOWTOPO_TRACE_PREP") != nullptr;
    auto t_ph = std::chrono::steady_clock::now();
    const auto phase = [&](const char* what) {
        if (!trace_prep) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[prep]   view: %s %.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_ph).count());
        t_ph = t;
    };
    if ((rc = ensure_mirrors(eng))) return rc;
    phase("mirrors");
    const int32_t V = eng->V;
    const int64_t M = eng->n_arcs;
    const std::vector<int64_t>& ptr = eng->h_in_ptr;
    const std::vector<int32_t>& src = eng->h_in_src;
    // peel: degree = distinct neighbours (the in-CSR merges parallel edges and drops loops)
    std::vector<uint8_t> keep((size_t)V, 1), att((size_t)V, 0);
    for (int32_t a : eng->h_attached) att[a] = 1;
    std::vector<int32_t> deg((size_t)V), stack;
    for (int32_t v = 0; v < V; ++v) {
        deg[v] = (int32_t)(ptr[v + 1] - ptr[v]);
        if (deg[v] <= 1 && !att[v]) stack.push_back(v);
    }
    int64_t peeled = 0, cut = 0;  // cut: edges to kept neighbours the peeled vertices took along
    while (!stack.empty()) {
        const int32_t x = stack.back();
        stack.pop_back();
        if (!keep[x]) continue;
        keep[x] = 0;
        ++peeled;
        cut += deg[x];  // its kept neighbours now (0 or 1): every other arc left with an earlier peel
        for (int64_t e = ptr[x]; e < ptr[x + 1]; ++e) {
            const int32_t y = src[e];
            if (keep[y] && --deg[y] <= 1 && !att[y]) stack.push_back(y);
        }
    }
    eng->pruned_vertices = peeled;
    phase("peel");
    eng->h_view_of.clear();
    eng->d_att_view = nullptr;
    eng->view_gen++;
    if (peeled == 0) {  // nothing to drop: relax over g (and do not peel again for this set)
        eng->gp = eng->g;
        eng->gp_arcs = eng->n_arcs;
        eng->prune_ready = true;
        return SHADOWTOPO_OK;
    }
    // the kept vertices renumbered densely in their original order, so the batch pools,
    // grids and flag scans cover only them (C5: 24 % fewer state rows, more batches per
    // group); every attached vertex is kept
    std::vector<int32_t> nid((size_t)V, -1);
    int32_t Vc = 0;
    for (int32_t v = 0; v < V; ++v)
        if (keep[v]) nid[v] = Vc++;
    // the filtered arrays, row order kept, with the builder's padding arcs at the end, built on
    // the device from the resident in-CSR (k_view_*: 2 ms on C5 where the host built and
    // uploaded them in 45 ms); the buffers are kept across attached sets at the graph's sizes
    const int64_t na0 = M - 2 * cut;  // kept arcs: every cut edge was two arcs
    const size_t na = (size_t)na0 + CSR_PAD;
    const int32_t A = eng->A;
    if (eng->view_cap_a < (size_t)std::max(A, 1)) {
        for (void* p : eng->prune_allocs) (void)hipFree(p);
        eng->prune_allocs.clear();
        eng->view_cap_a = 0;
        ViewBufs& vb = eng->vb;
        const size_t Mc = (size_t)M + CSR_PAD, Ac = (size_t)std::max(A, 1);
        if ((rc = dev_alloc(eng->prune_allocs, (void**)&vb.nid, 4 * (size_t)V)) ||
            (rc = dev_alloc(eng->prune_allocs, (void**)&vb.cnt, 4 * (size_t)V)) ||
            (rc = dev_alloc(eng->prune_allocs, (void**)&vb.vf, 8 * (size_t)V)) ||
            (rc = dev_alloc(eng->prune_allocs, (void**)&vb.loop, 4 * (size_t)V)) ||
            (rc = dev_alloc(eng->prune_allocs, (void**)&vb.att, 4 * Ac)) ||
            (rc = dev_alloc(eng->prune_allocs, (void**)&vb.ptr, 8 * ((size_t)V + 1))) ||
            (rc = dev_alloc(eng->prune_allocs, (void**)&vb.src, 4 * Mc)) ||
            (rc = dev_alloc(eng->prune_allocs, (void**)&vb.eid, 4 * Mc)) ||
            (rc = dev_alloc(eng->prune_allocs, (void**)&vb.w, 8 * Mc)) ||
            (rc = dev_alloc(eng->prune_allocs, (void**)&vb.r, 8 * Mc)) ||
            (rc = dev_alloc(eng->prune_allocs, (void**)&vb.w32, 4 * Mc)))
            return rc;
        eng->view_cap_a = Ac;
    }
    const ViewBufs& vb = eng->vb;
    HIP_TRY(hipMemcpyAsync(vb.nid, nid.data(), 4 * (size_t)V, hipMemcpyHostToDevice, s));
    const GraphDev& g0 = eng->g;
    const uint32_t wv = (uint32_t)(((int64_t)V + 3) / 4);  // one wave per vertex
    hipLaunchKernelGGL(k_view_count, dim3(wv), dim3(256), 0, s, g0.in_ptr, g0.in_src, vb.nid, V, vb.cnt);
    hipLaunchKernelGGL(k_view_scan, dim3(1), dim3(1024), 0, s, vb.cnt, Vc, vb.ptr);
    hipLaunchKernelGGL(k_view_fill, dim3(wv), dim3(256), 0, s, g0.in_ptr, g0.in_src, g0.in_eid, g0.in_w, g0.in_w32,
                       g0.in_r, vb.nid, V, (const int64_t*)vb.ptr, vb.src, vb.eid, vb.w, vb.w32, vb.r);
    hipLaunchKernelGGL(k_view_tables, dim3((uint32_t)((std::max(V, A) + 255) / 256)), dim3(256), 0, s, g0.vfac,
                       g0.loop_eid, vb.nid, V, eng->d_attached, A, na0, vb.vf, vb.loop, vb.att, vb.src, vb.eid, vb.w,
                       vb.w32, vb.r);
    HIP_TRY(hipGetLastError());
    // the view's arc count was derived from the peel; the scan's total must agree
    int64_t tot = -1;
    HIP_TRY(hipMemcpyAsync(&tot, vb.ptr + Vc, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));  // a pageable destination: the whole copy
    if (tot != na0) return fail(SHADOWTOPO_EINTERNAL, "pendant view: %lld arcs kept, %lld expected", (long long)tot,
                                (long long)na0);
    phase("device build");
    GraphDev gp = eng->g;
    int64_t* d_ptr = vb.ptr;
    int32_t *d_src = vb.src, *d_eid = vb.eid, *d_loop = vb.loop, *d_att = vb.att;
    double *d_w = vb.w, *d_r = vb.r, *d_vf = vb.vf;
    float* d_w32 = vb.w32;
    gp.in_ptr = d_ptr;
    gp.in_src = d_src;
    gp.in_eid = d_eid;
    gp.in_w = d_w;
    gp.in_r = d_r;
    gp.in_w32 = d_w32;
    gp.out_ptr = d_ptr;  // undirected: out-neighbours = in-neighbours
    gp.out_dst = d_src;
    gp.V = Vc;
    gp.Vp = (Vc + 63) / 64 * 64;
    gp.vfac = d_vf;
    gp.loop_eid = d_loop;
    gp.inc_ptr = nullptr;  // the self rule and the replay run on g, in the original ids
    gp.inc_eid = nullptr;
    gp.inc_lat = nullptr;
    eng->gp = gp;
    eng->gp_arcs = (int64_t)na - CSR_PAD;
    eng->h_view_of = std::move(nid);
    eng->d_att_view = d_att;
    eng->prune_ready = true;
    return SHADOWTOPO_OK;
}

// k_walk over the group's nbg batches: a block = 4 waves of TPW walk targets each, NC walk
// chains per lane
template <bool MG, int TPW, int NC>
void launch_walk_t(shadowtopo_engine* eng, int32_t nbg, const int32_t* att, int32_t A, double* dl, double* dr,
                   int32_t row_base, int32_t ls, hipStream_t s) {
    constexpr int TPB = TPW * (WALK_T / 64);
    hipLaunchKernelGGL((k_walk<MG, TPW, NC>), dim3((uint32_t)((eng->n_walk + TPB - 1) / TPB), nbg), dim3(WALK_T), 0, s,
                       *eng->rg, eng->d_arcinfo, eng->pools, att, eng->d_walk, eng->n_walk, A, dl, dr, row_base, ls);
}
// shape 1 (default): one walk target per wave, one chain per lane.  Walks are bound by the
// tree records' cache footprint (a batch's 16-byte records are ~100 MB on C4): the fewer
// targets a wave takes, the fewer batches are walked at once and the more record lines
// stay in the Infinity Cache.  C4L, compose + walks per build (r05i): 1 target / 1 chain
// 3.48 ms, 2 / 2 3.67, 2 / 1 4.18, 4 / 2 4.67; a chain that refills itself from the
// wave's targets lost the same way (8 targets per wave 5.8 ms, 16 6.7)
template <bool MG>
void launch_walk_m(shadowtopo_engine* eng, int32_t nbg, const int32_t* att, int32_t A, double* dl, double* dr,
                   int32_t row_base, int32_t ls, hipStream_t s) {
    if (eng->opt_walk_tpw == 2)
        launch_walk_t<MG, 2, 2>(eng, nbg, att, A, dl, dr, row_base, ls, s);
    else
        launch_walk_t<MG, 1, 1>(eng, nbg, att, A, dl, dr, row_base, ls, s);
}
// k_walk_lean: TPW targets per wave, NC walks per lane (OPT_WALK_TPW: 1 = 1 / 1, 2 = 2 / 2,
// 3 = 4 / 2, 4 = 8 / 2)
template <bool MG, int TPW, int NC>
void launch_walk_lean_t(shadowtopo_engine* eng, int32_t nbg, const int32_t* att, int32_t A, double* dl, double* dr,
                        uint32_t* dh, int32_t row_base, int32_t ls, hipStream_t s) {
    constexpr int TPB = TPW * (WALK_T / 64);
    hipLaunchKernelGGL((k_walk_lean<MG, TPW, NC>), dim3((uint32_t)((A + TPB - 1) / TPB), nbg), dim3(WALK_T), 0, s,
                       *eng->rg, eng->d_arcinfo, eng->pools, att, A, dl, dr, dh, row_base, ls);
}
template <bool MG>
void launch_walk_lean_m(shadowtopo_engine* eng, int32_t nbg, const int32_t* att, int32_t A, double* dl, double* dr,
                        uint32_t* dh, int32_t row_base, int32_t ls, hipStream_t s) {
    switch (eng->opt_walk_tpw) {
        case 2: launch_walk_lean_t<MG, 2, 2>(eng, nbg, att, A, dl, dr, dh, row_base, ls, s); break;
        case 3: launch_walk_lean_t<MG, 4, 2>(eng, nbg, att, A, dl, dr, dh, row_base, ls, s); break;
        case 4: launch_walk_lean_t<MG, 8, 2>(eng, nbg, att, A, dl, dr, dh, row_base, ls, s); break;
        default: launch_walk_lean_t<MG, 1, 1>(eng, nbg, att, A, dl, dr, dh, row_base, ls, s); break;
    }
}
hipError_t launch_walk_lean(shadowtopo_engine* eng, int32_t nbg, const int32_t* att, int32_t A, double* dl,
                            double* dr, uint32_t* dh, int32_t row_base, int32_t ls, hipStream_t s) {
    if (eng->multigraph)
        launch_walk_lean_m<true>(eng, nbg, att, A, dl, dr, dh, row_base, ls, s);
    else
        launch_walk_lean_m<false>(eng, nbg, att, A, dl, dr, dh, row_base, ls, s);
    return hipGetLastError();
}

hipError_t launch_walk(shadowtopo_engine* eng, int32_t nbg, const int32_t* att, int32_t A, double* dl, double* dr,
                       int32_t row_base, int32_t ls, hipStream_t s) {
    if (eng->multigraph)
        launch_walk_m<true>(eng, nbg, att, A, dl, dr, row_base, ls, s);
    else
        launch_walk_m<false>(eng, nbg, att, A, dl, dr, row_base, ls, s);
    return hipGetLastError();
}

int compute_rows_impl(shadowtopo_engine* eng, int32_t row_begin, int32_t row_end, double* lat, double* rel,
                      uint32_t* hops, uint8_t* kind, int32_t mem, hipStream_t s) {
    // MEM_HOST_LR: host rows of {lat, rel} pairs in `lat` (the shim's per-packet layout); the
    // staging rows are composed interleaved (element stride 2) and leave in one copy
    const bool lr = mem == SHADOWTOPO_MEM_HOST_LR;
    if (lr) mem = SHADOWTOPO_MEM_HOST;
    const int32_t ls = lr ? 2 : 1;
    const int32_t A = eng->A;
    const bool complete = (eng->flags & SHADOWTOPO_F_COMPLETE) != 0;
    int rc;
    // the self rule of these rows' diagonal pairs (rule 2 of the pair dispatch), inside every
    // computation: the reference computes the self path per query (topology.c:1545-1653),
    // so the matrix build includes it; timed with events once per attached set (the shim
    // reports it as the reference's selfPathTotalTime, topology.c:1608-1617) or with OPT_TIMING
    bool self_pending = false;
    if (!complete) {
        self_pending = eng->opt_timing || !eng->self_timed;
        if (self_pending) HIP_TRY(hipEventRecord(eng->ev_self[0], s));
        HIP_TRY(launch_self(eng, eng->g, row_begin, row_end, eng->d_self_lat, eng->d_self_rel, eng->d_self_hops,
                            eng->d_self_kind, s));
        if (self_pending) HIP_TRY(hipEventRecord(eng->ev_self[1], s));
        eng->st.self_paths += row_end - row_begin;
    }
    const auto t_att = std::chrono::steady_clock::now();
    // SHADOWTOPO_TRACE_PREP=1: the attached-set preparation's phases on stderr (diagnostics)
    static const bool trace_prep = getenv("SHADOWTOPO_TRACE_PREP") != nullptr;
    auto t_ph = t_att;
    const auto phase = [&](const char* what) {
        if (!trace_prep) return;
        const auto t = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(t - t_ph).count();
        if (ms > 0.05) fprintf(stderr, "[prep] %s %.2f ms\n", what, ms);
        t_ph = t;
    };
    if ((rc = ensure_pruned(eng, s))) return rc;
    phase("pendant view");
    eng->rg = eng->prune_ready ? &eng->gp : &eng->g;  // back to g for sssp (shadowtopo_sssp)
    // lean sparse rounds (D + the predecessor arc, 12 B per pair instead of 24; no predecessor
    // gathers in the rounds; hops, reliability and the taint come from a walk per pair after
    // the rounds, k_walk_lean) pay when the walks are cheap against the rounds: a walk costs
    // ~3.5 arc-row visits per hop (r05), the tree fold ~20 % of the rounds, so lean when the
    // graph has many arcs per attached target (C4: 60, C5: 72 -> lean; C3: 16 -> fold)
    {
        const int64_t arcs = eng->rg == &eng->g ? eng->n_arcs : eng->gp_arcs;
        eng->lean_next = !eng->dense && !complete && eng->opt_csr_variant == SHADOWTOPO_CSR_FULL &&
                         (eng->opt_csr_lean == 1 || (eng->opt_csr_lean == 2 && arcs >= 32 * (int64_t)A));
    }
    if (!eng->walk_ready && !complete) {
        // the targets whose pairs k_walk re-folds: vertex loss present (a factor != 1), or all
        // of them in a multigraph (lat from the get_eid edges)
        std::vector<int32_t> wl;
        for (int32_t i = 0; i < A; ++i)
            if (eng->multigraph || eng->h_vfac[(size_t)eng->h_attached[i]] != 1.0) wl.push_back(i);
        eng->n_walk = (int32_t)wl.size();
        if (!wl.empty()) {
            if (eng->walk_cap < wl.size()) {
                if (eng->d_walk) (void)hipFree(eng->d_walk);
                eng->d_walk = nullptr;
                eng->walk_cap = 0;
                HIP_TRY(hipMalloc((void**)&eng->d_walk, wl.size() * sizeof(int32_t)));
                eng->walk_cap = wl.size();
            }
            HIP_TRY(hipMemcpyAsync(eng->d_walk, wl.data(), wl.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
            HIP_TRY(hipStreamSynchronize(s));  // wl is a local
        }
        eng->walk_ready = true;
    }
    eng->st.walk_targets = eng->n_walk;
    phase("walk list");
    if ((eng->n_walk > 0 || eng->lean_next) &&
        (eng->arcinfo_of != eng->rg->in_src || eng->arcinfo_gen != eng->view_gen)) {
        // the walks' per-arc table, for the graph the rounds run on (rebuilt with the view)
        const int64_t na = eng->rg == &eng->g ? eng->n_arcs : eng->gp_arcs;
        if (eng->arcinfo_cap < (size_t)std::max<int64_t>(na, 1)) {
            if (eng->d_arcinfo) (void)hipFree(eng->d_arcinfo);
            eng->d_arcinfo = nullptr;
            eng->arcinfo_cap = 0;
            HIP_TRY(hipMalloc((void**)&eng->d_arcinfo, sizeof(ArcInfo) * (size_t)std::max<int64_t>(na, 1)));
            eng->arcinfo_cap = (size_t)std::max<int64_t>(na, 1);
        }
        if (na > 0)
            hipLaunchKernelGGL(k_arcinfo, dim3((uint32_t)std::min<int64_t>((na + 255) / 256, 8192)), dim3(256), 0, s,
                               eng->rg->in_src, eng->rg->in_eid, eng->rg->in_r, na, eng->d_arcinfo);
        HIP_TRY(hipGetLastError());
        eng->arcinfo_of = eng->rg->in_src;
        eng->arcinfo_gen = eng->view_gen;
    }
    phase("arc table");
    // host destinations: rows are composed into device staging and copied out per group;
    // into pinned (page-locked) host memory -- shadowtopo_host_alloc, as the topology shim
    // allocates its matrix -- the copy of group g runs on the copy stream behind group
    // g + 1's relaxation (two staging slots), into pageable memory it is a synchronous copy
    const bool pinned_out = mem == SHADOWTOPO_MEM_HOST && is_pinned(lat) && (lr || is_pinned(rel)) &&
                            (!hops || is_pinned(hops)) && (!kind || is_pinned(kind));
    int32_t nb = default_nb(eng, row_end - row_begin);
    {
        // a computation that fits one group would copy all its rows after its last round.  Cut
        // into opt_host_split groups, every group's copy but the last runs behind the next
        // group's rounds: sparse graphs whose rows are >= 64 MB (r05, with the host waits
        // polling: C3 25.0 -> 21.4 ms, C4 168 -> 141 ms in 4 groups, 6 / 8 no better; r04's
        // C4 loss to 4 groups was the blocking waits); dense graphs only when the rows outweigh
        // the arcs (C2's one sweep of 16 batches: 4.3 ms in one group, 5.4 in two)
        const int32_t need = (row_end - row_begin + KL - 1) / KL;
        const double row_bytes = (double)A * (16 + (hops ? 4 : 0) + (kind ? 1 : 0));
        const double bytes = row_bytes * (row_end - row_begin);
        if (pinned_out && eng->opt_host_groups > 0 && nb >= need)  // OPT_HOST_GROUPS: forced
            nb = std::max(1, (need + eng->opt_host_groups - 1) / eng->opt_host_groups);
        else if (pinned_out && eng->opt_host_split > 1 && nb >= need && bytes >= 64.0e6 &&
                 (!eng->dense || row_bytes >= 0.5 * (double)eng->n_arcs)) {
            // groups of at least 24 batches: smaller groups' rounds are latency-bound (C4's
            // 8-rank share, 20 batches: 23.1 ms in one group, 27.0 in four)
            const int32_t ng = std::min(eng->opt_host_split, need / 24);
            if (ng >= 2) nb = (need + ng - 1) / ng;
        }
    }
    {
        // groups of equal size: C5's 782 batches at 260 per group ran as 260 / 260 / 260 / 2,
        // and the last group's ~19 rounds over 2 batches were nearly all overhead
        const int32_t need = (row_end - row_begin + KL - 1) / KL;
        if (nb < need) {
            const int32_t ng = (need + nb - 1) / nb;
            nb = (need + ng - 1) / ng;
        }
    }
    if ((rc = ensure_batches(eng, nb)) == SHADOWTOPO_ENOMEM && eng->floor_ok) {
        // the 24 GB floor was free once, but something else has taken HBM since (another
        // engine or process on the device): size the pools from a fresh free-memory query
        (void)hipGetLastError();  // the failed hipMalloc's error, not a launch's
        eng->floor_ok = false;
        eng->floor_checked = true;
        free_batches(eng);  // what the failed attempt did allocate is free again: held = 0
        nb = default_nb(eng, row_end - row_begin);
        rc = ensure_batches(eng, nb);
    }
    if (rc) return rc;
    phase("pools");
    const int32_t group = nb * KL;
    if ((rc = ensure_vperm(eng, s))) return rc;
    // rows of a group go to batch lanes in locality order (CSR rounds, and the pruned dense
    // sweep, whose chunk skips need a batch's sources near each other; the unpruned dense
    // sweeps cost the same for any batch)
    const bool order = eng->opt_source_order && (!eng->dense || eng->vperm_ready) && !complete &&
                       row_end - row_begin > KL;
    if (order && (rc = ensure_locality(eng, s))) return rc;
    phase("source order");
    // host wall time of what depends on the attached set (zero when the set is unchanged)
    eng->st.attach_prep_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_att).count();
    std::vector<int32_t> lane_row;
    // a renumbered relaxation view: sources and targets in its ids
    const bool view = eng->rg == &eng->gp && !eng->h_view_of.empty();
    const int32_t* d_att_r = view ? eng->d_att_view : eng->d_attached;
    // device destinations (user buffers or staging)
    double *dl = lat, *dr = rel;
    uint32_t* dh = hops;
    uint8_t* dk = kind;
    const int nslots = pinned_out && row_end - row_begin > group ? 2 : 1;
    const size_t slot_bytes = ((size_t)group * A * (8 + 8 + (hops ? 4 : 0) + (kind ? 1 : 0)) + 255) & ~(size_t)255;
    if (mem == SHADOWTOPO_MEM_HOST) {
        const size_t need = slot_bytes * nslots + 64;
        if (eng->stage_bytes < need) {
            if (eng->copy_stream) HIP_TRY(hipStreamSynchronize(eng->copy_stream));
            if (eng->stage) (void)hipFree(eng->stage);
            eng->stage = nullptr;
            eng->stage_bytes = 0;
            HIP_TRY(hipMalloc(&eng->stage, need));
            eng->stage_bytes = need;
        }
        if (pinned_out && !eng->copy_stream) {
            HIP_TRY(hipStreamCreateWithFlags(&eng->copy_stream, hipStreamNonBlocking));
            for (int k = 0; k < 2; ++k) {
                HIP_TRY(hipEventCreateWithFlags(&eng->ev_comp[k], hipEventDisableTiming));
                HIP_TRY(hipEventCreateWithFlags(&eng->ev_copy[k], hipEventDisableTiming));
            }
        }
    }
    int64_t gidx = 0;
    for (int32_t r0 = row_begin; r0 < row_end; r0 += group, ++gidx) {
        const int32_t r1 = std::min(row_end, r0 + group);
        const int32_t nbg = (r1 - r0 + KL - 1) / KL;
        const int slot = (int)(gidx % nslots);
        int32_t row_base = row_begin;
        if (mem == SHADOWTOPO_MEM_HOST) {
            char* p = static_cast<char*>(eng->stage) + slot * slot_bytes;
            const size_t n = (size_t)group * A;
            dl = reinterpret_cast<double*>(p);
            dr = lr ? dl + 1 : reinterpret_cast<double*>(p + n * 8);
            dh = hops ? reinterpret_cast<uint32_t*>(p + n * 16) : nullptr;
            dk = kind ? reinterpret_cast<uint8_t*>(p + n * (hops ? 20 : 16)) : nullptr;
            row_base = r0;
            // the slot's previous rows (group g - 2) must have left before compose rewrites it
            if (pinned_out && gidx >= nslots) HIP_TRY(hipStreamWaitEvent(s, eng->ev_copy[slot], 0));
        }
        lane_row.assign((size_t)nbg * KL, -1);
        if (order) {  // the group's rows in key order (key_order)
            size_t n = 0;
            for (const int32_t row : eng->h_key_order)
                if (row >= r0 && row < r1) lane_row[n++] = row;
        } else {
            for (int32_t i = 0; i < r1 - r0; ++i) lane_row[i] = r0 + i;
        }
        for (size_t i = 0; i < lane_row.size(); ++i) {
            const int32_t row = lane_row[i];
            const int32_t v = row >= 0 ? eng->h_attached[row] : -1;
            eng->h_srcv[i] = (v >= 0 && view) ? eng->h_view_of[(size_t)v] : v;
            eng->h_row[i] = row;
        }
        HIP_TRY(hipMemcpyAsync(eng->pools.srcv, eng->h_srcv.data(), sizeof(int32_t) * KL * nbg,
                               hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(eng->pools.row, eng->h_row.data(), sizeof(int32_t) * KL * nbg,
                               hipMemcpyHostToDevice, s));
        // the pair compose (+ path walks) and the read-back of the tie-tainted sources (masks[1 + b])
        // and the walks' error word (masks[0]), into pinned host memory
        if (eng->h_masks_n < (size_t)nbg + 1) {
            if (eng->h_masks) (void)hipHostFree(eng->h_masks);
            eng->h_masks = nullptr;
            eng->h_masks_n = 0;
            HIP_TRY(hipHostMalloc((void**)&eng->h_masks, sizeof(unsigned long long) * (nb + 1), hipHostMallocDefault));
            eng->h_masks_n = (size_t)nb + 1;
        }
        const std::function<int()> enqueue_compose = [&]() -> int {
            HIP_TRY(hipMemsetAsync(eng->pools.err, 0, sizeof(unsigned long long) * (nbg + 1), s));
            if (eng->opt_timing) HIP_TRY(hipEventRecord(eng->ev_cmp[0], s));
            if (A > 0) {
                hipLaunchKernelGGL(k_compose, dim3((A + 63) / 64, nbg), dim3(COMPOSE_T), 0, s, *eng->rg, eng->pools,
                                   d_att_r, A, eng->d_self_lat, eng->d_self_rel, eng->d_self_hops,
                                   eng->d_self_kind, dl, dr, dh, dk, row_base, ls);
                HIP_TRY(hipGetLastError());
                if (eng->pools.P32) {  // lean rounds: every shortest-path pair's hops, rel and taint
                    HIP_TRY(launch_walk_lean(eng, nbg, d_att_r, A, dl, dr, dh, row_base, ls, s));
                } else if (eng->n_walk > 0) {  // the reference's full fold where the tree's is not it
                    HIP_TRY(launch_walk(eng, nbg, d_att_r, A, dl, dr, row_base, ls, s));
                }
            }
            if (eng->opt_timing) HIP_TRY(hipEventRecord(eng->ev_cmp[1], s));
            HIP_TRY(hipMemcpyAsync(eng->h_masks, eng->pools.err, sizeof(unsigned long long) * (nbg + 1),
                                   hipMemcpyDeviceToHost, s));
            return SHADOWTOPO_OK;
        };
        bool composed = false;
        if (!complete) {
            eng->unconverged = false;
            // speculative compose behind the dense delta rounds (not with the testing options
            // that act between the rounds and the compose)
            const bool spec = eng->opt_spec_compose && !eng->opt_test_scramble && !eng->opt_test_unconverged;
            if ((rc = run_rounds(eng, nbg, s, spec ? &enqueue_compose : nullptr, &composed))) return rc;
            // testing options: compose the state an iteration guard stopped at (every stream of
            // the device drained first: the rounds may have left work on the part streams), or
            // a scrambled tree
            if (eng->unconverged) HIP_TRY(hipDeviceSynchronize());
            if (eng->opt_test_scramble) {
                hipLaunchKernelGGL(k_scramble_tree, dim3(256, nbg), dim3(256), 0, s, *eng->rg, eng->pools,
                                   eng->opt_test_scramble);
                HIP_TRY(hipGetLastError());
            }
        }
        auto t0 = std::chrono::steady_clock::now();
        if (!composed) {
            if ((rc = enqueue_compose())) return rc;
            HIP_TRY(round_sync(eng, s));
        } else {
            eng->st.spec_composes++;
        }
        const unsigned long long* masks = eng->h_masks;
        eng->st.compose_ms +=
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (eng->opt_timing) {
            float ms = 0.0f;
            HIP_TRY(hipEventElapsedTime(&ms, eng->ev_cmp[0], eng->ev_cmp[1]));
            eng->st.compose_kernel_ms += ms;
        }
        if (self_pending) {
            float ms = 0.0f;
            HIP_TRY(hipEventElapsedTime(&ms, eng->ev_self[0], eng->ev_self[1]));
            eng->st.self_ms += ms;
            eng->self_timed = true;
            self_pending = false;
        }
        if (masks[0] || eng->unconverged)
            return fail(SHADOWTOPO_EINTERNAL,
                        !masks[0] ? "relaxation stopped at the iteration guard (composed for testing)" :
                        "a path walk left the predecessor tree (%s): the relaxation state is not a converged "
                        "shortest-path tree", masks[0] & 1 ? "arc or vertex out of range" : "hop count disagrees");
        std::vector<std::pair<int32_t, int32_t>> jobs;  // (vertex, row)
        for (int32_t b = 0; b < nbg; ++b) {
            for (int j = 0; j < KL; ++j) {
                const int32_t row = lane_row[(size_t)b * KL + j];
                if (row < 0) continue;
                if (complete) continue;
                if (eng->opt_force_replay || (masks[1 + b] >> j) & 1ull) jobs.emplace_back(eng->h_attached[row], row);
            }
        }
        if (!jobs.empty()) {
            auto t1 = std::chrono::steady_clock::now();
            if ((rc = ensure_replay(eng))) return rc;
            for (size_t k0 = 0; k0 < jobs.size(); k0 += REPLAY_SLOTS) {
                const int32_t nj = (int32_t)std::min<size_t>(REPLAY_SLOTS, jobs.size() - k0);
                for (int32_t k = 0; k < nj; ++k) {
                    eng->rp.srcv[k] = jobs[k0 + k].first;
                    eng->rp.row[k] = jobs[k0 + k].second;
                }
                hipLaunchKernelGGL(k_replay, dim3(nj), dim3(64), 0, s, eng->g, eng->rp, eng->d_attached, A, nj);
                HIP_TRY(hipGetLastError());
                hipLaunchKernelGGL(k_compose_replay, dim3((A + 255) / 256, nj), dim3(256), 0, s, eng->g, eng->rp,
                                   eng->d_attached, A, eng->d_self_lat, eng->d_self_rel, eng->d_self_hops,
                                   eng->d_self_kind, dl, dr, dh, dk, row_base, ls);
                HIP_TRY(hipGetLastError());
            }
            HIP_TRY(round_sync(eng, s));
            eng->st.replayed_sources += (int64_t)jobs.size();
            eng->st.replay_ms +=
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        }
        if (mem == SHADOWTOPO_MEM_HOST) {
            const size_t n = (size_t)(r1 - r0) * A;
            const size_t o = (size_t)(r0 - row_begin) * A;
            hipStream_t cs = pinned_out ? eng->copy_stream : s;
            if (pinned_out) {
                HIP_TRY(hipEventRecord(eng->ev_comp[slot], s));
                HIP_TRY(hipStreamWaitEvent(cs, eng->ev_comp[slot], 0));
            }
            if (lr) {
                HIP_TRY(hipMemcpyAsync(lat + 2 * o, dl, n * 16, hipMemcpyDeviceToHost, cs));
            } else {
                HIP_TRY(hipMemcpyAsync(lat + o, dl, n * 8, hipMemcpyDeviceToHost, cs));
                HIP_TRY(hipMemcpyAsync(rel + o, dr, n * 8, hipMemcpyDeviceToHost, cs));
            }
            if (hops) HIP_TRY(hipMemcpyAsync(hops + o, dh, n * 4, hipMemcpyDeviceToHost, cs));
            if (kind) HIP_TRY(hipMemcpyAsync(kind + o, dk, n, hipMemcpyDeviceToHost, cs));
            if (pinned_out)
                HIP_TRY(hipEventRecord(eng->ev_copy[slot], cs));
            else
                HIP_TRY(hipStreamSynchronize(s));  // pageable rows: the whole staged copy, host part included
        }
        eng->st.sources += r1 - r0;
        eng->st.batches += nbg;
        if (eng->pools.P32) eng->st.lean_groups++;
        eng->st.groups++;
        eng->st.group_batches = std::max<int64_t>(gidx == 0 ? 0 : eng->st.group_batches, nbg);
    }
    if (pinned_out) {  // the last group's rows have left
        HIP_TRY(hipEventRecord(eng->ev_spin, eng->copy_stream));
        HIP_TRY(spin_event(eng, eng->ev_spin));
    }
    return SHADOWTOPO_OK;
}

int ensure_mirrors(shadowtopo_engine* eng) {
    std::call_once(eng->mirrors_once, [eng] {
        const size_t V = (size_t)eng->V, M = (size_t)eng->n_arcs;
        eng->h_in_ptr.resize(V + 1);
        eng->h_in_src.resize(M);
        eng->h_in_eid.resize(M);
        eng->h_loop_eid.resize(V);
        // on the calling thread's device setting: restored below (shadowtopo_get_eid runs
        // on Shadow's worker threads, and the process may drive other devices)
        int prev = -1;
        (void)hipGetDevice(&prev);
        const bool ok = hipSetDevice(eng->device) == hipSuccess &&
                        hipMemcpy(eng->h_in_ptr.data(), eng->g.in_ptr, 8 * (V + 1), hipMemcpyDeviceToHost) == hipSuccess &&
                        (M == 0 || hipMemcpy(eng->h_in_src.data(), eng->g.in_src, 4 * M, hipMemcpyDeviceToHost) == hipSuccess) &&
                        (M == 0 || hipMemcpy(eng->h_in_eid.data(), eng->g.in_eid, 4 * M, hipMemcpyDeviceToHost) == hipSuccess) &&
                        hipMemcpy(eng->h_loop_eid.data(), eng->g.loop_eid, 4 * V, hipMemcpyDeviceToHost) == hipSuccess;
        if (prev >= 0) (void)hipSetDevice(prev);
        eng->mirrors_rc = ok ? 0 : fail(SHADOWTOPO_EDEVICE, "get_eid host mirrors");
    });
    return eng->mirrors_rc;
}

}  // namespace

extern "C" {

int shadowtopo_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* shadowtopo_last_error(void) { return g_err.c_str(); }


namespace {  // (internal linkage inside the extern "C" block)
// ---------------------------------------------------------------- engine creation helpers
// Host threads for the edge-list passes of shadowtopo_create: the box's CPU share, at most 16.
int host_workers(int64_t n_edges) {
    if (n_edges < (1 << 20)) return 1;
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, hw ? hw : 1u));
}

// The edge checks of topology.c:1070 and :1090 (plus endpoint range) over [a, z): the first
// failing edge, or z; loops counted into *loops.
int64_t first_bad_edge(int32_t V, int64_t a, int64_t z, const int32_t* src, const int32_t* dst, const double* lat,
                       const double* loss, int64_t* loops) {
    int64_t nl = 0;
    for (int64_t e = a; e < z; ++e) {
        nl += src[e] == dst[e];
        if (src[e] < 0 || src[e] >= V || dst[e] < 0 || dst[e] >= V || !(lat[e] > 0.0) || std::isinf(lat[e]) ||
            !(loss[e] >= 0.0 && loss[e] <= 1.0)) {
            *loops = nl;
            return e;
        }
    }
    *loops = nl;
    return z;
}

// Validate the edge list with W threads, each over its own slice; the error names the first
// failing edge in edge order, as one sequential scan would.
int validate_edges(int32_t V, int64_t n_edges, const int32_t* src, const int32_t* dst, const double* lat,
                   const double* loss, int64_t* n_loops) {
    const int W = host_workers(n_edges);
    std::vector<int64_t> bad((size_t)W, n_edges), loops((size_t)W, 0);
    auto work = [&](int w) {
        const int64_t a = n_edges * w / W, z = n_edges * (w + 1) / W;
        const int64_t e = first_bad_edge(V, a, z, src, dst, lat, loss, &loops[w]);
        bad[w] = e < z ? e : n_edges;
    };
    std::vector<std::thread> th;
    for (int w = 1; w < W; ++w) th.emplace_back(work, w);
    work(0);
    for (auto& t : th) t.join();
    int64_t e = n_edges, nl = 0;
    for (int w = 0; w < W; ++w) {
        e = std::min(e, bad[w]);
        nl += loops[w];
    }
    *n_loops = nl;
    if (e == n_edges) return SHADOWTOPO_OK;
    if (src[e] < 0 || src[e] >= V || dst[e] < 0 || dst[e] >= V)
        return fail(SHADOWTOPO_EINVAL, "edge %lld endpoint out of range", (long long)e);
    if (!(lat[e] > 0.0) || std::isinf(lat[e]))
        return fail(SHADOWTOPO_EINVAL, "edge %lld latency must be > 0 (topology.c:1070)", (long long)e);
    return fail(SHADOWTOPO_EINVAL, "edge %lld packetloss out of [0,1] (topology.c:1090)", (long long)e);
}

// Host -> device copies of the caller's (pageable) edge arrays through page-locked staging
// (tools/upload/upload_bench.hip, profiles/r03n_upload.jsonl, C2's 1.2 GB on the GPU box):
// hipMemcpy from pageable memory pins the source pages on first touch -- 80 ms, 15 GB/s for
// a fresh array (21 ms once pinned) -- while two threads filling a ring of four 8 MB
// page-locked buffers, each chunk's DMA issued in chunk order on one stream, move it at
// ~50 GB/s.  The ring is allocated once per process (hipHostMalloc costs ~3 ms per buffer)
// and kept; engine creations take it in turn.
struct UploadPart {
    void* dst;
    const void* src;
    size_t bytes;
};
#define GB_TRY_HIP(expr)                  \
    do {                                  \
        hipError_t e_ = (expr);           \
        if (e_ != hipSuccess) return e_;  \
    } while (0)
struct StagingRing {
    static constexpr size_t CH = (size_t)8 << 20;
    static constexpr int NB = 4;
    std::mutex mu;
    int device = -1;
    hipStream_t st = nullptr;
    void* buf[NB] = {};
    hipEvent_t ev[NB] = {};
};
StagingRing g_ring;

// the ring on `device` (caller holds R.mu)
hipError_t ring_ensure(StagingRing& R, int device) {
    constexpr int NB = StagingRing::NB;
    if (R.device != device) {  // first use, or another device: (re)create on this one
        if (R.st) (void)hipStreamDestroy(R.st);
        for (int k = 0; k < NB; ++k) {
            if (R.buf[k]) (void)hipHostFree(R.buf[k]);
            if (R.ev[k]) (void)hipEventDestroy(R.ev[k]);
            R.buf[k] = nullptr;
            R.ev[k] = nullptr;
        }
        R.st = nullptr;
        R.device = -1;
        GB_TRY_HIP(hipStreamCreateWithFlags(&R.st, hipStreamNonBlocking));
        for (int k = 0; k < NB; ++k) {
            GB_TRY_HIP(hipHostMalloc(&R.buf[k], StagingRing::CH, hipHostMallocDefault));
            GB_TRY_HIP(hipEventCreateWithFlags(&R.ev[k], hipEventDisableTiming));
        }
        R.device = device;
    }
    return hipSuccess;
}

hipError_t upload_staged(int device, const std::vector<UploadPart>& parts) {
    std::lock_guard<std::mutex> lk(g_ring.mu);
    StagingRing& R = g_ring;
    constexpr size_t CH = StagingRing::CH;
    constexpr int NB = StagingRing::NB;
    int W = 2;
#ifdef SHADOWTOPO_EXPERIMENTS
    if (const char* f = getenv("SHADOWTOPO_UPLOAD_FILLERS"))  // A/B knob
        if (atoi(f) >= 1 && atoi(f) <= NB) W = atoi(f);
#endif
    const bool tr = getenv("SHADOWTOPO_TRACE_BUILD") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    GB_TRY_HIP(ring_ensure(R, device));
    if (tr)
        fprintf(stderr, "[upload] ring setup %.2f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    std::vector<std::pair<size_t, size_t>> chunks;  // (part, offset)
    for (size_t p = 0; p < parts.size(); ++p)
        for (size_t o = 0; o < parts[p].bytes; o += CH) chunks.emplace_back(p, o);
    // chunk c fills buffer c % NB (after the DMA of chunk c - NB left it) on thread c % W, and
    // its DMA is issued in chunk order (a ticket), so the ring is reused in order
    std::atomic<size_t> ticket{0};
    std::atomic<int> failed{0};
    std::vector<hipError_t> err(W, hipSuccess);
    auto work = [&](int w) {
        hipError_t e = hipSetDevice(device);
        for (size_t c = (size_t)w; c < chunks.size(); c += W) {
            const int k = (int)(c % NB);
            if (e == hipSuccess && c >= (size_t)NB) e = hipEventSynchronize(R.ev[k]);
            if (e == hipSuccess) {
                const UploadPart& pt = parts[chunks[c].first];
                const size_t o = chunks[c].second, n = std::min(CH, pt.bytes - o);
                std::memcpy(R.buf[k], static_cast<const char*>(pt.src) + o, n);
                while (ticket.load(std::memory_order_acquire) != c && !failed.load(std::memory_order_relaxed))
                    std::this_thread::yield();
                e = hipMemcpyAsync(static_cast<char*>(pt.dst) + o, R.buf[k], n, hipMemcpyHostToDevice, R.st);
                if (e == hipSuccess) e = hipEventRecord(R.ev[k], R.st);
            }
            if (e != hipSuccess) failed.store(1, std::memory_order_relaxed);
            ticket.store(c + 1, std::memory_order_release);  // a failed chunk still passes the ticket on
        }
        err[w] = e;
    };
    std::vector<std::thread> helpers;
    for (int w = 1; w < W; ++w) helpers.emplace_back(work, w);
    work(0);
    for (auto& h : helpers) h.join();
    const hipError_t e = hipStreamSynchronize(R.st);
    if (tr)
        fprintf(stderr, "[upload] %d fillers, total %.2f ms\n", W,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    for (hipError_t x : err)
        if (x != hipSuccess) return x;
    return e;
}

// Device preparation (shadowtopo_prepare), one background thread per process at a time: the
// HIP runtime initialises a device lazily, at the first call that needs its queues (~85 ms on
// MI355X, measured at the first stream creation), and each of the first few streams of a
// process creates a hardware queue (~6-16 ms each); a code object loads at its first launch
// (~10 ms each).  The thread does all of it -- the staging ring (its stream is the first), a
// spare stream the next engine adopts, both code objects -- while the caller parses or
// validates the edge list.
struct Prep {
    std::mutex mu;
    std::thread th;
    int device = -1;              // the device the running or finished preparation is for
    hipStream_t spare = nullptr;  // an engine stream on `device`, adopted by the next create
    double ms = 0.0;
    ~Prep() {
        if (th.joinable()) th.join();
    }
};
Prep g_prep;

void prep_work(int device) {
    const auto t0 = std::chrono::steady_clock::now();
    if (hipSetDevice(device) == hipSuccess) {
        {
            std::lock_guard<std::mutex> lk(g_ring.mu);
            (void)ring_ensure(g_ring, device);
        }
        hipStream_t st = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) st = nullptr;
        hipFuncAttributes a;
        (void)graph_build::preload();
        (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_self<true>));
        g_prep.spare = st;  // read only after the thread is joined
    }
    g_prep.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// waits for a preparation of `device` (none running: returns at once); hands over its spare
// stream (nullptr if none) and how long it ran
hipStream_t prep_wait(int device, double* prep_ms) {
    std::lock_guard<std::mutex> lk(g_prep.mu);
    if (g_prep.th.joinable()) g_prep.th.join();
    hipStream_t st = nullptr;
    if (g_prep.device == device) {
        st = g_prep.spare;
        g_prep.spare = nullptr;
        *prep_ms = g_prep.ms;
    }
    return st;
}

}  // namespace

int shadowtopo_prepare(int32_t device) {
    if (device < 0 || device >= shadowtopo_device_count()) return fail(SHADOWTOPO_EINVAL, "device %d out of range", device);
    std::lock_guard<std::mutex> lk(g_prep.mu);
    if (g_prep.device == device && (g_prep.th.joinable() || g_prep.spare)) return SHADOWTOPO_OK;  // running or ready
    if (g_prep.th.joinable()) g_prep.th.join();
    if (g_prep.spare) {  // another device's spare stream
        (void)hipStreamDestroy(g_prep.spare);
        g_prep.spare = nullptr;
    }
    g_prep.device = device;
    g_prep.ms = 0.0;
    g_prep.th = std::thread(prep_work, device);
    return SHADOWTOPO_OK;
}

int shadowtopo_create(int32_t n_vertices, int64_t n_edges, const int32_t* edge_source, const int32_t* edge_target,
                      const double* edge_latency, const double* edge_packetloss, const double* vertex_packetloss,
                      uint32_t flags, int32_t device, shadowtopo_engine** out) {
    if (!out) return fail(SHADOWTOPO_EINVAL, "out is NULL");
    *out = nullptr;
    if (n_vertices <= 0 || n_edges < 0) return fail(SHADOWTOPO_EINVAL, "empty graph");
    if (n_edges > 0 && (!edge_source || !edge_target || !edge_latency || !edge_packetloss))
        return fail(SHADOWTOPO_EINVAL, "NULL edge array");
    const int32_t V = n_vertices;
    const bool directed = flags & SHADOWTOPO_F_DIRECTED;
    using clk = std::chrono::steady_clock;
    const auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
    auto t_phase = clk::now();
    // the device preparation runs while the edge list is validated (unless a caller started it
    // earlier); SHADOWTOPO_PRELOAD=0 (A/B knob) leaves all of it to the calls that need it
    const char* pl = getenv("SHADOWTOPO_PRELOAD");
    const bool prep = !(pl && pl[0] == '0');
    if (prep && device >= 0 && device < shadowtopo_device_count()) (void)shadowtopo_prepare(device);
    int64_t n_loops = 0;
    if (n_edges > 0) {
        const int rcv = validate_edges(V, n_edges, edge_source, edge_target, edge_latency, edge_packetloss, &n_loops);
        if (rcv) return rcv;
    }
    int ndev = shadowtopo_device_count();
    if (ndev <= 0) return fail(SHADOWTOPO_EDEVICE, "no HIP device visible");
    if (device < 0 || device >= ndev) return fail(SHADOWTOPO_EINVAL, "device %d out of range", device);
    double prep_ms = 0.0;
    const auto t_wait = clk::now();
    hipStream_t spare = prep ? prep_wait(device, &prep_ms) : nullptr;
    const double wait_ms = ms_since(t_wait);
    HIP_TRY(hipSetDevice(device));

    auto* eng = new (std::nothrow) shadowtopo_engine();
    if (!eng) {
        if (spare) (void)hipStreamDestroy(spare);
        return fail(SHADOWTOPO_ENOMEM, "engine alloc");
    }
    eng->own_stream = spare;
    if (!eng->own_stream && hipStreamCreateWithFlags(&eng->own_stream, hipStreamNonBlocking) != hipSuccess) {
        eng->own_stream = nullptr;
        shadowtopo_destroy(eng);
        return fail(SHADOWTOPO_EDEVICE, "stream create failed");
    }
    eng->st.prepare_ms = prep_ms;
    eng->st.create_prepare_wait_ms = wait_ms;
    eng->st.create_validate_ms = ms_since(t_phase);
    t_phase = clk::now();
    eng->V = V;
    eng->E = n_edges;
    eng->device = device;

    // The edge list goes to the device once; every derived table is built there
    // (graph_build.hip: stable radix sorts + segment kernels), so engine creation costs an
    // upload and a few sorts instead of host counting sorts over every arc.
    std::vector<double> vfac(V, 1.0);
    if (vertex_packetloss)
        for (int32_t v = 0; v < V; ++v)
            if (!std::isnan(vertex_packetloss[v])) vfac[v] = 1.0 - vertex_packetloss[v];
    int rc = 0;
    graph_build::Built gb;
    // the build's scratch, freed after the dense tables are allocated (graph_build.h)
    struct ScratchList {
        std::vector<void*> v;
        void release() {
            for (void* p : v) (void)hipFree(p);
            v.clear();
        }
        ~ScratchList() { release(); }
    } scratch;
    {
        int32_t *d_src = nullptr, *d_dst = nullptr;
        double *d_lat = nullptr, *d_loss = nullptr;
        const size_t ne = (size_t)std::max<int64_t>(n_edges, 1);
        // the edge buffers become the graph's igraph storage (graph_build::build works in
        // place): owned by the engine from here on
        hipError_t e = hipSuccess;
        for (auto& [p, bytes] : {std::pair<void**, size_t>{(void**)&d_src, ne * 4}, {(void**)&d_dst, ne * 4},
                                 {(void**)&d_lat, ne * 8}, {(void**)&d_loss, ne * 8}}) {
            if (e == hipSuccess) e = hipMalloc(p, bytes);
            if (e == hipSuccess) eng->graph_allocs.push_back(*p);
        }
        eng->st.create_alloc_ms = ms_since(t_phase);
        if (e == hipSuccess && n_edges > 0) {
            const size_t n = (size_t)n_edges;
            if (n * 24 >= ((size_t)64 << 20)) {  // small lists: the pageable copy's pinning is cheap
                e = upload_staged(device, {{d_src, edge_source, n * 4}, {d_dst, edge_target, n * 4},
                                           {d_lat, edge_latency, n * 8}, {d_loss, edge_packetloss, n * 8}});
            } else {
                e = hipMemcpy(d_src, edge_source, n * 4, hipMemcpyHostToDevice);
                if (e == hipSuccess) e = hipMemcpy(d_dst, edge_target, n * 4, hipMemcpyHostToDevice);
                if (e == hipSuccess) e = hipMemcpy(d_lat, edge_latency, n * 8, hipMemcpyHostToDevice);
                if (e == hipSuccess) e = hipMemcpy(d_loss, edge_packetloss, n * 8, hipMemcpyHostToDevice);
            }
        }
        eng->st.create_upload_ms = ms_since(t_phase);
        t_phase = clk::now();
        // the engine's stream builds the tables too (each further stream of a young process
        // costs a hardware queue's creation)
        hipStream_t bs = eng->own_stream;
        if (e == hipSuccess)
            e = graph_build::build(V, n_edges, n_loops, directed, CSR_PAD, d_src, d_dst, d_lat, d_loss, bs, gb,
                                   eng->graph_allocs, scratch.v);
        if (getenv("SHADOWTOPO_TRACE_BUILD")) fprintf(stderr, "[create] graph build %.2f ms\n", ms_since(t_phase));
        if (e != hipSuccess) {
            shadowtopo_destroy(eng);
            return fail(e == hipErrorOutOfMemory ? SHADOWTOPO_ENOMEM : SHADOWTOPO_EDEVICE, "graph build: %s",
                        hipGetErrorString(e));
        }
    }
    const int32_t multigraph = gb.multigraph;
    // completeness, topology.c:450-552
    if (flags & SHADOWTOPO_F_AUTO_COMPLETE)
        flags = (flags & ~SHADOWTOPO_F_COMPLETE) | (gb.complete ? SHADOWTOPO_F_COMPLETE : 0u);
    eng->flags = flags;
    eng->multigraph = multigraph;
    eng->n_arcs = gb.n_arcs;
    eng->self_blk = (directed ? n_edges : 2 * n_edges) >= 128 * (int64_t)V;
    eng->Vp = (V + 63) / 64 * 64;  // dense tiles of 64 destinations, 32-row LDS chunks
    {
        const double VV = (double)V * (double)V;
        const bool fits = (double)eng->Vp * eng->Vp * 24.0 <= 36.0e9;  // W, WR, WI, W32
        if (flags & SHADOWTOPO_F_FORCE_DENSE)
            eng->dense = fits ? 1 : 0;
        else if (flags & SHADOWTOPO_F_FORCE_CSR)
            eng->dense = 0;
        else
            eng->dense = (!(flags & SHADOWTOPO_F_COMPLETE) && fits && (double)eng->n_arcs >= 0.25 * VV) ? 1 : 0;
    }

    GraphDev& g = eng->g;
    g.V = V;
    g.Vp = eng->Vp;
    g.flags = flags;
    g.multigraph = multigraph;
    g.in_ptr = gb.in_ptr;
    g.in_src = gb.in_src;
    g.in_w = gb.in_w;
    g.in_w32 = gb.in_w32;
    g.in_r = gb.in_r;
    g.in_eid = gb.in_eid;
    g.inc_ptr = gb.inc_ptr;
    g.inc_eid = gb.inc_eid;
    g.inc_lat = gb.inc_lat;
    g.efrom = gb.efrom;
    g.eto = gb.eto;
    g.elat = gb.elat;
    g.erel = gb.erel;
    g.loop_eid = gb.loop_eid;
    eng->h_vfac = vfac;
    if ((rc = upload(eng, vfac, &g.vfac))) {
        shadowtopo_destroy(eng);
        return rc;
    }
    if (eng->dense) {
        const size_t Vp = (size_t)eng->Vp;
        double* W = nullptr;
        int32_t* WI = nullptr;
        float* W32 = nullptr;
        double* WR = nullptr;
        if ((rc = dev_alloc(eng->graph_allocs, (void**)&W, Vp * Vp * sizeof(double))) ||
            (rc = dev_alloc(eng->graph_allocs, (void**)&WR, Vp * Vp * sizeof(double))) ||
            (rc = dev_alloc(eng->graph_allocs, (void**)&WI, Vp * Vp * sizeof(int32_t))) ||
            (rc = dev_alloc(eng->graph_allocs, (void**)&W32, Vp * Vp * sizeof(float)))) {
            shadowtopo_destroy(eng);
            return rc;
        }
        if (getenv("SHADOWTOPO_TRACE_BUILD")) fprintf(stderr, "[create] dense alloc %.2f ms\n", ms_since(t_phase));
        const hipError_t e = graph_build::build_dense(eng->Vp, gb, W, WI, W32, WR, eng->own_stream);
        if (e != hipSuccess) {
            shadowtopo_destroy(eng);
            return fail(SHADOWTOPO_EDEVICE, "dense tables: %s", hipGetErrorString(e));
        }
        eng->d_W = W;
        eng->d_WI = WI;
        eng->d_WR = WR;
        eng->d_W32 = W32;
        if (getenv("SHADOWTOPO_TRACE_BUILD")) fprintf(stderr, "[create] dense tables %.2f ms\n", ms_since(t_phase));
    }
    scratch.release();
    if (getenv("SHADOWTOPO_TRACE_BUILD")) fprintf(stderr, "[create] scratch freed %.2f ms\n", ms_since(t_phase));
    // the arc heads were needed only for the dense tables
    for (auto& p : eng->graph_allocs)
        if (p == (void*)gb.arc_v) {
            (void)hipFree(p);
            p = nullptr;
        }
    if (directed) {
        g.out_ptr = gb.out_ptr;
        g.out_dst = gb.out_dst;
    } else {
        g.out_ptr = g.in_ptr;
        g.out_dst = g.in_src;
    }
    if (hipEventCreate(&eng->ev0) != hipSuccess || hipEventCreate(&eng->ev1) != hipSuccess ||
        hipEventCreate(&eng->evm) != hipSuccess || hipEventCreate(&eng->evm2) != hipSuccess ||
        hipEventCreate(&eng->ev_self[0]) != hipSuccess || hipEventCreate(&eng->ev_self[1]) != hipSuccess ||
        hipEventCreate(&eng->ev_cmp[0]) != hipSuccess || hipEventCreate(&eng->ev_cmp[1]) != hipSuccess ||
        hipEventCreateWithFlags(&eng->ev_spin, hipEventDisableTiming) != hipSuccess) {
        shadowtopo_destroy(eng);
        return fail(SHADOWTOPO_EDEVICE, "stream/event create failed");
    }
    {
        const char* tr = getenv("SHADOWTOPO_TRACE_ROUNDS");  // diagnostics: one stderr line per round
        eng->trace_rounds = tr && tr[0] == '1';
#ifdef SHADOWTOPO_EXPERIMENTS
        // A/B knobs of the experiments build (_exp/build_variant.sh), never read by the product
        const char* dd = getenv("SHADOWTOPO_DELTA_LIVE_DIV");
        if (dd && atoi(dd) > 0) eng->opt_delta_live_div = atoi(dd);
        const char* cb = getenv("SHADOWTOPO_DELTA_COLBOUND");  // A/B knob: 0, 1 or 2 (default)
        if (cb && cb[0] >= '0' && cb[0] <= '2') eng->opt_delta_colbound = cb[0] - '0';
        const char* sp = getenv("SHADOWTOPO_SWEEP_SPIRAL");  // A/B knob: 0 or 1 (default)
        if (sp && (sp[0] == '0' || sp[0] == '1')) eng->opt_sweep_spiral = sp[0] - '0';
        const char* w1 = getenv("SHADOWTOPO_SWEEP_WIN1");  // A/B knob: 0 .. 63, 8 default
        if (w1 && atoi(w1) >= 0 && atoi(w1) < 64) eng->opt_sweep_win1 = atoi(w1);
        const char* ss = getenv("SHADOWTOPO_SWEEP_SPLIT");  // A/B knob: 0 or 1 (default)
        if (ss && (ss[0] == '0' || ss[0] == '1')) eng->opt_sweep_split = ss[0] - '0';
        const char* sh = getenv("SHADOWTOPO_SWEEP_PARTS");  // A/B knob: 1 .. 4 (default 2)
        if (sh && sh[0] >= '1' && sh[0] <= '4') eng->opt_sweep_parts = sh[0] - '0';
        const char* cp = getenv("SHADOWTOPO_CHAIN_PARTS");  // A/B knob: 0 or 1 (default)
        if (cp && (cp[0] == '0' || cp[0] == '1')) eng->opt_chain_parts = cp[0] - '0';
        const char* fm = getenv("SHADOWTOPO_FUSE_MINDC");  // A/B knob: 0 or 1 (default)
        if (fm && (fm[0] == '0' || fm[0] == '1')) eng->opt_fuse_mindc = fm[0] - '0';
        const char* p0 = getenv("SHADOWTOPO_PART0_PERMILLE");  // A/B knob: part 0's share with 2 parts
        if (p0 && atoi(p0) > 0 && atoi(p0) < 1000) eng->opt_part0_permille = atoi(p0);
        const char* hs = getenv("SHADOWTOPO_HOST_SPLIT");
        if (hs && atoi(hs) > 0) eng->opt_host_split = atoi(hs);
#endif
    }
    eng->st.create_build_ms = ms_since(t_phase);
    if (getenv("SHADOWTOPO_TRACE_BUILD")) fprintf(stderr, "[create] build total %.2f ms\n", eng->st.create_build_ms);
    eng->st.n_vertices = V;
    eng->st.n_edges = n_edges;
    eng->st.n_arcs = eng->n_arcs;
    eng->st.device = device;
    eng->st.multigraph = multigraph;
    eng->st.dense = eng->dense;
    *out = eng;
    return SHADOWTOPO_OK;
}

void shadowtopo_destroy(shadowtopo_engine* eng) {
    if (!eng) return;
    (void)hipSetDevice(eng->device);
    if (eng->own_stream) (void)hipStreamSynchronize(eng->own_stream);
    if (eng->d_tlog) (void)hipFree(eng->d_tlog);
    if (eng->h_tlog) (void)hipHostFree(eng->h_tlog);
    for (auto e : eng->ev_dev) (void)hipEventDestroy(e);
    for (auto e : eng->ev_spec) (void)hipEventDestroy(e);
    if (eng->d_pk_scratch) (void)hipFree(eng->d_pk_scratch);
    free_batches(eng);
    for (void* p : eng->graph_allocs) (void)hipFree(p);
    for (void* p : eng->prune_allocs) (void)hipFree(p);
    for (void* p : eng->rp_allocs) (void)hipFree(p);
    if (eng->d_attached) (void)hipFree(eng->d_attached);
    if (eng->d_self_lat) (void)hipFree(eng->d_self_lat);
    if (eng->d_self_rel) (void)hipFree(eng->d_self_rel);
    if (eng->d_self_hops) (void)hipFree(eng->d_self_hops);
    if (eng->d_self_kind) (void)hipFree(eng->d_self_kind);
    if (eng->d_walk) (void)hipFree(eng->d_walk);
    if (eng->d_arcinfo) (void)hipFree(eng->d_arcinfo);
    for (int k = 0; k < 4; ++k)
        for (void* q : {(void*)eng->d_bweight[k], (void*)eng->d_border[k][0], (void*)eng->d_border[k][1]})
            if (q) (void)hipFree(q);
    if (eng->d_sweep_hits) (void)hipFree(eng->d_sweep_hits);
    if (eng->d_thrio) (void)hipFree(eng->d_thrio);
    if (eng->stage) (void)hipFree(eng->stage);
    if (eng->d_hitlog) (void)hipFree(eng->d_hitlog);
    if (eng->d_perm) (void)hipFree(eng->d_perm);
    if (eng->d_W32p) (void)hipFree(eng->d_W32p);
    if (eng->d_W16p) (void)hipFree(eng->d_W16p);
    if (eng->d_Wp) (void)hipFree(eng->d_Wp);
    if (eng->d_WIp) (void)hipFree(eng->d_WIp);
    if (eng->d_WRp) (void)hipFree(eng->d_WRp);
    if (eng->d_pos) (void)hipFree(eng->d_pos);
    if (eng->d_minW) (void)hipFree(eng->d_minW);
    if (eng->d_minD) (void)hipFree(eng->d_minD);
    if (eng->d_minW64) (void)hipFree(eng->d_minW64);
    if (eng->d_minDc) (void)hipFree(eng->d_minDc);
    if (eng->d_cmask) (void)hipFree(eng->d_cmask);
    if (eng->ev0) (void)hipEventDestroy(eng->ev0);
    if (eng->ev1) (void)hipEventDestroy(eng->ev1);
    if (eng->evm) (void)hipEventDestroy(eng->evm);
    if (eng->evm2) (void)hipEventDestroy(eng->evm2);
    if (eng->ev_spin) (void)hipEventDestroy(eng->ev_spin);
    for (auto e : eng->ev_self)
        if (e) (void)hipEventDestroy(e);
    for (auto e : eng->ev_cmp)
        if (e) (void)hipEventDestroy(e);
    if (eng->h_masks) (void)hipHostFree(eng->h_masks);
    if (eng->copy_stream) (void)hipStreamSynchronize(eng->copy_stream);
    for (int k = 0; k < 2; ++k) {
        if (eng->ev_comp[k]) (void)hipEventDestroy(eng->ev_comp[k]);
        if (eng->ev_copy[k]) (void)hipEventDestroy(eng->ev_copy[k]);
    }
    if (eng->copy_stream) (void)hipStreamDestroy(eng->copy_stream);
    for (int k = 0; k < 3; ++k) {
        if (eng->aux_stream[k]) (void)hipStreamDestroy(eng->aux_stream[k]);
        if (eng->ev_hp[k]) (void)hipEventDestroy(eng->ev_hp[k]);
    }
    for (auto e : eng->ev_sw)
        if (e) (void)hipEventDestroy(e);
    if (eng->ev_h0) (void)hipEventDestroy(eng->ev_h0);
    if (eng->own_stream) (void)hipStreamDestroy(eng->own_stream);
    delete eng;
}

int shadowtopo_set_attached(shadowtopo_engine* eng, const int32_t* attached, int32_t count) {
    if (!eng || count < 0 || (count > 0 && !attached)) return fail(SHADOWTOPO_EINVAL, "bad arguments");
    for (int32_t i = 0; i < count; ++i)
        if (attached[i] < 0 || attached[i] >= eng->V) return fail(SHADOWTOPO_EINVAL, "attached[%d] out of range", i);
    HIP_TRY(hipSetDevice(eng->device));
    HIP_TRY(hipStreamSynchronize(eng->own_stream));
    // the same list again (the shim sets it before every computation): keep the self paths,
    // the source order and the relaxation view
    if (eng->d_attached && count == eng->A && std::equal(attached, attached + count, eng->h_attached.begin()))
        return SHADOWTOPO_OK;
    eng->prune_ready = false;
    eng->rg = nullptr;
    const size_t n = (size_t)std::max(count, 1);
    // a new list of a size the buffers already hold reuses them (a hipFree waits for the
    // whole device; a new attach epoch pays for the rebuild of what depends on the list)
    if (n > eng->att_cap) {
        if (eng->d_attached) (void)hipFree(eng->d_attached);
        if (eng->d_self_lat) (void)hipFree(eng->d_self_lat);
        if (eng->d_self_rel) (void)hipFree(eng->d_self_rel);
        if (eng->d_self_hops) (void)hipFree(eng->d_self_hops);
        if (eng->d_self_kind) (void)hipFree(eng->d_self_kind);
        eng->d_attached = nullptr;
        eng->d_self_lat = eng->d_self_rel = nullptr;
        eng->d_self_hops = nullptr;
        eng->d_self_kind = nullptr;
        eng->att_cap = 0;
        HIP_TRY(hipMalloc((void**)&eng->d_attached, n * sizeof(int32_t)));
        HIP_TRY(hipMalloc((void**)&eng->d_self_lat, n * sizeof(double)));
        HIP_TRY(hipMalloc((void**)&eng->d_self_rel, n * sizeof(double)));
        HIP_TRY(hipMalloc((void**)&eng->d_self_hops, n * sizeof(uint32_t)));
        HIP_TRY(hipMalloc((void**)&eng->d_self_kind, n));
        eng->att_cap = n;
    }
    eng->h_attached.assign(attached, attached + count);
    eng->key_ready = false;
    eng->A = count;
    if (count > 0)
        HIP_TRY(hipMemcpy(eng->d_attached, attached, sizeof(int32_t) * count, hipMemcpyHostToDevice));
    eng->self_timed = false;
    eng->walk_ready = false;
    eng->st.n_attached = count;
    return SHADOWTOPO_OK;
}

int shadowtopo_set_option(shadowtopo_engine* eng, int32_t key, int64_t value) {
    if (!eng) return fail(SHADOWTOPO_EINVAL, "NULL engine");
    switch (key) {
        case SHADOWTOPO_OPT_BATCHES_IN_FLIGHT:
            if (value < 0 || value > 1024) return fail(SHADOWTOPO_EINVAL, "batches in flight out of range");
            eng->opt_nb = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_TIMING:
            eng->opt_timing = value ? 1 : 0;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_MAX_ROUNDS:
            eng->opt_max_rounds = value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_FORCE_REPLAY:
            eng->opt_force_replay = value ? 1 : 0;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_PROFILE:
            eng->opt_profile = value ? 1 : 0;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_DENSE_VARIANT:
            if (value != SHADOWTOPO_DENSE_F32 && value != SHADOWTOPO_DENSE_F64)
                return fail(SHADOWTOPO_EINVAL, "unknown dense variant %lld", (long long)value);
            eng->opt_dense_variant = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_DENSE_BATCHES_PER_WAVE:
            if (value != 1 && value != 2 && value != 4)
                return fail(SHADOWTOPO_EINVAL, "dense batches per wave must be 1, 2 or 4");
            eng->opt_dense_tb = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_CSR_VARIANT:
            // one sparse kernel family (k_relax / k_relax_wl / k_relax_wlp); the r01-r02
            // cross-check variants (changed-tail delta, stamped f32 keys, change records) were
            // slower on every config and are gone
            if (value != SHADOWTOPO_CSR_FULL && value != SHADOWTOPO_CSR_PUSH)
                return fail(SHADOWTOPO_EINVAL, "unknown CSR variant %lld", (long long)value);
            if (value == SHADOWTOPO_CSR_PUSH && (eng->flags & SHADOWTOPO_F_DIRECTED))
                return fail(SHADOWTOPO_EINVAL, "CSR_PUSH pushes along the in-lists: undirected graphs only");
            eng->opt_csr_variant = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_SOURCE_ORDER:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "source order must be 0 or 1");
            eng->opt_source_order = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_DENSE_PRUNE:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "dense prune must be 0 or 1");
            eng->opt_dense_prune = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_DENSE_SEED:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "dense seed must be 0 or 1");
            eng->opt_dense_seed = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_DEVICE_ROUNDS:
            if (value < 0 || value > 2) return fail(SHADOWTOPO_EINVAL, "device rounds must be 0, 1 or 2");
            eng->opt_device_rounds = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_PRUNE_PENDANT:
            if (value < 0 || value > 1) return fail(SHADOWTOPO_EINVAL, "prune must be 0 or 1");
            if (eng->opt_prune != (int32_t)value) {
                eng->opt_prune = (int32_t)value;
                eng->prune_ready = false;
                eng->rg = nullptr;
            }
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_GRID_X:
            if (value < 8 || value % 8 || value > ((int64_t)1 << 23))
                return fail(SHADOWTOPO_EINVAL, "grid x limit must be a multiple of 8 in [8, 2^23]");
            eng->opt_grid_x = value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_DENSE_W16:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "dense W16 must be 0 or 1");
            eng->opt_dense_w16 = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_CHAIN_PARTS:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "chain parts must be 0 or 1");
            eng->opt_chain_parts = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_SWEEP_PARTS:
            if (value < 1 || value > 4) return fail(SHADOWTOPO_EINVAL, "sweep parts must be 1 .. 4");
            eng->opt_sweep_parts = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_DENSE_SPEC:
            if (value < 0 || value > SPEC_MAX) return fail(SHADOWTOPO_EINVAL, "dense spec rounds must be in [0, 4]");
            eng->opt_dense_spec = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_DELTA_LIVE:
            if (value < 0 || value > 2) return fail(SHADOWTOPO_EINVAL, "delta live must be 0, 1 or 2");
            eng->opt_delta_live = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_WORKLIST:
            if (value < 0 || value > 2) return fail(SHADOWTOPO_EINVAL, "worklist must be 0, 1 or 2");
            eng->opt_worklist = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_HBM_SHARE:
            if (value < 1 || value > 1000) return fail(SHADOWTOPO_EINVAL, "HBM share must be in [1, 1000] per mille");
            eng->opt_hbm_share = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_CSR_LEAN:
            if (value < 0 || value > 2) return fail(SHADOWTOPO_EINVAL, "CSR lean must be 0, 1 or 2");
            eng->opt_csr_lean = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_HOST_GROUPS:
            if (value < 0 || value > 1024) return fail(SHADOWTOPO_EINVAL, "host groups must be in [0, 1024]");
            eng->opt_host_groups = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_SWEEP_WINDOWS:
            if (value < 0 || (value & 0xff) >= 64 || ((value >> 8) & 0xff) >= 64 || value >= (1 << 16))
                return fail(SHADOWTOPO_EINVAL, "sweep windows: bits 0-7 and 8-15 must each be in [0, 63]");
            eng->opt_sweep_win1 = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_SWEEP_GLDS:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "sweep glds must be 0 or 1");
            eng->opt_sweep_glds = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_SWEEP_WAVES:
            if (value != 4 && value != 8) return fail(SHADOWTOPO_EINVAL, "sweep waves must be 4 or 8");
            eng->opt_sweep_waves = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_DELTA_W16:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "delta w16 must be 0 or 1");
            eng->opt_delta_w16 = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_SEED_SKIP:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "seed skip must be 0 or 1");
            eng->opt_seed_skip = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_SWEEP_REFILTER:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "sweep refilter must be 0 or 1");
            eng->opt_sweep_refilter = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_SWEEP_STATS:
            eng->opt_sweep_stats = value ? 1 : 0;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_SPIN_US:
            if (value < 0 || value > 10000000) return fail(SHADOWTOPO_EINVAL, "spin must be in [0, 1e7] us");
            eng->opt_spin_us = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_SPEC_COMPOSE:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "speculative compose must be 0 or 1");
            eng->opt_spec_compose = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_CSR_INCREMENTAL:
            if (value < 0 || value > (1 << 20)) return fail(SHADOWTOPO_EINVAL, "CSR incremental must be in [0, 2^20]");
            eng->opt_csr_incremental = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_PART0_PERMILLE:
            if (value < 1 || value > 999) return fail(SHADOWTOPO_EINVAL, "part 0 share must be in [1, 999] per mille");
            eng->opt_part0_permille = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_WALK_TPW:
            if (value < 1 || value > 4) return fail(SHADOWTOPO_EINVAL, "walk shape must be 1 .. 4");
            eng->opt_walk_tpw = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_HEAVY_FIRST:
            if (value != 0 && value != 1) return fail(SHADOWTOPO_EINVAL, "heavy first must be 0 or 1");
            eng->opt_heavy_first = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_TEST_UNCONVERGED:
            eng->opt_test_unconverged = value ? 1 : 0;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_TEST_POOL_ENOMEM:
            eng->opt_test_pool_enomem = value ? 1 : 0;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_TEST_SCRAMBLE_TREE:
            if (value < 0 || value > 2) return fail(SHADOWTOPO_EINVAL, "scramble mode must be 0, 1 or 2");
            eng->opt_test_scramble = (int32_t)value;
            return SHADOWTOPO_OK;
        case SHADOWTOPO_OPT_DELTA_PERMILLE:
            if (value < 0 || value > 1000) return fail(SHADOWTOPO_EINVAL, "delta per mille must be in [0, 1000]");
            eng->opt_delta_permille = (int32_t)value;
            return SHADOWTOPO_OK;
        default:
            return fail(SHADOWTOPO_EINVAL, "unknown option %d", key);
    }
}

int shadowtopo_compute_rows(shadowtopo_engine* eng, int32_t row_begin, int32_t row_end, double* lat, double* rel,
                            uint32_t* hops, uint8_t* kind, int32_t mem, void* stream) {
    if (!eng) return fail(SHADOWTOPO_EINVAL, "NULL engine");
    if (!eng->d_attached) return fail(SHADOWTOPO_ESTATE, "shadowtopo_set_attached not called");
    if (row_begin < 0 || row_end > eng->A || row_begin > row_end) return fail(SHADOWTOPO_EINVAL, "bad row range");
    if (row_begin == row_end) return SHADOWTOPO_OK;
    if (mem != SHADOWTOPO_MEM_HOST && mem != SHADOWTOPO_MEM_DEVICE && mem != SHADOWTOPO_MEM_HOST_LR)
        return fail(SHADOWTOPO_EINVAL, "bad mem kind");
    if (!lat || (!rel) != (mem == SHADOWTOPO_MEM_HOST_LR)) return fail(SHADOWTOPO_EINVAL, "NULL output");
    HIP_TRY(hipSetDevice(eng->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : eng->own_stream;
    auto t0 = std::chrono::steady_clock::now();
    int rc = compute_rows_impl(eng, row_begin, row_end, lat, rel, hops, kind, mem, s);
    eng->st.wall_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int shadowtopo_sssp(shadowtopo_engine* eng, const int32_t* sources, int32_t n_sources, double* dist, int32_t* pred,
                    uint32_t* hops, uint8_t* tie) {
    if (!eng || n_sources < 0 || (n_sources > 0 && !sources)) return fail(SHADOWTOPO_EINVAL, "bad arguments");
    for (int32_t i = 0; i < n_sources; ++i)
        if (sources[i] < 0 || sources[i] >= eng->V) return fail(SHADOWTOPO_EINVAL, "source out of range");
    HIP_TRY(hipSetDevice(eng->device));
    hipStream_t s = eng->own_stream;
    int rc;
    eng->rg = &eng->g;  // full rows: every vertex, the unpruned graph (and pools sized for it)
    eng->lean_next = false;  // hops, predecessors and ties per vertex: the tree-fold state
    if ((rc = ensure_batches(eng, std::max(1, eng->nb_cap)))) return rc;
    const size_t V = (size_t)eng->V;
    double* d_dist = nullptr;
    int32_t* d_pred = nullptr;
    uint32_t* d_hops = nullptr;
    uint8_t* d_tie = nullptr;
    HIP_TRY(hipMalloc((void**)&d_dist, KL * V * 8));
    HIP_TRY(hipMalloc((void**)&d_pred, KL * V * 4));
    HIP_TRY(hipMalloc((void**)&d_hops, KL * V * 4));
    HIP_TRY(hipMalloc((void**)&d_tie, KL * V));
    for (int32_t i0 = 0; i0 < n_sources && rc == 0; i0 += KL) {
        const int32_t n = std::min(KL, n_sources - i0);
        for (int j = 0; j < KL; ++j) {
            eng->h_srcv[j] = j < n ? sources[i0 + j] : -1;
            eng->h_row[j] = -1;
        }
        if (hipMemcpyAsync(eng->pools.srcv, eng->h_srcv.data(), sizeof(int32_t) * KL, hipMemcpyHostToDevice, s) !=
            hipSuccess) {
            rc = fail(SHADOWTOPO_EDEVICE, "memcpy");
            break;
        }
        eng->rg = &eng->g;  // full rows: every vertex, the unpruned graph
        if ((rc = run_rounds(eng, 1, s))) break;
        hipLaunchKernelGGL(k_extract, dim3((eng->V + 255) / 256, n), dim3(256), 0, s, eng->g, eng->pools, n,
                           d_dist, d_pred, d_hops, d_tie);
        const size_t cnt = (size_t)n * V;
        const size_t o = (size_t)i0 * V;
        bool ok = hipGetLastError() == hipSuccess;
        if (ok && dist) ok = hipMemcpyAsync(dist + o, d_dist, cnt * 8, hipMemcpyDeviceToHost, s) == hipSuccess;
        if (ok && pred) ok = hipMemcpyAsync(pred + o, d_pred, cnt * 4, hipMemcpyDeviceToHost, s) == hipSuccess;
        if (ok && hops) ok = hipMemcpyAsync(hops + o, d_hops, cnt * 4, hipMemcpyDeviceToHost, s) == hipSuccess;
        if (ok && tie) ok = hipMemcpyAsync(tie + o, d_tie, cnt, hipMemcpyDeviceToHost, s) == hipSuccess;
        if (ok) ok = hipStreamSynchronize(s) == hipSuccess;
        if (!ok) rc = fail(SHADOWTOPO_EDEVICE, "sssp extract failed");
    }
    (void)hipFree(d_dist);
    (void)hipFree(d_pred);
    (void)hipFree(d_hops);
    (void)hipFree(d_tie);
    return rc;
}

// Large page-locked buffers (the shim's attached-pair matrix: C4 1.45 GB of {lat, rel}) are
// 2 MiB-aligned anonymous maps backed by transparent huge pages, then registered with the
// runtime.  Worker threads read them at random, one pair per packet: over 4 KiB pages every
// lookup is also a page walk, and page walks of 8 threads contend (a 1.45 GB random-pair read
// on the build container: 343 -> 68 ns per lookup per thread at 8 threads, 58 -> 56 at 1).
// Small buffers and a refused registration take hipHostMalloc.
namespace {
constexpr size_t kHugeAlign = size_t(2) << 20;
constexpr size_t kHugeMin = size_t(32) << 20;
std::mutex g_huge_mu;
std::vector<std::pair<void*, size_t>> g_huge;  // registered maps: base, length

void* huge_pinned(size_t bytes) {
    const size_t len = (bytes + kHugeAlign - 1) & ~(kHugeAlign - 1);
    void* raw = mmap(nullptr, len + kHugeAlign, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (raw == MAP_FAILED) return nullptr;
    const uintptr_t r = (uintptr_t)raw, a = (r + kHugeAlign - 1) & ~(uintptr_t)(kHugeAlign - 1);
    if (a > r) munmap(raw, a - r);
    if (r + len + kHugeAlign > a + len) munmap((void*)(a + len), r + len + kHugeAlign - (a + len));
    void* p = (void*)a;
    (void)madvise(p, len, MADV_HUGEPAGE);  // advisory: 4 KiB pages still work
    if (hipHostRegister(p, len, hipHostRegisterPortable) != hipSuccess) {
        (void)hipGetLastError();
        munmap(p, len);
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_huge_mu);
    g_huge.emplace_back(p, len);
    return p;
}
}  // namespace

int shadowtopo_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(SHADOWTOPO_EINVAL, "NULL argument");
    *out = nullptr;
    if (bytes >= kHugeMin && (*out = huge_pinned(bytes))) return SHADOWTOPO_OK;
    // portable: any device of the process (the shim's SHADOWTOPO_DEVICES engines) copies into it
    hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocPortable);
    if (e != hipSuccess) {
        *out = nullptr;
        return fail(SHADOWTOPO_ENOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
    }
    return SHADOWTOPO_OK;
}

void shadowtopo_host_free(void* p) {
    if (!p) return;
    size_t len = 0;
    {
        std::lock_guard<std::mutex> lk(g_huge_mu);
        for (size_t k = 0; k < g_huge.size(); k++)
            if (g_huge[k].first == p) {
                len = g_huge[k].second;
                g_huge[k] = g_huge.back();
                g_huge.pop_back();
                break;
            }
    }
    if (len) {
        (void)hipHostUnregister(p);
        munmap(p, len);
    } else {
        (void)hipHostFree(p);
    }
}

// ---------------------------------------------------------------- row exchange codec
// Multi-GPU (shard.RowExchange): every rank needs every rank's rows, and on a
// dense graph most pairs are a single arc from the source -- a value every rank can rebuild
// from its own replica of the graph.  A row block is packed as
//   header {u64 explicit pairs, u64 words} | mask[words] u64 | prefix[words] u32 (8-B padded)
//   | explicit entries {f64 lat, f64 rel, u32 hops, u32 0} in pair order
// where bit i of the mask says pair i equals pair_recon (the arc's value, below) bit for
// bit -- the packer compares, so the rebuilt value is the computed one whatever the rule
// that produced it -- and prefix[w] counts the explicit pairs before word w.  Pairs are the
// block's [rows][A] row-major order.  C2 at 8 ranks: 160 MB of rows per rank -> ~11 MB.
namespace {
constexpr int PK_WPB = 1024;  // words per scan block

struct PackHdr {
    unsigned long long n_explicit;
    unsigned long long n_words;
};

size_t pk_words(int64_t pairs) { return (size_t)((pairs + 63) / 64); }
size_t pk_mask_off() { return sizeof(PackHdr); }
size_t pk_prefix_off(size_t w) { return pk_mask_off() + w * 8; }
size_t pk_entry_off(size_t w) { return (pk_prefix_off(w) + w * 4 + 15) & ~(size_t)15; }

// the value of pair (s, t) if its path is the single arc s -> t (the dense sweep's seed
// winner): latency 0 + w, one hop, reliability vfac(s) * that arc's factor (compose's R(t)
// where the target has no vertex loss); false where there is no arc or s == t
__device__ __forceinline__ bool pair_recon(const double* __restrict__ W, const double* __restrict__ WR,
                                           const double* __restrict__ vfac, int32_t Vp, int32_t s, int32_t t,
                                           double& lat, double& rel) {
    if (s == t) return false;
    const double w = W[(size_t)s * Vp + t];
    if (!(w < dinf())) return false;
    lat = 0.0 + w;
    rel = vfac[s] * WR[(size_t)s * Vp + t];
    return true;
}

__global__ __launch_bounds__(256) void k_pack_mask(const double* __restrict__ W, const double* __restrict__ WR,
                                                   const double* __restrict__ vfac, int32_t Vp,
                                                   const int32_t* __restrict__ attached, int32_t row0, int32_t A,
                                                   int64_t pairs, const double* __restrict__ lat,
                                                   const double* __restrict__ rel, const uint32_t* __restrict__ hops,
                                                   unsigned long long* __restrict__ mask, uint32_t* __restrict__ cnt,
                                                   int64_t nwords) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwords) return;
    const int lane = threadIdx.x & 63;
    const int64_t i = w * 64 + lane;
    bool same = false;
    const bool valid = i < pairs;
    if (valid) {
        const int32_t row = (int32_t)(i / A), col = (int32_t)(i % A);
        double l, r;
        if (pair_recon(W, WR, vfac, Vp, attached[row0 + row], attached[col], l, r))
            same = hops[i] == 1u && __double_as_longlong(lat[i]) == __double_as_longlong(l) &&
                   __double_as_longlong(rel[i]) == __double_as_longlong(r);
    }
    const unsigned long long m = __ballot(same);
    const unsigned long long x = __ballot(valid && !same);
    if (lane == 0) {
        mask[w] = m;
        cnt[w] = (uint32_t)__popcll(x);
    }
}

// exclusive prefix of cnt over each block of PK_WPB words (pre), and the block totals
__global__ __launch_bounds__(256) void k_pack_scan(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ pre,
                                                   unsigned long long* __restrict__ bsum, int64_t nwords) {
    __shared__ uint32_t ws[256];
    const int64_t b0 = (int64_t)blockIdx.x * PK_WPB;
    uint32_t v[4], t = 0;
    for (int k = 0; k < 4; ++k) {
        const int64_t w = b0 + threadIdx.x * 4 + k;
        v[k] = w < nwords ? cnt[w] : 0u;
        t += v[k];
    }
    ws[threadIdx.x] = t;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive scan of the per-thread totals
        const uint32_t y = threadIdx.x >= (unsigned)o ? ws[threadIdx.x - o] : 0u;
        __syncthreads();
        ws[threadIdx.x] += y;
        __syncthreads();
    }
    uint32_t run = ws[threadIdx.x] - t;
    for (int k = 0; k < 4; ++k) {
        const int64_t w = b0 + threadIdx.x * 4 + k;
        if (w < nwords) pre[w] = run;
        run += v[k];
    }
    if (threadIdx.x == 255) bsum[blockIdx.x] = ws[255];
}

// block totals -> exclusive block offsets (one block, any count), the total into the header
__global__ __launch_bounds__(256) void k_pack_blocks(unsigned long long* __restrict__ bsum, int64_t nblk,
                                                     PackHdr* __restrict__ hdr, int64_t nwords) {
    __shared__ unsigned long long ws[256];
    unsigned long long carry = 0;
    for (int64_t c0 = 0; c0 < nblk; c0 += 256) {
        const int64_t j = c0 + threadIdx.x;
        const unsigned long long v = j < nblk ? bsum[j] : 0ull;
        ws[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) {
            const unsigned long long y = threadIdx.x >= (unsigned)o ? ws[threadIdx.x - o] : 0ull;
            __syncthreads();
            ws[threadIdx.x] += y;
            __syncthreads();
        }
        if (j < nblk) bsum[j] = carry + ws[threadIdx.x] - v;
        const unsigned long long tot = ws[255];
        __syncthreads();
        carry += tot;
    }
    if (threadIdx.x == 0) {
        hdr->n_explicit = carry;
        hdr->n_words = (unsigned long long)nwords;
    }
}

__global__ __launch_bounds__(256) void k_pack_scatter(int64_t pairs, const double* __restrict__ lat,
                                                      const double* __restrict__ rel,
                                                      const uint32_t* __restrict__ hops,
                                                      const unsigned long long* __restrict__ mask,
                                                      uint32_t* __restrict__ pre,
                                                      const unsigned long long* __restrict__ boff,
                                                      char* __restrict__ entries, int64_t nwords) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwords) return;
    const int lane = threadIdx.x & 63;
    const int64_t i = w * 64 + lane;
    const unsigned long long base = boff[w / PK_WPB] + pre[w];
    const unsigned long long m = mask[w];
    const bool expl = i < pairs && !((m >> lane) & 1ull);
    // lanes past the end are above every valid lane: ~m below a valid lane counts explicit pairs only
    const unsigned long long below = (lane ? (~0ull >> (64 - lane)) : 0ull);
    if (expl) {
        const unsigned long long k = base + (unsigned long long)__popcll(~m & below);
        char* e = entries + k * 24;
        *(double*)e = lat[i];
        *(double*)(e + 8) = rel[i];
        *(uint32_t*)(e + 16) = hops[i];
        *(uint32_t*)(e + 20) = 0u;
    }
    if (lane == 0) pre[w] = (uint32_t)base;  // the final prefix (wrapped past 2^32 pairs: guarded on the host)
}

__global__ __launch_bounds__(256) void k_unpack(const double* __restrict__ W, const double* __restrict__ WR,
                                                const double* __restrict__ vfac, int32_t Vp,
                                                const int32_t* __restrict__ attached, int32_t row0, int32_t A,
                                                int64_t pairs, const unsigned long long* __restrict__ mask,
                                                const uint32_t* __restrict__ pre, const char* __restrict__ entries,
                                                double* __restrict__ lat, double* __restrict__ rel,
                                                uint32_t* __restrict__ hops, int64_t nwords) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwords) return;
    const int lane = threadIdx.x & 63;
    const int64_t i = w * 64 + lane;
    if (i >= pairs) return;
    const unsigned long long m = mask[w];
    if ((m >> lane) & 1ull) {
        const int32_t row = (int32_t)(i / A), col = (int32_t)(i % A);
        double l = 0.0, r = 0.0;
        (void)pair_recon(W, WR, vfac, Vp, attached[row0 + row], attached[col], l, r);
        lat[i] = l;
        rel[i] = r;
        hops[i] = 1u;
    } else {
        const unsigned long long below = (lane ? (~0ull >> (64 - lane)) : 0ull);
        const unsigned long long k = (unsigned long long)pre[w] + (unsigned long long)__popcll(~m & below);
        const char* e = entries + k * 24;
        lat[i] = *(const double*)e;
        rel[i] = *(const double*)(e + 8);
        hops[i] = *(const uint32_t*)(e + 16);
    }
}
}  // namespace

size_t shadowtopo_packed_capacity(int32_t rows, int32_t A) {
    if (rows <= 0 || A <= 0) return 256;
    const int64_t pairs = (int64_t)rows * A;
    const size_t w = pk_words(pairs);
    return (pk_entry_off(w) + (size_t)pairs * 24 + 255) & ~(size_t)255;
}

int shadowtopo_pack_rows(shadowtopo_engine* eng, int32_t row_begin, int32_t row_end, const double* lat,
                         const double* rel, const uint32_t* hops, void* out, size_t cap, size_t* out_bytes,
                         void* stream) {
    if (!eng || !out || !out_bytes || row_begin < 0 || row_end > eng->A || row_begin > row_end)
        return fail(SHADOWTOPO_EINVAL, "bad arguments");
    if (!eng->dense || !eng->d_W || !eng->d_WR) return fail(SHADOWTOPO_ESTATE, "row packing needs a dense engine");
    const int32_t A = eng->A;
    const int64_t pairs = (int64_t)(row_end - row_begin) * A;
    if (pairs >= ((int64_t)1 << 32)) return fail(SHADOWTOPO_EINVAL, "row block over 2^32 pairs");
    if (cap < shadowtopo_packed_capacity(row_end - row_begin, A)) return fail(SHADOWTOPO_EINVAL, "payload buffer too small");
    if (pairs && (!lat || !rel || !hops)) return fail(SHADOWTOPO_EINVAL, "NULL rows");
    HIP_TRY(hipSetDevice(eng->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : eng->own_stream;
    const int64_t nw = (int64_t)pk_words(pairs);
    const int64_t nblk = (nw + PK_WPB - 1) / PK_WPB;
    char* o = static_cast<char*>(out);
    PackHdr* hdr = reinterpret_cast<PackHdr*>(o);
    auto* mask = reinterpret_cast<unsigned long long*>(o + pk_mask_off());
    auto* pre = reinterpret_cast<uint32_t*>(o + pk_prefix_off(nw));
    char* entries = o + pk_entry_off(nw);
    // scratch: the word counts and the block sums
    const size_t need = (size_t)nw * 4 + (size_t)(nblk + 1) * 8;
    if (eng->pk_scratch_n < need) {
        if (eng->d_pk_scratch) (void)hipFree(eng->d_pk_scratch);
        eng->d_pk_scratch = nullptr;
        eng->pk_scratch_n = 0;
        HIP_TRY(hipMalloc(&eng->d_pk_scratch, need));
        eng->pk_scratch_n = need;
    }
    auto* bsum = reinterpret_cast<unsigned long long*>(eng->d_pk_scratch);
    auto* cnt = reinterpret_cast<uint32_t*>(bsum + nblk + 1);
    if (nw > 0) {
        const uint32_t gw = (uint32_t)((nw + 3) / 4);
        hipLaunchKernelGGL(k_pack_mask, dim3(gw), dim3(256), 0, s, eng->d_W, eng->d_WR, eng->g.vfac, eng->Vp,
                           eng->d_attached, row_begin, A, pairs, lat, rel, hops, mask, cnt, nw);
        hipLaunchKernelGGL(k_pack_scan, dim3((uint32_t)nblk), dim3(256), 0, s, cnt, pre, bsum, nw);
    }
    hipLaunchKernelGGL(k_pack_blocks, dim3(1), dim3(256), 0, s, bsum, nblk, hdr, nw);
    if (nw > 0)
        hipLaunchKernelGGL(k_pack_scatter, dim3((uint32_t)((nw + 3) / 4)), dim3(256), 0, s, pairs, lat, rel, hops,
                           mask, pre, bsum, entries, nw);
    HIP_TRY(hipGetLastError());
    PackHdr h{};
    HIP_TRY(hipMemcpyAsync(&h, hdr, sizeof h, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *out_bytes = (pk_entry_off(nw) + (size_t)h.n_explicit * 24 + 255) & ~(size_t)255;
    eng->st.packed_pairs += pairs;
    eng->st.packed_explicit += (int64_t)h.n_explicit;
    return SHADOWTOPO_OK;
}

int shadowtopo_unpack_rows(shadowtopo_engine* eng, int32_t row_begin, int32_t row_end, const void* in, double* lat,
                           double* rel, uint32_t* hops, void* stream) {
    if (!eng || !in || row_begin < 0 || row_end > eng->A || row_begin > row_end)
        return fail(SHADOWTOPO_EINVAL, "bad arguments");
    if (!eng->dense || !eng->d_W || !eng->d_WR) return fail(SHADOWTOPO_ESTATE, "row unpacking needs a dense engine");
    const int32_t A = eng->A;
    const int64_t pairs = (int64_t)(row_end - row_begin) * A;
    if (pairs == 0) return SHADOWTOPO_OK;
    if (!lat || !rel || !hops) return fail(SHADOWTOPO_EINVAL, "NULL rows");
    HIP_TRY(hipSetDevice(eng->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : eng->own_stream;
    const int64_t nw = (int64_t)pk_words(pairs);
    const char* o = static_cast<const char*>(in);
    hipLaunchKernelGGL(k_unpack, dim3((uint32_t)((nw + 3) / 4)), dim3(256), 0, s, eng->d_W, eng->d_WR, eng->g.vfac,
                       eng->Vp, eng->d_attached, row_begin, A, pairs,
                       reinterpret_cast<const unsigned long long*>(o + pk_mask_off()),
                       reinterpret_cast<const uint32_t*>(o + pk_prefix_off(nw)), o + pk_entry_off(nw), lat, rel, hops,
                       nw);
    HIP_TRY(hipGetLastError());
    return SHADOWTOPO_OK;
}

// Sparse row exchange (r06, shard.RowExchange with hops16): no pair of a sparse graph's rows is
// rebuilt from the receiver's replica, so the exchange moves lat and rel in full and the hop
// counts as their low 16 bits -- 18 B per pair instead of 20.  A hop count >= 2^16 (a path
// longer than 65 535 arcs) sets the overflow word; the exchange then moves the high halves too.
namespace {
__global__ __launch_bounds__(256) void k_hops_narrow(const uint32_t* __restrict__ hops, int64_t n,
                                                     uint16_t* __restrict__ lo, uint16_t* __restrict__ hi,
                                                     uint32_t* __restrict__ overflow) {
    bool over = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t h = hops[i];
        lo[i] = (uint16_t)(h & 0xffffu);
        if (hi) hi[i] = (uint16_t)(h >> 16);
        over |= (h >> 16) != 0u;
    }
    if (__ballot(over) && (threadIdx.x & 63) == 0) atomicOr(overflow, 1u);
}

__global__ __launch_bounds__(256) void k_hops_widen(const uint16_t* __restrict__ lo, const uint16_t* __restrict__ hi,
                                                    int64_t n, uint32_t* __restrict__ hops) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        hops[i] = (uint32_t)lo[i] | (hi ? (uint32_t)hi[i] << 16 : 0u);
}

uint32_t hops_grid(int64_t n) { return (uint32_t)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192)); }
}  // namespace

int shadowtopo_hops_narrow(shadowtopo_engine* eng, const uint32_t* hops, int64_t n, uint16_t* lo, uint16_t* hi,
                           uint32_t* overflow, void* stream) {
    if (!eng || n < 0 || (n > 0 && (!hops || !lo || !overflow))) return fail(SHADOWTOPO_EINVAL, "bad arguments");
    if (n == 0) return SHADOWTOPO_OK;
    HIP_TRY(hipSetDevice(eng->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : eng->own_stream;
    hipLaunchKernelGGL(k_hops_narrow, dim3(hops_grid(n)), dim3(256), 0, s, hops, n, lo, hi, overflow);
    HIP_TRY(hipGetLastError());
    return SHADOWTOPO_OK;
}

int shadowtopo_hops_widen(shadowtopo_engine* eng, const uint16_t* lo, const uint16_t* hi, int64_t n, uint32_t* hops,
                          void* stream) {
    if (!eng || n < 0 || (n > 0 && (!lo || !hops))) return fail(SHADOWTOPO_EINVAL, "bad arguments");
    if (n == 0) return SHADOWTOPO_OK;
    HIP_TRY(hipSetDevice(eng->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : eng->own_stream;
    hipLaunchKernelGGL(k_hops_widen, dim3(hops_grid(n)), dim3(256), 0, s, lo, hi, n, hops);
    HIP_TRY(hipGetLastError());
    return SHADOWTOPO_OK;
}

int shadowtopo_self_rule_paths(shadowtopo_engine* eng, double* lat, double* rel, uint8_t* kind) {
    if (!eng || !lat || !rel || !kind) return fail(SHADOWTOPO_EINVAL, "bad arguments");
    if (!eng->d_attached) return fail(SHADOWTOPO_ESTATE, "set_attached first");
    HIP_TRY(hipSetDevice(eng->device));
    const int32_t A = eng->A;
    if (A == 0) return SHADOWTOPO_OK;
    // k_self with the version-independent rule, whatever the engine's self-pair flag
    GraphDev g = eng->g;
    g.flags &= ~SHADOWTOPO_F_SELF_DIJKSTRA_LOOP;
    void* buf = nullptr;
    HIP_TRY(hipMalloc(&buf, (size_t)A * 21));
    double* dl = (double*)buf;
    double* dr = dl + A;
    uint32_t* dh = (uint32_t*)(dr + A);
    uint8_t* dk = (uint8_t*)(dh + A);
    hipStream_t s = eng->own_stream;
    hipError_t e = launch_self(eng, g, 0, A, dl, dr, dh, dk, s);
    if (e == hipSuccess) e = hipMemcpyAsync(lat, dl, sizeof(double) * A, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(rel, dr, sizeof(double) * A, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(kind, dk, A, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(buf);
    if (e != hipSuccess) return fail(SHADOWTOPO_EDEVICE, "self-rule paths: %s", hipGetErrorString(e));
    return SHADOWTOPO_OK;
}

int shadowtopo_get_stats(const shadowtopo_engine* eng, shadowtopo_stats* out) {
    if (!eng || !out) return fail(SHADOWTOPO_EINVAL, "NULL argument");
    *out = eng->st;
    out->pruned_vertices = eng->prune_ready ? eng->pruned_vertices : 0;
    // the graph the relaxation rounds run on (the pendant-pruned view where one is in use)
    const bool view = eng->prune_ready && eng->rg == &eng->gp;
    out->relax_vertices = view ? (int64_t)eng->gp.V : (int64_t)eng->V;
    out->relax_arcs = view ? eng->gp_arcs : eng->n_arcs;
    return SHADOWTOPO_OK;
}

void shadowtopo_reset_stats(shadowtopo_engine* eng) {
    if (!eng) return;
    shadowtopo_stats keep = eng->st;
    eng->st = shadowtopo_stats{};
    eng->st.n_vertices = keep.n_vertices;
    eng->st.n_edges = keep.n_edges;
    eng->st.n_arcs = keep.n_arcs;
    eng->st.n_attached = keep.n_attached;
    eng->st.device = keep.device;
    eng->st.multigraph = keep.multigraph;
    eng->st.dense = keep.dense;
    eng->st.create_validate_ms = keep.create_validate_ms;
    eng->st.create_upload_ms = keep.create_upload_ms;
    eng->st.create_build_ms = keep.create_build_ms;
    eng->st.order_ms = keep.order_ms;
    eng->st.create_alloc_ms = keep.create_alloc_ms;
    eng->st.prepare_ms = keep.prepare_ms;
    eng->st.create_prepare_wait_ms = keep.create_prepare_wait_ms;
}

int shadowtopo_is_complete(const shadowtopo_engine* eng) {
    return eng && (eng->flags & SHADOWTOPO_F_COMPLETE) ? 1 : 0;
}

int64_t shadowtopo_get_eid(const shadowtopo_engine* eng, int32_t from, int32_t to) {
    if (!eng || from < 0 || to < 0 || from >= eng->V || to >= eng->V) return -1;
    if (ensure_mirrors(const_cast<shadowtopo_engine*>(eng))) return -1;
    if (from == to) return eng->h_loop_eid[from];
    const int64_t b = eng->h_in_ptr[to], e = eng->h_in_ptr[(size_t)to + 1];
    auto it = std::lower_bound(eng->h_in_src.begin() + b, eng->h_in_src.begin() + e, from);
    if (it == eng->h_in_src.begin() + e || *it != from) return -1;
    return eng->h_in_eid[(size_t)(it - eng->h_in_src.begin())];
}

}  // extern "C"
