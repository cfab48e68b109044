// graph_build.h -- device-side construction of the engine's resident graph (internal to
// libshadowtopo_hip; not part of the C ABI).  Replaces the host-side counting sorts of
// shadowtopo_create: the edge list goes to the GPU once and every derived table (the merged
// relaxation in-CSR, the out-CSR of directed graphs, igraph's incidence order, the per-vertex
// lowest self-loop, the completeness count and the dense V x V tables) is built there.
#ifndef SHADOWTOPO_GRAPH_BUILD_H
#define SHADOWTOPO_GRAPH_BUILD_H

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace graph_build {

// device arrays of the built graph, hipMalloc'd and recorded in `allocs` (the caller frees
// them); layouts are the ones engine.hip's GraphDev documents
struct Built {
    int64_t* in_ptr = nullptr;   // [V+1]
    int32_t* in_src = nullptr;   // [n_arcs + pad]
    double* in_w = nullptr;
    float* in_w32 = nullptr;
    double* in_r = nullptr;
    int32_t* in_eid = nullptr;
    int64_t n_arcs = 0;          // merged non-loop arcs (without the padding)
    int64_t* out_ptr = nullptr;  // directed only (undirected: the in-CSR)
    int32_t* out_dst = nullptr;
    int64_t* inc_ptr = nullptr;  // [V+1] igraph_incident(OUT) order
    int32_t* inc_eid = nullptr;
    double* inc_lat = nullptr;   // [inc] latency of each incidence entry (the self rule's contiguous scan)
    int32_t* efrom = nullptr;    // igraph storage: undirected from = max, to = min
    int32_t* eto = nullptr;
    double* elat = nullptr;
    double* erel = nullptr;      // 1 - packetloss
    int32_t* loop_eid = nullptr; // [V] lowest-id self-loop, -1 if none
    int32_t* arc_v = nullptr;    // [n_arcs] head of each merged arc (for the dense tables; freed by the caller)
    int32_t multigraph = 0;      // a merged run whose lowest-id edge is not its minimum latency
    int32_t complete = 0;        // _topology_isComplete's count rule (topology.c:450-552)
};

// d_src/d_dst/d_lat/d_loss: the GraphML edge list already on the device (E entries), in
// buffers the caller has recorded in `allocs`: they become the igraph storage in place
// (efrom/eto overwrite src/dst, erel overwrites packetloss, elat IS d_lat), so the build
// allocates and copies nothing for them; n_loops: self-loop edges among them (counted by
// the caller's validation pass); pad: padding arcs appended to the in-CSR (u = 0, w = +inf);
// scratch: the build's temporary device buffers, for the caller to hipFree once it has made
// its next large allocations (VRAM freed just before an allocation stalls it: the dense
// tables' allocation took 15-21 ms right after the 2.3 GB scratch of C2 was freed)
hipError_t build(int32_t V, int64_t E, int64_t n_loops, bool directed, int pad, int32_t* d_src, int32_t* d_dst,
                 double* d_lat, double* d_loss, hipStream_t s, Built& out, std::vector<void*>& allocs,
                 std::vector<void*>& scratch);

// dense tables [Vp][Vp] of the merged in-CSR, row = tail u, column = head v: W (latency,
// +inf where no arc), WI (in-arc index, -1), W32 (latency rounded toward -inf, NaN where no
// arc) and WR (the arc's reliability factor, 0 where no arc)
hipError_t build_dense(int32_t Vp, const Built& g, double* W, int32_t* WI, float* W32, double* WR, hipStream_t s);

// Loads this file's code object on the current device (the runtime does it at the first launch
// otherwise), so a caller can overlap it with host work.
hipError_t preload();

}  // namespace graph_build

#endif
