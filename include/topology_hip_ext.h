/*
 * topology_hip_ext.h -- extensions beyond Shadow's topology.h: engine configuration,
 * inspection for parity tooling, and the standalone stand-ins for the Shadow objects
 * the API takes (Address, Random), used when the library runs outside Shadow (tests,
 * bench).  Inside Shadow the real objects are passed and these constructors are unused.
 */
#ifndef SHADOWTOPO_TOPOLOGY_HIP_EXT_H
#define SHADOWTOPO_TOPOLOGY_HIP_EXT_H

#include <stdint.h>

#include "topology_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct topology_hip_info {
    int32_t n_vertices;
    int64_t n_edges;
    int32_t is_directed;
    int32_t is_complete;
    int32_t is_connected;
    int32_t cluster_count;
    int32_t prefers_direct_paths;
    int32_t n_attached;       /* unique attached vertices (sources/targets) */
    int32_t computed_for;     /* attached count the current matrix covers (0 = none) */
    int32_t device;
    double min_path_latency;  /* value handed to worker_updateMinTimeJump */
    double compute_seconds;   /* wall time of the eager attached-pair computation */
    int64_t compute_count;    /* source rows computed on the GPU */
    int32_t n_devices;        /* GPUs the attached-pair rows are sharded over */
    int32_t compute_failed;   /* 1 after a failed computation: queries fail without retrying it */
    /* the reference's path cache, emulated over the eager matrix (topology_hip.c cache_resolve) */
    int64_t dijkstra_runs;    /* _topology_computeSourcePaths calls the reference would have made */
    int64_t self_path_count;  /* _topology_computeShortestPathToSelf calls */
    int64_t cached_paths;     /* Paths in the cache */
    double self_seconds;      /* engine time of the self-path rule */
    /* IP -> vertex table read by the per-packet lookups with no lock (topology_hip.c iptab) */
    int64_t ip_table_slots;     /* slots of the live table */
    int64_t ip_tables_retired;  /* tables replaced by growth / tombstone rehash (freed with the topology) */
    int64_t ip_retired_bytes;   /* their bytes */
} topology_hip_info;

/* HIP device the engine uses (default: $SHADOWTOPO_DEVICE or 0); before the first query */
int topology_hip_set_device(Topology* top, int32_t device);
/* shard the attached-pair rows over several devices (one engine and one host thread per
 * entry; default: $SHADOWTOPO_DEVICES, e.g. "0,1,2,3,4,5,6,7"); before the first query */
int topology_hip_set_devices(Topology* top, const int32_t* devices, int32_t count);
/* alternative self-pair rule (see shadowtopo.h SHADOWTOPO_F_SELF_DIJKSTRA_LOOP) */
int topology_hip_set_self_rule(Topology* top, int32_t dijkstra_loop);
/* run the eager computation now instead of on the first query; 0 on success */
int topology_hip_prepare(Topology* top);
int topology_hip_get_info(Topology* top, topology_hip_info* out);
/* attached vertex list (vertex indices, attach order); returns count */
int32_t topology_hip_attached(Topology* top, int32_t* out, int32_t cap);
/* vertex an IP (network order) is attached to, -1 if none */
int32_t topology_hip_vertex_of_ip(Topology* top, uint32_t ip);
/* vertex index of a GraphML node id, -1 if none */
int32_t topology_hip_vertex_of_id(Topology* top, const char* id);
/* packet counter of the cached path between two attached vertices */
uint64_t topology_hip_packet_count(Topology* top, int32_t src_vertex, int32_t dst_vertex);
/* the emulated path cache's cell of an attached pair (parity / race tooling): bit 0 set when
 * (src, dst) is cached, bit 1 when (dst, src) is; both set would be a bug; -1 if unattached */
int32_t topology_hip_cached_cell(Topology* top, int32_t src_vertex, int32_t dst_vertex);
/* the parsed graph (for parity tooling): edge list + latency/packetloss, vertex loss (NaN
 * absent); arrays owned by the topology, valid until topology_free */
int topology_hip_edges(Topology* top, const int32_t** src, const int32_t** dst, const double** latency,
                       const double** packetloss, const double** vertex_packetloss);

/* standalone stand-ins for Shadow's Address / Random (shadow_hooks.c) */
Address* shadowtopo_address_new(const char* ipString, const char* name);
void shadowtopo_address_free(Address* a);
Random* shadowtopo_random_new(uint32_t seed);
void shadowtopo_random_free(Random* r);
/* last value the standalone worker_updateMinTimeJump received (-1 if never called) */
double shadowtopo_last_min_time_jump(void);
/* how many times the standalone worker_updateMinTimeJump was called */
long shadowtopo_min_time_jump_calls(void);
/* log verbosity of the standalone logger: 0 error .. 5 debug (default 3 = message) */
void shadowtopo_set_log_level(int level);

#ifdef __cplusplus
}
#endif

#endif
