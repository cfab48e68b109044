/*
 * topology_hip.h -- drop-in for Shadow's routing topology API.
 *
 * Same function names, argument meaning and error behaviour as
 * /root/reference/src/main/routing/topology.h:15-28; glib types spelled as their C
 * equivalents (gchar = char, gdouble = double, gboolean = int, guint64 = uint64_t), so a
 * Shadow build links libshadowtopo_hip.so in place of topology.c.
 *
 *   topology_new                        topology.h:17  (topology.c:2486-2510)
 *   topology_free                       topology.h:18  (topology.c:2441-2484)
 *   topology_attach                     topology.h:20  (topology.c:2371-2430)
 *   topology_detach                     topology.h:23  (topology.c:2432-2439)
 *   topology_isRoutable                 topology.h:25  (topology.c:2089-2092)
 *   topology_getLatency                 topology.h:26  (topology.c:2065-2075)
 *   topology_getReliability             topology.h:27  (topology.c:2077-2087)
 *   topology_incrementPathPacketCounter topology.h:28  (topology.c:2053-2063)
 *
 * Shadow functions this library calls (resolved from the Shadow executable at load
 * time; weak standalone defaults live in shadow_hooks.c):
 *   address_toNetworkIP      main/routing/address.h:78
 *   address_stringToIP       main/routing/address.h:94
 *   address_toHostIPString   main/routing/address.h:70
 *   address_toString         main/routing/address.h:96
 *   random_nextDouble        main/utility/random.h:42
 *   worker_updateMinTimeJump main/core/worker.h:57
 */
#ifndef SHADOWTOPO_TOPOLOGY_HIP_H
#define SHADOWTOPO_TOPOLOGY_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct _Topology Topology;
typedef struct _Address Address;
typedef struct _Random Random;

Topology* topology_new(const char* graphPath);
void topology_free(Topology* top);

void topology_attach(Topology* top, Address* address, Random* randomSourcePool, char* ipHint, char* citycodeHint,
                     char* countrycodeHint, char* geocodeHint, char* typeHint, uint64_t* bwDownOut,
                     uint64_t* bwUpOut);
void topology_detach(Topology* top, Address* address);

int topology_isRoutable(Topology* top, Address* srcAddress, Address* dstAddress);
double topology_getLatency(Topology* top, Address* srcAddress, Address* dstAddress);
double topology_getReliability(Topology* top, Address* srcAddress, Address* dstAddress);
void topology_incrementPathPacketCounter(Topology* top, Address* srcAddress, Address* dstAddress);

#ifdef __cplusplus
}
#endif

#endif
