/*
 * topology_hip.c -- Shadow's topology API (include/topology_hip.h) on top of the MI355X
 * engine (include/shadowtopo.h).
 *
 * Kept from the reference (/root/reference/src/main/routing/topology.c), restated in C
 * over flat arrays instead of igraph + glib:
 *   - GraphML load + validation            :371-399, :565-1210 (graphml.c, check_*)
 *   - host -> vertex attachment            :2094-2430 (find_attachment_vertex)
 *   - detach                               :2432-2439
 *   - getters / packet counter             :2053-2092
 *   - min-latency upcall                   :1374-1385
 *   - teardown logging                     :1266-1282, :1929-1967, path.c:62-75
 * Replaced: the lazy per-source igraph Dijkstra and the two-level GHashTable path cache
 * (:1284-1386, :1545-1927, :1969-2051).  On the first query (a worker thread, as in the
 * reference) the engine computes the whole attached-pair matrix once, eagerly, on the
 * GPU; after that every lookup is two array reads.  Pairs follow the canonical
 * ordered-pair rule of SURVEY.md 8.0 (the value the reference stores for (s,t) when s's
 * own computation runs first).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <math.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <sys/mman.h>
#include <time.h>

#include "graphml.h"
#include "shadowtopo.h"
#include "shim_log.h"
#include "topology_hip.h"
#include "topology_hip_ext.h"

/* Shadow functions (strong in Shadow, weak stand-ins in shadow_hooks.c) */
extern uint32_t address_toNetworkIP(Address* address);
extern in_addr_t address_stringToIP(const char* ipString);
extern char* address_toHostIPString(Address* address);
extern char* address_toString(Address* address);
extern double random_nextDouble(Random* random);
extern void worker_updateMinTimeJump(double minPathLatency);

#define TOPO_MAGIC 0x70B01060u
#define SHADOWTOPO_MAX_DEVICES 64

/* ------------------------------------------------------------ IP -> vertex table
 * virtualIP (topology.c:42-47, 1388-1405), read by the per-packet lookups with no lock
 * (SURVEY.md 8(f)3).  Every slot is ONE 64-bit word, ip << 32 | tag (tag 0: empty;
 * vertex + 1: live; IPT_DEAD: deleted), written by attach / detach under ip_lock (writer)
 * with a release store and read with an acquire load, so a lookup never sees a torn entry
 * and a detach costs one store (no rebuild).  Growth, and the rehash that drops tombstones,
 * builds a new table, publishes it with a release store and retires the old one, which a
 * lookup that loaded the old pointer may still be probing: retired tables are freed with the
 * topology.  What they hold is bounded: a table retired by growth is half the size of its
 * successor (all of them together < the live table), and a rehash at the same size needs
 * cap / 4 detaches since the last one (at most 32 bytes retained per detach). */
#define IPT_DEAD 0xFFFFFFFFu

typedef struct iptab {
    size_t cap;          /* slots, a power of two */
    size_t used, live;   /* writer-side counts (ip_lock): non-empty slots, live entries */
    struct iptab* next;  /* retired tables */
    _Atomic uint64_t slot[];
} iptab;

static size_t ip_slot(uint32_t ip, size_t cap) {
    uint64_t h = (uint64_t)ip * 0x9E3779B97F4A7C15ULL;
    return (size_t)(h >> 20) & (cap - 1);
}

static iptab* ipt_alloc(size_t cap) {
    iptab* t = calloc(1, sizeof(iptab) + cap * sizeof(uint64_t));
    if (t) t->cap = cap;
    return t;
}

/* lookups (any thread, no lock) */
static int32_t ipt_get(const iptab* t, uint32_t ip) {
    if (!t) return -1;
    for (size_t j = ip_slot(ip, t->cap);; j = (j + 1) & (t->cap - 1)) {
        const uint64_t w = atomic_load_explicit(&t->slot[j], memory_order_acquire);
        if (w == 0) return -1;
        const uint32_t tag = (uint32_t)w;
        if ((uint32_t)(w >> 32) == ip && tag != IPT_DEAD) return (int32_t)(tag - 1);
    }
}

/* writers hold ip_lock.  A table with room for one more entry (at most half its slots
 * non-empty): the current one, or a fresh one (twice the size when the live entries need
 * it) that replaces it */
static iptab* ipt_room(_Atomic(iptab*)* live, iptab** retired, size_t* nretired) {
    iptab* t = atomic_load_explicit(live, memory_order_relaxed);
    if (t && (t->used + 1) * 2 <= t->cap) return t;
    size_t cap = t ? t->cap : 256;
    while ((t ? t->live + 1 : 1) * 4 > cap) cap *= 2;
    iptab* n = ipt_alloc(cap);
    if (!n) return NULL;
    for (size_t i = 0; t && i < t->cap; i++) {
        const uint64_t w = atomic_load_explicit(&t->slot[i], memory_order_relaxed);
        if (w == 0 || (uint32_t)w == IPT_DEAD) continue;
        size_t j = ip_slot((uint32_t)(w >> 32), cap);
        while (atomic_load_explicit(&n->slot[j], memory_order_relaxed)) j = (j + 1) & (cap - 1);
        atomic_store_explicit(&n->slot[j], w, memory_order_relaxed);
        n->used++;
        n->live++;
    }
    atomic_store_explicit(live, n, memory_order_release);
    if (t) {
        t->next = *retired;
        *retired = t;
        (*nretired)++;
    }
    return n;
}

static int ipt_put(_Atomic(iptab*)* live, iptab** retired, size_t* nretired, uint32_t ip, int32_t v) {
    /* g_hash_table_replace */
    iptab* t = ipt_room(live, retired, nretired);
    if (!t) return -1;
    const uint64_t want = ((uint64_t)ip << 32) | (uint32_t)(v + 1);
    size_t tomb = (size_t)-1, j = ip_slot(ip, t->cap);
    for (;; j = (j + 1) & (t->cap - 1)) {
        const uint64_t w = atomic_load_explicit(&t->slot[j], memory_order_relaxed);
        if (w == 0) break;
        if ((uint32_t)w == IPT_DEAD) {
            if (tomb == (size_t)-1) tomb = j;
        } else if ((uint32_t)(w >> 32) == ip) {
            atomic_store_explicit(&t->slot[j], want, memory_order_release);
            return 0;
        }
    }
    if (tomb != (size_t)-1) j = tomb;
    else t->used++;
    atomic_store_explicit(&t->slot[j], want, memory_order_release);
    t->live++;
    return 0;
}

static void ipt_del(_Atomic(iptab*)* live, uint32_t ip) {
    iptab* t = atomic_load_explicit(live, memory_order_relaxed);
    if (!t) return;
    for (size_t j = ip_slot(ip, t->cap);; j = (j + 1) & (t->cap - 1)) {
        const uint64_t w = atomic_load_explicit(&t->slot[j], memory_order_relaxed);
        if (w == 0) return;
        if ((uint32_t)w != IPT_DEAD && (uint32_t)(w >> 32) == ip) {
            atomic_store_explicit(&t->slot[j], ((uint64_t)ip << 32) | IPT_DEAD, memory_order_release);
            t->live--;
            return;
        }
    }
}

/* ------------------------------------------------------------ state */
/* the attached-pair matrix: latency, reliability and pair kind (the API never exposes hop
 * counts, so they are not copied out); page-locked when the engine can provide it, so the
 * device rows arrive at full PCIe rate, a batch group's copy behind the next group's
 * computation (shadowtopo_host_alloc) */
typedef struct matrix {
    int32_t A;
    int pinned;
    double* lr;     /* {latency, reliability} per pair, interleaved (SHADOWTOPO_MEM_HOST_LR): a
                     * packet's getLatency and getReliability read one cache line */
    uint8_t* kind;
    /* undirected late attach: rows [0, partial) hold the reverse-direction entries in
     * columns >= fill_col until an old source's own row is needed (fill_old_rows rewrites
     * columns [fill_col, A) of those rows in place, then stores 0 here with release order).
     * fill_col = partial after one late attach; after several without a fill in between it
     * is the first unfilled column of the oldest unfilled matrix (those rows were copied
     * from it, reverse copies included) */
    _Atomic int32_t partial;
    int32_t fill_col;
    /* self_rule (the [s]-path igraph): the matrix diagonal holds the [s] path's value; these
     * hold the version-independent self-path rule's per attached index, which a self pair
     * takes when a query (s, s) cached it before s's Dijkstra did (else NULL) */
    double* srl_lat;
    double* srl_rel;
    uint8_t* srl_kind;
    struct matrix* next; /* retired matrices (readers may still hold them) */
} matrix;

/* ascending vertex list of one attach queue and how many of its vertices carry a usable IP */
typedef struct {
    int32_t* v;
    int32_t n, cap, nips;
} vlist;

/* string (lowercased) -> vlist */
typedef struct {
    char** keys;
    int32_t* vals;
    size_t cap, n;
    vlist* lists;
    int32_t nlists, caplists;
} strmap;

/* uint32 -> vlist */
typedef struct {
    uint32_t* keys;
    int32_t* vals; /* list index + 1, 0 = empty */
    size_t cap, n;
    vlist* lists;
    int32_t nlists, caplists;
} u32map;

/* attach hint indexes, built on the first attach */
typedef struct {
    in_addr_t* vip;      /* [V] address_stringToIP of the "ip" value ("" when absent): the LPM key */
    uint8_t* usable;     /* [V] ip attribute present and not NONE / ANY / LOOPBACK */
    int32_t nips_all;    /* vertices with a usable IP */
    strmap city, country, geo, type, city_type, country_type, geo_type;
    u32map exact;        /* usable IP -> vertices */
    int32_t (*trie)[2];  /* binary trie over vip[] (bit 31 first); leaves hold the first vertex */
    int32_t* leaf;
    int32_t ntrie, captrie;
} attach_index;

#define CTILE 64 /* packet counters: 64 x 64 tiles, allocated on first touch */

struct arena_slab;
typedef struct {
    pthread_mutex_t mu;
    struct arena_slab* head;
    size_t off;
} tile_arena;

struct _Topology {
    uint32_t magic;
    gml_graph* gml;
    int32_t V;
    int64_t E;
    int directed, complete, connected, clusters, prefer_direct;
    double* elat;  /* edge latency (ms) */
    double* eloss; /* edge packetloss */
    double* vloss; /* vertex packetloss, NaN = absent */
    const gml_attr *a_ip, *a_city, *a_country, *a_geo, *a_type, *a_bwdown, *a_bwup, *a_asn, *a_vloss;
    pthread_rwlock_t ip_lock; /* writers: attach / detach; readers: the attached list */
    _Atomic(iptab*) ips;      /* read with no lock (ipt_get) */
    iptab* ips_retired;
    size_t ips_nretired;
    _Atomic int32_t* att_index; /* [V] attached index or -1 (verticesWithAttachedHosts) */
    int32_t* attached;
    int32_t n_att, cap_att;
    pthread_mutex_t idx_lock;
    attach_index* aidx;
    pthread_mutex_t compute_lock;
    _Atomic(matrix*) mat;
    matrix* retired;
    int compute_failed; /* a failed computation is not retried (queries fail fast) */
    /* per-pair packet counters, keyed by attached indices (stable across late attaches):
     * crow[i / 64] -> [ctd] tile pointers -> 64 x 64 u64 (count + 1 once touched) */
    int32_t ctd;
    _Atomic(_Atomic(uint64_t*)*)* crow;
    tile_arena tiles; /* the counter and cache-cell tiles (arena_alloc) */
    shadowtopo_engine* eng;  /* engine on devices[0] */
    int32_t device;
    /* in-process multi-GPU: one engine per device, each computing a
     * contiguous block of source rows straight into the host matrix */
    int32_t ndev;
    int32_t devices[SHADOWTOPO_MAX_DEVICES];
    shadowtopo_engine* engs[SHADOWTOPO_MAX_DEVICES];
    /* the reference's path cache as a set of attached pairs (cache_resolve): bit j % 64 of
     * word i % 64 in the 64 x 64 tile (i / 64, j / 64), allocated on first store */
    _Atomic(_Atomic(uint64_t*)*)* srow;
    /* per attached source: the matrix size its Dijkstra store loop last ran for (one loop
     * per source and target list: concurrent misses on the same source claim their own pair
     * instead of repeating the O(A) loop) */
    _Atomic int32_t* src_loop;
    pthread_mutex_t min_lock; /* minimumPathLatency (the reference's pathCacheLock writer side) */
    int self_rule;
    double min_latency;
    double compute_s;
    int64_t compute_count;          /* source rows computed on the GPU */
    _Atomic int64_t dijkstra_runs;  /* _topology_computeSourcePaths calls the reference would make */
    _Atomic int64_t self_count;     /* _topology_computeShortestPathToSelf calls */
    _Atomic int64_t cached_paths;   /* Paths in the emulated cache */
};
/* ------------------------------------------------------------ attribute helpers
 * _topology_find{Vertex,Edge,Graph}Attribute{String,Double} (topology.c:284-369): a value
 * counts only if the attribute exists (exact name) and is non-empty / not NaN. */
static int vstr(const Topology* top, const gml_attr* a, int32_t v, const char** out) {
    (void)top;
    if (!a) return 0;
    const char* s = gml_str(a, v);
    if (!s || !s[0]) return 0;
    if (out) *out = s;
    return 1;
}

static int vnum(const gml_attr* a, int64_t i, double* out) {
    if (!a || a->type == GML_STRING) return 0;
    double x = gml_num(a, i);
    if (isnan(x)) return 0;
    if (out) *out = x;
    return 1;
}

static const char* vid(const Topology* top, int32_t v) { return top->gml->node_ids[v]; }

static const char* type_name(int t) {
    return t == GML_NUMERIC ? "NUMERIC" : t == GML_STRING ? "STRING" : t == GML_BOOLEAN ? "BOOLEAN" : "UNKOWN";
}

/* _topology_checkAttributeType, topology.c:554-563 */
static int check_type(const char* name, int parsed, int required) {
    if (parsed == required) {
        st_info("graph attribute '%s' with type '%s' is supported", name, type_name(parsed));
        return 1;
    }
    st_warning("graph attribute '%s' with type '%s' is supported, but we found unsupported type '%s'", name,
               type_name(required), type_name(parsed));
    return 0;
}

/* case-insensitive prefix match of the reference's attribute keys (topology.c:193-282) */
static int key_is(const char* name, const char* want, size_t len) { return strncasecmp(name, want, len) == 0; }

/* _topology_checkGraphAttributes, topology.c:565-722 -- note the reference ASSIGNS the
 * result of each type check (isSuccess = ...), so the last recognised attribute of each
 * loop decides; restated literally. */
static int check_attributes(Topology* top) {
    const gml_graph* g = top->gml;
    int ok = 1;
    st_message("checking graph attributes...");
    for (int i = 0; i < g->nattr; i++) {
        const gml_attr* a = &g->attrs[i];
        if (a->domain != GML_GRAPH) continue;
        if (key_is(a->name, "preferdirectpaths", 17))
            ok = check_type(a->name, a->type, GML_STRING);
        else
            st_warning("graph attribute '%s' is unsupported and will be ignored", a->name);
    }
    /* vertex attributes: the keys in order, then igraph's own "id" string attribute */
    for (int i = 0; i <= g->nattr; i++) {
        const char* name;
        int type;
        if (i < g->nattr) {
            if (g->attrs[i].domain != GML_NODE) continue;
            name = g->attrs[i].name;
            type = g->attrs[i].type;
        } else {
            name = "id";
            type = GML_STRING;
        }
        if (key_is(name, "id", 2) || key_is(name, "ip", 2) || key_is(name, "citycode", 8) ||
            key_is(name, "countrycode", 11) || key_is(name, "type", 4))
            ok = check_type(name, type, GML_STRING);
        else if (key_is(name, "asn", 3) || key_is(name, "bandwidthdown", 13) || key_is(name, "bandwidthup", 11) ||
                 key_is(name, "packetloss", 10))
            ok = check_type(name, type, GML_NUMERIC);
        else if (key_is(name, "geocode", 7)) {
            ok = check_type(name, type, GML_STRING);
            st_warning("vertex attribute '%s' has been renamed to 'countrycode' and is considered deprecated; "
                       "please use 'countrycode' and/or 'citycode' instead", name);
        } else
            st_info("vertex attribute '%s' is unsupported and will be ignored", name);
    }
    if (g->n == 0) { /* igraph adds the "id" attribute only when there are vertices */
        st_warning("the vertex attribute 'id' of type 'STRING' is required but not provided");
        ok = 0;
    }
    if (!gml_find(g, GML_NODE, "bandwidthdown")) {
        st_warning("the vertex attribute 'bandwidthdown' of type 'NUMERIC' is required but not provided");
        ok = 0;
    }
    if (!gml_find(g, GML_NODE, "bandwidthup")) {
        st_warning("the vertex attribute 'bandwidthup' of type 'NUMERIC' is required but not provided");
        ok = 0;
    }
    for (int i = 0; i < g->nattr; i++) {
        const gml_attr* a = &g->attrs[i];
        if (a->domain != GML_EDGE) continue;
        if (key_is(a->name, "latency", 7) || key_is(a->name, "jitter", 6) || key_is(a->name, "packetloss", 10))
            ok = check_type(a->name, a->type, GML_NUMERIC);
        else
            st_info("edge attribute '%s' is unsupported and will be ignored", a->name);
    }
    if (!gml_find(g, GML_EDGE, "latency")) {
        st_warning("the edge attribute 'latency' of type 'NUMERIC' is required but not provided");
        ok = 0;
    }
    if (!gml_find(g, GML_EDGE, "packetloss")) {
        st_warning("the edge attribute 'packetloss' of type 'NUMERIC' is required but not provided");
        ok = 0;
    }
    if (ok)
        st_message("successfully verified all graph, vertex, and edge attributes");
    else
        st_warning("we could not properly validate all graph, vertex, and edge attributes");
    return ok;
}

/* igraph_is_connected / igraph_clusters (mode STRONG), topology.c:738-749 */
static void connectivity(Topology* top) {
    const int32_t V = top->V;
    const int64_t E = top->E;
    const gml_graph* g = top->gml;
    if (V == 0) {
        top->connected = 0;
        top->clusters = 0;
        return;
    }
    /* forward and reverse CSR */
    int64_t* fp = calloc((size_t)V + 1, sizeof(int64_t));
    int64_t* rp = calloc((size_t)V + 1, sizeof(int64_t));
    int32_t* fa = malloc(sizeof(int32_t) * (size_t)(2 * E + 1));
    int32_t* ra = malloc(sizeof(int32_t) * (size_t)(2 * E + 1));
    for (int64_t e = 0; e < E; e++) {
        fp[g->src[e] + 1]++;
        rp[g->dst[e] + 1]++;
        if (!top->directed) {
            fp[g->dst[e] + 1]++;
            rp[g->src[e] + 1]++;
        }
    }
    for (int32_t v = 0; v < V; v++) {
        fp[v + 1] += fp[v];
        rp[v + 1] += rp[v];
    }
    int64_t* ff = malloc(sizeof(int64_t) * (size_t)V);
    int64_t* rf = malloc(sizeof(int64_t) * (size_t)V);
    memcpy(ff, fp, sizeof(int64_t) * (size_t)V);
    memcpy(rf, rp, sizeof(int64_t) * (size_t)V);
    for (int64_t e = 0; e < E; e++) {
        fa[ff[g->src[e]]++] = g->dst[e];
        ra[rf[g->dst[e]]++] = g->src[e];
        if (!top->directed) {
            fa[ff[g->dst[e]]++] = g->src[e];
            ra[rf[g->src[e]]++] = g->dst[e];
        }
    }
    /* Kosaraju: iterative DFS finish order on the forward graph, then reverse sweeps */
    int32_t* order = malloc(sizeof(int32_t) * (size_t)V);
    int32_t* stack = malloc(sizeof(int32_t) * (size_t)V);
    int64_t* it = malloc(sizeof(int64_t) * (size_t)V);
    uint8_t* seen = calloc((size_t)V, 1);
    int32_t no = 0;
    for (int32_t r = 0; r < V; r++) {
        if (seen[r]) continue;
        int32_t sp = 0;
        stack[sp++] = r;
        seen[r] = 1;
        it[r] = fp[r];
        while (sp) {
            int32_t v = stack[sp - 1];
            if (it[v] < fp[v + 1]) {
                int32_t w = fa[it[v]++];
                if (!seen[w]) {
                    seen[w] = 1;
                    it[w] = fp[w];
                    stack[sp++] = w;
                }
            } else {
                order[no++] = v;
                sp--;
            }
        }
    }
    int32_t* comp = malloc(sizeof(int32_t) * (size_t)V);
    for (int32_t v = 0; v < V; v++) comp[v] = -1;
    int32_t nc = 0;
    for (int32_t k = V - 1; k >= 0; k--) {
        int32_t r = order[k];
        if (comp[r] >= 0) continue;
        int32_t sp = 0;
        stack[sp++] = r;
        comp[r] = nc;
        while (sp) {
            int32_t v = stack[--sp];
            for (int64_t x = rp[v]; x < rp[v + 1]; x++) {
                int32_t w = ra[x];
                if (comp[w] < 0) {
                    comp[w] = nc;
                    stack[sp++] = w;
                }
            }
        }
        nc++;
    }
    top->clusters = nc;
    top->connected = (nc == 1);
    free(fp);
    free(rp);
    free(fa);
    free(ra);
    free(ff);
    free(rf);
    free(order);
    free(stack);
    free(it);
    free(seen);
    free(comp);
}

/* lowest-id self-loop per vertex (igraph_get_eid(v, v)) */
static int32_t* loop_edges(const Topology* top) {
    int32_t* le = malloc(sizeof(int32_t) * (size_t)top->V);
    for (int32_t v = 0; v < top->V; v++) le[v] = -1;
    for (int64_t e = top->E - 1; e >= 0; e--)
        if (top->gml->src[e] == top->gml->dst[e]) le[top->gml->src[e]] = (int32_t)e;
    return le;
}

/* _topology_isComplete, topology.c:450-552 */
static int is_complete(const Topology* top) {
    const int32_t V = top->V;
    int64_t* deg = calloc((size_t)V, sizeof(int64_t));
    for (int64_t e = 0; e < top->E; e++) {
        deg[top->gml->src[e]]++; /* OUT-incident (directed: tail) */
        if (!top->directed) deg[top->gml->dst[e]]++;
    }
    int32_t* le = loop_edges(top);
    int complete = 1;
    for (int32_t v = 0; v < V && complete; v++) {
        int64_t ecount = deg[v];
        if (!top->directed && le[v] >= 0) ecount -= 1;
        if (ecount < V) {
            st_info("Vert id=%ld has %ld incident edges to %ld total verts and thus this isn't a complete graph",
                    (long)v, (long)ecount, (long)V);
            complete = 0;
        }
    }
    if (complete) st_info("Determined this graph is complete.");
    free(deg);
    free(le);
    return complete;
}

/* _topology_checkGraphProperties, topology.c:724-809 */
static int check_properties(Topology* top) {
    st_message("checking graph properties...");
    if (!check_attributes(top)) {
        st_critical("topology validation failed because of problem with graph, vertex, or edge attributes");
        return 0;
    }
    connectivity(top);
    top->complete = is_complete(top);
    int prefer = 0;
    const gml_attr* pa = gml_find(top->gml, GML_GRAPH, "preferdirectpaths");
    if (pa && pa->type != GML_STRING) {
        /* the reference reaches igraph_cattribute_GAS on a non-string attribute here
         * (topology.c:292-293), which igraph's default error handler aborts on */
        st_critical("graph attribute 'preferdirectpaths' must be a string");
        return 0;
    }
    if (pa) {
        const char* value = gml_str(pa, 0);
        if (value && value[0]) {
            int yes = !strncasecmp(value, "true", 4) || !strncasecmp(value, "yes", 3) || !strncasecmp(value, "1", 1);
            if (yes) {
                st_message("If a direct path between any pair of nodes exists, Shadow will prefer it over shortest "
                           "path.");
                prefer = 1;
            } else {
                st_message("Shadow will always use shortest path between a pair of nodes, even if a direct path "
                           "exists (to override, set 'preferdirectpaths' to 'yes' or 'true' or '1' to enable)");
            }
        }
    }
    top->prefer_direct = prefer;
    st_message("topology graph is %s, %s, and %s with %u %s. It does%s prefer direct paths.",
               top->complete ? "complete" : "incomplete", top->directed ? "directed" : "undirected",
               top->connected ? "strongly connected" : "disconnected", (unsigned)top->clusters,
               top->clusters == 1 ? "cluster" : "clusters", top->prefer_direct ? "" : " not");
    if (!top->connected || top->clusters > 1) {
        st_critical("topology must be strongly connected with a single cluster; it is %sconnected with %i cluster%s",
                    top->connected ? "" : "dis", top->clusters, top->clusters == 1 ? "" : "s");
        return 0;
    }
    return 1;
}

/* _topology_checkGraphVerticesHelperHook, topology.c:811-978 */
static int check_vertices(Topology* top) {
    st_message("checking graph vertices...");
    int all_ok = 1;
    for (int32_t v = 0; v < top->V; v++) {
        int ok = 1;
        const char* id = vid(top, v);
        if (!id || !id[0]) {
            st_warning("required attribute 'id' on vertex %li is NULL", (long)v);
            ok = 0;
            id = "NULL";
        }
        double x;
        if (!top->a_bwdown) {
            st_warning("required attribute 'bandwidthdown' on vertex %li (id='%s') is missing", (long)v, id);
            ok = 0;
        } else if (!(vnum(top->a_bwdown, v, &x) && x > 0.0)) {
            st_warning("required attribute 'bandwidthdown' on vertex %li (id='%s') is NAN or negative", (long)v, id);
            ok = 0;
        }
        if (!top->a_bwup) {
            st_warning("required attribute 'bandwidthup' on vertex %li (id='%s') is missing", (long)v, id);
            ok = 0;
        } else if (!(vnum(top->a_bwup, v, &x) && x > 0.0)) {
            st_warning("required attribute 'bandwidthup' on vertex %li (id='%s') is NAN or negative", (long)v, id);
            ok = 0;
        }
        if (top->a_asn && vnum(top->a_asn, v, &x) && !(x > 0.0)) {
            st_warning("optional attribute 'asn' on vertex %li (id='%s') is non-positive", (long)v, id);
            ok = 0;
        }
        if (top->a_vloss && vnum(top->a_vloss, v, &x) && !(x >= 0.0 && x <= 1.0)) {
            st_warning("optional attribute 'packetloss' on vertex %li (id='%s') is out of range [0.0,1.0]", (long)v,
                       id);
            ok = 0;
        }
        if (!ok) all_ok = 0;
    }
    if (!all_ok) {
        st_warning("we had a problem validating vertex attributes");
        st_warning("unable to validate graph vertices");
        return 0;
    }
    st_message("%u graph vertices ok", (unsigned)top->V);
    return 1;
}

/* _topology_checkGraphEdgesHelperHook, topology.c:1041-1124 */
static int check_edges(Topology* top) {
    st_message("checking graph edges...");
    const gml_attr* al = gml_find(top->gml, GML_EDGE, "latency");
    const gml_attr* ap = gml_find(top->gml, GML_EDGE, "packetloss");
    const gml_attr* aj = gml_find(top->gml, GML_EDGE, "jitter");
    int all_ok = 1;
    for (int64_t e = 0; e < top->E; e++) {
        const char* from = vid(top, top->gml->src[e]);
        const char* to = vid(top, top->gml->dst[e]);
        double x;
        if (al && vnum(al, e, &x)) {
            if (!(x > 0.0)) {
                st_warning("required attribute 'latency' on edge %li (from '%s' to '%s') is non-positive", (long)e,
                           from, to);
                all_ok = 0;
            } else if (isinf(x)) {
                /* deviation: the reference accepts +inf here (topology.c:1066-1082); the engine
                 * needs finite latencies, so the graph fails at load time, not at the first query */
                st_warning("required attribute 'latency' on edge %li (from '%s' to '%s') is infinite", (long)e, from,
                           to);
                all_ok = 0;
            }
        } else {
            st_warning("required attribute 'latency' on edge %li (from '%s' to '%s') is missing or NAN", (long)e,
                       from, to);
            all_ok = 0;
        }
        if (ap && vnum(ap, e, &x)) {
            if (!(x >= 0.0 && x <= 1.0)) {
                st_warning("required attribute 'packetloss' on edge %li (from '%s' to '%s') is out of range [0.0,1.0]",
                           (long)e, from, to);
                all_ok = 0;
            }
        } else {
            st_warning("required attribute 'packetloss' on edge %li (from '%s' to '%s') is missing or NAN", (long)e,
                       from, to);
            all_ok = 0;
        }
        if (aj && vnum(aj, e, &x) && !(x >= 0.0)) {
            st_warning("optional attribute 'jitter' on edge %li (from '%s' to '%s') is negative", (long)e, from, to);
            all_ok = 0;
        }
    }
    if (!all_ok) {
        st_warning("we had a problem validating edge attributes");
        st_warning("unable to validate graph edges");
        return 0;
    }
    st_message("%u graph edges ok", (unsigned)top->E);
    return 1;
}

/* _topology_extractEdgeWeights (topology.c:1212-1246) + the per-vertex loss column */
static int extract(Topology* top) {
    const gml_attr* al = gml_find(top->gml, GML_EDGE, "latency");
    const gml_attr* ap = gml_find(top->gml, GML_EDGE, "packetloss");
    top->elat = malloc(sizeof(double) * (size_t)(top->E ? top->E : 1));
    top->eloss = malloc(sizeof(double) * (size_t)(top->E ? top->E : 1));
    top->vloss = malloc(sizeof(double) * (size_t)top->V);
    if (!top->elat || !top->eloss || !top->vloss) return 0;
    for (int64_t e = 0; e < top->E; e++) {
        top->elat[e] = gml_num(al, e);
        top->eloss[e] = gml_num(ap, e);
    }
    for (int32_t v = 0; v < top->V; v++) {
        double x;
        top->vloss[v] = vnum(top->a_vloss, v, &x) ? x : NAN;
    }
    return 1;
}

/* ------------------------------------------------------------ lifecycle */
static void mat_free(const matrix* m, void* p) {
    if (m->pinned)
        shadowtopo_host_free(p);
    else
        free(p);
}

static void free_matrix(matrix* m) {
    if (!m) return;
    mat_free(m, m->lr);
    mat_free(m, m->kind);
    free(m->srl_lat);
    free(m->srl_rel);
    free(m->srl_kind);
    free(m);
}

static void vl_push(vlist* l, int32_t v, int usable) {
    if (l->n == l->cap) {
        l->cap = l->cap ? l->cap * 2 : 8;
        l->v = realloc(l->v, sizeof(int32_t) * (size_t)l->cap);
    }
    l->v[l->n++] = v;
    if (usable) l->nips++;
}

static void strmap_free(strmap* m) {
    for (size_t i = 0; i < m->cap; i++) free(m->keys[i]);
    free(m->keys);
    free(m->vals);
    for (int32_t k = 0; k < m->nlists; k++) free(m->lists[k].v);
    free(m->lists);
}

static void free_index(attach_index* x) {
    if (!x) return;
    free(x->vip);
    free(x->usable);
    strmap* maps[] = {&x->city, &x->country, &x->geo, &x->type, &x->city_type, &x->country_type, &x->geo_type};
    for (size_t k = 0; k < sizeof maps / sizeof maps[0]; k++) strmap_free(maps[k]);
    free(x->exact.keys);
    free(x->exact.vals);
    for (int32_t k = 0; k < x->exact.nlists; k++) free(x->exact.lists[k].v);
    free(x->exact.lists);
    free(x->trie);
    free(x->leaf);
    free(x);
}

/* Zeroed tile memory for the counter and cache-cell tables, bumped out of 32 MiB anonymous
 * maps backed by transparent huge pages: worker threads touch the tiles at random, one pair
 * per packet, and over 4 KiB pages each touch is also a page walk (engine.hip:
 * shadowtopo_host_alloc has the measurement).  A tile is allocated once, on first touch, so
 * the arena takes a lock; a tile lost to a racing first touch stays unused until
 * topology_free unmaps the slabs. */
#define ARENA_SLAB ((size_t)32 << 20)
typedef struct arena_slab {
    struct arena_slab* next;
    size_t len;
} arena_slab;

static void* arena_alloc(tile_arena* ar, size_t bytes) {
    bytes = (bytes + 63) & ~(size_t)63;
    pthread_mutex_lock(&ar->mu);
    if (!ar->head || ar->off + bytes > ar->head->len) {
        size_t len = bytes + 64 > ARENA_SLAB ? ((bytes + 64 + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1)) : ARENA_SLAB;
        void* p = mmap(NULL, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) {
            pthread_mutex_unlock(&ar->mu);
            return NULL;
        }
        (void)madvise(p, len, MADV_HUGEPAGE);
        arena_slab* sl = p;
        sl->next = ar->head;
        sl->len = len;
        ar->head = sl;
        ar->off = 64;
    }
    void* r = (char*)ar->head + ar->off;
    ar->off += bytes;
    pthread_mutex_unlock(&ar->mu);
    return r;
}

static void arena_free(tile_arena* ar) {
    for (arena_slab* sl = ar->head; sl;) {
        arena_slab* n = sl->next;
        munmap(sl, sl->len);
        sl = n;
    }
    ar->head = NULL;
    pthread_mutex_destroy(&ar->mu);
}

/* tile (ti, tj) of `words` u64 in a rows -> tiles table, allocated on first touch with a
 * compare-and-swap (no lock); NULL when out of range or out of memory */
static uint64_t* tile_get(tile_arena* ar, _Atomic(_Atomic(uint64_t*)*)* rows, int32_t ctd, int32_t ti, int32_t tj,
                          size_t words) {
    if (!rows || ti >= ctd || tj >= ctd) return NULL;
    _Atomic(uint64_t*)* row = atomic_load_explicit(&rows[ti], memory_order_acquire);
    if (!row) {
        _Atomic(uint64_t*)* fresh = calloc((size_t)ctd, sizeof(*fresh));
        if (!fresh) return NULL;
        _Atomic(uint64_t*)* expect = NULL;
        if (atomic_compare_exchange_strong_explicit(&rows[ti], &expect, fresh, memory_order_acq_rel,
                                                    memory_order_acquire))
            row = fresh;
        else {
            free((void*)fresh);
            row = expect;
        }
    }
    uint64_t* tile = atomic_load_explicit(&row[tj], memory_order_acquire);
    if (!tile) {
        uint64_t* fresh = arena_alloc(ar, words * sizeof(uint64_t));
        if (!fresh) return NULL;
        uint64_t* expect = NULL;
        tile = atomic_compare_exchange_strong_explicit(&row[tj], &expect, fresh, memory_order_acq_rel,
                                                       memory_order_acquire)
                   ? fresh
                   : expect;
    }
    return tile;
}

/* the tile if it exists (readers: no allocation) */
static uint64_t* tile_peek(_Atomic(_Atomic(uint64_t*)*)* rows, int32_t ctd, int32_t ti, int32_t tj) {
    if (!rows || ti >= ctd || tj >= ctd) return NULL;
    _Atomic(uint64_t*)* row = atomic_load_explicit(&rows[ti], memory_order_acquire);
    return row ? atomic_load_explicit(&row[tj], memory_order_acquire) : NULL;
}

static void tiles_free(_Atomic(_Atomic(uint64_t*)*)* rows, int32_t ctd) {
    if (!rows) return;
    for (int32_t ti = 0; ti < ctd; ti++) {
        _Atomic(uint64_t*)* row = atomic_load(&rows[ti]);
        if (!row) continue;
        free((void*)row);
    }
    free((void*)rows);
}

/* counter cell of attached pair (i, j): one per cached Path, i.e. per unordered pair in
 * undirected graphs (the reference stores one direction, topology.c:1312-1318); the
 * stored value is count + 1 so a touched pair is non-zero. */
static _Atomic uint64_t* counter_slot(Topology* top, int32_t i, int32_t j) {
    if (!top->directed && j < i) {
        int32_t t = i;
        i = j;
        j = t;
    }
    uint64_t* tile = tile_get(&top->tiles, top->crow, top->ctd, i / CTILE, j / CTILE, CTILE * CTILE);
    return tile ? (_Atomic uint64_t*)&tile[(i % CTILE) * CTILE + (j % CTILE)] : NULL;
}

static uint64_t counter_peek(const Topology* top, int32_t i, int32_t j) {
    if (!top->directed && j < i) {
        int32_t t = i;
        i = j;
        j = t;
    }
    uint64_t* tile = tile_peek(top->crow, top->ctd, i / CTILE, j / CTILE);
    return tile ? atomic_load_explicit((_Atomic uint64_t*)&tile[(i % CTILE) * CTILE + (j % CTILE)],
                                       memory_order_relaxed)
                : 0;
}

/* The emulated path cache's stored set (cache_resolve): one 2-bit cell per unordered pair
 * {a <= b} -- bit 0: (a, b) is cached, bit 1: (b, a) -- in tile (a / 64, b / 64), word
 * 2 (a % 64) + (b % 64) / 32, so the direction that holds a pair is decided by ONE
 * compare-and-swap: _topology_shouldStorePath's "neither direction cached yet"
 * (topology.c:1309-1318) as an atomic claim, with no lock on the store path.  Directed graphs
 * too: the reference refuses (s, t) there as well once (t, s) is cached. */
#define STILE_WORDS(top) (2 * CTILE)

static _Atomic uint64_t* cell_word(const Topology* top, int32_t a, int32_t b, int alloc, int* shift) {
    /* the arena is the topology's mutable allocator state, not part of the query's const view */
    uint64_t* tile = alloc ? tile_get((tile_arena*)&top->tiles, top->srow, top->ctd, a / CTILE, b / CTILE, STILE_WORDS(top))
                           : tile_peek(top->srow, top->ctd, a / CTILE, b / CTILE);
    if (!tile) return NULL;
    *shift = 2 * (b % 32);
    return (_Atomic uint64_t*)&tile[2 * (a % CTILE) + (b % CTILE) / 32];
}

/* which direction of attached pair (i, j) is cached: 1 = (i, j), 2 = (j, i), 0 = neither */
static int cached_dir(const Topology* top, int32_t i, int32_t j) {
    int sh;
    const int32_t a = i < j ? i : j, b = i < j ? j : i;
    _Atomic uint64_t* w = cell_word(top, a, b, 0, &sh);
    const unsigned c = w ? (unsigned)((atomic_load_explicit(w, memory_order_acquire) >> sh) & 3u) : 0u;
    if (!c) return 0;
    if (i == j) return 1;
    /* bit 0 holds (a, b): the forward direction when i < j */
    return ((c & 1u) != 0) == (i < j) ? 1 : 2;
}

/* cache (i, j) unless the pair is cached already in either direction (directed graphs too,
 * topology.c:1311-1317); 1 when this call stored it */
static int cache_claim_bit(Topology* top, int32_t i, int32_t j, unsigned diag_bit) {
    int sh;
    const int32_t a = i < j ? i : j, b = i < j ? j : i;
    _Atomic uint64_t* w = cell_word(top, a, b, 1, &sh);
    if (!w) return 0;
    /* a self pair's cell: bit 0 = cached by s's Dijkstra (the [s] path) or by the default
     * rule's self path, bit 1 = cached by the self-path rule under self_rule */
    const uint64_t bit = (uint64_t)(i == j ? diag_bit : (i < j ? 1u : 2u)) << sh;
    uint64_t cur = atomic_load_explicit(w, memory_order_acquire);
    while (!((cur >> sh) & 3u))
        if (atomic_compare_exchange_weak_explicit(w, &cur, cur | bit, memory_order_acq_rel, memory_order_acquire))
            return 1;
    return 0;
}
static int cache_claim(Topology* top, int32_t i, int32_t j) { return cache_claim_bit(top, i, j, 1u); }

/* the self pair (i, i) was cached by the self-path rule under self_rule: it reads the
 * matrix's srl_* values instead of the diagonal */
static int diag_self_rule(const Topology* top, int32_t i) {
    int sh;
    _Atomic uint64_t* w = cell_word((Topology*)top, i, i, 0, &sh);
    return w && ((atomic_load_explicit(w, memory_order_acquire) >> sh) & 2u);
}

/* matrix cells are read by the getters while a late attach's fill_old_rows rewrites
 * others: relaxed atomic accesses (plain moves on x86-64) */
static inline double cell_d(const double* p) {
    uint64_t u = __atomic_load_n((const uint64_t*)p, __ATOMIC_RELAXED);
    double d;
    memcpy(&d, &u, sizeof d);
    return d;
}
static inline void cell_d_store(double* p, double d) {
    uint64_t u;
    memcpy(&u, &d, sizeof u);
    __atomic_store_n((uint64_t*)p, u, __ATOMIC_RELAXED);
}
static inline uint8_t cell_k(const uint8_t* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }

static char* path_string(const Topology* top, int32_t s, int32_t t, const matrix* m, int32_t i, int32_t j,
                         int srl, uint64_t count, char* buf, size_t len) {
    /* path_toString, path.c:62-75 (srl: a self pair cached by the self-path rule under
     * self_rule, whose values are the matrix's srl_*) */
    size_t o = (size_t)i * m->A + j;
    snprintf(buf, len,
             "SourceIndex=%ld DestinationIndex=%ld Latency=%f Reliability=%f PacketCount=%lu isDirect=%s", (long)s,
             (long)t, srl ? m->srl_lat[i] : cell_d(&m->lr[2 * o]), srl ? m->srl_rel[i] : cell_d(&m->lr[2 * o + 1]),
             (unsigned long)count, (!srl && cell_k(&m->kind[o]) == SHADOWTOPO_KIND_DIRECT) ? "True" : "False");
    (void)top;
    return buf;
}

void topology_free(Topology* top) {
    if (!top) return;
    matrix* m = atomic_load(&top->mat);
    if (m && top->srow && shadowtopo_log_enabled(ST_INFO)) {
        /* _topology_logAllCachedPaths (topology.c:1929-1967): every Path in the (emulated)
         * cache, with every packet counted on it (late attaches included) */
        char buf[512];
        for (int32_t ti = 0; ti < top->ctd; ti++) {
            for (int32_t tj = 0; tj < top->ctd; tj++) {
                uint64_t* tile = tile_peek(top->srow, top->ctd, ti, tj);
                if (!tile) continue;
                for (int32_t x = 0; x < STILE_WORDS(top); x++) {
                    for (uint64_t w = tile[x]; w; w &= w - 1) {
                        const int bit = __builtin_ctzll(w);
                        /* cell (a, b): bit 0 -> (a, b) cached, bit 1 -> (b, a) */
                        const int32_t a = ti * CTILE + x / 2, b = tj * CTILE + (x % 2) * 32 + bit / 2;
                        const int32_t i = (bit & 1) ? b : a, j = (bit & 1) ? a : b;
                        if (i >= m->A || j >= m->A) continue;
                        uint64_t c = counter_peek(top, i, j);
                        int32_t s = top->attached[i], t = top->attached[j];
                        const int srl = i == j && (bit & 1) && m->srl_lat != NULL;
                        st_info("Found path %s%s%s in cache: %s", vid(top, s), top->directed ? "->" : "<->",
                                vid(top, t), path_string(top, s, t, m, i, j, srl, c ? c - 1 : 0, buf, sizeof buf));
                    }
                }
            }
        }
    }
    /* topology.c:1276-1280; the Dijkstra seconds are the GPU computation's, the self-path
     * seconds the engine's self-rule kernel */
    shadowtopo_stats est;
    double self_s = 0.0;
    for (int32_t k = 0; k < top->ndev; k++)
        if (top->engs[k] && shadowtopo_get_stats(top->engs[k], &est) == SHADOWTOPO_OK) self_s += est.self_ms * 1e-3;
    st_message("path cache cleared, spent %f seconds computing %u shortest paths with dijkstra, "
               "and %f seconds computing %u shortest self paths",
               top->compute_s, (unsigned)atomic_load(&top->dijkstra_runs), self_s,
               (unsigned)atomic_load(&top->self_count));
    free_matrix(m);
    for (matrix* r = top->retired; r;) {
        matrix* n = r->next;
        free_matrix(r);
        r = n;
    }
    tiles_free(top->crow, top->ctd);
    tiles_free(top->srow, top->ctd);
    arena_free(&top->tiles);
    free(atomic_load(&top->ips));
    for (iptab* r = top->ips_retired; r;) {
        iptab* n = r->next;
        free(r);
        r = n;
    }
    free_index(top->aidx);
    for (int32_t k = 0; k < top->ndev; k++)
        if (top->engs[k]) shadowtopo_destroy(top->engs[k]);
    top->eng = NULL;
    free((void*)top->att_index);
    free(top->attached);
    free(top->elat);
    free(top->eloss);
    free(top->vloss);
    gml_free(top->gml);
    pthread_rwlock_destroy(&top->ip_lock);
    pthread_mutex_destroy(&top->compute_lock);
    pthread_mutex_destroy(&top->idx_lock);
    pthread_mutex_destroy(&top->min_lock);
    free((void*)top->src_loop);
    top->magic = 0;
    free(top);
}

/* SHADOWTOPO_DEVICES / topology_hip_set_devices: engines that share a device split its
 * batch-slot HBM budget (shadowtopo.h SHADOWTOPO_OPT_HBM_SHARE) */
static int32_t device_sharers(const Topology* top, int32_t k) {
    int32_t n = 0;
    for (int32_t j = 0; j < top->ndev; j++) n += top->devices[j] == top->devices[k];
    return n;
}

Topology* topology_new(const char* graphPath) {
    if (!graphPath) return NULL;
    Topology* top = calloc(1, sizeof(Topology));
    if (!top) return NULL;
    top->magic = TOPO_MAGIC;
    pthread_rwlock_init(&top->ip_lock, NULL);
    pthread_mutex_init(&top->compute_lock, NULL);
    pthread_mutex_init(&top->idx_lock, NULL);
    pthread_mutex_init(&top->min_lock, NULL);
    pthread_mutex_init(&top->tiles.mu, NULL);
    atomic_store(&top->ips, NULL);
    const char* dev = getenv("SHADOWTOPO_DEVICE");
    top->device = dev ? atoi(dev) : 0;
    top->ndev = 1;
    top->devices[0] = top->device;
    /* SHADOWTOPO_DEVICES: comma-separated device list, e.g. "0,1,2,3,4,5,6,7" */
    const char* devs = getenv("SHADOWTOPO_DEVICES");
    if (devs && *devs) {
        int32_t n = 0;
        for (const char* c = devs; *c && n < SHADOWTOPO_MAX_DEVICES;) {
            char* end = NULL;
            long d = strtol(c, &end, 10);
            if (end == c) break;
            top->devices[n++] = (int32_t)d;
            c = (*end == ',') ? end + 1 : end;
        }
        if (n > 0) {
            top->ndev = n;
            top->device = top->devices[0];
        }
    }
    atomic_store(&top->mat, NULL);
    /* the device's runtime initialisation, staging buffers and code objects on a background
     * thread while the file is parsed (shadowtopo_prepare); the engine is created later */
    if (top->device >= 0 && top->device < shadowtopo_device_count()) (void)shadowtopo_prepare(top->device);

    char err[512] = {0};
    st_message("reading graphml topology graph at '%s'...", graphPath);
    if (gml_parse_file(graphPath, &top->gml, err, sizeof err) != 0) {
        st_critical("reading graphml topology graph at '%s' failed: %s", graphPath, err);
        topology_free(top);
        st_critical("we failed to create the simulation topology because we were unable to validate the topology "
                    "graphml file");
        return NULL;
    }
    st_message("successfully read graphml topology graph at '%s'", graphPath);
    top->V = top->gml->n;
    top->E = top->gml->m;
    top->directed = top->gml->directed;
    top->a_ip = gml_find(top->gml, GML_NODE, "ip");
    top->a_city = gml_find(top->gml, GML_NODE, "citycode");
    top->a_country = gml_find(top->gml, GML_NODE, "countrycode");
    top->a_geo = gml_find(top->gml, GML_NODE, "geocode");
    top->a_type = gml_find(top->gml, GML_NODE, "type");
    top->a_bwdown = gml_find(top->gml, GML_NODE, "bandwidthdown");
    top->a_bwup = gml_find(top->gml, GML_NODE, "bandwidthup");
    top->a_asn = gml_find(top->gml, GML_NODE, "asn");
    top->a_vloss = gml_find(top->gml, GML_NODE, "packetloss");
    int ok = check_properties(top) && check_vertices(top) && check_edges(top);
    if (ok)
        st_message("successfully parsed graphml and validated topology: graph is %s with %u %s, %u %s, and %u %s",
                   top->connected ? "strongly connected" : "disconnected", (unsigned)top->clusters,
                   top->clusters == 1 ? "cluster" : "clusters", (unsigned)top->V, top->V == 1 ? "vertex" : "vertices",
                   (unsigned)top->E, top->E == 1 ? "edge" : "edges");
    if (!ok || !extract(top)) {
        topology_free(top);
        st_critical("we failed to create the simulation topology because we were unable to validate the topology "
                    "graphml file");
        return NULL;
    }
    top->att_index = malloc(sizeof(*top->att_index) * (size_t)(top->V > 0 ? top->V : 1));
    for (int32_t v = 0; v < top->V; v++) atomic_init(&top->att_index[v], -1);
    top->src_loop = malloc(sizeof(*top->src_loop) * (size_t)(top->V > 0 ? top->V : 1));
    for (int32_t v = 0; v < top->V; v++) atomic_init(&top->src_loop[v], 0);
    top->ctd = (top->V + CTILE - 1) / CTILE;
    top->crow = calloc((size_t)(top->ctd > 0 ? top->ctd : 1), sizeof(*top->crow));
    top->srow = calloc((size_t)(top->ctd > 0 ? top->ctd : 1), sizeof(*top->srow));
    return top;
}
/* ------------------------------------------------------------ attach
 * _topology_findAttachmentVertex + its hook (topology.c:2094-2369) scan every vertex per
 * host with five string compares (5e4 hosts x 1e6 vertices at C5).  Here the same
 * candidate queues come from indexes built once, on the first attach:
 * the ASCII-lowercased citycode / countrycode / geocode / type values and the three
 * (code, type) pairs map to ascending vertex lists with their usable-IP counts, the usable
 * vertex IPs map to their vertices (the exact-IP rule), and a binary trie over every
 * vertex's parsed IP answers the longest-prefix rule over the whole vertex set.  Queue
 * order (ascending vertex index), the usable-IP counts, the ~(a^b) match with its
 * 'bestMatch == 0' quirk and the round((n-1)*r) pick are the reference's, so the chosen
 * vertex and the consumed random stream are identical (tests/test_topology_shim.py checks
 * them against oracle/attach_ref.py, a restatement of the scan). */
static int usable_ip(in_addr_t ip) { return ip != INADDR_NONE && ip != INADDR_ANY && ip != INADDR_LOOPBACK; }

static uint64_t fnv1a(const char* s, size_t n) {
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 0; i < n; i++) h = (h ^ (uint8_t)s[i]) * 1099511628211ULL;
    return h;
}

/* g_ascii_strcasecmp equality == equality of the ASCII-lowercased strings (malloc'd) */
static char* ascii_lower(const char* s) {
    const size_t n = strlen(s);
    char* out = malloc(n + 1);
    if (!out) return NULL;
    for (size_t i = 0; i <= n; i++) out[i] = (char)((s[i] >= 'A' && s[i] <= 'Z') ? s[i] + 32 : s[i]);
    return out;
}

static vlist* strmap_get(const strmap* m, const char* key, size_t n) {
    if (!m->cap) return NULL;
    for (size_t j = fnv1a(key, n) & (m->cap - 1); m->keys[j]; j = (j + 1) & (m->cap - 1))
        if (!memcmp(m->keys[j], key, n) && m->keys[j][n] == 0) return &m->lists[m->vals[j]];
    return NULL;
}

static vlist* strmap_add(strmap* m, const char* key, size_t n) {
    vlist* l = strmap_get(m, key, n);
    if (l) return l;
    if ((m->n + 1) * 2 > m->cap) {
        size_t ncap = m->cap ? m->cap * 2 : 64;
        char** nk = calloc(ncap, sizeof(char*));
        int32_t* nv = calloc(ncap, sizeof(int32_t));
        for (size_t i = 0; i < m->cap; i++) {
            if (!m->keys[i]) continue;
            size_t j = fnv1a(m->keys[i], strlen(m->keys[i])) & (ncap - 1);
            while (nk[j]) j = (j + 1) & (ncap - 1);
            nk[j] = m->keys[i];
            nv[j] = m->vals[i];
        }
        free(m->keys);
        free(m->vals);
        m->keys = nk;
        m->vals = nv;
        m->cap = ncap;
    }
    if (m->nlists == m->caplists) {
        m->caplists = m->caplists ? m->caplists * 2 : 16;
        m->lists = realloc(m->lists, sizeof(vlist) * (size_t)m->caplists);
    }
    size_t j = fnv1a(key, n) & (m->cap - 1);
    while (m->keys[j]) j = (j + 1) & (m->cap - 1);
    m->keys[j] = strndup(key, n);
    m->vals[j] = m->nlists;
    memset(&m->lists[m->nlists], 0, sizeof(vlist));
    m->n++;
    return &m->lists[m->nlists++];
}

static vlist* u32map_get(const u32map* m, uint32_t k) {
    if (!m->cap) return NULL;
    for (size_t j = ip_slot(k, m->cap); m->vals[j]; j = (j + 1) & (m->cap - 1))
        if (m->keys[j] == k) return &m->lists[m->vals[j] - 1];
    return NULL;
}

static vlist* u32map_add(u32map* m, uint32_t k) {
    vlist* l = u32map_get(m, k);
    if (l) return l;
    if ((m->n + 1) * 2 > m->cap) {
        size_t ncap = m->cap ? m->cap * 2 : 64;
        uint32_t* nk = calloc(ncap, sizeof(uint32_t));
        int32_t* nv = calloc(ncap, sizeof(int32_t));
        for (size_t i = 0; i < m->cap; i++) {
            if (!m->vals[i]) continue;
            size_t j = ip_slot(m->keys[i], ncap);
            while (nv[j]) j = (j + 1) & (ncap - 1);
            nk[j] = m->keys[i];
            nv[j] = m->vals[i];
        }
        free(m->keys);
        free(m->vals);
        m->keys = nk;
        m->vals = nv;
        m->cap = ncap;
    }
    if (m->nlists == m->caplists) {
        m->caplists = m->caplists ? m->caplists * 2 : 16;
        m->lists = realloc(m->lists, sizeof(vlist) * (size_t)m->caplists);
    }
    size_t j = ip_slot(k, m->cap);
    while (m->vals[j]) j = (j + 1) & (m->cap - 1);
    m->keys[j] = k;
    m->vals[j] = ++m->nlists;
    memset(&m->lists[m->nlists - 1], 0, sizeof(vlist));
    m->n++;
    return &m->lists[m->nlists - 1];
}

static int32_t trie_node(attach_index* x) {
    if (x->ntrie == x->captrie) {
        x->captrie = x->captrie ? x->captrie * 2 : 1024;
        x->trie = realloc(x->trie, sizeof(*x->trie) * (size_t)x->captrie);
        x->leaf = realloc(x->leaf, sizeof(int32_t) * (size_t)x->captrie);
    }
    x->trie[x->ntrie][0] = x->trie[x->ntrie][1] = 0;
    x->leaf[x->ntrie] = -1;
    return x->ntrie++;
}

/* key "<len(a)>:<a>|<b>" (unambiguous for any byte values), malloc'd */
static char* pair_key(const char* a, const char* b) {
    const size_t n = strlen(a) + strlen(b) + 24;
    char* k = malloc(n);
    if (k) snprintf(k, n, "%zu:%s|%s", strlen(a), a, b);
    return k;
}

static attach_index* build_index(Topology* top) {
    attach_index* x = calloc(1, sizeof(attach_index));
    const int32_t V = top->V;
    x->vip = malloc(sizeof(in_addr_t) * (size_t)(V ? V : 1));
    x->usable = calloc((size_t)(V ? V : 1), 1);
    trie_node(x); /* root */
    for (int32_t v = 0; v < V; v++) {
        const char *ipS = NULL, *s[4] = {NULL, NULL, NULL, NULL};
        int ipF = vstr(top, top->a_ip, v, &ipS);
        vstr(top, top->a_city, v, &s[0]);
        vstr(top, top->a_country, v, &s[1]);
        vstr(top, top->a_geo, v, &s[2]);
        vstr(top, top->a_type, v, &s[3]);
        /* LPM key: VAS(graph, "ip", v) parsed, "" (INADDR_NONE) when absent (topology.c:2232-2235) */
        x->vip[v] = address_stringToIP(top->a_ip ? gml_str(top->a_ip, v) : "");
        const in_addr_t ip = ipF ? address_stringToIP(ipS) : INADDR_NONE;
        const int u = ipF && usable_ip(ip);
        x->usable[v] = (uint8_t)u;
        x->nips_all += u;
        if (u) vl_push(u32map_add(&x->exact, ip), v, 1);
        char* l[4] = {NULL, NULL, NULL, NULL};
        for (int k = 0; k < 4; k++)
            if (s[k]) l[k] = ascii_lower(s[k]);
        strmap* single[3] = {&x->city, &x->country, &x->geo};
        strmap* paired[3] = {&x->city_type, &x->country_type, &x->geo_type};
        for (int k = 0; k < 3; k++) {
            if (!l[k]) continue;
            vl_push(strmap_add(single[k], l[k], strlen(l[k])), v, u);
            char* key = l[3] ? pair_key(l[k], l[3]) : NULL;
            if (key) vl_push(strmap_add(paired[k], key, strlen(key)), v, u);
            free(key);
        }
        if (l[3]) vl_push(strmap_add(&x->type, l[3], strlen(l[3])), v, u);
        for (int k = 0; k < 4; k++) free(l[k]);
        /* trie insert, bit 31 first; a leaf keeps its first (lowest) vertex */
        int32_t node = 0;
        for (int b = 31; b >= 0; b--) {
            const int bit = (int)((x->vip[v] >> b) & 1u);
            if (!x->trie[node][bit]) {
                int32_t c = trie_node(x);
                x->trie[node][bit] = c;
            }
            node = x->trie[node][bit];
        }
        if (x->leaf[node] < 0) x->leaf[node] = v;
    }
    return x;
}

static attach_index* attach_index_of(Topology* top) {
    pthread_mutex_lock(&top->idx_lock);
    if (!top->aidx) top->aidx = build_index(top);
    attach_index* x = top->aidx;
    pthread_mutex_unlock(&top->idx_lock);
    return x;
}

/* a hint's queue (NULL hint or no vertex with that value: empty) */
static vlist* queue_of(const strmap* m, const char* hint) {
    if (!hint) return NULL;
    char* l = ascii_lower(hint);
    vlist* q = l ? strmap_get(m, l, strlen(l)) : NULL;
    free(l);
    return q;
}

static vlist* pair_queue_of(const strmap* m, const char* a, const char* b) {
    if (!a || !b) return NULL;
    char *la = ascii_lower(a), *lb = ascii_lower(b);
    char* key = (la && lb) ? pair_key(la, lb) : NULL;
    vlist* q = key ? strmap_get(m, key, strlen(key)) : NULL;
    free(la);
    free(lb);
    free(key);
    return q;
}

/* _topology_getLongestPrefixMatch (topology.c:2219-2246) over one queue, in queue order */
static int32_t lpm_scan(const attach_index* x, const vlist* q, in_addr_t requested) {
    in_addr_t best_match = 0;
    int32_t chosen = -1;
    for (int32_t k = 0; k < q->n; k++) {
        const in_addr_t match = ~(x->vip[q->v[k]] ^ requested);
        if (match > best_match || best_match == 0) {
            best_match = match;
            chosen = q->v[k];
        }
    }
    return chosen;
}

/* the same over every vertex: max ~(vip ^ req) == min (vip ^ req), the first vertex with
 * that value; if even the best match is 0 every vertex replaced the previous one, so the
 * reference returns the last vertex */
static int32_t lpm_all(const attach_index* x, int32_t V, in_addr_t requested) {
    if (V <= 0) return -1;
    int32_t node = 0;
    uint32_t xr = 0;
    for (int b = 31; b >= 0; b--) {
        const int want = (int)((requested >> b) & 1u);
        if (x->trie[node][want]) {
            node = x->trie[node][want];
        } else {
            node = x->trie[node][want ^ 1];
            xr |= 1u << b;
        }
    }
    if ((in_addr_t)~xr == 0) return V - 1;
    return x->leaf[node];
}

static int32_t find_attachment_vertex(Topology* top, Random* rnd, const char* ipHint, const char* cityHint,
                                      const char* countryHint, const char* geoHint, const char* typeHint) {
    const attach_index* x = attach_index_of(top);
    int requested_usable = 0;
    in_addr_t requested = 0;
    if (ipHint) {
        in_addr_t ip = address_stringToIP(ipHint);
        if (usable_ip(ip)) {
            requested_usable = 1;
            requested = ip;
        }
    }
    const vlist* q = NULL;
    int32_t n = top->V; /* ALL: every vertex, in order */
    int use_lpm = 0;
    const vlist* exact = requested_usable ? u32map_get(&x->exact, requested) : NULL;
    if (exact && exact->n > 0) {
        /* exact IP matches: every other queue was cleared, LPM is skipped (topology.c:2138-2160, 2318) */
        q = exact;
        n = exact->n;
    } else {
        const vlist* cand[7] = {
            pair_queue_of(&x->city_type, cityHint, typeHint), queue_of(&x->city, cityHint),
            pair_queue_of(&x->country_type, countryHint, typeHint), queue_of(&x->country, countryHint),
            pair_queue_of(&x->geo_type, geoHint, typeHint), queue_of(&x->geo, geoHint), queue_of(&x->type, typeHint)};
        for (int k = 0; k < 7 && !q; k++)
            if (cand[k] && cand[k]->n > 0) q = cand[k];
        if (q) {
            n = q->n;
            use_lpm = requested_usable && q->nips > 0;
        } else {
            use_lpm = ipHint && x->nips_all > 0;
        }
    }
    if (n <= 0) return -1;
    if (use_lpm) return q ? lpm_scan(x, q, requested) : lpm_all(x, top->V, requested);
    double r = random_nextDouble(rnd);
    int index_range = n - 1;
    int chosen_index = (int)round((double)(index_range * r));
    if (chosen_index < 0 || chosen_index >= n) return -1;
    return q ? q->v[chosen_index] : chosen_index;
}

void topology_attach(Topology* top, Address* address, Random* randomSourcePool, char* ipHint, char* citycodeHint,
                     char* countrycodeHint, char* geocodeHint, char* typeHint, uint64_t* bwDownOut,
                     uint64_t* bwUpOut) {
    if (!top || !address) return;
    uint32_t node_ip = address_toNetworkIP(address);
    int32_t v = find_attachment_vertex(top, randomSourcePool, ipHint, citycodeHint, countrycodeHint, geocodeHint,
                                       typeHint);
    if (v < 0) {
        st_error("no attachment vertex for address '%s'", address_toHostIPString(address));
        return;
    }
    pthread_rwlock_wrlock(&top->ip_lock);
    if (ipt_put(&top->ips, &top->ips_retired, &top->ips_nretired, node_ip, v))
        st_critical("out of memory for the IP table; address '%s' stays unconnected", address_toHostIPString(address));
    if (atomic_load_explicit(&top->att_index[v], memory_order_relaxed) < 0) {
        if (top->n_att == top->cap_att) {
            top->cap_att = top->cap_att ? top->cap_att * 2 : 256;
            top->attached = realloc(top->attached, sizeof(int32_t) * (size_t)top->cap_att);
        }
        top->attached[top->n_att] = v;
        atomic_store_explicit(&top->att_index[v], top->n_att, memory_order_release);
        top->n_att++;
    }
    pthread_rwlock_unlock(&top->ip_lock);
    double x;
    if (bwUpOut) *bwUpOut = vnum(top->a_bwup, v, &x) ? (uint64_t)x : 0;
    if (bwDownOut) *bwDownOut = vnum(top->a_bwdown, v, &x) ? (uint64_t)x : 0;
    if (!shadowtopo_log_enabled(ST_MESSAGE)) return;
    const char *ipS = NULL, *cityS = NULL, *countryS = NULL, *geoS = NULL, *typeS = NULL;
    vstr(top, top->a_ip, v, &ipS);
    vstr(top, top->a_city, v, &cityS);
    vstr(top, top->a_country, v, &countryS);
    vstr(top, top->a_geo, v, &geoS);
    vstr(top, top->a_type, v, &typeS);
#define NS(x) ((x) ? (x) : "(null)")
    st_message("attached address '%s' to vertex %li ('%s') with attributes (ip=%s, citycode=%s, countrycode=%s, "
               "geocode=%s, type=%s) using hints (ip=%s, citycode=%s, countrycode=%s, geocode=%s, type=%s)",
               address_toHostIPString(address), (long)v, vid(top, v), NS(ipS), NS(cityS), NS(countryS), NS(geoS),
               NS(typeS), NS(ipHint), NS(citycodeHint), NS(countrycodeHint), NS(geocodeHint), NS(typeHint));
#undef NS
}

void topology_detach(Topology* top, Address* address) {
    if (!top || !address) return;
    uint32_t ip = address_toNetworkIP(address);
    pthread_rwlock_wrlock(&top->ip_lock);
    ipt_del(&top->ips, ip);  /* one tombstone store: lookups see it at once, nothing is rebuilt */
    pthread_rwlock_unlock(&top->ip_lock);
}
/* ------------------------------------------------------------ eager computation */
static int ensure_engine(Topology* top) {
    if (top->eng) return 0;
    uint32_t flags = 0;
    if (top->directed) flags |= SHADOWTOPO_F_DIRECTED;
    if (top->complete) flags |= SHADOWTOPO_F_COMPLETE;
    if (top->prefer_direct) flags |= SHADOWTOPO_F_PREFER_DIRECT;
    if (top->self_rule) flags |= SHADOWTOPO_F_SELF_DIJKSTRA_LOOP;
    for (int32_t k = 0; k < top->ndev; k++) {
        int rc = shadowtopo_create(top->V, top->E, top->gml->src, top->gml->dst, top->elat, top->eloss, top->vloss,
                                   flags, top->devices[k], &top->engs[k]);
        if (rc == SHADOWTOPO_OK)
            rc = shadowtopo_set_option(top->engs[k], SHADOWTOPO_OPT_HBM_SHARE, 1000 / device_sharers(top, k));
        if (rc != SHADOWTOPO_OK) {
            st_critical("GPU topology engine unavailable on device %d (%d): %s", (int)top->devices[k], rc,
                        shadowtopo_last_error());
            for (int32_t j = 0; j <= k; j++) {
                if (top->engs[j]) shadowtopo_destroy(top->engs[j]);
                top->engs[j] = NULL;
            }
            return -1;
        }
    }
    top->eng = top->engs[0];
    return 0;
}

/* one device's share of the rows: source rows [r0, r1) of the attached list, written to
 * out + (row - r0) * A (host memory) */
typedef struct {
    shadowtopo_engine* eng;
    const int32_t* attached;
    int32_t A, r0, r1;
    double* lr;
    uint8_t* kind;
    int rc;
    char err[256];
} row_block;

static void* compute_block(void* arg) {
    row_block* w = arg;
    w->rc = shadowtopo_set_attached(w->eng, w->attached, w->A);
    if (w->rc == SHADOWTOPO_OK && w->r1 > w->r0)
        w->rc = shadowtopo_compute_rows(w->eng, w->r0, w->r1, w->lr, NULL, NULL, w->kind, SHADOWTOPO_MEM_HOST_LR,
                                        NULL);
    if (w->rc != SHADOWTOPO_OK) snprintf(w->err, sizeof w->err, "%s", shadowtopo_last_error());
    return NULL;
}

/* rows [r0, r1) of the pair matrix over `attached` (A targets) into m's rows, sharded over
 * the devices (device k takes the contiguous k-th block, its own thread) */
static int compute_rows_sharded(Topology* top, const int32_t* attached, int32_t A, int32_t r0, int32_t r1,
                                matrix* m) {
    int32_t nd = top->ndev;
    row_block blocks[SHADOWTOPO_MAX_DEVICES];
    pthread_t th[SHADOWTOPO_MAX_DEVICES];
    const int32_t rows = r1 - r0;
    const int32_t per = (rows + nd - 1) / nd;
    for (int32_t k = 0; k < nd; k++) {
        row_block* b = &blocks[k];
        b->eng = top->engs[k];
        b->attached = attached;
        b->A = A;
        b->r0 = r0 + (k * per < rows ? k * per : rows);
        b->r1 = r0 + ((k + 1) * per < rows ? (k + 1) * per : rows);
        const size_t o = (size_t)b->r0 * (size_t)A;
        b->lr = m->lr + 2 * o;
        b->kind = m->kind + o;
        b->rc = 0;
        b->err[0] = 0;
    }
    int spawned[SHADOWTOPO_MAX_DEVICES] = {0};
    for (int32_t k = 1; k < nd; k++) spawned[k] = pthread_create(&th[k], NULL, compute_block, &blocks[k]) == 0;
    compute_block(&blocks[0]);
    for (int32_t k = 1; k < nd; k++) {
        if (spawned[k])
            pthread_join(th[k], NULL);
        else
            compute_block(&blocks[k]);
    }
    for (int32_t k = 0; k < nd; k++) {
        if (blocks[k].rc != SHADOWTOPO_OK) {
            st_critical("attached-pair computation failed on device %d (%d): %s", (int)top->devices[k],
                        blocks[k].rc, blocks[k].err);
            return -1;
        }
    }
    return 0;
}

static matrix* alloc_matrix(int32_t A) {
    matrix* m = calloc(1, sizeof(matrix));
    if (!m) return NULL;
    size_t n = (size_t)A * (size_t)A;
    m->A = A;
    /* page-locked first; plain malloc when the driver refuses (the copy is then slower) */
    void *pl = NULL, *pk = NULL;
    if (shadowtopo_host_alloc(2 * sizeof(double) * (n ? n : 1), &pl) == SHADOWTOPO_OK &&
        shadowtopo_host_alloc(n ? n : 1, &pk) == SHADOWTOPO_OK) {
        m->pinned = 1;
        m->lr = pl;
        m->kind = pk;
    } else {
        shadowtopo_host_free(pl);
        shadowtopo_host_free(pk);
        m->pinned = 0;
        m->lr = malloc(2 * sizeof(double) * (n ? n : 1));
        m->kind = malloc(n ? n : 1);
    }
    if (!m->lr || !m->kind) {
        st_critical("out of host memory for the %d x %d attached-pair matrix", A, A);
        free_matrix(m);
        return NULL;
    }
    return m;
}

/* The matrix for the first A attached vertices (`attached`, a private copy).
 * Late attach (`old` covers the first old->A of them): in an undirected graph only the new
 * rows are computed (the new sources against every target); an old source's entry for a
 * new target takes the new target's own entry for it (the reverse direction), which is
 * exactly what the reference returns once the new host's paths are cached first
 * (_topology_getPathEntry tries (t, s) for undirected graphs, topology.c:1987-1990), and
 * the old block is kept as computed.  Directed graphs recompute every row. */
static matrix* compute_matrix(Topology* top, const int32_t* attached, int32_t A, const matrix* old) {
    if (ensure_engine(top)) return NULL;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    matrix* m = alloc_matrix(A);
    if (!m) return NULL;
    const int32_t A0 = (old && !top->directed && old->A < A) ? old->A : 0;
    if (compute_rows_sharded(top, attached, A, A0, A, m)) {
        free_matrix(m);
        return NULL;
    }
    if (top->self_rule) {
        m->srl_lat = malloc(sizeof(double) * (size_t)(A ? A : 1));
        m->srl_rel = malloc(sizeof(double) * (size_t)(A ? A : 1));
        m->srl_kind = malloc((size_t)(A ? A : 1));
        if (!m->srl_lat || !m->srl_rel || !m->srl_kind ||
            shadowtopo_self_rule_paths(top->engs[0], m->srl_lat, m->srl_rel, m->srl_kind) != SHADOWTOPO_OK) {
            st_critical("self-path rule values: %s", shadowtopo_last_error());
            free_matrix(m);
            return NULL;
        }
    }
    for (int32_t i = 0; i < A0; i++) {
        const size_t src = (size_t)i * (size_t)A0, dst = (size_t)i * (size_t)A;
        memcpy(m->lr + 2 * dst, old->lr + 2 * src, 2 * sizeof(double) * (size_t)A0);
        memcpy(m->kind + dst, old->kind + src, (size_t)A0);
        for (int32_t j = A0; j < A; j++) {
            const size_t o = dst + (size_t)j, r = (size_t)j * (size_t)A + (size_t)i;
            m->lr[2 * o] = m->lr[2 * r];
            m->lr[2 * o + 1] = m->lr[2 * r + 1];
            m->kind[o] = m->kind[r];
        }
    }
    /* an old matrix that was never filled passes its reverse copies on */
    m->fill_col = (A0 > 0 && atomic_load_explicit(&old->partial, memory_order_acquire) > 0) ? old->fill_col : A0;
    atomic_store_explicit(&m->partial, A0, memory_order_release);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    top->compute_s += (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    top->compute_count += A - A0;
    /* the running minimum handed to worker_updateMinTimeJump is folded in as paths enter
     * the emulated cache (cache_resolve), as the reference does */
    st_info("computed %d x %d attached-pair matrix (%d new rows) on %d device(s) (first %d) in %f seconds", A, A,
            A - A0, (int)top->ndev, (int)top->device, top->compute_s);
    return m;
}

/* the matrix covering attached index `need`; computed on the first query that needs it */
static matrix* current_matrix(Topology* top, int32_t need) {
    matrix* m = atomic_load_explicit(&top->mat, memory_order_acquire);
    if (m && m->A > need) return m;
    pthread_mutex_lock(&top->compute_lock);
    m = atomic_load_explicit(&top->mat, memory_order_acquire);
    if ((!m || m->A <= need) && !top->compute_failed) {
        /* a private copy of the attached list: a concurrent attach may grow (realloc) it */
        pthread_rwlock_rdlock(&top->ip_lock);
        const int32_t A = top->n_att;
        int32_t* att = malloc(sizeof(int32_t) * (size_t)(A ? A : 1));
        if (att && A) memcpy(att, top->attached, sizeof(int32_t) * (size_t)A);
        pthread_rwlock_unlock(&top->ip_lock);
        matrix* nm = (att && A > need) ? compute_matrix(top, att, A, m) : NULL;
        free(att);
        if (nm) {
            if (m) {
                m->next = top->retired;
                top->retired = m;
            }
            atomic_store_explicit(&top->mat, nm, memory_order_release);
            m = nm;
        } else {
            /* fail once, loudly: later queries return -1 without retrying the GPU work */
            if (A > need) {
                top->compute_failed = 1;
                st_critical("attached-pair computation failed; every later query fails without a retry");
            }
            m = NULL;
        }
    } else if (!m || m->A <= need) {
        m = NULL;
    }
    pthread_mutex_unlock(&top->compute_lock);
    return m;
}

/* Rows [0, m->partial) of an undirected late-attach matrix with their own entries for the
 * columns the late attach added (compute_matrix copied the reverse direction there):
 * needed once an old source's entry for a new target is read (the reference reruns that
 * source's Dijkstra against the grown target list).  In place, under compute_lock (once per
 * matrix: a thread that waited finds partial == 0), with relaxed atomic cell stores; then
 * partial = 0 with release order.  No reader reads those cells before: cache_resolve fills
 * before it returns such an entry, and every (i, t) it caches is claimed after the fill. */
static int fill_old_rows(Topology* top, matrix* m) {
    if (atomic_load_explicit(&m->partial, memory_order_acquire) <= 0) return 0;
    pthread_mutex_lock(&top->compute_lock);
    const int32_t P = atomic_load_explicit(&m->partial, memory_order_acquire), A = m->A;
    int rc = P <= 0 ? 0 : -1;
    if (P > 0) {
        int32_t* att = malloc(sizeof(int32_t) * (size_t)A);
        matrix tmp;
        memset(&tmp, 0, sizeof tmp);
        tmp.A = A;
        tmp.lr = malloc(2 * sizeof(double) * (size_t)P * (size_t)A);
        tmp.kind = malloc((size_t)P * (size_t)A);
        if (att && tmp.lr && tmp.kind) {
            pthread_rwlock_rdlock(&top->ip_lock);
            memcpy(att, top->attached, sizeof(int32_t) * (size_t)A);  /* attach order: a stable prefix */
            pthread_rwlock_unlock(&top->ip_lock);
            struct timespec t0, t1;
            clock_gettime(CLOCK_MONOTONIC, &t0);
            if (ensure_engine(top) == 0 && compute_rows_sharded(top, att, A, 0, P, &tmp) == 0) {
                /* columns [fill_col, P) of rows [fill_col, P) are own entries already: the
                 * rewrite stores the same values there */
                for (int32_t i = 0; i < P; i++)
                    for (int32_t t = m->fill_col; t < A; t++) {
                        const size_t o = (size_t)i * (size_t)A + (size_t)t;
                        cell_d_store(&m->lr[2 * o], tmp.lr[2 * o]);
                        cell_d_store(&m->lr[2 * o + 1], tmp.lr[2 * o + 1]);
                        __atomic_store_n(&m->kind[o], tmp.kind[o], __ATOMIC_RELAXED);
                    }
                atomic_store_explicit(&m->partial, 0, memory_order_release);
                top->compute_count += P;
                rc = 0;
            }
            clock_gettime(CLOCK_MONOTONIC, &t1);
            top->compute_s += (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
        }
        free(att);
        free(tmp.lr);
        free(tmp.kind);
    }
    pthread_mutex_unlock(&top->compute_lock);
    if (rc) st_critical("recomputing the rows of hosts attached before a late attach failed");
    return rc;
}

/* the running minimum (topology.c:1374-1385: `minimumPathLatency == 0 || lower`), and the
 * upcall after the lock is released, as the reference makes it */
static void note_min_latency(Topology* top, double mn) {
    pthread_mutex_lock(&top->min_lock);
    const int upd = top->min_latency == 0 || mn < top->min_latency;
    if (upd) top->min_latency = mn;
    const double cur = top->min_latency;
    pthread_mutex_unlock(&top->min_lock);
    if (upd) worker_updateMinTimeJump(cur);
}

/* The reference's path cache over the eager matrix.  Every value is computed up front; what
 * follows the reference's query order is WHICH pairs are cached and in which direction, so
 * a getter returns exactly the entry the reference would (_topology_getPathEntry tries
 * (s, t), then (t, s) in undirected graphs, topology.c:1983-1990; after a successful miss
 * (s, t), then (t, s) in any graph, :2033-2038 -- so in a directed graph whose (t, s) was
 * cached first, (s, t) misses every time, reruns s's Dijkstra and returns (t, s)), the minimum handed to
 * worker_updateMinTimeJump changes when the reference's would (:1374-1385), the teardown
 * log lists the reference's cached Paths (:1929-1967), and the Dijkstra / self-path counts
 * are the reference's.  A miss (:1992-2045) replays the reference's branch, which the pair's
 * kind already encodes (k_compose's dispatch of the same rules):
 *   DIRECT    -> _topology_lookupDirectPath: (s, t) alone;
 *   s == t    -> _topology_computeShortestPathToSelf: (s, s);
 *   otherwise -> _topology_computeSourcePaths (:1655-1875): one Dijkstra from s, storing
 *                (s, t') for every attached t' that igraph reaches and that
 *                _topology_shouldStorePath accepts (:1309-1334: neither direction cached
 *                yet; not a non-direct path where the graph prefers an existing direct
 *                edge), t' = s included with the configured self value.
 * No lock: each store is an atomic claim of its pair (cache_claim), so concurrent misses
 * serialise per pair exactly as some order of the reference's would; the O(A) store loop
 * runs once per source and target list (src_loop), a concurrent miss on the same source
 * claiming just its own pair.  Returns the cached direction in (si, sj), or -1 when the
 * pair has no path. */
static int cache_resolve(Topology* top, matrix** mp, int32_t i, int32_t j, int32_t* si, int32_t* sj) {
    matrix* m = *mp;
    int d = cached_dir(top, i, j);
    if (top->directed && d == 2) d = 0; /* a directed lookup tries (s, t) only (:1983-1986) */
    if (!d) {
        /* a late attach may have published a larger matrix meanwhile: its target list is the
         * one the reference's Dijkstra would use now */
        matrix* cur = atomic_load_explicit(&top->mat, memory_order_acquire);
        if (cur && cur->A > (i > j ? i : j)) *mp = m = cur;
        const int32_t A = m->A;
        /* an old source's own entries before any of them is cached (or, below, read) */
        if (i < atomic_load_explicit(&m->partial, memory_order_acquire) && fill_old_rows(top, m)) return -1;
        const uint8_t k = cell_k(&m->kind[(size_t)i * A + j]);
        double mn = 0.0;
        int64_t stored = 0;
        int noted = 0;   /* the Dijkstra branch hands each lowering store to the upcall itself */
        int success = 1; /* the reference's `success` (:2009-2031) */
        if (k == SHADOWTOPO_KIND_DIRECT || top->complete) {
            /* a complete graph without the edge: get_eid fails, nothing is stored */
            if (k != SHADOWTOPO_KIND_DIRECT)
                success = 0;
            else if (cache_claim(top, i, j)) {
                mn = cell_d(&m->lr[2 * ((size_t)i * A + j)]);
                stored = 1;
            }
        } else if (i == j) {
            /* _topology_computeShortestPathToSelf (topology.c:1545-1653); under self_rule the
             * diagonal holds the [s] path's value, the self rule's is in srl_* */
            atomic_fetch_add_explicit(&top->self_count, 1, memory_order_relaxed);
            const uint8_t ks = top->self_rule ? m->srl_kind[i] : k;
            if (ks == SHADOWTOPO_KIND_NONE)
                success = 0; /* no incident edge: no self path */
            else if (cache_claim_bit(top, i, i, top->self_rule ? 2u : 1u)) {
                mn = top->self_rule ? m->srl_lat[i] : cell_d(&m->lr[2 * ((size_t)i * A + i)]);
                stored = 1;
            }
        } else {
            atomic_fetch_add_explicit(&top->dijkstra_runs, 1, memory_order_relaxed);
            int32_t ran = atomic_load_explicit(&top->src_loop[i], memory_order_acquire);
            int mine = 0;
            while (ran < A && !(mine = atomic_compare_exchange_weak_explicit(&top->src_loop[i], &ran, A,
                                                                             memory_order_acq_rel,
                                                                             memory_order_acquire))) {
            }
            const uint8_t* kr = m->kind + (size_t)i * A;
            const int32_t t0 = mine ? 0 : j, t1 = mine ? A : j + 1;
            /* the running minimum at the loop's start (0: none yet); a store at or above what
             * this loop has seen cannot lower the minimum, which only falls (other threads'
             * stores included), so only the others take the lock -- each lowering store makes
             * its own upcall, in store order, as _topology_storePathInCache does (:1374-1385) */
            pthread_mutex_lock(&top->min_lock);
            double seen = top->min_latency == 0 ? INFINITY : top->min_latency;
            pthread_mutex_unlock(&top->min_lock);
            noted = 1;
            for (int32_t t = t0; t < t1; t++) {
                /* the source itself: the igraph that returns [] for it stores nothing
                 * (topology.c:1815, the default rule); the one that returns [s] stores its
                 * self-loop path (self_rule) */
                if (t == i && !top->self_rule) continue;
                /* reachable targets only (an empty igraph path is never stored); a pair whose
                 * rule is the direct edge is not stored from a Dijkstra run */
                const uint8_t kt = cell_k(&kr[t]);
                if (kt == SHADOWTOPO_KIND_NONE || kt == SHADOWTOPO_KIND_DIRECT) continue;
                if (!cache_claim(top, i, t)) continue;
                const double l = cell_d(&m->lr[2 * ((size_t)i * A + t)]);
                if (l < seen) {
                    note_min_latency(top, l);
                    seen = l;
                }
                stored++;
            }
            /* [s] without a self-loop: _topology_computePathProperties fails for the source's
             * own target, so every Dijkstra run of s returns FALSE (:1857) after storing the
             * rest, and the query fails (:2040-2045) */
            if (top->self_rule && cell_k(&kr[i]) == SHADOWTOPO_KIND_NONE) success = 0;
        }
        if (stored) {
            atomic_fetch_add_explicit(&top->cached_paths, stored, memory_order_relaxed);
            if (!noted) note_min_latency(top, mn);
        }
        if (!success) return -1;
        d = cached_dir(top, i, j); /* (s, t), else (t, s), directed or not (:2033-2038) */
        if (!d) return -1;
    }
    *si = d == 1 ? i : j;
    *sj = d == 1 ? j : i;
    /* the entry's own row: a matrix whose rows [0, partial) still hold reverse copies in the
     * late attach's columns is swapped for the current one (filled before any of those
     * entries was cached) or filled now (an entry cached before the late attach) */
    int32_t p = atomic_load_explicit(&m->partial, memory_order_acquire);
    if (*si < p && *sj >= m->fill_col) {
        matrix* cur = atomic_load_explicit(&top->mat, memory_order_acquire);
        if (cur && cur->A > (*si > *sj ? *si : *sj)) *mp = m = cur;
        p = atomic_load_explicit(&m->partial, memory_order_acquire);
        if (*si < p && *sj >= m->fill_col && fill_old_rows(top, m)) return -1;
    }
    return 0;
}

static int32_t connected_vertex(Topology* top, Address* a) {
    /* _topology_getConnectedVertexIndex, topology.c:1388-1405, with no lock (ipt_get) */
    int32_t v = ipt_get(atomic_load_explicit(&top->ips, memory_order_acquire), address_toNetworkIP(a));
    if (v < 0) st_warning("address %s is not connected to the topology", address_toHostIPString(a));
    return v;
}

/* _topology_getPathEntry, topology.c:1969-2051: returns the matrix and pair offset */
static matrix* path_entry(Topology* top, Address* src, Address* dst, size_t* off, int32_t* ri, int32_t* rj,
                          int* srl) {
    int32_t vs = connected_vertex(top, src);
    if (vs < 0) {
        st_critical("invalid vertex %i, source address %s is not connected to topology", (int)vs,
                    address_toString(src));
        return NULL;
    }
    int32_t vd = connected_vertex(top, dst);
    if (vd < 0) {
        st_critical("invalid vertex %i, destination address %s is not connected to topology", (int)vd,
                    address_toString(dst));
        return NULL;
    }
    int32_t i = atomic_load_explicit(&top->att_index[vs], memory_order_acquire);
    int32_t j = atomic_load_explicit(&top->att_index[vd], memory_order_acquire);
    matrix* m = (i >= 0 && j >= 0) ? current_matrix(top, i > j ? i : j) : NULL;
    if (m) {
        /* a packet makes four calls on one pair (isRoutable, getLatency, getReliability,
         * increment; worker.c:267-279): start the pair's value line (either direction, the
         * cache decides which one holds it) and its counter on the first call, while the
         * cache cell is read, instead of three dependent DRAM misses */
        const size_t A = (size_t)m->A;
        __builtin_prefetch(&m->lr[2 * ((size_t)i * A + (size_t)j)]);
        __builtin_prefetch(&m->lr[2 * ((size_t)j * A + (size_t)i)]);
        const int32_t a = (!top->directed && j < i) ? j : i, b = a == i ? j : i;
        const uint64_t* ct = tile_peek(top->crow, top->ctd, a / CTILE, b / CTILE);
        if (ct) __builtin_prefetch(&ct[(a % CTILE) * CTILE + (b % CTILE)], 1);
    }
    int32_t si, sj;
    if (m && cache_resolve(top, &m, i, j, &si, &sj) == 0) {
        *off = (size_t)si * (size_t)m->A + (size_t)sj;
        if (ri) *ri = si;
        if (rj) *rj = sj;
        if (srl) *srl = si == sj && m->srl_lat && diag_self_rule(top, si);
        return m;
    }
    st_error("unable to find path between node %s at %s (vertex %i) and node %s at %s (vertex %i)",
             address_toString(src), vid(top, vs), (int)vs, address_toString(dst), vid(top, vd), (int)vd);
    return NULL;
}

double topology_getLatency(Topology* top, Address* srcAddress, Address* dstAddress) {
    size_t o;
    int32_t i;
    int srl = 0;
    matrix* m = path_entry(top, srcAddress, dstAddress, &o, &i, NULL, &srl);
    return m ? (srl ? m->srl_lat[i] : cell_d(&m->lr[2 * o])) : -1.0;
}

double topology_getReliability(Topology* top, Address* srcAddress, Address* dstAddress) {
    size_t o;
    int32_t i;
    int srl = 0;
    matrix* m = path_entry(top, srcAddress, dstAddress, &o, &i, NULL, &srl);
    return m ? (srl ? m->srl_rel[i] : cell_d(&m->lr[2 * o + 1])) : -1.0;
}

int topology_isRoutable(Topology* top, Address* srcAddress, Address* dstAddress) {
    return topology_getLatency(top, srcAddress, dstAddress) > -1 ? 1 : 0;
}

void topology_incrementPathPacketCounter(Topology* top, Address* srcAddress, Address* dstAddress) {
    size_t o;
    int32_t i, j;
    matrix* m = path_entry(top, srcAddress, dstAddress, &o, &i, &j, NULL);
    if (!m) {
        st_error("unable to find path between node %s and node %s", address_toString(srcAddress),
                 address_toString(dstAddress));
        return;
    }
    _Atomic uint64_t* c = counter_slot(top, i, j);
    if (!c) return;
    uint64_t expect = atomic_load_explicit(c, memory_order_relaxed);
    if (expect == 0) {
        /* first touch: 0 -> 2 (touched + one packet) */
        if (atomic_compare_exchange_strong(c, &expect, 2)) return;
    }
    atomic_fetch_add_explicit(c, 1, memory_order_relaxed);
}
/* ------------------------------------------------------------ extensions */
int topology_hip_set_device(Topology* top, int32_t device) {
    if (!top || top->eng) return -1;
    top->device = device;
    top->ndev = 1;
    top->devices[0] = device;
    return 0;
}

int topology_hip_set_devices(Topology* top, const int32_t* devices, int32_t count) {
    if (!top || top->eng || !devices || count < 1 || count > SHADOWTOPO_MAX_DEVICES) return -1;
    for (int32_t k = 0; k < count; k++) top->devices[k] = devices[k];
    top->ndev = count;
    top->device = devices[0];
    return 0;
}

int topology_hip_set_self_rule(Topology* top, int32_t dijkstra_loop) {
    if (!top || top->eng) return -1;
    top->self_rule = dijkstra_loop ? 1 : 0;
    return 0;
}

int topology_hip_prepare(Topology* top) {
    if (!top) return -1;
    if (top->n_att == 0) return 0;
    return current_matrix(top, top->n_att - 1) ? 0 : -1;
}

int topology_hip_get_info(Topology* top, topology_hip_info* out) {
    if (!top || !out) return -1;
    memset(out, 0, sizeof *out);
    out->n_vertices = top->V;
    out->n_edges = top->E;
    out->is_directed = top->directed;
    out->is_complete = top->complete;
    out->is_connected = top->connected;
    out->cluster_count = top->clusters;
    out->prefers_direct_paths = top->prefer_direct;
    out->n_attached = top->n_att;
    matrix* m = atomic_load(&top->mat);
    out->computed_for = m ? m->A : 0;
    out->device = top->device;
    out->n_devices = top->ndev;
    pthread_mutex_lock(&top->min_lock);
    out->min_path_latency = top->min_latency;
    pthread_mutex_unlock(&top->min_lock);
    out->compute_seconds = top->compute_s;
    out->compute_count = top->compute_count;
    out->dijkstra_runs = atomic_load(&top->dijkstra_runs);
    out->self_path_count = atomic_load(&top->self_count);
    out->cached_paths = atomic_load(&top->cached_paths);
    shadowtopo_stats est;
    for (int32_t k = 0; k < top->ndev; k++)
        if (top->engs[k] && shadowtopo_get_stats(top->engs[k], &est) == SHADOWTOPO_OK)
            out->self_seconds += est.self_ms * 1e-3;
    out->compute_failed = top->compute_failed;
    pthread_rwlock_rdlock(&top->ip_lock);
    const iptab* it = atomic_load(&top->ips);
    out->ip_table_slots = it ? (int64_t)it->cap : 0;
    out->ip_tables_retired = (int64_t)top->ips_nretired;
    for (const iptab* r = top->ips_retired; r; r = r->next) out->ip_retired_bytes += (int64_t)(sizeof(iptab) + r->cap * 8);
    pthread_rwlock_unlock(&top->ip_lock);
    return 0;
}

int32_t topology_hip_attached(Topology* top, int32_t* out, int32_t cap) {
    if (!top) return -1;
    int32_t n = top->n_att < cap ? top->n_att : cap;
    if (out && n > 0) memcpy(out, top->attached, sizeof(int32_t) * (size_t)n);
    return top->n_att;
}

int32_t topology_hip_vertex_of_ip(Topology* top, uint32_t ip) {
    if (!top) return -1;
    int32_t v = ipt_get(atomic_load_explicit(&top->ips, memory_order_acquire), ip);
    return v;
}

int32_t topology_hip_vertex_of_id(Topology* top, const char* id) {
    if (!top || !id) return -1;
    for (int32_t v = 0; v < top->V; v++)
        if (!strcmp(top->gml->node_ids[v], id)) return v;
    return -1;
}

uint64_t topology_hip_packet_count(Topology* top, int32_t src_vertex, int32_t dst_vertex) {
    if (!top || src_vertex < 0 || dst_vertex < 0 || src_vertex >= top->V || dst_vertex >= top->V) return 0;
    int32_t i = atomic_load(&top->att_index[src_vertex]), j = atomic_load(&top->att_index[dst_vertex]);
    if (i < 0 || j < 0) return 0;
    uint64_t c = counter_peek(top, i, j);
    return c ? c - 1 : 0;
}

int32_t topology_hip_cached_cell(Topology* top, int32_t src_vertex, int32_t dst_vertex) {
    if (!top || src_vertex < 0 || dst_vertex < 0 || src_vertex >= top->V || dst_vertex >= top->V) return -1;
    int32_t i = atomic_load(&top->att_index[src_vertex]), j = atomic_load(&top->att_index[dst_vertex]);
    if (i < 0 || j < 0) return -1;
    int sh;
    const int32_t a = i < j ? i : j, b = i < j ? j : i;
    _Atomic uint64_t* w = cell_word(top, a, b, 0, &sh);
    const unsigned c = w ? (unsigned)((atomic_load_explicit(w, memory_order_acquire) >> sh) & 3u) : 0u;
    if (i <= j) return (int32_t)c;
    return (int32_t)(((c & 1u) << 1) | ((c >> 1) & 1u)); /* bit 0 = (src, dst) */
}

int topology_hip_edges(Topology* top, const int32_t** src, const int32_t** dst, const double** latency,
                       const double** packetloss, const double** vertex_packetloss) {
    if (!top) return -1;
    if (src) *src = top->gml->src;
    if (dst) *dst = top->gml->dst;
    if (latency) *latency = top->elat;
    if (packetloss) *packetloss = top->eloss;
    if (vertex_packetloss) *vertex_packetloss = top->vloss;
    return 0;
}
