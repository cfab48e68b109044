/*
 * graphml.h -- streaming GraphML reader for the topology shim.
 *
 * Replaces igraph_read_graph_graphml + the igraph C attribute table as used by
 * _topology_loadGraph (/root/reference/src/main/routing/topology.c:371-399):
 *   - vertex index = order of first appearance of a node id (<node> or <edge> endpoint),
 *     edge index = <edge> element order (igraph's node trie);
 *   - the node id string is the string vertex attribute "id";
 *   - <key attr.type> int/long/float/double -> numeric (double), boolean -> boolean,
 *     string -> string; missing numeric = <default> or NaN, missing string = <default> or "";
 *   - only the first <graph> element is read (igraph's index 0).
 * Output goes straight to flat arrays (edge list + per-attribute columns).
 */
#ifndef SHADOWTOPO_GRAPHML_H
#define SHADOWTOPO_GRAPHML_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { GML_NUMERIC = 1, GML_STRING = 2, GML_BOOLEAN = 3 };
enum { GML_GRAPH = 1, GML_NODE = 2, GML_EDGE = 4 };

typedef struct gml_attr {
    char* name;      /* attr.name (or the key id if absent) */
    char* key_id;    /* GraphML key id */
    int type;        /* GML_NUMERIC / GML_STRING / GML_BOOLEAN */
    int domain;      /* GML_GRAPH / GML_NODE / GML_EDGE (one per attr; for="all" makes three) */
    int has_default;
    double num_default;
    char* str_default;
    /* per element values (vertex or edge domain); graph domain uses element 0 */
    double* num;     /* numeric / boolean */
    char** str;      /* string (NULL = default) */
    int64_t cap;
} gml_attr;

typedef struct gml_graph {
    int directed;
    int32_t n;
    int64_t m;
    int32_t* src;
    int32_t* dst;
    char** node_ids;
    int nattr;
    gml_attr* attrs;
} gml_graph;

/* returns 0 on success; on failure fills err */
int gml_parse_buffer(const char* buf, size_t len, gml_graph** out, char* err, size_t errlen);
int gml_parse_file(const char* path, gml_graph** out, char* err, size_t errlen);
void gml_free(gml_graph* g);

/* exact-name lookup (igraph_cattribute_has_attr semantics), NULL if absent */
const gml_attr* gml_find(const gml_graph* g, int domain, const char* name);
/* value accessors: string returns the stored value, default, or "" */
const char* gml_str(const gml_attr* a, int64_t i);
double gml_num(const gml_attr* a, int64_t i);

#ifdef __cplusplus
}
#endif

#endif
