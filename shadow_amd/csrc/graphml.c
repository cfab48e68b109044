/*
 * graphml.c -- streaming GraphML reader (see graphml.h for the igraph semantics it keeps).
 * A single forward scan over the file buffer: no DOM, no libxml2; node ids are interned
 * in an open-addressing hash, data values go straight into per-attribute columns.
 */
#define _GNU_SOURCE
#include "graphml.h"

#include <ctype.h>
#include <errno.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

/* ------------------------------------------------------------ string -> id hash */
typedef struct {
    char** keys;
    int32_t* vals;
    uint64_t* hs;  /* each key's hash: probes compare it before the string (one miss, not two) */
    size_t cap;
    size_t n;
} strhash;

static uint64_t fnv1a(const char* s, size_t len) {
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 0; i < len; i++) {
        h ^= (unsigned char)s[i];
        h *= 1099511628211ULL;
    }
    return h;
}

static int sh_grow(strhash* h) {
    size_t ncap = h->cap ? h->cap * 2 : 1024;
    char** nk = (char**)calloc(ncap, sizeof(char*));
    int32_t* nv = (int32_t*)calloc(ncap, sizeof(int32_t));
    uint64_t* nh = (uint64_t*)calloc(ncap, sizeof(uint64_t));
    if (!nk || !nv || !nh) {
        free(nk);
        free(nv);
        free(nh);
        return -1;
    }
    for (size_t i = 0; i < h->cap; i++) {
        if (!h->keys[i]) continue;
        size_t j = h->hs[i] & (ncap - 1);
        while (nk[j]) j = (j + 1) & (ncap - 1);
        nk[j] = h->keys[i];
        nv[j] = h->vals[i];
        nh[j] = h->hs[i];
    }
    free(h->keys);
    free(h->vals);
    free(h->hs);
    h->keys = nk;
    h->vals = nv;
    h->hs = nh;
    h->cap = ncap;
    return 0;
}

/* returns the id for key s (inserting `next` if absent); *inserted set accordingly, and
 * *key the table's own copy of the string */
static int sh_intern(strhash* h, const char* s, int32_t next, int32_t* out, int* inserted, char** key) {
    if ((h->n + 1) * 2 > h->cap && sh_grow(h)) return -1;
    const size_t len = strlen(s);
    const uint64_t hv = fnv1a(s, len);
    size_t j = hv & (h->cap - 1);
    while (h->keys[j]) {
        if (h->hs[j] == hv && strcmp(h->keys[j], s) == 0) {
            *out = h->vals[j];
            *inserted = 0;
            *key = h->keys[j];
            return 0;
        }
        j = (j + 1) & (h->cap - 1);
    }
    h->keys[j] = (char*)malloc(len + 1);
    if (!h->keys[j]) return -1;
    memcpy(h->keys[j], s, len + 1);
    h->vals[j] = next;
    h->hs[j] = hv;
    h->n++;
    *out = next;
    *inserted = 1;
    *key = h->keys[j];
    return 0;
}

static void sh_free(strhash* h) {
    /* keys are owned by node_ids */
    free(h->keys);
    free(h->vals);
    free(h->hs);
}

/* ------------------------------------------------------------ growable text */
typedef struct {
    char* s;
    size_t n, cap;
} sbuf;

static int sb_add(sbuf* b, const char* p, size_t len) {
    if (b->n + len + 1 > b->cap) {
        size_t nc = b->cap ? b->cap * 2 : 256;
        while (nc < b->n + len + 1) nc *= 2;
        char* ns = (char*)realloc(b->s, nc);
        if (!ns) return -1;
        b->s = ns;
        b->cap = nc;
    }
    memcpy(b->s + b->n, p, len);
    b->n += len;
    b->s[b->n] = 0;
    return 0;
}

/* decode XML entities in place-copy */
static int sb_add_decoded(sbuf* b, const char* p, size_t len) {
    size_t i = 0;
    while (i < len) {
        if (p[i] == '&') {
            const char* semi = memchr(p + i, ';', len - i);
            if (semi) {
                size_t el = (size_t)(semi - (p + i)) + 1;
                char tmp[8];
                size_t tl = 0;
                if (el == 4 && !strncmp(p + i, "&lt;", 4)) {
                    tmp[0] = '<';
                    tl = 1;
                } else if (el == 4 && !strncmp(p + i, "&gt;", 4)) {
                    tmp[0] = '>';
                    tl = 1;
                } else if (el == 5 && !strncmp(p + i, "&amp;", 5)) {
                    tmp[0] = '&';
                    tl = 1;
                } else if (el == 6 && !strncmp(p + i, "&quot;", 6)) {
                    tmp[0] = '"';
                    tl = 1;
                } else if (el == 6 && !strncmp(p + i, "&apos;", 6)) {
                    tmp[0] = '\'';
                    tl = 1;
                } else if (el > 3 && p[i + 1] == '#') {
                    unsigned long cp = (p[i + 2] == 'x' || p[i + 2] == 'X') ? strtoul(p + i + 3, NULL, 16)
                                                                           : strtoul(p + i + 2, NULL, 10);
                    if (cp < 0x80) {
                        tmp[tl++] = (char)cp;
                    } else if (cp < 0x800) {
                        tmp[tl++] = (char)(0xC0 | (cp >> 6));
                        tmp[tl++] = (char)(0x80 | (cp & 0x3F));
                    } else if (cp < 0x10000) {
                        tmp[tl++] = (char)(0xE0 | (cp >> 12));
                        tmp[tl++] = (char)(0x80 | ((cp >> 6) & 0x3F));
                        tmp[tl++] = (char)(0x80 | (cp & 0x3F));
                    } else {
                        tmp[tl++] = (char)(0xF0 | (cp >> 18));
                        tmp[tl++] = (char)(0x80 | ((cp >> 12) & 0x3F));
                        tmp[tl++] = (char)(0x80 | ((cp >> 6) & 0x3F));
                        tmp[tl++] = (char)(0x80 | (cp & 0x3F));
                    }
                }
                if (tl) {
                    if (sb_add(b, tmp, tl)) return -1;
                    i += el;
                    continue;
                }
            }
        }
        size_t j = i + 1;
        while (j < len && p[j] != '&') j++;
        if (sb_add(b, p + i, j - i)) return -1;
        i = j;
    }
    return 0;
}

/* ------------------------------------------------------------ parser */
typedef struct {
    char* id;
    char* name;
    int type;
    int domains;
    int has_default;
    char* def;
} keydef;

typedef struct {
    const char* p;
    const char* end;
    gml_graph* g;
    strhash ids;
    int64_t ids_cap;
    keydef* keys;
    int nkeys, capkeys;
    int in_graph;        /* inside the first <graph> */
    int graph_done;
    int skip_depth;      /* nested (hierarchical) graph content is ignored */
    int cur_dom;         /* GML_NODE / GML_EDGE / GML_GRAPH of the element owning <data> */
    int64_t cur_idx;
    int in_data;
    sbuf data_key;       /* key of the open <data> (reused buffer) */
    sbuf tagbuf;         /* the current tag's attribute names and values (reused buffer) */
    int in_key;          /* index into keys while inside <key> */
    int in_default;
    sbuf text;
    int64_t edge_cap;
    char* err;
    size_t errlen;
} pstate;

static int perr(pstate* s, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(s->err, s->errlen, fmt, ap);
    va_end(ap);
    return -1;
}

static const char* local_name(const char* n) {
    const char* c = strrchr(n, ':');
    return c ? c + 1 : n;
}

/* A parsed tag.  Attribute names and decoded values live in the parser's reusable tag
 * buffer (NUL-separated), so a tag costs no allocation: the file's ~3e7 attributes of a
 * C5-sized topology took two mallocs and two frees each when every string was its own
 * allocation. */
typedef struct {
    char name[64];
    int nattr;
    const char* an[16];
    const char* av[16];
    int self_close;
    int is_end;
} tag;

static const char* tag_get(const tag* t, const char* name) {
    for (int i = 0; i < t->nattr; i++)
        if (!strcmp(local_name(t->an[i]), name)) return t->av[i];
    return NULL;
}

/* parse a tag starting after '<'; s->p points at the name (or '/') */
static int parse_tag(pstate* s, tag* t) {
    t->nattr = 0;
    t->self_close = 0;
    t->is_end = 0;
    sbuf* tb = &s->tagbuf;
    tb->n = 0;
    size_t aoff[16], voff[16];
    const char* p = s->p;
    if (p < s->end && *p == '/') {
        t->is_end = 1;
        p++;
    }
    size_t k = 0;
    while (p < s->end && !isspace((unsigned char)*p) && *p != '>' && *p != '/') {
        if (k + 1 < sizeof t->name) t->name[k++] = *p;
        p++;
    }
    t->name[k] = 0;
    for (;;) {
        while (p < s->end && isspace((unsigned char)*p)) p++;
        if (p >= s->end) return perr(s, "unterminated tag <%s", t->name);
        if (*p == '>') {
            p++;
            break;
        }
        if (*p == '/' && p + 1 < s->end && p[1] == '>') {
            t->self_close = 1;
            p += 2;
            break;
        }
        const char* an = p;
        while (p < s->end && *p != '=' && !isspace((unsigned char)*p) && *p != '>') p++;
        size_t anl = (size_t)(p - an);
        while (p < s->end && isspace((unsigned char)*p)) p++;
        if (p >= s->end || *p != '=') return perr(s, "malformed attribute in <%s", t->name);
        p++;
        while (p < s->end && isspace((unsigned char)*p)) p++;
        if (p >= s->end || (*p != '"' && *p != '\'')) return perr(s, "unquoted attribute in <%s", t->name);
        char q = *p++;
        const char* av = p;
        while (p < s->end && *p != q) p++;
        if (p >= s->end) return perr(s, "unterminated attribute value in <%s", t->name);
        if (t->nattr < 16) {
            /* name NUL value NUL, as offsets: the buffer may move while it grows */
            aoff[t->nattr] = tb->n;
            if (sb_add(tb, an, anl)) return perr(s, "out of memory");
            tb->n++;
            voff[t->nattr] = tb->n;
            if (sb_add_decoded(tb, av, (size_t)(p - av)) || sb_add(tb, "", 0)) return perr(s, "out of memory");
            tb->n++;
            t->nattr++;
        }
        p++;
    }
    for (int i = 0; i < t->nattr; i++) {
        t->an[i] = tb->s + aoff[i];
        t->av[i] = tb->s + voff[i];
    }
    s->p = p;
    return 0;
}

int gml_strtod(const char* s, double* out); /* numparse.cpp: strtod's value, faster */

static double parse_num(const char* txt, double def) {
    if (!txt) return def;
    while (*txt && isspace((unsigned char)*txt)) txt++;
    if (!*txt) return def;
    double v;
    return gml_strtod(txt, &v) ? v : def;
}

static int parse_bool(const char* txt, double def) {
    if (!txt) return (int)def;
    while (*txt && isspace((unsigned char)*txt)) txt++;
    if (!*txt) return (int)def;
    if (!strncasecmp(txt, "true", 4) || !strncasecmp(txt, "yes", 3) || !strncmp(txt, "1", 1)) return 1;
    return 0;
}

static int attr_reserve(gml_attr* a, int64_t need) {
    if (need <= a->cap) return 0;
    int64_t nc = a->cap ? a->cap : 1024;
    while (nc < need) nc *= 2;
    if (a->type == GML_STRING) {
        char** ns = (char**)realloc(a->str, sizeof(char*) * (size_t)nc);
        if (!ns) return -1;
        for (int64_t i = a->cap; i < nc; i++) ns[i] = NULL;
        a->str = ns;
    } else {
        double* nn = (double*)realloc(a->num, sizeof(double) * (size_t)nc);
        if (!nn) return -1;
        for (int64_t i = a->cap; i < nc; i++) nn[i] = a->num_default;
        a->num = nn;
    }
    a->cap = nc;
    return 0;
}

static int add_attr(pstate* s, const keydef* k, int dom) {
    gml_graph* g = s->g;
    gml_attr* na = (gml_attr*)realloc(g->attrs, sizeof(gml_attr) * (size_t)(g->nattr + 1));
    if (!na) return perr(s, "out of memory");
    g->attrs = na;
    gml_attr* a = &g->attrs[g->nattr++];
    memset(a, 0, sizeof *a);
    a->name = strdup(k->name);
    a->key_id = strdup(k->id);
    a->type = k->type;
    a->domain = dom;
    a->has_default = k->has_default;
    if (k->type == GML_STRING) {
        a->str_default = strdup(k->has_default && k->def ? k->def : "");
        a->num_default = NAN;
    } else if (k->type == GML_BOOLEAN) {
        a->num_default = k->has_default ? (double)parse_bool(k->def, 0) : 0.0;
    } else {
        a->num_default = k->has_default ? parse_num(k->def, NAN) : NAN;
    }
    if (dom == GML_GRAPH && attr_reserve(a, 1)) return perr(s, "out of memory");
    return 0;
}

static int finish_key(pstate* s, int ki) {
    keydef* k = &s->keys[ki];
    if (k->domains & GML_GRAPH && add_attr(s, k, GML_GRAPH)) return -1;
    if (k->domains & GML_NODE && add_attr(s, k, GML_NODE)) return -1;
    if (k->domains & GML_EDGE && add_attr(s, k, GML_EDGE)) return -1;
    return 0;
}

static int vertex_of(pstate* s, const char* name, int32_t* out) {
    gml_graph* g = s->g;
    int ins = 0;
    char* key = NULL;
    if (sh_intern(&s->ids, name, g->n, out, &ins, &key)) return perr(s, "out of memory");
    if (ins) {
        if (g->n >= s->ids_cap) {
            int64_t nc = s->ids_cap ? s->ids_cap * 2 : 1024;
            char** ni = (char**)realloc(g->node_ids, sizeof(char*) * (size_t)nc);
            if (!ni) return perr(s, "out of memory");
            g->node_ids = ni;
            s->ids_cap = nc;
        }
        /* the hash owns one copy; node_ids shares it */
        g->node_ids[g->n] = key;
        g->n++;
    }
    return 0;
}

static int store_data(pstate* s) {
    const char* txt = s->text.s ? s->text.s : "";
    const char* dk = s->data_key.s ? s->data_key.s : "";
    for (int i = 0; i < s->g->nattr; i++) {
        gml_attr* a = &s->g->attrs[i];
        if (a->domain != s->cur_dom || strcmp(a->key_id, dk)) continue;
        int64_t idx = s->cur_dom == GML_GRAPH ? 0 : s->cur_idx;
        if (attr_reserve(a, idx + 1)) return perr(s, "out of memory");
        if (a->type == GML_STRING) {
            free(a->str[idx]);
            a->str[idx] = strdup(txt);
        } else if (a->type == GML_BOOLEAN) {
            a->num[idx] = (double)parse_bool(txt, a->num_default);
        } else {
            a->num[idx] = parse_num(txt, a->num_default);
        }
        return 0;
    }
    return 0; /* undeclared key: igraph warns and ignores */
}

static int handle_start(pstate* s, tag* t) {
    const char* n = local_name(t->name);
    if (s->skip_depth > 0) {
        if (!t->self_close && !strcmp(n, "graph")) s->skip_depth++;
        return 0;
    }
    if (!strcmp(n, "key")) {
        if (s->nkeys == s->capkeys) {
            int nc = s->capkeys ? s->capkeys * 2 : 16;
            keydef* nk = (keydef*)realloc(s->keys, sizeof(keydef) * (size_t)nc);
            if (!nk) return perr(s, "out of memory");
            s->keys = nk;
            s->capkeys = nc;
        }
        keydef* k = &s->keys[s->nkeys];
        memset(k, 0, sizeof *k);
        const char* id = tag_get(t, "id");
        const char* an = tag_get(t, "attr.name");
        const char* at = tag_get(t, "attr.type");
        const char* fo = tag_get(t, "for");
        k->id = strdup(id ? id : "");
        k->name = strdup(an ? an : (id ? id : ""));
        if (!at || !strcmp(at, "string"))
            k->type = GML_STRING;
        else if (!strcmp(at, "boolean"))
            k->type = GML_BOOLEAN;
        else if (!strcmp(at, "int") || !strcmp(at, "long") || !strcmp(at, "float") || !strcmp(at, "double"))
            k->type = GML_NUMERIC;
        else
            k->type = GML_STRING;
        if (!fo || !strcmp(fo, "all"))
            k->domains = GML_GRAPH | GML_NODE | GML_EDGE;
        else if (!strcmp(fo, "node"))
            k->domains = GML_NODE;
        else if (!strcmp(fo, "edge"))
            k->domains = GML_EDGE;
        else if (!strcmp(fo, "graph"))
            k->domains = GML_GRAPH;
        else
            k->domains = 0;
        s->nkeys++;
        if (t->self_close) return finish_key(s, s->nkeys - 1);
        s->in_key = s->nkeys;
        return 0;
    }
    if (!strcmp(n, "default") && s->in_key) {
        s->in_default = 1;
        s->text.n = 0;
        if (s->text.s) s->text.s[0] = 0;
        if (t->self_close) {
            s->keys[s->in_key - 1].has_default = 1;
            s->keys[s->in_key - 1].def = strdup("");
            s->in_default = 0;
        }
        return 0;
    }
    if (!strcmp(n, "graph")) {
        if (s->in_graph || s->graph_done) {
            if (!t->self_close) s->skip_depth = 1;
            return 0;
        }
        const char* ed = tag_get(t, "edgedefault");
        s->g->directed = !(ed && !strcmp(ed, "undirected"));
        if (t->self_close) {
            s->graph_done = 1;
            return 0;
        }
        s->in_graph = 1;
        s->cur_dom = GML_GRAPH;
        s->cur_idx = 0;
        return 0;
    }
    if (!s->in_graph) return 0;
    if (!strcmp(n, "node")) {
        const char* id = tag_get(t, "id");
        if (!id) return perr(s, "<node> without id");
        int32_t v;
        if (vertex_of(s, id, &v)) return -1;
        if (!t->self_close) {
            s->cur_dom = GML_NODE;
            s->cur_idx = v;
        }
        return 0;
    }
    if (!strcmp(n, "edge")) {
        const char* a = tag_get(t, "source");
        const char* b = tag_get(t, "target");
        if (!a || !b) return perr(s, "<edge> without source/target");
        int32_t va, vb;
        if (vertex_of(s, a, &va) || vertex_of(s, b, &vb)) return -1;
        gml_graph* g = s->g;
        if (g->m >= s->edge_cap) {
            int64_t nc = s->edge_cap ? s->edge_cap * 2 : 4096;
            int32_t* ns = (int32_t*)realloc(g->src, sizeof(int32_t) * (size_t)nc);
            if (!ns) return perr(s, "out of memory");
            g->src = ns;
            int32_t* nd = (int32_t*)realloc(g->dst, sizeof(int32_t) * (size_t)nc);
            if (!nd) return perr(s, "out of memory");
            g->dst = nd;
            s->edge_cap = nc;
        }
        g->src[g->m] = va;
        g->dst[g->m] = vb;
        if (!t->self_close) {
            s->cur_dom = GML_EDGE;
            s->cur_idx = g->m;
        }
        g->m++;
        return 0;
    }
    if (!strcmp(n, "data")) {
        const char* k = tag_get(t, "key");
        s->data_key.n = 0;
        if (sb_add(&s->data_key, k ? k : "", k ? strlen(k) : 0)) return perr(s, "out of memory");
        s->text.n = 0;
        if (s->text.s) s->text.s[0] = 0;
        if (t->self_close) return store_data(s);
        s->in_data = 1;
        return 0;
    }
    return 0;
}

static int handle_end(pstate* s, const char* name) {
    const char* n = local_name(name);
    if (s->skip_depth > 0) {
        if (!strcmp(n, "graph")) s->skip_depth--;
        return 0;
    }
    if (!strcmp(n, "default") && s->in_default) {
        keydef* k = &s->keys[s->in_key - 1];
        k->has_default = 1;
        free(k->def);
        k->def = strdup(s->text.s ? s->text.s : "");
        s->in_default = 0;
        return 0;
    }
    if (!strcmp(n, "key") && s->in_key) {
        int ki = s->in_key - 1;
        s->in_key = 0;
        return finish_key(s, ki);
    }
    if (!strcmp(n, "data") && s->in_data) {
        s->in_data = 0;
        return store_data(s);
    }
    if ((!strcmp(n, "node") || !strcmp(n, "edge")) && s->in_graph) {
        s->cur_dom = GML_GRAPH;
        s->cur_idx = 0;
        return 0;
    }
    if (!strcmp(n, "graph") && s->in_graph) {
        s->in_graph = 0;
        s->graph_done = 1;
    }
    return 0;
}

int gml_parse_buffer(const char* buf, size_t len, gml_graph** out, char* err, size_t errlen) {
    pstate s;
    memset(&s, 0, sizeof s);
    char dummy[8];
    s.err = err ? err : dummy;
    s.errlen = err ? errlen : sizeof dummy;
    s.p = buf;
    s.end = buf + len;
    s.g = (gml_graph*)calloc(1, sizeof(gml_graph));
    if (!s.g) return perr(&s, "out of memory");
    s.g->directed = 1;
    int rc = 0;
    int saw_graph = 0;
    while (s.p < s.end && rc == 0) {
        const char* lt = memchr(s.p, '<', (size_t)(s.end - s.p));
        const char* stop = lt ? lt : s.end;
        if ((s.in_data || s.in_default) && stop > s.p) rc = sb_add_decoded(&s.text, s.p, (size_t)(stop - s.p));
        if (!lt || rc) break;
        s.p = lt + 1;
        if (s.p < s.end && *s.p == '?') {
            const char* e = strstr(s.p, "?>");
            s.p = e ? e + 2 : s.end;
        } else if (s.end - s.p >= 3 && !strncmp(s.p, "!--", 3)) {
            const char* e = strstr(s.p, "-->");
            s.p = e ? e + 3 : s.end;
        } else if (s.end - s.p >= 8 && !strncmp(s.p, "![CDATA[", 8)) {
            const char* b = s.p + 8;
            const char* e = strstr(b, "]]>");
            if (!e) {
                rc = perr(&s, "unterminated CDATA");
                break;
            }
            if (s.in_data || s.in_default) rc = sb_add(&s.text, b, (size_t)(e - b));
            s.p = e + 3;
        } else if (s.p < s.end && *s.p == '!') {
            const char* e = memchr(s.p, '>', (size_t)(s.end - s.p));
            s.p = e ? e + 1 : s.end;
        } else {
            tag t;
            rc = parse_tag(&s, &t);
            if (rc == 0) {
                if (!strcmp(local_name(t.name), "graph") && !t.is_end) saw_graph = 1;
                rc = t.is_end ? handle_end(&s, t.name) : handle_start(&s, &t);
            }
        }
    }
    free(s.text.s);
    free(s.data_key.s);
    free(s.tagbuf.s);
    for (int i = 0; i < s.nkeys; i++) {
        free(s.keys[i].id);
        free(s.keys[i].name);
        free(s.keys[i].def);
    }
    free(s.keys);
    sh_free(&s.ids);
    if (rc == 0 && !saw_graph) rc = perr(&s, "no <graph> element");
    if (rc) {
        gml_free(s.g);
        return -1;
    }
    *out = s.g;
    return 0;
}

int gml_parse_file(const char* path, gml_graph** out, char* err, size_t errlen) {
    FILE* f = fopen(path, "rb");
    if (!f) {
        snprintf(err, errlen, "fopen('%s'): %s", path, strerror(errno));
        return -1;
    }
    if (fseek(f, 0, SEEK_END) != 0) {
        fclose(f);
        snprintf(err, errlen, "fseek failed");
        return -1;
    }
    long sz = ftell(f);
    rewind(f);
    char* buf = (char*)malloc((size_t)sz + 1);
    if (!buf) {
        fclose(f);
        snprintf(err, errlen, "out of memory (%ld bytes)", sz);
        return -1;
    }
    size_t rd = fread(buf, 1, (size_t)sz, f);
    fclose(f);
    buf[rd] = 0;
    int rc = gml_parse_buffer(buf, rd, out, err, errlen);
    free(buf);
    return rc;
}

void gml_free(gml_graph* g) {
    if (!g) return;
    for (int i = 0; i < g->nattr; i++) {
        gml_attr* a = &g->attrs[i];
        if (a->str)
            for (int64_t k = 0; k < a->cap; k++) free(a->str[k]);
        free(a->str);
        free(a->num);
        free(a->name);
        free(a->key_id);
        free(a->str_default);
    }
    free(g->attrs);
    if (g->node_ids)
        for (int32_t v = 0; v < g->n; v++) free(g->node_ids[v]);
    free(g->node_ids);
    free(g->src);
    free(g->dst);
    free(g);
}

const gml_attr* gml_find(const gml_graph* g, int domain, const char* name) {
    if (domain == GML_NODE && !strcmp(name, "id")) return NULL; /* handled by node_ids */
    for (int i = 0; i < g->nattr; i++)
        if (g->attrs[i].domain == domain && !strcmp(g->attrs[i].name, name)) return &g->attrs[i];
    return NULL;
}

const char* gml_str(const gml_attr* a, int64_t i) {
    if (!a) return "";
    if (a->type != GML_STRING) return "";
    if (i < a->cap && a->str[i]) return a->str[i];
    return a->str_default ? a->str_default : "";
}

double gml_num(const gml_attr* a, int64_t i) {
    if (!a) return NAN;
    if (a->type == GML_STRING) return NAN;
    if (i < a->cap) return a->num[i];
    return a->num_default;
}
