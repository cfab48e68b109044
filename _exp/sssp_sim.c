// Offline model of batched (64 sources per wave) pull relaxation schedules on a CSR graph:
// counts rounds, (vertex, batch) visits, 512-B row reads and 64-B line reads per schedule,
// so alternatives to round-synchronous Bellman-Ford can be priced before writing kernels.
// usage: sssp_sim graph.bin nbatches delta_ms [mode]
// graph.bin: int32 V, int64 arcs, int64 ptr[V+1], int32 src[arcs], double w[arcs],
//            int32 nsrc, int32 sources[nsrc]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int32_t V;
static int64_t M;
static int64_t* ptr;
static int32_t* src;
static double* w;

#define KL 64

typedef struct {
    long rounds, visits, rows, lines, lane_visits, changes, scans, pendl, pendl16, lines16;
} stat_t;

static void report(const char* name, stat_t s, int nb) {
    printf("%-28s rounds %6ld  visits/vb %6.2f  rows/arcb %6.2f  lines/arcb(x8) %6.2f  lanevisits/vs %5.2f  changes/vs %5.2f\n",
           name, s.rounds, (double)s.visits / nb / V, (double)s.rows / nb / M, (double)s.lines / nb / M / 8.0,
           (double)s.lane_visits / nb / V / KL, (double)s.changes / nb / V / KL);
}

// Jacobi / Gauss-Seidel Bellman-Ford, activation = any in-neighbour changed in any lane
static stat_t bf(const int32_t* srcs, int gs) {
    stat_t st = {0};
    double* D = malloc(sizeof(double) * V * KL);
    double* Dn = malloc(sizeof(double) * V * KL);
    uint64_t* ch = calloc(V, 8);
    uint64_t* chn = calloc(V, 8);
    for (long i = 0; i < (long)V * KL; i++) D[i] = INFINITY;
    for (int l = 0; l < KL; l++)
        if (srcs[l] >= 0) {
            D[(long)srcs[l] * KL + l] = 0;
            ch[srcs[l]] |= 1ull << l;
        }
    for (;;) {
        memcpy(Dn, D, sizeof(double) * V * KL);
        double* R = gs ? Dn : D;
        int any = 0;
        memset(chn, 0, 8 * (size_t)V);
        for (int32_t v = 0; v < V; v++) {
            uint64_t need = 0;
            for (int64_t x = ptr[v]; x < ptr[v + 1]; x++) need |= ch[src[x]];
            if (gs)
                for (int64_t x = ptr[v]; x < ptr[v + 1]; x++) need |= chn[src[x]];
            if (!need) continue;
            st.visits++;
            st.rows += ptr[v + 1] - ptr[v];
            {
                int gq = 0, g16 = 0;
                for (int gI = 0; gI < 8; gI++)
                    if ((need >> (8 * gI)) & 0xff) gq++;
                for (int gI = 0; gI < 4; gI++)
                    if ((need >> (16 * gI)) & 0xffff) g16++;
                st.pendl += (ptr[v + 1] - ptr[v]) * gq;
                st.pendl16 += (ptr[v + 1] - ptr[v]) * g16;
            }
            for (int64_t x = ptr[v]; x < ptr[v + 1]; x++) {
                uint64_t cm = ch[src[x]] | (gs ? chn[src[x]] : 0);
                if (cm) st.scans++;  // changed-only pull: rows of changed tails
                for (int gI = 0; gI < 4; gI++)
                    if ((cm >> (16 * gI)) & 0xffff) st.lines16++;
                for (int gI = 0; gI < 8; gI++)
                    if ((cm >> (8 * gI)) & 0xff) st.lines++;
            }
            uint64_t m = 0;
            for (int l = 0; l < KL; l++) {
                if (srcs[l] == v) continue;
                double b = Dn[(long)v * KL + l];
                for (int64_t x = ptr[v]; x < ptr[v + 1]; x++) {
                    double c = R[(long)src[x] * KL + l] + w[x];
                    if (c < b) b = c;
                }
                if (b < Dn[(long)v * KL + l]) {
                    Dn[(long)v * KL + l] = b;
                    m |= 1ull << l;
                }
            }
            st.lane_visits += __builtin_popcountll(need);
            if (m) {
                chn[v] = m;
                any = 1;
                st.changes += __builtin_popcountll(m);
            }
        }
        st.rounds++;
        if (getenv("SIM_VERBOSE")) {
            static long pv = 0, pr = 0;
            printf("  round %ld visits %ld rows %ld\n", st.rounds, st.visits - pv, st.rows - pr);
            pv = st.visits;
            pr = st.rows;
        }
        memcpy(D, Dn, sizeof(double) * V * KL);
        uint64_t* t = ch;
        ch = chn;
        chn = t;
        if (!any) break;
    }
    free(D);
    free(Dn);
    free(ch);
    free(chn);
    return st;
}

// Bucketed pull (delta-stepping per lane): a changed (u, lane) propagates only once
// d(u) < T(lane); each lane's threshold advances by delta when it has no propagating pair
// left.  A destination is pulled for the lanes with a propagating in-neighbour; cost is
// counted as full rows (any lane) and as 64-B lines (8-lane groups with a lane).
static int g_shared = 0;
static stat_t bucket(const int32_t* srcs, double delta, int changed_only) {
    stat_t st = {0};
    double* D = malloc(sizeof(double) * V * KL);
    uint64_t* dirty = calloc(V, 8);
    uint64_t* prop = calloc(V, 8);
    double T[KL];
    for (long i = 0; i < (long)V * KL; i++) D[i] = INFINITY;
    for (int l = 0; l < KL; l++) {
        T[l] = delta;
        if (srcs[l] >= 0) {
            D[(long)srcs[l] * KL + l] = 0;
            dirty[srcs[l]] |= 1ull << l;
        }
    }
    for (;;) {
        // propagating set
        uint64_t lanes_with_prop = 0, lanes_with_dirty = 0;
        for (int32_t u = 0; u < V; u++) {
            uint64_t p = 0, d = dirty[u];
            lanes_with_dirty |= d;
            while (d) {
                int l = __builtin_ctzll(d);
                d &= d - 1;
                if (D[(long)u * KL + l] < T[l]) p |= 1ull << l;
            }
            prop[u] = p;
            lanes_with_prop |= p;
        }
        if (!lanes_with_dirty) break;
        // lanes without propagating pairs advance their threshold (a round with no work
        // for them; shared rounds count once)
        if (g_shared) {
            if (!lanes_with_prop)
                for (int l = 0; l < KL; l++) T[l] += delta;
            if (!lanes_with_prop) continue;
        }
        for (int l = 0; l < KL && !g_shared; l++)
            if (!((lanes_with_prop >> l) & 1) && ((lanes_with_dirty >> l) & 1)) {
                // jump straight to the next bucket holding a dirty pair of this lane
                double mn = INFINITY;
                for (int32_t u = 0; u < V; u++)
                    if ((dirty[u] >> l) & 1) mn = fmin(mn, D[(long)u * KL + l]);
                T[l] = (floor(mn / delta) + 1) * delta;
            }
        if (!lanes_with_prop) continue;  // thresholds moved, no round spent
        st.rounds++;
        for (int32_t u = 0; u < V; u++) dirty[u] &= ~prop[u];
        for (int32_t v = 0; v < V; v++) {
            uint64_t need = 0;
            long nch = 0;
            for (int64_t x = ptr[v]; x < ptr[v + 1]; x++) {
                need |= prop[src[x]];
                if (prop[src[x]]) nch++;
            }
            for (int l = 0; l < KL; l++)
                if (srcs[l] == v) need &= ~(1ull << l);
            if (!need) continue;
            st.visits++;
            st.scans += ptr[v + 1] - ptr[v];
            st.rows += changed_only ? nch : ptr[v + 1] - ptr[v];
            int groups = 0;
            for (int gI = 0; gI < 8; gI++)
                if ((need >> (8 * gI)) & 0xff) groups++;
            st.lines += (changed_only ? nch : ptr[v + 1] - ptr[v]) * groups;
            st.lane_visits += __builtin_popcountll(need);
            uint64_t m = need;
            while (m) {
                int l = __builtin_ctzll(m);
                m &= m - 1;
                double b = D[(long)v * KL + l];
                for (int64_t x = ptr[v]; x < ptr[v + 1]; x++)
                    if ((prop[src[x]] >> l) & 1) {
                        double c = D[(long)src[x] * KL + l] + w[x];
                        if (c < b) b = c;
                    }
                if (b < D[(long)v * KL + l]) {
                    D[(long)v * KL + l] = b;
                    dirty[v] |= 1ull << l;
                    st.changes++;
                }
            }
        }
    }
    free(D);
    free(dirty);
    free(prop);
    return st;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s graph.bin nbatches delta [mode]\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    int32_t nsrc;
    if (fread(&V, 4, 1, f) != 1 || fread(&M, 8, 1, f) != 1) return 1;
    ptr = malloc(8 * ((size_t)V + 1));
    src = malloc(4 * (size_t)M);
    w = malloc(8 * (size_t)M);
    if (fread(ptr, 8, V + 1, f) != (size_t)V + 1 || fread(src, 4, M, f) != (size_t)M ||
        fread(w, 8, M, f) != (size_t)M || fread(&nsrc, 4, 1, f) != 1)
        return 1;
    int32_t* sources = malloc(4 * (size_t)nsrc);
    if (fread(sources, 4, nsrc, f) != (size_t)nsrc) return 1;
    fclose(f);
    int nb = atoi(argv[2]);
    double delta = atof(argv[3]);
    const char* mode = argc > 4 ? argv[4] : "all";
    g_shared = getenv("SIM_SHARED") != NULL;
    int lanes = argc > 5 ? atoi(argv[5]) : KL;  // sources per batch (rest of the lanes idle)
    int32_t* s2 = malloc(4 * (size_t)nb * KL);
    for (int b = 0; b < nb; b++)
        for (int l = 0; l < KL; l++) s2[b * KL + l] = l < lanes ? sources[(size_t)b * lanes + l] : -1;
    sources = s2;
    printf("V=%d arcs=%ld batches=%d delta=%g\n", V, (long)M, nb, delta);
    stat_t acc[4];
    memset(acc, 0, sizeof acc);
    for (int b = 0; b < nb; b++) {
        const int32_t* s = sources + (size_t)b * KL;
        stat_t r[4];
        memset(r, 0, sizeof r);
        if (strstr(mode, "all") || strstr(mode, "bf")) r[0] = bf(s, 0);
        if (strstr(mode, "all") || strstr(mode, "gs")) r[1] = bf(s, 1);
        if (strstr(mode, "all") || strstr(mode, "bk")) r[2] = bucket(s, delta, 0);
        if (strstr(mode, "all") || strstr(mode, "bc")) r[3] = bucket(s, delta, 1);
        for (int k = 0; k < 4; k++) {
            acc[k].rounds = acc[k].rounds > r[k].rounds ? acc[k].rounds : r[k].rounds;
            acc[k].visits += r[k].visits;
            acc[k].rows += r[k].rows;
            acc[k].lines += r[k].lines;
            acc[k].lane_visits += r[k].lane_visits;
            acc[k].changes += r[k].changes;
            acc[k].scans += r[k].scans;
            acc[k].pendl += r[k].pendl;
            acc[k].pendl16 += r[k].pendl16;
            acc[k].lines16 += r[k].lines16;
        }
    }
    printf("BF jacobi changed-only rows/arcb %.2f lines(x8) %.2f; GS %.2f %.2f\n", (double)acc[0].scans / nb / M,
           (double)acc[0].lines / nb / M / 8.0, (double)acc[1].scans / nb / M, (double)acc[1].lines / nb / M / 8.0);
    for (int k = 0; k < 2; k++)
        printf("%s: pend-masked f64 lines(x8) %.2f  f32 lines(x16->f64 row eq /16*2) %.2f  changed-only f32 %.2f\n",
               k ? "GS" : "J", (double)acc[k].pendl / nb / M / 8.0, (double)acc[k].pendl16 / nb / M / 8.0,
               (double)acc[k].lines16 / nb / M / 8.0);
    report("BF jacobi", acc[0], nb);
    report("BF gauss-seidel", acc[1], nb);
    report("bucket pull (all in-arcs)", acc[2], nb);
    report("bucket pull (changed only)", acc[3], nb);
    printf("bucket changed-only scans/arcb %.2f\n", (double)acc[3].scans / nb / M);
    return 0;
}
