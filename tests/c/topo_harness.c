/*
 * topo_harness.c -- a C caller of the drop-in API (include/topology_hip.h), the way Shadow
 * links it: GraphML ingest, host attachment with hints, then per-packet lookups from N
 * worker threads (worker.c:267-279 calls getLatency / getReliability / increment per
 * packet).  Prints one JSON line with the timings.
 *
 *   topo_harness GRAPHML HOSTS THREADS QUERIES_PER_THREAD [HINTMODE]
 *     HINTMODE 0: no hints (random vertex), 1: type + country hints, 2: IP hints
 *     QUERIES_PER_THREAD 0: ingest + attach only (no GPU needed)
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "topology_hip.h"
#include "topology_hip_ext.h"

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

typedef struct {
    Topology* top;
    Address** hosts;
    int nh;
    long queries;
    unsigned seed;
    double sum;
    long routable;
    double secs;
    int warm_only; /* run the untimed warm pass only */
} worker_t;

static int g_warm = 0; /* TOPO_HARNESS_WARM=1: one untimed pass first (the emulated cache warm) */

static void* worker(void* arg) {
    worker_t* w = arg;
    unsigned s = w->seed;
    if (w->warm_only) {
        unsigned s2 = w->seed + 7919u;
        for (long q = 0; q < w->queries; q++) {
            Address* a = w->hosts[rand_r(&s2) % w->nh];
            Address* b = w->hosts[rand_r(&s2) % w->nh];
            if (topology_isRoutable(w->top, a, b)) (void)topology_getLatency(w->top, a, b);
        }
        return NULL;
    }
    /* the tallies stay in locals: the workers' structs share cache lines, and a store to
       them per query made the threads' lookups pay for false sharing */
    double sum = 0.0;
    long routable = 0;
    double t0 = now();
    for (long q = 0; q < w->queries; q++) {
        Address* a = w->hosts[rand_r(&s) % w->nh];
        Address* b = w->hosts[rand_r(&s) % w->nh];
        /* the per-packet sequence of worker.c:267-279 */
        if (topology_isRoutable(w->top, a, b)) {
            routable++;
            sum += topology_getLatency(w->top, a, b) + topology_getReliability(w->top, a, b);
            topology_incrementPathPacketCounter(w->top, a, b);
        }
    }
    w->sum = sum;
    w->routable = routable;
    w->secs = now() - t0;
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s GRAPHML HOSTS THREADS QUERIES_PER_THREAD [HINTMODE]\n", argv[0]);
        return 2;
    }
    const int nh = atoi(argv[2]), nt = atoi(argv[3]);
    const long nq = atol(argv[4]);
    const int mode = argc > 5 ? atoi(argv[5]) : 0;
    g_warm = getenv("TOPO_HARNESS_WARM") && atoi(getenv("TOPO_HARNESS_WARM")) > 0;
    shadowtopo_set_log_level(1);
    double t0 = now();
    Topology* top = topology_new(argv[1]);
    double t_ingest = now() - t0;
    if (!top) {
        printf("{\"error\": \"topology_new failed\"}\n");
        return 1;
    }
    topology_hip_info inf;
    topology_hip_get_info(top, &inf);
    Address** hosts = malloc(sizeof(Address*) * (size_t)nh);
    Random* rnd = shadowtopo_random_new(12345);
    static const char* types[] = {"client", "relay", "server"};
    static const char* cc[] = {"US", "DE", "FR", "BR", "JP"};
    char ip[32], hint[32];
    t0 = now();
    for (int k = 0; k < nh; k++) {
        snprintf(ip, sizeof ip, "11.%d.%d.%d", (k >> 16) & 255, (k >> 8) & 255, (k & 255) + 0);
        if ((k & 255) == 0) snprintf(ip, sizeof ip, "12.%d.%d.1", (k >> 16) & 255, (k >> 8) & 255);
        hosts[k] = shadowtopo_address_new(ip, "host");
        if (mode == 1)
            topology_attach(top, hosts[k], rnd, NULL, NULL, (char*)cc[k % 5], NULL, (char*)types[k % 3], NULL, NULL);
        else if (mode == 2) {
            snprintf(hint, sizeof hint, "10.%d.%d.%d", (k * 7) & 255, (k * 13) & 255, (k * 29) & 255);
            topology_attach(top, hosts[k], rnd, hint, NULL, NULL, NULL, NULL, NULL, NULL);
        } else
            topology_attach(top, hosts[k], rnd, NULL, NULL, NULL, NULL, NULL, NULL, NULL);
    }
    double t_attach = now() - t0;
    topology_hip_get_info(top, &inf);
    double t_prepare = 0, lookup_ns = 0, sum = 0;
    long long runs_warm = -1, paths_warm = -1;
    long routable = 0;
    if (nq > 0) {
        t0 = now();
        int rc = topology_hip_prepare(top);
        t_prepare = now() - t0;
        if (g_warm) { /* the warm pass alone (its misses), then the timed pass's on top */
            worker_t* wp = calloc((size_t)nt, sizeof(worker_t));
            pthread_t* tp = malloc(sizeof(pthread_t) * (size_t)nt);
            for (int i = 0; i < nt; i++) {
                wp[i] = (worker_t){top, hosts, nh, nq, 1000u + (unsigned)i, 0.0, 0, 0.0};
                wp[i].warm_only = 1;
                pthread_create(&tp[i], NULL, worker, &wp[i]);
            }
            for (int i = 0; i < nt; i++) pthread_join(tp[i], NULL);
            free(wp);
            free(tp);
            topology_hip_get_info(top, &inf);
            runs_warm = inf.dijkstra_runs;
            paths_warm = inf.cached_paths;
        }
        worker_t* ws = calloc((size_t)nt, sizeof(worker_t));
        pthread_t* th = malloc(sizeof(pthread_t) * (size_t)nt);
        for (int i = 0; i < nt; i++) {
            ws[i] = (worker_t){top, hosts, nh, nq, 1000u + (unsigned)i, 0.0, 0, 0.0};
            pthread_create(&th[i], NULL, worker, &ws[i]);
        }
        double worst = 0;
        for (int i = 0; i < nt; i++) {
            pthread_join(th[i], NULL);
            sum += ws[i].sum;
            routable += ws[i].routable;
            if (ws[i].secs > worst) worst = ws[i].secs;
        }
        /* one "lookup" = one topology call; a routable packet makes four */
        long calls = (long)nt * nq + 3 * routable;
        lookup_ns = worst * 1e9 / ((double)calls / nt);
        if (rc) fprintf(stderr, "prepare failed (no GPU?)\n");
        free(ws);
        free(th);
    }
    topology_hip_get_info(top, &inf);
    printf("{\"vertices\": %d, \"edges\": %lld, \"hosts\": %d, \"attached\": %d, \"ingest_s\": %.4f, "
           "\"attach_s\": %.4f, \"attach_us_per_host\": %.3f, \"prepare_s\": %.4f, \"threads\": %d, "
           "\"queries_per_thread\": %ld, \"ns_per_call_per_thread\": %.2f, \"routable\": %ld, \"checksum\": %.6e, "
           "\"compute_failed\": %d, \"warm\": %d, \"dijkstra_runs\": %lld, \"cached_paths\": %lld, "
           "\"dijkstra_runs_after_warm\": %lld, \"cached_paths_after_warm\": %lld}\n",
           inf.n_vertices, (long long)inf.n_edges, nh, inf.n_attached, t_ingest, t_attach, t_attach * 1e6 / nh,
           t_prepare, nt, nq, lookup_ns, routable, sum, inf.compute_failed, g_warm, (long long)inf.dijkstra_runs,
           (long long)inf.cached_paths, runs_warm, paths_warm);
    topology_free(top);
    for (int k = 0; k < nh; k++) shadowtopo_address_free(hosts[k]);
    free(hosts);
    shadowtopo_random_free(rnd);
    return 0;
}
