/*
 * topo_race.c -- concurrency stress of the drop-in's lock-free path cache:
 * several worker threads call topology_getLatency / getReliability /
 * incrementPathPacketCounter over overlapping pairs of a small host set, in two phases
 * (phase 2 after a late attach, so the late-attach matrix and the old rows' fill are
 * resolved by racing workers).  Every returned (latency, reliability) is written out for
 * the test (tests/test_topology_gpu.py) to check against the oracle; the increments made
 * are counted so the test can check that none is lost.
 *
 *   topo_race GRAPHML HINTS_FILE H1 H2 THREADS QUERIES_PER_THREAD OUT_FILE
 *     HINTS_FILE: one IP hint per line (host k is attached with hint k); H1 hosts in phase
 *     1, H1 + H2 in phase 2
 *   OUT_FILE: binary records {int32 phase, int32 i, int32 j, int32 pad, double lat, double rel}
 *   stdout: one JSON line {"increments", "cached_paths", "compute_failed"}, then one line
 *   "P a b cell count" per unordered host pair (topology_hip_cached_cell / _packet_count)
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "topology_hip.h"
#include "topology_hip_ext.h"

uint32_t address_toNetworkIP(Address* address); /* Shadow's (shadow_hooks.c stand-in here) */

typedef struct {
    int32_t phase, i, j, pad;
    double lat, rel;
} rec_t;

typedef struct {
    Topology* top;
    Address** hosts;
    int nh, phase;
    long queries;
    unsigned seed;
    rec_t* out;
    long nout, incs;
} worker_t;

static pthread_barrier_t g_start;

static void* worker(void* arg) {
    worker_t* w = arg;
    unsigned s = w->seed;
    pthread_barrier_wait(&g_start); /* all threads enter the first misses together */
    for (long q = 0; q < w->queries; q++) {
        const int i = (int)(rand_r(&s) % (unsigned)w->nh), j = (int)(rand_r(&s) % (unsigned)w->nh);
        Address *a = w->hosts[i], *b = w->hosts[j];
        const double lat = topology_getLatency(w->top, a, b);
        const double rel = topology_getReliability(w->top, a, b);
        w->out[w->nout++] = (rec_t){w->phase, i, j, 0, lat, rel};
        if (rand_r(&s) & 1) {
            topology_incrementPathPacketCounter(w->top, a, b);
            w->incs++;
        }
    }
    return NULL;
}

static long run_phase(Topology* top, Address** hosts, int nh, int nt, long nq, int phase, FILE* fo) {
    worker_t* ws = calloc((size_t)nt, sizeof(worker_t));
    pthread_t* th = malloc(sizeof(pthread_t) * (size_t)nt);
    pthread_barrier_init(&g_start, NULL, (unsigned)nt);
    for (int t = 0; t < nt; t++) {
        ws[t] = (worker_t){top, hosts, nh, phase, nq, 77u * (unsigned)t + 1000u * (unsigned)phase, NULL, 0, 0};
        ws[t].out = malloc(sizeof(rec_t) * (size_t)nq);
        pthread_create(&th[t], NULL, worker, &ws[t]);
    }
    long incs = 0;
    for (int t = 0; t < nt; t++) {
        pthread_join(th[t], NULL);
        fwrite(ws[t].out, sizeof(rec_t), (size_t)ws[t].nout, fo);
        incs += ws[t].incs;
        free(ws[t].out);
    }
    pthread_barrier_destroy(&g_start);
    free(ws);
    free(th);
    return incs;
}

int main(int argc, char** argv) {
    if (argc < 8) {
        fprintf(stderr, "usage: %s GRAPHML HINTS H1 H2 THREADS QUERIES OUT\n", argv[0]);
        return 2;
    }
    const int h1 = atoi(argv[3]), h2 = atoi(argv[4]), nt = atoi(argv[5]);
    const long nq = atol(argv[6]);
    shadowtopo_set_log_level(1);
    Topology* top = topology_new(argv[1]);
    if (!top) {
        printf("{\"error\": \"topology_new failed\"}\n");
        return 1;
    }
    FILE* fh = fopen(argv[2], "r");
    FILE* fo = fopen(argv[7], "wb");
    if (!fh || !fo) return 1;
    const int nh = h1 + h2;
    Address** hosts = malloc(sizeof(Address*) * (size_t)nh);
    Random* rnd = shadowtopo_random_new(7);
    char hint[64], ip[32];
    long incs = 0;
    for (int k = 0; k < nh; k++) {
        if (!fgets(hint, sizeof hint, fh)) return 1;
        hint[strcspn(hint, "\r\n")] = 0;
        snprintf(ip, sizeof ip, "11.%d.%d.%d", (k >> 16) & 255, (k >> 8) & 255, (k & 255) + 1);
        hosts[k] = shadowtopo_address_new(ip, "host");
        topology_attach(top, hosts[k], rnd, hint, NULL, NULL, NULL, NULL, NULL, NULL);
        if (k == h1 - 1) incs += run_phase(top, hosts, h1, nt, nq, 1, fo);
    }
    incs += run_phase(top, hosts, nh, nt, nq, 2, fo);
    fclose(fo);
    fclose(fh);
    topology_hip_info inf;
    topology_hip_get_info(top, &inf);
    printf("{\"increments\": %ld, \"cached_paths\": %lld, \"compute_failed\": %d}\n", incs,
           (long long)inf.cached_paths, inf.compute_failed);
    /* per unordered host pair: the emulated cache's cell and the cached Path's packet count */
    for (int a = 0; a < nh; a++)
        for (int b = a; b < nh; b++) {
            const int32_t va = topology_hip_vertex_of_ip(top, address_toNetworkIP(hosts[a]));
            const int32_t vb = topology_hip_vertex_of_ip(top, address_toNetworkIP(hosts[b]));
            printf("P %d %d %d %llu\n", a, b, topology_hip_cached_cell(top, va, vb),
                   (unsigned long long)topology_hip_packet_count(top, va, vb));
        }
    topology_free(top);
    for (int k = 0; k < nh; k++) shadowtopo_address_free(hosts[k]);
    free(hosts);
    shadowtopo_random_free(rnd);
    return 0;
}
