/*
 * shim_asan.c -- the drop-in's host paths under AddressSanitizer / UBSan (no GPU needed):
 * GraphML ingest and validation of each file on the command line (rejected files included),
 * then for each accepted graph: attaches with no hints, type + country hints and IP hints,
 * detaches and re-attaches (the lock-free IP table's tombstones and growth), IP lookups,
 * and topology_free.  Queries are not made (they need the GPU).  The test
 * (tests/test_topology_shim.py) compiles the shim's C sources into this program with the
 * sanitizers, so the instrumented copies are the ones that run.
 *
 *   shim_asan HOSTS GRAPHML...
 *   stdout: one line per file: "<path> rejected" or "<path> ok <vertices> <attached>"
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "topology_hip.h"
#include "topology_hip_ext.h"

uint32_t address_toNetworkIP(Address* address); /* Shadow's (shadow_hooks.c stand-in here) */

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s HOSTS GRAPHML...\n", argv[0]);
        return 2;
    }
    const int nh = atoi(argv[1]);
    shadowtopo_set_log_level(0);
    static const char* types[] = {"client", "relay", "server", ""};
    static const char* cc[] = {"US", "DE", "FR", "BR", "JP"};
    for (int f = 2; f < argc; f++) {
        Topology* top = topology_new(argv[f]);
        if (!top) {
            printf("%s rejected\n", argv[f]);
            continue;
        }
        Address** hosts = calloc((size_t)nh, sizeof(Address*));
        Random* rnd = shadowtopo_random_new(777u + (uint32_t)f);
        char ip[32], hint[32];
        for (int k = 0; k < nh; k++) {
            snprintf(ip, sizeof ip, "11.%d.%d.%d", (k >> 16) & 255, (k >> 8) & 255, (k & 255) + 1 > 255 ? 1 : (k & 255) + 1);
            hosts[k] = shadowtopo_address_new(ip, "host");
            switch (k % 3) {
                case 0:
                    topology_attach(top, hosts[k], rnd, NULL, NULL, NULL, NULL, NULL, NULL, NULL);
                    break;
                case 1:
                    topology_attach(top, hosts[k], rnd, NULL, NULL, (char*)cc[k % 5], NULL, (char*)types[k % 4], NULL,
                                    NULL);
                    break;
                default:
                    snprintf(hint, sizeof hint, "10.%d.%d.%d", (k * 7) & 3, (k * 13) & 255, (k * 29) & 255);
                    topology_attach(top, hosts[k], rnd, hint, NULL, NULL, NULL, NULL, NULL, NULL);
            }
        }
        /* churn: detach every third host, look every host up, attach the detached ones again */
        for (int k = 0; k < nh; k += 3) topology_detach(top, hosts[k]);
        long found = 0;
        for (int k = 0; k < nh; k++) found += topology_hip_vertex_of_ip(top, address_toNetworkIP(hosts[k])) >= 0;
        for (int k = 0; k < nh; k += 3) topology_attach(top, hosts[k], rnd, NULL, NULL, NULL, NULL, NULL, NULL, NULL);
        topology_hip_info inf;
        topology_hip_get_info(top, &inf);
        printf("%s ok %d %d %ld\n", argv[f], inf.n_vertices, inf.n_attached, found);
        topology_free(top);
        for (int k = 0; k < nh; k++) shadowtopo_address_free(hosts[k]);
        free(hosts);
        shadowtopo_random_free(rnd);
    }
    return 0;
}
