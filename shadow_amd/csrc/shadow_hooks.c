/*
 * shadow_hooks.c -- standalone defaults for the Shadow functions the topology shim calls,
 * plus the shim's logger.
 *
 * Every Shadow function here is a WEAK definition: when libshadowtopo_hip.so is loaded
 * into Shadow, the executable's strong definitions (main/routing/address.c:122,145,
 * main/utility/random.c:39-43, main/core/worker.c:412-415) take precedence through normal
 * ELF symbol interposition, and the Address/Random stand-ins below are never used.
 * Outside Shadow (tests, bench) they give the library something to call.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <netinet/in.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "shim_log.h"
#include "topology_hip_ext.h"

/* stand-in layouts (Shadow's real ones: address.c:21-40, random.c:15-18) */
struct _Address {
    uint32_t ip; /* network order, first member as in Shadow */
    char ipString[INET_ADDRSTRLEN];
    char name[64];
    char idString[128];
};

struct _Random {
    unsigned int seedState;
    unsigned int initialSeed;
};

/* the last upcall's value; worker threads upcall concurrently (Shadow's master takes a lock,
 * master.c:148-159), so the stand-in keeps it in one atomic word */
static _Atomic double g_last_min_jump = -1.0;
static _Atomic long g_min_jump_calls = 0;
static int g_log_level = -1;

__attribute__((weak)) uint32_t address_toNetworkIP(Address* address) { return address->ip; }

__attribute__((weak)) in_addr_t address_stringToIP(const char* ipString) {
    struct in_addr a;
    if (ipString && inet_pton(AF_INET, ipString, &a) == 1) return a.s_addr;
    return INADDR_NONE;
}

__attribute__((weak)) char* address_toHostIPString(Address* address) { return address->ipString; }

__attribute__((weak)) char* address_toString(Address* address) { return address->idString; }

/* random.c:32-43: rand_r over the pool's seed state, scaled by RAND_MAX */
__attribute__((weak)) double random_nextDouble(Random* random) {
    int v = rand_r(&random->seedState);
    return (double)(((double)v) / ((double)RAND_MAX));
}

__attribute__((weak)) void worker_updateMinTimeJump(double minPathLatency) {
    atomic_store_explicit(&g_last_min_jump, minPathLatency, memory_order_relaxed);
    atomic_fetch_add_explicit(&g_min_jump_calls, 1, memory_order_relaxed);
}

Address* shadowtopo_address_new(const char* ipString, const char* name) {
    Address* a = (Address*)calloc(1, sizeof(Address));
    if (!a) return NULL;
    struct in_addr in;
    if (!ipString || inet_pton(AF_INET, ipString, &in) != 1) {
        free(a);
        return NULL;
    }
    a->ip = in.s_addr;
    snprintf(a->ipString, sizeof a->ipString, "%s", ipString);
    snprintf(a->name, sizeof a->name, "%s", name ? name : "host");
    snprintf(a->idString, sizeof a->idString, "%s-%s (eth,mac=0)", a->name, a->ipString);
    return a;
}

void shadowtopo_address_free(Address* a) { free(a); }

Random* shadowtopo_random_new(uint32_t seed) {
    Random* r = (Random*)calloc(1, sizeof(Random));
    if (!r) return NULL;
    r->seedState = seed;
    r->initialSeed = seed;
    return r;
}

void shadowtopo_random_free(Random* r) { free(r); }

double shadowtopo_last_min_time_jump(void) { return atomic_load_explicit(&g_last_min_jump, memory_order_relaxed); }

/* the stand-in's upcall count (the tests compare it with the reference model's upcalls) */
long shadowtopo_min_time_jump_calls(void) { return atomic_load_explicit(&g_min_jump_calls, memory_order_relaxed); }

void shadowtopo_set_log_level(int level) { g_log_level = level; }

int shadowtopo_log_enabled(int level) {
    if (g_log_level < 0) {
        const char* e = getenv("SHADOWTOPO_LOG_LEVEL");
        g_log_level = e ? atoi(e) : ST_WARNING;
    }
    return level <= g_log_level;
}

void shadowtopo_log(int level, const char* func, const char* fmt, ...) {
    static const char* names[] = {"error", "critical", "warning", "message", "info", "debug"};
    if (!shadowtopo_log_enabled(level)) return;
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    fprintf(stderr, "[shadowtopo] [%s] [%s] %s\n", names[level < 0 ? 0 : (level > 5 ? 5 : level)], func, buf);
}
